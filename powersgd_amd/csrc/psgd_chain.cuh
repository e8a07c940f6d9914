// Panel helpers shared by the orthonormalisation kernels (psgd_small.hip) and the projection
// form's in-pass Cholesky-QR (psgd_final.cuh): panel row loads/stores, fp64 wave sums, the
// Cholesky-QR chain with LAPACK column signs, and the exact Householder QR (geqr2 + org2r)
// that rejected panels take (reference powersgd/orthogonalization.py:8, torch.linalg.qr).
#pragma once

#include "psgd_stream.cuh"

namespace psgd {

// a panel row of r floats: one 16-byte (or 8-byte) access when r == R in {2, 4, 8}
template <int R>
__device__ __forceinline__ void ld_row(const float* __restrict__ p, int r, float (&v)[R]) {
    ld_factor<R>(gconst<float>(p), r, v);
}
template <int R>
__device__ __forceinline__ void st_row(float* __restrict__ p, int r, const float (&v)[R]) {
    const gptr<float> g = gmut<float>(p);
    if constexpr (R % 4 == 0) {
        if (r == R) {
#pragma unroll
            for (int c = 0; c < R; c += 4) {
                const v4f x = {v[c], v[c + 1], v[c + 2], v[c + 3]};
                *(gptr<v4f>)(g + c) = x;
            }
            return;
        }
    } else if constexpr (R == 2) {
        if (r == 2) {
            const v2f x = {v[0], v[1]};
            *(gptr<v2f>)g = x;
            return;
        }
    }
#pragma unroll
    for (int c = 0; c < R; ++c)
        if (c < r) g[c] = v[c];
}

// Sum of NV values over a workgroup of NW waves, broadcast to every thread (fixed order).
template <typename A, int NV, int NW>
__device__ __forceinline__ void block_sum_nw(A (&v)[NV], A* red) {
#pragma unroll
    for (int i = 0; i < NV; ++i)
        for (int s = 32; s > 0; s >>= 1) v[i] += __shfl_xor(v[i], s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) red[wave * NV + i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        A t = red[i];
        for (int w = 1; w < NW; ++w) t += red[w * NV + i];
        v[i] = t;
    }
}

// rout (optional): the r x r factor R of the QR (geqr2's upper triangle), row-major
template <int R, int NT = kBlock>
__device__ void householder_q(float* A, int64_t k, int r, float* red, float* tau, float* rout = nullptr) {
    const int tid = threadIdx.x;
    for (int j = 0; j < r; ++j) {
        float s1[1] = {0.f};
        for (int64_t i = j + 1 + tid; i < k; i += NT) {
            const float x = A[i * r + j];
            s1[0] = fmaf(x, x, s1[0]);
        }
        block_sum_nw<float, 1, NT / 64>(s1, red);
        const float alpha = A[int64_t(j) * r + j];
        float tj = 0.f;
        if (s1[0] != 0.f) {
            const float xnorm = sqrtf(s1[0]);
            const float beta = -copysignf(hypotf(alpha, xnorm), alpha);
            tj = (beta - alpha) / beta;
            const float scal = 1.f / (alpha - beta);
            for (int64_t i = j + 1 + tid; i < k; i += NT) A[i * r + j] *= scal;
            __syncthreads();
            if (tid == 0) A[int64_t(j) * r + j] = beta;
        }
        if (tid == 0) tau[j] = tj;
        __syncthreads();
        if (tj != 0.f && j + 1 < r) {
            // w_c = A[j,c] + sum_{i>j} v_i A[i,c] ; A[i,c] -= tau v_i w_c   (c > j)
            float w[R];
#pragma unroll
            for (int c = 0; c < R; ++c) w[c] = 0.f;
            for (int64_t i = j + 1 + tid; i < k; i += NT) {
                const float vi = A[i * r + j];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > j && c < r) w[c] = fmaf(vi, A[i * r + c], w[c]);
            }
            block_sum_nw<float, R, NT / 64>(w, red);
#pragma unroll
            for (int c = 0; c < R; ++c)
                if (c > j && c < r) w[c] += A[int64_t(j) * r + c];
            __syncthreads();
            for (int64_t i = j + tid; i < k; i += NT) {
                const float vi = i == j ? 1.f : A[i * r + j];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > j && c < r) A[i * r + c] -= tj * vi * w[c];
            }
            __syncthreads();
        }
    }
    if (rout) {
        for (int e = tid; e < r * r; e += NT) {
            const int i = e / r, j = e - (e / r) * r;
            rout[e] = i <= j ? A[int64_t(i) * r + j] : 0.f;
        }
        __syncthreads();  // read before org2r overwrites the upper triangle
    }
    // org2r: Q = H_0 H_1 ... H_{r-1} I[:, :r], built in place, last reflector first
    for (int j = r - 1; j >= 0; --j) {
        const float tj = tau[j];
        if (j + 1 < r && tj != 0.f) {
            float w[R];
#pragma unroll
            for (int c = 0; c < R; ++c) w[c] = 0.f;
            for (int64_t i = j + 1 + tid; i < k; i += NT) {
                const float vi = A[i * r + j];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > j && c < r) w[c] = fmaf(vi, A[i * r + c], w[c]);
            }
            block_sum_nw<float, R, NT / 64>(w, red);
#pragma unroll
            for (int c = 0; c < R; ++c)
                if (c > j && c < r) w[c] += A[int64_t(j) * r + c];
            __syncthreads();
            for (int64_t i = j + tid; i < k; i += NT) {
                const float vi = i == j ? 1.f : A[i * r + j];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > j && c < r) A[i * r + c] -= tj * vi * w[c];
            }
            __syncthreads();
        }
        for (int64_t i = j + 1 + tid; i < k; i += NT) A[i * r + j] *= -tj;
        for (int64_t i = tid; i < j; i += NT) A[i * r + j] = 0.f;
        if (tid == 0) A[int64_t(j) * r + j] = 1.f - tj;
        __syncthreads();
    }
}


// fp64 all-reduce over the 64 lanes with DPP row rotations + gfx950 half-row swaps on the
// two 32-bit halves (the fixed order of wave_allsum; no ds_bpermute round trips)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, uint32_t(b), CTRL, 0xf, 0xf, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, uint32_t(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((uint64_t(hi) << 32) | lo);
}
__device__ __forceinline__ double wave_allsum_f64(double v) {
    v += dpp_f64<0x128>(v);
    v += dpp_f64<0x124>(v);
    v += dpp_f64<0x122>(v);
    v += dpp_f64<0x121>(v);
    {
        const uint64_t b = __double_as_longlong(v);
        const auto l = __builtin_amdgcn_permlane16_swap(uint32_t(b), uint32_t(b), false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(uint32_t(b >> 32), uint32_t(b >> 32), false, false);
        v = __longlong_as_double((uint64_t(h[0]) << 32) | l[0]) + __longlong_as_double((uint64_t(h[1]) << 32) | l[1]);
    }
    {
        const uint64_t b = __double_as_longlong(v);
        const auto l = __builtin_amdgcn_permlane32_swap(uint32_t(b), uint32_t(b), false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(uint32_t(b >> 32), uint32_t(b >> 32), false, false);
        v = __longlong_as_double((uint64_t(h[0]) << 32) | l[0]) + __longlong_as_double((uint64_t(h[1]) << 32) | l[1]);
    }
    return v;
}

// A sign pivot |T_jj| within this of 1 marks a column LAPACK leaves unreflected (tau = 0)
// or nearly so; orthonormal-column entries of a real panel sit far below it.
constexpr double kSignTol = 1e-5;


// The r x r work of Cholesky-QR on one wave (a serial fp64 latency chain; the other waves
// would only compete for the fp64 pipes): Cholesky of the Gram g (upper, NG entries), M =
// R^-1, and LAPACK's column signs D from the top block T = X[0:r] M (`top`: the top R x R rows
// in LDS, or null: loaded from st). Lane 0 publishes M D (m_sh, R x R), ok and R' = D R.
template <int R>
__device__ __forceinline__ void chol_chain(const double* g, const float* top, const float* st, int r, int64_t k,
                                           double* m_sh, int* ok_sh, float* rfac) {
        double Rm[R][R];
        double inv[R];  // 1 / R_jj: one division per column, products elsewhere (the chain is
                        // serial; each fp64 division is a ~10-instruction dependent sequence)
        bool ok = true;
        {
            double G[R][R];
            int e = 0;
#pragma unroll
            for (int c = 0; c < R; ++c)
#pragma unroll
                for (int b = c; b < R; ++b) {
                    G[c][b] = g[e];
                    G[b][c] = g[e];
                    ++e;
                }
#pragma unroll
            for (int j = 0; j < R; ++j) {
#pragma unroll
                for (int b = 0; b < R; ++b) Rm[j][b] = 0.0;
            }
#pragma unroll
            for (int j = 0; j < R; ++j) {
                inv[j] = 1.0;
                if (j < r) {
                    double piv = G[j][j];
#pragma unroll
                    for (int l = 0; l < R; ++l)
                        if (l < j) piv -= Rm[l][j] * Rm[l][j];
                    ok = ok && piv > 1e-8 * G[j][j] && piv > 0.0;
                    const double d = sqrt(piv > 0.0 ? piv : 1.0);
                    Rm[j][j] = d;
                    inv[j] = 1.0 / d;
#pragma unroll
                    for (int b = 0; b < R; ++b)
                        if (b > j && b < r) {
                            double v = G[j][b];
#pragma unroll
                            for (int l = 0; l < R; ++l)
                                if (l < j) v -= Rm[l][j] * Rm[l][b];
                            Rm[j][b] = v * inv[j];
                        }
                }
            }
        }
        // M = R^-1 (upper triangular, back substitution column by column)
        double M[R][R];
#pragma unroll
        for (int c = 0; c < R; ++c) {
#pragma unroll
            for (int i = R - 1; i >= 0; --i) {
                double v = (i == c) ? 1.0 : 0.0;
#pragma unroll
                for (int l = 0; l < R; ++l)
                    if (l > i && l < r) v -= Rm[i][l] * M[l][c];
                M[i][c] = (i < r && c < r) ? v * inv[i] : 0.0;
            }
        }
        // LAPACK column signs from the top block T = X[0:r] M
        double T[R][R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            float x[R];
            if (top) {
#pragma unroll
                for (int c = 0; c < R; ++c) x[c] = top[(i < r ? i : 0) * R + c];  // LDS, written before a barrier
            } else {
                ld_row<R>(st + int64_t(i < r ? i : 0) * r, r, x);
            }
#pragma unroll
            for (int c = 0; c < R; ++c) {
                double v = 0.0;
#pragma unroll
                for (int l = 0; l < R; ++l) v += double(x[l]) * M[l][c];
                T[i][c] = v;
            }
        }
        double sgn[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            if (j < r) {
                const bool nonneg = T[j][j] >= 0.0;
                // |T_jj| = 1 is LAPACK's xnorm == 0 column (tau = 0, beta = alpha, no flip):
                // the reconstruction cannot tell it from a tiny trailing sub-column, so such
                // panels (e.g. upper trapezoidal) take the exact Householder recursion
                ok = ok && !(j < k - 1 && fabs(T[j][j]) > 1.0 - kSignTol);
                sgn[j] = (j == k - 1) ? (nonneg ? 1.0 : -1.0) : (nonneg ? -1.0 : 1.0);
                T[j][j] -= sgn[j];
                const double ip = 1.0 / T[j][j];
#pragma unroll
                for (int i = 0; i < R; ++i)
                    if (i > j && i < r) {
                        const double l = T[i][j] * ip;
#pragma unroll
                        for (int b = 0; b < R; ++b)
                            if (b > j && b < r) T[i][b] -= l * T[j][b];
                    }
            } else {
                sgn[j] = 1.0;
            }
        }
        if ((threadIdx.x & 63) == 0) {
#pragma unroll
            for (int i = 0; i < R; ++i)
#pragma unroll
                for (int c = 0; c < R; ++c) m_sh[i * R + c] = M[i][c] * sgn[c];
            *ok_sh = ok ? 1 : 0;
            if (rfac && ok) {  // X = Q (D R): R' = D R
#pragma unroll
                for (int i = 0; i < R; ++i)
#pragma unroll
                    for (int c = 0; c < R; ++c)
                        if (i < r && c < r) rfac[i * r + c] = i <= c ? float(sgn[i] * Rm[i][c]) : 0.f;
            }
        }
}


}  // namespace psgd
