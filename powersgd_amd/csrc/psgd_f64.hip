// fp64 gradients: the reference's own error-feedback test dtype (tests/powersgd_test.py:38,
// torch.set_default_dtype(torch.float64)). There the P/Q factors follow the default dtype
// (powersgd.py:241-251), so gradients, factors and every product are fp64. This file is the
// codec for that case, kernel for kernel the fp32 path's structure (psgd_stream.cuh,
// psgd_small.hip) without its fusions:
//
//   k_f64_even   Q_part = G_k^T X per (64-column strip, 256-row chunk) tile, one partial per
//                wave (no atomics)                           reference powersgd.py:185-193
//   k_f64_reduce fixed-order sum of the partials -> Q state + history copy
//   k_f64_odd    P = G_k X, one wave per row, xor-butterfly column sum (bitwise the same in
//                every lane)                                 reference powersgd.py:185-193
//   k_f64_orth   rank 1: joint norm over the shape group; rank > 1: Householder QR
//                (LAPACK dgeqr2 + dorg2r conventions)        reference orthogonalization.py:4-8
//   k_f64_apply  residual = G_0 - sum_k P_k Q_k^T, output = sum_k alpha P_k Qbar_k^T
//                                                            reference powersgd.py:195-230
//   k_flat_pack_f64  uncompressed tensors: flat = x / W, x = 0  reference powersgd.py:22-31
//
// G_k = G_0 - sum_{j<k} P_j Q_j^T is formed on the fly, as in the fp32 path (the reference's
// in-place baddbmm_, :195-202, element by element). fp64 is a parity path (the reference's
// test dtype, not a BASELINE workload): coalesced 8-byte loads, no MFMA (the fp64 MFMA would
// not pay at rank <= 32 products that are HBM-bound anyway).
#include <hip/hip_runtime.h>

#include <cmath>

#include "psgd_internal.h"

namespace psgd {

namespace {

__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s);  // identical result in every lane
    return v;
}

// Sum of NV doubles over the 256-thread workgroup in a fixed order (wave butterflies, then
// waves 0..3 in order), broadcast to every thread. `red` holds kWaves * NV doubles.
template <int NV>
__device__ __forceinline__ void block_sum64(double (&v)[NV], double* red) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_sum64(v[i]);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) red[wave * NV + i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        double t = red[i];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) t += red[w * NV + i];
        v[i] = t;
    }
}

// (P_k Q_k^T)[i, j] for one term, c-ordered dot
template <int R>
__device__ __forceinline__ double term_dot(const double* p, const double* q, int r) {
    double t = 0.0;
#pragma unroll
    for (int c = 0; c < R; ++c)
        if (c < r) t = c == 0 ? p[0] * q[0] : fma(p[c], q[c], t);
    return t;
}

}  // namespace

// ------------------------------------------------------------------ even product --
template <int R>
__global__ __launch_bounds__(kBlock) void k_f64_even(F64Args a) {
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = d.r;
    const int64_t n = d.n, m = d.m;
    const int64_t col = int64_t(t.strip) * kF64Cols + lane;
    const bool active = col < m;
    const int64_t cc = active ? col : 0;
    const double* G = static_cast<const double*>(a.grads[d.tensor]);
    const int64_t i0 = int64_t(t.chunk) * kF64Rows, i1 = n < i0 + kF64Rows ? n : i0 + kF64Rows;
    double acc[R];
#pragma unroll
    for (int c = 0; c < R; ++c) acc[c] = 0.0;
    for (int64_t i = i0 + wave; i < i1; i += kWaves) {
        double g = G[i * m + cc];
        for (int k = 0; k < a.nres; ++k)
            g -= term_dot<R>(a.res.p[k] + d.poff + i * r, a.res.q[k] + d.qoff + cc * r, r);
        const double* x = a.x + d.poff + i * r;
#pragma unroll
        for (int c = 0; c < R; ++c)
            if (c < r) acc[c] = fma(g, x[c], acc[c]);
    }
    if (active) {
        double* dst = a.part + a.part_off[t.mat] + ((int64_t(t.chunk) * kWaves + wave) * m + col) * r;
#pragma unroll
        for (int c = 0; c < R; ++c)
            if (c < r) dst[c] = acc[c];
    }
}

// one wave per item of kRedElems (64) consecutive Q elements; partials summed in order
__global__ __launch_bounds__(64) void k_f64_reduce(F64Args a) {
    const RedItem it = a.items[blockIdx.x];
    const MatDesc d = a.mats[it.mat];
    const int64_t len = d.m * d.r;
    const int64_t e = int64_t(it.start) + threadIdx.x;
    if (e >= len) return;
    const int np = d.nchunk * kWaves;
    const double* p = a.part + a.part_off[it.mat] + e;
    double s = 0.0;
    for (int c = 0; c < np; ++c) s += p[int64_t(c) * len];
    a.y[d.qoff + e] = s;
    a.yh[d.qoff + e] = s;
}

// ------------------------------------------------------------------- odd product --
template <int R>
__global__ __launch_bounds__(kBlock) void k_f64_odd(F64Args a) {
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = d.r;
    const int64_t n = d.n, m = d.m;
    const double* G = static_cast<const double*>(a.grads[d.tensor]);
    constexpr int kRowsPerWave = kF64OddRows / kWaves;
    for (int u = 0; u < kRowsPerWave; ++u) {
        const int64_t i = int64_t(t.chunk) * kF64OddRows + wave * kRowsPerWave + u;
        if (i >= n) break;  // wave-uniform
        double acc[R];
#pragma unroll
        for (int c = 0; c < R; ++c) acc[c] = 0.0;
        for (int64_t j = lane; j < m; j += 64) {
            double g = G[i * m + j];
            for (int k = 0; k < a.nres; ++k)
                g -= term_dot<R>(a.res.p[k] + d.poff + i * r, a.res.q[k] + d.qoff + j * r, r);
            const double* x = a.x + d.qoff + j * r;
#pragma unroll
            for (int c = 0; c < R; ++c)
                if (c < r) acc[c] = fma(g, x[c], acc[c]);
        }
#pragma unroll
        for (int c = 0; c < R; ++c) acc[c] = wave_sum64(acc[c]);
        if (lane < r) {
            double v = acc[0];
#pragma unroll
            for (int c = 1; c < R; ++c) v = lane == c ? acc[c] : v;
            a.y[d.poff + i * r + lane] = v;
            a.yh[d.poff + i * r + lane] = v;
        }
    }
}

// ------------------------------------------------------------------------- apply --
template <int R>
__global__ __launch_bounds__(kBlock) void k_f64_apply(F64Args a) {
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    const int r = d.r;
    const int64_t n = d.n, m = d.m;
    double* G = static_cast<double*>(a.grads[d.tensor]);
    double* O = static_cast<double*>(a.out) + d.out_off;
    const int64_t i0 = int64_t(t.chunk) * d.chunk_rows;
    const int64_t i1 = n < i0 + d.chunk_rows ? n : i0 + d.chunk_rows;
    const int64_t e1 = i1 * m;
    const double alpha = a.alpha;
    for (int64_t e = i0 * m + threadIdx.x; e < e1; e += kBlock) {
        const int64_t i = e / m, j = e - i * m;
        double g = G[e];
        double o = 0.0;
        for (int k = 0; k < a.nres; ++k) {
            g -= term_dot<R>(a.res.p[k] + d.poff + i * r, a.res.q[k] + d.qoff + j * r, r);   // :195-202
            o += alpha * term_dot<R>(a.apx.p[k] + d.poff + i * r, a.apx.q[k] + d.qoff + j * r, r);  // :211-219
        }
        G[e] = g;
        O[e] = o;
    }
}

// ---------------------------------------------------------------- orthonormalise --
// One 256-thread workgroup per unit. Rank 1: x /= max(||x||_F over the whole shape group,
// 1e-16). Rank > 1: Q of the reduced Householder QR of the [k, r] panel, in place — dgeqr2
// (dlarfg: beta = -sign(alpha) * hypot(alpha, ||x||), tau = 0 when ||x|| == 0) then dorg2r.
template <int R>
__global__ __launch_bounds__(kBlock) void k_f64_orth(F64OrthArgs a) {
    __shared__ double red[kWaves * (R > 1 ? R : 1)];
    __shared__ double tau[R];
    const OrthUnit u = a.units[blockIdx.x];
    double* A = a.state + u.off;
    const int tid = threadIdx.x;
    const int64_t k = u.k;
    const int r = u.r;
    const int64_t total = k * r * u.count;
    if (a.save)
        for (int64_t e = tid; e < total; e += kBlock) a.save[u.off + e] = A[e];
    if (r == 1) {  // a rank-1 shape group (also inside a wider plan: min(shape) == 1)
        double ss[1] = {0.0};
        for (int64_t e = tid; e < total; e += kBlock) ss[0] = fma(A[e], A[e], ss[0]);
        block_sum64<1>(ss, red);
        const double nrm = sqrt(ss[0]);
        const double dv = nrm > 1e-16 ? nrm : 1e-16;
        for (int64_t e = tid; e < total; e += kBlock) {
            const double v = A[e] / dv;
            A[e] = v;
            a.hx[u.off + e] = v;
        }
        return;
    }
    if constexpr (R > 1) {
        __syncthreads();  // the save copy reads A before it is overwritten
        // ---- dgeqr2
        for (int j = 0; j < r; ++j) {
            double sg[1] = {0.0};
            for (int64_t i = j + 1 + tid; i < k; i += kBlock) sg[0] = fma(A[i * r + j], A[i * r + j], sg[0]);
            block_sum64<1>(sg, red);
            const double alpha = A[int64_t(j) * r + j];
            const double xnorm = sqrt(sg[0]);
            double tj = 0.0;
            if (xnorm != 0.0) {
                const double beta = -copysign(hypot(alpha, xnorm), alpha);
                tj = (beta - alpha) / beta;
                const double scal = 1.0 / (alpha - beta);
                for (int64_t i = j + 1 + tid; i < k; i += kBlock) A[i * r + j] *= scal;
                __syncthreads();
                if (tid == 0) A[int64_t(j) * r + j] = beta;
            }
            if (tid == 0) tau[j] = tj;
            __syncthreads();
            if (tj != 0.0 && j + 1 < r) {  // H_j applied to columns j+1..r-1 (dlarf)
                double w[R];
#pragma unroll
                for (int c = 0; c < R; ++c) w[c] = 0.0;
                for (int64_t i = j + tid; i < k; i += kBlock) {
                    const double v = i == j ? 1.0 : A[i * r + j];
#pragma unroll
                    for (int c = 0; c < R; ++c)
                        if (c > j && c < r) w[c] = fma(v, A[i * r + c], w[c]);
                }
                block_sum64<R>(w, red);
                for (int64_t i = j + tid; i < k; i += kBlock) {
                    const double v = i == j ? 1.0 : A[i * r + j];
#pragma unroll
                    for (int c = 0; c < R; ++c)
                        if (c > j && c < r) A[i * r + c] -= tj * v * w[c];
                }
                __syncthreads();
            }
        }
        // ---- dorg2r: Q in place, reflectors applied in reverse
        for (int j = r - 1; j >= 0; --j) {
            const double tj = tau[j];
            if (j + 1 < r) {
                double w[R];
#pragma unroll
                for (int c = 0; c < R; ++c) w[c] = 0.0;
                for (int64_t i = j + tid; i < k; i += kBlock) {
                    const double v = i == j ? 1.0 : A[i * r + j];
#pragma unroll
                    for (int c = 0; c < R; ++c)
                        if (c > j && c < r) w[c] = fma(v, A[i * r + c], w[c]);
                }
                block_sum64<R>(w, red);
                for (int64_t i = j + tid; i < k; i += kBlock) {
                    const double v = i == j ? 1.0 : A[i * r + j];
#pragma unroll
                    for (int c = 0; c < R; ++c)
                        if (c > j && c < r) A[i * r + c] -= tj * v * w[c];
                }
                __syncthreads();
            }
            for (int64_t i = j + 1 + tid; i < k; i += kBlock) A[i * r + j] *= -tj;
            for (int64_t i = tid; i < j; i += kBlock) A[i * r + j] = 0.0;
            if (tid == 0) A[int64_t(j) * r + j] = 1.0 - tj;
            __syncthreads();
        }
        for (int64_t e = tid; e < total; e += kBlock) a.hx[u.off + e] = A[e];
    }
}

// ------------------------------------------------------------------- flat pack ----
__global__ __launch_bounds__(kBlock) void k_flat_pack_f64(FlatArgs a) {
    const FlatItem it = a.items[blockIdx.x];
    const FlatEntry en = a.entries[it.entry];
    double* x = static_cast<double*>(a.tensors[en.tensor]);
    double* f = static_cast<double*>(a.flat) + en.off;
    const int64_t end = it.start + kFlatItem < en.numel ? it.start + kFlatItem : en.numel;
    for (int64_t j = it.start + threadIdx.x; j < end; j += kBlock) {
        const double v = x[j];
        f[j] = a.world != 1 ? v / double(a.world) : v;
        x[j] = 0.0;
    }
}

hipError_t launch_flat_pack_f64(const FlatArgs& a, hipStream_t s) {
    if (a.nitems == 0) return hipSuccess;
    k_flat_pack_f64<<<a.nitems, kBlock, 0, s>>>(a);
    return hipGetLastError();
}

// ------------------------------------------------------------------- launchers ----
#define PSGD_F64_R(KERNEL, GRID, BLOCK, ARG)                      \
    switch (R) {                                                  \
        case 1: KERNEL<1><<<GRID, BLOCK, 0, s>>>(ARG); break;     \
        case 2: KERNEL<2><<<GRID, BLOCK, 0, s>>>(ARG); break;     \
        case 4: KERNEL<4><<<GRID, BLOCK, 0, s>>>(ARG); break;     \
        case 8: KERNEL<8><<<GRID, BLOCK, 0, s>>>(ARG); break;     \
        case 16: KERNEL<16><<<GRID, BLOCK, 0, s>>>(ARG); break;   \
        case 32: KERNEL<32><<<GRID, BLOCK, 0, s>>>(ARG); break;   \
        default: return hipErrorInvalidValue;                     \
    }

hipError_t launch_f64_product(bool even, int R, const F64Args& a, int ntiles, hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    if (even) {
        PSGD_F64_R(k_f64_even, ntiles, kBlock, a)
    } else {
        PSGD_F64_R(k_f64_odd, ntiles, kBlock, a)
    }
    return hipGetLastError();
}

hipError_t launch_f64_reduce(int /*R*/, const F64Args& a, int nitems, hipStream_t s) {
    if (nitems == 0) return hipSuccess;
    k_f64_reduce<<<nitems, 64, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_f64_apply(int R, const F64Args& a, int ntiles, hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    PSGD_F64_R(k_f64_apply, ntiles, kBlock, a)
    return hipGetLastError();
}

hipError_t launch_f64_orth(int R, const F64OrthArgs& a, int nunits, hipStream_t s) {
    if (nunits == 0) return hipSuccess;
    PSGD_F64_R(k_f64_orth, nunits, kBlock, a)
    return hipGetLastError();
}
#undef PSGD_F64_R

}  // namespace psgd
