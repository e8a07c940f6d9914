// Streaming kernels of the PowerSGD hot path, written for CDNA4 (gfx950, wave64).
//
// All three kernels walk the same tiles: a tile is (matrix, column strip, row chunk).
// Inside a 256-thread workgroup every lane OWNS a fixed group of V consecutive columns
// (V = 4 -> 16-byte fp32 / 8-byte bf16 vector loads) and the workgroup's 4 waves x RW row
// phases walk the chunk's rows. Rows are contiguous in HBM, so every wave-instruction
// reads L*V*sizeof(T) contiguous bytes per row (L = lanes per row, up to 64 -> 1 KiB).
// Per-column factor values (Q-layout panels, [m, r]) are kept in registers for the whole
// tile; per-row factor values (P-layout panels, [n, r]) are broadcast loads (one address
// per row group, L1-resident).
//
//   k_product<EVEN>  reference powersgd.py:185-202
//     even: Y[j,:] = sum_i Gk[i,j] X[i,:]   (Q = Gk^T P)   -> per-lane column accumulators,
//           reduced over the workgroup's row phases in LDS -> one partial per row chunk.
//     odd:  Y[i,:] = sum_j Gk[i,j] X[j,:]   (P = Gk Q)     -> per-row dot, reduced across
//           the L lanes of the row -> one partial per column strip.
//     Gk = G0 - sum_{j<k} P_j Q_j^T is formed ON THE FLY from the untouched gradient
//     (same per-element arithmetic as the reference's baddbmm_, :195-202), so the
//     iteration reads the gradient once and writes nothing back.
//   k_apply          reference powersgd.py:195-230 (all iterations at once)
//     residual = G0 - sum_k P_k Q_k^T (local factors)  -> written over the gradient
//     output   = sum_k alpha * P_k Qbar_k^T            -> written to the flat output
//     One read + two writes per element: the only pass that writes the gradient matrix.
//
// Template parameters: T = storage type (float / bf16 bits), R = rank bucket (runtime
// r <= R; c >= r lanes hold zeros), K/NI = number of terms (-1: runtime count, Q-layout
// panels re-read from L1 instead of cached in registers), V = vector width (runtime branch
// per matrix, wave-uniform).
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include "psgd_internal.h"

namespace psgd {

using bf16_t = uint16_t;

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
    return __bfloat16_as_ushort(__float2bfloat16(f));  // RNE, NaN preserving
}

template <typename T>
struct Io;

template <>
struct Io<float> {
    static __device__ __forceinline__ void ld(const float* p, float (&v)[4]) {
        const float4 x = *reinterpret_cast<const float4*>(p);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
    static __device__ __forceinline__ void ld(const float* p, float (&v)[1]) { v[0] = *p; }
    static __device__ __forceinline__ void st(float* p, const float (&v)[4]) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
    static __device__ __forceinline__ void st(float* p, const float (&v)[1]) { *p = v[0]; }
};

template <>
struct Io<bf16_t> {
    static __device__ __forceinline__ void ld(const bf16_t* p, float (&v)[4]) {
        const uint2 x = *reinterpret_cast<const uint2*>(p);
        v[0] = __uint_as_float(x.x << 16);
        v[1] = __uint_as_float(x.x & 0xffff0000u);
        v[2] = __uint_as_float(x.y << 16);
        v[3] = __uint_as_float(x.y & 0xffff0000u);
    }
    static __device__ __forceinline__ void ld(const bf16_t* p, float (&v)[1]) { v[0] = bf2f(*p); }
    static __device__ __forceinline__ void st(bf16_t* p, const float (&v)[4]) {
        uint2 x;
        x.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
        x.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
        *reinterpret_cast<uint2*>(p) = x;
    }
    static __device__ __forceinline__ void st(bf16_t* p, const float (&v)[1]) { *p = f2bf(v[0]); }
};

// r (<= R) consecutive fp32 factor values; zeros for c >= r. When r == R the row start is
// R-aligned (every panel offset is a multiple of r), so R in {2,4,8,...} uses vector loads.
template <int R>
__device__ __forceinline__ void ld_factor(const float* __restrict__ p, int r, float (&v)[R]) {
    if (r == R) {
        if constexpr (R % 4 == 0) {
#pragma unroll
            for (int c = 0; c < R; c += 4) {
                const float4 x = *reinterpret_cast<const float4*>(p + c);
                v[c] = x.x; v[c + 1] = x.y; v[c + 2] = x.z; v[c + 3] = x.w;
            }
        } else if constexpr (R == 2) {
            const float2 x = *reinterpret_cast<const float2*>(p);
            v[0] = x.x; v[1] = x.y;
        } else {
#pragma unroll
            for (int c = 0; c < R; ++c) v[c] = p[c];
        }
    } else {
#pragma unroll
        for (int c = 0; c < R; ++c) v[c] = c < r ? p[c] : 0.f;
    }
}

// sum_c a[c] * b[c] as an fma chain in c order (the order of a rank-r dot in the
// reference's batched GEMM for one output element).
template <int R>
__device__ __forceinline__ float dotr(const float (&a)[R], const float (&b)[R]) {
    float t = a[0] * b[0];
#pragma unroll
    for (int c = 1; c < R; ++c) t = fmaf(a[c], b[c], t);
    return t;
}

struct TileGeom {
    int lane, wave, L, sub, ql;
    int64_t n, m, col0, row_begin, row_end, first_row;
    int stride;
    bool active;
};

template <int V>
__device__ __forceinline__ TileGeom tile_geom(const MatDesc& d, const Tile& t) {
    TileGeom g;
    g.lane = threadIdx.x & 63;
    g.wave = threadIdx.x >> 6;
    g.L = d.lanes;
    const int rw = 64 / g.L;
    g.sub = g.lane / g.L;
    g.ql = g.lane - g.sub * g.L;
    g.n = d.n;
    g.m = d.m;
    g.col0 = (int64_t(t.strip) * g.L + g.ql) * V;
    g.active = g.col0 < g.m;  // V == 4 only when m % 4 == 0: the whole vector is in range
    g.row_begin = int64_t(t.chunk) * d.chunk_rows;
    g.row_end = g.n < g.row_begin + d.chunk_rows ? g.n : g.row_begin + d.chunk_rows;
    g.stride = kWaves * rw;
    g.first_row = g.row_begin + g.wave * rw + g.sub;
    return g;
}

constexpr int kUnroll = 4;  // rows in flight per lane

// ------------------------------------------------------------------ product -------
template <typename T, int R, int K, bool EVEN, int V>
__device__ __forceinline__ void product_tile(const ProductArgs& a, const MatDesc& d, const Tile& t,
                                             float* lds) {
    const TileGeom g = tile_geom<V>(d, t);
    const int r = d.r;
    const T* __restrict__ G = static_cast<const T*>(a.grads[d.tensor]);
    const int nres = K >= 0 ? K : a.nres;
    constexpr int KC = K > 0 ? K : 1;  // register-cached terms

    // Q-layout values at this lane's columns (clamped to a valid column when inactive).
    const int64_t ccol = g.active ? g.col0 : 0;
    float bq[KC][V][R];
    if constexpr (K > 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int v = 0; v < V; ++v) ld_factor<R>(a.res.q[k] + d.qoff + (ccol + v) * r, r, bq[k][v]);
    }
    float xq[EVEN ? 1 : V][R];
    if constexpr (!EVEN) {
#pragma unroll
        for (int v = 0; v < V; ++v) ld_factor<R>(a.x + d.qoff + (ccol + v) * r, r, xq[v]);
    }
    float acc[EVEN ? V : 1][R];
#pragma unroll
    for (int v = 0; v < (EVEN ? V : 1); ++v)
#pragma unroll
        for (int c = 0; c < R; ++c) acc[v][c] = 0.f;

    for (int64_t row = g.first_row; row < g.row_end; row += kUnroll * g.stride) {
        float x[kUnroll][V];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t rr = row + u * g.stride;
            if (g.active && rr < g.row_end) {
                Io<T>::ld(G + rr * g.m + g.col0, x[u]);
            } else {
#pragma unroll
                for (int v = 0; v < V; ++v) x[u][v] = 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t rr = row + u * g.stride;
            const bool valid = g.active && rr < g.row_end;
            const int64_t rc = rr < g.row_end ? rr : g.row_begin;  // clamped for factor loads
            // error feedback of the previous iterations, formed on the fly
            for (int k = 0; k < nres; ++k) {
                float ap[R];
                ld_factor<R>(a.res.p[k] + d.poff + rc * r, r, ap);
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    float b[R];
                    if constexpr (K > 0) {
#pragma unroll
                        for (int c = 0; c < R; ++c) b[c] = bq[k < KC ? k : 0][v][c];
                    } else {
                        ld_factor<R>(a.res.q[k] + d.qoff + (ccol + v) * r, r, b);
                    }
                    x[u][v] = x[u][v] - dotr<R>(ap, b);
                }
            }
            if (!valid) {
#pragma unroll
                for (int v = 0; v < V; ++v) x[u][v] = 0.f;
            }
            if constexpr (EVEN) {
                float xp[R];
                ld_factor<R>(a.x + d.poff + rc * r, r, xp);
#pragma unroll
                for (int v = 0; v < V; ++v)
#pragma unroll
                    for (int c = 0; c < R; ++c) acc[v][c] = fmaf(x[u][v], xp[c], acc[v][c]);
            } else {
                float dot[R];
#pragma unroll
                for (int c = 0; c < R; ++c) {
                    float s = x[u][0] * xq[0][c];
#pragma unroll
                    for (int v = 1; v < V; ++v) s = fmaf(x[u][v], xq[v][c], s);
                    dot[c] = s;
                }
                for (int s = g.L >> 1; s > 0; s >>= 1) {
#pragma unroll
                    for (int c = 0; c < R; ++c) dot[c] += __shfl_xor(dot[c], s);
                }
                if (g.ql == 0 && rr < g.row_end) {
                    float* dst = a.part + d.part_odd + (int64_t(t.strip) * g.n + rr) * r;
#pragma unroll
                    for (int c = 0; c < R; ++c)
                        if (c < r) dst[c] = dot[c];
                }
            }
        }
    }

    if constexpr (EVEN) {
        // reduce the RW row phases inside the wave (lanes ql, ql+L, ...)
        for (int s = g.L; s < 64; s <<= 1) {
#pragma unroll
            for (int v = 0; v < V; ++v)
#pragma unroll
                for (int c = 0; c < R; ++c) acc[v][c] += __shfl_xor(acc[v][c], s);
        }
        const int width = g.L * V * R;  // floats per wave
        if (g.sub == 0) {
#pragma unroll
            for (int v = 0; v < V; ++v)
#pragma unroll
                for (int c = 0; c < R; ++c) lds[g.wave * width + (g.ql * V + v) * R + c] = acc[v][c];
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < width; idx += kBlock) {
            float s = lds[idx];
#pragma unroll
            for (int w = 1; w < kWaves; ++w) s += lds[w * width + idx];
            const int c = idx % R;
            const int64_t col = int64_t(t.strip) * g.L * V + idx / R;
            if (c < r && col < g.m) a.part[d.part_even + (int64_t(t.chunk) * g.m + col) * r + c] = s;
        }
    }
}

template <typename T, int R, int K, bool EVEN>
__global__ __launch_bounds__(kBlock) void k_product(ProductArgs a) {
    // ranks above 8 always take the scalar (V = 1) layout (the plan guarantees d.vec == 0)
    __shared__ float lds[EVEN ? kWaves * 64 * (R <= 8 ? 4 : 1) * R : 1];
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    if constexpr (R <= 8) {
        if (d.vec) {
            product_tile<T, R, K, EVEN, 4>(a, d, t, lds);
            return;
        }
    }
    product_tile<T, R, K, EVEN, 1>(a, d, t, lds);
}

// ------------------------------------------------------------------ apply ---------
template <typename T, int R, int NI, bool SHARED, int V>
__device__ __forceinline__ void apply_tile(const ApplyArgs& a, const MatDesc& d, const Tile& t) {
    const TileGeom g = tile_geom<V>(d, t);
    const int r = d.r;
    T* __restrict__ G = static_cast<T*>(a.grads[d.tensor]);
    T* __restrict__ O = static_cast<T*>(a.out) + d.out_off;
    const int nt = NI > 0 ? NI : a.nterms;
    constexpr int NC = NI > 0 ? NI : 1;
    constexpr int NA = (NI > 0 && !SHARED) ? NI : 1;
    const int64_t ccol = g.active ? g.col0 : 0;

    float bq[NC][V][R];
    float ba[NA][V][R];
    if constexpr (NI > 0) {
#pragma unroll
        for (int k = 0; k < NI; ++k)
#pragma unroll
            for (int v = 0; v < V; ++v) {
                ld_factor<R>(a.res.q[k] + d.qoff + (ccol + v) * r, r, bq[k][v]);
                if constexpr (!SHARED) ld_factor<R>(a.apx.q[k] + d.qoff + (ccol + v) * r, r, ba[k][v]);
            }
    }
    const float alpha = a.alpha;

    for (int64_t row = g.first_row; row < g.row_end; row += kUnroll * g.stride) {
        float x[kUnroll][V];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t rr = row + u * g.stride;
            if (g.active && rr < g.row_end) {
                Io<T>::ld(G + rr * g.m + g.col0, x[u]);
            } else {
#pragma unroll
                for (int v = 0; v < V; ++v) x[u][v] = 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t rr = row + u * g.stride;
            const int64_t rc = rr < g.row_end ? rr : g.row_begin;
            float o[V];
#pragma unroll
            for (int v = 0; v < V; ++v) o[v] = 0.f;
            for (int k = 0; k < nt; ++k) {
                float ap[R];
                ld_factor<R>(a.res.p[k] + d.poff + rc * r, r, ap);
                float aa[R];
                if constexpr (!SHARED) ld_factor<R>(a.apx.p[k] + d.poff + rc * r, r, aa);
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    float b[R];
                    if constexpr (NI > 0) {
#pragma unroll
                        for (int c = 0; c < R; ++c) b[c] = bq[k < NC ? k : 0][v][c];
                    } else {
                        ld_factor<R>(a.res.q[k] + d.qoff + (ccol + v) * r, r, b);
                    }
                    const float tk = dotr<R>(ap, b);
                    x[u][v] = x[u][v] - tk;  // reference :195-202 (alpha = -1)
                    if constexpr (SHARED) {
                        o[v] = o[v] + tk;    // world size 1: Qbar == Q_local, alpha = 1
                    } else {
                        float bb[R];
                        if constexpr (NI > 0) {
#pragma unroll
                            for (int c = 0; c < R; ++c) bb[c] = ba[k < NA ? k : 0][v][c];
                        } else {
                            ld_factor<R>(a.apx.q[k] + d.qoff + (ccol + v) * r, r, bb);
                        }
                        o[v] = o[v] + alpha * dotr<R>(aa, bb);  // reference :211-219
                    }
                }
            }
            if (g.active && rr < g.row_end) {
                Io<T>::st(G + rr * g.m + g.col0, x[u]);
                Io<T>::st(O + rr * g.m + g.col0, o);
            }
        }
    }
}

template <typename T, int R, int NI, bool SHARED>
__global__ __launch_bounds__(kBlock) void k_apply(ApplyArgs a) {
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    if constexpr (R <= 8) {
        if (d.vec) {
            apply_tile<T, R, NI, SHARED, 4>(a, d, t);
            return;
        }
    }
    apply_tile<T, R, NI, SHARED, 1>(a, d, t);
}

// ------------------------------------------------------------------ dispatch ------
template <typename T, int R>
hipError_t dispatch_product_r(bool even, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    const dim3 grid(ntiles), block(kBlock);
    constexpr bool kCache = R <= 8;
    const int K = (kCache && nres <= 3) ? nres : -1;
#define PSGD_P(KK)                                                                       \
    do {                                                                                 \
        if (even)                                                                        \
            k_product<T, R, KK, true><<<grid, block, 0, s>>>(a);                         \
        else                                                                             \
            k_product<T, R, KK, false><<<grid, block, 0, s>>>(a);                        \
    } while (0)
    if constexpr (kCache) {
        switch (K) {
            case 0: PSGD_P(0); break;
            case 1: PSGD_P(1); break;
            case 2: PSGD_P(2); break;
            case 3: PSGD_P(3); break;
            default: PSGD_P(-1); break;
        }
    } else {
        PSGD_P(-1);
    }
#undef PSGD_P
    return hipGetLastError();
}

template <typename T>
hipError_t dispatch_product(int R, bool even, int nres, const ProductArgs& a, int ntiles,
                            hipStream_t s) {
    switch (R) {
        case 1: return dispatch_product_r<T, 1>(even, nres, a, ntiles, s);
        case 2: return dispatch_product_r<T, 2>(even, nres, a, ntiles, s);
        case 4: return dispatch_product_r<T, 4>(even, nres, a, ntiles, s);
        case 8: return dispatch_product_r<T, 8>(even, nres, a, ntiles, s);
        case 16: return dispatch_product_r<T, 16>(even, nres, a, ntiles, s);
        case 32: return dispatch_product_r<T, 32>(even, nres, a, ntiles, s);
        default: return hipErrorInvalidValue;
    }
}

template <typename T, int R>
hipError_t dispatch_apply_r(int nterms, bool shared, const ApplyArgs& a, int ntiles, hipStream_t s) {
    const dim3 grid(ntiles), block(kBlock);
    constexpr bool kCache = R <= 8;
    const int NI = (kCache && nterms <= 4) ? nterms : -1;
#define PSGD_A(NN)                                                                       \
    do {                                                                                 \
        if (shared)                                                                      \
            k_apply<T, R, NN, true><<<grid, block, 0, s>>>(a);                           \
        else                                                                             \
            k_apply<T, R, NN, false><<<grid, block, 0, s>>>(a);                          \
    } while (0)
    if constexpr (kCache) {
        switch (NI) {
            case 1: PSGD_A(1); break;
            case 2: PSGD_A(2); break;
            case 3: PSGD_A(3); break;
            case 4: PSGD_A(4); break;
            default: PSGD_A(-1); break;
        }
    } else {
        PSGD_A(-1);
    }
#undef PSGD_A
    return hipGetLastError();
}

template <typename T>
hipError_t dispatch_apply(int R, int nterms, bool shared, const ApplyArgs& a, int ntiles,
                          hipStream_t s) {
    switch (R) {
        case 1: return dispatch_apply_r<T, 1>(nterms, shared, a, ntiles, s);
        case 2: return dispatch_apply_r<T, 2>(nterms, shared, a, ntiles, s);
        case 4: return dispatch_apply_r<T, 4>(nterms, shared, a, ntiles, s);
        case 8: return dispatch_apply_r<T, 8>(nterms, shared, a, ntiles, s);
        case 16: return dispatch_apply_r<T, 16>(nterms, shared, a, ntiles, s);
        case 32: return dispatch_apply_r<T, 32>(nterms, shared, a, ntiles, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace psgd
