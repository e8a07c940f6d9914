// Small-panel kernels: orthonormalisation of the in-factor, deterministic reduction of the
// product partials, and the flat pack of uncompressed tensors.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "psgd_internal.h"
#include "psgd_stream.cuh"
#include "psgd_chain.cuh"

namespace psgd {

// Diagnostic-only phase stamps (tools/orth_stamps.hip builds this file with PSGD_STAMPS;
// the library build never executes a stamp).
#ifdef PSGD_STAMPS
__device__ unsigned long long g_stamps[64];
#define PSGD_STAMP(i)                                                                         \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        unsigned long long t_;                                                                \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        if (threadIdx.x == 0 && blockIdx.x == 0) g_stamps[i] = t_;                            \
        __builtin_amdgcn_sched_barrier(0);                                                    \
    } while (0)
#else
#define PSGD_STAMP(i) \
    do {              \
    } while (0)
#endif

// Sum NV floats over a workgroup of NW waves; result in every thread. `red` holds
// 2 * NW * SLOT floats (double-buffered by `phase`, so one barrier per call suffices).
// SLOT is the largest NV the kernel sums: the two buffers sit at fixed offsets, so calls
// of different widths never overlap the buffer the previous call is still being read from.
template <int NV, int NW, int SLOT>
__device__ __forceinline__ void wg_sum(float (&v)[NV], float* red, int& phase) {
    static_assert(NV <= SLOT, "wg_sum: NV exceeds the buffer slot");
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_allsum(v[i]);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float* buf = red + phase * NW * SLOT;
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) buf[wave * NV + i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        float s = buf[i];
#pragma unroll
        for (int w = 1; w < NW; ++w) s += buf[w * NV + i];
        v[i] = s;
    }
    phase ^= 1;
}

// ---------------------------------------------------------------- block reductions
template <typename A, int NV>
__device__ __forceinline__ void block_sum(A (&v)[NV], A* red) {
    // red: LDS scratch of kWaves * NV elements; result broadcast to every thread's v
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
        A s = red[i];
        for (int w = 1; w < kWaves; ++w) s += red[w * NV + i];
        v[i] = s;
    }
}

// ---------------------------------------------------------------- orthonormalise
// reference powersgd/orthogonalization.py:4-8.
//   rank 1 : x /= max(||x||_F over the WHOLE shape group, 1e-16)
//   rank>1 : x = Q of the Householder QR of each [k, r] panel — LAPACK geqr2 + org2r
//            conventions (beta = -sign(alpha)*||col||, tau = 0 for an all-zero column,
//            so a zero panel yields the leading identity columns, as torch.linalg.qr does).
// The panel is staged in LDS when it fits, else worked on in place in the history buffer.
template <int R>
__global__ __launch_bounds__(kBlock) void k_orth(OrthArgs a, int64_t lds_floats) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __shared__ double redd[kWaves];
    __shared__ float red[kWaves * (R > 1 ? R : 1)];
    __shared__ float tau[(R + 3) / 4 * 4];  // keep the static LDS a multiple of 16 bytes
    const OrthUnit u = a.units[blockIdx.x];
    float* st = a.state + u.off;
    float* hx = a.hx + u.off;
    const int64_t total = u.k * u.r * u.count;
    const int tid = threadIdx.x;
    if (a.save) {
        float* sv = a.save + u.off;
        for (int64_t i = tid; i < total; i += kBlock) sv[i] = st[i];
    }
    if (u.r == 1) {
        double s[1] = {0.0};
        for (int64_t i = tid; i < total; i += kBlock) {
            const double x = st[i];
            s[0] += x * x;
        }
        block_sum<double, 1>(s, redd);
        const float nrm = float(sqrt(s[0]));
        const float d = nrm > 1e-16f ? nrm : 1e-16f;  // torch.maximum(norm, eps)
        for (int64_t i = tid; i < total; i += kBlock) {
            const float x = st[i] / d;
            st[i] = x;
            hx[i] = x;
        }
        return;
    }
    if constexpr (R > 1) {
        const bool in_lds = total <= lds_floats;
        float* A = in_lds ? smem : hx;
        for (int64_t i = tid; i < total; i += kBlock) A[i] = st[i];
        __syncthreads();
        householder_q<R>(A, u.k, u.r, red, tau);
        for (int64_t i = tid; i < total; i += kBlock) {
            const float x = A[i];
            st[i] = x;
            if (in_lds) hx[i] = x;
        }
    }
}

// ----------------------------------------------------------- fast orthonormalise
constexpr int kOrthThreads = 1024;
constexpr int kOrthWaves = kOrthThreads / 64;

// rank 1: x /= max(||x||, 1e-16) over the whole shape group (two streaming passes, the
// second one from L2). Optionally saves the pre-normalisation values.
template <int NT = kOrthThreads>
__device__ void orth_joint_norm(const OrthArgs& a, const OrthUnit& u, double* rd) {
    float* __restrict__ st = a.state + u.off;
    float* __restrict__ hx = a.hx + u.off;
    float* __restrict__ sv = a.save ? a.save + u.off : nullptr;
    const int64_t total = u.k * u.count;
    const int tid = threadIdx.x;
    constexpr int U = 8;
    float part = 0.f;
    // a group of at most U1 * NT values (every rank-1 group of cfg2 at W > 1): all loads in
    // one round trip, no second pass; the per-thread order of the sums is the batched loop's
    constexpr int U1 = 16;
    if (total <= int64_t(U1) * NT) {
        float x[U1];
#pragma unroll
        for (int q = 0; q < U1; ++q) {  // unconditional loads from clamped indices (no branches)
            const int64_t i = tid + int64_t(q) * NT;
            x[q] = st[i < total ? i : 0];
        }
#pragma unroll
        for (int q = 0; q < U1; ++q) {
            const int64_t i = tid + int64_t(q) * NT;
            keep(x[q]);
            x[q] = i < total ? x[q] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < U1; ++q) part = fmaf(x[q], x[q], part);
        double s = wave_allsum(part);
        if ((tid & 63) == 0) rd[tid >> 6] = s;
        __syncthreads();
        s = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += rd[w];
        const float nrm = float(sqrt(s));
        const float d = nrm > 1e-16f ? nrm : 1e-16f;
        if (a.rfac)
            for (int c = tid; c < u.count; c += NT) a.rfac[u.off + int64_t(c) * u.k] = d;
#pragma unroll
        for (int q = 0; q < U1; ++q) {
            const int64_t i = tid + int64_t(q) * NT;
            if (i < total) {
                if (sv) sv[i] = x[q];
                const float y = x[q] / d;
                st[i] = y;
                hx[i] = y;
            }
        }
        return;
    }
    for (int64_t base = tid; base < total; base += int64_t(U) * NT) {
        float x[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {  // unconditional loads from clamped indices (no branches)
            const int64_t i = base + int64_t(q) * NT;
            x[q] = st[i < total ? i : 0];
        }
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int64_t i = base + int64_t(q) * NT;
            keep(x[q]);
            x[q] = i < total ? x[q] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < U; ++q) part = fmaf(x[q], x[q], part);
    }
    // block sum in double (wave partials in fp32 are exact enough: <= 64 * U terms each)
    double s = wave_allsum(part);
    if ((tid & 63) == 0) rd[tid >> 6] = s;
    __syncthreads();
    s = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += rd[w];
    const float nrm = float(sqrt(s));
    const float d = nrm > 1e-16f ? nrm : 1e-16f;  // torch.maximum(norm, eps)
    if (a.rfac)  // x = (x / d) d: R' = d for every panel of the group
        for (int c = tid; c < u.count; c += NT) a.rfac[u.off + int64_t(c) * u.k] = d;
    for (int64_t base = tid; base < total; base += int64_t(U) * NT) {
        float x[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int64_t i = base + int64_t(q) * NT;
            x[q] = st[i < total ? i : 0];
        }
#pragma unroll
        for (int q = 0; q < U; ++q) keep(x[q]);
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int64_t i = base + int64_t(q) * NT;
            if (i < total) {
                if (sv) sv[i] = x[q];
                const float y = x[q] / d;
                st[i] = y;
                hx[i] = y;
            }
        }
    }
}

// rank > 1: the k x r panel lives in registers (thread t owns rows t + 1024 q, q < RPT);
// LAPACK geqr2 + org2r as 3r - 1 workgroup reductions.
template <int R, int RPT>
__global__ __launch_bounds__(kOrthThreads) void k_orth_reg(OrthArgs a) {
    constexpr int kSlot = R > 2 ? R : 2;  // widest wg_sum below
    __shared__ __attribute__((aligned(16))) float red[2 * kOrthWaves * kSlot];
    const OrthUnit u = a.units[blockIdx.x];
    if (u.r == 1) {
        orth_joint_norm(a, u, reinterpret_cast<double*>(red));
        return;
    }
    if constexpr (R > 1) {
        PSGD_STAMP(0);
        const int r = u.r;
        const int64_t k = u.k;
        const int tid = threadIdx.x;
        float* __restrict__ st = a.state + u.off;
        float* __restrict__ sv = a.save ? a.save + u.off : nullptr;
        float A[RPT][R];
        // every load first (all in flight together), then the save-copy stores
#pragma unroll
        for (int q = 0; q < RPT; ++q) {  // unconditional loads from clamped indices (no branches)
            const int64_t i = tid + int64_t(q) * kOrthThreads;
            const int64_t ic = i < k ? i : 0;
#pragma unroll
            for (int c = 0; c < R; ++c) A[q][c] = st[ic * r + (c < r ? c : 0)];
        }
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int64_t i = tid + int64_t(q) * kOrthThreads;
#pragma unroll
            for (int c = 0; c < R; ++c) {
                keep(A[q][c]);
                A[q][c] = (i < k && c < r) ? A[q][c] : 0.f;
            }
        }
        if (sv) {
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int64_t i = tid + int64_t(q) * kOrthThreads;
                if (i < k) {
#pragma unroll
                    for (int c = 0; c < R; ++c)
                        if (c < r) sv[i * r + c] = A[q][c];
                }
            }
        }
        PSGD_STAMP(1);
        int phase = 0;
        float tau[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            tau[j] = 0.f;
            if (j >= r) continue;
            PSGD_STAMP(2 + 2 * j);
            float v2[2] = {0.f, 0.f};  // sum_{i>j} A[i][j]^2, alpha = A[j][j]
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int64_t i = tid + int64_t(q) * kOrthThreads;
                const float x = A[q][j];
                if (i > j && i < k) v2[0] = fmaf(x, x, v2[0]);
                if (i == j) v2[1] = x;
            }
            wg_sum<2, kOrthWaves, kSlot>(v2, red, phase);
            PSGD_STAMP(3 + 2 * j);
            const float alpha = v2[1];
            float tj = 0.f;
            if (v2[0] != 0.f) {
                const float beta = -copysignf(hypotf(alpha, sqrtf(v2[0])), alpha);
                tj = (beta - alpha) / beta;
                const float scal = 1.f / (alpha - beta);
#pragma unroll
                for (int q = 0; q < RPT; ++q) {
                    const int64_t i = tid + int64_t(q) * kOrthThreads;
                    if (i > j && i < k) A[q][j] *= scal;
                    if (i == j) A[q][j] = beta;
                }
            }
            tau[j] = tj;
            if (tj != 0.f && j + 1 < r) {  // apply H_j to A[j:, j+1:]
                float w[R];
#pragma unroll
                for (int c = 0; c < R; ++c) w[c] = 0.f;
#pragma unroll
                for (int q = 0; q < RPT; ++q) {
                    const int64_t i = tid + int64_t(q) * kOrthThreads;
                    const float vi = i == j ? 1.f : ((i > j && i < k) ? A[q][j] : 0.f);
#pragma unroll
                    for (int c = j + 1; c < R; ++c) w[c] = fmaf(vi, A[q][c], w[c]);
                }
                wg_sum<R, kOrthWaves, kSlot>(w, red, phase);
#pragma unroll
                for (int q = 0; q < RPT; ++q) {
                    const int64_t i = tid + int64_t(q) * kOrthThreads;
                    const float vi = i == j ? 1.f : ((i > j && i < k) ? A[q][j] : 0.f);
#pragma unroll
                    for (int c = j + 1; c < R; ++c) A[q][c] -= tj * vi * w[c];
                }
            }
        }
        PSGD_STAMP(40);
        // org2r: Q = H_0 ... H_{r-1} I[:, :r]
#pragma unroll
        for (int j = R - 1; j >= 0; --j) {
            if (j >= r) continue;
            const float tj = tau[j];
            if (j + 1 < r && tj != 0.f) {
                float w[R];
#pragma unroll
                for (int c = 0; c < R; ++c) w[c] = 0.f;
#pragma unroll
                for (int q = 0; q < RPT; ++q) {
                    const int64_t i = tid + int64_t(q) * kOrthThreads;
                    const float vi = i == j ? 1.f : ((i > j && i < k) ? A[q][j] : 0.f);
#pragma unroll
                    for (int c = j + 1; c < R; ++c) w[c] = fmaf(vi, A[q][c], w[c]);
                }
                wg_sum<R, kOrthWaves, kSlot>(w, red, phase);
#pragma unroll
                for (int q = 0; q < RPT; ++q) {
                    const int64_t i = tid + int64_t(q) * kOrthThreads;
                    const float vi = i == j ? 1.f : ((i > j && i < k) ? A[q][j] : 0.f);
#pragma unroll
                    for (int c = j + 1; c < R; ++c) A[q][c] -= tj * vi * w[c];
                }
            }
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int64_t i = tid + int64_t(q) * kOrthThreads;
                if (i > j && i < k) A[q][j] *= -tj;
                else if (i == j) A[q][j] = 1.f - tj;
                else if (i < j) A[q][j] = 0.f;
            }
        }
        PSGD_STAMP(41);
        float* __restrict__ hx = a.hx + u.off;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int64_t i = tid + int64_t(q) * kOrthThreads;
            if (i < k) {
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c < r) {
                        st[i * r + c] = A[q][c];
                        hx[i * r + c] = A[q][c];
                    }
            }
        }
        PSGD_STAMP(42);
    }
}

// ------------------------------------------------- WY-form Householder (fast path) ----
// LAPACK geqr2 + org2r semantics with two latency cuts (stamps: each workgroup reduction
// costs ~1k cycles, the arithmetic is negligible):
//  * per column j ONE reduction gathers ||A[j+1:, j]||^2, alpha = A[j][j], the dots
//    d_c = A[j+1:, j] . A[j+1:, c] and A[j][c] (c > j): w_c = A[j][c] + scal * d_c is the
//    same quantity as LAPACK's slarf w = v^T C with v = [1; scal * A[j+1:, j]];
//  * Q = H_0 ... H_{r-1} [I; 0] = [I; 0] - V T V1^T (compact WY, LAPACK slarft: T upper
//    triangular from tau and V^T V), i.e. ONE more reduction instead of r - 1 in org2r.
// NW = waves per panel: NW = 1 -> one wave per panel (4 panels per 256-thread workgroup,
// no barriers); NW = 4/8/16 -> the whole workgroup of 64*NW threads works on one panel
// (rows tid + 64*NW*q, cross-wave sums through LDS). More waves per panel means fewer rows
// per wave and several waves per SIMD to hide each other's latency.
template <int NV, int NW, int SLOT>
__device__ __forceinline__ void grp_sum(float (&v)[NV], float* red, int& phase) {
    static_assert(NV <= SLOT, "grp_sum: NV exceeds the buffer slot");
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_allsum(v[i]);
    if constexpr (NW > 1) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        float* buf = red + phase * (NW + 1) * SLOT;
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < NV; ++i) buf[wave * NV + i] = v[i];
        }
        __syncthreads();
        if constexpr (NW * NV <= 64) {  // few partials: every thread adds them itself
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                float sum = buf[i];
#pragma unroll
                for (int w = 1; w < NW; ++w) sum += buf[w * NV + i];
                v[i] = sum;
            }
        } else {  // thread i adds partial i over the waves (same order), then all read
            if (threadIdx.x < NV) {
                float sum = buf[threadIdx.x];
#pragma unroll
                for (int w = 1; w < NW; ++w) sum += buf[w * NV + threadIdx.x];
                buf[NW * NV + threadIdx.x] = sum;
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = buf[NW * NV + i];
        }
        phase ^= 1;
    }
}

// rank-1 unit handled by the NW waves of its panel group
template <int NW>
__device__ void joint_norm_grp(const OrthArgs& a, const OrthUnit& u, float* red) {
    constexpr int NT = 64 * NW;
    const int t = NW == 1 ? (threadIdx.x & 63) : threadIdx.x;
    float* __restrict__ st = a.state + u.off;
    float* __restrict__ hx = a.hx + u.off;
    float* __restrict__ sv = a.save ? a.save + u.off : nullptr;
    const int64_t total = u.k * u.count;
    constexpr int U = 8;
    float part[1] = {0.f};
    for (int64_t base = t; base < total; base += int64_t(U) * NT) {
        float x[U];
#pragma unroll
        for (int q = 0; q < U; ++q) x[q] = st[base + q * NT < total ? base + q * NT : 0];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            keep(x[q]);
            part[0] = fmaf(base + q * NT < total ? x[q] : 0.f, base + q * NT < total ? x[q] : 0.f, part[0]);
        }
    }
    int phase = 0;
    grp_sum<1, NW, 1>(part, red, phase);
    const float nrm = sqrtf(part[0]);
    const float d = nrm > 1e-16f ? nrm : 1e-16f;  // torch.maximum(norm, eps)
    for (int64_t base = t; base < total; base += int64_t(U) * NT) {
        float x[U];
#pragma unroll
        for (int q = 0; q < U; ++q) x[q] = st[base + q * NT < total ? base + q * NT : 0];
#pragma unroll
        for (int q = 0; q < U; ++q) keep(x[q]);
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int64_t i = base + q * NT;
            if (i < total) {
                if (sv) sv[i] = x[q];
                const float y = x[q] / d;
                st[i] = y;
                hx[i] = y;
            }
        }
    }
}


template <int R, int RPT, int NW>
__global__ __launch_bounds__(NW == 1 ? kBlock : 64 * NW) void k_orth_wy(OrthArgs a, int nunits) {
    constexpr int kRed = (2 * R + 2) > (2 * R * R) ? (2 * R + 2) : (2 * R * R);  // largest sum
    __shared__ __attribute__((aligned(16))) float red[2 * (NW + 1) * kRed];
    constexpr int NT = 64 * NW;  // threads per panel
    const int unit = NW == 1 ? blockIdx.x * kWaves + (threadIdx.x >> 6) : blockIdx.x;
    if (unit >= nunits) return;  // NW == 1 only: whole waves leave, no barrier follows
    const OrthUnit u = a.units[unit];
    if (u.r == 1) {
        joint_norm_grp<NW>(a, u, red);
        return;
    }
    PSGD_STAMP(0);
    const int r = u.r;
    const int k = int(u.k);
    const int t = NW == 1 ? (threadIdx.x & 63) : threadIdx.x;
    const int nq = (k + NT - 1) / NT;  // row slots in use (uniform); slot q holds row t + q*NT
    float* __restrict__ st = a.state + u.off;
    float* __restrict__ sv = a.save ? a.save + u.off : nullptr;
    // Rows >= k are zero, so they add nothing to any sum and stay zero under every update;
    // rows in slots q >= 1 are >= NT > R, i.e. strictly below every diagonal element: only
    // slot 0 needs the diagonal cases (i == j / i < j).
    float A[RPT][R];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {  // whole rows, from clamped (always valid) row indices
        const int i = t + q * NT;
        ld_row<R>(st + int64_t(i < k ? i : 0) * r, r, A[q]);
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const int i = t + q * NT;
#pragma unroll
        for (int c = 0; c < R; ++c) {
            keep(A[q][c]);
            A[q][c] = i < k ? A[q][c] : 0.f;
        }
    }
    if (sv) {
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int i = t + q * NT;
            if (q < nq && i < k) st_row<R>(sv + int64_t(i) * r, r, A[q]);
        }
    }
    PSGD_STAMP(1);
    int phase = 0;
    float tau[R];
    // ---- geqr2: A <- R (rows < r) and V (strictly below the diagonal, unit diagonal implied)
#pragma unroll
    for (int j = 0; j < R; ++j) {
        tau[j] = 0.f;
        if (j >= r) continue;
        // v[0] = sum_{i>j} A[i][j]^2, v[1] = alpha, v[2+c] = d_c (c > j), v[2+R+c] = A[j][c] (c > j)
        float v[2 + 2 * R];
#pragma unroll
        for (int e = 0; e < 2 + 2 * R; ++e) v[e] = 0.f;
        {
            const float x = A[0][j];
            const float xb = t > j ? x : 0.f;
            v[0] = xb * xb;
            v[1] = t == j ? x : 0.f;
#pragma unroll
            for (int c = j + 1; c < R; ++c) {
                v[2 + c] = xb * A[0][c];
                v[2 + R + c] = t == j ? A[0][c] : 0.f;
            }
        }
#pragma unroll
        for (int q = 1; q < RPT; ++q) {
            if (q < nq) {  // uniform: unused row slots do nothing
                const float x = A[q][j];
                v[0] = fmaf(x, x, v[0]);
    #pragma unroll
                for (int c = j + 1; c < R; ++c) v[2 + c] = fmaf(x, A[q][c], v[2 + c]);
            }
        }
        grp_sum<2 + 2 * R, NW, kRed>(v, red, phase);
        const float alpha = v[1];
        if (v[0] != 0.f) {  // LAPACK slarfg: xnorm == 0 -> tau = 0, H_j = I
            const float beta = -copysignf(hypotf(alpha, sqrtf(v[0])), alpha);
            const float tj = (beta - alpha) / beta;
            const float scal = 1.f / (alpha - beta);
            tau[j] = tj;
            float w[R];
#pragma unroll
            for (int c = j + 1; c < R; ++c) w[c] = v[2 + R + c] + scal * v[2 + c];
            {
                const bool below = t > j;
                const float vi = below ? A[0][j] * scal : (t == j ? 1.f : 0.f);
                A[0][j] = below ? vi : (t == j ? beta : A[0][j]);
#pragma unroll
                for (int c = j + 1; c < R; ++c) A[0][c] -= tj * vi * w[c];
            }
#pragma unroll
            for (int q = 1; q < RPT; ++q) {
                if (q < nq) {  // uniform: unused row slots do nothing
                    const float vi = A[q][j] * scal;
                    A[q][j] = vi;
    #pragma unroll
                    for (int c = j + 1; c < R; ++c) A[q][c] -= tj * vi * w[c];
                }
            }
        }
    }
    PSGD_STAMP(40);
    // ---- slarft: T from tau and S = V^T V; V1 = rows 0..r-1 of V, broadcast in the same sum
    float sv2[2 * R * R];  // [0, R*R): S[a][b] (a < b); [R*R, 2R*R): V[row a][col b]
#pragma unroll
    for (int e = 0; e < 2 * R * R; ++e) sv2[e] = 0.f;
    {
        float vr[R];  // row t of V (slot 0 holds the diagonal cases)
#pragma unroll
        for (int c = 0; c < R; ++c) vr[c] = (c < r) ? (t == c ? 1.f : (t > c ? A[0][c] : 0.f)) : 0.f;
#pragma unroll
        for (int a2 = 0; a2 < R; ++a2)
#pragma unroll
            for (int b = a2 + 1; b < R; ++b) sv2[a2 * R + b] = vr[a2] * vr[b];
#pragma unroll
        for (int a2 = 0; a2 < R; ++a2)
#pragma unroll
            for (int b = 0; b < R; ++b) sv2[R * R + a2 * R + b] = t == a2 ? vr[b] : 0.f;
    }
#pragma unroll
    for (int q = 1; q < RPT; ++q) {
        if (q < nq) {  // uniform: unused row slots do nothing
    #pragma unroll
            for (int a2 = 0; a2 < R; ++a2)
    #pragma unroll
                for (int b = a2 + 1; b < R; ++b) sv2[a2 * R + b] = fmaf(A[q][a2], A[q][b], sv2[a2 * R + b]);
        }
    }
    grp_sum<2 * R * R, NW, kRed>(sv2, red, phase);
    float T[R][R];
#pragma unroll
    for (int a2 = 0; a2 < R; ++a2)
#pragma unroll
        for (int b = 0; b < R; ++b) T[a2][b] = 0.f;
#pragma unroll
    for (int j = 0; j < R; ++j) {
        if (j >= r) continue;
        // T[0:j, j] = -tau_j * T[0:j, 0:j] * S[0:j, j];  T[j][j] = tau_j
        float y[R];
#pragma unroll
        for (int a2 = 0; a2 < R; ++a2) y[a2] = a2 < j ? -tau[j] * sv2[a2 * R + j] : 0.f;
#pragma unroll
        for (int a2 = 0; a2 < R; ++a2) {
            if (a2 >= j) continue;
            float acc = 0.f;
#pragma unroll
            for (int b = 0; b < R; ++b)
                if (b >= a2 && b < j) acc = fmaf(T[a2][b], y[b], acc);
            T[a2][j] = acc;
        }
        T[j][j] = tau[j];
    }
    // M = T V1^T  (r x r):  M[l][c] = sum_b T[l][b] * V[c][b]
    float M[R][R];
#pragma unroll
    for (int l = 0; l < R; ++l)
#pragma unroll
        for (int c = 0; c < R; ++c) {
            float acc = 0.f;
#pragma unroll
            for (int b = 0; b < R; ++b) acc = fmaf(T[l][b], sv2[R * R + c * R + b], acc);
            M[l][c] = acc;
        }
    // Q[i][c] = [i == c] - sum_l V[i][l] * M[l][c]
    float* __restrict__ hx = a.hx + u.off;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        if (q < nq) {  // uniform: unused row slots do nothing
            const int i = t + q * NT;
            float vr[R];
    #pragma unroll
            for (int c = 0; c < R; ++c) {
                if (q == 0)
                    vr[c] = (c < r) ? (i == c ? 1.f : (i > c ? A[0][c] : 0.f)) : 0.f;
                else
                    vr[c] = A[q][c];  // c >= r columns are zero
            }
            float qrow[R];
    #pragma unroll
            for (int c = 0; c < R; ++c) {
                float acc = 0.f;
    #pragma unroll
                for (int l = 0; l < R; ++l) acc = fmaf(vr[l], M[l][c], acc);
                qrow[c] = (i == c ? 1.f : 0.f) - acc;
            }
            if (i < k) {
                st_row<R>(st + int64_t(i) * r, r, qrow);
                st_row<R>(hx + int64_t(i) * r, r, qrow);
            }
        }
    }
    PSGD_STAMP(42);
}

// register budget of the WY kernel (checked with -Rpass-analysis=kernel-resource-usage:
// no spills for these pairs at the launch bounds used)
__host__ __device__ constexpr bool orth_wy_ok(int R, int RPT) {
    return R <= 4 ? R * RPT <= 32 : R * RPT <= 16;
}

template <int R, int RPT, int NW>
void launch_orth_wy_one(const OrthArgs& a, int nunits, hipStream_t s) {
    if constexpr (orth_wy_ok(R, RPT) && !(R == 8 && NW == 16)) {  // R=8 x 1024 threads spills
        const int blocks = NW == 1 ? (nunits + kWaves - 1) / kWaves : nunits;
        k_orth_wy<R, RPT, NW><<<blocks, NW == 1 ? kBlock : 64 * NW, 0, s>>>(a, nunits);
    }
}

template <int R, int NW>
hipError_t launch_orth_wy_r(int rpt, const OrthArgs& a, int nunits, hipStream_t s) {
    switch (rpt) {
        case 1: launch_orth_wy_one<R, 1, NW>(a, nunits, s); break;
        case 2: launch_orth_wy_one<R, 2, NW>(a, nunits, s); break;
        case 4: launch_orth_wy_one<R, 4, NW>(a, nunits, s); break;
        case 8: launch_orth_wy_one<R, 8, NW>(a, nunits, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int R>
hipError_t launch_orth_wy_nw(int nw, int rpt, const OrthArgs& a, int nunits, hipStream_t s) {
    switch (nw) {
        case 1: return launch_orth_wy_r<R, 1>(rpt, a, nunits, s);
        case 4: return launch_orth_wy_r<R, 4>(rpt, a, nunits, s);
        case 8: return launch_orth_wy_r<R, 8>(rpt, a, nunits, s);
        default: return launch_orth_wy_r<R, 16>(rpt, a, nunits, s);
    }
}

// Picks the fast WY kernel when the panel slice fits in registers; returns false otherwise.
// Waves per panel: as few as keep every wave at <= 8 rows (1 wave up to 512 rows ... 16 waves
// up to 8192 rows).
bool launch_orth_wy(const OrthArgs& a, int nunits, int R, int64_t kmax, hipStream_t s, hipError_t* err) {
    if (R < 2 || R > 8) return false;
    const int nw_max = R == 8 ? 8 : 16;  // R = 8 needs > 128 VGPRs: no 1024-thread groups
    int nw = 1;
    while (nw < nw_max && int64_t(64) * nw * 8 < kmax) nw = nw == 1 ? 4 : nw * 2;
    int64_t rpt = 1;
    while (rpt * 64 * nw < kmax) rpt <<= 1;
    if (rpt > 8 || !orth_wy_ok(R, int(rpt))) return false;
    *err = R == 2 ? launch_orth_wy_nw<2>(nw, int(rpt), a, nunits, s)
         : R == 4 ? launch_orth_wy_nw<4>(nw, int(rpt), a, nunits, s)
                  : launch_orth_wy_nw<8>(nw, int(rpt), a, nunits, s);
    return true;
}

// Register budget: 1024-thread workgroups get at most 128 VGPRs, so the panel slice a
// thread holds is capped at kOrthRegFloats floats (no spills for any instantiated pair).
// (checked with -Rpass-analysis=kernel-resource-usage: ranks 16/32 spill, so they take the
// LDS kernel above).
__host__ __device__ constexpr bool orth_reg_ok(int R, int RPT) {
    return R == 1 || (R <= 4 && R * RPT <= 32) || (R == 8 && RPT <= 2);
}

template <int R, int RPT>
void launch_orth_reg_one(const OrthArgs& a, int nunits, hipStream_t s) {
    if constexpr (orth_reg_ok(R, RPT)) k_orth_reg<R, RPT><<<nunits, kOrthThreads, 0, s>>>(a);
}

template <int R>
hipError_t launch_orth_reg_r(int rpt, const OrthArgs& a, int nunits, hipStream_t s) {
    switch (rpt) {
        case 1: launch_orth_reg_one<R, 1>(a, nunits, s); break;
        case 2: launch_orth_reg_one<R, 2>(a, nunits, s); break;
        case 4: launch_orth_reg_one<R, 4>(a, nunits, s); break;
        case 8: launch_orth_reg_one<R, 8>(a, nunits, s); break;
        case 16: launch_orth_reg_one<R, 16>(a, nunits, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_orth_r(int R, const OrthArgs& a, int nunits, int64_t lds_floats, hipStream_t s) {
    const size_t bytes = size_t(lds_floats) * sizeof(float);
    switch (R) {
        case 1: k_orth<1><<<nunits, kBlock, 0, s>>>(a, 0); break;
        case 2: k_orth<2><<<nunits, kBlock, bytes, s>>>(a, lds_floats); break;
        case 4: k_orth<4><<<nunits, kBlock, bytes, s>>>(a, lds_floats); break;
        case 8: k_orth<8><<<nunits, kBlock, bytes, s>>>(a, lds_floats); break;
        case 16: k_orth<16><<<nunits, kBlock, bytes, s>>>(a, lds_floats); break;
        case 32: k_orth<32><<<nunits, kBlock, bytes, s>>>(a, lds_floats); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

static bool env_orth_wy() {
    static const bool on = [] {
        const char* v = std::getenv("PSGD_ORTH_WY");
        return !(v && v[0] == '0');
    }();
    return on;
}


// ------------------------------------------- Cholesky QR with LAPACK signs (fast path) ----
// Q of the Householder QR of a k x r panel X (reference orthogonalization.py:8,
// torch.linalg.qr) computed as Q = X R^-1 D:
//   * Gram G = X^T X accumulated in fp64 (one pass over the panel, ONE workgroup
//     reduction) and its Cholesky factor R (fp64, every thread redundantly);
//   * D = the column signs LAPACK's geqr2 gives (beta = -sign(alpha) ||x||, and beta =
//     alpha for a reflector with nothing below the diagonal): read off the top r x r block
//     of X R^-1 by the LU recursion of Ballard et al., "Reconstructing Householder vectors
//     from Tall-Skinny QR" (s_j = -sign(pivot_j); last column of a square panel: +sign);
//   * Q = X (R^-1 D) row by row (fp64, rounded once to fp32).
// With the Gram in fp64, the loss of orthogonality is ~kappa^2 * 1e-16: below fp32
// rounding for kappa < 1e4. A panel with a pivot under 1e-8 of its column's squared norm
// (kappa >~ 1e4, a zero or rank-deficient panel) takes the exact Householder path instead
// (householder_q above, in place in the history buffer), so zero panels still give the
// leading identity columns. One workgroup per panel, no register-resident panel: the
// second pass re-reads it from L2.
template <int NV, int NW>
__device__ __forceinline__ void block_sum_f64(double (&v)[NV], double* red) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_allsum_f64(v[i]);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) red[wave * NV + i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        double t = red[i];
        for (int w = 1; w < NW; ++w) t += red[w * NV + i];
        v[i] = t;
    }
}

// NT threads per panel: 512 for r <= 4 (a 4096-row panel is one batch of loads per pass;
// the kernel is latency-bound, one workgroup per panel), 256 for r = 8 (registers).
template <int R>
struct CholNT {
    static constexpr int value = R <= 4 ? 512 : 256;
};

// RC = R: the panel has exactly R columns (compile-time rank: the r x r arithmetic is
// branch-free straight-line fp64 that the compiler interleaves; it is a serial latency
// chain per workgroup, so this matters); RC = 0: any r <= R at run time.
// rows per thread per load batch of k_orth_chol (ranks 2 / 4). Larger batches (fewer round
// trips on long panels) measured slower: 16 / 12 rows, k_orth_chol<2> 8.5 -> 9.5 us (cfg4),
// <4> 6.3 -> 6.8 us (profiles/r04/t); likewise the whole panel held in registers (r04/l)
#ifndef PSGD_CHOL_U2
#define PSGD_CHOL_U2 8
#endif
// panels of one load batch keep their rows in registers for the second pass (no L2 re-read):
// rank 4 only (k_orth_chol<4> 6.48 -> 6.26 us on cfg3's P panels; rank 2 +0.3 us on cfg4's,
// profiles/r05/orth)
#ifndef PSGD_CHOL_RES
#define PSGD_CHOL_RES 1
#endif
#ifndef PSGD_CHOL_U4
#define PSGD_CHOL_U4 8
#endif

// Gram sums through LDS (NT x NG fp64 partials: 40 KB at rank 4) for r <= 4
template <int R>
constexpr bool kGramLds = R <= 4;

// KU: rows per thread per load batch (0: the PSGD_CHOL_U* default of the rank)
template <int R, int RC, int KU = 0>
__device__ __forceinline__ void orth_chol_panel(const OrthArgs& a, const OrthUnit& u, double* redd, float* red,
                                                float* tau, double* gpart, float* top_sh) {
    constexpr int NG = R * (R + 1) / 2;
    constexpr int NT = CholNT<R>::value;
    const int r = RC > 0 ? RC : u.r;
    const int64_t k = u.k;
    const int tid = threadIdx.x;
    float* __restrict__ st = a.state + u.off;
    float* __restrict__ hx = a.hx + u.off;
    float* __restrict__ sv = a.save ? a.save + u.off : nullptr;

    // rows in batches of kU per thread, all loads of a batch issued together (clamped
    // rows, masked afterwards): the panel was just written by another kernel, so each
    // batch costs one L2/MALL round trip rather than one per row
    constexpr int kU = KU > 0 ? KU : R <= 2 ? PSGD_CHOL_U2 : R <= 4 ? PSGD_CHOL_U4 : 4;
    double g[NG];
#pragma unroll
    for (int e = 0; e < NG; ++e) g[e] = 0.0;
    // PSGD_CHOL_RES: a panel of one batch keeps its rows in registers for the second pass
    constexpr bool kRes = PSGD_CHOL_RES != 0 && (R == 4 || KU > 0);
    const bool res = kRes && k <= int64_t(kU) * NT;
    float xr[kRes ? kU : 1][R];
    for (int64_t i0 = tid; i0 < k; i0 += int64_t(kU) * NT) {
        float x[kU][R];
#pragma unroll
        for (int q = 0; q < kU; ++q) {
            const int64_t i = i0 + int64_t(q) * NT;
            ld_row<R>(st + (i < k ? i : 0) * r, r, x[q]);
        }
#pragma unroll
        for (int q = 0; q < kU; ++q) {
            const int64_t i = i0 + int64_t(q) * NT;
#pragma unroll
            for (int c = 0; c < R; ++c) {
                keep(x[q][c]);
                x[q][c] = i < k ? x[q][c] : 0.f;
            }
            if (sv && i < k) st_row<R>(sv + i * r, r, x[q]);
            if (kGramLds<R> && i < r) {  // the top r rows: the sign recursion's input, from LDS
#pragma unroll
                for (int c = 0; c < R; ++c) top_sh[i * R + c] = x[q][c];
            }
            int e = 0;
#pragma unroll
            for (int c = 0; c < R; ++c)
#pragma unroll
                for (int b = c; b < R; ++b) g[e++] += double(x[q][c]) * double(x[q][b]);
            if constexpr (kRes) {
#pragma unroll
                for (int c = 0; c < R; ++c) xr[q][c] = x[q][c];
            }
        }
    }
    PSGD_STAMP(11);
    if constexpr (kGramLds<R>) {
        // workgroup Gram sums: every thread's NG partials to LDS (entry-major), then wave w
        // sums entries w, w + NW, ... (lane l: threads l, l + 64, ... in order, then the wave
        // tree): at most two fp64 wave reductions per wave instead of NG (the DPP trees of NG
        // fp64 values on every wave were ~40 % of a small panel's kernel time). Fixed order.
        constexpr int NW = NT / 64;
#pragma unroll
        for (int e = 0; e < NG; ++e) gpart[e * NT + tid] = g[e];
        __syncthreads();
        const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
        for (int e0 = 0; e0 < NG; e0 += NW) {
            const int e = e0 + wave;
            if (e < NG) {
                double t = gpart[e * NT + lane];
#pragma unroll
                for (int w = 1; w < NW; ++w) t += gpart[e * NT + w * 64 + lane];
                t = wave_allsum_f64(t);
                if (lane == 0) redd[e] = t;
            }
        }
        __syncthreads();
        if ((tid >> 6) == 0) {
#pragma unroll
            for (int e = 0; e < NG; ++e) g[e] = redd[e];
        }
    } else {
        block_sum_f64<NG, NT / 64>(g, redd);
    }
    PSGD_STAMP(12);

    __shared__ double m_sh[R * R];
    __shared__ int ok_sh;
    if ((tid >> 6) == 0) chol_chain<R>(g, kGramLds<R> ? top_sh : nullptr, st, r, k, m_sh, &ok_sh,
                                       a.rfac ? a.rfac + u.off : nullptr);
    __syncthreads();
    PSGD_STAMP(13);
    if (!ok_sh) {  // exact Householder (geqr2 + org2r) in place in the history buffer
        for (int64_t i = tid; i < k * r; i += NT) hx[i] = st[i];
        __syncthreads();
        householder_q<R, NT>(hx, k, r, red, tau, a.rfac ? a.rfac + u.off : nullptr);
        for (int64_t i = tid; i < k * r; i += NT) st[i] = hx[i];
        return;
    }
    double M[R][R];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int c = 0; c < R; ++c) M[i][c] = m_sh[i * R + c];
    __syncthreads();  // every thread has read the top block before any row is overwritten
    for (int64_t i0 = tid; i0 < k; i0 += int64_t(kU) * NT) {
        float x[kU][R];
        if (kRes && res) {
#pragma unroll
            for (int q = 0; q < kU; ++q)
#pragma unroll
                for (int c = 0; c < R; ++c) x[q][c] = xr[kRes ? q : 0][c];
        } else {
#pragma unroll
            for (int q = 0; q < kU; ++q) {
                const int64_t i = i0 + int64_t(q) * NT;
                ld_row<R>(st + (i < k ? i : 0) * r, r, x[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < kU; ++q) {
            const int64_t i = i0 + int64_t(q) * NT;
#pragma unroll
            for (int c = 0; c < R; ++c) keep(x[q][c]);
            float y[R];
#pragma unroll
            for (int c = 0; c < R; ++c) {
                double v = 0.0;
#pragma unroll
                for (int l = 0; l < R; ++l) v += double(x[q][l]) * M[l][c];
                y[c] = float(v);
            }
            if (i < k) {
                st_row<R>(st + i * r, r, y);
                st_row<R>(hx + i * r, r, y);
            }
        }
    }
}

// KU > 0: load batches of KU rows per thread (the rank-4 instance for panels above one default
// batch: 4608-row Q panels at world size > 1 stay one batch, kept in registers)
template <int R, int KU = 0>
__global__ __launch_bounds__(CholNT<R>::value) void k_orth_chol(OrthArgs a) {
    constexpr int NT = CholNT<R>::value;
    __shared__ double redd[NT / 64 * (R * (R + 1) / 2)];
    __shared__ float red[NT / 64 * R];
    __shared__ float tau[(R + 3) / 4 * 4];
    PSGD_STAMP(9);
    __shared__ double gpart[kGramLds<R> ? NT * (R * (R + 1) / 2) : 1];
    __shared__ float top_sh[R * R];
    const OrthUnit u = a.units[blockIdx.x];
    PSGD_STAMP(10);
    if (u.r == 1)  // rank-1 group of a mixed-rank plan: the reference's joint norm, not QR
        orth_joint_norm<NT>(a, u, redd);
    else if (u.r == R)
        orth_chol_panel<R, R, KU>(a, u, redd, red, tau, gpart, top_sh);
    else
        orth_chol_panel<R, 0, KU>(a, u, redd, red, tau, gpart, top_sh);
    PSGD_STAMP(14);
}

// ------------------------------------------- Cholesky-QR for ranks 9-16 on fp64 MFMA ----
// Same algorithm and LAPACK sign reconstruction as k_orth_chol, restructured for a 16-column
// panel, where per-thread r x r register arrays no longer fit:
//  * Gram G = X^T X with v_mfma_f64_16x16x4_f64: a wave loads 4 rows x 16 columns (lane
//    l = X[row0 + l/16][l%16]); that one value is both the A operand (A[i][kk] = X[kk][i])
//    and the B operand (B[kk][j] = X[kk][j]), so each row is read once and the matrix core
//    forms all 256 products. 16 waves accumulate their own rows; partials summed via LDS in
//    a fixed order (bitwise reproducible).
//  * The 16 x 16 chain (Cholesky, R^-1, the signs' LU recursion on the top block) runs on
//    wave 0 with lane-parallel LDS updates.
//  * Y = X M' (M' = R^-1 D) again on the matrix core, transposed: D[c'][rr] = sum M'[l][c]
//    X[row0+rr][l] with a column permutation c = pi(c'); lane l loads X[row0 + l%16][4(l/16)
//    .. +3] (one 16-B load) and writes Y[row0 + l%16][4(l/16) .. +3].
//  * v_mfma_f64_16x16x4_f64 layouts (cdna_hip_programming.md): A[i][k] in lane i + 16k,
//    B[k][j] in lane j + 16k, D[i][j] in lane j + 16 (i % 4), item i / 4.
// Columns >= r (a narrower matrix in the rank-16 bucket) are zero in X and identity in the
// padded Gram, so they do not disturb the first r columns.
typedef double f64x4_t __attribute__((ext_vector_type(4)));
constexpr int kC16NT = 512;
constexpr int kC16W = kC16NT / 64;

__device__ __forceinline__ void lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// R = 16 or 32: NB = R / 16 column blocks of 16; the Gram is NB (NB + 1) / 2 MFMA blocks
// (upper), the apply NB x NB blocks of four MFMAs.
template <int R>
__device__ __forceinline__ void orth_chol_wide(const OrthArgs& a) {
    constexpr int NB = R / 16;
    constexpr int NBLK = NB * (NB + 1) / 2;
    constexpr int RR = R * R;
    constexpr int PER = RR / 64;  // r x r entries per lane of wave 0
    // per-wave Gram partials; after the wave sum the same storage holds M', T and X's top block
    constexpr int kScratch = (kC16W * NBLK * 256 > 3 * RR) ? kC16W * NBLK * 256 : 3 * RR;
    __shared__ double scratch[kScratch];
    __shared__ double wsh[RR];  // G, then R (upper, row-major)
    __shared__ double gdiag[R];
    __shared__ double rd[kC16W];
    __shared__ float red[kC16W * R];
    __shared__ float tau[R];
    __shared__ int ok_sh;
    double* gsh = scratch;
    double* msh = scratch;           // M' = R^-1 D (row-major M'[l][c])
    double* tsh = scratch + RR;      // top block T = X[0:r] R^-1
    double* xsh = scratch + 2 * RR;  // top block of X
    const OrthUnit u = a.units[blockIdx.x];
    if (u.r == 1) {  // rank-1 group of a mixed-rank plan: the reference's joint norm
        orth_joint_norm<kC16NT>(a, u, rd);
        return;
    }
    const int r = u.r;
    const int64_t k = u.k;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ri = lane & 15, kq = lane >> 4;
    float* __restrict__ st = a.state + u.off;
    float* __restrict__ hx = a.hx + u.off;
    float* __restrict__ sv = a.save ? a.save + u.off : nullptr;

    // ---- Gram: wave w takes row quads w, w + 16, ...; kG quads per batch, loads in flight
    constexpr int kG = NB == 1 ? 12 : 6;
    f64x4_t g[NBLK];
#pragma unroll
    for (int bl = 0; bl < NBLK; ++bl) g[bl] = f64x4_t{0.0, 0.0, 0.0, 0.0};
    const int64_t nq = (k + 3) >> 2;
    for (int64_t q0 = wave; q0 < nq; q0 += int64_t(kG) * kC16W) {
        float v[kG][NB];
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int64_t row = (q0 + int64_t(q) * kC16W) * 4 + kq;
#pragma unroll
            for (int cb = 0; cb < NB; ++cb) {
                const int c = 16 * cb + ri;
                v[q][cb] = st[(row < k ? row : 0) * r + (c < r ? c : 0)];
            }
        }
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int64_t row = (q0 + int64_t(q) * kC16W) * 4 + kq;
#pragma unroll
            for (int cb = 0; cb < NB; ++cb) {
                keep(v[q][cb]);
                const int c = 16 * cb + ri;
                const bool ok = c < r && row < k;
                v[q][cb] = ok ? v[q][cb] : 0.f;
                if (sv && ok) sv[row * r + c] = v[q][cb];
            }
            int bl = 0;
#pragma unroll
            for (int ca = 0; ca < NB; ++ca)
#pragma unroll
                for (int cb = ca; cb < NB; ++cb) {
                    g[bl] = __builtin_amdgcn_mfma_f64_16x16x4f64(double(v[q][ca]), double(v[q][cb]), g[bl], 0, 0, 0);
                    ++bl;
                }
        }
    }
#pragma unroll
    for (int bl = 0; bl < NBLK; ++bl)
#pragma unroll
        for (int e = 0; e < 4; ++e) gsh[(wave * NBLK + bl) * 256 + e * 64 + lane] = g[bl][e];
    __syncthreads();
    for (int t = tid; t < NBLK * 256; t += kC16NT) {  // fixed-order wave sum; f64 D layout
        const int bl = t >> 8, el = t & 255;
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kC16W; ++w) s += gsh[(w * NBLK + bl) * 256 + el];
        int ca = 0, cb = 0, x = bl;  // block index -> (ca <= cb)
        while (x >= NB - ca) { x -= NB - ca; ++ca; }
        cb = ca + x;
        const int e = el >> 6, l = el & 63;
        const int i = 16 * ca + (l >> 4) + 4 * e, j = 16 * cb + (l & 15);
        if (i >= r || j >= r) s = (i == j) ? 1.0 : 0.0;  // identity padding
        wsh[i * R + j] = s;
        if (i == j) gdiag[i] = s;
    }
    __syncthreads();  // gsh is dead from here on (msh / tsh / xsh reuse it)

    if (wave == 0) {
        // top block of X (rows 0..r-1), in flight during the factorisation
        float xt[PER];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = lane + 64 * q, i = e / R, l = e % R;
            xt[q] = st[(i < r ? i : 0) * r + (l < r ? l : 0)];
        }
        // Cholesky G = R^T R (upper R in place), lane-parallel trailing updates
        bool ok = true;
        for (int j = 0; j < R; ++j) {
            lds_fence();
            const double piv = wsh[j * R + j];
            ok = ok && (j >= r || (piv > 1e-8 * gdiag[j] && piv > 0.0));
            const double d = sqrt(piv > 0.0 ? piv : 1.0);
            lds_fence();
            if (lane < R && lane > j) wsh[j * R + lane] = wsh[j * R + lane] / d;
            if (lane == j) wsh[j * R + j] = d;
            lds_fence();
#pragma unroll 4
            for (int q = 0; q < PER; ++q) {
                const int e = lane + 64 * q, i = e / R, b = e % R;
                if (i > j && b >= i) wsh[e] = wsh[e] - wsh[j * R + i] * wsh[j * R + b];
            }
        }
        lds_fence();
        // M = R^-1: lane c owns column c (back substitution; the column lives in LDS, where
        // only lane c touches it, so no register array of R doubles is needed)
        if (lane < R) {
            const int c = lane;
            for (int i = R - 1; i >= 0; --i) {
                double v = (i == c) ? 1.0 : 0.0;
                for (int l = i + 1; l < R; ++l) v -= wsh[i * R + l] * msh[l * R + c];
                msh[i * R + c] = v / wsh[i * R + i];
            }
            for (int i = 0; i < R; ++i)
                if (i >= r || c >= r) msh[i * R + c] = 0.0;
        }
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            keep(xt[q]);
            const int e = lane + 64 * q, i = e / R, l = e % R;
            xsh[e] = (i < r && l < r) ? double(xt[q]) : 0.0;
        }
        lds_fence();
        // T = X[0:r] M
#pragma unroll 1
        for (int q = 0; q < PER; ++q) {
            const int e = lane + 64 * q, i = e / R, c = e % R;
            double v = 0.0;
#pragma unroll 16
            for (int l = 0; l < R; ++l) v += xsh[i * R + l] * msh[l * R + c];
            tsh[e] = v;
        }
        // LAPACK's column signs: the LU recursion of k_orth_chol, lane-parallel
        double sg = 1.0;  // lane c < r ends with sgn[c]
        for (int j = 0; j < r; ++j) {
            lds_fence();
            const double tjj = tsh[j * R + j];
            const bool nonneg = tjj >= 0.0;
            ok = ok && !(j < k - 1 && fabs(tjj) > 1.0 - kSignTol);  // see orth_chol_panel
            const double sj = (j == k - 1) ? (nonneg ? 1.0 : -1.0) : (nonneg ? -1.0 : 1.0);
            if (lane == j) sg = sj;
            const double piv = tjj - sj;
#pragma unroll 4
            for (int q = 0; q < PER; ++q) {
                const int e = lane + 64 * q, i = e / R, b = e % R;
                if (i > j && i < r && b > j && b < r) tsh[e] = tsh[e] - (tsh[i * R + j] / piv) * tsh[j * R + b];
            }
        }
        lds_fence();
        if (lane < R) {
#pragma unroll
            for (int i = 0; i < R; ++i) msh[i * R + lane] = msh[i * R + lane] * sg;
        }
        if (lane == 0) ok_sh = ok ? 1 : 0;
    }
    __syncthreads();
    if (!ok_sh && !(a.flags & 1)) {  // exact Householder (geqr2 + org2r) in place in hx
        for (int64_t i = tid; i < k * r; i += kC16NT) hx[i] = st[i];
        __syncthreads();
        householder_q<R, kC16NT>(hx, k, r, red, tau);
        for (int64_t i = tid; i < k * r; i += kC16NT) st[i] = hx[i];
        return;
    }

    // ---- Y = X M' on the matrix core: 16-row blocks, wave w takes blocks w, w + 16, ...
    // Output block cb, inner block lb, MFMA e covers inner columns l = 16 lb + 4 kk + e:
    // A[i = ri][kk = kq] = M'[16 lb + 4 kq + e][16 cb + pi(ri)], pi(i) = 4 (i & 3) + (i >> 2):
    // the f64 D layout puts row (l>>4) + 4e in lane l, item e, so this output-column
    // permutation hands lane l the four contiguous columns 16 cb + 4 kq .. + 3 of its row
    double am[NB][NB][4];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
#pragma unroll
        for (int lb = 0; lb < NB; ++lb)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                am[cb][lb][e] = msh[(16 * lb + 4 * kq + e) * R + 16 * cb + 4 * (ri & 3) + (ri >> 2)];
    __syncthreads();  // the top block was read (wave 0) before any row is overwritten
    constexpr int kA = NB == 1 ? 6 : 3;
    const int64_t nb = (k + 15) >> 4;
    // 16-B rows: one load per lane per block and column block (state offsets of a
    // mixed-rank plan need not be multiples of 4 floats)
    const bool vec = r == R && ((reinterpret_cast<uintptr_t>(st) | reinterpret_cast<uintptr_t>(hx)) & 15) == 0;
    for (int64_t b0 = wave; b0 < nb; b0 += int64_t(kA) * kC16W) {
        float x[kA][NB][4];
#pragma unroll
        for (int q = 0; q < kA; ++q) {
            const int64_t row = (b0 + int64_t(q) * kC16W) * 16 + ri;
            const int64_t rc = row < k ? row : 0;
#pragma unroll
            for (int lb = 0; lb < NB; ++lb) {
                if (vec) {
                    const float4 t = *reinterpret_cast<const float4*>(st + rc * R + 16 * lb + 4 * kq);
                    x[q][lb][0] = t.x; x[q][lb][1] = t.y; x[q][lb][2] = t.z; x[q][lb][3] = t.w;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int c = 16 * lb + 4 * kq + e;
                        x[q][lb][e] = st[rc * r + (c < r ? c : 0)];
                    }
                }
            }
        }
#pragma unroll
        for (int q = 0; q < kA; ++q) {
            const int64_t row = (b0 + int64_t(q) * kC16W) * 16 + ri;
#pragma unroll
            for (int lb = 0; lb < NB; ++lb)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    keep(x[q][lb][e]);
                    x[q][lb][e] = (16 * lb + 4 * kq + e < r) ? x[q][lb][e] : 0.f;
                }
#pragma unroll
            for (int cb = 0; cb < NB; ++cb) {
                f64x4_t y = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int lb = 0; lb < NB; ++lb)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        y = __builtin_amdgcn_mfma_f64_16x16x4f64(am[cb][lb][e], double(x[q][lb][e]), y, 0, 0, 0);
                // lane l holds D[kq + 4e][ri] = Y[row0 + ri][16 cb + pi(kq + 4e) = 16 cb + 4 kq + e]
                if (row < k) {
                    if (vec) {
                        const float4 o = make_float4(float(y[0]), float(y[1]), float(y[2]), float(y[3]));
                        *reinterpret_cast<float4*>(st + row * R + 16 * cb + 4 * kq) = o;
                        *reinterpret_cast<float4*>(hx + row * R + 16 * cb + 4 * kq) = o;
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int c = 16 * cb + 4 * kq + e;
                            if (c < r) {
                                st[row * r + c] = float(y[e]);
                                hx[row * r + c] = float(y[e]);
                            }
                        }
                    }
                }
            }
        }
    }
}

__global__ __launch_bounds__(kC16NT) void k_orth_chol16(OrthArgs a) { orth_chol_wide<16>(a); }
__global__ __launch_bounds__(kC16NT) void k_orth_chol32(OrthArgs a) { orth_chol_wide<32>(a); }

// ------------------------------------------- folded Cholesky-QR (projection form) ----
// The Q panels of a two-iteration rank-2/4 step at world size 1: k_reduce left each item's
// upper Gram (fp64) beside the reduced factor, so no pass over the panel forms it. Workgroup
// (unit, slice) sums its unit's item partials (lane-strided in item order, then the wave
// tree: fixed order, the same in every slice), runs k_orth_chol's chain (Cholesky, R^-1,
// LAPACK signs from the top rows) and writes X = raw M D for its kChainRows rows (the same
// fp64 row products as k_orth_chol's second pass): the panel is read once, spread over
// ceil(k / kChainRows) CUs instead of one. A panel the chain rejects takes the exact
// Householder recursion in slice 0 (the other slices return).
// rows per thread of k_orth_chain: 1 (one 512-row slice per workgroup; cfg3 0.0911-0.0912 ->
// 0.0908 ms against 2, 4 slower: 0.0914-0.0915, profiles/r05/orth/r05ar_chain_rows.txt)
#ifndef PSGD_CHAIN_NT
#define PSGD_CHAIN_NT 512
#endif
#ifndef PSGD_CHAIN_ROWS
#define PSGD_CHAIN_ROWS 1
#endif
template <int R>
__global__ __launch_bounds__(PSGD_CHAIN_NT) void k_orth_chain(ChainArgs a) {
    constexpr int NT = PSGD_CHAIN_NT;
    constexpr int NG = R * (R + 1) / 2;
    constexpr int kRows = PSGD_CHAIN_ROWS;  // rows per thread: kChainRows = kRows NT
    __shared__ double m_sh[R * R];
    __shared__ int ok_sh;
    __shared__ float top_sh[R * R];
    __shared__ float red[NT / 64 * R];
    __shared__ float tau[(R + 3) / 4 * 4];
    const OrthUnit u = a.units[blockIdx.x];
    const int r = R;  // the plan folds only panels of exactly R columns
    const int64_t k = u.k;
    const int64_t row0 = int64_t(blockIdx.y) * kRows * NT;
    if (row0 >= k) return;  // uniform: short panels use fewer slices
    const int tid = threadIdx.x, lane = tid & 63;
    const float* raw = a.raw + u.off;
    // this slice's rows go out first (in flight during the partial sums and the chain)
    float x[kRows][R];
#pragma unroll
    for (int q = 0; q < kRows; ++q) {
        const int64_t i = row0 + tid + int64_t(q) * NT;
        ld_row<R>(raw + (i < k ? i : 0) * r, r, x[q]);
    }
    if (tid < R * R) top_sh[tid] = raw[tid];  // the top R rows (k >= r)
    double g[NG];
    if (tid < 64) {
        const int ib = a.uitems[2 * blockIdx.x], ie = a.uitems[2 * blockIdx.x + 1];
#pragma unroll
        for (int e = 0; e < NG; ++e) g[e] = 0.0;
        for (int it0 = ib + lane; it0 < ie; it0 += 64) {
#pragma unroll
            for (int e = 0; e < NG; ++e) g[e] += a.gram[int64_t(it0) * kGramStride + e];
        }
#pragma unroll
        for (int e = 0; e < NG; ++e) g[e] = wave_allsum_f64(g[e]);
    }
    __syncthreads();  // top_sh
    if (tid < 64) chol_chain<R>(g, top_sh, raw, r, k, m_sh, &ok_sh, blockIdx.y == 0 ? a.rfac + u.off : nullptr);
    __syncthreads();
    float* st = a.state + u.off;
    float* hx = a.hx + u.off;
    if (!ok_sh) {
        if (blockIdx.y != 0) return;
        // exact Householder (geqr2 + org2r) in the history buffer, then the state
        for (int64_t i = tid; i < k * r; i += NT) hx[i] = raw[i];
        __syncthreads();
        householder_q<R, NT>(hx, k, r, red, tau, a.rfac + u.off);
        for (int64_t i = tid; i < k * r; i += NT) st[i] = hx[i];
        return;
    }
    double M[R][R];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int c = 0; c < R; ++c) M[i][c] = m_sh[i * R + c];
#pragma unroll
    for (int q = 0; q < kRows; ++q) {
        const int64_t i = row0 + tid + int64_t(q) * NT;
#pragma unroll
        for (int c = 0; c < R; ++c) keep(x[q][c]);
        float y[R];
#pragma unroll
        for (int c = 0; c < R; ++c) {
            double v = 0.0;
#pragma unroll
            for (int l = 0; l < R; ++l) v += double(x[q][l]) * M[l][c];
            y[c] = float(v);
        }
        if (i < k) {
            st_row<R>(st + i * r, r, y);
            st_row<R>(hx + i * r, r, y);
        }
    }
}

hipError_t launch_orth_chain(const ChainArgs& a, int nunits, int64_t max_rows, int R, hipStream_t s) {
    if (nunits == 0) return hipSuccess;
    auto grid = [&](int nt) { return dim3(unsigned(nunits), unsigned((max_rows + PSGD_CHAIN_ROWS * nt - 1) / (PSGD_CHAIN_ROWS * nt))); };
    switch (R) {
        case 2: k_orth_chain<2><<<grid(PSGD_CHAIN_NT), PSGD_CHAIN_NT, 0, s>>>(a); break;
        case 4: k_orth_chain<4><<<grid(PSGD_CHAIN_NT), PSGD_CHAIN_NT, 0, s>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// rank 4, panels longer than one default batch (8 x 512 rows) up to 10 x 512: the 10-row
// batch instance (W > 1 Q panels of ResNet-50: k_orth_chol<4> ~1 us faster; on the <= 4096-row
// P panels the default batch stays faster, profiles/r05/orth)
#ifndef PSGD_CHOL_U4L
#define PSGD_CHOL_U4L 10
#endif
constexpr int kCholKU4Long = PSGD_CHOL_U4L > PSGD_CHOL_U4 ? PSGD_CHOL_U4L : PSGD_CHOL_U4 + 1;
// rank 4, panels of at most 4 x 512 rows (ResNet-50's P panels): 4-row batches, no clamped loads
#ifndef PSGD_CHOL_U4S
#define PSGD_CHOL_U4S 4
#endif
constexpr int kCholKU4Short = PSGD_CHOL_U4S > 0 ? PSGD_CHOL_U4S : 1;
// rank 2, panels up to 22 x 512 rows (LLaMA's 11008-row Q panels) in one register-resident batch
#ifndef PSGD_CHOL_U2L
#define PSGD_CHOL_U2L 22
#endif
constexpr int kCholKU2Long = PSGD_CHOL_U2L > PSGD_CHOL_U2 ? PSGD_CHOL_U2L : PSGD_CHOL_U2 + 1;
hipError_t launch_orth_chol(const OrthArgs& a, int nunits, int R, int64_t kmax, hipStream_t s) {
    switch (R) {
        case 2:
            if (PSGD_CHOL_U2L > PSGD_CHOL_U2 && kmax > int64_t(PSGD_CHOL_U2) * CholNT<2>::value && kmax <= int64_t(kCholKU2Long) * CholNT<2>::value)
                k_orth_chol<2, kCholKU2Long><<<nunits, CholNT<2>::value, 0, s>>>(a);
            else
                k_orth_chol<2><<<nunits, CholNT<2>::value, 0, s>>>(a);
            break;
        case 4:
            if (PSGD_CHOL_U4S > 0 && PSGD_CHOL_U4S < PSGD_CHOL_U4 && kmax <= int64_t(kCholKU4Short) * CholNT<4>::value)
                k_orth_chol<4, kCholKU4Short><<<nunits, CholNT<4>::value, 0, s>>>(a);
            else if (PSGD_CHOL_U4L > PSGD_CHOL_U4 && kmax > int64_t(PSGD_CHOL_U4) * CholNT<4>::value && kmax <= int64_t(kCholKU4Long) * CholNT<4>::value)
                k_orth_chol<4, kCholKU4Long><<<nunits, CholNT<4>::value, 0, s>>>(a);
            else
                k_orth_chol<4><<<nunits, CholNT<4>::value, 0, s>>>(a);
            break;
        case 8: k_orth_chol<8><<<nunits, CholNT<8>::value, 0, s>>>(a); break;
        case 16: k_orth_chol16<<<nunits, kC16NT, 0, s>>>(a); break;
        case 32: k_orth_chol32<<<nunits, kC16NT, 0, s>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------ paper-code Gram-Schmidt (variant) ----
// paper-code/gradient_reducers.py:945-956 (RankKReducer / HalfRankKReducer), per matrix:
//   for i: col_i /= sqrt(sum col_i^2) + 1e-8 ; rest -= (col_i . rest) col_i
// (the eps is ADDED to the norm, unlike the reference codec's max(norm, eps)). One
// workgroup per panel, in place, column sums as fixed-order workgroup reductions.
template <int R>
__global__ __launch_bounds__(kBlock) void k_orth_mgs(OrthArgs a) {
    __shared__ float red[kWaves * R];
    const OrthUnit u = a.units[blockIdx.x];
    const int r = u.r;
    const int64_t k = u.k;
    const int tid = threadIdx.x;
    float* __restrict__ x = a.state + u.off;
    for (int i = 0; i < r; ++i) {
        float s1[1] = {0.f};
        for (int64_t row = tid; row < k; row += kBlock) {
            const float v = x[row * r + i];
            s1[0] = fmaf(v, v, s1[0]);
        }
        block_sum_nw<float, 1, kWaves>(s1, red);
        const float den = sqrtf(s1[0]) + 1e-8f;
        for (int64_t row = tid; row < k; row += kBlock) x[row * r + i] = x[row * r + i] / den;
        __syncthreads();
        if (i + 1 < r) {
            float dt[R];
#pragma unroll
            for (int c = 0; c < R; ++c) dt[c] = 0.f;
            for (int64_t row = tid; row < k; row += kBlock) {
                const float ci = x[row * r + i];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > i && c < r) dt[c] = fmaf(ci, x[row * r + c], dt[c]);
            }
            block_sum_nw<float, R, kWaves>(dt, red);
            for (int64_t row = tid; row < k; row += kBlock) {
                const float ci = x[row * r + i];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > i && c < r) x[row * r + c] -= dt[c] * ci;
            }
            __syncthreads();
        }
    }
}

hipError_t launch_orth_mgs(const OrthArgs& a, int nunits, int R, hipStream_t s) {
    switch (R) {
        case 1: k_orth_mgs<1><<<nunits, kBlock, 0, s>>>(a); break;
        case 2: k_orth_mgs<2><<<nunits, kBlock, 0, s>>>(a); break;
        case 4: k_orth_mgs<4><<<nunits, kBlock, 0, s>>>(a); break;
        case 8: k_orth_mgs<8><<<nunits, kBlock, 0, s>>>(a); break;
        case 16: k_orth_mgs<16><<<nunits, kBlock, 0, s>>>(a); break;
        case 32: k_orth_mgs<32><<<nunits, kBlock, 0, s>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_orth(const OrthArgs& a, int nunits, int R, int64_t kmax, bool chol, hipStream_t s) {
    // register-resident path when the longest rank>1 panel fits RPT * R <= 128 floats/thread
    int64_t rpt = 1;
    while (rpt * kOrthThreads < kmax) rpt <<= 1;
    if (R == 1) return launch_orth_reg_r<1>(1, a, nunits, s);
    static const int diag = [] {
        const char* e = std::getenv("PSGD_ORTH_DIAG");
        return e ? std::atoi(e) : 0;
    }();
    if (chol && R <= 32) {
        OrthArgs b = a;
        b.flags = diag;
        return launch_orth_chol(b, nunits, R, kmax, s);
    }
    hipError_t err = hipSuccess;
    if (env_orth_wy() && launch_orth_wy(a, nunits, R, kmax, s, &err)) return err;
    if (rpt <= 16 && orth_reg_ok(R, int(rpt))) {
        switch (R) {
            case 2: return launch_orth_reg_r<2>(int(rpt), a, nunits, s);
            case 4: return launch_orth_reg_r<4>(int(rpt), a, nunits, s);
            case 8: return launch_orth_reg_r<8>(int(rpt), a, nunits, s);
            default: break;
        }
    }
    constexpr int64_t kLdsCap = 60 * 1024 / 4;  // dynamic LDS floats (stays under the 64 KiB default)
    const int64_t panel = kmax * R;
    const int64_t lds = panel < kLdsCap ? panel : kLdsCap;
    return launch_orth_r(R, a, nunits, lds, s);
}

// ---------------------------------------------------------------- partial reduction
// Sums the partials of each factor element in a FIXED order (the even product's segments down
// a column strip, the odd product's column strips): bitwise reproducible, no atomics.

// One item = up to 64 * per consecutive elements of one factor (per = 4, or 1 for factors with
// many partials: RedItem::per) with one partial layout (RedItem::pbase / pstride / np).
// per = 4: one 16-byte load per partial when the item's partial runs are 16-byte aligned (lane
// l owns elements 4l .. 4l+3), else four 256-byte wave loads (lane l owns l, l+64, l+128,
// l+192). Wave w adds the partials [w*np/4, (w+1)*np/4) of each element in order, then wave 0
// adds the four wave sums in order: every element is summed in the same fixed order on every
// run, whatever the layout.
#ifndef PSGD_RED_SHORT
#define PSGD_RED_SHORT 8
#endif
__device__ __forceinline__ int red_elem(bool vec, int lane, int j) { return vec ? 4 * lane + j : lane + 64 * j; }

__global__ __launch_bounds__(kBlock) void k_reduce(ReduceArgs a) {
    __shared__ float red[kWaves * kRedItem];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (int(blockIdx.x) >= a.nmain) {  // fused normalisation of the in-factor (rank 1)
        if (wave != 0) return;
        const RedItem it = a.nitems[blockIdx.x - a.nmain];
        const MatDesc d = a.mats[it.mat];
        const int64_t base = (a.even ? d.poff : d.qoff) + it.start;
        float x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // in flight together with the norm's loads
            const int e = red_elem(false, lane, j);
            x[j] = a.raw[base + (e < it.cnt ? e : 0)];
        }
        const float dn = group_norm_ss(a.ss_in, a.grng_in, d.group);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = red_elem(false, lane, j);
            if (j < it.per && e < it.cnt) {
                const float v = x[j] / dn;  // matrix.div_(max(norm, eps))
                a.xstate[base + e] = v;
                a.hx[base + e] = v;
            }
        }
        return;
    }
    const RedItem it = a.items[blockIdx.x];
    const MatDesc d = a.mats[it.mat];
    const int per = it.per, cnt = it.cnt;
    const int64_t ps = it.pstride;
    const bool vec = per == 4 && ((it.pbase | ps | int64_t(cnt)) & 3) == 0;  // uniform per workgroup
    const int np = it.np;
    const int c0 = wave * np / kWaves, c1 = (wave + 1) * np / kWaves;
    // wave 0's first group-norm loads go out before the partials' (group_norm_ss's order:
    // lane-strided sums from 0, then the wave tree), so the two round trips overlap
    const bool nrm = a.ss_in != nullptr && wave == 0;
    int gb = 0, ge = 0;
    float ssv = 0.f;
    if (nrm) {
        gb = a.grng_in[2 * d.group];
        ge = a.grng_in[2 * d.group + 1];
        ssv = gb + lane < ge ? a.ss_in[gb + lane] : 0.f;
    }
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    // loads issued 16 at a time (clamped, unconditional): the partials were just written on
    // other XCDs, so each batch is one MALL round trip
    const gptr<const float> pb = gconst<float>(a.part) + it.pbase;
    if (vec) {
        const int e0 = red_elem(true, lane, 0);
        const gptr<const float> p = pb + (e0 < cnt ? e0 : 0);
        // batches of kB partials; a wave with at most PSGD_RED_SHORT partials issues only that
        // many loads (no clamped repeats): k_reduce 6.2 -> 5.5-5.7 us on cfg3,
        // cfg3 / cfg2 steps 0.0910 / 0.0757-0.0760 -> 0.0905-0.0907 / 0.0754-0.0756 ms
        // (profiles/r05/reduce)
        auto run = [&](auto KB) {
            constexpr int kB = decltype(KB)::value;
            for (int c = c0; c < c1; c += kB) {
                float v[kB][4];
#pragma unroll
                for (int q = 0; q < kB; ++q) {
                    const v4f x = *(gptr<const v4f>)(p + int64_t(c + q < c1 ? c + q : c0) * ps);
                    v[q][0] = x.x; v[q][1] = x.y; v[q][2] = x.z; v[q][3] = x.w;
                }
#pragma unroll
                for (int q = 0; q < kB; ++q)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        keep(v[q][j]);
                        s[j] += c + q < c1 ? v[q][j] : 0.f;
                    }
            }
        };
        if (PSGD_RED_SHORT > 0 && c1 - c0 <= PSGD_RED_SHORT)
            run(std::integral_constant<int, (PSGD_RED_SHORT > 0 ? PSGD_RED_SHORT : 1)>{});
        else
            run(std::integral_constant<int, 16>{});
    } else if (per == 4) {
        int ec[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = red_elem(false, lane, j);
            ec[j] = e < cnt ? e : 0;
        }
        constexpr int kB = 4;
        for (int c = c0; c < c1; c += kB) {
            float v[kB][4];
#pragma unroll
            for (int q = 0; q < kB; ++q)
#pragma unroll
                for (int j = 0; j < 4; ++j) v[q][j] = pb[int64_t(c + q < c1 ? c + q : c0) * ps + ec[j]];
#pragma unroll
            for (int q = 0; q < kB; ++q)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    keep(v[q][j]);
                    s[j] += c + q < c1 ? v[q][j] : 0.f;
                }
        }
    } else {
        // many partials per element (np > kRedWide, e.g. the odd-even pass's row blocks): 32 of
        // a wave's partials in flight at once (two round trips where 16 took four on 256
        // partials; the sum order is the same)
        const gptr<const float> p = pb + (lane < cnt ? lane : 0);
        constexpr int kB = 32;
        for (int c = c0; c < c1; c += kB) {
            float v[kB];
#pragma unroll
            for (int q = 0; q < kB; ++q) v[q] = p[int64_t(c + q < c1 ? c + q : c0) * ps];
#pragma unroll
            for (int q = 0; q < kB; ++q) {
                keep(v[q]);
                s[0] += c + q < c1 ? v[q] : 0.f;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (j < per) red[wave * kRedItem + j * 64 + lane] = s[j];
    __syncthreads();
    if (wave != 0) return;
    float nv = 1.f;
    if (nrm) {
        for (int i = gb + lane + 64; i < ge; i += 64) ssv += a.ss_in[i];
        nv = sqrtf(wave_allsum(ssv));
        nv = nv > 1e-16f ? nv : 1e-16f;
    }
    const int64_t dbase = (a.even ? d.qoff : d.poff) + it.start;
    float sq = 0.f;
    float tv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        tv[j] = 0.f;
        if (j >= per) continue;
        const int o = j * 64 + lane;
        float t = ((red[o] + red[kRedItem + o]) + red[2 * kRedItem + o]) + red[3 * kRedItem + o];
        if (nrm) t = t / nv;  // G^T (x / d) == (G^T x) / d up to rounding
        const int e = red_elem(vec, lane, j);
        if (e < cnt) {
            a.yloc[dbase + e] = t;
            a.state[dbase + e] = t;
            if (a.xout) st_slot(a.xout + dbase + e, t);
            sq = fmaf(t, t, sq);
            tv[j] = t;
        }
    }
    if (a.ss_out) {  // this output is the next iteration's in-factor: its sum of squares
        const float v = wave_allsum(sq);
        if (lane == 0) a.ss_out[blockIdx.x] = v;
    }
    if (a.gram) {
        // folded orthonormalisation: the upper Gram of this item's rows (r in {2, 4}; items
        // start on a row and hold whole rows). The outputs go to LDS in element order (wave 0
        // alone: its own earlier reads of `red` are ordered before these writes), then lane l
        // takes rows l, l + 64, ...; fp64 products and sums, one fixed-order wave tree per entry.
        const int r = a.gram_r, ng = r * (r + 1) / 2;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < per) red[vec ? 4 * lane + j : lane + 64 * j] = tv[j];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int nrow = 64 * per / r;
        double g[kGramStride];
#pragma unroll
        for (int e = 0; e < kGramStride; ++e) g[e] = 0.0;
        auto rows = [&](auto RT) {  // compile-time r: register-indexed Gram entries
            constexpr int RC = decltype(RT)::value;
            for (int row = lane; row < nrow; row += 64) {
                float x[RC];
#pragma unroll
                for (int c = 0; c < RC; ++c) x[c] = red[row * RC + c];
                int e = 0;
#pragma unroll
                for (int c = 0; c < RC; ++c)
#pragma unroll
                    for (int b = c; b < RC; ++b) g[e++] += double(x[c]) * double(x[b]);
            }
        };
        if (r == 4)
            rows(std::integral_constant<int, 4>{});
        else
            rows(std::integral_constant<int, 2>{});
#pragma unroll
        for (int e = 0; e < kGramStride; ++e) {
            if (e < ng) {
                const double t = wave_allsum_f64(g[e]);
                if (lane == 0) a.gram[int64_t(blockIdx.x) * kGramStride + e] = t;
            }
        }
    }
}

hipError_t launch_reduce(const ReduceArgs& a, int nitems, hipStream_t s) {
    k_reduce<<<nitems, kBlock, 0, s>>>(a);  // nitems = nmain + nnorm
    return hipGetLastError();
}

// ---------------------------------------------------------------- one-shot all-reduce
// The reference's SUM all-reduce of an out-factor (powersgd.py:204-209), one node, one
// process per GPU, stream-ordered with no host round trip. Cross-GPU visibility, step by step:
//  1. the kernels before this one wrote the LOCAL factor into this rank's exchange slot with
//     system-scope stores (st_slot: `sc0 sc1`, write-through; the flat region with PSGD_ST_AUX
//     = sc0 | nt | sc1): no byte of the slot waits in any of the eight L2s for a writeback;
//  2. this launch starts only after they completed (same stream, barrier bit): every one of those
//     stores has been acknowledged by memory;
//  3. workgroup 0 then stores this rank's epoch flag (system scope, `sc0 sc1`);
//  4. peers poll the flag with system-scope loads and read the slot ONLY with system-scope loads
//     (`sc0 sc1`, which no non-coherent cache level serves), so they see the bytes of (1).
// This is the write-through hand-off of MI355X_MICROARCH.md (visibility table, first row: stores
// all write-through, drained before ONE lane's flag store, flag polled and payload loaded with
// coherent loads) at system scope, with the kernel boundary as the drain. It needs no release
// fence: one here would write back only this workgroup's XCD L2, which (1) leaves clean.
// The wait is bounded: a peer that never arrives sets the sticky error word (host-mapped, read by
// the next psgd_aggregate_ipc call, which then fails) instead of hanging the queue.
#ifndef PSGD_XCHG_FLAG_ORDER
#define PSGD_XCHG_FLAG_ORDER __ATOMIC_RELAXED
#endif
// System-scope (sc0 | sc1) 16-byte loads: they miss in every non-coherent cache level.
constexpr int kSysAux = 17;
constexpr int kXchgUnroll = 8;  // peers whose loads are in flight together

__device__ __forceinline__ void xchg_sum_quad(const XchgArgs& a, int64_t src_byte, uint32_t lim, float (&s)[4]) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    for (int w0 = 0; w0 < a.world; w0 += kXchgUnroll) {
        v4u v[kXchgUnroll];
#pragma unroll
        for (int u = 0; u < kXchgUnroll; ++u) {
            const bool on = w0 + u < a.world;  // past the last peer: an empty descriptor, no access
            const rsrc_t rs = make_rsrc(a.peers[on ? w0 + u : w0] + a.slot_off, on ? lim : 0u);
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, uint32_t(src_byte), 0, kSysAux);
        }
#pragma unroll
        for (int u = 0; u < kXchgUnroll; ++u)
            if (w0 + u < a.world)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float x = __uint_as_float(v[u][j]);
                    s[j] = w0 + u == 0 ? x : s[j] + x;  // rank order
                }
    }
}

__global__ __launch_bounds__(kBlock) void k_xchg(XchgArgs a) {
    const int tid = threadIdx.x;
    // the slot bytes were written through by the PREVIOUS kernels of this stream (steps 1-2
    // above): the flag is a plain system-scope store, no fence
    if (blockIdx.x == 0 && tid == 0)
        __hip_atomic_store(a.own_flag, (uint64_t(a.own_nonce) << 32) | a.epoch, PSGD_XCHG_FLAG_ORDER,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    bool dead = false;
    if (tid < a.world && tid != a.rank) {  // lane w polls peer w: the W round trips overlap
        const uint64_t* f = reinterpret_cast<const uint64_t*>(a.peers[tid] + a.flag_off);
        const uint32_t want = a.nonces[tid];  // this session's flags only
        uint32_t spins = 0;
        for (;;) {
            // the device copy of the sticky error word, loaded beside the flag (no extra round
            // trip): an earlier exchange of this rank gave up, so the ranks' epochs have drifted
            // apart and this exchange is invalid whatever the flags say
            const int32_t gone = __hip_atomic_load(a.err_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t fv = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (gone) {
                dead = true;
                break;
            }
            if (uint32_t(fv >> 32) == want && (fv & 0xffffffffull) >= a.epoch) break;
            if (++spins > a.spin_limit) {
                // host-mapped sticky word (vector store, system scope) and its device copy: the
                // results of this step are invalid and the host refuses every later exchange step
                __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(a.err_dev, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                dead = true;
                break;
            }
            __builtin_amdgcn_s_sleep(10);
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    if (__syncthreads_or(dead)) {
        // an invalid exchange returns NaN sums, never plausible stale ones: the
        // factor (and, on the last iteration, the flat tensors) of this workgroup's share
        const float nan = __builtin_nanf("");
        if (a.items) {
            const RedItem it = a.items[blockIdx.x];
            const MatDesc d = a.mats[it.mat];
            const int64_t e = (a.even ? d.qoff : d.poff) + it.start + tid;
            if (tid < it.cnt) a.dst[e] = a.dst2[e] = nan;
            return;
        }
        const int64_t stride = int64_t(gridDim.x) * kBlock;
        for (int64_t i = int64_t(blockIdx.x) * kBlock + tid; i < a.n + a.nflat; i += stride) {
            if (i < a.n) a.dst[i] = nan;
            else a.flat_dst[i - a.n] = nan;
        }
        return;
    }
    if (a.items) {  // one reduction item per workgroup (<= 256 consecutive factor elements)
        __shared__ float wsq[kWaves];
        __shared__ float xv[kRedItem];
        const RedItem it = a.items[blockIdx.x];
        const MatDesc d = a.mats[it.mat];
        const int64_t e = (a.even ? d.qoff : d.poff) + it.start + tid;
        float sq = 0.f, s = 0.f;
        if (tid < it.cnt) {
            for (int w0 = 0; w0 < a.world; w0 += kXchgUnroll) {  // the peers' loads in flight together
                float v[kXchgUnroll];
#pragma unroll
                for (int u = 0; u < kXchgUnroll; ++u)  // uniform guard: no load past the last peer
                    v[u] = w0 + u < a.world
                               ? __hip_atomic_load(reinterpret_cast<const float*>(a.peers[w0 + u] + a.slot_off) + e,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                               : 0.f;
#pragma unroll
                for (int u = 0; u < kXchgUnroll; ++u)
                    if (w0 + u < a.world) s = w0 + u == 0 ? v[u] : s + v[u];  // rank order
            }
            a.dst[e] = s;
            a.dst2[e] = s;
            sq = s * s;
        }
        if (a.ss_out) {
            sq = wave_allsum(sq);
            if ((tid & 63) == 0) wsq[tid >> 6] = sq;
            __syncthreads();
            if (tid == 0) a.ss_out[blockIdx.x] = ((wsq[0] + wsq[1]) + wsq[2]) + wsq[3];
        }
        if (a.gram) {
            // the item's rows (it starts on a row and holds whole rows of r elements): lane l
            // of wave 0 takes rows l, l + 64, ...; fp64 products, one wave tree per entry
            xv[tid] = s;
            __syncthreads();
            if (tid >= 64) return;
            const int r = a.gram_r, nrow = it.cnt / r;
            double g[kGramStride];
#pragma unroll
            for (int k = 0; k < kGramStride; ++k) g[k] = 0.0;
            for (int row = tid; row < nrow; row += 64) {
                int k = 0;
                for (int c = 0; c < r; ++c)
                    for (int b = c; b < r; ++b) {
                        const double prod = double(xv[row * r + c]) * double(xv[row * r + b]);
#pragma unroll
                        for (int q = 0; q < kGramStride; ++q)
                            if (q == k) g[q] += prod;
                        ++k;
                    }
            }
            const int ng = r * (r + 1) / 2;
#pragma unroll
            for (int k = 0; k < kGramStride; ++k) {
                if (k < ng) {
                    const double t = wave_allsum_f64(g[k]);
                    if (tid == 0) a.gram[int64_t(blockIdx.x) * kGramStride + k] = t;
                }
            }
        }
        return;
    }
    // quads of the factor, then quads of the flat region; buffer bounds zero-fill a ragged tail
    const int64_t qf = (a.n + 3) / 4, qt = qf + (a.nflat + 3) / 4;
    const int64_t stride = int64_t(gridDim.x) * kBlock;
    for (int64_t q = int64_t(blockIdx.x) * kBlock + tid; q < qt; q += stride) {
        const bool fac = q < qf;
        const int64_t e0 = fac ? 4 * q : 4 * (q - qf);  // element index in dst / flat_dst
        const int64_t cnt = fac ? a.n : a.nflat;
        const int64_t base = fac ? 0 : a.flat_off;
        const uint32_t lim = uint32_t((base + cnt) * int64_t(sizeof(float)));
        float s[4];
        xchg_sum_quad(a, (base + e0) * int64_t(sizeof(float)), lim, s);
        float* d = fac ? a.dst : a.flat_dst;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (e0 + j < cnt) d[e0 + j] = s[j];
    }
}

hipError_t launch_xchg(const XchgArgs& a, hipStream_t s) {
    if (a.items) {
        k_xchg<<<a.nitems < 1 ? 1 : a.nitems, kBlock, 0, s>>>(a);
        return hipGetLastError();
    }
    const int64_t quads = (a.n + 3) / 4 + (a.nflat + 3) / 4;
    const int64_t blocks = (quads + kBlock - 1) / kBlock;
    // at least one workgroup (it raises the flag), at most one per CU
    k_xchg<<<int(blocks < 1 ? 1 : blocks < 256 ? blocks : 256), kBlock, 0, s>>>(a);
    return hipGetLastError();
}

// ---------------------------------------------------------------- flat pack
// reference powersgd.py:22-31 + utils.py:6-10, :43-49: flat = x / W (division, as div_),
// then x = 0. One read + two writes per element.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_flat_pack(FlatArgs a) {
    flat_pack_item<T, kBlock>(a, blockIdx.x);
}

hipError_t launch_flat_pack(int dtype, const FlatArgs& a, hipStream_t s) {
    if (a.nitems == 0) return hipSuccess;
    if (dtype == 2) return launch_flat_pack_f64(a, s);
    if (dtype == 0)
        k_flat_pack<float><<<a.nitems, kBlock, 0, s>>>(a);
    else
        k_flat_pack<bf16_t><<<a.nitems, kBlock, 0, s>>>(a);
    return hipGetLastError();
}

// ---------------------------------------------------------------- DDP run tables
// The DDP comm hook's two bucket passes (powersgd_amd/ddp.py): ADD folds a bucket
// of fresh gradients into the per-parameter error-feedback residual (what autograd's
// accumulation into p.grad does in the reference flow, README.md:39-42: one add in the
// gradient dtype, bf16 rounded to nearest even), GATHER copies the averaged gradients back into
// the bucket's layout. One item per workgroup: 16 coalesced elements per thread, every load in
// flight before any store.
template <typename T>
struct RunMath {  // fp32 / fp64: native adds
    using A = T;
    static __device__ __forceinline__ A up(T x) { return x; }
    static __device__ __forceinline__ T down(A x) { return x; }
};
template <>
struct RunMath<bf16_t> {
    using A = float;
    static __device__ __forceinline__ A up(bf16_t x) { return bf2f(x); }
    static __device__ __forceinline__ bf16_t down(A x) { return f2bf(x); }
};

template <typename T, bool ADD>
__global__ __launch_bounds__(kBlock) void k_runs(RunsArgs a) {
    using M = RunMath<T>;
    const RunItem it = a.items[blockIdx.x];
    T* t = static_cast<T*>(a.tensors[it.tensor]) + it.toff;
    T* b = static_cast<T*>(a.bucket) + it.boff;
    constexpr int PER = kRunItem / kBlock;
    T v[PER], w[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int j = q * kBlock + int(threadIdx.x);
        const int jj = j < it.cnt ? j : 0;  // clamped, unconditional
        if constexpr (ADD) {
            v[q] = b[jj];
            w[q] = t[jj];
        } else {
            v[q] = t[jj];
        }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int j = q * kBlock + int(threadIdx.x);
        if (j < it.cnt) {
            if constexpr (ADD)
                t[j] = M::down(M::up(w[q]) + M::up(v[q]));  // residual + fresh gradient
            else
                b[j] = v[q];
        }
    }
}

template <typename T>
hipError_t launch_runs_t(bool add, const RunsArgs& a, hipStream_t s) {
    if (add)
        k_runs<T, true><<<a.nitems, kBlock, 0, s>>>(a);
    else
        k_runs<T, false><<<a.nitems, kBlock, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_runs(int dtype, bool add, const RunsArgs& a, hipStream_t s) {
    if (a.nitems <= 0) return hipSuccess;
    if (dtype == 0) return launch_runs_t<float>(add, a, s);
    if (dtype == 2) return launch_runs_t<double>(add, a, s);
    return launch_runs_t<bf16_t>(add, a, s);
}

}  // namespace psgd
