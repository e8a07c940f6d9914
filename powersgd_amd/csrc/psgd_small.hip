// Small-panel kernels: orthonormalisation of the in-factor, deterministic reduction of the
// product partials, and the flat pack of uncompressed tensors.
#include <hip/hip_runtime.h>

#include "psgd_internal.h"
#include "psgd_stream.cuh"

namespace psgd {

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
__device__ void householder_q(float* A, int64_t k, int r, float* red, float* tau) {
    const int tid = threadIdx.x;
    for (int j = 0; j < r; ++j) {
        float s1[1] = {0.f};
        for (int64_t i = j + 1 + tid; i < k; i += kBlock) {
            const float x = A[i * r + j];
            s1[0] = fmaf(x, x, s1[0]);
        }
        block_sum<float, 1>(s1, red);
        const float alpha = A[int64_t(j) * r + j];
        float tj = 0.f;
        if (s1[0] != 0.f) {
            const float xnorm = sqrtf(s1[0]);
            const float beta = -copysignf(hypotf(alpha, xnorm), alpha);
            tj = (beta - alpha) / beta;
            const float scal = 1.f / (alpha - beta);
            for (int64_t i = j + 1 + tid; i < k; i += kBlock) A[i * r + j] *= scal;
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
            for (int64_t i = j + 1 + tid; i < k; i += kBlock) {
                const float vi = A[i * r + j];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > j && c < r) w[c] = fmaf(vi, A[i * r + c], w[c]);
            }
            block_sum<float, R>(w, red);
#pragma unroll
            for (int c = 0; c < R; ++c)
                if (c > j && c < r) w[c] += A[int64_t(j) * r + c];
            __syncthreads();
            for (int64_t i = j + tid; i < k; i += kBlock) {
                const float vi = i == j ? 1.f : A[i * r + j];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > j && c < r) A[i * r + c] -= tj * vi * w[c];
            }
            __syncthreads();
        }
    }
    // org2r: Q = H_0 H_1 ... H_{r-1} I[:, :r], built in place, last reflector first
    for (int j = r - 1; j >= 0; --j) {
        const float tj = tau[j];
        if (j + 1 < r && tj != 0.f) {
            float w[R];
#pragma unroll
            for (int c = 0; c < R; ++c) w[c] = 0.f;
            for (int64_t i = j + 1 + tid; i < k; i += kBlock) {
                const float vi = A[i * r + j];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > j && c < r) w[c] = fmaf(vi, A[i * r + c], w[c]);
            }
            block_sum<float, R>(w, red);
#pragma unroll
            for (int c = 0; c < R; ++c)
                if (c > j && c < r) w[c] += A[int64_t(j) * r + c];
            __syncthreads();
            for (int64_t i = j + tid; i < k; i += kBlock) {
                const float vi = i == j ? 1.f : A[i * r + j];
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c > j && c < r) A[i * r + c] -= tj * vi * w[c];
            }
            __syncthreads();
        }
        for (int64_t i = j + 1 + tid; i < k; i += kBlock) A[i * r + j] *= -tj;
        for (int64_t i = tid; i < j; i += kBlock) A[i * r + j] = 0.f;
        if (tid == 0) A[int64_t(j) * r + j] = 1.f - tj;
        __syncthreads();
    }
}

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

hipError_t launch_orth(const OrthArgs& a, int nunits, int R, int64_t panel, hipStream_t s) {
    constexpr int64_t kLdsCap = 60 * 1024 / 4;  // dynamic LDS floats (stays under the 64 KiB default)
    const int64_t lds = R > 1 ? (panel < kLdsCap ? panel : kLdsCap) : 0;
    return launch_orth_r(R, a, nunits, lds, s);
}

// ---------------------------------------------------------------- partial reduction
// Sums the partials of each factor element in a FIXED order (row chunks for even
// iterations, column strips for odd ones): bitwise reproducible, no atomics.
__global__ __launch_bounds__(kBlock) void k_reduce(ReduceArgs a) {
    const RedItem it = a.items[blockIdx.x];
    const MatDesc d = a.mats[it.mat];
    const int64_t len = (a.even ? d.m : d.n) * d.r;
    const int64_t e = int64_t(it.start) + threadIdx.x;
    if (e >= len) return;
    float s;
    int64_t dst;
    if (a.even) {
        const float* p = a.part + d.part_even + e;
        s = p[0];
        for (int c = 1; c < d.nchunk; ++c) s += p[int64_t(c) * len];
        dst = d.qoff + e;
    } else {
        const float* p = a.part + d.part_odd + e;
        s = p[0];
        for (int c = 1; c < d.nstrip; ++c) s += p[int64_t(c) * len];
        dst = d.poff + e;
    }
    a.yloc[dst] = s;
    a.state[dst] = s;
}

hipError_t launch_reduce(const ReduceArgs& a, int nitems, hipStream_t s) {
    k_reduce<<<nitems, kBlock, 0, s>>>(a);
    return hipGetLastError();
}

// ---------------------------------------------------------------- flat pack
// reference powersgd.py:22-31 + utils.py:6-10, :43-49: flat = x / W (division, as div_),
// then x = 0. One read + two writes per element.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_flat_pack(FlatArgs a) {
    const int64_t chunk = int64_t(blockIdx.x) * kBlock * 4;
    const FlatEntry* ents = a.entries;
    // entry lookup: binary search on dense offsets (count is small)
    int lo = 0, hi = a.count - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (ents[mid].off <= chunk) lo = mid; else hi = mid - 1;
    }
    const float w = float(a.world);
    for (int q = 0; q < 4; ++q) {
        const int64_t e = chunk + int64_t(q) * kBlock + threadIdx.x;
        if (e >= a.total) return;
        int i = lo;
        while (i + 1 < a.count && ents[i + 1].off <= e) ++i;
        T* x = static_cast<T*>(a.tensors[ents[i].tensor]);
        const int64_t j = e - ents[i].off;
        float v[1];
        Io<T>::ld(x + j, v);
        if (a.world != 1) v[0] = v[0] / w;
        Io<T>::st(static_cast<T*>(a.flat) + e, v);
        const float z[1] = {0.f};
        Io<T>::st(x + j, z);
    }
}

hipError_t launch_flat_pack(int dtype, const FlatArgs& a, hipStream_t s) {
    if (a.total == 0) return hipSuccess;
    const int64_t blocks = (a.total + kBlock * 4 - 1) / (kBlock * 4);
    if (dtype == 0)
        k_flat_pack<float><<<dim3(unsigned(blocks)), kBlock, 0, s>>>(a);
    else
        k_flat_pack<bf16_t><<<dim3(unsigned(blocks)), kBlock, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace psgd
