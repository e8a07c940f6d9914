// Streaming-bandwidth ceilings for the codec's two access mixes (diagnostic tool, not part
// of the library), at the cfg2 gradient size (102 MB) so MALL effects match the bench:
//   read  : sum of G                                   [even product]
//   r1w2  : a = G; out = 0.5 a; G = a - out (in place)  [fused final pass / k_apply]
//   copy  : out = G
// Each variant with plain and non-temporal stores, several grid sizes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bw_ceiling.hip -o tools/bw_ceiling
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_read(const v4f* __restrict__ g, float* out, long n4) {
    float s = 0.f;
    const long stride = long(gridDim.x) * 256;
    for (long b = long(blockIdx.x) * 256 + threadIdx.x; b < n4; b += stride * U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + u * stride;
            x[u] = i < n4 ? g[i] : v4f{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) s += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_r1w2(v4f* __restrict__ g, v4f* __restrict__ out, long n4) {
    const long stride = long(gridDim.x) * 256;
    for (long b = long(blockIdx.x) * 256 + threadIdx.x; b < n4; b += stride * U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + u * stride;
            x[u] = i < n4 ? g[i] : v4f{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + u * stride;
            if (i < n4) {
                const v4f o = x[u] * 0.5f;
                if (NT) {
                    __builtin_nontemporal_store(o, out + i);
                    __builtin_nontemporal_store(x[u] - o, g + i);
                } else {
                    out[i] = o;
                    g[i] = x[u] - o;
                }
            }
        }
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const v4f* __restrict__ g, v4f* __restrict__ out, long n4) {
    const long stride = long(gridDim.x) * 256;
    for (long b = long(blockIdx.x) * 256 + threadIdx.x; b < n4; b += stride * U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + u * stride;
            x[u] = i < n4 ? g[i] : v4f{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + u * stride;
            if (i < n4) {
                if (NT)
                    __builtin_nontemporal_store(x[u], out + i);
                else
                    out[i] = x[u];
            }
        }
    }
}

// block-chunked: block b owns elements [b C, (b + 1) C) (float4 units) and walks them with
// U loads in flight per thread (the tiled kernels' pattern)
template <int U>
__global__ __launch_bounds__(256) void k_r1w2_chunk(v4f* __restrict__ g, v4f* __restrict__ out, long n4, long C) {
    extern __shared__ float occ_limiter[];  // dynamic LDS only caps blocks per CU
    if (C < 0) occ_limiter[threadIdx.x] = 0.f;
    const long lo = long(blockIdx.x) * C, hi = lo + C < n4 ? lo + C : n4;
    for (long b = lo + threadIdx.x; b < hi; b += 256 * U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + u * 256;
            x[u] = i < hi ? g[i] : v4f{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + u * 256;
            if (i < hi) {
                const v4f o = x[u] * 0.5f;
                out[i] = o;
                g[i] = x[u] - o;
            }
        }
    }
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                      \
        }                                                                  \
    } while (0)

template <class F>
static float time_it(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) f();
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / reps;  // us per launch
}

int main() {
    const long bytes = 102228128L / 16 * 16;
    const long n4 = bytes / 16;
    v4f *g, *o;
    float* sink;
    CK(hipMalloc(&g, bytes));
    CK(hipMalloc(&o, bytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(g, 0, bytes));
    CK(hipMemset(o, 0, bytes));
    const int grids[] = {1024, 2048, 4096, 8192, 16384};
    for (int gr : grids) {
        float t;
        t = time_it([&] { k_read<4><<<gr, 256>>>(g, sink, n4); }, 50);
        printf("read      grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, bytes / t / 1e3);
        t = time_it([&] { k_read<8><<<gr, 256>>>(g, sink, n4); }, 50);
        printf("read U8   grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, bytes / t / 1e3);
        t = time_it([&] { k_copy<4, false><<<gr, 256>>>(g, o, n4); }, 50);
        printf("copy      grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 2 * bytes / t / 1e3);
        t = time_it([&] { k_copy<4, true><<<gr, 256>>>(g, o, n4); }, 50);
        printf("copy nt   grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 2 * bytes / t / 1e3);
        t = time_it([&] { k_r1w2<4, false><<<gr, 256>>>(g, o, n4); }, 50);
        printf("r1w2      grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 3 * bytes / t / 1e3);
        t = time_it([&] { k_r1w2<4, true><<<gr, 256>>>(g, o, n4); }, 50);
        printf("r1w2 nt   grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 3 * bytes / t / 1e3);
    }
    for (long C : {1024L, 4096L, 16384L, 65536L}) {
        const int gr = int((n4 + C - 1) / C);
        float t = time_it([&] { k_r1w2_chunk<4><<<gr, 256>>>(g, o, n4, C); }, 50);
        printf("r1w2 chunk %6ld KB grid %6d  %7.2f us  %6.0f GB/s\n", C * 16 / 1024, gr, t, 3 * bytes / t / 1e3);
        t = time_it([&] { k_r1w2_chunk<8><<<gr, 256>>>(g, o, n4, C); }, 50);
        printf("r1w2 chunk U8 %6ld KB grid %6d  %7.2f us  %6.0f GB/s\n", C * 16 / 1024, gr, t, 3 * bytes / t / 1e3);
    }
    // occupancy: blocks (= waves per SIMD) per CU capped through dynamic LDS
    CK(hipFuncSetAttribute((const void*)k_r1w2_chunk<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)k_r1w2_chunk<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)k_r1w2_chunk<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    for (int bpc : {1, 2, 3, 4, 8}) {
        const size_t lds = bpc >= 8 ? 0 : size_t(160 * 1024 / bpc - 1024);
        const long C = 4096;
        const int gr = int((n4 + C - 1) / C);
        float t4 = time_it([&] { k_r1w2_chunk<4><<<gr, 256, lds>>>(g, o, n4, C); }, 30);
        float t8 = time_it([&] { k_r1w2_chunk<8><<<gr, 256, lds>>>(g, o, n4, C); }, 30);
        float t16 = time_it([&] { k_r1w2_chunk<16><<<gr, 256, lds>>>(g, o, n4, C); }, 30);
        CK(hipGetLastError());
        printf("r1w2 %d waves/SIMD: U4 %6.0f  U8 %6.0f  U16 %6.0f GB/s\n", bpc, 3 * bytes / t4 / 1e3,
               3 * bytes / t8 / 1e3, 3 * bytes / t16 / 1e3);
    }
    // the codec's step mix: read pass then r1w2 pass, alternating (MALL reuse of G)
    for (int gr : {4096, 8192}) {
        float t = time_it([&] {
            k_read<4><<<gr, 256>>>(g, sink, n4);
            k_r1w2<4, false><<<gr, 256>>>(g, o, n4);
        }, 50);
        printf("read+r1w2 grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 4 * bytes / t / 1e3);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
