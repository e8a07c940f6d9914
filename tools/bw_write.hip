// Write-only streaming ceiling (diagnostic tool, not part of the library): the access mix of
// k_lowrank_out (the W > 1 output pass: a rank-r product written over the gradient's shape),
// 102 MB like cfg2, under each store cache policy the library uses, several grid sizes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bw_write.hip -o tools/bw_write
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U, int AUX>
__global__ __launch_bounds__(256) void k_write(float* __restrict__ out, long n4, float a) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, int(n4 * 16 > 0x7fffffff ? 0x7fffffff : n4 * 16), 0x00020000);
    const long stride = long(gridDim.x) * 256;
    for (long b = long(blockIdx.x) * 256 + threadIdx.x; b < n4; b += stride * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + u * stride;
            if (i < n4) {
                const float v = a * float(i & 1023);
                const v4u x = {__float_as_uint(v), __float_as_uint(v + 1.f), __float_as_uint(v + 2.f),
                               __float_as_uint(v + 3.f)};
                __builtin_amdgcn_raw_buffer_store_b128(x, r, uint32_t(i * 16), 0, AUX);
            }
        }
    }
}

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));               \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

template <int U, int AUX>
float timeit(float* out, long n4, int grid, float* scratch, size_t sbytes) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 20; ++rep) {
        // evict: write a 512 MB scratch buffer between reps (cold Infinity Cache)
        (void)hipMemsetAsync(scratch, rep & 0xff, sbytes, 0);
        (void)hipEventRecord(e0, 0);
        k_write<U, AUX><<<grid, 256, 0, 0>>>(out, n4, 0.5f);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep >= 2 && ms < best) best = ms;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return best * 1e3f;
}

int main() {
    const long bytes = 102228128L / 16 * 16;
    const long n4 = bytes / 16;
    float *out, *scratch;
    const size_t sbytes = size_t(512) << 20;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&scratch, sbytes));
    const int grids[] = {1024, 2048, 4096, 8192, 16384};
    for (int gr : grids) {
        float t;
        t = timeit<4, 0>(out, n4, gr, scratch, sbytes);
        printf("write plain       U4 grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, bytes / t / 1e3);
        t = timeit<4, 2>(out, n4, gr, scratch, sbytes);
        printf("write nt          U4 grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, bytes / t / 1e3);
        t = timeit<4, 19>(out, n4, gr, scratch, sbytes);
        printf("write sc0|nt|sc1  U4 grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, bytes / t / 1e3);
        t = timeit<8, 19>(out, n4, gr, scratch, sbytes);
        printf("write sc0|nt|sc1  U8 grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, bytes / t / 1e3);
        t = timeit<4, 17>(out, n4, gr, scratch, sbytes);
        printf("write sc0|sc1     U4 grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, bytes / t / 1e3);
    }
    CK(hipFree(out));
    CK(hipFree(scratch));
    return 0;
}
