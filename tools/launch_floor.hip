// Per-launch floor of a chain of dependent kernels (diagnostic tool, not part of the library):
// what a small plan's step (cfg5: seven dependent launches on 8 MB) cannot go below however
// fast each kernel's own work is. Each launch reads a small buffer the previous launch wrote
// (one dependent memory round trip through L2/MALL) and writes its own; 7 launches per step,
// 200 steps back to back on one stream, timed with events.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_empty() {}

// read n floats the previous launch wrote, write n floats for the next one
__global__ __launch_bounds__(256) void k_hop(const float* __restrict__ in, float* __restrict__ out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[i] * 0.5f + 1.f;
}

// the same plus a streaming read of `bytes_per_wg` per workgroup (a small plan's share)
__global__ __launch_bounds__(256) void k_hop_stream(const float* __restrict__ in, float* __restrict__ out, int n,
                                                    const float4* __restrict__ g, int per_wg4) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    float s = 0.f;
    const float4* p = g + size_t(blockIdx.x) * per_wg4;
    for (int k = threadIdx.x; k < per_wg4; k += 256) {
        const float4 v = p[k];
        s += v.x + v.y + v.z + v.w;
    }
    if (i < n) out[i] = in[i] * 0.5f + (s == 12345.f ? 1.f : 0.f);
}

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                        \
        }                                                                    \
    } while (0)

int main() {
    constexpr int kLaunches = 7, kSteps = 200;
    const int grids[] = {64, 256, 1024};
    float *a, *b, *g;
    const int n = 1 << 20;
    const size_t gbytes = size_t(8) << 20;  // cfg5's 8 MB gradient
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&g, gbytes));
    CK(hipMemset(a, 0, n * 4));
    CK(hipMemset(b, 0, n * 4));
    CK(hipMemset(g, 0, gbytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 3; ++mode) {
        for (int gr : grids) {
            const int nn = gr * 256;
            const int per_wg4 = int(gbytes / 16 / gr);
            auto step = [&]() {
                for (int l = 0; l < kLaunches; ++l) {
                    float* in = (l & 1) ? b : a;
                    float* out = (l & 1) ? a : b;
                    if (mode == 0)
                        k_empty<<<gr, 256>>>();
                    else if (mode == 1)
                        k_hop<<<gr, 256>>>(in, out, nn);
                    else
                        k_hop_stream<<<gr, 256>>>(in, out, nn, reinterpret_cast<const float4*>(g), per_wg4);
                }
            };
            for (int w = 0; w < 20; ++w) step();
            CK(hipEventRecord(e0, 0));
            for (int s = 0; s < kSteps; ++s) step();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const float us_launch = ms * 1e3f / (kSteps * kLaunches);
            const char* name = mode == 0 ? "empty" : mode == 1 ? "hop (1 dependent round trip)" : "hop + 8 MB read";
            printf("%-30s grid %5d: %6.2f us per launch, %6.2f us per 7-launch step\n", name, gr, us_launch,
                   us_launch * kLaunches);
        }
    }
    return 0;
}
