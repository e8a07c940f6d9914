// Read-bandwidth microbenchmark for the two gradient access shapes of the products
// (diagnostic tool, not part of the library):
//   ROW  : a wave-instruction reads 1 KB of ONE row (64 lanes x 16 B)       [even product, apply]
//   MFMA : a wave-instruction reads 64 B of each of 16 rows (lane = ri + 16 cq) [odd MFMA A-operand]
// Tiles of 64 rows x 256 columns, 256 threads (4 waves x 16 rows); U = 16-byte loads in
// flight per lane before they are consumed.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/read_patterns.hip -o tools/read_patterns
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_row(const float* __restrict__ g, float* out, int n, int m) {
    const int strips = m / 256;
    const int tile = blockIdx.x, strip = tile % strips, chunk = tile / strips;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float* base = g + (size_t)(chunk * 64 + wave * 16) * m + strip * 256 + lane * 4;
    float s = 0.f;
    for (int r0 = 0; r0 < 16; r0 += U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = *(const v4f*)(base + (size_t)(r0 + u) * m);
#pragma unroll
        for (int u = 0; u < U; ++u) s += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int U>
__global__ __launch_bounds__(256) void k_mfma(const float* __restrict__ g, float* out, int n, int m) {
    const int strips = m / 256;
    const int tile = blockIdx.x, strip = tile % strips, chunk = tile / strips;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ri = lane & 15, cq = lane >> 4;
    const float* base = g + (size_t)(chunk * 64 + wave * 16 + ri) * m + strip * 256 + cq * 4;
    float s = 0.f;
    for (int j0 = 0; j0 < 256; j0 += 16 * U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = *(const v4f*)(base + j0 + 16 * u);
#pragma unroll
        for (int u = 0; u < U; ++u) s += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    if (s == 12345.f) out[threadIdx.x] = s;
}

// MFMA layout but each lane covers 64 contiguous bytes of its row (4 consecutive 16-B
// loads): lane (ri, cq) reads columns 64 cq + 16 u .. (k-step mapping permuted).
template <int U>
__global__ __launch_bounds__(256) void k_mfma_perm(const float* __restrict__ g, float* out, int n, int m) {
    const int strips = m / 256;
    const int tile = blockIdx.x, strip = tile % strips, chunk = tile / strips;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ri = lane & 15, cq = lane >> 4;
    const float* base = g + (size_t)(chunk * 64 + wave * 16 + ri) * m + strip * 256 + cq * 64;
    float s = 0.f;
    for (int j0 = 0; j0 < 64; j0 += 4 * U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = *(const v4f*)(base + j0 + 4 * u);
#pragma unroll
        for (int u = 0; u < U; ++u) s += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    if (s == 12345.f) out[threadIdx.x] = s;
}

__global__ void k_touch(const v4f* __restrict__ p, size_t n, float* out) {  // read-only flush
    v4f s = {0.f, 0.f, 0.f, 0.f};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i];
    if (s.x == 12345.f) out[0] = s.y;
}

template <typename P, typename F>
float best_us(P pre, F launch) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int rep = 0; rep < 30; ++rep) {
        pre();
        (void)hipEventRecord(e0, 0);
        launch();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 2 && ms < best) best = ms;
    }
    return best * 1e3f;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2048;
    const int m = argc > 2 ? atoi(argv[2]) : 12288;
    const size_t bytes = (size_t)n * m * 4;
    float *g, *out, *flush;
    (void)hipMalloc(&g, bytes);
    (void)hipMalloc(&out, 4096);
    (void)hipMalloc(&flush, 512 << 20);
    (void)hipMemset(g, 0, bytes);
    const int tiles = (n / 64) * (m / 256);
    (void)hipMemset(flush, 0, 512 << 20);
    (void)hipDeviceSynchronize();
    auto run = [&](const char* name, auto kern) {
        const float cold = best_us([&] { hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, 0,
                                                            (const v4f*)flush, (size_t(512) << 20) / 16, out); },
                                   [&] { hipLaunchKernelGGL(kern, dim3(tiles), dim3(256), 0, 0, g, out, n, m); });
        const float warm = best_us([&] {}, [&] { hipLaunchKernelGGL(kern, dim3(tiles), dim3(256), 0, 0, g, out, n, m); });
        printf("%-16s cold %8.2f us %7.1f GB/s | back-to-back %8.2f us %7.1f GB/s\n", name, cold,
               bytes / (cold * 1e3), warm, bytes / (warm * 1e3));
    };
    run("row U=4", k_row<4>);
    run("row U=8", k_row<8>);
    run("row U=16", k_row<16>);
    run("mfma U=4", k_mfma<4>);
    run("mfma U=8", k_mfma<8>);
    run("mfma U=16", k_mfma<16>);
    run("mfma_perm U=4", k_mfma_perm<4>);
    run("mfma_perm U=16", k_mfma_perm<16>);
    return 0;
}
