// Read-once / write-twice streaming rate by row-segment width (diagnostic tool, not part of the
// library): k_apply on bf16 gradients (cfg4: 4096 x 11008 and 4096 x 4096, one read of G, the
// residual written in place, the output written to a second buffer) reaches 0.68-0.71 of 8 TB/s
// where the fp32 form reaches 0.78. A bf16 lane owns 4 columns = 8 bytes, so one wave
// instruction covers a 512-byte segment of a row where fp32 covers 1 KB. This probe streams the
// same bytes (cold: 4 rotating buffer sets) with
//   seg512   lane = 8 B,  one instruction per 512-byte row segment      (bf16 k_apply today)
//   seg1k    lane = 16 B, one instruction per 1 KB segment               (fp32 k_apply)
//   seg1k2   lane = 2 x 8 B, two instructions covering one 1 KB segment   (bf16, paired columns)
// tiles of 64 rows x one segment per 256-thread block, U rows in flight per lane, rows of
// `rowbytes` bytes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/seg_r1w2.hip -o tools/seg_r1w2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
constexpr int U = 4;

// MODE 0: 8 B per lane (512 B / instruction); 1: 16 B per lane (1 KB); 2: two 8 B (1 KB, 2 instr)
template <int MODE>
__global__ __launch_bounds__(256) void k_seg(char* g, char* out, long rows, long rowbytes) {
    constexpr long seg = MODE == 0 ? 512 : 1024;
    const long segs = rowbytes / seg;
    const long tile = blockIdx.x, s = tile % segs, chunk = tile / segs;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long r0 = chunk * 64 + wave * 16;
    for (int rb = 0; rb < 16; rb += U) {
        if constexpr (MODE == 1) {
            v4u x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = *(const v4u*)(g + (r0 + rb + u) * rowbytes + s * seg + lane * 16);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long o = (r0 + rb + u) * rowbytes + s * seg + lane * 16;
                v4u y = x[u] + 1u;
                __builtin_nontemporal_store(y, (v4u*)(g + o));
                __builtin_nontemporal_store(x[u], (v4u*)(out + o));
            }
        } else {
            constexpr int H = MODE == 2 ? 2 : 1;
            v2u x[U][H];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int h = 0; h < H; ++h)
                    x[u][h] = *(const v2u*)(g + (r0 + rb + u) * rowbytes + s * seg + h * 512 + lane * 8);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int h = 0; h < H; ++h) {
                    const long o = (r0 + rb + u) * rowbytes + s * seg + h * 512 + lane * 8;
                    v2u y = x[u][h] + 1u;
                    __builtin_nontemporal_store(y, (v2u*)(g + o));
                    __builtin_nontemporal_store(x[u][h], (v2u*)(out + o));
                }
        }
    }
}

int main() {
    // cfg4's larger matrix: 4096 rows x 11008 bf16 (22016 B); rows padded to a 1 KB multiple
    const long rows = 5632, rowbytes = 22528;  // ~127 MB per buffer (cfg4: 124 MB of bf16 gradient)
    const long bytes = rows * rowbytes;
    constexpr int SETS = 4;
    std::vector<char*> g(SETS), o(SETS);
    for (int k = 0; k < SETS; ++k) {
        CK(hipMalloc(&g[k], bytes));
        CK(hipMalloc(&o[k], bytes));
        CK(hipMemset(g[k], 1, bytes));
        CK(hipMemset(o[k], 0, bytes));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto kern, long seg) {
        const long tiles = (rows / 64) * (rowbytes / seg);
        for (int w = 0; w < 8; ++w) kern<<<tiles, 256>>>(g[w % SETS], o[w % SETS], rows, rowbytes);
        CK(hipDeviceSynchronize());
        constexpr int N = 40;
        CK(hipEventRecord(e0));
        for (int i = 0; i < N; ++i) kern<<<tiles, 256>>>(g[i % SETS], o[i % SETS], rows, rowbytes);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / N;
        std::printf("%-8s %8.1f us per pass, %7.1f GB/s r1w2 (%.3f of 8 TB/s), %ld tiles\n", name, us,
                    3.0 * bytes / (us * 1e3), 3.0 * bytes / (us * 1e3) / 8000.0, tiles);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("seg512", k_seg<0>, 512);
        run("seg1k", k_seg<1>, 1024);
        run("seg1k2", k_seg<2>, 1024);
    }
    return 0;
}
