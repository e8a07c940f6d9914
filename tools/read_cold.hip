// Cold read ceilings of the even product's access patterns (diagnostic tool, not part of the
// library). Every timed launch reads a 102 MB buffer that has not been touched for >= 1 GB of
// other traffic (NS rotating sets, each 102 MB, with NS x 102 MB >> the 256 MB Infinity Cache),
// so no byte is an Infinity-Cache hit. Patterns, on an n x m fp32 matrix (m = 4608):
//   linear : grid-stride 16-byte loads, 8 in flight per lane
//   rowblk : one workgroup per block of consecutive full rows (the final pass's order)
//   tiles  : 32-row x 256-column tiles, chunk-major / strip-minor (the round-2 even product)
//   walk   : 512-thread workgroups, 2 or 4 per CU, each walks an equal (strip, row) range down
//            its strips with U rows in flight per lane (k_even)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/read_cold.hip -o tools/read_cold
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                   \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_linear(const v4f* __restrict__ g, float* out, long n4) {
    float s = 0.f;
    const long stride = long(gridDim.x) * 256;
    for (long b = long(blockIdx.x) * 256 + threadIdx.x; b < n4; b += stride * U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + stride * u;
            x[u] = i < n4 ? g[i] : v4f{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) s += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int U>
__global__ __launch_bounds__(256) void k_rowblk(const v4f* __restrict__ g, float* out, long n4, long per) {
    const long b0 = long(blockIdx.x) * per, b1 = b0 + per < n4 ? b0 + per : n4;
    float s = 0.f;
    for (long b = b0 + threadIdx.x; b < b1; b += 256L * U) {
        v4f x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = b + 256L * u;
            x[u] = i < b1 ? g[i] : v4f{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) s += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int U>
__global__ __launch_bounds__(256) void k_tiles(const float* __restrict__ g, float* out, int n, int m, int rows) {
    const int nstrip = (m + 255) / 256;
    const int strip = blockIdx.x % nstrip, chunk = blockIdx.x / nstrip;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = strip * 256 + 4 * lane;
    const int r0 = chunk * rows, r1 = min(n, r0 + rows);
    float s = 0.f;
    if (col < m) {
        for (int i = r0 + wave; i < r1; i += 4 * U) {
            v4f x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int rr = i + 4 * u;
                x[u] = rr < r1 ? *reinterpret_cast<const v4f*>(g + long(rr) * m + col) : v4f{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) s += x[u].x + x[u].y + x[u].z + x[u].w;
        }
    }
    if (s == 12345.f) out[threadIdx.x] = s;
}

// workgroup w reads the (strip, row) units [w * total / nwg, (w + 1) * total / nwg), strips
// in order, each strip's rows in order; 8 waves, row i of a strip to wave i % 8
template <int U>
__global__ __launch_bounds__(512) void k_walk(const float* __restrict__ g, float* out, int n, int m) {
    const int nstrip = m / 256;
    const long total = long(nstrip) * n;
    const long u0 = long(blockIdx.x) * total / gridDim.x, u1 = long(blockIdx.x + 1) * total / gridDim.x;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float s = 0.f;
    long u = u0;
    while (u < u1) {
        const int strip = int(u / n);
        const long rb = u % n;
        const long re = (u1 - long(strip) * n) < n ? (u1 - long(strip) * n) : n;
        const float* base = g + strip * 256 + 4 * lane;
        for (long i = rb + wave; i < re; i += 8 * U) {
            v4f x[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const long rr = i + 8 * k;
                x[k] = *reinterpret_cast<const v4f*>(base + (rr < re ? rr : rb) * m);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) s += x[k].x + x[k].y + x[k].z + x[k].w;
        }
        u += re - rb;
    }
    if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
    const int m = 4608, n = 5547;  // 102.2 MB fp32
    const long elems = long(n) * m, n4 = elems / 4;
    constexpr int NS = 12;          // 1.2 GB of sets: every timed read is cold
    std::vector<float*> gs(NS);
    float* sink;
    for (int i = 0; i < NS; ++i) {
        CK(hipMalloc(&gs[i], elems * 4));
        CK(hipMemset(gs[i], 0, elems * 4));
    }
    CK(hipMalloc(&sink, 4096));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int k = 0;
    auto time_it = [&](auto launch, int reps) {
        for (int i = 0; i < NS; ++i) launch();  // warm-up round
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        for (int i = 0; i < reps; ++i) launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        return ms * 1000.f / reps;
    };
    auto report = [&](const char* what, float us) {
        printf("%-44s %8.2f us  %6.0f GB/s\n", what, us, double(elems) * 4 / (us * 1e-6) / 1e9);
    };
    char name[128];
    for (int gr : {2048, 4096, 8192}) {
        snprintf(name, sizeof name, "linear U8 grid %d", gr);
        report(name, time_it([&] { k_linear<8><<<gr, 256>>>((const v4f*)gs[k++ % NS], sink, n4); }, 48));
    }
    for (int rows : {8, 16, 32}) {
        const long per = long(rows) * m / 4;
        const int gr = int((n4 + per - 1) / per);
        snprintf(name, sizeof name, "rowblk %d rows grid %d", rows, gr);
        report(name, time_it([&] { k_rowblk<4><<<gr, 256>>>((const v4f*)gs[k++ % NS], sink, n4, per); }, 48));
    }
    for (int rows : {32, 64}) {
        const int gr = (m / 256) * ((n + rows - 1) / rows);
        snprintf(name, sizeof name, "tiles %d rows grid %d", rows, gr);
        report(name, time_it([&] { k_tiles<4><<<gr, 256>>>(gs[k++ % NS], sink, n, m, rows); }, 48));
    }
    for (int wpc : {2, 3, 4}) {
        snprintf(name, sizeof name, "walk U4 %d wg/CU", wpc);
        report(name, time_it([&] { k_walk<4><<<256 * wpc, 512>>>(gs[k++ % NS], sink, n, m); }, 48));
        snprintf(name, sizeof name, "walk U8 %d wg/CU", wpc);
        report(name, time_it([&] { k_walk<8><<<256 * wpc, 512>>>(gs[k++ % NS], sink, n, m); }, 48));
    }
    // the same patterns over 4 rotating sets (408 MB: partly Infinity-Cache resident)
    {
        int k4 = 0;
        auto t4 = [&](auto launch) {
            for (int i = 0; i < 8; ++i) launch();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(a);
            for (int i = 0; i < 48; ++i) launch();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, a, b);
            return ms * 1000.f / 48;
        };
        report("4-set linear U8 grid 4096", t4([&] { k_linear<8><<<4096, 256>>>((const v4f*)gs[k4++ % 4], sink, n4); }));
        report("4-set walk U4 4 wg/CU", t4([&] { k_walk<4><<<1024, 512>>>(gs[k4++ % 4], sink, n, m); }));
    }
    return 0;
}
