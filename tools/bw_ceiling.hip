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

// the fused final pass's access pattern without its arithmetic: rows of m floats, row groups
// of T lanes (4 columns each, S segments of 4T columns), RB rows per group per batch, 256
// threads, `rows` rows per block; r1w2 on every element
template <int S, int RB>
__global__ __launch_bounds__(256) void k_r1w2_rows(float* __restrict__ g, float* __restrict__ out, int m, int T,
                                                   int rows, int n) {
    extern __shared__ float occ_rows[];  // dynamic LDS only caps blocks per CU
    if (rows < 0) occ_rows[threadIdx.x] = 0.f;
    const int tid = threadIdx.x, rg = tid / T, tt = tid - rg * T, RGS = 256 / T;
    const long row0 = long(blockIdx.x) * rows;
    for (int b = 0; b * RGS * RB < rows; ++b) {
        v4f x[RB][S];
#pragma unroll
        for (int u = 0; u < RB; ++u)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const long row = row0 + (long(b) * RGS + rg) * RB + u;
                const int c = (s * T + tt) * 4;
                x[u][s] = (row < n && c < m) ? *(const v4f*)(g + row * m + c) : v4f{0, 0, 0, 0};
            }
#pragma unroll
        for (int u = 0; u < RB; ++u)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const long row = row0 + (long(b) * RGS + rg) * RB + u;
                const int c = (s * T + tt) * 4;
                if (row < n && c < m) {
                    const v4f o = x[u][s] * 0.5f;
                    *(v4f*)(out + row * m + c) = o;
                    *(v4f*)(g + row * m + c) = x[u][s] - o;
                }
            }
    }
}

// the same pattern through buffer descriptors (the codec's loads/stores: raw buffer
// b128 with 32-bit byte offsets, rsrc word 3 = 0x00020000)
template <int S, int RB>
__global__ __launch_bounds__(256) void k_r1w2_rows_buf(float* __restrict__ g, float* __restrict__ out, int m, int T,
                                                       int rows, int n) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const int nbytes = int(long(n) * m * 4);
    const __amdgpu_buffer_rsrc_t gs = __builtin_amdgcn_make_buffer_rsrc(g, 0, nbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(out, 0, nbytes, 0x00020000);
    const int tid = threadIdx.x, rg = tid / T, tt = tid - rg * T, RGS = 256 / T;
    const long row0 = long(blockIdx.x) * rows;
    for (int b = 0; b * RGS * RB < rows; ++b) {
        v4u x[RB][S];
        unsigned off[RB][S];
#pragma unroll
        for (int u = 0; u < RB; ++u)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const long row = row0 + (long(b) * RGS + rg) * RB + u;
                const int c = (s * T + tt) * 4;
                off[u][s] = (row < n && c < m) ? unsigned((row * m + c) * 4) : 0x80000000u;
                x[u][s] = __builtin_amdgcn_raw_buffer_load_b128(gs, off[u][s], 0, 0);
            }
#pragma unroll
        for (int u = 0; u < RB; ++u)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                v4f xv = __builtin_bit_cast(v4f, x[u][s]);
                const v4f o = xv * 0.5f;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, o), os, off[u][s], 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, xv - o), gs, off[u][s], 0, 0);
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

// Even-product access pattern: one workgroup per tile of `rows` rows x 256 columns (64 lanes x
// 16 B) of an n x m fp32 matrix; wave w reads rows w, w + 4, ... with U rows in flight per lane
template <int U>
__global__ __launch_bounds__(256) void k_read_tiles(const float* __restrict__ g, float* out, int n, int m, int rows) {
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
// Row-major blocks: one workgroup per block of `rows` consecutive full rows, read as one
// contiguous range (the final pass's / a row-layout product's order)
template <int U>
__global__ __launch_bounds__(256) void k_read_rowblk(const v4f* __restrict__ g, float* out, long n4, long per) {
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
    {
        // (n, m, T, S) as the final pass's geometry picks them, ~100 MB each
        struct Case { int n, m, T, S; };
        const Case cs[] = {{49152, 512, 32, 4}, {49152, 512, 128, 1}, {5120, 4608, 256, 5}, {40960, 576, 32, 5},
                           {40960, 576, 256, 1}};
        for (const Case& c : cs) {
            for (int rows_blk : {16, 32, 64}) {
                const int rgs = 256 / c.T;
                const int rows = (rows_blk + 2 * rgs - 1) / (2 * rgs) * (2 * rgs);
                const int gr = (c.n + rows - 1) / rows;
                float* gf = (float*)g;
                float* of = (float*)o;
                float t = 0.f;
                switch (c.S) {
                    case 1: t = time_it([&] { k_r1w2_rows<1, 2><<<gr, 256>>>(gf, of, c.m, c.T, rows, c.n); }, 30); break;
                    case 4: t = time_it([&] { k_r1w2_rows<4, 2><<<gr, 256>>>(gf, of, c.m, c.T, rows, c.n); }, 30); break;
                    case 5: t = time_it([&] { k_r1w2_rows<5, 2><<<gr, 256>>>(gf, of, c.m, c.T, rows, c.n); }, 30); break;
                }
                CK(hipGetLastError());
                const double nb = 3.0 * c.n * double(c.m) * 4;
                printf("rows n %5d m %4d T %3d S %d rows/blk %3d grid %5d  %7.2f us  %6.0f GB/s\n", c.n, c.m, c.T, c.S,
                       rows, gr, t, nb / t / 1e3);
            }
        }
    }
    {
        float* gf = (float*)g;
        float* of = (float*)o;
        float t1 = time_it([&] { k_r1w2_rows_buf<4, 2><<<3072, 256>>>(gf, of, 512, 32, 16, 49152); }, 30);
        float t2 = time_it([&] { k_r1w2_rows_buf<5, 2><<<320, 256>>>(gf, of, 4608, 256, 16, 5120); }, 30);
        float t3 = time_it([&] { k_r1w2_rows<4, 2><<<3072, 256>>>(gf, of, 512, 32, 16, 49152); }, 30);
        float t4 = time_it([&] { k_r1w2_rows<5, 2><<<320, 256>>>(gf, of, 4608, 256, 16, 5120); }, 30);
        CK(hipGetLastError());
        printf("rows buffer ops: m512 T32 S4 %6.0f GB/s   m4608 T256 S5 %6.0f GB/s (global: %6.0f %6.0f)\n",
               3.0 * 49152 * 512 * 4 / t1 / 1e3, 3.0 * 5120 * 4608 * 4 / t2 / 1e3, 3.0 * 49152 * 512 * 4 / t3 / 1e3,
               3.0 * 5120 * 4608 * 4 / t4 / 1e3);
    }
    CK(hipFuncSetAttribute((const void*)k_r1w2_rows<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)k_r1w2_rows<5, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    for (int bpc : {1, 2, 3}) {
        const size_t lds = size_t(160 * 1024 / bpc - 1024);
        float* gf = (float*)g;
        float* of = (float*)o;
        float t1 = time_it([&] { k_r1w2_rows<4, 2><<<3072, 256, lds>>>(gf, of, 512, 32, 16, 49152); }, 30);
        float t2 = time_it([&] { k_r1w2_rows<5, 2><<<320, 256, lds>>>(gf, of, 4608, 256, 16, 5120); }, 30);
        CK(hipGetLastError());
        printf("rows %d waves/SIMD: m512 T32 S4 %6.0f GB/s   m4608 T256 S5 %6.0f GB/s\n", bpc,
               3.0 * 49152 * 512 * 4 / t1 / 1e3, 3.0 * 5120 * 4608 * 4 / t2 / 1e3);
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
    // COLD ceilings: 4 independent (G, out) pairs of the same size rotated per launch, so
    // between two uses of a pair ~600 MB stream through the chip (> the 256 MiB Infinity
    // Cache): the rate a step gets when the gradients arrive cold from a backward pass
    {
        constexpr int NS = 4;
        v4f *gs[NS], *os[NS];
        for (int i = 0; i < NS; ++i) {
            CK(hipMalloc(&gs[i], bytes));
            CK(hipMalloc(&os[i], bytes));
            CK(hipMemset(gs[i], 0, bytes));
            CK(hipMemset(os[i], 0, bytes));
        }
        int k = 0;
        for (int gr : {4096, 8192, 16384}) {
            float t;
            t = time_it([&] { k_read<8><<<gr, 256>>>(gs[k % NS], sink, n4); ++k; }, 40);
            printf("COLD read U8    grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, bytes / t / 1e3);
            t = time_it([&] { k_copy<4, false><<<gr, 256>>>(gs[k % NS], os[k % NS], n4); ++k; }, 40);
            printf("COLD copy       grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 2 * bytes / t / 1e3);
            t = time_it([&] { k_copy<4, true><<<gr, 256>>>(gs[k % NS], os[k % NS], n4); ++k; }, 40);
            printf("COLD copy nt    grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 2 * bytes / t / 1e3);
            t = time_it([&] { k_r1w2<4, false><<<gr, 256>>>(gs[k % NS], os[k % NS], n4); ++k; }, 40);
            printf("COLD r1w2       grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 3 * bytes / t / 1e3);
            t = time_it([&] { k_r1w2<4, true><<<gr, 256>>>(gs[k % NS], os[k % NS], n4); ++k; }, 40);
            printf("COLD r1w2 nt    grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 3 * bytes / t / 1e3);
        }
        for (int gr : {4096, 8192}) {
            float t = time_it([&] {
                k_read<4><<<gr, 256>>>(gs[k % NS], sink, n4);
                k_r1w2<4, false><<<gr, 256>>>(gs[k % NS], os[k % NS], n4);
                ++k;
            }, 40);
            printf("COLD read+r1w2  grid %5d  %7.2f us  %6.0f GB/s\n", gr, t, 4 * bytes / t / 1e3);
        }
        // even-product tile pattern vs contiguous row blocks, cold, 5120 x 4608 and 49152 x 512
        {
            struct Sh { int n, m; };
            for (Sh sh : {Sh{5120, 4608}, Sh{49152, 512}, Sh{20480, 1152}}) {
                for (int rows : {32, 64, 128}) {
                    const int nstrip = (sh.m + 255) / 256, nchunk = (sh.n + rows - 1) / rows;
                    const float* gf = (const float*)gs[k % NS];
                    float t = time_it([&] { k_read_tiles<4><<<nstrip * nchunk, 256>>>((const float*)gs[k % NS], sink, sh.n, sh.m, rows); ++k; }, 40);
                    (void)gf;
                    const double nb = double(sh.n) * sh.m * 4;
                    printf("COLD tiles n %5d m %4d rows %3d grid %6d  %7.2f us  %6.0f GB/s\n", sh.n, sh.m, rows,
                           nstrip * nchunk, t, nb / t / 1e3);
                    const long per = long(rows) * sh.m / 4;
                    const long n4s = long(sh.n) * sh.m / 4;
                    const int gr = int((n4s + per - 1) / per);
                    t = time_it([&] { k_read_rowblk<4><<<gr, 256>>>(gs[k % NS], sink, n4s, per); ++k; }, 40);
                    printf("COLD rowblk n %5d m %4d rows %3d grid %6d  %7.2f us  %6.0f GB/s\n", sh.n, sh.m, rows, gr, t,
                           nb / t / 1e3);
                }
            }
        }
        for (int i = 0; i < NS; ++i) {
            CK(hipFree(gs[i]));
            CK(hipFree(os[i]));
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
