// Streaming kernels of the PowerSGD hot path, written for CDNA4 (gfx950, wave64).
//
// k_apply (and the odd lane-column product) walk lane-column tiles: a tile is (matrix, column
// strip, row chunk) and inside a 256-thread workgroup every lane OWNS V consecutive columns
// (V = 4 -> 16-byte fp32 / 8-byte bf16 vector loads) while the 4 waves x RW row phases walk
// the chunk's rows. A wave-instruction reads L*V*sizeof(T) contiguous bytes of one row
// (L = lanes per row, up to 64 -> 1 KiB). Q-layout factor values ([m, r], per column) stay
// in registers for the whole tile; P-layout values ([n, r], per row) are broadcast loads.
//
//   k_product<ODD>    reference powersgd.py:185-202, P = Gk Q: a row layout with a lane
//     reduce-scatter on full-width strips (r <= 4), lane-column tiles with lane sums on narrow
//     ones; k_odd_mfma (matrix cores, below) for r 5-16. The even product Q = Gk^T P is the
//     persistent k_even (psgd_even.cuh).
//     Gk = G0 - sum_{j<k} P_j Q_j^T is formed ON THE FLY from the untouched gradient (the
//     reference's baddbmm_, :195-202, element by element), so an iteration reads the
//     gradient once and writes nothing back.
//   k_apply           reference powersgd.py:195-230, all iterations at once:
//     residual = G0 - sum_k P_k Q_k^T (local factors)  -> written over the gradient,
//     output   = sum_k alpha P_k Qbar_k^T              -> written to the flat output.
//     One read + two writes per element: the only pass that writes matrix-sized data.
//
// Codegen rules applied throughout (see cdna_hip_programming.md): every global pointer is
// cast to address space 1 (global_load/store, not flat_*); loads are unconditional from
// clamped in-range addresses and masked with selects afterwards (no exec-mask branch per
// load); cross-lane sums use DPP row rotations and the gfx950 permlane16/32 swaps.
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "psgd_internal.h"

namespace psgd {

#define PSGD_G __attribute__((address_space(1)))
template <typename T>
using gptr = PSGD_G T*;

template <typename T>
__device__ __forceinline__ gptr<const T> gconst(const void* p) {
    return (gptr<const T>)(static_cast<const T*>(p));
}
template <typename T>
__device__ __forceinline__ gptr<T> gmut(void* p) {
    return (gptr<T>)(static_cast<T*>(p));
}

using bf16_t = uint16_t;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
    return __bfloat16_as_ushort(__float2bfloat16(f));  // RNE, NaN preserving (v_cvt_pk_bf16_f32)
}

// Pin a loaded value: an empty asm that consumes it. Issued after a batch of loads, it stops
// LLVM from sinking a load into the branch of the select that masks it (which costs an
// exec-mask branch and a vmcnt(0) wait per load).
__device__ __forceinline__ void keep(float& v) { asm volatile("" : "+v"(v)); }

// A store into this rank's IPC exchange slot (psgd_aggregate_ipc), which peers read over xGMI
// with system-scope loads after this kernel has completed and k_xchg has raised the epoch flag.
// System scope lowers to a vector `global_store_dword ... sc0 sc1`: write-through, the line
// leaves (is dropped from) this XCD's L2 (MI355X_MICROARCH.md, the store-flavour row of the
// visibility table), so the peer's read never depends on a writeback of the eight L2s at kernel
// end. The flat region is written through with kStAuxSlot (sc0 | sc1) for the same reason.
__device__ __forceinline__ void st_slot(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Streaming outputs (residual, output, flat pack) go through buffer descriptors with an explicit
// cache policy (gfx950 CPol bits: sc0 = 1, nt = 2, sc1 = 16). Default sc0 | nt | sc1: the
// 200+ MB a final pass writes must not sit dirty in the Infinity Cache, where the NEXT step's
// cold gradient reads would pay for their write-back: the following even product ran 30 -> 23.6
// us, and the rank-4 final pass itself 60 -> 53 us, against nt alone (profiles/r03/st_aux.txt;
// plain stores were worse still, 33 us). Build-time knob for A/B runs.
#ifndef PSGD_ST_AUX
#define PSGD_ST_AUX 19
#endif
// The output stores (the averaged gradient the optimizer reads next) of the fused world-size-1
// final pass of LARGE plans take nt alone (FinalArgs::out_nt, chosen by the plan): measured
// against sc0 | nt | sc1 (profiles/r04/g, r04/h), cfg2 cold 0.082 -> 0.076 ms, warm and
// post-backward likewise faster, cfg3 and cfg4 unchanged; the small plans (cfg1, cfg5:
// everything fits the Infinity Cache) were 2-4 % slower with it and keep the write-through
// policy. Plain stores sat between the two. The residual (read again only after the next
// backward pass) always streams write-through, and so do k_apply and k_lowrank_out: nt made the
// write-only k_lowrank_out slower (19.6 -> 23.0 us, cfg2 W > 1), and k_apply's run-time choice
// cost a wave per SIMD of occupancy for no measured gain (profiles/r04/o).
constexpr int kStAuxOutNt = 2;
// The flat buffer of the uncompressed tensors is, at world size > 1 over the IPC exchange, this
// rank's exchange slot that peers read over xGMI: its stores keep a fixed write-through policy
// (sc0 | sc1, no nt: MI355X_MICROARCH.md, never nt on hand-off stores), independent of the
// PSGD_ST_AUX build knob, so no A/B build can hand peers stale bytes.
constexpr int kStAuxSlot = 17;
static_assert((kStAuxSlot & 17) == 17, "IPC exchange slot stores (flat region) must be write-through: sc0 | sc1");
// A kernel launch that honours g_kernel_timing (psgd_internal.h)
template <typename... Args>
inline void timed_launch(void (*k)(Args...), dim3 grid, dim3 block, hipStream_t s, Args... args) {
    if (g_kernel_timing)
        hipExtLaunchKernelGGL(k, grid, block, 0, s, g_kernel_timing->start, g_kernel_timing->stop, 0, args...);
    else
        hipLaunchKernelGGL(k, grid, block, 0, s, args...);
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOob = 0x80000000u;  // beyond every descriptor (num_records < 2^31)

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, int(bytes), 0x00020000);
}

template <typename T>
struct StIo;

template <>
struct StIo<float> {
    template <int AUX = PSGD_ST_AUX>
    static __device__ __forceinline__ void st4(rsrc_t r, uint32_t off, const float (&v)[4]) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u x = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
        __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, AUX);
    }
    template <int AUX = PSGD_ST_AUX>
    static __device__ __forceinline__ void st1(rsrc_t r, uint32_t off, float v) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, AUX);
    }
};

template <>
struct StIo<bf16_t> {
    template <int AUX = PSGD_ST_AUX>
    static __device__ __forceinline__ void st4(rsrc_t r, uint32_t off, const float (&v)[4]) {
        typedef unsigned v2u_ __attribute__((ext_vector_type(2)));
        const v2u_ x = {uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16),
                        uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16)};
        __builtin_amdgcn_raw_buffer_store_b64(x, r, off, 0, AUX);
    }
    template <int AUX = PSGD_ST_AUX>
    static __device__ __forceinline__ void st1(rsrc_t r, uint32_t off, float v) {
        __builtin_amdgcn_raw_buffer_store_b16(f2bf(v), r, off, 0, AUX);
    }
};
// V consecutive elements at byte offset `off` of descriptor r
template <typename T, int AUX = PSGD_ST_AUX>
__device__ __forceinline__ void st_vec(rsrc_t r, uint32_t off, const float (&v)[4]) {
    StIo<T>::template st4<AUX>(r, off, v);
}
template <typename T, int AUX = PSGD_ST_AUX>
__device__ __forceinline__ void st_vec(rsrc_t r, uint32_t off, const float (&v)[1]) {
    StIo<T>::template st1<AUX>(r, off, v[0]);
}

template <typename T>
struct Io;

template <>
struct Io<float> {
    static __device__ __forceinline__ void ld(gptr<const float> p, float (&v)[4]) {
        const v4f x = *(gptr<const v4f>)p;
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
    static __device__ __forceinline__ void ld(gptr<const float> p, float (&v)[1]) { v[0] = *p; }
};

template <>
struct Io<bf16_t> {
    static __device__ __forceinline__ void ld(gptr<const bf16_t> p, float (&v)[4]) {
        const v2u x = *(gptr<const v2u>)p;
        v[0] = __uint_as_float(x.x << 16);
        v[1] = __uint_as_float(x.x & 0xffff0000u);
        v[2] = __uint_as_float(x.y << 16);
        v[3] = __uint_as_float(x.y & 0xffff0000u);
    }
    static __device__ __forceinline__ void ld(gptr<const bf16_t> p, float (&v)[1]) { v[0] = bf2f(*p); }
};

// r (<= R) consecutive fp32 factor values, zeros for c >= r. When r == R the row start is
// R-aligned (every panel offset is a multiple of r): vector loads for R in {2, 4, 8}.
template <int R>
__device__ __forceinline__ void ld_factor(gptr<const float> p, int r, float (&v)[R]) {
    if constexpr (R == 1) {
        v[0] = p[0];
    } else {
        if (r == R) {
            if constexpr (R % 4 == 0) {
#pragma unroll
                for (int c = 0; c < R; c += 4) {
                    const v4f x = *(gptr<const v4f>)(p + c);
                    v[c] = x.x; v[c + 1] = x.y; v[c + 2] = x.z; v[c + 3] = x.w;
                }
            } else if constexpr (R == 2) {
                const v2f x = *(gptr<const v2f>)p;
                v[0] = x.x; v[1] = x.y;
            } else {
#pragma unroll
                for (int c = 0; c < R; ++c) v[c] = p[c];
            }
        } else {
#pragma unroll
            for (int c = 0; c < R; ++c) v[c] = p[c < r ? c : 0];
#pragma unroll
            for (int c = 0; c < R; ++c) {
                keep(v[c]);
                v[c] = c < r ? v[c] : 0.f;
            }
        }
    }
}

// sum_c a[c] * b[c] as an fma chain in c order (the order of a rank-r dot of one output
// element in the reference's batched GEMM).
template <int R>
__device__ __forceinline__ float dotr(const float (&a)[R], const float (&b)[R]) {
    float t = a[0] * b[0];
#pragma unroll
    for (int c = 1; c < R; ++c) t = fmaf(a[c], b[c], t);
    return t;
}

// ------------------------------------------------------------ cross-lane sums -------
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// Coset all-reduce steps: v + v(partner at distance s). Rotations within 16-lane rows
// (row_ror) are equivalent to xor-partners once applied for every power of two up to 8;
// s = 16 / 32 use the gfx950 half-exchanges. `on` is wave-uniform: a disabled step is a
// select, not a branch, so independent sums interleave freely.
__device__ __forceinline__ float swap16_sum(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
__device__ __forceinline__ float swap32_sum(float v) {
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// sum over the lanes that share lane / L (aligned groups of L lanes); L = 1..64, power of
// 2. Groups smaller than a 16-lane row need partners INSIDE the group: quad_perm xor 1 /
// xor 2, then row_half_mirror (l -> 7 - l) and row_mirror (l -> 15 - l), whose partner lies
// in the other half of the 8 / 16 group (all of whose lanes already hold the same sum).
__device__ __forceinline__ float sum_within(float v, int L) {
    float t;
    t = v + dpp<0xB1>(v);  v = L > 1 ? t : v;   // quad_perm [1,0,3,2]
    t = v + dpp<0x4E>(v);  v = L > 2 ? t : v;   // quad_perm [2,3,0,1]
    t = v + dpp<0x141>(v); v = L > 4 ? t : v;   // row_half_mirror
    t = v + dpp<0x140>(v); v = L > 8 ? t : v;   // row_mirror
    t = swap16_sum(v);     v = L > 16 ? t : v;
    t = swap32_sum(v);     v = L > 32 ? t : v;
    return v;
}
// sum over the lanes that share lane % L (partners lane ^ s, L <= s < 64)
__device__ __forceinline__ float sum_across(float v, int L) {
    float t;
    t = v + dpp<0x121>(v); v = L <= 1 ? t : v;
    t = v + dpp<0x122>(v); v = L <= 2 ? t : v;
    t = v + dpp<0x124>(v); v = L <= 4 ? t : v;
    t = v + dpp<0x128>(v); v = L <= 8 ? t : v;
    t = swap16_sum(v);     v = L <= 16 ? t : v;
    t = swap32_sum(v);     v = L <= 32 ? t : v;
    return v;
}

// All-reduce of one float over the 64 lanes: 4 DPP row rotations (within rows of 16 lanes),
// then the gfx950 half-exchanges v_permlane16_swap / v_permlane32_swap. No LDS traffic.
__device__ __forceinline__ float wave_allsum(float v) {
    v += dpp<0x128>(v);  // row_ror:8
    v += dpp<0x124>(v);  // row_ror:4
    v += dpp<0x122>(v);  // row_ror:2
    v += dpp<0x121>(v);  // row_ror:1
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Joint norm of a rank-1 group from per-item sums of squares (reference
// orthogonalization.py:5-6: max(||x||, eps)); every wave that evaluates it uses the same
// fixed order (lane-strided partial sums, then the DPP/permlane wave tree), so all agree
// bitwise. Group g's items are grng[2g] .. grng[2g+1].
__device__ __forceinline__ float group_norm_ss(const float* ss, const int32_t* grng, int group) {
    const int lane = threadIdx.x & 63;
    const int b = grng[2 * group], e = grng[2 * group + 1];
    float acc = 0.f;
    for (int i = b + lane; i < e; i += 64) acc += ss[i];
    const float nrm = sqrtf(wave_allsum(acc));
    return nrm > 1e-16f ? nrm : 1e-16f;
}

// Plain sum of the sum-of-squares partials [rng[2 i], rng[2 i + 1]) (same wave order as
// group_norm_ss; one matrix's items for the rank-1 projection form)
__device__ __forceinline__ float range_ss(const float* ss, const int32_t* rng, int i) {
    const int lane = threadIdx.x & 63;
    const int b = rng[2 * i], e = rng[2 * i + 1];
    float acc = 0.f;
    for (int k = b + lane; k < e; k += 64) acc += ss[k];
    return wave_allsum(acc);
}

// One flat-pack item (kFlatItem consecutive elements of one uncompressed tensor; reference
// powersgd.py:22-31 + utils.py:6-10, :43-49): flat = x / W (division, as div_; an exact
// copy at W = 1), then x = 0. NT threads; one read + two writes per element.
template <typename T, int NT>
__device__ __forceinline__ void flat_pack_item(const FlatArgs& a, int item) {
    constexpr int PER = kFlatItem / NT;
    const FlatItem it = a.items[item];
    const FlatEntry en = a.entries[it.entry];
    const gptr<T> x = gmut<T>(a.tensors[en.tensor]);
    // this item's ranges of the tensor and of the flat buffer (stores past them drop)
    const uint32_t nb = uint32_t((en.numel - it.start < kFlatItem ? en.numel - it.start : kFlatItem) * sizeof(T));
    const rsrc_t rx = make_rsrc(static_cast<T*>(a.tensors[en.tensor]) + it.start, nb);
    const rsrc_t rf = make_rsrc(static_cast<T*>(a.flat) + en.off + it.start, nb);
    const float w = float(a.world);
    float v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int64_t j = it.start + int64_t(q) * NT + threadIdx.x;
        float t[1];
        Io<T>::ld(x + (j < en.numel ? j : 0), t);  // clamped, unconditional
        v[q] = t[0];
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) keep(v[q]);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int64_t j = it.start + int64_t(q) * NT + threadIdx.x;
        if (j < en.numel) {
            const uint32_t off = uint32_t(int64_t(q) * NT + threadIdx.x) * uint32_t(sizeof(T));
            StIo<T>::template st1<kStAuxSlot>(rf, off, a.world != 1 ? v[q] / w : v[q]);
            StIo<T>::st1(rx, off, 0.f);
        }
    }
}

struct TileGeom {
    int lane, wave, L, sub, ql;
    int64_t n, m, row_begin, row_end, first_row;
    int32_t col0, ccol;  // this lane's first column; clamped copy that is always in range
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
    g.col0 = (t.strip * g.L + g.ql) * V;
    g.active = g.col0 < g.m;  // V == 4 only when m % 4 == 0: the whole vector is in range
    g.ccol = g.active ? g.col0 : 0;
    g.row_begin = int64_t(t.chunk) * d.chunk_rows;
    g.row_end = g.n < g.row_begin + d.chunk_rows ? g.n : g.row_begin + d.chunk_rows;
    g.stride = kWaves * rw;
    g.first_row = g.row_begin + g.wave * rw + g.sub;
    return g;
}

constexpr int kUnroll = 4;  // rows in flight per lane (k_apply, odd lane-column product)

// ------------------------------------------------- odd product, row layout (VALU) --
// For full-width strips (256 columns = 64 lanes x 4) and r <= 4: a wave takes 16 rows; each
// wave-instruction reads 1 KB of ONE row; lane l forms the r partial dots of its 4 columns
// for each row (16 r values), and a butterfly REDUCE-SCATTER over the 64 lanes leaves every
// lane with the total of one (row, column) item. Halving step on lane bit b: the value list
// is split in halves (a = first, b = second); lanes with bit b = 0 keep a, the others keep
// b, and each receives its partner's copy of the half it keeps. Bits 5 and 4 use the gfx950
// half-row swaps (v_permlane32_swap / v_permlane16_swap: one instruction per pair), bit 3
// DPP row_ror:8 (= xor 8), bit 2 row_ror:12 / row_ror:4 (the partner above / below), bits 1
// and 0 DPP quad_perm xor patterns. ~40 VALU per 16 rows at r = 1, against 16 dependent
// 16x16x4 MFMAs of which 15/16 of the columns are padding.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
constexpr int kDppXor1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;  // quad_perm [2,3,0,1]

template <int NV>
__device__ __forceinline__ void halve_swap32(float (&v)[NV]) {
#pragma unroll
    for (int i = 0; i < NV / 2; ++i) {
        const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + NV / 2]), false, false);
        v[i] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
}
template <int NV>
__device__ __forceinline__ void halve_swap16(float (&v)[NV]) {
#pragma unroll
    for (int i = 0; i < NV / 2; ++i) {
        const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + NV / 2]), false, false);
        v[i] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
}
// lane bit B in {0, 1, 2, 3}: DPP partner exchange inside 16-lane rows
template <int NV, int B>
__device__ __forceinline__ void halve_dpp(float (&v)[NV], int lane) {
    const bool hi = (lane >> B) & 1;
#pragma unroll
    for (int i = 0; i < NV / 2; ++i) {
        const float a = v[i], b = v[i + NV / 2];
        const float kept = hi ? b : a, send = hi ? a : b;
        float recv;
        if constexpr (B == 3) recv = dppf<0x128>(send);                      // row_ror:8
        else if constexpr (B == 2) {
            // row_ror:N delivers lane (l - N) mod 16: low lanes take l + 4 (ror 12), high
            // ones l - 4 (ror 4). Both moves must run with every lane active (a DPP read
            // from a disabled lane yields 0): pinned before the select, so the compiler
            // cannot turn the select into a divergent branch around them.
            float r4 = dppf<0x124>(send), r12 = dppf<0x12C>(send);
            keep(r4);
            keep(r12);
            recv = hi ? r4 : r12;
        }
        else if constexpr (B == 1) recv = dppf<kDppXor2>(send);
        else recv = dppf<kDppXor1>(send);
        v[i] = kept + recv;
    }
}

// NV = 16 R values per lane -> one total per lane (lanes sharing lane >> (6 - log2 NV) agree)
template <int NV>
__device__ __forceinline__ float reduce_scatter(float (&v)[NV], int lane) {
    halve_swap32<NV>(v);
    halve_swap16<NV / 2>(reinterpret_cast<float(&)[NV / 2]>(v));
    halve_dpp<NV / 4, 3>(reinterpret_cast<float(&)[NV / 4]>(v), lane);
    halve_dpp<NV / 8, 2>(reinterpret_cast<float(&)[NV / 8]>(v), lane);
    if constexpr (NV >= 32) halve_dpp<NV / 16, 1>(reinterpret_cast<float(&)[NV / 16]>(v), lane);
    if constexpr (NV >= 64) halve_dpp<NV / 32, 0>(reinterpret_cast<float(&)[NV / 32]>(v), lane);
    float t = v[0];
    if constexpr (NV < 32) t = t + dppf<kDppXor2>(t);  // remaining lanes hold partial sums
    if constexpr (NV < 64) t = t + dppf<kDppXor1>(t);
    return t;
}

template <typename T, int R, int K>
__device__ __forceinline__ void odd_rows_tile(const ProductArgs& a, const MatDesc& d, const Tile& t) {
    static_assert(R <= 4, "row-layout odd product: r <= 4");
    constexpr int RB = R == 4 ? 8 : 16;                 // rows per batch
    constexpr int NV = RB * R;                          // values reduced per batch (16 or 32)
    constexpr int SH = NV == 16 ? 2 : 1;                // lanes >> SH share one item
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = d.r;
    const int64_t n = d.n, m = d.m;
    const int32_t col0 = t.strip * 256 + 4 * lane;
    const bool active = col0 < m;
    const int32_t ccol = active ? col0 : 0;
    const int64_t row_begin = int64_t(t.chunk) * d.chunk_rows;
    const int64_t row_end = n < row_begin + d.chunk_rows ? n : row_begin + d.chunk_rows;
    const gptr<const T> G = gconst<T>(a.grads[t.tensor]);
    const int nres = K >= 0 ? K : a.nres;
    constexpr int KC = K > 0 ? K : 1;

    float xq[4][R];  // X[col][c] of this lane's columns (zero when inactive)
#pragma unroll
    for (int v = 0; v < 4; ++v) ld_factor<R>(gconst<float>(a.x) + d.qoff + (ccol + v) * r, r, xq[v]);
    float bq[KC][4][R];
    if constexpr (K > 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int v = 0; v < 4; ++v)
                ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + (ccol + v) * r, r, bq[k][v]);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int c = 0; c < R; ++c) xq[v][c] = active ? xq[v][c] : 0.f;

    for (int64_t i0 = row_begin + wave * RB; i0 < row_end; i0 += kWaves * RB) {
        const int nrow = row_end - i0 < RB ? int(row_end - i0) : RB;
        // error-feedback rows P_k[i0 .. i0 + RB) (RB * r <= 32 floats, contiguous): lane l
        // holds element l; row u's values are broadcast with readlane (wave-uniform)
        float pk[KC];
        if constexpr (K > 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int e = lane < nrow * r ? lane : 0;
                pk[k] = gconst<float>(a.res.p[k])[d.poff + i0 * r + e];
            }
        }
        float x[RB][4];
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            const int64_t i = i0 + u;
            Io<T>::ld(G + (i < row_end ? i : row_begin) * m + ccol, x[u]);  // clamped, unconditional
        }
        float sv[NV];
#pragma unroll
        for (int u = 0; u < RB; ++u) {
#pragma unroll
            for (int v = 0; v < 4; ++v) keep(x[u][v]);
            if constexpr (K > 0) {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    float ap[R];
#pragma unroll
                    for (int c = 0; c < R; ++c) {
                        const int src = u * r + (c < r ? c : 0);
                        const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pk[k]), src < 64 ? src : 0));
                        ap[c] = c < r ? w : 0.f;
                    }
#pragma unroll
                    for (int v = 0; v < 4; ++v) x[u][v] = x[u][v] - dotr<R>(ap, bq[k][v]);
                }
            } else {
                const int64_t ic = i0 + u < row_end ? i0 + u : row_begin;
                for (int k = 0; k < nres; ++k) {  // many terms: factor rows from L1/L2
                    float ap[R];
                    ld_factor<R>(gconst<float>(a.res.p[k]) + d.poff + ic * r, r, ap);
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        float b[R];
                        ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + (ccol + v) * r, r, b);
                        x[u][v] = x[u][v] - dotr<R>(ap, b);
                    }
                }
            }
            const bool valid = u < nrow;
#pragma unroll
            for (int c = 0; c < R; ++c) {
                float s = x[u][0] * xq[0][c];
#pragma unroll
                for (int v = 1; v < 4; ++v) s = fmaf(x[u][v], xq[v][c], s);
                sv[c * RB + u] = valid ? s : 0.f;
            }
        }
        const float tot = reduce_scatter<NV>(sv, lane);
        const int item = lane >> SH, c = item / RB, u = item % RB;
        if ((lane & ((1 << SH) - 1)) == 0 && c < r && u < nrow)
            gmut<float>(a.part)[d.part_odd + (int64_t(t.strip) * n + i0 + u) * r + c] = tot;
    }
}

// ------------------------------------------------- odd product, lane-column tiles --
// P = Gk Q on strips narrower than 256 columns (or without the vector layout): each lane forms
// the r partial dots of its V columns of a row; the row's lanes are summed with DPP and the
// strip's partial of the row is stored by the row's first lane.
template <typename T, int R, int K, int V>
__device__ __forceinline__ void odd_cols_tile(const ProductArgs& a, const MatDesc& d, const Tile& t) {
    const TileGeom g = tile_geom<V>(d, t);
    const int r = d.r;
    const gptr<const T> G = gconst<T>(a.grads[t.tensor]);
    const int nres = K >= 0 ? K : a.nres;
    constexpr int KC = K > 0 ? K : 1;  // register-cached terms
    const gptr<const float> xq_base = gconst<float>(a.x) + d.qoff;

    float bq[KC][V][R];
    if constexpr (K > 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int v = 0; v < V; ++v)
                ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + (g.ccol + v) * r, r, bq[k][v]);
    }
    float xq[V][R];
#pragma unroll
    for (int v = 0; v < V; ++v) ld_factor<R>(xq_base + (g.ccol + v) * r, r, xq[v]);

    for (int64_t row = g.first_row; row < g.row_end; row += int64_t(kUnroll) * g.stride) {
        // the rows' error-feedback factor rows travel with the gradient rows (loaded inside
        // the row loop they were a chain of dependent round trips per batch)
        float x[kUnroll][V];
        int64_t rc[kUnroll];
        float apu[KC][kUnroll][R];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t rr = row + u * g.stride;
            rc[u] = rr < g.row_end ? rr : g.row_begin;  // clamped: every load is in range
            Io<T>::ld(G + rc[u] * g.m + g.ccol, x[u]);
        }
        if constexpr (K > 0) {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
#pragma unroll
                for (int k = 0; k < K; ++k)
                    ld_factor<R>(gconst<float>(a.res.p[k]) + d.poff + int32_t(rc[u]) * r, r, apu[k][u]);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const bool valid = g.active && (row + u * g.stride) < g.row_end;
            const int32_t prow = int32_t(rc[u]) * r;
            // error feedback of the previous iterations, formed on the fly
            for (int k = 0; k < nres; ++k) {
                float ap[R];
                if constexpr (K > 0) {
#pragma unroll
                    for (int c = 0; c < R; ++c) ap[c] = apu[k < KC ? k : 0][u][c];
                } else {
                    ld_factor<R>(gconst<float>(a.res.p[k]) + d.poff + prow, r, ap);
                }
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    float bb[R];
                    if constexpr (K > 0) {
#pragma unroll
                        for (int c = 0; c < R; ++c) bb[c] = bq[k < KC ? k : 0][v][c];
                    } else {
                        ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + (g.ccol + v) * r, r, bb);
                    }
                    x[u][v] = x[u][v] - dotr<R>(ap, bb);
                }
            }
#pragma unroll
            for (int v = 0; v < V; ++v) x[u][v] = valid ? x[u][v] : 0.f;
            float dot[R];
#pragma unroll
            for (int c = 0; c < R; ++c) {
                float sacc = x[u][0] * xq[0][c];
#pragma unroll
                for (int v = 1; v < V; ++v) sacc = fmaf(x[u][v], xq[v][c], sacc);
                dot[c] = sum_within(sacc, g.L);
            }
            const int64_t rr = row + u * g.stride;
            if (g.ql == 0 && rr < g.row_end) {
                gptr<float> dst = gmut<float>(a.part) + d.part_odd + (int64_t(t.strip) * g.n + rr) * r;
#pragma unroll
                for (int c = 0; c < R; ++c)
                    if (c < r) dst[c] = dot[c];
            }
        }
    }
}

template <typename T, int R, int K>
__global__ __launch_bounds__(kBlock) void k_product_odd(ProductArgs a) {
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    if constexpr (R <= 4) {
        if (d.vec && d.lanes == 64) {  // full-width strips: row layout + reduce-scatter
            odd_rows_tile<T, R, K>(a, d, t);
            return;
        }
    }
    if constexpr (R <= 8) {
        if (d.vec) {
            odd_cols_tile<T, R, K, 4>(a, d, t);
            return;
        }
    }
    odd_cols_tile<T, R, K, 1>(a, d, t);
}

// ------------------------------------------------------- odd product on MFMA -------
// P[i, c] = sum_j Gk[i, j] X[j, c] with v_mfma_f32_16x16x4_f32 (exact fp32 fma chains).
// A wave owns 16 rows; lane l = (ri = l & 15, cq = l >> 4) loads G[i0+ri][j0+4cq .. +3]
// (16 rows x 64 contiguous bytes per wave-instruction) and those four values are the
// A-operands of four 16x16x4 products whose B-operand is X[j0+4cq+e][c = ri]: the matrix
// core does the reduction over columns that a VALU version needs cross-lane sums for. The
// error-feedback correction (A_t B_t^T)[i, j] of the same 16 x 16 sub-tile is one MFMA per
// term and 4 factor columns, produced directly in the layout of the loaded fragment
// (D[row=j][col=i] of B_t[16x4] . A_t^T[4x16]).
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kOddSW = 256;            // max MFMA strip width (columns)
constexpr int kOddXT = kOddSW + 4;      // padded row of the transposed X strip in LDS

// Gradient reads of the odd product go through a buffer descriptor that spans exactly the
// tile's region (from the strip's first column of row0 to the strip's last column of the
// tile's last row): the hardware range check returns 0 for rows past the tile, and a slot
// whose columns lie past the strip gets offset kOob (also 0, and no memory traffic). Every
// load is therefore unconditional, unclamped and unmasked.

template <typename T>
struct BufIo;

template <>
struct BufIo<float> {
    static __device__ __forceinline__ void ld4(rsrc_t r, uint32_t off, float (&v)[4]) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
        v[0] = __uint_as_float(x[0]); v[1] = __uint_as_float(x[1]);
        v[2] = __uint_as_float(x[2]); v[3] = __uint_as_float(x[3]);
    }
    static __device__ __forceinline__ float ld1(rsrc_t r, uint32_t off) {
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
    }
};

template <>
struct BufIo<bf16_t> {
    static __device__ __forceinline__ void ld4(rsrc_t r, uint32_t off, float (&v)[4]) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        v[0] = __uint_as_float(x[0] << 16);
        v[1] = __uint_as_float(x[0] & 0xffff0000u);
        v[2] = __uint_as_float(x[1] << 16);
        v[3] = __uint_as_float(x[1] & 0xffff0000u);
    }
    static __device__ __forceinline__ float ld1(rsrc_t r, uint32_t off) {
        return __uint_as_float(uint32_t(__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0)) << 16);
    }
};

// Stage n factor values into LDS: ld(idx) (a global load from a clamped, always valid address)
// for B strides of the workgroup at once, then st(idx, value). A plain element loop waits one
// L2 round trip per element: apply_tile_mfma's rank-32 tiles 122.7 -> 107.4 us with it. (The
// odd product's staging, behind its tile's gradient loads, measured slower batched: 84 -> 93.5
// us at rank 16, profiles/r06/wide/em4.)
template <int B, typename Ld, typename St>
__device__ __forceinline__ void stage_lds(int n, Ld ld, St st) {
    for (int base = threadIdx.x; base < n; base += B * kBlock) {
        float v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int idx = base + u * kBlock;
            v[u] = ld(idx < n ? idx : n - 1);
        }
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int idx = base + u * kBlock;
            if (idx < n) st(idx, v[u]);
        }
    }
}

// A wave owns row blocks rb (16 rows each: rows row0 + 16 (wave + 4 rb) + ri) of the tile
// and works in ROUNDS of 16 slots (one 16-byte load per lane each), all issued together:
//   WIDE   (strip > 64 columns): a round = 1 row block x 16 k-steps (the whole strip row);
//   NARROW (strip <= 64 columns): a round = 4 row blocks x 4 k-steps.
// tile_elems <= 16384 makes a wave's whole share one round; the first round is issued
// before the factor strips are staged in LDS.
constexpr int kOddSlots = 16;

template <typename T, int VEC, int RC, int K, bool WIDE>
__device__ __forceinline__ void odd_mfma_tile(const ProductArgs& a, const MatDesc& d, const Tile& t,
                                              float* xt, float* bs) {
    constexpr int QN = WIDE ? 1 : 4;     // row blocks per round
    constexpr int KN = kOddSlots / QN;   // k-steps per round
    constexpr int s = sizeof(T);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ri = lane & 15, cq = lane >> 4;
    const int r = d.r;
    const int64_t n = d.n;
    const int32_t m = int32_t(d.m);
    const int32_t j_begin = t.strip * d.odd_sw;
    const int32_t j_end = m < j_begin + d.odd_sw ? m : j_begin + d.odd_sw;
    const int32_t sw = j_end - j_begin;
    const int64_t row0 = int64_t(t.chunk) * d.odd_chunk_rows;
    const int64_t row_end = n < row0 + d.odd_chunk_rows ? n : row0 + d.odd_chunk_rows;
    const int nt = K >= 0 ? K : a.nres;
    constexpr int KC = K > 0 ? K : 1;
    constexpr int RP = 4 * RC;           // factor columns held per strip row in LDS
    constexpr int RB = RP > 16 ? 2 : 1;  // 16-column blocks of the product (rank 32: two)
    const int nks = (sw + 15) >> 4;      // 16-column k-steps of the strip
    const int nrb = int((row_end - row0 - wave * 16 + kWaves * 16 - 1) / (kWaves * 16));  // >= 0

    const uint32_t nrec = uint32_t(((row_end - row0 - 1) * m + sw) * s);
    const T* gbase = static_cast<const T*>(a.grads[t.tensor]) + row0 * m + j_begin;
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(gbase), 0, int(nrec), 0x00020000);

    float x[kOddSlots][4];
    float at[QN][KC][RC];
    auto issue = [&](int rb0) {
        if constexpr (K > 0) {  // error-feedback rows P_k[i][cq + 4b] (clamped, pinned later)
#pragma unroll
            for (int q = 0; q < QN; ++q) {
                const int64_t i = row0 + wave * 16 + int64_t(rb0 + q) * (kWaves * 16) + ri;
                const int64_t ic = i < row_end ? i : row0;
#pragma unroll
                for (int k = 0; k < K; ++k)
#pragma unroll
                    for (int bb = 0; bb < RC; ++bb) {
                        const int c = cq + 4 * bb;
                        at[q][k][bb] = gconst<float>(a.res.p[k])[d.poff + ic * r + (c < r ? c : 0)];
                    }
            }
        }
#pragma unroll
        for (int sl = 0; sl < kOddSlots; ++sl) {
            const int q = sl / KN, ks = sl % KN;
            const uint32_t roff = uint32_t((wave * 16 + (rb0 + q) * (kWaves * 16) + ri) * int64_t(m)) * s;
            const int32_t jj = ks * 16 + 4 * cq;
            if constexpr (VEC) {
                BufIo<T>::ld4(rs, jj < sw ? roff + uint32_t(jj) * s : kOob, x[sl]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    x[sl][e] = BufIo<T>::ld1(rs, jj + e < sw ? roff + uint32_t(jj + e) * s : kOob);
            }
        }
    };

    auto process = [&](int rb0) {
        f32x4_t acc[QN][RB];
#pragma unroll
        for (int q = 0; q < QN; ++q)
#pragma unroll
            for (int ob = 0; ob < RB; ++ob) acc[q][ob] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        if constexpr (K > 0) {
#pragma unroll
            for (int q = 0; q < QN; ++q) {
                const bool rv = row0 + wave * 16 + int64_t(rb0 + q) * (kWaves * 16) + ri < row_end;
#pragma unroll
                for (int k = 0; k < K; ++k)
#pragma unroll
                    for (int bb = 0; bb < RC; ++bb) {
                        keep(at[q][k][bb]);
                        at[q][k][bb] = (rv && cq + 4 * bb < r) ? at[q][k][bb] : 0.f;
                    }
            }
        }
#pragma unroll
        for (int sl = 0; sl < kOddSlots; ++sl) {
            const int q = sl / KN, ks = sl % KN;
            if (ks < nks) {  // wave-uniform; the loads were all issued before
                const int32_t js = ks * 16;
                const int32_t jj = js + 4 * cq;
                if constexpr (K > 0) {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        f32x4_t corr = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int bb = 0; bb < RC; ++bb) {
                            const int c = cq + 4 * bb;
                            const int32_t jr = js + ri;
                            const bool ok = jr < sw && c < r;
                            const float av = bs[(k * kOddSW + (jr < sw ? jr : 0)) * RP + c];
                            corr = __builtin_amdgcn_mfma_f32_16x16x4f32(ok ? av : 0.f, at[q][k][bb], corr, 0, 0, 0);
                        }
#pragma unroll
                        for (int e = 0; e < 4; ++e) x[sl][e] -= corr[e];
                    }
                } else {
                    const int64_t i = row0 + wave * 16 + int64_t(rb0 + q) * (kWaves * 16) + ri;
                    const bool rv = i < row_end;
                    const int64_t ic = rv ? i : row0;
                    for (int k = 0; k < nt; ++k) {  // many terms: panels straight from L1/L2
                        const gptr<const float> Bq = gconst<float>(a.res.q[k]) + d.qoff;
                        f32x4_t corr = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int bb = 0; bb < RC; ++bb) {
                            const int c = cq + 4 * bb;
                            const int32_t jr = js + ri;
                            const bool ok = jr < sw && c < r;
                            const float av = Bq[int64_t(j_begin + (ok ? jr : 0)) * r + (ok ? c : 0)];
                            const float pv = gconst<float>(a.res.p[k])[d.poff + ic * r + (c < r ? c : 0)];
                            corr = __builtin_amdgcn_mfma_f32_16x16x4f32(ok ? av : 0.f, (rv && c < r) ? pv : 0.f,
                                                                        corr, 0, 0, 0);
                        }
#pragma unroll
                        for (int e = 0; e < 4; ++e) x[sl][e] -= corr[e];
                    }
                }
                // xt rows are zero-padded to a multiple of 4 columns: one aligned 16-byte read
#pragma unroll
                for (int ob = 0; ob < RB; ++ob) {
                    const int c = 16 * ob + ri;
                    const v4f bx4 = *reinterpret_cast<const v4f*>(xt + (c < r ? c : 0) * kOddXT + (jj < sw ? jj : 0));
                    const bool okx = c < r && jj < sw;
                    acc[q][ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[sl][0], okx ? bx4.x : 0.f, acc[q][ob], 0, 0, 0);
                    acc[q][ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[sl][1], okx ? bx4.y : 0.f, acc[q][ob], 0, 0, 0);
                    acc[q][ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[sl][2], okx ? bx4.z : 0.f, acc[q][ob], 0, 0, 0);
                    acc[q][ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[sl][3], okx ? bx4.w : 0.f, acc[q][ob], 0, 0, 0);
                }
            }
        }
        // acc[q][ob][e] = partial P[i0 + 4 cq + e][c = 16 ob + ri] of row block rb0 + q
        gptr<float> part = gmut<float>(a.part) + d.part_odd + int64_t(t.strip) * n * r;
#pragma unroll
        for (int ob = 0; ob < RB; ++ob) {
            const int c = 16 * ob + ri;
            if (c < r) {
#pragma unroll
                for (int q = 0; q < QN; ++q) {
                    const int64_t i0 = row0 + wave * 16 + int64_t(rb0 + q) * (kWaves * 16);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int64_t ii = i0 + 4 * cq + e;
                        if (ii < row_end) part[ii * r + c] = acc[q][ob][e];
                    }
                }
            }
        }
    };

    // Stage the strip's factor panels once per tile: xt[c][j] = X[j_begin + j][c]
    // (transposed: a lane's four B-operands of one k-step are one ds_read_b128) and
    // bs[k][j][c] = B_k[j_begin + j][c] for the error-feedback correction. This thread's X values
    // (at most RP) are loaded BEFORE the tile's gradient loads, so that waiting for them (vmcnt
    // counts in order) does not also wait for the gradient rows.
    {
        const gptr<const float> X = gconst<float>(a.x) + d.qoff + int64_t(j_begin) * r;
        const int nx = sw * r;  // <= kOddSW * RP = kBlock * RP
        // rank 32 and K >= 2: none (2 waves per SIMD would become 1). Rank 16, K = 1 (the
        // I = 2 odd product): 83.5 -> 74.8 us (profiles/r06/wide/em9)
        constexpr int NXP = (RP <= 16 && K <= 1) ? RP : 0;
        float xs[NXP > 0 ? NXP : 1];
#pragma unroll
        for (int u = 0; u < NXP; ++u) {
            const int idx = int(threadIdx.x) + u * kBlock;
            xs[u] = X[idx < nx ? idx : 0];
        }
        // ... and the first error-feedback panel's (a term loaded after the gradient rows waits
        // for them)
        constexpr bool BP = K == 1 && NXP > 0;
        float bp[BP ? NXP : 1];
        if constexpr (BP) {
            const gptr<const float> Bq = gconst<float>(a.res.q[0]) + d.qoff + int64_t(j_begin) * r;
#pragma unroll
            for (int u = 0; u < NXP; ++u) {
                const int idx = int(threadIdx.x) + u * kBlock;
                bp[u] = Bq[idx < nx ? idx : 0];
            }
        }
        issue(0);  // in flight while the strips are staged
        if constexpr (BP) {
#pragma unroll
            for (int u = 0; u < NXP; ++u) {
                const int idx = int(threadIdx.x) + u * kBlock;
                if (idx < nx) {
                    const int j = idx / r, c = idx - j * r;
                    bs[j * RP + c] = bp[u];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < NXP; ++u) {
            const int idx = int(threadIdx.x) + u * kBlock;
            if (idx < nx) {
                const int j = idx / r, c = idx - j * r;
                xt[c * kOddXT + j] = xs[u];
            }
        }
        for (int idx = int(threadIdx.x) + NXP * kBlock; idx < nx; idx += kBlock) {
            const int j = idx / r, c = idx - j * r;
            xt[c * kOddXT + j] = X[idx];
        }
        const int swp = (sw + 3) & ~3;
        for (int idx = threadIdx.x; idx < (swp - sw) * r; idx += kBlock) {
            const int j = sw + idx / r, c = idx % r;
            xt[c * kOddXT + j] = 0.f;
        }
        if constexpr (K > 0) {
#pragma unroll
            for (int k = BP ? 1 : 0; k < K; ++k) {
                const gptr<const float> Bq = gconst<float>(a.res.q[k]) + d.qoff + int64_t(j_begin) * r;
                for (int idx = threadIdx.x; idx < sw * r; idx += kBlock) {
                    const int j = idx / r, c = idx - j * r;
                    bs[(k * kOddSW + j) * RP + c] = Bq[idx];
                }
            }
        }
        __syncthreads();
    }

    if (nrb > 0) process(0);
    for (int rb0 = QN; rb0 < nrb; rb0 += QN) {
        issue(rb0);
        process(rb0);
    }
}

template <typename T, int RC, int K>
__global__ __launch_bounds__(kBlock) void k_odd_mfma(ProductArgs a) {
    __shared__ __attribute__((aligned(16))) float xt[RC * 4 * kOddXT];
    __shared__ __attribute__((aligned(16))) float bs[(K > 0 ? K : 1) * kOddSW * 4 * RC];
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    const bool wide = d.odd_sw > 64;
    if (d.vec) {
        if (wide) odd_mfma_tile<T, 1, RC, K, true>(a, d, t, xt, bs);
        else odd_mfma_tile<T, 1, RC, K, false>(a, d, t, xt, bs);
    } else {
        if (wide) odd_mfma_tile<T, 0, RC, K, true>(a, d, t, xt, bs);
        else odd_mfma_tile<T, 0, RC, K, false>(a, d, t, xt, bs);
    }
}

template <typename T>
hipError_t dispatch_odd_mfma(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    const dim3 grid(ntiles), block(kBlock);
    const int K = nres <= 3 ? nres : -1;
#define PSGD_O(RC)                                                                       \
    do {                                                                                 \
        switch (K) {                                                                     \
            case 0: k_odd_mfma<T, RC, 0><<<grid, block, 0, s>>>(a); break;               \
            case 1: k_odd_mfma<T, RC, 1><<<grid, block, 0, s>>>(a); break;               \
            case 2: k_odd_mfma<T, RC, 2><<<grid, block, 0, s>>>(a); break;               \
            case 3: k_odd_mfma<T, RC, 3><<<grid, block, 0, s>>>(a); break;               \
            default: k_odd_mfma<T, RC, -1><<<grid, block, 0, s>>>(a); break;             \
        }                                                                                \
    } while (0)
    if (R <= 4)
        PSGD_O(1);
    else if (R <= 8)
        PSGD_O(2);
    else if (R <= 16)
        PSGD_O(4);
    else if (R <= 32)
        PSGD_O(8);
    else
        return hipErrorInvalidValue;
#undef PSGD_O
    return hipGetLastError();
}

// ------------------------------------------------------------------ apply ---------
template <typename T, int R, int NI, bool SHARED, int V, bool ONT = false>
__device__ __forceinline__ void apply_tile(const ApplyArgs& a, const MatDesc& d, const Tile& t) {
    const TileGeom g = tile_geom<V>(d, t);
    const int r = d.r;
    const gptr<T> G = gmut<T>(a.grads[t.tensor]);
    // residual and output destinations: this tile's rows through buffer descriptors (streaming
    // cache policy, 32-bit offsets from the tile's first row)
    T* const Dp = static_cast<T*>(a.rdst ? a.rdst[d.tensor] : a.grads[t.tensor]);
    T* const Op = a.odst ? static_cast<T*>(a.odst[d.tensor]) : static_cast<T*>(a.out) + d.out_off;
    const uint32_t tb = uint32_t((g.row_end - g.row_begin) * g.m * int64_t(sizeof(T)));
    const rsrc_t rD = make_rsrc(Dp + g.row_begin * g.m, tb);
    const rsrc_t rO = make_rsrc(Op + g.row_begin * g.m, tb);
    const int nt = NI > 0 ? NI : a.nterms;
    constexpr int NC = NI > 0 ? NI : 1;
    constexpr int NA = (NI > 0 && !SHARED) ? NI : 1;

    float bq[NC][V][R];
    float ba[NA][V][R];
    if constexpr (NI > 0) {
#pragma unroll
        for (int k = 0; k < NI; ++k)
#pragma unroll
            for (int v = 0; v < V; ++v) {
                ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + (g.ccol + v) * r, r, bq[k][v]);
                if constexpr (!SHARED)
                    ld_factor<R>(gconst<float>(a.apx.q[k]) + d.qoff + (g.ccol + v) * r, r, ba[k][v]);
            }
    }
    const float alpha = a.alpha;

    // batches of kUnroll rows: all gradient rows AND their error-feedback factor rows are
    // loaded before the first is consumed (factor rows loaded inside the term loop were a
    // chain of kUnroll dependent round trips per batch)
    struct Batch {
        float x[kUnroll][V];
        int64_t rc[kUnroll];
        float ap[NC][kUnroll][R];
        float aa[NA][kUnroll][R];
    };
    auto load = [&](Batch& b, int64_t row) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t rr = row + u * g.stride;
            b.rc[u] = rr < g.row_end ? rr : g.row_begin;
            Io<T>::ld(G + b.rc[u] * g.m + g.ccol, b.x[u]);
        }
        if constexpr (NI > 0) {
#pragma unroll
            for (int k = 0; k < NI; ++k)
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const int32_t prow = int32_t(b.rc[u]) * r;
                    ld_factor<R>(gconst<float>(a.res.p[k]) + d.poff + prow, r, b.ap[k][u]);
                    if constexpr (!SHARED) ld_factor<R>(gconst<float>(a.apx.p[k]) + d.poff + prow, r, b.aa[k][u]);
                }
        }
    };
    auto process = [&](Batch& b, int64_t row) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int32_t prow = int32_t(b.rc[u]) * r;
            float o[V];
#pragma unroll
            for (int v = 0; v < V; ++v) o[v] = 0.f;
            for (int k = 0; k < nt; ++k) {
                float ap[R], aa[R];
                if constexpr (NI > 0) {
#pragma unroll
                    for (int c = 0; c < R; ++c) {
                        ap[c] = b.ap[k < NC ? k : 0][u][c];
                        aa[c] = b.aa[k < NA ? k : 0][u][c];
                    }
                } else {
                    ld_factor<R>(gconst<float>(a.res.p[k]) + d.poff + prow, r, ap);
                    if constexpr (!SHARED) ld_factor<R>(gconst<float>(a.apx.p[k]) + d.poff + prow, r, aa);
                }
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    float bv[R];
                    if constexpr (NI > 0) {
#pragma unroll
                        for (int c = 0; c < R; ++c) bv[c] = bq[k < NC ? k : 0][v][c];
                    } else {
                        ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + (g.ccol + v) * r, r, bv);
                    }
                    const float tk = dotr<R>(ap, bv);
                    b.x[u][v] = b.x[u][v] - tk;  // reference :195-202 (alpha = -1)
                    if constexpr (SHARED) {
                        o[v] = o[v] + tk;        // world size 1: Qbar == Q_local, alpha = 1
                    } else {
                        float bb[R];
                        if constexpr (NI > 0) {
#pragma unroll
                            for (int c = 0; c < R; ++c) bb[c] = ba[k < NA ? k : 0][v][c];
                        } else {
                            ld_factor<R>(gconst<float>(a.apx.q[k]) + d.qoff + (g.ccol + v) * r, r, bb);
                        }
                        o[v] = o[v] + alpha * dotr<R>(aa, bb);  // reference :211-219
                    }
                }
            }
            if (g.active && row + u * g.stride < g.row_end) {
                const uint32_t off = uint32_t((b.rc[u] - g.row_begin) * g.m + g.col0) * uint32_t(sizeof(T));
                st_vec<T>(rD, off, b.x[u]);
                st_vec<T, ONT ? kStAuxOutNt : PSGD_ST_AUX>(rO, off, o);
            }
        }
    };
    for (int64_t row = g.first_row; row < g.row_end; row += kUnroll * g.stride) {
        Batch b;
        load(b, row);
        process(b, row);
    }
}

// Ranks 16 / 32: the reconstruction T = sum_k P_k Q_k^T of a tile on the matrix cores
// (v_mfma_f32_16x16x4_f32), the residual G - T and the output T (world size 1) or
// alpha * sum_k Pbar_k Qbar_k^T (world size > 1) streamed as the VALU form does. A wave takes
// 16-row blocks of the tile's 64-column strip; lane l = (ri = l & 15, cq = l >> 4) holds rows
// b0 + 4 cq + v (v = 0..3) x columns c0 + 4 ri .. +3 of the block: one 16-byte gradient load,
// residual store and output store per row (4 rows x 256 B per wave instruction), which is
// exactly the accumulator layout of four products D_e (column offset e) with A[i][k] =
// P_k[b0 + i][rank(k)] and B[k][n] = Q_k[c0 + 4 n + e][rank(k)]. Lane row cq owns ranks
// cq * R/4 .. +R/4 (contiguous: one or two 16-byte LDS reads per product set). The strip's factor
// columns (every term, both sets) are staged in LDS once per tile. The VALU form of these ranks
// (one column per lane, r FMAs and r factor loads per element) ran at 0.08 of HBM at rank 16 and
// 0.013 at rank 32 (profiles/r06/wide/em1).
constexpr int kApplyMfmaSets = 4;  // staged (term, set) panels: nterms x (1 shared, 2 split) <= 4
template <int R>
struct ApplyMfmaLds {
    static constexpr int RP = R + 4;  // padded LDS row (floats)
    static constexpr int floats = kApplyMfmaSets * 64 * RP;
};

template <typename T, int R, bool SHARED, bool ONT>
__device__ __forceinline__ void apply_tile_mfma(const ApplyArgs& a, const MatDesc& d, const Tile& t, float* qs) {
    constexpr int KQ = R / 4;
    constexpr int RP = ApplyMfmaLds<R>::RP;
    constexpr int NS = SHARED ? 1 : 2;
    constexpr uint32_t s = sizeof(T);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ri = lane & 15, cq = lane >> 4;
    const int r = d.r;
    const int nt = a.nterms;
    const int32_t m = int32_t(d.m);
    const int L = d.lanes;
    const int32_t cb = t.strip * L;  // V = 1 strips of L <= 64 columns
    const int32_t col = cb + 4 * ri;
    const bool active = 4 * ri < L && col < m;  // m % 4 == 0: a quad is wholly in or out
    const int64_t row_begin = int64_t(t.chunk) * d.chunk_rows;
    const int64_t row_end = d.n < row_begin + d.chunk_rows ? d.n : row_begin + d.chunk_rows;
    // stage qs[set * nt + k][j][c] = Q_k[cb + j][c] of the set (0 past the strip or the rank)
    auto qidx = [&](int idx, int& c, int& j, int& sk) {
        c = idx % R;
        j = (idx / R) % 64;
        sk = idx / (64 * R);
    };
    stage_lds<8>(
        NS * nt * 64 * R,
        [&](int idx) {
            int c, j, sk;
            qidx(idx, c, j, sk);
            const int set = sk / nt, k = sk - set * nt;
            const float* q = set == 0 ? a.res.q[k] : a.apx.q[k];
            const bool ok = c < r && cb + j < m && j < L;
            const float v = gconst<float>(q)[d.qoff + (ok ? int64_t(cb + j) * r + c : 0)];
            return ok ? v : 0.f;
        },
        [&](int idx, float v) {
            int c, j, sk;
            qidx(idx, c, j, sk);
            qs[(sk * 64 + j) * RP + c] = v;
        });
    __syncthreads();
    T* const Gp = static_cast<T*>(a.grads[t.tensor]);
    T* const Dp = static_cast<T*>(a.rdst ? a.rdst[d.tensor] : a.grads[t.tensor]);
    T* const Op = a.odst ? static_cast<T*>(a.odst[d.tensor]) : static_cast<T*>(a.out) + d.out_off;
    const uint32_t tb = uint32_t((row_end - row_begin) * int64_t(m) * int64_t(s));
    const rsrc_t rG = make_rsrc(Gp + row_begin * m, tb);
    const rsrc_t rD = make_rsrc(Dp + row_begin * m, tb);
    const rsrc_t rO = make_rsrc(Op + row_begin * m, tb);
    const uint32_t cofs = active ? uint32_t(col) * s : kOob;
    const uint32_t rstride = uint32_t(m) * s;
    const bool pvec = r == R && (d.poff & 3) == 0;
    const float alpha = a.alpha;
    for (int64_t b0 = row_begin + 16 * wave; b0 < row_end; b0 += 16 * kWaves) {
        const uint32_t rb = uint32_t(b0 - row_begin + 4 * cq);
        float x[4][4];
#pragma unroll
        for (int v = 0; v < 4; ++v) BufIo<T>::ld4(rG, (rb + v) * rstride + cofs, x[v]);
        const int64_t pi = b0 + ri < row_end ? b0 + ri : row_begin;  // A-operand row (clamped)
        f32x4_t tacc[NS][4];
#pragma unroll
        for (int st = 0; st < NS; ++st)
#pragma unroll
            for (int e = 0; e < 4; ++e) tacc[st][e] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        for (int st = 0; st < NS; ++st) {
            for (int k = 0; k < nt; ++k) {
                const gptr<const float> P = gconst<float>(st == 0 ? a.res.p[k] : a.apx.p[k]) + d.poff + pi * r;
                float pa[KQ];
                if (pvec) {
#pragma unroll
                    for (int j = 0; j < KQ; j += 4) {
                        const v4f w = *(gptr<const v4f>)(P + cq * KQ + j);
                        pa[j] = w.x; pa[j + 1] = w.y; pa[j + 2] = w.z; pa[j + 3] = w.w;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < KQ; ++j) {
                        const int c = cq * KQ + j;
                        pa[j] = P[c < r ? c : 0];
                    }
#pragma unroll
                    for (int j = 0; j < KQ; ++j) {
                        keep(pa[j]);
                        pa[j] = cq * KQ + j < r ? pa[j] : 0.f;
                    }
                }
                const float* qk = qs + ((st * nt + k) * 64 + 4 * ri) * RP + cq * KQ;
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < KQ; j += 4) {
                        const v4f bq = *reinterpret_cast<const v4f*>(qk + e * RP + j);
                        tacc[st][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[j], bq.x, tacc[st][e], 0, 0, 0);
                        tacc[st][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[j + 1], bq.y, tacc[st][e], 0, 0, 0);
                        tacc[st][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[j + 2], bq.z, tacc[st][e], 0, 0, 0);
                        tacc[st][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[j + 3], bq.w, tacc[st][e], 0, 0, 0);
                    }
            }
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            float xo[4], oo[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                xo[e] = x[v][e] - tacc[0][e][v];  // reference :195-202
                oo[e] = SHARED ? tacc[0][e][v] : alpha * tacc[NS - 1][e][v];  // :211-219
            }
            const uint32_t off = (rb + v) * rstride + cofs;
            st_vec<T>(rD, off, xo);
            st_vec<T, ONT ? kStAuxOutNt : PSGD_ST_AUX>(rO, off, oo);
        }
    }
    __syncthreads();  // qs is staged again by the next tile of this workgroup (none today)
}

// ONT: the output stores nt only (world size 1, plans above PSGD_OUT_NT_MB: the averaged
// gradient the optimizer reads next does not sit dirty in the Infinity Cache ahead of the next
// step's cold reads); a compile-time instance, so the store form costs no registers
template <typename T, int R, int NI, bool SHARED, bool ONT = false>
__global__ __launch_bounds__(kBlock) void k_apply(ApplyArgs a) {
    // blocks [0, nitems): uncompressed tensors (first, so they run beside the first wave of
    // tiles rather than in the launch tail); then the tiles
    const int nf = a.flat.nitems;
    if (int(blockIdx.x) < nf) {
        flat_pack_item<T, kBlock>(a.flat, blockIdx.x);
        return;
    }
    const Tile t = a.tiles[blockIdx.x - nf];
    const MatDesc d = a.mats[t.mat];
    if constexpr (R <= 8) {
        if (d.vec) {
            apply_tile<T, R, NI, SHARED, 4, ONT>(a, d, t);
            return;
        }
    }
    if constexpr (R >= 16) {
        __shared__ __attribute__((aligned(16))) float qs[ApplyMfmaLds<R>::floats];
        constexpr int NS = SHARED ? 1 : 2;
        const uintptr_t rows = reinterpret_cast<uintptr_t>(a.grads[t.tensor]) |
                               reinterpret_cast<uintptr_t>(a.rdst ? a.rdst[d.tensor] : a.grads[t.tensor]) |
                               reinterpret_cast<uintptr_t>(a.odst ? static_cast<T*>(a.odst[d.tensor])
                                                                  : static_cast<T*>(a.out) + d.out_off);
        if ((d.m & 3) == 0 && (rows & (4 * sizeof(T) - 1)) == 0 && a.nterms * NS <= kApplyMfmaSets) {
            apply_tile_mfma<T, R, SHARED, ONT>(a, d, t, qs);
            return;
        }
    }
    apply_tile<T, R, NI, SHARED, 1, ONT>(a, d, t);
}

// ------------------------------------------------------------------ dispatch ------
template <typename T, int R>
hipError_t dispatch_odd_r(int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    constexpr bool kCache = R <= 8;
    const int K = (kCache && nres <= 3) ? nres : -1;
    const dim3 grid(ntiles), block(kBlock);
    if constexpr (kCache) {
        switch (K) {
            case 0: k_product_odd<T, R, 0><<<grid, block, 0, s>>>(a); break;
            case 1: k_product_odd<T, R, 1><<<grid, block, 0, s>>>(a); break;
            case 2: k_product_odd<T, R, 2><<<grid, block, 0, s>>>(a); break;
            case 3: k_product_odd<T, R, 3><<<grid, block, 0, s>>>(a); break;
            default: k_product_odd<T, R, -1><<<grid, block, 0, s>>>(a); break;
        }
    } else {
        k_product_odd<T, R, -1><<<grid, block, 0, s>>>(a);
    }
    return hipGetLastError();
}

template <typename T>
hipError_t dispatch_odd(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    switch (R) {
        case 1: return dispatch_odd_r<T, 1>(nres, a, ntiles, s);
        case 2: return dispatch_odd_r<T, 2>(nres, a, ntiles, s);
        case 4: return dispatch_odd_r<T, 4>(nres, a, ntiles, s);
        case 8: return dispatch_odd_r<T, 8>(nres, a, ntiles, s);
        case 16: return dispatch_odd_r<T, 16>(nres, a, ntiles, s);
        case 32: return dispatch_odd_r<T, 32>(nres, a, ntiles, s);
        default: return hipErrorInvalidValue;
    }
}

template <typename T, int R>
hipError_t dispatch_apply_r(int nterms, bool shared, const ApplyArgs& a, int ntiles, hipStream_t s) {
    const dim3 grid(ntiles + a.flat.nitems), block(kBlock);
    // register-cached factor terms: up to 4 at ranks <= 8; ranks 16 / 32 take the matrix-core
    // tiles (apply_tile_mfma, any term count), whose fallback loads factor rows per element
    constexpr bool kCache = R <= 8;
    constexpr int kMaxNI = 4;
    // world size > 1 (two term sets: local and all-reduced) caches fewer: the 4-term rank-4
    // and rank-8 instances spilled VGPRs to scratch (tools/regs.py), the per-use loads do not
    const int maxni = shared ? kMaxNI : (R <= 2 ? 4 : R == 4 ? 3 : 2);
    const int NI = (kCache && nterms <= maxni) ? nterms : -1;
#define PSGD_A(NN)                                                                       \
    do {                                                                                 \
        if (shared && a.out_nt)                                                          \
            timed_launch(&k_apply<T, R, NN, true, true>, grid, block, s, a);             \
        else if (shared)                                                                 \
            timed_launch(&k_apply<T, R, NN, true>, grid, block, s, a);                   \
        else                                                                             \
            timed_launch(&k_apply<T, R, NN, false>, grid, block, s, a);                  \
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
