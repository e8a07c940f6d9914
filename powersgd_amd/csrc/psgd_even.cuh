// k_even — the even power iteration's product Q = G_k^T X (reference powersgd.py:185-193, with
// the error feedback of :195-202 formed on the fly), as a PERSISTENT streaming pass (gfx950).
//
// The plan cuts the gradient bytes of all matrices (or of one bucket of shape groups) into
// equal ranges, one per workgroup, walking matrices -> column strips -> rows. A range is a short
// list of segments (Seg: rows [row0, row1) of one strip); a strip is cut only where a
// workgroup's range ends. Inside a segment every lane OWNS V consecutive columns (V = 4: 16-byte
// fp32 / 8-byte bf16 loads) and the NW waves x (64 / L) row phases walk the rows, kEvenU rows in
// flight per lane; the factor rows X[i, :] travel with the gradient rows. At the end of a
// segment the row phases are summed (DPP inside a wave, then the waves in index order through
// LDS) into ONE column partial per segment: the partial slab is (workgroups + strips) x strip
// width x r floats instead of one per small tile, and k_reduce sums a handful of partials per
// element, always in the same order (bitwise reproducible, no float atomics).
//
// Against the tile grid it replaces (13k short-lived waves of ~8 KB each, 63 % of wave time
// parked in s_waitcnt/barrier, 13 MB of rank-4 partials), the persistent form keeps every
// wave streaming the same strip for hundreds of rows and pays the tile epilogue once per
// segment (a few per workgroup).
#pragma once

#include "psgd_stream.cuh"

namespace psgd {

// Threads per workgroup and gradient rows in flight per lane (build-time knobs for A/B runs).
// The plan launches PSGD_EVEN_WPC (default 4) workgroups per CU, fewer on small plans (at least
// PSGD_EVEN_MIN gradient elements each).
#ifndef PSGD_EVEN_NT
#define PSGD_EVEN_NT 512
#endif
#ifndef PSGD_EVEN_U
#define PSGD_EVEN_U 4
#endif
// bf16 full-width strips: a lane's 4 columns are one 8-byte load, so a row batch carries half the
// bytes of fp32's (rows in flight per lane of even_seg_full)
#ifndef PSGD_EVEN_U_BF16
#define PSGD_EVEN_U_BF16 PSGD_EVEN_U
#endif
// rank 4, narrow strips (V = 4, fewer than 64 lanes per row): rows in flight per lane. 3 keeps
// the rank-4 instance at 80 VGPRs (6 waves per SIMD: 3 workgroups per CU instead of 2); its
// full-width path alone needs 70. cfg3 k_even 23.06 -> 22.4 us (profiles/r05/even_occ)
#ifndef PSGD_EVEN_U_NR4
#define PSGD_EVEN_U_NR4 3
#endif
constexpr int kEvenNT = PSGD_EVEN_NT;
constexpr int kEvenNW = kEvenNT / 64;
constexpr int kEvenU = PSGD_EVEN_U;

// Wave-uniform copies (v_readfirstlane): LLVM cannot prove that threadIdx.x >> 6 or a value
// loaded from a uniform address is the same in every lane, and keeps them in VGPRs, which turns
// buffer-descriptor loads into waterfall loops and the in-factor rows into vector loads.
__device__ __forceinline__ int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni(int64_t x) {
    const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int32_t(uint32_t(x))));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int32_t(uint32_t(uint64_t(x) >> 32))));
    return int64_t((uint64_t(hi) << 32) | lo);
}
__device__ __forceinline__ const void* uni(const void* p) {
    return reinterpret_cast<const void*>(uni(int64_t(reinterpret_cast<uintptr_t>(p))));
}
__device__ __forceinline__ Seg uni(const Seg& s) {
    Seg u;
    u.m = uni(s.m);
    u.poff = uni(s.poff);
    u.qoff = uni(s.qoff);
    u.part = uni(s.part);
    u.row0 = uni(s.row0);
    u.row1 = uni(s.row1);
    u.strip = uni(s.strip);
    u.tensor = uni(s.tensor);
    u.ss = uni(s.ss);
    u.r = uni(s.r);
    u.lanes = uni(s.lanes);
    u.vec = uni(s.vec);
    return u;
}

// The waves' column partials red[wave][strip column][R] (written and synchronised by the caller)
// summed in wave-index order into ONE partial [strip columns][r] of the segment at sg.part
// (r == R: one contiguous run, 16-byte stores of 4 consecutive sums). `cols` = strip width.
template <int R>
__device__ __forceinline__ void even_store(const ProductArgs& a, const Seg& sg, int cols, const float* red) {
    const int tid = threadIdx.x;
    const int r = sg.r;
    const int64_t m = sg.m;
    const int width = cols * R;  // floats per wave
    gptr<float> part = gmut<float>(a.part) + sg.part;
    const int64_t cbase = int64_t(sg.strip) * cols;
    if (r == R && (width & 3) == 0 && cbase + cols <= m && (sg.part & 3) == 0) {
        for (int i4 = tid * 4; i4 < width; i4 += kEvenNT * 4) {
            v4f s = *reinterpret_cast<const v4f*>(red + i4);
#pragma unroll
            for (int w = 1; w < kEvenNW; ++w) s += *reinterpret_cast<const v4f*>(red + w * width + i4);
            *(gptr<v4f>)(part + i4) = s;
        }
    } else {
        for (int idx = tid; idx < width; idx += kEvenNT) {
            float s = red[idx];
#pragma unroll
            for (int w = 1; w < kEvenNW; ++w) s += red[w * width + idx];
            const int c = idx % R;
            const int64_t jc = idx / R;
            if (c < r && cbase + jc < m) part[jc * r + c] = s;
        }
    }
    __syncthreads();  // `red` is written again by the next segment
}

// End of a segment: the rank-1 norm fold's share of sum_rows X^2 (strip-0 segments), the row
// phases summed (DPP inside a wave, then the waves in index order through LDS) and ONE partial
// [strip columns][r] stored at sg.part (even_store).
template <int R, int V>
__device__ __forceinline__ void even_epilogue(const ProductArgs& a, const Seg& sg, int L, float (&acc)[V][R],
                                              float* red, float* ssl) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane / L, ql = lane - sub * L;
    const int64_t rb = sg.row0, re = sg.row1;
    // rank-1 iteration 0 with the norm folded: this strip-0 segment's share of the RAW
    // in-factor's sum of squares (rows in a fixed lane-strided order, then waves in order)
    if constexpr (R == 1) {
        if (a.ss0 && sg.ss >= 0) {
            const float* xp = a.x + sg.poff;
            float sq = 0.f;
            for (int64_t row = rb + tid; row < re; row += kEvenNT) {
                const float v = xp[row];
                sq = fmaf(v, v, sq);
            }
            sq = wave_allsum(sq);
            if (lane == 0) ssl[wave] = sq;
        }
    }
    // row phases inside the wave, then the waves in index order
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
        for (int c = 0; c < R; ++c) acc[v][c] = sum_across(acc[v][c], L);
    const int width = L * V * R;  // floats per wave: the strip's columns x R
    if (sub == 0) {
#pragma unroll
        for (int v = 0; v < V; ++v)
#pragma unroll
            for (int c = 0; c < R; ++c) red[wave * width + (ql * V + v) * R + c] = acc[v][c];
    }
    __syncthreads();
    if constexpr (R == 1) {
        if (a.ss0 && sg.ss >= 0 && tid == 0) {
            float tot = ssl[0];
#pragma unroll
            for (int w = 1; w < kEvenNW; ++w) tot += ssl[w];
            a.ss0[sg.ss] = tot;
        }
    }
    even_store<R>(a, sg, L * V, red);
}

// A wave-uniform row of R factor values through the scalar data cache (s_load_dwordx1/2/4/8):
// the in-factor rows of a full-width strip are the same for all 64 lanes, so they cost SGPRs
// (used directly as FMA operands), not VGPRs or vector-memory slots.
#define PSGD_C __attribute__((address_space(4)))
template <int R>
__device__ __forceinline__ void ld_row_s(const float* base, int64_t off, float (&v)[R]) {
    const PSGD_C float* p = (const PSGD_C float*)(base) + off;
    if constexpr (R == 1) {
        v[0] = p[0];
    } else if constexpr (R == 2) {
        const v2f x = *(const PSGD_C v2f*)p;
        v[0] = x.x;
        v[1] = x.y;
    } else {
#pragma unroll
        for (int c = 0; c < R; c += 4) {
            const v4f x = *(const PSGD_C v4f*)(p + c);
            v[c] = x.x; v[c + 1] = x.y; v[c + 2] = x.z; v[c + 3] = x.w;
        }
    }
}

// Full-width strip (256 columns: 64 lanes x 4, r == R): every row a wave touches is
// wave-uniform, so the in-factor rows come through the scalar cache, and the gradient rows
// through a buffer descriptor spanning the segment's rows (rows past the segment and columns
// past the matrix load 0 without a clamp or a branch). 32-bit offsets from the segment's first
// row; the loop state is scalar. Same arithmetic order as even_seg.
template <typename T, int R, int K>
__device__ __forceinline__ void even_seg_full(const ProductArgs& a, const Seg& sg, const void* gp, float* red,
                                              float* ssl) {
    constexpr uint32_t s = sizeof(T);
    constexpr int U = s == 2 ? PSGD_EVEN_U_BF16 : kEvenU;
    const int lane = threadIdx.x & 63, wave = uni(int32_t(threadIdx.x >> 6));
    const int32_t m = int32_t(sg.m);
    const int32_t col0 = sg.strip * 256 + 4 * lane;
    const bool active = col0 < m;
    const int32_t rb = sg.row0, re = sg.row1;
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(static_cast<const T*>(gp) + int64_t(rb) * m), 0, int(uint32_t(re - rb) * uint32_t(m) * s),
        0x00020000);
    const uint32_t cofs = active ? uint32_t(col0) * s : kOob;
    const uint32_t rstride = uint32_t(m) * s;  // bytes per row
    const float* xb = a.x + sg.poff;
    constexpr int KC = K > 0 ? K : 1;
    const int nres = K >= 0 ? K : a.nres;
    float bq[KC][4][R];  // Q_k values of this lane's columns
    if constexpr (K > 0) {
        const int32_t cc = active ? col0 : 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int v = 0; v < 4; ++v) ld_factor<R>(gconst<float>(a.res.q[k]) + sg.qoff + (cc + v) * R, R, bq[k][v]);
    }
    float acc[4][R];
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int c = 0; c < R; ++c) acc[v][c] = 0.f;

    for (int32_t row = rb + wave; row < re; row += U * kEvenNW) {
        float x[U][4];
        float xs[U][R];
        float ap[KC][U][R];
#pragma unroll
        for (int u = 0; u < U; ++u)
            BufIo<T>::ld4(rs, uint32_t(row + u * kEvenNW - rb) * rstride + cofs, x[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t ru = row + u * kEvenNW;
            const int32_t xr = ru < re ? ru : rb;  // clamped (the gradient row loads 0)
            ld_row_s<R>(xb, int64_t(xr) * R, xs[u]);
            if constexpr (K > 0) {
#pragma unroll
                for (int k = 0; k < K; ++k) ld_row_s<R>(a.res.p[k] + sg.poff, int64_t(xr) * R, ap[k][u]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int v = 0; v < 4; ++v) keep(x[u][v]);
            if constexpr (K != 0) {
                // error feedback of the earlier iterations (reference :195-202), element by element;
                // rows past the segment and inactive columns must stay 0 afterwards
                const int32_t ru = row + u * kEvenNW;
                const int32_t xr = ru < re ? ru : rb;
                const bool valid = active && ru < re;
                for (int k = 0; k < nres; ++k) {
                    float pk[R];
                    if constexpr (K > 0) {
#pragma unroll
                        for (int c = 0; c < R; ++c) pk[c] = ap[k < KC ? k : 0][u][c];
                    } else {
                        ld_row_s<R>(a.res.p[k] + sg.poff, int64_t(xr) * R, pk);
                    }
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        float qk[R];
                        if constexpr (K > 0) {
#pragma unroll
                            for (int c = 0; c < R; ++c) qk[c] = bq[k < KC ? k : 0][v][c];
                        } else {
                            const int32_t cc = active ? col0 : 0;
                            ld_factor<R>(gconst<float>(a.res.q[k]) + sg.qoff + (cc + v) * R, R, qk);
                        }
                        x[u][v] = x[u][v] - dotr<R>(pk, qk);
                    }
                }
#pragma unroll
                for (int v = 0; v < 4; ++v) x[u][v] = valid ? x[u][v] : 0.f;
            }
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
                for (int c = 0; c < R; ++c) acc[v][c] = fmaf(x[u][v], xs[u][c], acc[v][c]);
        }
    }
    even_epilogue<R, 4>(a, sg, 64, acc, red, ssl);
}

template <typename T, int R, int K, int V>
__device__ __forceinline__ void even_seg(const ProductArgs& a, const Seg& sg, const void* gp, float* red,
                                         float* ssl) {
    constexpr uint32_t s = sizeof(T);
    constexpr int U = (R == 4 && V == 4) ? PSGD_EVEN_U_NR4 : R <= 8 ? kEvenU : R == 16 ? 2 : 1;  // fewer rows in flight at ranks 16/32
    const int tid = threadIdx.x, lane = tid & 63, wave = uni(int32_t(tid >> 6));
    const int L = sg.lanes, rw = 64 / L;
    const int sub = lane / L, ql = lane - sub * L;
    const int r = sg.r;
    const int32_t m = int32_t(sg.m);
    const int32_t col0 = (sg.strip * L + ql) * V;
    const bool active = col0 < m;  // V == 4 only when m % 4 == 0: the whole vector is in range
    const int32_t ccol = active ? col0 : 0;
    const int32_t rb = sg.row0, re = sg.row1;
    const int stride = kEvenNW * rw;
    // gradient rows through a buffer descriptor spanning the segment's rows (rows past it and
    // columns past the matrix load 0); 32-bit offsets from the segment's first row
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(static_cast<const T*>(gp) + int64_t(rb) * m), 0, int(uint32_t(re - rb) * uint32_t(m) * s),
        0x00020000);
    const uint32_t rstride = uint32_t(m) * s;
    const gptr<const float> xp = gconst<float>(a.x) + sg.poff;
    const int nres = K >= 0 ? K : a.nres;
    constexpr int KC = K > 0 ? K : 1;  // register-cached error-feedback terms

    float bq[KC][V][R];  // Q_k values of this lane's columns (constant over the segment)
    if constexpr (K > 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int v = 0; v < V; ++v) ld_factor<R>(gconst<float>(a.res.q[k]) + sg.qoff + (ccol + v) * r, r, bq[k][v]);
    }
    float acc[V][R];
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
        for (int c = 0; c < R; ++c) acc[v][c] = 0.f;

    for (int32_t row = rb + wave * rw + sub; row < re + sub; row += U * stride) {
        float x[U][V];
        float xr[U][R];
        float ap[KC][U][R];
        // every load of the batch is issued before any is consumed (no exec-mask branch per
        // load: rows past the segment are out of the descriptor's range and load 0)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t off = active ? uint32_t(row + u * stride - rb) * rstride + uint32_t(col0) * s : kOob;
            if constexpr (V == 4) {
                BufIo<T>::ld4(rs, off, x[u]);
            } else {
                x[u][0] = BufIo<T>::ld1(rs, off);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t ru = row + u * stride;
            const int32_t xi = ru < re ? ru : rb;  // clamped factor row
            ld_factor<R>(xp + xi * r, r, xr[u]);
            if constexpr (K > 0) {
#pragma unroll
                for (int k = 0; k < K; ++k) ld_factor<R>(gconst<float>(a.res.p[k]) + sg.poff + xi * r, r, ap[k][u]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int v = 0; v < V; ++v) keep(x[u][v]);
            if constexpr (K != 0) {
                // error feedback of the earlier iterations (reference :195-202), element by
                // element; rows past the segment and inactive columns must stay 0 afterwards
                const int32_t ru = row + u * stride;
                const int32_t xi = ru < re ? ru : rb;
                const bool valid = active && ru < re;
                for (int k = 0; k < nres; ++k) {
                    float pk[R];
                    if constexpr (K > 0) {
#pragma unroll
                        for (int c = 0; c < R; ++c) pk[c] = ap[k < KC ? k : 0][u][c];
                    } else {
                        ld_factor<R>(gconst<float>(a.res.p[k]) + sg.poff + xi * r, r, pk);
                    }
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        float qk[R];
                        if constexpr (K > 0) {
#pragma unroll
                            for (int c = 0; c < R; ++c) qk[c] = bq[k < KC ? k : 0][v][c];
                        } else {
                            ld_factor<R>(gconst<float>(a.res.q[k]) + sg.qoff + (ccol + v) * r, r, qk);
                        }
                        x[u][v] = x[u][v] - dotr<R>(pk, qk);
                    }
                }
#pragma unroll
                for (int v = 0; v < V; ++v) x[u][v] = valid ? x[u][v] : 0.f;
            }
#pragma unroll
            for (int v = 0; v < V; ++v)
#pragma unroll
                for (int c = 0; c < R; ++c) acc[v][c] = fmaf(x[u][v], xr[u][c], acc[v][c]);
        }
    }
    even_epilogue<R, V>(a, sg, L, acc, red, ssl);
}

// Ranks 9-32, first iteration (no error-feedback terms), m % 4 == 0 and 16-byte rows: the
// column sums Q[j, c] = sum_i G[i, j] X[i, c] on the matrix cores (v_mfma_f32_16x16x4_f32,
// exact fp32 FMA chains). Every wave spans the strip's 64 columns: lane l = (ri = l & 15,
// cq = l >> 4) loads G[i + cq][c0 + 4 ri .. +3] (one 16-byte load, 4 rows x 256 B per wave
// instruction; 8 bytes for bf16), and the four values are the A-operands (A[column quad ri][k =
// row cq]) of four products whose B-operand is X[i + cq][16 cb + ri]: one accumulator per column
// offset e and 16-rank block cb, D_e[4 cq + v][ri] = the partial of column c0 + 4 (4 cq + v) + e,
// rank 16 cb + ri. The waves take 4-row groups in turn (kEvenU groups in flight per lane) and
// meet in even_store. The VALU form of these ranks (one column per lane, the factor row as
// vector loads) read G at 0.14 of HBM at rank 16.
#ifndef PSGD_EVEN_U_MFMA
#define PSGD_EVEN_U_MFMA 4
#endif
#ifndef PSGD_EVEN_U_MFMA32
#define PSGD_EVEN_U_MFMA32 3  // rank 32 (k_even<float, 32, 0> 35.1 us; 3 waves per SIMD without
                              // the 8 spilled VGPRs: 38.7-40.7 us, profiles/r06/wide/em2)
#endif
// VEC = false (m % 4 != 0 or an unaligned gradient): four element loads per lane instead.
template <typename T, int R, bool VEC>
__device__ __forceinline__ void even_seg_mfma(const ProductArgs& a, const Seg& sg, const void* gp, float* red) {
    static_assert(R == 16 || R == 32, "16-rank blocks");
    constexpr int RB = R / 16;
    constexpr int U = R == 32 ? PSGD_EVEN_U_MFMA32 : PSGD_EVEN_U_MFMA;
    constexpr uint32_t s = sizeof(T);
    const int lane = threadIdx.x & 63, wave = uni(int32_t(threadIdx.x >> 6));
    const int ri = lane & 15, cq = lane >> 4;
    const int r = sg.r;
    const int L = sg.lanes;  // strip width (V = 1 strips: one column per lane of the VALU form)
    const int32_t m = int32_t(sg.m);
    const int32_t c0 = sg.strip * L;
    const int32_t col = c0 + 4 * ri;
    const bool active = 4 * ri < L && col < m;  // VEC (m % 4 == 0): a quad is wholly in or out
    const int32_t rb = sg.row0, re = sg.row1;
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(static_cast<const T*>(gp) + int64_t(rb) * m), 0, int(uint32_t(re - rb) * uint32_t(m) * s),
        0x00020000);
    const uint32_t cofs = active ? uint32_t(col) * s : kOob;
    uint32_t eofs[4];  // !VEC: per column of the quad
#pragma unroll
    for (int e = 0; e < 4; ++e) eofs[e] = (4 * ri + e < L && col + e < m) ? uint32_t(col + e) * s : kOob;
    const uint32_t rstride = uint32_t(m) * s;
    const gptr<const float> xp = gconst<float>(a.x) + sg.poff;
    f32x4_t acc[RB][4];
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[cb][e] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int32_t ngroups = (re - rb + 3) >> 2;
    for (int32_t g = wave; g < ngroups; g += U * kEvenNW) {
        float x[U][4];
        float b[U][RB];
        // every load of the batch before any is consumed; rows past the segment load 0 (range)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t ro = uint32_t(4 * (g + u * kEvenNW) + cq) * rstride;
            if constexpr (VEC) {
                BufIo<T>::ld4(rs, ro + cofs, x[u]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) x[u][e] = BufIo<T>::ld1(rs, ro + eofs[e]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t row = rb + 4 * (g + u * kEvenNW) + cq;
            const int32_t xi = row < re ? row : rb;
#pragma unroll
            for (int cb = 0; cb < RB; ++cb) {
                const int c = 16 * cb + ri;
                b[u][cb] = xp[int64_t(xi) * r + (c < r ? c : 0)];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t row = rb + 4 * (g + u * kEvenNW) + cq;
#pragma unroll
            for (int e = 0; e < 4; ++e) keep(x[u][e]);
#pragma unroll
            for (int cb = 0; cb < RB; ++cb) {
                keep(b[u][cb]);
                const float bv = (row < re && 16 * cb + ri < r) ? b[u][cb] : 0.f;
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[cb][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[u][e], bv, acc[cb][e], 0, 0, 0);
            }
        }
    }
    // red[wave][strip column][R]: column 16 cq + 4 v + e of the strip, rank 16 cb + ri
    const int width = L * R;
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int cl = 16 * cq + 4 * v + e;
                if (cl < L) red[wave * width + cl * R + 16 * cb + ri] = acc[cb][e][v];
            }
    __syncthreads();
    even_store<R>(a, sg, L, red);
}

// Occupancy targets (waves per SIMD) per rank: the full-width path's registers, so that
// every CU keeps enough 1 KB row loads in flight (PSGD_EVEN_WPE_R<rank> overrides for A/B runs)
#ifndef PSGD_EVEN_WPE_R1
#define PSGD_EVEN_WPE_R1 8
#endif
#ifndef PSGD_EVEN_WPE_R2
#define PSGD_EVEN_WPE_R2 6
#endif
#ifndef PSGD_EVEN_WPE_R4
#define PSGD_EVEN_WPE_R4 6
#endif
// bf16 gradients: the narrow-strip paths' 16-bit loads and conversions need more registers; at
// the fp32 targets the rank-2/4 instances spilled VGPRs to scratch (tools/regs.py), so one wave
// per SIMD fewer there
#ifndef PSGD_EVEN_WPE_BF16_R2
#define PSGD_EVEN_WPE_BF16_R2 5
#endif
#ifndef PSGD_EVEN_WPE_BF16_R4
#define PSGD_EVEN_WPE_BF16_R4 4
#endif
// ranks 16 / 32, first iteration (the matrix-core form and its scalar-column fallback)
#ifndef PSGD_EVEN_WPE_MFMA
#define PSGD_EVEN_WPE_MFMA 4
#endif
template <typename T, int R, int K>
struct EvenWpe {
    static constexpr bool kBf = sizeof(T) == 2;
    static constexpr int value = K != 0 ? 1
                                 : R >= 16 ? PSGD_EVEN_WPE_MFMA
                                 : R == 1 ? PSGD_EVEN_WPE_R1
                                 : R == 2 ? (kBf ? PSGD_EVEN_WPE_BF16_R2 : PSGD_EVEN_WPE_R2)
                                 : R == 4 ? (kBf ? PSGD_EVEN_WPE_BF16_R4 : PSGD_EVEN_WPE_R4)
                                          : 1;
};

template <typename T, int R, int K>
__global__ __launch_bounds__(kEvenNT)
__attribute__((amdgpu_waves_per_eu(EvenWpe<T, R, K>::value))) void k_even(ProductArgs a) {
    // ranks above 8 always take the scalar (V = 1) layout (the plan guarantees vec == 0)
    __shared__ __attribute__((aligned(16))) float red[kEvenNW * 64 * (R <= 8 ? 4 : 1) * R];
    __shared__ float ssl[kEvenNW];
    if (int(blockIdx.x) >= a.nwg) {  // uncompressed tensors (reference utils.py:43-47)
        flat_pack_item<T, kEvenNT>(a.flat, int(blockIdx.x) - a.nwg);
        return;
    }
#ifdef PSGD_EVEN_STAMPS
    // diagnostic build: entry time, then the end of each of the first kEvenStamps - 2 segments
    unsigned long long* const stp = a.stamps ? a.stamps + size_t(blockIdx.x) * kEvenStamps : nullptr;
    if (stp && threadIdx.x == 0) {
        stp[0] = __builtin_amdgcn_s_memrealtime();
        stp[kEvenStamps - 1] = (uint64_t(uint32_t(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)))) << 32) |
                               uint32_t(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));
    }
#endif
    const int rg = int(blockIdx.x);
    const int s0 = a.wg_seg[rg], s1 = a.wg_seg[rg + 1];
    if (s0 >= s1) return;
    // the next segment's descriptor and gradient pointer are loaded while this one streams
    Seg nx = a.segs[s0];
    const void* ng = a.grads[nx.tensor];
    for (int si = s0; si < s1; ++si) {
        const Seg sg = uni(nx);
        const void* gp = uni(ng);
        if (si + 1 < s1) {
            nx = a.segs[si + 1];
            ng = a.grads[nx.tensor];
        }
        bool done = false;
        if constexpr (R >= 16 && K == 0) {
            // the matrix cores, with 16-byte row quads when m % 4 == 0 and the base is aligned
            if ((sg.m & 3) == 0 && (reinterpret_cast<uintptr_t>(gp) & (4 * sizeof(T) - 1)) == 0)
                even_seg_mfma<T, R, true>(a, sg, gp, red);
            else
                even_seg_mfma<T, R, false>(a, sg, gp, red);
            done = true;
        }
        if constexpr (R <= 8) {
            if (sg.vec == 2) {
                even_seg_full<T, R, K>(a, sg, gp, red, ssl);
                done = true;
            } else if (sg.vec) {
                even_seg<T, R, K, 4>(a, sg, gp, red, ssl);
                done = true;
            }
        }
        if constexpr (!(R >= 16 && K == 0)) {
            if (!done) even_seg<T, R, K, 1>(a, sg, gp, red, ssl);
        }
#ifdef PSGD_EVEN_STAMPS
        if (stp && threadIdx.x == 0 && si - s0 < kEvenStamps - 2) stp[1 + si - s0] = __builtin_amdgcn_s_memrealtime();
#endif
    }
}

template <typename T, int R>
hipError_t dispatch_even_r(int nres, const ProductArgs& a, int nwg0, hipStream_t s) {
    const int nwg = nwg0 + a.flat.nitems;
    // register-cached error-feedback terms: up to 3 at ranks <= 4, 1 at rank 8 (more spill at
    // the 256-VGPR cap of a 512-thread workgroup)
    constexpr bool kCache = R <= 8;
    const int K = (kCache && nres <= (R <= 4 ? 3 : 1)) ? nres : -1;
    const dim3 grid(nwg), block(kEvenNT);
    if constexpr (kCache) {
        switch (K) {
            case 0: k_even<T, R, 0><<<grid, block, 0, s>>>(a); break;
            case 1: k_even<T, R, 1><<<grid, block, 0, s>>>(a); break;
            case 2:
                if constexpr (R <= 4) k_even<T, R, 2><<<grid, block, 0, s>>>(a);
                break;
            case 3:
                if constexpr (R <= 4) k_even<T, R, 3><<<grid, block, 0, s>>>(a);
                break;
            default: k_even<T, R, -1><<<grid, block, 0, s>>>(a); break;
        }
    } else if (nres == 0) {  // ranks 16 / 32, first iteration: the matrix-core instance
        k_even<T, R, 0><<<grid, block, 0, s>>>(a);
    } else {
        k_even<T, R, -1><<<grid, block, 0, s>>>(a);
    }
    return hipGetLastError();
}

// workgroups of the first-iteration instance (K = 0, static ranges) resident per CU: the plan's
// default workgroups per CU, so that the whole grid is one wave of resident workgroups (measured:
// rank 4 fp32 3 per CU 22.0 us against 22.7 at 4; bf16 rank 2 2 per CU 24.6 against 28.0;
// profiles/r05/even_occ)
template <typename T>
int even_resident(int R) {
    int n = 0;
    hipError_t e = hipErrorInvalidValue;
    switch (R) {
        case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_even<T, 1, 0>, kEvenNT, 0); break;
        case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_even<T, 2, 0>, kEvenNT, 0); break;
        case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_even<T, 4, 0>, kEvenNT, 0); break;
        case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_even<T, 8, 0>, kEvenNT, 0); break;
        case 16: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_even<T, 16, 0>, kEvenNT, 0); break;
        case 32: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_even<T, 32, 0>, kEvenNT, 0); break;
        default: break;
    }
    return e == hipSuccess ? n : 0;
}

template <typename T>
hipError_t dispatch_even(int R, int nres, const ProductArgs& a, int nwg, hipStream_t s) {
    if (nwg + a.flat.nitems <= 0) return hipSuccess;
    switch (R) {
        case 1: return dispatch_even_r<T, 1>(nres, a, nwg, s);
        case 2: return dispatch_even_r<T, 2>(nres, a, nwg, s);
        case 4: return dispatch_even_r<T, 4>(nres, a, nwg, s);
        case 8: return dispatch_even_r<T, 8>(nres, a, nwg, s);
        case 16: return dispatch_even_r<T, 16>(nres, a, nwg, s);
        case 32: return dispatch_even_r<T, 32>(nres, a, nwg, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace psgd
