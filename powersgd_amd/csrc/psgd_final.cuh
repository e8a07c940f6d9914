// Final-pass kernels (gfx950, wave64).
//
// k_final_odd — the LAST power iteration when it is odd (P = G_k X, reference
// powersgd.py:185-202 with the transposed views) fused with the final pass (:195-230).
// A row group of T threads (T = 4..64 lanes of one wave, or 2 / 4 whole waves) owns one
// gradient row at a time: thread t holds columns 4 (s T + t) .. +3 of segments s < S in
// registers, so
//   1. g = G_0[i, :] - sum_{j<k} P_j[i] Q_j^T        (error feedback, formed on the fly)
//   2. P[i, :] = g . X                                 (thread dots + DPP / LDS row sum)
//   3. residual[i, :] = g - P[i] X^T                   (from the same registers)
//      output[i, :]   = sum_{j<=k} P_j[i] Q_j^T        (world size 1 only)
// The gradient is read ONCE for the last iteration and its finalisation together: the
// separate odd product + partial reduction + k_apply read it twice and ran three launches.
// The factor panels of a row group's columns (X and the earlier terms' Q_j) stay in
// registers for all rows of the workgroup's row block.
//
// k_lowrank_out — output = alpha * sum_k Pbar_k Qbar_k^T for world size > 1 after a fused
// final iteration (the all-reduced factor of the last iteration is only known after the
// collective, :204-219): writes the output, reads no gradient.
#pragma once

#include "psgd_stream.cuh"

namespace psgd {

// Rows per row group per batch (each batch double-buffered: the next batch's loads are in
// flight while this one reduces and stores): 1 (ranks 1/2: 2 measured 0.6-2 us slower on the
// ResNet-50 and Llama final passes, profiles/r03/v, profiles/r03/x; fewer registers per row). Workgroup size: 256
// threads (rank 4: PSGD_FIN_NT4 below).
#ifndef PSGD_FIN_RB12
#define PSGD_FIN_RB12 1
#endif
template <int R>
struct FinRB {
    static constexpr int value = R == 4 ? 1 : PSGD_FIN_RB12;
};
// rank 4: PSGD_FIN_NT4 threads per workgroup. 256 with up to 5 register segments per thread
// (187 VGPRs, 2 waves per SIMD; PSGD_PROJ4_WPE) against 512 with 3 (128 VGPRs, 4 waves per
// SIMD): fewer idle lanes on the 9c-column rows (4608 columns: 1280 slots for 1152 quads
// instead of 1536), cfg3 k_final_proj 53.9-54.6 -> 51.7-52.5 us, step 0.0938-0.0941 -> 0.0923-
// 0.0925 ms (profiles/r05/fin_nt4). At 3 waves per SIMD the instance spills (168 + 29 VGPRs)
#ifndef PSGD_FIN_NT4
#define PSGD_FIN_NT4 256
#endif
#ifndef PSGD_PROJ4_WPE
#define PSGD_PROJ4_WPE 2
#endif
template <int R>
struct FinNT {
    static constexpr int value = R == 4 ? PSGD_FIN_NT4 : 256;
};

// Gradient / output rows go through buffer descriptors spanning exactly one matrix: a
// slot past the row end or past the matrix gets offset kOob, which loads 0 and drops the
// store in hardware (no clamping, no branches). The plan keeps a fused matrix below 2^31
// bytes.
// Four consecutive row elements [c, c+4) at element offset `e` (= row * m + c): one vector
// access with the vector layout (m % 4 == 0, aligned), else four scalar accesses.
template <typename T, bool VEC>
__device__ __forceinline__ void fin_ld(rsrc_t rs, uint32_t e, bool ok, int32_t c, int32_t m, float (&v)[4]) {
    constexpr uint32_t s = sizeof(T);
    if constexpr (VEC) {
        BufIo<T>::ld4(rs, ok ? e * s : kOob, v);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = BufIo<T>::ld1(rs, (ok && c + q < m) ? (e + q) * s : kOob);
    }
}
template <typename T, bool VEC, int AUX = PSGD_ST_AUX>
__device__ __forceinline__ void fin_st(rsrc_t rs, uint32_t e, bool ok, int32_t c, int32_t m, const float (&v)[4]) {
    constexpr uint32_t s = sizeof(T);
    if constexpr (VEC) {
        StIo<T>::template st4<AUX>(rs, ok ? e * s : kOob, v);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) StIo<T>::template st1<AUX>(rs, (ok && c + q < m) ? (e + q) * s : kOob, v[q]);
    }
}

// P_0 rows of a row block staged in LDS by the projection form: kFinRowsMax (psgd_internal.h)
constexpr int kProjRows = kFinRowsMax;

// PJ (projection form, two power iterations at world size 1, K = 0): X = orth(Q_0) with
// Q_0 = X R' (R' = the QR factor the orthonormalisation left in a.proj_r), so the reference's
// output P_0 Q_0^T + P_1 X^T with P_1 = (G - P_0 Q_0^T) X is exactly G X X^T and the residual
// G - G X X^T (reference powersgd.py:185-230 with I = 2): the row pass needs X alone, no error
// feedback term per element. The P state the reference keeps is P_1 = G X - P_0 R'^T (X^T X
// = I), formed per row from the row sum.
// Rank 1 (PJ, R = 1): the joint group norm N makes X = Q_0 / N orthonormal only over the whole
// shape group, so X^T X = 1 fails per matrix. With c = Q_0,i . X = ||Q_0,i||^2 / N the
// reference's output P_0 Q_0^T + P_1 X^T is exactly s X^T per row, s = G X + (N - c) P_0, its
// residual G - s X^T, and its P state G X - c P_0 (single-matrix groups: N = c, the pure
// projection). c comes from the even reduction's per-item sums of squares of the matrix.
// OE (odd-even pass, rank 1, world size 1, k_final_oe): the odd iteration k's rows as above, but
// instead of storing the residual g - P x^T it accumulates the NEXT (even) iteration's raw
// product: column partials sum_rows (g - P x^T) P over the row block (reference :185-202 for
// iteration k + 1 with its in-factor P_k before the joint norm, which the reduction divides
// out), and sum_rows P^2 for that norm. The gradient is read once for both iterations.
template <typename T, int R, int K, int SMAX, bool VEC, int NT, int RB, bool PJ = false, bool OE = false>
__device__ __forceinline__ void final_odd_tile(const FinalArgs& a, const MatDesc& d, const Tile& t,
                                               float* red, float* rqs = nullptr, float* oered = nullptr) {
    static_assert(!OE || (R == 1 && !PJ), "the odd-even pass is rank 1, K-term form");
    constexpr int KC = K > 0 ? K : 1;
    constexpr int NW = NT / 64;
    const int r = d.r;
    const int32_t m = int32_t(d.m);
    const int Tg = d.fin_T, S = d.fin_S;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rg = tid / Tg, tt = tid - rg * Tg;
    const int RGS = NT / Tg;
    const int64_t frows = OE ? d.oe_rows : PJ ? d.fin_rows : d.fin_rows_kt;
    const int64_t row0 = int64_t(t.chunk) * frows;
    const int64_t row_end = d.n < row0 + frows ? d.n : row0 + frows;
    const int nres = K >= 0 ? K : a.nres;
    const uint32_t nbytes = uint32_t(d.n * d.m * int64_t(sizeof(T)));
    const rsrc_t gs = __builtin_amdgcn_make_buffer_rsrc(a.grads[t.tensor], 0, int(nbytes), 0x00020000);
    const rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(static_cast<T*>(a.out) + d.out_off, 0, int(nbytes),
                                                        0x00020000);
    const gptr<const float> X = gconst<float>(a.x) + d.qoff;

    int32_t ccol[SMAX];
    bool act[SMAX];
#pragma unroll
    for (int s = 0; s < SMAX; ++s) {
        const int32_t c = (s * Tg + tt) * 4;
        act[s] = s < S && c < m;
        ccol[s] = act[s] ? c : 0;
    }
    // one batch: rows ib .. ib + RB of row group rg, with their error-feedback factor rows.
    // Every load of a batch is issued unconditionally (rows past the block end and
    // segments past the row end load 0 through kOob / clamped factor rows), so the number
    // of loads in flight is the same on every path and the waits stay counted, not full
    struct Batch {
        float g[RB][SMAX][4];
        float ap[KC][RB][R];
    };
    auto load = [&](Batch& bt, int b) {
        const int64_t ib = row0 + (int64_t(b) * RGS + rg) * RB;
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            const uint32_t rowe = uint32_t((ib + u) * int64_t(m));
#pragma unroll
            for (int s = 0; s < SMAX; ++s)
                fin_ld<T, VEC>(gs, rowe + uint32_t(ccol[s]), act[s] && ib + u < row_end, ccol[s], m, bt.g[u][s]);
        }
        if constexpr (K > 0) {
#pragma unroll
            for (int u = 0; u < RB; ++u) {
                const int64_t ic = ib + u < row_end ? ib + u : row0;  // factor rows: clamped
#pragma unroll
                for (int k = 0; k < K; ++k)
                    ld_factor<R>(gconst<float>(a.res.p[k]) + d.poff + ic * r, r, bt.ap[k][u]);
            }
        }
    };
    // The first batch's gradient rows go out before the factor panels, the norm and the
    // projection rows are loaded: a small block's prologue (panels, norm partials, P_0 rows:
    // dependent round trips) then overlaps the gradient's HBM latency instead of preceding it.
    Batch ga, gb;
    load(ga, 0);
    // rank-1 joint norm of the raw in-factor (world size 1, fused): x / max(||x||, eps)
    // (rank-1 plans only: fused_norm, psgd_plan.cpp; compile-time false above rank 1)
    const bool norm = R == 1 && a.ss_in != nullptr;
    const float dn = norm ? group_norm_ss(a.ss_in, a.grng_in, d.group) : 1.f;
    float cfac = 0.f, kfac = 0.f;  // rank-1 projection: c and N - c of this matrix
    if constexpr (PJ && R == 1) {
        cfac = range_ss(a.ss_in, a.mrng_in, t.mat) / dn;
        kfac = dn - cfac;
    }
    if (norm && t.chunk == 0) {  // row block 0 publishes this matrix's normalised in-factor
        for (int64_t e = tid; e < d.m * r; e += NT) {
            const float v = X[e] / dn;
            a.xstate[d.qoff + e] = v;
            a.hx[d.qoff + e] = v;
        }
    }

    // PJ: R' of this matrix (r x r, row-major at its Q-layout offset; zero outside r x r)
    // and the block's first kProjRows rows of P_0, staged in LDS: only the row-group leaders
    // read them, once per row, with no global load (and vmcnt wait) inside the row loop
    if constexpr (PJ) {
        if (tid < R * R) {
            const int c = tid / R, l = tid - (tid / R) * R;
            if constexpr (R == 1)
                rqs[tid] = cfac;
            else
                rqs[tid] = (c < r && l < r) ? a.proj_r[d.qoff + c * r + l] : 0.f;
        }
        const int nst = int(row_end - row0) * R;  // the plan keeps row blocks <= kProjRows rows
        for (int e = tid; e < nst; e += NT) {
            const int i = e / R, l = e - (e / R) * R;
            rqs[R * R + e] = l < r ? a.proj_p0[d.poff + (row0 + i) * r + l] : 0.f;
        }
        __syncthreads();
    }
    // factor row of column c (clamped to column 0 past the end of a ragged row)
    auto fcol = [&](int s, int v) { return ccol[s] + v < m ? ccol[s] + v : 0; };
    float xq[SMAX][4][R];
    float bq[KC][SMAX][4][R];
    {
        // every panel load issued unconditionally (clamped columns) before any is consumed:
        // a load under a lane condition becomes a branch with its own wait, i.e. a chain of
        // SMAX * 4 * (K + 1) round trips before the first gradient row
#pragma unroll
        for (int s = 0; s < SMAX; ++s)
#pragma unroll
            for (int v = 0; v < 4; ++v) ld_factor<R>(X + fcol(s, v) * r, r, xq[s][v]);
        if constexpr (K > 0) {
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int s = 0; s < SMAX; ++s)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + fcol(s, v) * r, r, bq[k][s][v]);
        }
#pragma unroll
        for (int s = 0; s < SMAX; ++s)
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
                for (int c = 0; c < R; ++c) keep(xq[s][v][c]);
#pragma unroll
        for (int s = 0; s < SMAX; ++s)
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
                for (int c = 0; c < R; ++c) {
                    const float w = norm ? xq[s][v][c] / dn : xq[s][v][c];  // matrix.div_ (:6)
                    xq[s][v][c] = (act[s] && ccol[s] + v < m) ? w : 0.f;
                    // rank 1, pinned: LLVM otherwise sinks the division and the select into
                    // the row loop and re-executes them on every batch
                    if constexpr (R == 1) keep(xq[s][v][c]);
                }
    }
    // factor values of the 4 columns of segment s (registers)
    auto segx = [&](int s, float (&o)[4][R]) {
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int c = 0; c < R; ++c) o[v][c] = xq[s][v][c];
    };
    auto segb = [&](int k, int s, float (&o)[4][R]) {
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int c = 0; c < R; ++c) o[v][c] = bq[k < KC ? k : 0][s][v][c];
    };

    // OE: this thread's columns' partial of the next product, and (row-group leaders) sum P^2
    float cacc[OE ? SMAX : 1][4];
    float ssacc = 0.f;
#pragma unroll
    for (int s = 0; s < (OE ? SMAX : 1); ++s)
#pragma unroll
        for (int v = 0; v < 4; ++v) cacc[s][v] = 0.f;
    // segments past S load zeros (kOob) and drop their stores; their arithmetic is skipped
    // by a uniform branch
    auto seg_on = [&](int s) { return s < S; };
    auto process = [&](Batch& bt, int b) {
        const int64_t ib = row0 + (int64_t(b) * RGS + rg) * RB;
        int64_t ic[RB];
#pragma unroll
        for (int u = 0; u < RB; ++u) ic[u] = ib + u < row_end ? ib + u : row0;  // factor rows: clamped
        auto& g = bt.g;
        auto& ap = bt.ap;
        float dot[RB][R];
#pragma unroll
        for (int u = 0; u < RB; ++u) {
#pragma unroll
            for (int s = 0; s < SMAX; ++s)
#pragma unroll
                for (int v = 0; v < 4; ++v) keep(g[u][s][v]);
#pragma unroll
            for (int c = 0; c < R; ++c) dot[u][c] = 0.f;
#pragma unroll
            for (int s = 0; s < SMAX; ++s) {
                if (seg_on(s)) {
                    // error feedback of the earlier iterations (reference :195-202), same
                    // per-element arithmetic as the product and k_apply
                    if constexpr (K > 0) {
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            float b[4][R];
                            segb(k, s, b);
#pragma unroll
                            for (int v = 0; v < 4; ++v) g[u][s][v] = g[u][s][v] - dotr<R>(ap[k][u], b[v]);
                        }
                    } else if constexpr (K < 0) {
                        for (int k = 0; k < nres; ++k) {
                            float pa[R];
                            ld_factor<R>(gconst<float>(a.res.p[k]) + d.poff + ic[u] * r, r, pa);
#pragma unroll
                            for (int v = 0; v < 4; ++v) {
                                float qb[R];
                                ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + fcol(s, v) * r, r, qb);
                                g[u][s][v] = g[u][s][v] - dotr<R>(pa, qb);
                            }
                        }
                    }
                    float xs[4][R];
                    segx(s, xs);
#pragma unroll
                    for (int v = 0; v < 4; ++v)
#pragma unroll
                        for (int c = 0; c < R; ++c) dot[u][c] = fmaf(g[u][s][v], xs[v][c], dot[u][c]);
                }
            }
        }
        // row sums over the T threads of the row group (fixed order: DPP tree, then waves
        // in index order)
        if (Tg <= 64) {
#pragma unroll
            for (int u = 0; u < RB; ++u)
#pragma unroll
                for (int c = 0; c < R; ++c) dot[u][c] = sum_within(dot[u][c], Tg);
        } else {
            float* buf = red + (b & 1) * NW * RB * R;
#pragma unroll
            for (int u = 0; u < RB; ++u)
#pragma unroll
                for (int c = 0; c < R; ++c) {
                    dot[u][c] = wave_allsum(dot[u][c]);
                    if (lane == 0) buf[wave * RB * R + u * R + c] = dot[u][c];
                }
            __syncthreads();
            const int w0 = rg * (Tg >> 6), nw = Tg >> 6;
#pragma unroll
            for (int u = 0; u < RB; ++u)
#pragma unroll
                for (int c = 0; c < R; ++c) {
                    float sum = buf[w0 * RB * R + u * R + c];
                    for (int w = 1; w < nw; ++w) sum += buf[(w0 + w) * RB * R + u * R + c];
                    dot[u][c] = sum;
                }
        }
        // the local out-factor rows (history + the reference-visible P state, :189-193)
        if (tt == 0) {
#pragma unroll
            for (int u = 0; u < RB; ++u)
                if (ib + u < row_end) {
                    float p0[PJ ? R : 1];  // PJ: this row of P_0 (LDS; blocks <= kProjRows rows)
                    if constexpr (PJ) {
                        const int li = int(ib + u - row0);
#pragma unroll
                        for (int l = 0; l < R; ++l) p0[l] = rqs[R * R + li * R + l];
                    }
#pragma unroll
                    for (int c = 0; c < R; ++c)
                        if (c < r) {
                            const int64_t e = d.poff + (ib + u) * r + c;
                            float y = dot[u][c];
                            if constexpr (PJ) {  // P_1 = G X - P_0 R'^T
                                float t = 0.f;
#pragma unroll
                                for (int l = 0; l < R; ++l) t = fmaf(p0[l], rqs[c * R + l], t);
                                y = y - t;
                            }
                            a.yloc[e] = y;
                            a.state[e] = y;
                            if constexpr (OE) ssacc = fmaf(y, y, ssacc);
                            if constexpr (!PJ && !OE) {  // the exchange (W > 1) never takes the projection form
                                if (a.xout) st_slot(a.xout + e, y);
                            }
                        }
                }
        }
        // residual (and output at world size 1) from the registers
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            float pr[R];
#pragma unroll
            for (int c = 0; c < R; ++c) pr[c] = c < r ? dot[u][c] : 0.f;
            const bool valid = ib + u < row_end;
            if constexpr (PJ && R == 1) {  // s = G X + (N - c) P_0 (every thread of the row group)
                const int li = valid ? int(ib + u - row0) : 0;
                pr[0] = fmaf(kfac, rqs[R * R + li * R], pr[0]);
            }
            const uint32_t rowe = uint32_t((ib + u) * int64_t(m));
#pragma unroll
            for (int s = 0; s < SMAX; ++s) {
                if (seg_on(s)) {
                    float res[4], o[4];
                    float xs[4][R];
                    segx(s, xs);
                    float bs[K > 0 ? K : 1][4][R];
                    if constexpr (K > 0) {
                        if (a.write_out) {
#pragma unroll
                            for (int k = 0; k < K; ++k) segb(k, s, bs[k]);
                        }
                    }
                    if constexpr (OE) {
                        // the next iteration's raw product (rows past the block: P taken as 0,
                        // so they add nothing whatever their error-feedback terms made of g)
                        const float pv = valid ? pr[0] : 0.f;
#pragma unroll
                        for (int v = 0; v < 4; ++v) cacc[s][v] = fmaf(g[u][s][v] - pv * xs[v][0], pv, cacc[s][v]);
                        continue;
                    }
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        const float tl = dotr<R>(pr, xs[v]);
                        res[v] = g[u][s][v] - tl;
                        if (PJ || a.write_out) {  // PJ: world size 1, always
                            float acc = 0.f;
                            if constexpr (K > 0) {
#pragma unroll
                                for (int k = 0; k < K; ++k) acc = acc + dotr<R>(ap[k][u], bs[k][v]);
                            } else if constexpr (K < 0) {
                                for (int k = 0; k < nres; ++k) {
                                    float pa[R], qb[R];
                                    ld_factor<R>(gconst<float>(a.res.p[k]) + d.poff + ic[u] * r, r, pa);
                                    ld_factor<R>(gconst<float>(a.res.q[k]) + d.qoff + fcol(s, v) * r, r, qb);
                                    acc = acc + dotr<R>(pa, qb);
                                }
                            }
                            o[v] = PJ ? tl : acc + tl;
                        }
                    }
                    const bool ok = valid && act[s];
                    fin_st<T, VEC>(gs, rowe + uint32_t(ccol[s]), ok, ccol[s], m, res);
                    if (PJ || a.write_out) {
                        if (a.out_nt)
                            fin_st<T, VEC, kStAuxOutNt>(os, rowe + uint32_t(ccol[s]), ok, ccol[s], m, o);
                        else
                            fin_st<T, VEC>(os, rowe + uint32_t(ccol[s]), ok, ccol[s], m, o);
                    }
                }
            }
        }
    };

    // software pipeline: the next batch's rows are in flight while this batch reduces,
    // synchronises and stores (the workgroup barrier no longer idles the memory system)
    const int64_t rows = row_end - row0;
    const int nb = int((rows + int64_t(RGS) * RB - 1) / (int64_t(RGS) * RB));
    for (int b = 0; b < nb; b += 2) {
        load(gb, b + 1);
        process(ga, b);
        load(ga, b + 2);
        if (b + 1 < nb) process(gb, b + 1);
    }
    if constexpr (OE) {
        // the row groups' partials summed in row-group order (fixed), one [m] partial per block
        float* ssl = oered + NT * SMAX * 4;
#pragma unroll
        for (int s = 0; s < SMAX; ++s)
#pragma unroll
            for (int v = 0; v < 4; ++v) oered[((rg * Tg + tt) * SMAX + s) * 4 + v] = cacc[s][v];
        if (tt == 0) ssl[rg] = ssacc;
        __syncthreads();
        if (rg == 0) {
            float* part = a.oe_part + d.oe_part + int64_t(t.chunk) * m;
#pragma unroll
            for (int s = 0; s < SMAX; ++s)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    float sum = oered[(tt * SMAX + s) * 4 + v];
                    for (int g2 = 1; g2 < RGS; ++g2) sum += oered[((g2 * Tg + tt) * SMAX + s) * 4 + v];
                    if (act[s] && ccol[s] + v < m) part[ccol[s] + v] = sum;
                }
            if (tt == 0) {
                float tot = ssl[0];
                for (int g2 = 1; g2 < RGS; ++g2) tot += ssl[g2];
                a.oe_ss[d.oe_blk0 + t.chunk] = tot;
            }
        }
    }
}

template <typename T, int R, int K, int SMAX, bool PJ = false>
__device__ __forceinline__ void final_odd_block(const FinalArgs& a) {
    constexpr int NT = FinNT<R>::value, RB = FinRB<R>::value;
    // batch row sums (2 buffers)
    constexpr int kRed = 2 * (NT / 64) * RB * R;
    __shared__ float red[kRed];
    __shared__ float rqs[PJ ? R * R + kProjRows * R : 1];
    // blocks [0, nitems): uncompressed tensors (first: beside the first wave of row blocks,
    // not in the launch tail); then the row blocks
    const int nf = a.flat.nitems;
    if (int(blockIdx.x) < nf) {
        flat_pack_item<T, NT>(a.flat, blockIdx.x);
        return;
    }
    const Tile t = a.tiles[blockIdx.x - nf];
    const MatDesc d = a.mats[t.mat];
    if (d.vec)
        final_odd_tile<T, R, K, SMAX, true, NT, RB, PJ>(a, d, t, red, rqs);
    else
        final_odd_tile<T, R, K, SMAX, false, NT, RB, PJ>(a, d, t, red, rqs);
}

template <typename T, int R, int K, int SMAX>
__global__ __launch_bounds__(FinNT<R>::value) void k_final_odd(FinalArgs a) {
    final_odd_block<T, R, K, SMAX, false>(a);
}

// Odd-even pass (rank 1, world size 1, an odd iteration followed by an even one inside a step:
// I >= 3): the odd iteration's rows plus the next iteration's column partials, one gradient pass
template <typename T, int K, int SMAX>
__global__ __launch_bounds__(FinNT<1>::value) void k_final_oe(FinalArgs a) {
    constexpr int NT = FinNT<1>::value, RB = FinRB<1>::value;
    __shared__ float red[2 * (NT / 64) * RB];
    __shared__ float oered[NT * SMAX * 4 + NT];
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    if (d.vec)
        final_odd_tile<T, 1, K, SMAX, true, NT, RB, false, true>(a, d, t, red, nullptr, oered);
    else
        final_odd_tile<T, 1, K, SMAX, false, NT, RB, false, true>(a, d, t, red, nullptr, oered);
}

#ifndef PSGD_PROJ1_WPE
#define PSGD_PROJ1_WPE 1
#endif
// Projection form: rank 4 at PSGD_PROJ4_WPE waves per SIMD (2: the 256-thread, 5-segment
// instance's 187 VGPRs; see PSGD_FIN_NT4), rank 1 at PSGD_PROJ1_WPE, rank 2 uncapped
template <typename T, int R, int SMAX>
__global__ __launch_bounds__(FinNT<R>::value) __attribute__((amdgpu_waves_per_eu(R == 4 ? PSGD_PROJ4_WPE : R == 1 ? PSGD_PROJ1_WPE : 1))) void k_final_proj(
    FinalArgs a) {
    final_odd_block<T, R, 0, SMAX, true>(a);
}

// output = sum_k alpha * (A_k B_k^T) on the lane-column tiles (same order as k_apply's
// output term, reference :211-219). kLowrankUR rows per lane in flight: cfg2 over the
// multi-GPU code path 21.1 -> 20.4 us (profiles/r04/r; the write-only ceiling of the same
// bytes is ~17.9 us, profiles/r04/q)
#ifndef PSGD_LOWRANK_UR
#define PSGD_LOWRANK_UR 4
#endif
constexpr int kLowrankUR = PSGD_LOWRANK_UR;
template <typename T, int R, int NI, int V>
__device__ __forceinline__ void lowrank_tile(const ApplyArgs& a, const MatDesc& d, const Tile& t) {
    const TileGeom g = tile_geom<V>(d, t);
    const int r = d.r;
    const rsrc_t rO = make_rsrc(static_cast<T*>(a.out) + d.out_off + g.row_begin * g.m,
                                uint32_t((g.row_end - g.row_begin) * g.m * int64_t(sizeof(T))));
    const int nt = NI > 0 ? NI : a.nterms;
    constexpr int NC = NI > 0 ? NI : 1;
    float ba[NC][V][R];
    if constexpr (NI > 0) {
#pragma unroll
        for (int k = 0; k < NI; ++k)
#pragma unroll
            for (int v = 0; v < V; ++v)
                ld_factor<R>(gconst<float>(a.apx.q[k]) + d.qoff + (g.ccol + v) * r, r, ba[k][v]);
    }
    const float alpha = a.alpha;
    if constexpr (NI > 0 && kLowrankUR > 1) {
        // kLowrankUR rows per lane in flight: their P-factor loads first, then the stores (the
        // same per-element arithmetic and order as the loop below)
        for (int64_t row0 = g.first_row; row0 < g.row_end; row0 += int64_t(kLowrankUR) * g.stride) {
            float pa[kLowrankUR][NI][R];
#pragma unroll
            for (int u = 0; u < kLowrankUR; ++u) {
                const int64_t row = row0 + int64_t(u) * g.stride;
                const int32_t prow = int32_t(row < g.row_end ? row : row0) * r;
#pragma unroll
                for (int k = 0; k < NI; ++k) ld_factor<R>(gconst<float>(a.apx.p[k]) + d.poff + prow, r, pa[u][k]);
            }
#pragma unroll
            for (int u = 0; u < kLowrankUR; ++u) {
                const int64_t row = row0 + int64_t(u) * g.stride;
                float o[V];
#pragma unroll
                for (int v = 0; v < V; ++v) o[v] = 0.f;
#pragma unroll
                for (int k = 0; k < NI; ++k)
#pragma unroll
                    for (int v = 0; v < V; ++v) o[v] = o[v] + alpha * dotr<R>(pa[u][k], ba[k][v]);
                if (g.active && row < g.row_end) {
                    const uint32_t off = uint32_t((row - g.row_begin) * g.m + g.col0) * uint32_t(sizeof(T));
                    st_vec<T>(rO, off, o);
                }
            }
        }
        return;
    }
    for (int64_t row = g.first_row; row < g.row_end; row += g.stride) {
        const int32_t prow = int32_t(row) * r;
        float o[V];
#pragma unroll
        for (int v = 0; v < V; ++v) o[v] = 0.f;
        for (int k = 0; k < nt; ++k) {
            float aa[R];
            ld_factor<R>(gconst<float>(a.apx.p[k]) + d.poff + prow, r, aa);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                float bb[R];
                if constexpr (NI > 0) {
#pragma unroll
                    for (int c = 0; c < R; ++c) bb[c] = ba[k < NC ? k : 0][v][c];
                } else {
                    ld_factor<R>(gconst<float>(a.apx.q[k]) + d.qoff + (g.ccol + v) * r, r, bb);
                }
                o[v] = o[v] + alpha * dotr<R>(aa, bb);
            }
        }
        if (g.active) {
            const uint32_t off = uint32_t((row - g.row_begin) * g.m + g.col0) * uint32_t(sizeof(T));
            st_vec<T>(rO, off, o);
        }
    }
}

template <typename T, int R, int NI>
__global__ __launch_bounds__(kBlock) void k_lowrank_out(ApplyArgs a) {
    const Tile t = a.tiles[blockIdx.x];
    const MatDesc d = a.mats[t.mat];
    if constexpr (R <= 8) {
        if (d.vec) {
            lowrank_tile<T, R, NI, 4>(a, d, t);
            return;
        }
    }
    lowrank_tile<T, R, NI, 1>(a, d, t);
}

// ------------------------------------------------------------------ dispatch ------
// SMAX (register segments) is the smallest instantiated bucket >= the plan's max fin_S.
// ntiles == 0: no launch; `*waves` (if non-null) receives the resident waves per SIMD of
// the instance that would run (the plan only fuses at >= 2).
template <typename T, int R, int SMAX, int K, bool PJ = false>
hipError_t launch_final_k(const FinalArgs& a, int ntiles, hipStream_t s, int* waves) {
    constexpr int NT = FinNT<R>::value;
    if (waves) {  // resident waves per SIMD; 0 when the instance spills to scratch
        const void* fn;
        if constexpr (PJ)
            fn = reinterpret_cast<const void*>(&k_final_proj<T, R, SMAX>);
        else
            fn = reinterpret_cast<const void*>(&k_final_odd<T, R, K, SMAX>);
        int blocks = 0;
        hipFuncAttributes fa{};
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, NT, 0);
        if (e == hipSuccess) e = hipFuncGetAttributes(&fa, fn);
        if (e != hipSuccess) return e;
        *waves = fa.localSizeBytes > 0 ? 0 : blocks * (NT / 64) / 4;
    }
    if (ntiles == 0) return hipSuccess;
    if constexpr (PJ)
        timed_launch(&k_final_proj<T, R, SMAX>, dim3(ntiles + a.flat.nitems), dim3(NT), s, a);
    else
        timed_launch(&k_final_odd<T, R, K, SMAX>, dim3(ntiles + a.flat.nitems), dim3(NT), s, a);
    return hipGetLastError();
}

// Earlier terms cached in registers: up to 1 always, up to 3 on narrow rows (SMAX <= 3,
// e.g. the 4-iteration LSTM config); otherwise read per use from L1/L2 (K = -1).
// ntiles == 0: no launch; `*waves` (if non-null) receives the resident waves per SIMD of
// the instance that would run (the plan only fuses at >= 2).
template <typename T, int R, int SMAX>
hipError_t dispatch_final_k(int nres, const FinalArgs& a, int ntiles, hipStream_t s, int* waves) {
    if (nres == kFinProj) return launch_final_k<T, R, SMAX, 0, true>(a, ntiles, s, waves);
    if constexpr (R == 4) {
        return hipErrorInvalidValue;  // rank 4: the projection form only (psgd_plan.cpp, set_vec)
    } else {
        switch (nres) {
            case 0: return launch_final_k<T, R, SMAX, 0>(a, ntiles, s, waves);
            case 1: return launch_final_k<T, R, SMAX, 1>(a, ntiles, s, waves);
            case 2:
                if constexpr (SMAX <= 3) return launch_final_k<T, R, SMAX, 2>(a, ntiles, s, waves);
                break;
            case 3:
                if constexpr (SMAX <= 3) return launch_final_k<T, R, SMAX, 3>(a, ntiles, s, waves);
                break;
            default: break;
        }
        return launch_final_k<T, R, SMAX, -1>(a, ntiles, s, waves);
    }
}

// Instantiated (R, SMAX) pairs: the ones that can keep two waves per SIMD without scratch
// (tools/regs.py); any other request returns hipErrorInvalidValue and the plan keeps the
// unfused final iteration.
template <typename T, int R>
hipError_t dispatch_final_r(int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s, int* waves) {
    if (smax <= 2) return dispatch_final_k<T, R, 2>(nres, a, ntiles, s, waves);
    if (smax <= 3) return dispatch_final_k<T, R, 3>(nres, a, ntiles, s, waves);
    if constexpr (R == 4 && PSGD_FIN_NT4 == 256) {
        if (smax <= 5 && nres == kFinProj) return launch_final_k<T, R, 5, 0, true>(a, ntiles, s, waves);
    }
    if constexpr (R <= 2) {
        if (smax <= 5) return dispatch_final_k<T, R, 5>(nres, a, ntiles, s, waves);
        if (smax <= 12 && (nres <= 1 || nres == kFinProj)) {
            if (nres == kFinProj) return launch_final_k<T, R, 12, 0, true>(a, ntiles, s, waves);
            return nres == 0 ? launch_final_k<T, R, 12, 0>(a, ntiles, s, waves)
                             : launch_final_k<T, R, 12, 1>(a, ntiles, s, waves);
        }
    }
    return hipErrorInvalidValue;
}

template <typename T>
hipError_t dispatch_final(int R, int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s,
                          int* waves) {
    switch (R) {
        case 1: return dispatch_final_r<T, 1>(nres, smax, a, ntiles, s, waves);
        case 2: return dispatch_final_r<T, 2>(nres, smax, a, ntiles, s, waves);
        case 4: return dispatch_final_r<T, 4>(nres, smax, a, ntiles, s, waves);
        default: return hipErrorInvalidValue;
    }
}

template <typename T, int SMAX, int K>
hipError_t launch_oe_k(const FinalArgs& a, int ntiles, hipStream_t s, int* waves) {
    constexpr int NT = FinNT<1>::value;
    if (waves) {  // resident waves per SIMD; 0 when the instance spills to scratch
        const void* fn = reinterpret_cast<const void*>(&k_final_oe<T, K, SMAX>);
        int blocks = 0;
        hipFuncAttributes fa{};
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, NT, 0);
        if (e == hipSuccess) e = hipFuncGetAttributes(&fa, fn);
        if (e != hipSuccess) return e;
        *waves = fa.localSizeBytes > 0 ? 0 : blocks * (NT / 64) / 4;
    }
    if (ntiles == 0) return hipSuccess;
    k_final_oe<T, K, SMAX><<<ntiles, NT, 0, s>>>(a);
    return hipGetLastError();
}

// odd-even pass instances: SMAX buckets 2 / 3 / 5, earlier terms cached up to 3 (K = -1 beyond)
template <typename T>
hipError_t dispatch_final_oe(int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s, int* waves) {
    auto by_k = [&](auto SM) -> hipError_t {
        constexpr int SMX = decltype(SM)::value;
        switch (nres) {
            case 1: return launch_oe_k<T, SMX, 1>(a, ntiles, s, waves);
            case 2: return launch_oe_k<T, SMX, 2>(a, ntiles, s, waves);
            case 3: return launch_oe_k<T, SMX, 3>(a, ntiles, s, waves);
            default: return launch_oe_k<T, SMX, -1>(a, ntiles, s, waves);
        }
    };
    if (smax <= 2) return by_k(std::integral_constant<int, 2>{});
    if (smax <= 3) return by_k(std::integral_constant<int, 3>{});
    if (smax <= 5) return by_k(std::integral_constant<int, 5>{});
    return hipErrorInvalidValue;
}

template <typename T, int R>
hipError_t dispatch_lowrank_r(int nterms, const ApplyArgs& a, int ntiles, hipStream_t s) {
    const dim3 grid(ntiles), block(kBlock);
    switch (R <= 8 ? nterms : -1) {
        case 1: k_lowrank_out<T, R, 1><<<grid, block, 0, s>>>(a); break;
        case 2: k_lowrank_out<T, R, 2><<<grid, block, 0, s>>>(a); break;
        case 4: k_lowrank_out<T, R, 4><<<grid, block, 0, s>>>(a); break;
        default: k_lowrank_out<T, R, -1><<<grid, block, 0, s>>>(a); break;
    }
    return hipGetLastError();
}

template <typename T>
hipError_t dispatch_lowrank(int R, int nterms, const ApplyArgs& a, int ntiles, hipStream_t s) {
    switch (R) {
        case 1: return dispatch_lowrank_r<T, 1>(nterms, a, ntiles, s);
        case 2: return dispatch_lowrank_r<T, 2>(nterms, a, ntiles, s);
        case 4: return dispatch_lowrank_r<T, 4>(nterms, a, ntiles, s);
        case 8: return dispatch_lowrank_r<T, 8>(nterms, a, ntiles, s);
        case 16: return dispatch_lowrank_r<T, 16>(nterms, a, ntiles, s);
        case 32: return dispatch_lowrank_r<T, 32>(nterms, a, ntiles, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace psgd
