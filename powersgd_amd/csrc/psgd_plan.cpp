// Host side of libpsgd: the codec plan (layout of groups, factor buffers, tiles) and the
// C ABI declared in include/psgd.h. No torch: plain pointers, hipStream_t as void*.
//
// Layout mirrors the reference exactly where it is observable:
//   - matrices = tensor.view(shape[0], -1), grouped by matrix shape in first-appearance order
//     (reference powersgd/powersgd.py:253-263, :283-289);
//   - P state = concat over groups of [count, n, r], Q state = concat of [count, m, r],
//     r = min(rank, n, m) (:130-144, :237-251);
//   - iteration parity = (step * num_iters_per_step + it) % 2 (:174).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <unistd.h>
#include <algorithm>
#include <cmath>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "psgd.h"
#include "psgd_internal.h"

namespace psgd {
hipError_t launch_even_f32(int R, int nres, const ProductArgs& a, int nwg, hipStream_t s);
hipError_t launch_even_bf16(int R, int nres, const ProductArgs& a, int nwg, hipStream_t s);
int even_resident_f32(int R);
int even_resident_bf16(int R);
hipError_t launch_product_odd_f32(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s);
hipError_t launch_product_odd_bf16(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s);
hipError_t launch_apply_f32(int R, int nterms, bool shared, const ApplyArgs& a, int ntiles, hipStream_t s);
hipError_t launch_apply_bf16(int R, int nterms, bool shared, const ApplyArgs& a, int ntiles, hipStream_t s);
hipError_t launch_odd_mfma_f32(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s);
hipError_t launch_odd_mfma_bf16(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s);
hipError_t launch_final_odd_f32(int R, int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s,
                               int* waves);
hipError_t launch_final_odd_bf16(int R, int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s,
                                int* waves);
hipError_t launch_lowrank_out_f32(int R, int nterms, const ApplyArgs& a, int ntiles, hipStream_t s);
hipError_t launch_lowrank_out_bf16(int R, int nterms, const ApplyArgs& a, int ntiles, hipStream_t s);
hipError_t launch_final_oe_f32(int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s, int* waves);
hipError_t launch_final_oe_bf16(int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s, int* waves);
hipError_t launch_final_oe(int dtype, int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s, int* waves) {
    return dtype == PSGD_F32 ? launch_final_oe_f32(nres, smax, a, ntiles, s, waves)
                             : launch_final_oe_bf16(nres, smax, a, ntiles, s, waves);
}

hipError_t launch_final_odd(int dtype, int R, int nres, int smax, const FinalArgs& a, int ntiles,
                            hipStream_t s, int* waves) {
    return dtype == PSGD_F32 ? launch_final_odd_f32(R, nres, smax, a, ntiles, s, waves)
                             : launch_final_odd_bf16(R, nres, smax, a, ntiles, s, waves);
}
hipError_t launch_lowrank_out(int dtype, int R, int nterms, const ApplyArgs& a, int ntiles, hipStream_t s) {
    return dtype == PSGD_F32 ? launch_lowrank_out_f32(R, nterms, a, ntiles, s)
                             : launch_lowrank_out_bf16(R, nterms, a, ntiles, s);
}
hipError_t launch_odd_mfma(int dtype, int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dtype == PSGD_F32 ? launch_odd_mfma_f32(R, nres, a, ntiles, s)
                             : launch_odd_mfma_bf16(R, nres, a, ntiles, s);
}
hipError_t launch_even(int dtype, int R, int nres, const ProductArgs& a, int nwg, hipStream_t s) {
    return dtype == PSGD_F32 ? launch_even_f32(R, nres, a, nwg, s) : launch_even_bf16(R, nres, a, nwg, s);
}
hipError_t launch_product_odd(int dtype, int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dtype == PSGD_F32 ? launch_product_odd_f32(R, nres, a, ntiles, s)
                             : launch_product_odd_bf16(R, nres, a, ntiles, s);
}
hipError_t launch_apply(int dtype, int R, int nterms, bool shared, const ApplyArgs& a, int ntiles,
                        hipStream_t s) {
    return dtype == PSGD_F32 ? launch_apply_f32(R, nterms, shared, a, ntiles, s)
                             : launch_apply_bf16(R, nterms, shared, a, ntiles, s);
}
}  // namespace psgd

using namespace psgd;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define PSGD_HIP(expr)                                                                   \
    do {                                                                                 \
        const hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess)                                                            \
            return fail(PSGD_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }
int64_t pow2ceil(int64_t x) {
    int64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}
size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

int64_t env_int(const char* name, int64_t dflt) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    return std::atoll(v);
}

struct Geom {
    int lanes, nstrip, nchunk, chunk_rows;
    int64_t part_even, part_odd, ntiles;
};

// Tile geometry of one matrix for a vector width (see psgd_stream.cuh).
Geom geometry(int64_t n, int64_t m, int r, int vec, int64_t tile_elems) {
    const int V = vec ? 4 : 1;
    const int64_t nq = (m + V - 1) / V;
    Geom g;
    g.lanes = int(std::min<int64_t>(64, pow2ceil(nq)));
    const int rows_pass = kWaves * (64 / g.lanes);
    g.nstrip = int((nq + g.lanes - 1) / g.lanes);
    int64_t cr = tile_elems / (int64_t(g.lanes) * V);
    // a small matrix must still spread over several workgroups (its tile is a serial chain)
    cr = std::min<int64_t>(cr, std::max<int64_t>(rows_pass, round_up((n + 7) / 8, rows_pass)));
    cr = std::max<int64_t>(cr, rows_pass);
    cr = round_up(cr, rows_pass);
    cr = std::min(cr, round_up(n, rows_pass));
    g.chunk_rows = int(cr);
    g.nchunk = int((n + cr - 1) / cr);
    g.part_even = int64_t(g.nchunk) * m * r;
    g.part_odd = int64_t(g.nstrip) * n * r;
    g.ntiles = int64_t(g.nchunk) * g.nstrip;
    return g;
}

struct OddGeom {
    int sw, chunk_rows, nstrip, nchunk;
};

// MFMA odd-product tiles: strips of up to 256 columns (kOddSW, psgd_stream.cuh), chunks of
// 64 * g rows (4 waves x 16-row groups x g) sized to about tile_elems elements.
OddGeom odd_geometry(int64_t n, int64_t m, int64_t tile_elems) {
    OddGeom g;
    g.sw = int(std::min<int64_t>(256, round_up(m, 16)));
    const int64_t rows_pass = 16 * kWaves;
    int64_t groups = std::max<int64_t>(1, tile_elems / (rows_pass * g.sw));
    // a small matrix must still spread over several workgroups (as geometry())
    groups = std::min(groups, std::max<int64_t>(1, ((n + 7) / 8 + rows_pass - 1) / rows_pass));
    int64_t cr = std::min(groups * rows_pass, round_up(n, rows_pass));
    g.chunk_rows = int(cr);
    g.nstrip = int((m + g.sw - 1) / g.sw);
    g.nchunk = int((n + cr - 1) / cr);
    return g;
}

struct FinGeom {
    int T, S, rows;
    int64_t ntiles;
};

// Fused final odd pass (psgd_final.cuh): row groups of T threads (4 columns each, S
// segments), fin_rb(R) rows per group per batch, blocks of about fin_elems elements.
#ifndef PSGD_FIN_RB12
#define PSGD_FIN_RB12 1
#endif
int fin_rb(int R) { return R == 4 ? 1 : PSGD_FIN_RB12; }   // == FinRB<R>
#ifndef PSGD_FIN_NT4
#define PSGD_FIN_NT4 256  // == psgd_final.cuh
#endif
int fin_nt(int R) { return R == 4 ? PSGD_FIN_NT4 : 256; }  // == FinNT<R>
// scap = 0: the widest row group (T = min(threads, 4-column units rounded up to a power of
// two), fewest segments). scap > 0: the row group with the fewest idle lanes among
// S <= scap (ties: the narrower group — more rows per batch and, at T <= 64, a row sum
// within one wave instead of across waves through LDS); e.g. m = 576: T = 32, S = 5 (10 %
// idle) rather than T = 256, S = 1 (44 % idle).
FinGeom fin_geometry(int64_t n, int64_t m, int R, int64_t fin_elems, int scap = 0) {
    FinGeom g;
    const int nt = fin_nt(R), rb = fin_rb(R);
    const int64_t q4 = (m + 3) / 4;
    g.T = int(std::min<int64_t>(nt, pow2ceil(q4)));
    g.S = int((q4 + g.T - 1) / g.T);
    if (scap > 0) {
        int64_t best = int64_t(g.S) * g.T;
        for (int T = g.T / 2; T >= 4; T /= 2) {
            const int64_t S = (q4 + T - 1) / T;
            if (S > scap) break;
            if (S * T <= best) {
                best = S * T;
                g.T = T;
                g.S = int(S);
            }
        }
    }
    const int64_t batch = int64_t(nt / g.T) * rb;  // rows per workgroup batch
    int64_t rows = round_up(std::max<int64_t>(1, (fin_elems + m - 1) / m), batch);
    // a small matrix must still spread over several workgroups
    rows = std::min(rows, std::max(batch, round_up((n + 7) / 8, batch)));
    rows = std::min(rows, round_up(n, batch));
    // at most kFinRowsMax rows (a multiple of batch)
    rows = std::min(rows, std::max(batch, kFinRowsMax / batch * batch));
    g.rows = int(rows);
    g.ntiles = (n + rows - 1) / rows;
    return g;
}

int fin_bucket(int s) { return s <= 2 ? 2 : s <= 3 ? 3 : s <= 5 ? 5 : s <= 12 ? 12 : 0; }
// widest register-segment instance of the K-term final kernels per rank bucket (psgd_final.cuh)
int fin_smax_inst(int R) { return R <= 2 || PSGD_FIN_NT4 == 256 ? 5 : 3; }

// Device-resident pointer tables (gradients, destinations) without a host synchronisation.
// kSlots tables live in the caller's workspace; a call whose pointer set matches a slot uses
// it as is (callers that rotate a few gradient sets, or get fresh tensors from the caching
// allocator, hit after the first round). A miss takes the least recently used slot and
// uploads into it with hipMemcpyAsync ON THE LAUNCH STREAM from a pinned staging copy, so
// the copy is ordered after every earlier launch on that stream that may still read the
// slot, and the host never waits (the reference hands tensors to torch ops, which never
// synchronise either). Calls of one plan must be ordered on one stream (as torch's are).
struct TableCache {
    static constexpr int kSlots = 4;
    size_t n = 0;              // pointers per table
    char* dev = nullptr;       // kSlots * n pointers inside the workspace
    std::vector<void*> host[kSlots];
    uint64_t stamp[kSlots] = {};
    uint64_t clock = 0;
    int cur = -1;
    void** pinned = nullptr;   // kSlots * n staging pointers (hipHostMalloc)
    hipEvent_t ev[kSlots] = {};
    bool live[kSlots] = {};

    static size_t bytes(size_t n) { return size_t(kSlots) * std::max<size_t>(n, 1) * sizeof(void*); }
    void bind(char* d, size_t count) {
        release();
        dev = d;
        n = count;
        for (auto& h : host) h.clear();
        cur = -1;
    }
    void release() {
        for (int i = 0; i < kSlots; ++i) {
            if (live[i]) (void)hipEventSynchronize(ev[i]);
            if (ev[i]) (void)hipEventDestroy(ev[i]);
            ev[i] = nullptr;
            live[i] = false;
        }
        if (pinned) (void)hipHostFree(pinned);
        pinned = nullptr;
    }
    ~TableCache() { release(); }
    bool match(int i, void* const* p) const {
        if (host[i].size() != n) return false;
        for (size_t k = 0; k < n; ++k)
            if (host[i][k] != p[k]) return false;
        return true;
    }
    // 0 on success, else a hipError_t
    hipError_t select(void* const* p, hipStream_t s) {
        ++clock;
        if (cur >= 0 && match(cur, p)) {
            stamp[cur] = clock;
            return hipSuccess;
        }
        int victim = 0;
        for (int i = 0; i < kSlots; ++i) {
            if (match(i, p)) {
                cur = i;
                stamp[i] = clock;
                return hipSuccess;
            }
            if (stamp[i] < stamp[victim]) victim = i;
        }
        if (!pinned) {
            hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&pinned), bytes(n), hipHostMallocDefault);
            if (e != hipSuccess) {
                pinned = nullptr;
                return e;
            }
            for (int i = 0; i < kSlots; ++i)
                if ((e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming)) != hipSuccess) return e;
        }
        // the staging slot may still feed the previous upload into this slot
        if (live[victim]) {
            const hipError_t e = hipEventSynchronize(ev[victim]);
            if (e != hipSuccess) return e;
        }
        void** stage = pinned + size_t(victim) * n;
        std::copy(p, p + n, stage);
        hipError_t e = hipMemcpyAsync(dev + size_t(victim) * n * sizeof(void*), stage, n * sizeof(void*),
                                      hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipEventRecord(ev[victim], s);
        if (e != hipSuccess) return e;
        live[victim] = true;
        host[victim].assign(p, p + n);
        stamp[victim] = clock;
        cur = victim;
        return hipSuccess;
    }
    void* const* table() const { return reinterpret_cast<void* const*>(dev + size_t(cur) * n * sizeof(void*)); }
};

struct DevScope {  // make `dev` current for the scope, restore afterwards
    int prev = -1;
    explicit DevScope(int dev) {
        (void)hipGetDevice(&prev);
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DevScope() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

// ---------------------------------------------------- process-lifetime IPC exchange arena ---
// Exchange buffers of the one-shot all-reduce (psgd_ipc_*) are REGIONS of per-device chunks that
// this process allocates once and never frees, and every peer chunk is mapped once per process
// and never unmapped (round 6). A session (psgd_ipc_create .. psgd_ipc_close) takes a region,
// zeroes its header and draws a fresh nonce; a later session of the same size gets the same
// region back. There is no hipFree -> hipMalloc -> hipIpcOpenMemHandle cycle between two
// sessions of one process, so a peer can never be handed a mapping of a freed buffer (the
// round-5 r05a-new mismatch: the second same-size session after a closed one read stale sums,
// which a cached mapping of the first session's freed allocation, whose flags still carried
// higher epochs than the new session's, produces exactly). The nonce check at open and the
// nonce-tagged flags stay as guards.
struct XchgChunk {
    int device = -1;
    char* base = nullptr;
    size_t bytes = 0;
    hipIpcMemHandle_t handle{};
};

class XchgArena {
  public:
    static constexpr size_t kAlign = 4096;
    static constexpr size_t kMinChunk = size_t(64) << 20;

    // a region of at least `bytes` on `device`: first fit in a free range, else a new chunk
    int acquire(int device, size_t bytes, int* chunk, size_t* off) {
        std::lock_guard<std::mutex> lock(mu_);
        bytes = (bytes + kAlign - 1) & ~(kAlign - 1);
        for (size_t i = 0; i < free_.size(); ++i) {
            Range& f = free_[i];
            if (chunks_[size_t(f.chunk)].device != device || f.bytes < bytes) continue;
            *chunk = f.chunk;
            *off = f.off;
            f.off += bytes;
            f.bytes -= bytes;
            if (f.bytes == 0) free_.erase(free_.begin() + long(i));
            ++reuses_;
            return PSGD_OK;
        }
        XchgChunk c;
        c.device = device;
        c.bytes = std::max(kMinChunk, (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1));
        if (hipMalloc(reinterpret_cast<void**>(&c.base), c.bytes) != hipSuccess)
            return fail(PSGD_ERR_DEVICE, "hipMalloc of the IPC exchange arena failed");
        if (hipIpcGetMemHandle(&c.handle, c.base) != hipSuccess) {
            (void)hipFree(c.base);  // never exported: no peer can map it
            return fail(PSGD_ERR_DEVICE, "hipIpcGetMemHandle of the IPC exchange arena failed");
        }
        chunks_.push_back(c);
        ++allocs_;
        *chunk = int(chunks_.size()) - 1;
        *off = 0;
        if (c.bytes > bytes) free_.push_back(Range{*chunk, bytes, c.bytes - bytes});
        return PSGD_OK;
    }
    // give a region back (its bytes stay allocated and exported; adjacent free ranges merge)
    void release(int chunk, size_t off, size_t bytes) {
        std::lock_guard<std::mutex> lock(mu_);
        bytes = (bytes + kAlign - 1) & ~(kAlign - 1);
        Range r{chunk, off, bytes};
        for (size_t i = 0; i < free_.size();) {
            Range& f = free_[i];
            if (f.chunk == r.chunk && (f.off + f.bytes == r.off || r.off + r.bytes == f.off)) {
                r.off = std::min(r.off, f.off);
                r.bytes += f.bytes;
                free_.erase(free_.begin() + long(i));
                i = 0;
            } else {
                ++i;
            }
        }
        free_.push_back(r);
    }
    XchgChunk chunk(int i) {
        std::lock_guard<std::mutex> lock(mu_);
        return chunks_[size_t(i)];
    }
    // the process's mapping of a peer chunk: opened at the first session that needs it, kept
    // for the life of the process (the peer never frees the chunk either)
    int map_peer(int device, const hipIpcMemHandle_t& h, char** base) {
        std::lock_guard<std::mutex> lock(mu_);
        std::string key(reinterpret_cast<const char*>(&h), sizeof(h));
        key += std::to_string(device);
        auto it = peers_.find(key);
        if (it != peers_.end()) {
            *base = it->second;
            return PSGD_OK;
        }
        void* v = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&v, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return fail(PSGD_ERR_DEVICE, std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
        ++opens_;
        *base = static_cast<char*>(v);
        peers_.emplace(key, *base);
        return PSGD_OK;
    }
    void counters(int64_t* out) {
        std::lock_guard<std::mutex> lock(mu_);
        out[0] = allocs_;   // chunks allocated (hipMalloc) by this process
        out[1] = opens_;    // peer chunks mapped (hipIpcOpenMemHandle) by this process
        out[2] = reuses_;   // regions served from already-allocated chunks
        out[3] = 0;         // chunks freed: never
    }

  private:
    struct Range {
        int chunk;
        size_t off, bytes;
    };
    std::mutex mu_;
    std::vector<XchgChunk> chunks_;
    std::vector<Range> free_;
    std::map<std::string, char*> peers_;
    int64_t allocs_ = 0, opens_ = 0, reuses_ = 0;
};

XchgArena& xchg_arena() {
    static XchgArena* a = new XchgArena();  // never destroyed: chunks and mappings live to exit
    return *a;
}

}  // namespace

namespace psgd {
int comm_fail(int code, const char* msg) { return fail(code, msg); }
thread_local const KernelTiming* g_kernel_timing = nullptr;
}  // namespace psgd

// Persistent even product (k_even): workgroups per launch (CUs x workgroups per CU), at least
// kEvenMinElems gradient elements per workgroup (small plans use fewer, fuller workgroups), at
// most kMaxBuckets buckets (each bucket launch spreads over the whole chip).
constexpr int kCUs = 256;                // MI355X
constexpr int kEvenWpcMax = 16;          // k_even workgroups per CU (PSGD_EVEN_WPC cap)
constexpr int kEvenWgMax = kEvenWpcMax * kCUs;  // workgroups per launch (capacity)
constexpr int kMaxBuckets = 8;

struct psgd_plan {
    int rank = 0, iters = 0, dtype = 0;
    std::vector<std::vector<int64_t>> shapes;
    struct Group {
        int64_t n, m;
        int r;
        std::vector<int> tensors;
        int64_t poff, qoff;
    };
    std::vector<Group> groups;
    std::vector<MatDesc> mats;  // group order
    std::vector<int> base_vec;  // vector path possible by shape (m % 4 == 0, r <= 8)
    std::vector<int> vec_now;   // currently active vector flags
    std::vector<int64_t> out_off;
    int64_t out_total = 0, ptot = 0, qtot = 0, fmax = 0;
    int rbucket = 1;
    int64_t tile_elems = 16384;
    std::vector<Tile> tiles;     // lane-column tiles of every matrix (apply, low-rank output)
    std::vector<Tile> tiles_ov;  // lane-column tiles of the odd-VALU matrices
    std::vector<Tile> tiles_om;  // MFMA tiles of the odd-MFMA matrices
    std::vector<Tile> tiles_fin; // row blocks of the fused final odd pass
    // the K-term form's own row blocks when they differ from the projection form's (MatDesc::
    // fin_rows_kt); empty: the K-term form uses tiles_fin
    std::vector<Tile> tiles_fin_kt;
    bool fin_ok = false;         // every matrix fits the fused final odd pass (K-term form)
    bool fin_proj = false;       // ... in its projection form (I = 2, psgd_aggregate only)
    bool orth_chol = true;       // PSGD_ORTH_CHOL, read at set_vec (Cholesky-QR vs Householder)
    int fin_smax = 0;
    int64_t fin_elems = 32768, tiles_fin_cap = 0;
    int64_t fin_elems_kt = 32768, tiles_fin_kt_cap = 0;
    // output stores of the fused final pass nt only (psgd_stream.cuh kStAuxOutNt): plans whose
    // gradients exceed PSGD_OUT_NT_MB (default 32) MB; smaller plans keep the write-through policy
    int32_t out_nt = 0;
    int64_t tiles_cap = 0, tiles_om_cap = 0;
    // even product (k_even): segments, per-workgroup segment ranges (wg_seg[w] .. wg_seg[w+1]),
    // workgroups per CU and the minimum elements per workgroup (read at create)
    std::vector<Seg> segs;
    std::vector<int32_t> wg_seg;
    int even_wpc = 4;
    int64_t even_segc = 4096;  // k_even cost model: elements-equivalent of one segment's fixed cost
    int64_t even_min = 16384;
    int64_t segs_cap = 0, even_part_cap = 0, ss0_cap = 0;
    // odd-even pass (k_final_oe: rank 1, world size 1, I >= 3): an odd iteration followed by an
    // even one inside a step in ONE gradient pass; its partials (per K-term row block, [m]) are
    // summed by k_reduce over red_oe, the blocks' sums of P^2 (oe_ss) give the even iteration's
    // joint norm (grng_oe: per group its block range), and the items' sums of squares feed the
    // next fused iteration (grng_oe_items: per group its red_oe range)
    bool oe_ok = false;
    std::vector<RedItem> red_oe;
    std::vector<Tile> tiles_oe;  // its row blocks (MatDesc::oe_rows rows)
    std::vector<int32_t> grng_oe, grng_oe_items;
    int64_t oe_part_floats = 0;
    int32_t oe_blocks = 0;
    size_t o_oe_part = 0, o_oe_ss = 0, o_red_oe = 0, o_grng_oe = 0, o_grng_oe_items = 0, o_tiles_oe = 0;
    bool oe_at(int64_t step, int it, bool agg) const {  // iteration `it` runs the odd-even pass
        return oe_ok && agg && it >= 1 && it + 1 < iters && !even(step, it);
    }
    // reduction items (rebuilt with the geometry): even items follow the segmentation
    std::vector<RedItem> red_even, red_odd;
    std::vector<int32_t> grng_even, grng_odd;  // per group: [begin, end) of its reduction items
    int64_t red_even_cap = 0, red_odd_cap = 0;
    std::vector<OrthUnit> units_p, units_q;
    std::vector<OrthUnit> munits_p, munits_q;  // one unit per MATRIX (paper-code Gram-Schmidt)
    size_t o_munits_p = 0, o_munits_q = 0, o_rdst = 0, o_odst = 0;
    TableCache grad_tab, rdst_tab, odst_tab;  // device pointer tables (gradients, destinations)
    int64_t panel_p = 0, panel_q = 0;
    int64_t part_odd_floats = 0;  // odd partials [odd strips][n][r] per matrix; even ones follow
    double unc_floats = 0, comp_floats = 0;
    size_t o_ptrs = 0, o_mats = 0, o_tiles = 0, o_tiles_ov = 0, o_tiles_om = 0, o_tiles_fin = 0, o_tiles_fin_kt = 0, o_red_even = 0,
           o_red_odd = 0, o_units_p = 0, o_units_q = 0, o_hist = 0, o_part = 0, o_grng_even = 0,
           o_grng_odd = 0, o_ss = 0, ss_stride = 0, o_ss0 = 0, o_grng_ss0 = 0, o_segs = 0, o_wg_seg = 0,
           ws_bytes = 0;
    // rank-1 iteration-0 norm fold: per strip-0 segment a sum-of-squares slot, and per group the
    // [begin, end) slot range
    std::vector<int32_t> grng_ss0;
    // Buckets of whole shape groups (W > 1 overlap, psgd_plan_set_buckets): per bucket the
    // [begin, end) range of every launch list (all are in matrix order) and of the P/Q buffers.
    struct Span {
        int32_t tiles[2], ov[2], om[2], fin[2], fin_kt[2], re[2], ro[2], up[2], uq[2], wg[2];
        int64_t p[2], q[2];
    };
    std::vector<int32_t> bucket_gend;              // exclusive group end per bucket
    std::vector<int32_t> bucket_wg;                // per bucket [begin, end) of its k_even workgroups
    std::vector<Span> spans;
    std::vector<int32_t> unit_group_p, unit_group_q;
    Span full_span() const {
        Span sp{};
        sp.tiles[1] = int32_t(tiles.size());
        sp.ov[1] = int32_t(tiles_ov.size());
        sp.om[1] = int32_t(tiles_om.size());
        sp.fin[1] = int32_t(tiles_fin.size());
        sp.fin_kt[1] = int32_t(tiles_fin_kt.size());
        sp.re[1] = int32_t(red_even.size());
        sp.ro[1] = int32_t(red_odd.size());
        sp.up[1] = int32_t(units_p.size());
        sp.uq[1] = int32_t(units_q.size());
        sp.wg[1] = int32_t(wg_seg.empty() ? 0 : wg_seg.size() - 1);
        sp.p[1] = ptot;
        sp.q[1] = qtot;
        return sp;
    }
    void build_spans() {
        spans.clear();
        int32_t g0 = 0;
        for (size_t b = 0; b < bucket_gend.size(); ++b) {
            const int32_t g1 = bucket_gend[b];
            auto in = [&](int32_t mat) { const int32_t g = mats[mat].group; return g >= g0 && g < g1; };
            auto range = [&](const auto& v, auto key, int32_t (&r)[2]) {
                r[0] = int32_t(v.size());
                r[1] = 0;
                for (size_t i = 0; i < v.size(); ++i)
                    if (key(v[i])) {
                        r[0] = std::min(r[0], int32_t(i));
                        r[1] = int32_t(i) + 1;
                    }
                if (r[1] == 0) r[0] = 0;
            };
            Span sp{};
            auto tk = [&](const Tile& t) { return in(t.mat); };
            auto rk = [&](const RedItem& it) { return in(it.mat); };
            range(tiles, tk, sp.tiles);
            range(tiles_ov, tk, sp.ov);
            range(tiles_om, tk, sp.om);
            range(tiles_fin, tk, sp.fin);
            range(tiles_fin_kt, tk, sp.fin_kt);
            range(red_even, rk, sp.re);
            range(red_odd, rk, sp.ro);
            range(unit_group_p, [&](int32_t g) { return g >= g0 && g < g1; }, sp.up);
            range(unit_group_q, [&](int32_t g) { return g >= g0 && g < g1; }, sp.uq);
            sp.wg[0] = bucket_wg[2 * b];
            sp.wg[1] = bucket_wg[2 * b + 1];
            sp.p[0] = groups[g0].poff;
            sp.q[0] = groups[g0].qoff;
            sp.p[1] = g1 < int32_t(groups.size()) ? groups[g1].poff : ptot;
            sp.q[1] = g1 < int32_t(groups.size()) ? groups[g1].qoff : qtot;
            spans.push_back(sp);
            g0 = g1;
        }
    }

    // fp64 plans (psgd_f64.hip): even tiles (64-column strip, 256-row chunk), odd tiles
    // (16-row blocks), apply tiles (row chunks of ~16k elements), even partial offsets
    std::vector<Tile> f64_even, f64_odd, f64_apply;
    std::vector<int64_t> f64_part_off;
    int64_t f64_part = 0;
    size_t o_f64_even = 0, o_f64_odd = 0, o_f64_apply = 0, o_f64_partoff = 0, o_f64_part = 0;
    bool bound = false;
    int device = -1;
    float* P = nullptr;
    float* Q = nullptr;
    char* ws = nullptr;
    void* out_now = nullptr;  // psgd_aggregate's output buffer (fused final pass)
    // benchmark timing of the final pass: event pairs recorded on the launch stream
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
    size_t ev_used = 0;
    // one-shot IPC all-reduce (psgd_ipc_*, psgd_aggregate_ipc): this rank's exchange buffer
    // (hipMalloc'd so that it can be exported: flags header + 2 parities x iters slots), the
    // peers' opened mappings, the slot size (floats: factor region, then the flat region)
    char* ipc_buf = nullptr;      // this session's region of the process's exchange arena
    int ipc_chunk = -1;           // the region: arena chunk, byte offset and size
    size_t ipc_off = 0, ipc_bytes = 0;
    std::vector<void*> ipc_peer;
    int ipc_world = 0, ipc_rank = -1;
    int64_t ipc_slot = 0, ipc_flat_off = 0, ipc_flat_cap = 0;
    size_t o_ipc_ptrs = 0, o_ipc_nonce = 0;
    uint32_t ipc_nonce = 0;  // this rank's exchange session (psgd_ipc_create)
    // sticky timeout word of the exchange waits: pinned host memory mapped into the device
    // (k_xchg stores 1 with a system-scope store), so every psgd_aggregate_ipc call can check it
    // without synchronising; cleared only by psgd_ipc_close
    int32_t* xerr_host = nullptr;
    int32_t* xerr_dev = nullptr;
    bool xerr_set() const { return xerr_host && __atomic_load_n(xerr_host, __ATOMIC_ACQUIRE) != 0; }
    float* xout_now = nullptr;  // set per iteration by psgd_aggregate_ipc (exchange slot)
    unsigned long long* stamp_buf = nullptr;  // diagnostic k_even stamps (PSGD_EVEN_STAMPS)
    size_t stamp_words = 0;
    // history slot of the RAW in-factor the rank-1 norm fold reads: 1 (the local reduction's
    // output, world size 1) or 2 (the exchange's summed copy, psgd_aggregate_ipc)
    int raw_slot = 1;
    // psgd_aggregate_ipc, ranks 2/4, two iterations: the exchange of iteration 0 left the summed
    // Q panels' Gram partials, so iteration 1 orthonormalises with k_orth_chain
    bool xgram_now = false;
    int64_t xslot_off(int64_t step, int it) const {  // byte offset of a slot in every buffer
        return kXchgHeader + ((step & 1) * iters + it) * ipc_slot * int64_t(sizeof(float));
    }
    float* xslot(int64_t step, int it) const { return reinterpret_cast<float*>(ipc_buf + xslot_off(step, it)); }
    size_t o_rq = 0;  // R' of the last iteration's in-factor panels (projection form), Q layout
    // folded orthonormalisation of the projection form's Q panels (k_orth_chain): every Q unit
    // a single panel of exactly rbucket in {2, 4} columns; per-item Gram partials and per-unit
    // item ranges
    bool qfold_ok = false;
    size_t o_gram = 0, o_uitems = 0;
    std::vector<int32_t> uitems, red_even_b, red_even_e;
    std::vector<int32_t> mrng_even;  // per matrix [begin, end) of its even reduction items
    size_t o_mrng = 0;
    bool qfold(int64_t step, bool agg) const { return qfold_ok && iters == 2 && proj_final(step, agg); }

    ~psgd_plan() {
        for (auto& e : ev_pool) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        // the exchange region goes back to the process's arena (never freed, never unmapped:
        // a peer's mapping stays valid; teardown is still collective, psgd_ipc_close + barrier,
        // so that no peer kernel reads the region when a later session re-zeroes it)
        if (ipc_buf) xchg_arena().release(ipc_chunk, ipc_off, ipc_bytes);
        if (xerr_host) (void)hipHostFree(xerr_host);
        if (stamp_buf) (void)hipFree(stamp_buf);
    }

    float* hist(int which, int k) const {  // 0: X (orthonormal in-factor), 1: Y local, 2: Y reduced
        return reinterpret_cast<float*>(ws + o_hist) + (int64_t(which) * iters + k) * fmax;
    }
    double* hist64(int which, int k) const {  // the same history, fp64 plans
        return reinterpret_cast<double*>(ws + o_hist) + (int64_t(which) * iters + k) * fmax;
    }
    bool f64() const { return dtype == PSGD_F64; }
    void set_f64_tiles() {
        f64_even.clear();
        f64_odd.clear();
        f64_apply.clear();
        f64_part_off.clear();
        f64_part = 0;
        vec_now = base_vec;
        red_even.clear();
        red_odd.clear();
        for (size_t i = 0; i < mats.size(); ++i) {
            MatDesc& d = mats[i];
            d.vec = 0;
            d.nstrip = int32_t((d.m + kF64Cols - 1) / kF64Cols);
            d.nchunk = int32_t((d.n + kF64Rows - 1) / kF64Rows);
            d.chunk_rows = int32_t(std::max<int64_t>(1, 16384 / d.m));  // apply: ~16k elements per tile
            for (int c = 0; c < d.nchunk; ++c)
                for (int st = 0; st < d.nstrip; ++st) f64_even.push_back(Tile{int32_t(i), st, c, 0});
            for (int64_t b = 0; b * kF64OddRows < d.n; ++b) f64_odd.push_back(Tile{int32_t(i), 0, int32_t(b), 0});
            for (int64_t b = 0; b * d.chunk_rows < d.n; ++b) f64_apply.push_back(Tile{int32_t(i), 0, int32_t(b), 0});
            f64_part_off.push_back(f64_part);
            f64_part += int64_t(d.nchunk) * kWaves * d.m * d.r;
            // k_f64_reduce: 64 consecutive Q elements per item (start only)
            for (int64_t s = 0; s < d.m * d.r; s += kRedElems)
                red_even.push_back(RedItem{int32_t(i), int32_t(s), 1, int32_t(std::min<int64_t>(kRedElems, d.m * d.r - s)), 0, 0, 0});
        }
    }
    template <typename T>
    T* dev(size_t off) const { return reinterpret_cast<T*>(ws + off); }
    bool even(int64_t step, int it) const { return ((step * iters + it) % 2) == 0; }

    // Even-product segmentation (k_even) and every reduction item list, for the current strip
    // geometry and buckets. Per bucket (or the whole plan), the gradient elements of its
    // matrices (walked matrix -> strip -> row) are cut into nwg equal ranges, one per workgroup;
    // a segment ends at a strip end or at a workgroup's range end. Partials: per strip, its
    // segments' [W x r] slabs in row order (W = lanes x V strip columns).
    void build_reduction() {
        segs.clear();
        wg_seg.clear();
        bucket_wg.clear();
        red_even.clear();
        red_odd.clear();
        red_even_b.assign(mats.size(), 0);
        red_even_e.assign(mats.size(), 0);
        grng_even.assign(2 * groups.size(), 0);
        grng_odd.assign(2 * groups.size(), 0);
        grng_ss0.assign(2 * groups.size(), 0);
        std::vector<int32_t> ends = bucket_gend;
        if (ends.empty()) ends.push_back(int32_t(groups.size()));
        // pass 1: segments per bucket
        std::vector<std::vector<int32_t>> nseg(mats.size());  // per matrix, per strip: segment count
        for (size_t i = 0; i < mats.size(); ++i) nseg[i].assign(size_t(mats[i].nstrip), 0);
        size_t mi = 0;
        for (int32_t g1 : ends) {
            size_t m0 = mi;
            while (mi < mats.size() && mats[mi].group < g1) ++mi;
            int64_t total = 0;
            for (size_t i = m0; i < mi; ++i) total += mats[i].n * mats[i].m;
            int64_t nwg_launch = std::max<int64_t>(
                1, std::min<int64_t>(int64_t(even_wpc) * kCUs, (total + even_min - 1) / std::max<int64_t>(even_min, 1)));
            const int64_t nwg = nwg_launch;  // ranges cut below, one per workgroup
            bucket_wg.push_back(int32_t(wg_seg.size()));
            int64_t cum = 0, w = 0;
            wg_seg.push_back(int32_t(segs.size()));
            auto make = [&](size_t i, int s, int64_t r0, int64_t r1) {
                const MatDesc& d = mats[i];
                Seg sg{};
                sg.m = d.m;
                sg.poff = d.poff;
                sg.qoff = d.qoff;
                sg.row0 = int32_t(r0);
                sg.row1 = int32_t(r1);
                sg.strip = s;
                sg.tensor = d.tensor;
                sg.ss = -1;
                sg.r = d.r;
                sg.lanes = d.lanes;
                sg.vec = d.vec;
                // full-width strips of an r == R matrix take k_even's scalar-row fast path
                if (d.vec && d.lanes == 64 && d.r == rbucket && rbucket <= 8) sg.vec = 2;
                sg.part = int64_t(i);  // matrix index for now (pass 2)
                segs.push_back(sg);
                ++nseg[i][size_t(s)];
            };
            // Cost model (round 4, the per-workgroup stamps of profiles/r04/b): a workgroup's
            // time is its gradient loads plus a fixed cost per segment (descriptor loads, a
            // fresh load batch, the epilogue: ~1.5-2 us, i.e. even_segc elements at one
            // workgroup's streaming rate), and a scalar-column strip (V = 1: 256 B per wave
            // load instead of 1 KB) costs 4x per element. Equal COST ranges instead of equal
            // bytes: the first workgroup used to take the five narrow segments of conv1 and the
            // first 64-row matrices and finish last (22 us against p99 19 us).
            const int64_t segc = even_segc;
            // (ranks 16 / 32: m % 4 == 0 strips stream 16-byte row quads on the matrix cores,
            // even_seg_mfma, at the vector rate)
            auto rowc = [&](const MatDesc& d, int64_t cols) {
                return cols * ((d.vec || (rbucket >= 16 && d.m % 4 == 0)) ? 1 : 4);
            };
            int64_t totw = nwg * segc;
            for (size_t i = m0; i < mi; ++i) {
                const MatDesc& d = mats[i];
                const int64_t W = int64_t(d.lanes) * (d.vec ? 4 : 1);
                for (int s = 0; s < d.nstrip; ++s) totw += d.n * rowc(d, std::min<int64_t>(W, d.m - s * W)) + segc;
            }
            // (a dispatch-order skew, more cost to low block indices, was measured and does not
            // help: the late blocks finish late whatever their share, profiles/r04/e)
            auto wbound = [&](int64_t ww) { return ww + 1 >= nwg ? totw : (ww + 1) * totw / nwg; };
            for (size_t i = m0; i < mi; ++i) {
                const MatDesc& d = mats[i];
                const int64_t W = int64_t(d.lanes) * (d.vec ? 4 : 1);
                for (int s = 0; s < d.nstrip; ++s) {
                    const int64_t cols = std::min<int64_t>(W, d.m - s * W);
                    const int64_t rc = rowc(d, cols);
                    // k_even addresses a segment with 32-bit offsets: at most 2^30 bytes each
                    const int64_t es = dtype == PSGD_BF16 ? 2 : 4;
                    const int64_t seg_max = std::max<int64_t>(1, ((int64_t(1) << 30) / (d.m * es)) - 64);
                    int64_t r0 = 0;
                    while (r0 < d.n) {
                        int64_t take = std::min(d.n - r0, seg_max);
                        if (w < nwg - 1) {
                            // rows to this range's end, after paying the segment's fixed cost
                            const int64_t fit = (wbound(w) - cum - segc + rc / 2) / rc;
                            if (fit <= 0) {
                                ++w;
                                wg_seg.push_back(int32_t(segs.size()));
                                continue;
                            }
                            take = std::min(take, fit);
                        }
                        make(i, s, r0, r0 + take);
                        cum += segc + take * rc;
                        r0 += take;
                        if (w < nwg - 1 && cum >= wbound(w)) {  // this range is full
                            ++w;
                            wg_seg.push_back(int32_t(segs.size()));
                        }
                    }
                }
            }
            while (int64_t(wg_seg.size()) - bucket_wg.back() < nwg + 1) wg_seg.push_back(int32_t(segs.size()));
            bucket_wg.push_back(int32_t(wg_seg.size()) - 1);
        }
        // wg_seg holds nwg + 1 bounds per bucket; the buckets' ranges are concatenated so that
        // workgroup w of the whole launch reads wg_seg[w], wg_seg[w + 1]: drop each bucket's
        // closing bound except the last
        {
            std::vector<int32_t> flat;
            std::vector<int32_t> bw;
            for (size_t b = 0; b * 2 < bucket_wg.size(); ++b) {
                const int32_t lo = bucket_wg[2 * b], hi = bucket_wg[2 * b + 1];
                bw.push_back(int32_t(flat.size()));
                for (int32_t k = lo; k < hi; ++k) flat.push_back(wg_seg[size_t(k)]);
                bw.push_back(int32_t(flat.size()));
            }
            flat.push_back(int32_t(segs.size()));
            wg_seg.swap(flat);
            bucket_wg.swap(bw);
        }
        // pass 2: partial slabs (per matrix, per strip, segments in row order) and ss slots
        std::vector<std::vector<int64_t>> base(mats.size());
        int64_t off = (part_odd_floats + 3) & ~int64_t(3);
        for (size_t i = 0; i < mats.size(); ++i) {
            const MatDesc& d = mats[i];
            const int64_t W = int64_t(d.lanes) * (d.vec ? 4 : 1);
            base[i].assign(size_t(d.nstrip), 0);
            for (int s = 0; s < d.nstrip; ++s) {
                base[i][size_t(s)] = off;
                off += (int64_t(nseg[i][size_t(s)]) * W * d.r + 3) & ~int64_t(3);
            }
        }
        std::vector<std::vector<int32_t>> kseg(mats.size());
        for (size_t i = 0; i < mats.size(); ++i) kseg[i].assign(size_t(mats[i].nstrip), 0);
        int32_t ss = 0;
        // strip-0 segments get consecutive slots in matrix order (a group's slots contiguous)
        std::vector<std::vector<int32_t>> s0(mats.size());
        for (Seg& sg : segs) {
            const size_t i = size_t(sg.part);
            const MatDesc& d = mats[i];
            const int64_t W = int64_t(d.lanes) * (d.vec ? 4 : 1);
            const int32_t k = kseg[i][size_t(sg.strip)]++;
            sg.part = base[i][size_t(sg.strip)] + int64_t(k) * W * d.r;
            if (sg.strip == 0) s0[i].push_back(int32_t(&sg - segs.data()));
        }
        for (size_t i = 0; i < mats.size(); ++i) {
            const int g = mats[i].group;
            if (i == 0 || mats[i - 1].group != g) grng_ss0[2 * g] = ss;
            for (int32_t si : s0[i]) segs[size_t(si)].ss = ss++;
            grng_ss0[2 * g + 1] = ss;
        }
        // reduction items: even ones per strip (its segments' partials), odd ones per matrix
        for (size_t i = 0; i < mats.size(); ++i) {
            const MatDesc& d = mats[i];
            const int g = d.group;
            const bool first = i == 0 || mats[i - 1].group != g;
            if (first) {
                grng_even[2 * g] = int32_t(red_even.size());
                grng_odd[2 * g] = int32_t(red_odd.size());
            }
            const int64_t W = int64_t(d.lanes) * (d.vec ? 4 : 1);
            red_even_b[i] = int32_t(red_even.size());
            for (int s = 0; s < d.nstrip; ++s) {
                const int np = nseg[i][size_t(s)];
                const int pe = np > kRedWide ? 1 : 4;
                const int64_t e0 = s * W * d.r, e1 = std::min<int64_t>((s + 1) * W, d.m) * d.r;
                for (int64_t e = e0; e < e1; e += 64 * pe)
                    red_even.push_back(RedItem{int32_t(i), int32_t(e), pe, int32_t(std::min<int64_t>(64 * pe, e1 - e)),
                                               base[i][size_t(s)] + (e - e0), int32_t(W * d.r), np});
            }
            red_even_e[i] = int32_t(red_even.size());
            const int npo = d.odd_nstrip;
            const int po = npo > kRedWide ? 1 : 4;
            for (int64_t e = 0; e < d.n * d.r; e += 64 * po)
                red_odd.push_back(RedItem{int32_t(i), int32_t(e), po, int32_t(std::min<int64_t>(64 * po, d.n * d.r - e)),
                                          d.part_odd + e, int32_t(d.n * d.r), npo});
            grng_even[2 * g + 1] = int32_t(red_even.size());
            grng_odd[2 * g + 1] = int32_t(red_odd.size());
        }
        mrng_even.clear();
        for (size_t i = 0; i < mats.size(); ++i) {
            mrng_even.push_back(red_even_b[i]);
            mrng_even.push_back(red_even_e[i]);
        }
        // folded orthonormalisation: per Q unit (one matrix each) its even item range
        uitems.clear();
        if (qfold_ok) {
            for (const OrthUnit& u : units_q)
                for (size_t i = 0; i < mats.size(); ++i)
                    if (mats[i].qoff == u.off) {
                        uitems.push_back(red_even_b[i]);
                        uitems.push_back(red_even_e[i]);
                    }
        }
    }

    void set_vec(const std::vector<int>& vec) {
        vec_now = vec;
        tiles.clear();
        tiles_ov.clear();
        tiles_om.clear();
        tiles_fin.clear();
        tiles_fin_kt.clear();
        // PSGD_FUSE_FINAL: 0 off; 1 (default) the fused forms (K-term at ranks 1-2, projection at
        // ranks 1/2/4). The rank-4 K-term form (two register panels: 253 VGPRs, one 512-thread
        // workgroup per CU, profiles/r04/regs_final_f32.txt) measured 0.152 vs 0.119 ms for the
        // unfused world-size > 1 step (profiles/r03/k) and is not built
        const int64_t fuse_mode = env_int("PSGD_FUSE_FINAL", 1);
        if (fuse_mode != 0 && fuse_mode != 1) {  // 2 was the removed rank-4 K-term form
            static bool warned = false;
            if (!warned)
                std::fprintf(stderr, "psgd: PSGD_FUSE_FINAL=%lld is not a mode (0 or 1); using 1\n",
                             static_cast<long long>(fuse_mode));
            warned = true;
        }
        const bool use_mfma = env_int("PSGD_ODD_MFMA", 1) != 0;
        const bool use_rows = env_int("PSGD_ODD_ROWS", 1) != 0;
        int64_t podd = 0;
        for (size_t i = 0; i < mats.size(); ++i) {
            MatDesc& d = mats[i];
            const Geom g = geometry(d.n, d.m, d.r, vec[i], tile_elems);
            d.vec = vec[i];
            d.lanes = g.lanes;
            d.nstrip = g.nstrip;
            d.nchunk = g.nchunk;
            d.chunk_rows = g.chunk_rows;
            const OddGeom og = odd_geometry(d.n, d.m, tile_elems);
            // the MFMA kernel addresses a tile through a buffer descriptor (< 2^31 bytes)
            const int64_t span = ((int64_t(og.chunk_rows) - 1) * d.m + og.sw) * (dtype == PSGD_BF16 ? 2 : 4);
            // r <= 4: every odd tile stays in ONE k_product_odd launch (row layout with a
            // reduce-scatter on full-width strips, lane sums on narrow ones); the MFMA kernel
            // pays for itself only for wider factors (16 output columns per instruction)
            const bool valu = use_rows && d.r <= 4;
            d.odd_mfma = (use_mfma && !valu && d.r <= 32 && span < (int64_t(1) << 31)) ? 1 : 0;
            for (int c = 0; c < g.nchunk; ++c)
                for (int s = 0; s < g.nstrip; ++s) {
                    tiles.push_back(Tile{int32_t(i), s, c, d.tensor});
                    if (!d.odd_mfma) tiles_ov.push_back(Tile{int32_t(i), s, c, d.tensor});
                }
            if (d.odd_mfma) {
                d.odd_sw = og.sw;
                d.odd_chunk_rows = og.chunk_rows;
                d.odd_nstrip = og.nstrip;
                for (int c = 0; c < og.nchunk; ++c)
                    for (int s = 0; s < og.nstrip; ++s) tiles_om.push_back(Tile{int32_t(i), s, c, d.tensor});
            } else {
                d.odd_sw = d.odd_chunk_rows = 0;
                d.odd_nstrip = g.nstrip;
            }
            // odd partials [odd strips][n][r], 16-byte aligned slabs (k_reduce's vector loads)
            d.part_odd = podd = (podd + 3) & ~int64_t(3);
            podd += int64_t(d.odd_nstrip) * d.n * d.r;
            d.part_even = 0;
        }
        part_odd_floats = podd;
        fin_ok = false;
        fin_proj = false;
        orth_chol = env_int("PSGD_ORTH_CHOL", 1) != 0;
        // buffer descriptors address one matrix: keep each below 2^31 bytes
        bool small = true;
        for (const MatDesc& d : mats) small = small && d.n * d.m * (dtype == PSGD_BF16 ? 2 : 4) < (int64_t(1) << 31);
        int smax = 0;
        for (const MatDesc& d : mats) smax = std::max(smax, fin_geometry(d.n, d.m, rbucket, 0).S);
        // >= 2 waves per SIMD resident (the register arrays scale with S * 4 * r)
        auto fits = [&](int nres) {
            int waves = 0;
            FinalArgs none{};
            return fin_bucket(smax) > 0 &&
                   launch_final_odd(dtype, rbucket, nres, fin_bucket(smax), none, 0, nullptr, &waves) == hipSuccess &&
                   waves >= 2;
        };
        if (fuse_mode != 0 && small && rbucket <= 2) fin_ok = fits(iters - 1);
        // the K-term form exists for ranks 1-2 only (dispatch_final_k<4> refuses any K-term nres)
        assert(!fin_ok || rbucket <= 2);
        // Projection form (psgd_final.cuh): two power iterations at world size 1, ranks 2 and 4,
        // the last iteration's in-factor orthonormalised by Cholesky-QR (which leaves R').
        // Same register-panel geometry as the K-term form, so both can share the tile list.
        // Rank 1 (the joint group norm folded into the kernels, psgd_aggregate): the same form with
        // the per-matrix correction of psgd_final.cuh; it needs the folded norm's sums of squares.
        const bool proj_r1 = rbucket == 1 && env_int("PSGD_FUSE_NORM", 1) != 0 && env_int("PSGD_FIN_PROJ1", 1) != 0;
        if (fuse_mode != 0 && small && iters == 2 && (((rbucket == 2 || rbucket == 4) && orth_chol) || proj_r1) &&
            env_int("PSGD_FIN_PROJ", 1) != 0)
            fin_proj = fits(kFinProj);
        fin_smax = 0;
        if (fin_ok || fin_proj) {
            // segments per row up to the kernel bucket the widest groups already need
            // (at most 5: the exact-S bodies), for fewer idle lanes
            const int scap = std::min(fin_bucket(smax), 5);
            // row blocks: the projection form's fin_elems; the K-term form's fin_elems_kt (its own
            // list only when both forms exist and the sizes differ; fin_rows_kt = fin_rows else)
            const int64_t fe = fin_proj ? fin_elems : fin_elems_kt;
            const bool two = fin_proj && fin_ok && fin_elems_kt != fin_elems;
            for (size_t i = 0; i < mats.size(); ++i) {
                MatDesc& d = mats[i];
                const FinGeom fg = fin_geometry(d.n, d.m, rbucket, fe, scap);
                d.fin_T = fg.T;
                d.fin_S = fg.S;
                d.fin_rows = fg.rows;
                d.fin_rows_kt = fg.rows;
                fin_smax = std::max(fin_smax, fg.S);
                for (int64_t b = 0; b < fg.ntiles; ++b) tiles_fin.push_back(Tile{int32_t(i), 0, int32_t(b), d.tensor});
                if (two) {
                    const FinGeom fk = fin_geometry(d.n, d.m, rbucket, fin_elems_kt, scap);
                    d.fin_rows_kt = fk.rows;
                    for (int64_t b = 0; b < fk.ntiles; ++b)
                        tiles_fin_kt.push_back(Tile{int32_t(i), 0, int32_t(b), d.tensor});
                }
            }
        }
        build_oe();
        build_reduction();
        if (!bucket_gend.empty()) build_spans();
    }
    void build_oe() {
        oe_ok = false;
        red_oe.clear();
        tiles_oe.clear();
        grng_oe.assign(2 * groups.size(), 0);
        grng_oe_items.assign(2 * groups.size(), 0);
        oe_part_floats = 0;
        oe_blocks = 0;
        if (!fin_ok || rbucket != 1 || iters < 3 || f64() || env_int("PSGD_OE", 1) == 0) return;
        int waves = 0;
        FinalArgs none{};
        if (launch_final_oe(dtype, iters - 2, fin_bucket(fin_smax), none, 0, nullptr, &waves) != hipSuccess || waves < 2)
            return;
        for (size_t i = 0; i < mats.size(); ++i) {
            MatDesc& d = mats[i];
            const int g = d.group;
            const bool first = i == 0 || mats[i - 1].group != g;
            if (first) {
                grng_oe[2 * g] = oe_blocks;
                grng_oe_items[2 * g] = int32_t(red_oe.size());
            }
            // one K-term row block per odd-even block (2 / 4 / 8 blocks merged: fewer partials
            // for the reduction but a slower pass, cfg5 0.0322 / 0.0333 / 0.041 against 0.0307 ms,
            // profiles/r05)
            d.oe_rows = int32_t(std::min<int64_t>(d.n, int64_t(d.fin_rows_kt)));
            const int32_t nb = int32_t((d.n + d.oe_rows - 1) / d.oe_rows);
            for (int32_t b = 0; b < nb; ++b) tiles_oe.push_back(Tile{int32_t(i), 0, b, d.tensor});
            d.oe_blk0 = oe_blocks;
            d.oe_part = oe_part_floats;
            oe_blocks += nb;
            oe_part_floats += int64_t(nb) * d.m;  // rank 1: [m] per block
            const int pe = nb > kRedWide ? 1 : 4;
            for (int64_t e = 0; e < d.m; e += 64 * pe)
                red_oe.push_back(RedItem{int32_t(i), int32_t(e), pe, int32_t(std::min<int64_t>(64 * pe, d.m - e)),
                                         d.oe_part + e, int32_t(d.m), nb});
            grng_oe[2 * g + 1] = oe_blocks;
            grng_oe_items[2 * g + 1] = int32_t(red_oe.size());
        }
        oe_ok = true;
    }
    // the last iteration of `step` runs fused (odd, and every matrix fits); `agg`: the caller
    // is psgd_aggregate (world size 1, output written), where the projection form also applies
    bool fused_final(int64_t step, bool agg) const { return (fin_ok || (agg && fin_proj)) && !even(step, iters - 1); }
    // the fused last iteration takes the projection form
    bool proj_final(int64_t step, bool agg) const { return agg && fin_proj && !even(step, iters - 1); }
    bool fused_final_at(int64_t step, int it, bool agg) const { return it == iters - 1 && fused_final(step, agg); }

    int upload_tiles() const;
};

struct psgd_flat {
    int dtype = 0;
    std::vector<FlatEntry> entries;  // non-empty tensors only
    std::vector<FlatItem> items;
    int32_t count = 0;
    int64_t total = 0;
    size_t o_ptrs = 0, o_ents = 0, o_items = 0, ws_bytes = 0;
    bool bound = false;
    int device = -1;
    char* ws = nullptr;
    TableCache tab;  // device pointer tables of the tensors
};

// DDP bucket <-> parameter tensors (psgd_runs_*, include/psgd.h): the work items of one run
// table and the device pointer tables of the tensors it addresses
struct psgd_runs {
    int dtype = 0;
    int32_t ntensors = 0;
    std::vector<RunItem> items;
    int64_t bucket_numel = 0;  // one past the last bucket element any run touches
    size_t o_ptrs = 0, o_items = 0, ws_bytes = 0;
    bool bound = false;
    int device = -1;
    char* ws = nullptr;
    TableCache tab;
};

namespace {

int upload(void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return PSGD_OK;
    PSGD_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return PSGD_OK;
}

// Select (or upload, stream-ordered) the gradient pointer table; switch matrices whose
// gradient is not vector-aligned to the scalar path (rare: views into unaligned flat buffers;
// only that re-tiling synchronises, because the tile tables are rewritten in place).
int refresh_pointers(psgd_plan* p, void* const* grads, hipStream_t stream) {
    const size_t nt = p->shapes.size();
    for (size_t i = 0; i < nt; ++i)
        if (!grads[i]) return fail(PSGD_ERR_VALUE, "null gradient pointer");
    const uintptr_t need = p->dtype == PSGD_F32 ? 16 : 8;
    bool same_vec = true;
    for (size_t i = 0; same_vec && i < p->mats.size(); ++i)
        same_vec = p->vec_now[i] == int(p->base_vec[i] && (reinterpret_cast<uintptr_t>(grads[p->mats[i].tensor]) % need == 0));
    if (!same_vec) {
        std::vector<int> vec(p->mats.size());
        for (size_t i = 0; i < p->mats.size(); ++i)
            vec[i] = p->base_vec[i] && (reinterpret_cast<uintptr_t>(grads[p->mats[i].tensor]) % need == 0);
        PSGD_HIP(hipStreamSynchronize(stream));  // earlier launches may still read the tile tables
        p->set_vec(vec);
        if (int st = p->upload_tiles()) return st;
    }
    PSGD_HIP(p->grad_tab.select(grads, stream));
    return PSGD_OK;
}

}  // namespace

int psgd_plan::upload_tiles() const {
    // the lists follow the geometry and the buckets: never past the capacities carved at create
    if (int64_t(segs.size()) > segs_cap || int64_t(wg_seg.size()) > int64_t(kMaxBuckets) * kEvenWgMax + 1 ||
        int64_t(red_even.size()) > red_even_cap || int64_t(red_odd.size()) > red_odd_cap ||
        int64_t(tiles_fin.size()) > tiles_fin_cap || int64_t(tiles_fin_kt.size()) > tiles_fin_kt_cap)
        return fail(PSGD_ERR_STATE, "internal: work lists exceed their workspace capacity");
    if (int st = upload(dev<void>(o_mats), mats.data(), mats.size() * sizeof(MatDesc))) return st;
    if (int st = upload(dev<void>(o_tiles), tiles.data(), tiles.size() * sizeof(Tile))) return st;
    if (int st = upload(dev<void>(o_tiles_ov), tiles_ov.data(), tiles_ov.size() * sizeof(Tile))) return st;
    if (int st = upload(dev<void>(o_tiles_fin), tiles_fin.data(), tiles_fin.size() * sizeof(Tile))) return st;
    if (int st = upload(dev<void>(o_tiles_fin_kt), tiles_fin_kt.data(), tiles_fin_kt.size() * sizeof(Tile))) return st;
    if (int st = upload(dev<void>(o_tiles_om), tiles_om.data(), tiles_om.size() * sizeof(Tile))) return st;
    if (int st = upload(dev<void>(o_segs), segs.data(), segs.size() * sizeof(Seg))) return st;
    if (int st = upload(dev<void>(o_wg_seg), wg_seg.data(), wg_seg.size() * sizeof(int32_t))) return st;
    if (int st = upload(dev<void>(o_red_even), red_even.data(), red_even.size() * sizeof(RedItem))) return st;
    if (int st = upload(dev<void>(o_red_odd), red_odd.data(), red_odd.size() * sizeof(RedItem))) return st;
    if (int st = upload(dev<void>(o_grng_even), grng_even.data(), grng_even.size() * sizeof(int32_t))) return st;
    if (int st = upload(dev<void>(o_grng_odd), grng_odd.data(), grng_odd.size() * sizeof(int32_t))) return st;
    if (int st = upload(dev<void>(o_grng_ss0), grng_ss0.data(), grng_ss0.size() * sizeof(int32_t))) return st;
    if (qfold_ok)
        if (int st = upload(dev<void>(o_uitems), uitems.data(), uitems.size() * sizeof(int32_t))) return st;
    if (int st = upload(dev<void>(o_mrng), mrng_even.data(), mrng_even.size() * sizeof(int32_t))) return st;
    if (oe_ok && o_red_oe) {
        if (int st = upload(dev<void>(o_tiles_oe), tiles_oe.data(), tiles_oe.size() * sizeof(Tile))) return st;
        if (int st = upload(dev<void>(o_red_oe), red_oe.data(), red_oe.size() * sizeof(RedItem))) return st;
        if (int st = upload(dev<void>(o_grng_oe), grng_oe.data(), grng_oe.size() * sizeof(int32_t))) return st;
        if (int st = upload(dev<void>(o_grng_oe_items), grng_oe_items.data(), grng_oe_items.size() * sizeof(int32_t)))
            return st;
    }
    return PSGD_OK;
}

namespace {

void fill_terms(const psgd_plan* p, int64_t step, int count, Terms& res) {
    for (int j = 0; j < count; ++j) {
        const bool e = p->even(step, j);
        // local rank-r term of iteration j: even -> (P_j = X_j, Q_j = Y_j); odd -> (P_j = Y_j, Q_j = X_j)
        res.p[j] = e ? p->hist(0, j) : p->hist(1, j);
        res.q[j] = e ? p->hist(1, j) : p->hist(0, j);
    }
    for (int j = count; j < kMaxTerms; ++j) res.p[j] = res.q[j] = nullptr;
}

}  // namespace

extern "C" {

int psgd_version(void) { return 100; }

const char* psgd_last_error(void) { return g_err.c_str(); }

int psgd_should_compress(const int64_t* shape, int32_t ndim, int32_t rank, int32_t iters,
                         double min_rate, int32_t* out) {
    if (!shape || !out || ndim < 1) return fail(PSGD_ERR_VALUE, "shape must have at least one dim");
    int64_t numel = 1, sum = 0, mn = shape[0];
    for (int i = 0; i < ndim; ++i) {
        numel *= shape[i];
        sum += shape[i];
        mn = std::min(mn, shape[i]);
    }
    const double r = double(std::min<int64_t>(rank, mn));
    const double avg = 0.5 * double(iters) * r * double(sum);  // reference :292-294
    if (avg == 0.0) return fail(PSGD_ERR_VALUE, "zero average compressed size (division by zero)");
    *out = (double(numel) / avg > min_rate) ? 1 : 0;  // reference :101-105
    return PSGD_OK;
}

int psgd_plan_create(const int64_t* dims, const int32_t* ndims, int32_t num_tensors, int32_t rank,
                     int32_t iters, int32_t dtype, psgd_plan** out_plan) {
    if (!out_plan) return fail(PSGD_ERR_VALUE, "out_plan is null");
    *out_plan = nullptr;
    if (num_tensors < 1 || !dims || !ndims) return fail(PSGD_ERR_INDEX, "list index out of range (no tensors)");
    if (rank < 1) return fail(PSGD_ERR_VALUE, "rank must be >= 1");
    if (iters < 1 || iters > PSGD_MAX_ITERS) return fail(PSGD_ERR_VALUE, "num_iters_per_step must be in [1, 16]");
    if (dtype != PSGD_F32 && dtype != PSGD_BF16 && dtype != PSGD_F64)
        return fail(PSGD_ERR_DTYPE, "dtype must be fp32, bf16 or fp64");

    auto* p = new psgd_plan();
    p->rank = rank;
    p->iters = iters;
    p->dtype = dtype;
    p->tile_elems = 0;  // set below from the compressed size
    std::map<std::pair<int64_t, int64_t>, int> gid;
    const int64_t* d = dims;
    for (int t = 0; t < num_tensors; ++t) {
        const int nd = ndims[t];
        if (nd < 1) {
            delete p;
            return fail(PSGD_ERR_INDEX, "tuple index out of range (0-dim tensor)");
        }
        std::vector<int64_t> s(d, d + nd);
        d += nd;
        int64_t numel = 1;
        for (int64_t x : s) numel *= x;
        if (numel <= 0) {
            delete p;
            return fail(PSGD_ERR_LAYOUT, "cannot view an empty tensor as a matrix");
        }
        const int64_t n = s[0], m = numel / n;
        auto key = std::make_pair(n, m);
        auto it = gid.find(key);
        if (it == gid.end()) {
            it = gid.emplace(key, int(p->groups.size())).first;
            psgd_plan::Group g;
            g.n = n;
            g.m = m;
            g.r = int(std::min<int64_t>(rank, std::min(n, m)));
            g.poff = g.qoff = 0;
            p->groups.push_back(g);
        }
        p->groups[it->second].tensors.push_back(t);
        p->shapes.push_back(std::move(s));
        // compression_rate bookkeeping (reference :265-275, on the ORIGINAL shape)
        int64_t sum = 0, mn = p->shapes.back()[0];
        for (int64_t x : p->shapes.back()) {
            sum += x;
            mn = std::min(mn, x);
        }
        p->unc_floats += double(numel);
        p->comp_floats += 0.5 * iters * double(std::min<int64_t>(rank, mn)) * double(sum);
    }
    int maxr = 1;
    for (auto& g : p->groups) maxr = std::max(maxr, g.r);
    {
        // about 3k tiles (12 per CU) on large problems, never below 4k elements per tile: the
        // cold even product on ResNet-50 is fastest at 8k-element tiles (profiles/r02/tile_sweep.txt)
        int64_t total = 0;
        for (auto& g : p->groups) total += int64_t(g.tensors.size()) * g.n * g.m;
        // small plans (<= 4M elements): about one tile per CU (cfg5 4096 x 512: 8192-element
        // tiles 0.038 -> 0.033 ms/step with the final blocks below; profiles/r02b/small)
        const int64_t dflt = total <= (int64_t(1) << 22)
                                 ? std::min<int64_t>(16384, std::max<int64_t>(4096, total / 256))
                                 : std::min<int64_t>(16384, std::max<int64_t>(4096, total / 3072));
        p->tile_elems = std::max<int64_t>(1024, env_int("PSGD_TILE_ELEMS", dflt));
    }
    if (maxr > 32) {
        delete p;
        return fail(PSGD_ERR_VALUE, "effective rank above 32 is not supported by this build");
    }
    p->rbucket = int(pow2ceil(maxr));
    {
        // Fused final pass: ~1500 row blocks on ResNet-50 (about three rounds of the
        // resident workgroups); the sweeps in profiles/r01 put the optimum at 16-24k
        // elements per block.
        int64_t total = 0;
        for (auto& g : p->groups) total += int64_t(g.tensors.size()) * g.n * g.m;
        // Rank 1 (256-thread row groups): twice as many, smaller blocks (ResNet-50: ~8k elements,
        // ~3000 blocks): cfg2 0.0818 -> 0.0771 ms, final pass 55.7 -> 51.4 us; rank 4 (512-thread
        // groups) slower there, 0.097 -> 0.103 ms (profiles/r04/g)
        const int64_t per = maxr <= 1 ? 3072 : 1536;
        const int64_t gbytes = total * (p->dtype == PSGD_BF16 ? 2 : p->dtype == PSGD_F64 ? 8 : 4);
        p->out_nt = gbytes > env_int("PSGD_OUT_NT_MB", 32) * (int64_t(1) << 20) ? 1 : 0;
        const int64_t dflt = total <= (int64_t(1) << 22)
                                 ? std::min<int64_t>(16384, std::max<int64_t>(4096, total / 256))
                                 : std::min<int64_t>(65536, std::max<int64_t>(4096, total / per));
        p->fin_elems = std::max<int64_t>(1024, env_int("PSGD_FIN_ELEMS", dflt));
        // the K-term form (world size > 1, and world size 1 beyond two iterations) keeps ~16k at
        // every rank: cfg2 over the multi-GPU code path 0.0932-0.0959 -> 0.0916-0.0918 ms
        // (profiles/r04/o)
        const int64_t dflt_kt = total <= (int64_t(1) << 22) ? dflt
                                                            : std::min<int64_t>(65536, std::max<int64_t>(4096, total / 1536));
        p->fin_elems_kt = std::max<int64_t>(1024, env_int("PSGD_FIN_ELEMS_KT", env_int("PSGD_FIN_ELEMS", dflt_kt)));
        // persistent even product: workgroups per CU, minimum gradient elements per workgroup
        // default: the first-iteration instance's resident workgroups per CU (capped at 4), so the
        // grid is one wave of resident workgroups (rank 4: 3 since the narrow-strip path fits 6
        // waves per SIMD; bf16 ranks 2 / 4: 2)
        int resident = p->dtype == PSGD_F32 ? even_resident_f32(p->rbucket) : even_resident_bf16(p->rbucket);
        resident = resident > 0 ? std::min(resident, 4) : 4;
        p->even_wpc = int(std::min<int64_t>(kEvenWpcMax, std::max<int64_t>(1, env_int("PSGD_EVEN_WPC", resident))));
        p->even_min = std::max<int64_t>(1024, env_int("PSGD_EVEN_MIN", 16384));
        // segment cost: rank 4 writes 4 floats per column per segment, so fewer, longer
        // segments pay there (cfg3 k_even 23.3-23.8 -> 22.7 us at 8192); neutral at rank 1
        // (profiles/r04/j)
        p->even_segc = std::max<int64_t>(0, env_int("PSGD_EVEN_SEGC", maxr >= 4 ? 8192 : 4096));
    }

    // output layout: dense, tensor order (what torch.cat / unflatten produce); a matrix
    // whose segment is not 16-byte aligned takes the scalar path
    p->out_off.assign(num_tensors, 0);
    for (int t = 0; t < num_tensors; ++t) {
        int64_t numel = 1;
        for (int64_t x : p->shapes[t]) numel *= x;
        p->out_off[t] = p->out_total;
        p->out_total += numel;
    }
    int64_t poff = 0, qoff = 0;
    for (size_t gi = 0; gi < p->groups.size(); ++gi) {
        auto& g = p->groups[gi];
        g.poff = poff;
        g.qoff = qoff;
        for (size_t b = 0; b < g.tensors.size(); ++b) {
            MatDesc md{};
            md.n = g.n;
            md.m = g.m;
            md.r = g.r;
            md.poff = poff + int64_t(b) * g.n * g.r;
            md.qoff = qoff + int64_t(b) * g.m * g.r;
            md.out_off = p->out_off[g.tensors[b]];
            md.tensor = g.tensors[b];
            md.group = int(gi);
            p->mats.push_back(md);
            p->base_vec.push_back((dtype != PSGD_F64 && g.m % 4 == 0 && g.r <= 8 && md.out_off % 4 == 0) ? 1 : 0);
        }
        poff += int64_t(g.tensors.size()) * g.n * g.r;
        qoff += int64_t(g.tensors.size()) * g.m * g.r;
        // orthonormalisation units (reference orthogonalize() is called per group batch, :188)
        if (g.r == 1) {
            p->units_p.push_back(OrthUnit{g.poff, g.n, 1, int32_t(g.tensors.size())});
            p->units_q.push_back(OrthUnit{g.qoff, g.m, 1, int32_t(g.tensors.size())});
            p->unit_group_p.push_back(int32_t(gi));
            p->unit_group_q.push_back(int32_t(gi));
        } else {
            for (size_t b = 0; b < g.tensors.size(); ++b) {
                p->units_p.push_back(OrthUnit{g.poff + int64_t(b) * g.n * g.r, g.n, g.r, 1});
                p->units_q.push_back(OrthUnit{g.qoff + int64_t(b) * g.m * g.r, g.m, g.r, 1});
                p->unit_group_p.push_back(int32_t(gi));
                p->unit_group_q.push_back(int32_t(gi));
            }
            p->panel_p = std::max(p->panel_p, g.n);  // longest rank>1 panel (rows)
            p->panel_q = std::max(p->panel_q, g.m);
        }
    }
    p->ptot = poff;
    p->qtot = qoff;
    p->fmax = std::max(poff, qoff);

    // capacities of every list set_vec may build (either vector width, up to kMaxBuckets
    // buckets): tiles, segments, reduction items, partial slabs
    int64_t total = 0, strips_max = 0, strip_elems = 0, red_even_cap = 0, red_odd_cap = 0, part_odd_cap = 0, wr_max = 0;
    for (size_t i = 0; i < p->mats.size(); ++i) {
        const MatDesc& md = p->mats[i];
        total += md.n * md.m;
        const OddGeom og = odd_geometry(md.n, md.m, p->tile_elems);
        int64_t ns = 0, se = 0, re = 0, po = og.nstrip;
        for (int v : {p->base_vec[i], 0}) {
            const Geom g = geometry(md.n, md.m, md.r, v, p->tile_elems);
            const int64_t W = int64_t(g.lanes) * (v ? 4 : 1);
            ns = std::max<int64_t>(ns, g.nstrip);
            se = std::max<int64_t>(se, g.nstrip * (W * md.r + 3));
            re = std::max<int64_t>(re, (md.m * md.r + 63) / 64 + g.nstrip);
            po = std::max<int64_t>(po, g.nstrip);
            wr_max = std::max<int64_t>(wr_max, W * md.r + 3);
        }
        p->tiles_cap += std::max(geometry(md.n, md.m, md.r, p->base_vec[i], p->tile_elems).ntiles,
                                 geometry(md.n, md.m, md.r, 0, p->tile_elems).ntiles);
        p->tiles_om_cap += int64_t(og.nstrip) * og.nchunk;
        int64_t cap = 0, cap_kt = 0;
        for (int sc = 0; sc <= 5; ++sc) {  // any segment cap set_vec may pick
            cap_kt = std::max(cap_kt, fin_geometry(md.n, md.m, p->rbucket, p->fin_elems_kt, sc).ntiles);
            cap = std::max(cap, fin_geometry(md.n, md.m, p->rbucket, p->fin_elems, sc).ntiles);
        }
        p->tiles_fin_cap += std::max(cap, cap_kt);
        p->tiles_fin_kt_cap += cap_kt;
        strips_max += ns;
        strip_elems += se;
        red_even_cap += re;
        red_odd_cap += (md.n * md.r + 63) / 64;
        part_odd_cap += po * md.n * md.r + 3;
    }
    {
        const int64_t nb = std::min<int64_t>(kMaxBuckets, int64_t(p->groups.size()));
        const int64_t wg = std::min<int64_t>(int64_t(p->even_wpc) * kCUs, total / p->even_min + 1);
        // segments beyond one per strip: one per workgroup boundary (strip walk), up to two per
        // workgroup (row blocks across strips, ragged strips)
        const int64_t extra = 2 * nb * wg;
        p->segs_cap = strips_max + extra;
        p->ss0_cap = int64_t(p->mats.size()) + extra;
        p->even_part_cap = strip_elems + extra * wr_max;
        p->red_even_cap = red_even_cap;
        p->red_odd_cap = red_odd_cap;
    }
    // folded orthonormalisation (projection form): every Q unit one panel of rbucket columns
    p->qfold_ok = !p->f64() && (p->rbucket == 2 || p->rbucket == 4) && !p->units_q.empty() &&
                  env_int("PSGD_QFOLD", 1) != 0;
    for (const OrthUnit& u : p->units_q) p->qfold_ok = p->qfold_ok && u.r == p->rbucket && u.count == 1;
    const int64_t part_cap = part_odd_cap + 4 + p->even_part_cap;
    if (p->f64()) {
        p->set_f64_tiles();  // fp64: its own kernels and tiles (psgd_f64.hip), no fused forms
        p->red_even_cap = std::max<int64_t>(p->red_even_cap, int64_t(p->red_even.size()));
    } else {
        p->set_vec(p->base_vec);
    }

    size_t off = 0;
    auto carve = [&](size_t bytes) {
        const size_t o = off;
        off = align256(off + bytes);
        return o;
    };
    p->o_ptrs = carve(TableCache::bytes(size_t(num_tensors)));
    p->o_mats = carve(p->mats.size() * sizeof(MatDesc));
    p->o_tiles = carve(size_t(p->tiles_cap) * sizeof(Tile));
    p->o_tiles_ov = carve(size_t(p->tiles_cap) * sizeof(Tile));
    p->o_tiles_om = carve(size_t(std::max<int64_t>(p->tiles_om_cap, 1)) * sizeof(Tile));
    p->o_tiles_fin = carve(size_t(std::max<int64_t>(p->tiles_fin_cap, 1)) * sizeof(Tile));
    p->o_tiles_fin_kt = carve(size_t(std::max<int64_t>(p->tiles_fin_kt_cap, 1)) * sizeof(Tile));
    p->o_segs = carve(size_t(std::max<int64_t>(p->segs_cap, 1)) * sizeof(Seg));
    p->o_wg_seg = carve((size_t(kMaxBuckets) * kEvenWgMax + 1) * sizeof(int32_t));
    p->o_red_even = carve(size_t(std::max<int64_t>(p->red_even_cap, 1)) * sizeof(RedItem));
    p->o_red_odd = carve(size_t(std::max<int64_t>(p->red_odd_cap, 1)) * sizeof(RedItem));
    p->o_units_p = carve(p->units_p.size() * sizeof(OrthUnit));
    p->o_units_q = carve(p->units_q.size() * sizeof(OrthUnit));
    for (const MatDesc& md : p->mats) {
        p->munits_p.push_back(OrthUnit{md.poff, md.n, md.r, 1});
        p->munits_q.push_back(OrthUnit{md.qoff, md.m, md.r, 1});
    }
    p->o_munits_p = carve(p->munits_p.size() * sizeof(OrthUnit));
    p->o_munits_q = carve(p->munits_q.size() * sizeof(OrthUnit));
    p->o_ipc_ptrs = carve(size_t(kMaxRanks) * sizeof(void*));
    p->o_ipc_nonce = carve(size_t(kMaxRanks) * sizeof(uint32_t));
    p->o_rq = carve(size_t(std::max<int64_t>(p->fmax, 1)) * sizeof(float));
    p->o_rdst = carve(TableCache::bytes(size_t(num_tensors)));
    p->o_odst = carve(TableCache::bytes(size_t(num_tensors)));
    p->o_grng_even = carve(std::max<size_t>(2 * p->groups.size(), 1) * sizeof(int32_t));
    p->o_grng_odd = carve(std::max<size_t>(2 * p->groups.size(), 1) * sizeof(int32_t));
    p->o_mrng = carve(std::max<size_t>(2 * p->mats.size(), 1) * sizeof(int32_t));
    p->ss_stride = size_t(std::max<int64_t>({p->red_even_cap, p->red_odd_cap, int64_t(p->red_oe.size())}));
    if (p->oe_ok) {  // the odd-even pass's layout (geometry-independent: fixed at create)
        p->o_oe_part = carve(size_t(p->oe_part_floats) * sizeof(float));
        p->o_tiles_oe = carve(std::max<size_t>(p->tiles_oe.size(), 1) * sizeof(Tile));
        p->o_oe_ss = carve(size_t(std::max(p->oe_blocks, 1)) * sizeof(float));
        p->o_red_oe = carve(std::max<size_t>(p->red_oe.size(), 1) * sizeof(RedItem));
        p->o_grng_oe = carve(std::max<size_t>(2 * p->groups.size(), 1) * sizeof(int32_t));
        p->o_grng_oe_items = carve(std::max<size_t>(2 * p->groups.size(), 1) * sizeof(int32_t));
    }
    p->o_ss = carve(2 * std::max<size_t>(p->ss_stride, 1) * sizeof(float));
    p->o_ss0 = carve(size_t(std::max<int64_t>(p->ss0_cap, 1)) * sizeof(float));
    p->o_grng_ss0 = carve(std::max<size_t>(2 * p->groups.size(), 1) * sizeof(int32_t));
    p->o_hist = carve(size_t(3) * iters * size_t(p->fmax) * (p->f64() ? sizeof(double) : sizeof(float)));
    p->o_f64_even = carve(std::max<size_t>(p->f64_even.size(), 1) * sizeof(Tile));
    p->o_f64_odd = carve(std::max<size_t>(p->f64_odd.size(), 1) * sizeof(Tile));
    p->o_f64_apply = carve(std::max<size_t>(p->f64_apply.size(), 1) * sizeof(Tile));
    p->o_f64_partoff = carve(std::max<size_t>(p->f64_part_off.size(), 1) * sizeof(int64_t));
    p->o_f64_part = carve(size_t(std::max<int64_t>(p->f64_part, 1)) * sizeof(double));
    p->o_part = carve(size_t(part_cap) * sizeof(float));
    if (p->qfold_ok) {
        p->o_gram = carve(size_t(p->red_even_cap) * kGramStride * sizeof(double));
        p->o_uitems = carve(2 * p->units_q.size() * sizeof(int32_t));
    }
    p->ws_bytes = off;
    *out_plan = p;
    return PSGD_OK;
}

int psgd_plan_destroy(psgd_plan* plan) {
    delete plan;
    return PSGD_OK;
}

int psgd_plan_num_groups(const psgd_plan* p, int32_t* out) {
    if (!p || !out) return fail(PSGD_ERR_VALUE, "null argument");
    *out = int32_t(p->groups.size());
    return PSGD_OK;
}

int psgd_plan_group(const psgd_plan* p, int32_t g, int64_t* n, int64_t* m, int32_t* r, int32_t* count) {
    if (!p || g < 0 || g >= int32_t(p->groups.size())) return fail(PSGD_ERR_VALUE, "group index out of range");
    const auto& gr = p->groups[g];
    if (n) *n = gr.n;
    if (m) *m = gr.m;
    if (r) *r = gr.r;
    if (count) *count = int32_t(gr.tensors.size());
    return PSGD_OK;
}

int psgd_plan_factor_numel(const psgd_plan* p, int64_t* pn, int64_t* qn) {
    if (!p) return fail(PSGD_ERR_VALUE, "null plan");
    if (pn) *pn = p->ptot;
    if (qn) *qn = p->qtot;
    return PSGD_OK;
}

int psgd_plan_output_offset(const psgd_plan* p, int32_t i, int64_t* off) {
    if (!p || !off || i < 0 || i >= int32_t(p->out_off.size())) return fail(PSGD_ERR_VALUE, "tensor index out of range");
    *off = p->out_off[i];
    return PSGD_OK;
}

int psgd_plan_output_numel(const psgd_plan* p, int64_t* numel) {
    if (!p || !numel) return fail(PSGD_ERR_VALUE, "null argument");
    *numel = p->out_total;
    return PSGD_OK;
}

int psgd_plan_workspace_bytes(const psgd_plan* p, int64_t* bytes) {
    if (!p || !bytes) return fail(PSGD_ERR_VALUE, "null argument");
    *bytes = int64_t(p->ws_bytes);
    return PSGD_OK;
}

int psgd_plan_compression_rate(const psgd_plan* p, double* rate, double* unc, double* comp) {
    if (!p) return fail(PSGD_ERR_VALUE, "null plan");
    if (rate) *rate = p->unc_floats / p->comp_floats;
    if (unc) *unc = p->unc_floats;
    if (comp) *comp = p->comp_floats;
    return PSGD_OK;
}

int psgd_plan_bind(psgd_plan* p, int32_t device, void* P, void* Q, void* workspace) {
    if (!p || !P || !Q || !workspace) return fail(PSGD_ERR_VALUE, "null argument");
    if (reinterpret_cast<uintptr_t>(workspace) % 16) return fail(PSGD_ERR_LAYOUT, "workspace must be 16-byte aligned");
    DevScope scope(device);
    p->device = device;
    p->P = static_cast<float*>(P);  // fp64 plans: double buffers (see P64/Q64)
    p->Q = static_cast<float*>(Q);
    p->ws = static_cast<char*>(workspace);
    const size_t nt = p->shapes.size();
    p->grad_tab.bind(p->dev<char>(p->o_ptrs), nt);
    p->rdst_tab.bind(p->dev<char>(p->o_rdst), nt);
    p->odst_tab.bind(p->dev<char>(p->o_odst), nt);
    if (int st = p->upload_tiles()) return st;
    if (int st = upload(p->dev<void>(p->o_units_p), p->units_p.data(), p->units_p.size() * sizeof(OrthUnit))) return st;
    if (int st = upload(p->dev<void>(p->o_munits_p), p->munits_p.data(), p->munits_p.size() * sizeof(OrthUnit))) return st;
    if (int st = upload(p->dev<void>(p->o_munits_q), p->munits_q.data(), p->munits_q.size() * sizeof(OrthUnit))) return st;
    if (int st = upload(p->dev<void>(p->o_units_q), p->units_q.data(), p->units_q.size() * sizeof(OrthUnit))) return st;
    PSGD_HIP(hipMemset(p->dev<void>(p->o_ss0), 0, size_t(std::max<int64_t>(p->ss0_cap, 1)) * sizeof(float)));
    if (p->f64()) {
        if (int st = upload(p->dev<void>(p->o_f64_even), p->f64_even.data(), p->f64_even.size() * sizeof(Tile))) return st;
        if (int st = upload(p->dev<void>(p->o_f64_odd), p->f64_odd.data(), p->f64_odd.size() * sizeof(Tile))) return st;
        if (int st = upload(p->dev<void>(p->o_f64_apply), p->f64_apply.data(), p->f64_apply.size() * sizeof(Tile))) return st;
        if (int st = upload(p->dev<void>(p->o_f64_partoff), p->f64_part_off.data(), p->f64_part_off.size() * sizeof(int64_t)))
            return st;
    }
    p->bound = true;
    return PSGD_OK;
}

int psgd_out_factor(const psgd_plan* p, int64_t step, int32_t it, int32_t* which) {
    if (!p || !which) return fail(PSGD_ERR_VALUE, "null argument");
    if (step < 0 || it < 0 || it >= p->iters) return fail(PSGD_ERR_VALUE, "step/iteration out of range");
    *which = p->even(step, it) ? 0 : 1;
    return PSGD_OK;
}

// World size 1 inside psgd_aggregate, every group rank 1, iteration >= 1: the joint-norm
// orthonormalisation of the in-factor is folded into the neighbouring reductions (no
// orthonormalisation launch): the previous reduction leaves per-item sums of squares, the
// product runs on the raw in-factor, and this iteration's reduction divides by the norm and
// writes the normalised in-factor (reference powersgd.py:186-188 + orthogonalization.py:5-6).
static bool fused_norm(const psgd_plan* p, bool fuse, int it) {
    return fuse && p->rbucket == 1 && it >= 1;
}

static bool norm0_fold() {
    static const bool on = env_int("PSGD_FUSE_NORM0", 1) != 0;
    return on;
}

// Timing (benchmarks): HIP events of the final pass (k_apply, or the fused final odd kernel):
// recorded by the kernel's own dispatch (timed_launch) for the fp32/bf16 kernels, or around the
// launch on its stream (fp64 apply).
struct TimedScope {
    KernelTiming kt{};
    explicit TimedScope(const std::pair<hipEvent_t, hipEvent_t>* ev) {
        if (ev) {
            kt = KernelTiming{ev->first, ev->second};
            g_kernel_timing = &kt;
        }
    }
    ~TimedScope() { g_kernel_timing = nullptr; }
};
static int timing_begin(psgd_plan* p, hipStream_t s, std::pair<hipEvent_t, hipEvent_t>** ev, bool direct);
static int timing_begin(psgd_plan* p, hipStream_t s, std::pair<hipEvent_t, hipEvent_t>** ev) {
    return timing_begin(p, s, ev, false);
}
static int timing_begin(psgd_plan* p, hipStream_t s, std::pair<hipEvent_t, hipEvent_t>** ev, bool direct) {
    *ev = nullptr;
    if (!p->timing) return PSGD_OK;
    if (p->ev_used == p->ev_pool.size()) {
        std::pair<hipEvent_t, hipEvent_t> e;
        // no system-scope fence: a system-scope release writes back the L2s around the timed
        // kernel (~5.6 us of idle queue per event in the traces) that a plain step never pays
        PSGD_HIP(hipEventCreateWithFlags(&e.first, hipEventDisableSystemFence));
        PSGD_HIP(hipEventCreateWithFlags(&e.second, hipEventDisableSystemFence));
        p->ev_pool.push_back(e);
    }
    *ev = &p->ev_pool[p->ev_used++];
    if (!direct) PSGD_HIP(hipEventRecord((*ev)->first, s));
    return PSGD_OK;
}

// ---------------------------------------------------------------- fp64 plans ------
// The same iteration structure as the fp32 path below, on psgd_f64.hip's kernels: orthonormalise
// the in-factor (saving the all-reduced values of the previous iteration), product with
// G_k formed on the fly, and for even iterations the fixed-order partial reduction.
static void fill_terms64(const psgd_plan* p, int64_t step, int count, TermsF64& res) {
    for (int j = 0; j < count; ++j) {
        const bool e = p->even(step, j);
        res.p[j] = e ? p->hist64(0, j) : p->hist64(1, j);
        res.q[j] = e ? p->hist64(1, j) : p->hist64(0, j);
    }
    for (int j = count; j < kMaxTerms; ++j) res.p[j] = res.q[j] = nullptr;
}

static int compress_f64(psgd_plan* p, void* const* grads, int64_t step, int32_t it, hipStream_t s) {
    if (int st = refresh_pointers(p, grads, s)) return st;
    const bool even = p->even(step, it);
    double* P = reinterpret_cast<double*>(p->P);
    double* Q = reinterpret_cast<double*>(p->Q);
    double* in = even ? P : Q;
    double* out = even ? Q : P;
    F64OrthArgs oa{};
    oa.units = p->dev<OrthUnit>(even ? p->o_units_p : p->o_units_q);
    oa.state = in;
    oa.hx = p->hist64(0, it);
    oa.save = it > 0 ? p->hist64(2, it - 1) : nullptr;  // keep the all-reduced factor of it-1
    PSGD_HIP(launch_f64_orth(p->rbucket, oa, int(even ? p->units_p.size() : p->units_q.size()), s));
    F64Args a{};
    a.mats = p->dev<MatDesc>(p->o_mats);
    a.grads = p->grad_tab.table();
    a.x = p->hist64(0, it);
    a.part = p->dev<double>(p->o_f64_part);
    a.part_off = p->dev<int64_t>(p->o_f64_partoff);
    a.y = out;
    a.yh = p->hist64(1, it);
    fill_terms64(p, step, it, a.res);
    a.nres = it;
    if (even) {
        a.tiles = p->dev<Tile>(p->o_f64_even);
        PSGD_HIP(launch_f64_product(true, p->rbucket, a, int(p->f64_even.size()), s));
        a.items = p->dev<RedItem>(p->o_red_even);
        PSGD_HIP(launch_f64_reduce(p->rbucket, a, int(p->red_even.size()), s));
    } else {
        a.tiles = p->dev<Tile>(p->o_f64_odd);
        PSGD_HIP(launch_f64_product(false, p->rbucket, a, int(p->f64_odd.size()), s));
    }
    return PSGD_OK;
}

static int decompress_f64(psgd_plan* p, void* const* grads, void* out, int64_t step, int32_t world, hipStream_t s) {
    if (int st = refresh_pointers(p, grads, s)) return st;
    const int I = p->iters;
    F64Args a{};
    a.mats = p->dev<MatDesc>(p->o_mats);
    a.tiles = p->dev<Tile>(p->o_f64_apply);
    a.grads = p->grad_tab.table();
    a.out = out;
    fill_terms64(p, step, I, a.res);
    double* last = reinterpret_cast<double*>(p->even(step, I - 1) ? p->Q : p->P);
    for (int k = 0; k < I; ++k) {
        const bool e = p->even(step, k);
        double* ybar = k + 1 < I ? p->hist64(2, k) : last;  // all-reduced factor of iteration k
        a.apx.p[k] = e ? p->hist64(0, k) : ybar;
        a.apx.q[k] = e ? ybar : p->hist64(0, k);
    }
    a.nres = I;
    a.alpha = 1.0 / double(world);  // reference alpha = 1 / num_workers (:218)
    std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
    if (int st = timing_begin(p, s, &ev)) return st;
    PSGD_HIP(launch_f64_apply(p->rbucket, a, int(p->f64_apply.size()), s));
    if (ev) PSGD_HIP(hipEventRecord(ev->second, s));
    return PSGD_OK;
}

// Diagnostic (PSGD_EVEN_STAMPS=<file>, with a library built -DPSGD_EVEN_STAMPS): after every
// k_even launch, synchronise and append its per-workgroup stamps to <file>: one line per launch,
// "nwg", then per workgroup its segments' gradient bytes and the kEvenStamps words
// (tools/even_stamps.py). Never set in a timed run.
static int even_stamps_begin(psgd_plan* p, ProductArgs& pa) {
    static const char* path = std::getenv("PSGD_EVEN_STAMPS");
    if (!path || !*path) return PSGD_OK;
    const size_t words = size_t(std::max(pa.nwg, 1)) * kEvenStamps;
    if (p->stamp_words < words) {
        if (p->stamp_buf) (void)hipFree(p->stamp_buf);
        p->stamp_buf = nullptr;
        PSGD_HIP(hipMalloc(reinterpret_cast<void**>(&p->stamp_buf), words * sizeof(unsigned long long)));
        p->stamp_words = words;
    }
    PSGD_HIP(hipMemset(p->stamp_buf, 0, words * sizeof(unsigned long long)));
    pa.stamps = p->stamp_buf;
    return PSGD_OK;
}

static int even_stamps_end(psgd_plan* p, const ProductArgs& pa, hipStream_t s) {
    if (!pa.stamps) return PSGD_OK;
    PSGD_HIP(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(size_t(pa.nwg) * kEvenStamps);
    PSGD_HIP(hipMemcpy(h.data(), pa.stamps, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    FILE* f = std::fopen(std::getenv("PSGD_EVEN_STAMPS"), "a");
    if (!f) return PSGD_OK;
    const int64_t esz = p->dtype == PSGD_BF16 ? 2 : 4;
    const int32_t w0 = int32_t((pa.wg_seg - p->dev<int32_t>(p->o_wg_seg)));
    std::fprintf(f, "%d", pa.nwg);
    for (int w = 0; w < pa.nwg; ++w) {
        int64_t bytes = 0;
        const int32_t b = p->wg_seg[size_t(w0 + w)], e = p->wg_seg[size_t(w0 + w + 1)];
        for (int32_t k = b; k < e; ++k) {
            const Seg& sg = p->segs[size_t(k)];
            const int64_t cols = std::min<int64_t>(int64_t(sg.lanes) * (sg.vec ? 4 : 1), sg.m - int64_t(sg.strip) * sg.lanes * (sg.vec ? 4 : 1));
            bytes += int64_t(sg.row1 - sg.row0) * cols * esz;
        }
        std::fprintf(f, " %d:%lld", e - b, static_cast<long long>(bytes));
        for (int k = 0; k < kEvenStamps; ++k) std::fprintf(f, ":%llu", h[size_t(w) * kEvenStamps + k]);
    }
    std::fprintf(f, "\n");
    std::fclose(f);
    return PSGD_OK;
}

static int compress_impl(psgd_plan* p, void* const* grads, int64_t step, int32_t it, hipStream_t s,
                         bool fuse, bool write_out, const FlatArgs* fl = nullptr,
                         const psgd_plan::Span* span = nullptr) {
    if (p->f64()) return compress_f64(p, grads, step, it, s);
    if (int st = refresh_pointers(p, grads, s)) return st;
    const psgd_plan::Span sp = span ? *span : p->full_span();
    const bool even = p->even(step, it);
    float* in = even ? p->P : p->Q;
    float* out = even ? p->Q : p->P;
    const bool fused = fused_norm(p, fuse, it);
    // rank 1, iteration 0, even: the joint norm of the (raw) state P is folded into the even
    // product (per-chunk sums of squares) and its reduction (divide, write normalised P)
    const bool fused0 = norm0_fold() && p->rbucket == 1 && it == 0 && even && !p->fused_final_at(step, it, write_out);
    // projection form of the fused last iteration: its orthonormalisation leaves R' in o_rq
    const bool proj = it == p->iters - 1 && p->proj_final(step, write_out);
    // folded orthonormalisation of the projection form: the even reduction leaves Gram
    // partials and k_orth_chain (no Gram pass, panel rows over several workgroups) replaces
    // k_orth_chol
    const bool qf = p->qfold(step, write_out);
    const bool xg = p->xgram_now && it == 1 && !even;  // the exchange left the summed Q's Gram
    float* ss = p->dev<float>(p->o_ss);

    if ((qf && proj) || xg) {
        ChainArgs ca{};
        ca.units = p->dev<OrthUnit>(p->o_units_q) + sp.uq[0];
        ca.uitems = p->dev<int32_t>(p->o_uitems) + 2 * sp.uq[0];
        ca.gram = p->dev<double>(p->o_gram);
        // the even iteration's reduced Q: k_reduce's yloc (world size 1) or the exchange's
        // summed copy (history slot 2, psgd_aggregate_ipc)
        ca.raw = xg ? p->hist(2, it - 1) : p->hist(1, it - 1);
        ca.state = in;
        ca.hx = p->hist(0, it);
        ca.rfac = p->dev<float>(p->o_rq);
        PSGD_HIP(launch_orth_chain(ca, sp.uq[1] - sp.uq[0], p->panel_q, p->rbucket, s));
    } else if (!fused && !fused0) {
        OrthArgs oa{};
        const int32_t* ur = even ? sp.up : sp.uq;
        oa.units = p->dev<OrthUnit>(even ? p->o_units_p : p->o_units_q) + ur[0];
        oa.state = in;
        oa.hx = p->hist(0, it);
        oa.save = it > 0 ? p->hist(2, it - 1) : nullptr;  // keep the all-reduced factor of it-1
        oa.rfac = proj ? p->dev<float>(p->o_rq) : nullptr;
        const int nunits = ur[1] - ur[0];
        if (nunits > 0) PSGD_HIP(launch_orth(oa, nunits, p->rbucket, even ? p->panel_p : p->panel_q, p->orth_chol, s));
    }

    // where the previous iteration's reduction left the per-item sums of squares of its
    // out-factor (this iteration's raw in-factor) and the per-group item ranges (after an
    // odd-even pass the previous even reduction ran over its own item list)
    const float* prev_ss = ss + size_t((it - 1) & 1) * p->ss_stride;
    const bool oe_prev2 = !even && it >= 2 && p->oe_at(step, it - 2, write_out) && fused_norm(p, fuse, it - 2);
    const int32_t* prev_grng = p->dev<int32_t>(even ? p->o_grng_odd : oe_prev2 ? p->o_grng_oe_items : p->o_grng_even);
    // odd-even pass: this odd iteration and the next (even) one's product in one gradient pass
    // (k_final_oe); its P rows need no reduction, the even iteration reduces its partials
    if (fused && span == nullptr && p->oe_at(step, it, write_out)) {
        FinalArgs fa{};
        fa.mats = p->dev<MatDesc>(p->o_mats);
        fa.tiles = p->dev<Tile>(p->o_tiles_oe);
        const int nfin = int(p->tiles_oe.size());
        fa.grads = p->grad_tab.table();
        fa.x = p->hist(p->raw_slot, it - 1);
        fill_terms(p, step, it, fa.res);
        fa.nres = it;
        fa.yloc = p->hist(1, it);
        fa.state = out;
        fa.ss_in = prev_ss;
        fa.grng_in = prev_grng;
        fa.xstate = in;
        fa.hx = p->hist(0, it);
        fa.ntiles = nfin;
        fa.oe_part = p->dev<float>(p->o_oe_part);
        fa.oe_ss = p->dev<float>(p->o_oe_ss);
        PSGD_HIP(launch_final_oe(p->dtype, it, fin_bucket(p->fin_smax), fa, nfin, s, nullptr));
        return PSGD_OK;
    }
    const bool oe_prev = even && it >= 1 && span == nullptr && p->oe_at(step, it - 1, write_out) && fused_norm(p, fuse, it - 1);
    if (it == p->iters - 1 && p->fused_final(step, write_out)) {
        // last iteration, odd: product + residual (+ output at world size 1) in one pass
        FinalArgs fa{};
        fa.out_nt = p->out_nt;
        fa.mats = p->dev<MatDesc>(p->o_mats);
        // the K-term form on its own row blocks when the plan has them (MatDesc::fin_rows_kt)
        const bool own_kt = !proj && !p->tiles_fin_kt.empty();
        const int32_t(&fr)[2] = own_kt ? sp.fin_kt : sp.fin;
        fa.tiles = p->dev<Tile>(own_kt ? p->o_tiles_fin_kt : p->o_tiles_fin) + fr[0];
        fa.grads = p->grad_tab.table();
        fa.out = p->out_now;
        fa.x = fused ? p->hist(p->raw_slot, it - 1) : p->hist(0, it);
        fill_terms(p, step, it, fa.res);
        fa.nres = it;
        fa.write_out = write_out ? 1 : 0;
        fa.yloc = p->hist(1, it);
        fa.state = out;
        fa.xout = p->xout_now;
        if (fused) {
            fa.ss_in = prev_ss;  // the in-factor Q came from an even iteration's reduction
            fa.grng_in = prev_grng;
            fa.xstate = in;
            fa.hx = p->hist(0, it);
        }
        const int nfin = fr[1] - fr[0];
        if (proj) {  // no error-feedback terms: P_0 and R' only (rank 1: P_0 and the matrix's c)
            fa.proj_p0 = p->hist(0, 0);
            fa.proj_r = p->dev<float>(p->o_rq);
            fa.mrng_in = p->dev<int32_t>(p->o_mrng);
            fill_terms(p, step, 0, fa.res);
            fa.nres = kFinProj;
        }
        fa.ntiles = nfin;
        if (fl && write_out) fa.flat = *fl;  // uncompressed tensors ride in the same launch
        if (nfin + fa.flat.nitems == 0) return PSGD_OK;
        std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
        if (int st = timing_begin(p, s, &ev, true)) return st;  // benchmark timing: the final pass
        TimedScope ts(ev);
        PSGD_HIP(launch_final_odd(p->dtype, p->rbucket, fa.nres, fin_bucket(p->fin_smax), fa, nfin, s));
        return PSGD_OK;
    }

    ProductArgs pa{};
    pa.mats = p->dev<MatDesc>(p->o_mats);
    pa.grads = p->grad_tab.table();
    pa.x = fused ? p->hist(p->raw_slot, it - 1) : fused0 ? in : p->hist(0, it);  // fused: the raw factor
    pa.part = p->dev<float>(p->o_part);
    if (fused0) pa.ss0 = p->dev<float>(p->o_ss0);
    fill_terms(p, step, it, pa.res);
    pa.nres = it;
    if (oe_prev) {
        // the product of this even iteration was accumulated by the odd-even pass
    } else if (even) {
        // persistent k_even: this span's workgroups [wg[0], wg[1]) of the segmentation
        pa.segs = p->dev<Seg>(p->o_segs);
        pa.wg_seg = p->dev<int32_t>(p->o_wg_seg) + sp.wg[0];
        pa.nwg = sp.wg[1] - sp.wg[0];
        // world size > 1 (no output written here): the first iteration's launch also packs the
        // uncompressed tensors, ahead of every collective
        if (fl && !write_out && it == 0) pa.flat = *fl;
        if (int st = even_stamps_begin(p, pa)) return st;
        PSGD_HIP(launch_even(p->dtype, p->rbucket, it, pa, pa.nwg, s));
        if (int st = even_stamps_end(p, pa, s)) return st;
    } else {
        if (sp.ov[1] > sp.ov[0]) {
            pa.tiles = p->dev<Tile>(p->o_tiles_ov) + sp.ov[0];
            PSGD_HIP(launch_product_odd(p->dtype, p->rbucket, it, pa, sp.ov[1] - sp.ov[0], s));
        }
        if (sp.om[1] > sp.om[0]) {
            pa.tiles = p->dev<Tile>(p->o_tiles_om) + sp.om[0];
            PSGD_HIP(launch_odd_mfma(p->dtype, p->rbucket, it, pa, sp.om[1] - sp.om[0], s));
        }
    }

    ReduceArgs ra{};
    ra.mats = pa.mats;
    const int32_t* rr = even ? sp.re : sp.ro;  // this parity's items (out-factor side)
    const int32_t* rn = even ? sp.ro : sp.re;  // the other parity's items (in-factor side)
    ra.items = p->dev<RedItem>(even ? p->o_red_even : p->o_red_odd) + rr[0];
    ra.part = pa.part;
    ra.yloc = p->hist(1, it);
    ra.state = out;
    ra.even = even ? 1 : 0;
    ra.nmain = rr[1] - rr[0];
    if (oe_prev) {  // the odd-even pass's block partials, per matrix [blocks][m]
        ra.items = p->dev<RedItem>(p->o_red_oe);
        ra.part = p->dev<float>(p->o_oe_part);
        ra.nmain = int32_t(p->red_oe.size());
    }
    if (fused0) {  // normalise the state P in place + history copy (P-side items)
        ra.ss_in = pa.ss0;
        ra.grng_in = p->dev<int32_t>(p->o_grng_ss0);
        ra.nitems = p->dev<RedItem>(p->o_red_odd) + sp.ro[0];
        ra.nnorm = sp.ro[1] - sp.ro[0];
        ra.raw = in;
        ra.xstate = in;
        ra.hx = p->hist(0, it);
    }
    if (fused) {  // in-factor items: the other parity's item list (in-factor side)
        ra.ss_in = oe_prev ? p->dev<float>(p->o_oe_ss) : prev_ss;  // odd-even: the blocks' sums of P^2
        ra.grng_in = oe_prev ? p->dev<int32_t>(p->o_grng_oe) : prev_grng;
        ra.nitems = p->dev<RedItem>(even ? p->o_red_odd : p->o_red_even) + rn[0];
        ra.nnorm = rn[1] - rn[0];
        ra.raw = p->hist(p->raw_slot, it - 1);
        ra.xstate = in;
        ra.hx = p->hist(0, it);
    }
    // ss_out is indexed by the launch's block (item) index: offset like the item list
    if (fused_norm(p, fuse, it + 1) && it + 1 < p->iters) ra.ss_out = ss + size_t(it & 1) * p->ss_stride + rr[0];
    ra.xout = p->xout_now;
    if (qf && even && it + 2 == p->iters) {  // the Q panels' Gram for k_orth_chain
        ra.gram = p->dev<double>(p->o_gram) + size_t(rr[0]) * kGramStride;
        ra.gram_r = p->rbucket;
    }
    if (ra.nmain + ra.nnorm > 0) PSGD_HIP(launch_reduce(ra, ra.nmain + ra.nnorm, s));
    return PSGD_OK;
}

int psgd_compress(psgd_plan* p, void* const* grads, int64_t step, int32_t it, void* stream) {
    if (!p || !grads) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (step < 0 || it < 0 || it >= p->iters) return fail(PSGD_ERR_VALUE, "step/iteration out of range");
    DevScope scope(p->device);
    return compress_impl(p, grads, step, it, static_cast<hipStream_t>(stream), false, false);
}

static int decompress_impl(psgd_plan* p, void* const* grads, void* out, int64_t step, int32_t world,
                           hipStream_t s, bool fuse, const FlatArgs* fl = nullptr,
                           const psgd_plan::Span* span = nullptr) {
    if (p->f64()) return decompress_f64(p, grads, out, step, world, s);
    if (int st = refresh_pointers(p, grads, s)) return st;
    const psgd_plan::Span sp = span ? *span : p->full_span();
    const int nt = sp.tiles[1] - sp.tiles[0];
    const int I = p->iters;
    ApplyArgs aa{};
    aa.mats = p->dev<MatDesc>(p->o_mats);
    aa.tiles = p->dev<Tile>(p->o_tiles) + sp.tiles[0];
    aa.grads = p->grad_tab.table();
    aa.out = out;
    fill_terms(p, step, I, aa.res);
    float* last = p->even(step, I - 1) ? p->Q : p->P;  // all-reduced factor of the last iteration
    for (int k = 0; k < kMaxTerms; ++k) aa.apx.p[k] = aa.apx.q[k] = nullptr;
    for (int k = 0; k < I; ++k) {
        const bool e = p->even(step, k);
        // fused (world 1): the reduced factor was never copied to hist(2): use hist(1)
        float* ybar = k + 1 < I ? p->hist(fused_norm(p, fuse, k + 1) ? 1 : 2, k) : last;
        aa.apx.p[k] = e ? p->hist(0, k) : ybar;
        aa.apx.q[k] = e ? ybar : p->hist(0, k);
    }
    aa.nterms = I;
    aa.alpha = float(1.0 / double(world));  // reference alpha = 1 / num_workers (:218)
    aa.out_nt = world == 1 ? p->out_nt : 0;
    if (p->fused_final(step, false)) {
        // the residual was written by the fused last iteration: output only
        aa.ntiles = nt;
        if (nt > 0) PSGD_HIP(launch_lowrank_out(p->dtype, p->rbucket, I, aa, nt, s));
        return PSGD_OK;
    }
    aa.ntiles = nt;
    if (fl) aa.flat = *fl;  // uncompressed tensors ride in the same launch
    if (nt + aa.flat.nitems == 0) return PSGD_OK;
    std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
    if (int st = timing_begin(p, s, &ev, true)) return st;
    TimedScope ts(ev);
    PSGD_HIP(launch_apply(p->dtype, p->rbucket, I, world == 1, aa, nt, s));
    return PSGD_OK;
}

int psgd_decompress(psgd_plan* p, void* const* grads, void* out, int64_t step, int32_t world,
                    void* stream) {
    if (!p || !grads || !out) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (step < 0 || world < 1) return fail(PSGD_ERR_VALUE, "step/world size out of range");
    if (reinterpret_cast<uintptr_t>(out) % 16) return fail(PSGD_ERR_LAYOUT, "output buffer must be 16-byte aligned");
    DevScope scope(p->device);
    return decompress_impl(p, grads, out, step, world, static_cast<hipStream_t>(stream), false);
}

// ------------------------------------------------------------- buckets (W > 1) ---
int psgd_plan_set_buckets(psgd_plan* p, int32_t nbuckets, const int32_t* group_end) {
    if (!p) return fail(PSGD_ERR_VALUE, "null plan");
    if (nbuckets < 0 || (nbuckets > 0 && !group_end)) return fail(PSGD_ERR_VALUE, "bad bucket list");
    const int32_t ng = int32_t(p->groups.size());
    int32_t prev = 0;
    for (int b = 0; b < nbuckets; ++b) {
        if (group_end[b] <= prev || group_end[b] > ng) return fail(PSGD_ERR_VALUE, "bucket group ends must increase");
        prev = group_end[b];
    }
    if (nbuckets > 0 && prev != ng) return fail(PSGD_ERR_VALUE, "the last bucket must end at the last group");
    if (nbuckets > kMaxBuckets) return fail(PSGD_ERR_VALUE, "at most 8 buckets");
    DevScope scope(p->device);
    if (p->bound) PSGD_HIP(hipDeviceSynchronize());  // the tile tables are rewritten below
    p->bucket_gend.assign(group_end, group_end + nbuckets);
    p->spans.clear();
    if (!p->f64()) {
        p->set_vec(p->vec_now);  // per-bucket segmentation of the even product, spans
        if (p->bound)
            if (int st = p->upload_tiles()) return st;
    }
    return PSGD_OK;
}

int psgd_plan_bucket_range(const psgd_plan* p, int32_t b, int64_t* p_off, int64_t* p_len, int64_t* q_off,
                           int64_t* q_len) {
    if (!p || b < 0 || b >= int32_t(std::max<size_t>(p->spans.size(), 1))) return fail(PSGD_ERR_VALUE, "bucket out of range");
    const psgd_plan::Span sp = p->spans.empty() ? p->full_span() : p->spans[b];
    if (p_off) *p_off = sp.p[0];
    if (p_len) *p_len = sp.p[1] - sp.p[0];
    if (q_off) *q_off = sp.q[0];
    if (q_len) *q_len = sp.q[1] - sp.q[0];
    return PSGD_OK;
}

static int bucket_span(const psgd_plan* p, int32_t b, psgd_plan::Span* sp) {
    if (p->f64()) return fail(PSGD_ERR_DTYPE, "buckets are not supported for fp64 plans");
    if (p->spans.empty()) {
        if (b != 0) return fail(PSGD_ERR_VALUE, "bucket out of range");
        *sp = p->full_span();
        return PSGD_OK;
    }
    if (b < 0 || b >= int32_t(p->spans.size())) return fail(PSGD_ERR_VALUE, "bucket out of range");
    *sp = p->spans[b];
    return PSGD_OK;
}

int psgd_compress_bucket(psgd_plan* p, void* const* grads, int64_t step, int32_t it, int32_t bucket, void* stream) {
    if (!p || !grads) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (step < 0 || it < 0 || it >= p->iters) return fail(PSGD_ERR_VALUE, "step/iteration out of range");
    psgd_plan::Span sp;
    if (int st = bucket_span(p, bucket, &sp)) return st;
    DevScope scope(p->device);
    return compress_impl(p, grads, step, it, static_cast<hipStream_t>(stream), false, false, nullptr, &sp);
}

int psgd_decompress_bucket(psgd_plan* p, void* const* grads, void* out, int64_t step, int32_t world, int32_t bucket,
                           void* stream) {
    if (!p || !grads || !out) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (step < 0 || world < 1) return fail(PSGD_ERR_VALUE, "step/world size out of range");
    if (reinterpret_cast<uintptr_t>(out) % 16) return fail(PSGD_ERR_LAYOUT, "output buffer must be 16-byte aligned");
    psgd_plan::Span sp;
    if (int st = bucket_span(p, bucket, &sp)) return st;
    DevScope scope(p->device);
    return decompress_impl(p, grads, out, step, world, static_cast<hipStream_t>(stream), false, nullptr, &sp);
}

// ------------------------------------------------- one-shot all-reduce over IPC ---
// an exchange handle: the HIP IPC handle of the arena chunk, the region's byte offset in it,
// then the session nonce (last, 4 bytes)
constexpr size_t kHandleBytes = sizeof(hipIpcMemHandle_t) + sizeof(uint64_t) + sizeof(uint32_t);

int psgd_ipc_handle_bytes(int64_t* bytes) {
    if (!bytes) return fail(PSGD_ERR_VALUE, "null argument");
    *bytes = int64_t(kHandleBytes);
    return PSGD_OK;
}

int psgd_ipc_create(psgd_plan* p, int64_t flat_numel, void* handle_out) {
    if (!p || !handle_out) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (p->f64()) return fail(PSGD_ERR_DTYPE, "the IPC all-reduce takes fp32/bf16 plans");
    if (flat_numel < 0) return fail(PSGD_ERR_VALUE, "negative flat size");
    if (!p->ipc_peer.empty()) return fail(PSGD_ERR_STATE, "exchange session open (psgd_ipc_close first)");
    DevScope scope(p->device);
    auto a64 = [](int64_t x) { return (x + 63) & ~int64_t(63); };
    const int64_t flat_off = a64(std::max<int64_t>(p->fmax, 1));
    const int64_t slot = flat_off + a64(flat_numel);
    const size_t bytes = size_t(kXchgHeader) + size_t(2 * p->iters * slot) * sizeof(float);
    // a region of the process's arena: this plan's previous region when it is large enough (a
    // re-opened session), else a new one (the old one goes back to the arena)
    if (p->ipc_buf && p->ipc_bytes < bytes) {
        xchg_arena().release(p->ipc_chunk, p->ipc_off, p->ipc_bytes);
        p->ipc_buf = nullptr;
    }
    if (!p->ipc_buf) {
        int chunk = -1;
        size_t off = 0;
        if (int st = xchg_arena().acquire(p->device, bytes, &chunk, &off)) return st;
        p->ipc_chunk = chunk;
        p->ipc_off = off;
        p->ipc_bytes = bytes;
        p->ipc_buf = xchg_arena().chunk(chunk).base + off;
    }
    p->ipc_flat_off = flat_off;
    p->ipc_flat_cap = flat_numel;
    p->ipc_slot = slot;
    PSGD_HIP(hipMemset(p->ipc_buf, 0, bytes));  // flags at epoch 0, error word clear
    if (!p->xerr_host) {
        PSGD_HIP(hipHostMalloc(reinterpret_cast<void**>(&p->xerr_host), sizeof(int32_t),
                               hipHostMallocMapped | hipHostMallocCoherent));
        PSGD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&p->xerr_dev), p->xerr_host, 0));
    }
    __atomic_store_n(p->xerr_host, 0, __ATOMIC_RELEASE);
    // a fresh session nonce (never 0: a zeroed header never matches), in the header and the handle
    {
        static std::atomic<uint32_t> counter{0};
        uint64_t z = uint64_t(std::chrono::steady_clock::now().time_since_epoch().count()) ^
                     (uint64_t(reinterpret_cast<uintptr_t>(p->ipc_buf)) << 7) ^ (uint64_t(getpid()) << 40) ^
                     (uint64_t(counter.fetch_add(1)) * 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p->ipc_nonce = uint32_t(z ^ (z >> 31)) | 1u;
    }
    PSGD_HIP(hipMemcpy(p->ipc_buf + kXchgNonceOff, &p->ipc_nonce, sizeof(uint32_t), hipMemcpyHostToDevice));
    PSGD_HIP(hipDeviceSynchronize());  // zeroed before any peer can open and poll it
    const XchgChunk c = xchg_arena().chunk(p->ipc_chunk);
    char* h = static_cast<char*>(handle_out);
    const uint64_t off64 = uint64_t(p->ipc_off);
    std::memcpy(h, &c.handle, sizeof(hipIpcMemHandle_t));
    std::memcpy(h + sizeof(hipIpcMemHandle_t), &off64, sizeof(uint64_t));
    std::memcpy(h + sizeof(hipIpcMemHandle_t) + sizeof(uint64_t), &p->ipc_nonce, sizeof(uint32_t));
    return PSGD_OK;
}

int psgd_ipc_open(psgd_plan* p, int32_t world, int32_t rank, const void* handles) {
    if (!p || !handles) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->ipc_buf) return fail(PSGD_ERR_STATE, "psgd_ipc_create first");
    if (!p->ipc_peer.empty()) return fail(PSGD_ERR_STATE, "peers already open (psgd_ipc_close first)");
    if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return fail(PSGD_ERR_VALUE, "bad world/rank");
    DevScope scope(p->device);
    const char* hb = static_cast<const char*>(handles);
    std::vector<void*> peer(size_t(world), nullptr);
    std::vector<uint32_t> nonce(size_t(world), 0);
    const XchgChunk own = xchg_arena().chunk(p->ipc_chunk);
    for (int w = 0; w < world; ++w) {
        hipIpcMemHandle_t h;
        uint64_t off = 0;
        const char* e = hb + size_t(w) * kHandleBytes;
        std::memcpy(&h, e, sizeof(h));
        std::memcpy(&off, e + sizeof(h), sizeof(uint64_t));
        std::memcpy(&nonce[w], e + sizeof(h) + sizeof(uint64_t), sizeof(uint32_t));
        if (w == rank) {
            peer[w] = p->ipc_buf;
            if (nonce[w] != p->ipc_nonce || off != uint64_t(p->ipc_off) ||
                std::memcmp(&h, &own.handle, sizeof(h)) != 0)
                return fail(PSGD_ERR_VALUE, "handle list: this rank's entry is not its own exchange handle");
            continue;
        }
        // the peer's chunk, mapped once per process (no unmap / remap between sessions)
        char* base = nullptr;
        if (int st = xchg_arena().map_peer(p->device, h, &base)) return st;
        peer[w] = base + off;
        // the mapping must reach THIS session's region of rank w: its header carries the nonce the
        // handle announced (a stale mapping, or an offset into another session's region, does not)
        uint32_t seen = 0;
        const hipError_t e2 = hipMemcpy(&seen, static_cast<char*>(peer[w]) + kXchgNonceOff, sizeof(uint32_t),
                                        hipMemcpyDeviceToHost);
        if (e2 != hipSuccess || seen != nonce[w])
            return fail(PSGD_ERR_STATE, "the mapping of rank " + std::to_string(w) +
                                            "'s exchange buffer does not reach this session's buffer (stale IPC mapping)");
    }
    p->ipc_peer = peer;
    p->ipc_world = world;
    p->ipc_rank = rank;
    if (int st = upload(p->dev<void>(p->o_ipc_nonce), nonce.data(), size_t(world) * sizeof(uint32_t))) return st;
    return upload(p->dev<void>(p->o_ipc_ptrs), p->ipc_peer.data(), size_t(world) * sizeof(void*));
}

int psgd_ipc_close(psgd_plan* p) {
    if (!p) return fail(PSGD_ERR_VALUE, "null plan");
    if (p->ipc_peer.empty()) return PSGD_OK;
    DevScope scope(p->device);
    PSGD_HIP(hipDeviceSynchronize());  // no kernel of this rank still reads a peer buffer
    // the peer mappings stay in the process's arena (mapped once, never unmapped)
    p->ipc_peer.clear();
    p->ipc_world = 0;
    p->ipc_rank = -1;
    if (p->xerr_host) __atomic_store_n(p->xerr_host, 0, __ATOMIC_RELEASE);  // a fresh exchange
    PSGD_HIP(hipMemset(static_cast<char*>(p->ipc_buf) + kXchgErrOff, 0, sizeof(int32_t)));
    return PSGD_OK;
}

int psgd_ipc_debug(psgd_plan* p, int32_t w, psgd_ipc_info* info) {
    if (!p || !info) return fail(PSGD_ERR_VALUE, "null argument");
    std::memset(info, 0, sizeof(*info));
    int64_t c[4];
    xchg_arena().counters(c);
    info->arena_allocs = c[0];
    info->arena_opens = c[1];
    info->arena_reuses = c[2];
    info->arena_frees = c[3];
    info->own_va = uint64_t(reinterpret_cast<uintptr_t>(p->ipc_buf));
    info->own_nonce = p->ipc_nonce;
    if (p->ipc_peer.empty()) return PSGD_OK;
    if (w < 0 || w >= p->ipc_world) return fail(PSGD_ERR_VALUE, "peer out of range");
    DevScope scope(p->device);
    info->peer_va = uint64_t(reinterpret_cast<uintptr_t>(p->ipc_peer[size_t(w)]));
    uint32_t seen = 0;
    PSGD_HIP(hipMemcpy(&seen, static_cast<char*>(p->ipc_peer[size_t(w)]) + kXchgNonceOff, sizeof(uint32_t),
                       hipMemcpyDeviceToHost));
    info->peer_nonce_seen = seen;
    return PSGD_OK;
}

int psgd_ipc_status(psgd_plan* p, int32_t* timed_out) {
    if (!p || !timed_out) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    DevScope scope(p->device);
    PSGD_HIP(hipDeviceSynchronize());  // every enqueued exchange wait has ended
    *timed_out = p->xerr_set() ? 1 : 0;  // sticky until psgd_ipc_close
    return PSGD_OK;
}

// ------------------------------------------------- building blocks (reducer variants) ---
static int check_terms(int32_t nterms, const float* const* a, const float* const* b) {
    if (nterms < 0 || nterms > kMaxTerms) return fail(PSGD_ERR_VALUE, "term count out of range");
    for (int k = 0; k < nterms; ++k)
        if (!a || !b || !a[k] || !b[k]) return fail(PSGD_ERR_VALUE, "null term buffer");
    return PSGD_OK;
}

int psgd_product(psgd_plan* p, void* const* grads, int32_t odd, const float* x, float* y, int32_t nterms,
                 const float* const* term_p, const float* const* term_q, void* stream) {
    if (!p || !grads || !x || !y) return fail(PSGD_ERR_VALUE, "null argument");
    if (p->f64()) return fail(PSGD_ERR_DTYPE, "the building blocks take fp32/bf16 plans");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (int st = check_terms(nterms, term_p, term_q)) return st;
    DevScope scope(p->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int st = refresh_pointers(p, grads, s)) return st;
    ProductArgs pa{};
    pa.mats = p->dev<MatDesc>(p->o_mats);
    pa.grads = p->grad_tab.table();
    pa.x = x;
    pa.part = p->dev<float>(p->o_part);
    for (int k = 0; k < nterms; ++k) {
        pa.res.p[k] = term_p[k];
        pa.res.q[k] = term_q[k];
    }
    pa.nres = nterms;
    if (!odd) {
        pa.segs = p->dev<Seg>(p->o_segs);
        pa.wg_seg = p->dev<int32_t>(p->o_wg_seg);
        pa.nwg = int(p->wg_seg.size()) - 1;
        PSGD_HIP(launch_even(p->dtype, p->rbucket, nterms, pa, pa.nwg, s));
    } else {
        if (!p->tiles_ov.empty()) {
            pa.tiles = p->dev<Tile>(p->o_tiles_ov);
            PSGD_HIP(launch_product_odd(p->dtype, p->rbucket, nterms, pa, int(p->tiles_ov.size()), s));
        }
        if (!p->tiles_om.empty()) {
            pa.tiles = p->dev<Tile>(p->o_tiles_om);
            PSGD_HIP(launch_odd_mfma(p->dtype, p->rbucket, nterms, pa, int(p->tiles_om.size()), s));
        }
    }
    ReduceArgs ra{};
    ra.mats = pa.mats;
    ra.items = p->dev<RedItem>(odd ? p->o_red_odd : p->o_red_even);
    ra.part = pa.part;
    ra.yloc = y;
    ra.state = y;
    ra.even = odd ? 0 : 1;
    ra.nmain = int(odd ? p->red_odd.size() : p->red_even.size());
    PSGD_HIP(launch_reduce(ra, ra.nmain, s));
    return PSGD_OK;
}

int psgd_orthogonalize(psgd_plan* p, int32_t which, float* buf, int32_t mode, void* stream) {
    if (!p || !buf) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (mode != 0 && mode != 1) return fail(PSGD_ERR_VALUE, "mode must be 0 (reference) or 1 (paper-code)");
    if (p->f64()) return fail(PSGD_ERR_DTYPE, "the building blocks take fp32/bf16 plans");
    DevScope scope(p->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    OrthArgs oa{};
    oa.state = buf;
    oa.hx = p->hist(0, 0);  // scratch copy
    if (mode == 1) {
        oa.units = p->dev<OrthUnit>(which ? p->o_munits_p : p->o_munits_q);
        PSGD_HIP(launch_orth_mgs(oa, int(p->mats.size()), p->rbucket, s));
    } else {
        oa.units = p->dev<OrthUnit>(which ? p->o_units_p : p->o_units_q);
        const int nunits = int(which ? p->units_p.size() : p->units_q.size());
        PSGD_HIP(launch_orth(oa, nunits, p->rbucket, which ? p->panel_p : p->panel_q, p->orth_chol, s));
    }
    return PSGD_OK;
}

// select (or upload, stream-ordered) a per-tensor destination table; every pointer must keep
// the vector layout's alignment where the matrix uses it
static int refresh_table(psgd_plan* p, void* const* ptrs, TableCache& tab, hipStream_t s) {
    const uintptr_t need = p->dtype == PSGD_F32 ? 16 : 8;
    for (const MatDesc& md : p->mats) {
        if (!ptrs[md.tensor]) return fail(PSGD_ERR_VALUE, "null destination pointer");
        if (md.vec && reinterpret_cast<uintptr_t>(ptrs[md.tensor]) % need)
            return fail(PSGD_ERR_LAYOUT, "destination tensor is not aligned for the vector layout");
    }
    PSGD_HIP(tab.select(ptrs, s));
    return PSGD_OK;
}

int psgd_reconstruct(psgd_plan* p, void* const* grads, void* const* resid_out, void* const* out, int32_t nterms,
                     const float* const* term_p, const float* const* term_q, const float* const* avg_p,
                     const float* const* avg_q, float alpha, void* stream) {
    if (!p || !grads || !out) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (nterms < 1) return fail(PSGD_ERR_VALUE, "at least one term");
    if (p->f64()) return fail(PSGD_ERR_DTYPE, "the building blocks take fp32/bf16 plans");
    if (int st = check_terms(nterms, term_p, term_q)) return st;
    if (int st = check_terms(nterms, avg_p, avg_q)) return st;
    DevScope scope(p->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int st = refresh_pointers(p, grads, s)) return st;
    if (resid_out)
        if (int st = refresh_table(p, resid_out, p->rdst_tab, s)) return st;
    if (int st = refresh_table(p, out, p->odst_tab, s)) return st;
    ApplyArgs aa{};
    aa.mats = p->dev<MatDesc>(p->o_mats);
    aa.tiles = p->dev<Tile>(p->o_tiles);
    aa.grads = p->grad_tab.table();
    aa.rdst = resid_out ? p->rdst_tab.table() : nullptr;
    aa.odst = p->odst_tab.table();
    bool shared = alpha == 1.0f;
    for (int k = 0; k < nterms; ++k) {
        aa.res.p[k] = term_p[k];
        aa.res.q[k] = term_q[k];
        aa.apx.p[k] = avg_p[k];
        aa.apx.q[k] = avg_q[k];
        shared = shared && avg_p[k] == term_p[k] && avg_q[k] == term_q[k];
    }
    aa.nterms = nterms;
    aa.alpha = alpha;
    aa.ntiles = int32_t(p->tiles.size());
    PSGD_HIP(launch_apply(p->dtype, p->rbucket, nterms, shared, aa, int(p->tiles.size()), s));
    return PSGD_OK;
}

int psgd_plan_fused_final(const psgd_plan* p, int64_t step, int32_t aggregate, int32_t* fused) {
    if (!p || !fused) return fail(PSGD_ERR_VALUE, "null argument");
    if (step < 0) return fail(PSGD_ERR_VALUE, "step out of range");
    *fused = p->proj_final(step, aggregate != 0) ? 2 : p->fused_final(step, aggregate != 0) ? 1 : 0;
    return PSGD_OK;
}

int psgd_plan_odd_even(const psgd_plan* p, int64_t step, int32_t it, int32_t* on) {
    if (!p || !on) return fail(PSGD_ERR_VALUE, "null argument");
    if (step < 0 || it < 0 || it >= p->iters) return fail(PSGD_ERR_VALUE, "step/iteration out of range");
    static const bool fuse = env_int("PSGD_FUSE_NORM", 1) != 0;  // as aggregate_impl
    *on = p->oe_at(step, it, true) && fused_norm(p, fuse, it) ? 1 : 0;
    return PSGD_OK;
}

int psgd_plan_set_timing(psgd_plan* p, int32_t enable) {
    if (!p) return fail(PSGD_ERR_VALUE, "null plan");
    p->timing = enable != 0;
    p->ev_used = 0;
    return PSGD_OK;
}

int psgd_plan_timing_read(psgd_plan* p, double* total_ms, int32_t* launches) {
    if (!p || !total_ms || !launches) return fail(PSGD_ERR_VALUE, "null argument");
    DevScope scope(p->device);
    double sum = 0.0;
    for (size_t i = 0; i < p->ev_used; ++i) {
        PSGD_HIP(hipEventSynchronize(p->ev_pool[i].second));
        float ms = 0.f;
        PSGD_HIP(hipEventElapsedTime(&ms, p->ev_pool[i].first, p->ev_pool[i].second));
        sum += ms;
    }
    *total_ms = sum;
    *launches = int32_t(p->ev_used);
    p->ev_used = 0;
    return PSGD_OK;
}

static int bucket_span(const psgd_plan* p, int32_t b, psgd_plan::Span* sp);
static int aggregate_entry(psgd_plan* p, void* const* grads, void* out, int64_t step, hipStream_t s,
                           const FlatArgs* fl, const psgd_flat* f);
static int flat_args(psgd_flat* f, void* const* tensors, void* flat, int32_t world, hipStream_t s, FlatArgs* out);

static int aggregate_impl(psgd_plan* p, void* const* grads, void* out, int64_t step, hipStream_t s,
                          const FlatArgs* fl, const psgd_plan::Span* span = nullptr) {
    static const bool fuse = env_int("PSGD_FUSE_NORM", 1) != 0;
    p->out_now = out;
    for (int it = 0; it < p->iters; ++it)
        if (int st = compress_impl(p, grads, step, it, s, fuse, true, fl, span)) return st;
    if (p->fused_final(step, true)) return PSGD_OK;  // output written by the fused last iteration
    return decompress_impl(p, grads, out, step, 1, s, fuse, fl, span);
}

int psgd_aggregate(psgd_plan* p, void* const* grads, void* out, int64_t step, void* stream) {
    if (!p || !grads || !out) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (step < 0) return fail(PSGD_ERR_VALUE, "step out of range");
    if (reinterpret_cast<uintptr_t>(out) % 16) return fail(PSGD_ERR_LAYOUT, "output buffer must be 16-byte aligned");
    DevScope scope(p->device);
    return aggregate_entry(p, grads, out, step, static_cast<hipStream_t>(stream), nullptr, nullptr);
}

// ------------------------------------------------------------------ flat pack ------
int psgd_flat_create(const int64_t* numels, int32_t count, int32_t dtype, psgd_flat** out) {
    if (!out) return fail(PSGD_ERR_VALUE, "null argument");
    *out = nullptr;
    if (count < 0 || (count > 0 && !numels)) return fail(PSGD_ERR_VALUE, "bad tensor list");
    if (dtype != PSGD_F32 && dtype != PSGD_BF16 && dtype != PSGD_F64)
        return fail(PSGD_ERR_DTYPE, "dtype must be fp32, bf16 or fp64");
    auto* f = new psgd_flat();
    f->dtype = dtype;
    f->count = count;
    for (int i = 0; i < count; ++i) {
        if (numels[i] < 0) {
            delete f;
            return fail(PSGD_ERR_VALUE, "negative numel");
        }
        // empty tensors occupy no flat range: no lookup entry (their pointer slot stays)
        if (numels[i] > 0) f->entries.push_back(FlatEntry{f->total, numels[i], i, 0});
        f->total += numels[i];
    }
    for (size_t e = 0; e < f->entries.size(); ++e)
        for (int64_t st = 0; st < f->entries[e].numel; st += kFlatItem) f->items.push_back(FlatItem{int32_t(e), 0, st});
    f->o_ptrs = 0;
    f->o_ents = align256(TableCache::bytes(size_t(std::max(count, 1))));
    f->o_items = align256(f->o_ents + std::max<size_t>(f->entries.size(), 1) * sizeof(FlatEntry));
    f->ws_bytes = align256(f->o_items + std::max<size_t>(f->items.size(), 1) * sizeof(FlatItem));
    *out = f;
    return PSGD_OK;
}

int psgd_flat_destroy(psgd_flat* f) {
    delete f;
    return PSGD_OK;
}

int psgd_flat_workspace_bytes(const psgd_flat* f, int64_t* bytes) {
    if (!f || !bytes) return fail(PSGD_ERR_VALUE, "null argument");
    *bytes = int64_t(f->ws_bytes);
    return PSGD_OK;
}

int psgd_flat_bind(psgd_flat* f, int32_t device, void* workspace) {
    if (!f || !workspace) return fail(PSGD_ERR_VALUE, "null argument");
    DevScope scope(device);
    f->device = device;
    f->ws = static_cast<char*>(workspace);
    f->tab.bind(f->ws + f->o_ptrs, size_t(f->count));
    if (int st = upload(f->ws + f->o_ents, f->entries.data(), f->entries.size() * sizeof(FlatEntry))) return st;
    if (int st = upload(f->ws + f->o_items, f->items.data(), f->items.size() * sizeof(FlatItem))) return st;
    f->bound = true;
    return PSGD_OK;
}

// Device-side arguments of a flat pack (selects or uploads the pointer table, stream-ordered).
static int flat_args(psgd_flat* f, void* const* tensors, void* flat, int32_t world, hipStream_t s,
                     FlatArgs* out) {
    PSGD_HIP(f->tab.select(tensors, s));
    FlatArgs& a = *out;
    a = FlatArgs{};
    a.entries = reinterpret_cast<const FlatEntry*>(f->ws + f->o_ents);
    a.items = reinterpret_cast<const FlatItem*>(f->ws + f->o_items);
    a.tensors = f->tab.table();
    a.flat = flat;
    a.nitems = int32_t(f->items.size());
    a.world = world;
    return PSGD_OK;
}

int psgd_flat_pack(psgd_flat* f, void* const* tensors, void* flat, int32_t world, void* stream) {
    if (!f || (!tensors && f->count > 0) || (!flat && f->total > 0)) return fail(PSGD_ERR_VALUE, "null argument");
    if (!f->bound) return fail(PSGD_ERR_STATE, "flat plan is not bound");
    if (world < 1) return fail(PSGD_ERR_VALUE, "world size must be >= 1");
    if (f->total == 0) return PSGD_OK;
    DevScope scope(f->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    FlatArgs a;
    if (int st = flat_args(f, tensors, flat, world, s, &a)) return st;
    PSGD_HIP(launch_flat_pack(f->dtype, a, s));
    return PSGD_OK;
}

// ------------------------------------------------------ DDP run tables (psgd_runs) --
int psgd_runs_create(const int64_t* bucket_off, const int32_t* tensor, const int64_t* tensor_off,
                     const int64_t* len, int32_t nruns, int32_t ntensors, int32_t dtype, psgd_runs** out) {
    if (!out) return fail(PSGD_ERR_VALUE, "null argument");
    *out = nullptr;
    if (nruns < 0 || ntensors < 0 || (nruns > 0 && (!bucket_off || !tensor || !tensor_off || !len)))
        return fail(PSGD_ERR_VALUE, "bad run table");
    if (dtype != PSGD_F32 && dtype != PSGD_BF16 && dtype != PSGD_F64)
        return fail(PSGD_ERR_DTYPE, "dtype must be fp32, bf16 or fp64");
    auto* r = new psgd_runs();
    r->dtype = dtype;
    r->ntensors = ntensors;
    for (int32_t k = 0; k < nruns; ++k) {
        if (len[k] < 0 || bucket_off[k] < 0 || tensor_off[k] < 0 || tensor[k] < 0 || tensor[k] >= ntensors) {
            delete r;
            return fail(PSGD_ERR_VALUE, "run " + std::to_string(k) + " out of range");
        }
        for (int64_t e = 0; e < len[k]; e += kRunItem)
            r->items.push_back(RunItem{bucket_off[k] + e, tensor_off[k] + e, tensor[k],
                                       int32_t(std::min<int64_t>(kRunItem, len[k] - e))});
        r->bucket_numel = std::max(r->bucket_numel, bucket_off[k] + len[k]);
    }
    if (r->items.size() > size_t(INT32_MAX)) {
        delete r;
        return fail(PSGD_ERR_VALUE, "run table too large for one launch");
    }
    r->o_ptrs = 0;
    r->o_items = align256(TableCache::bytes(size_t(std::max(ntensors, 1))));
    r->ws_bytes = align256(r->o_items + std::max<size_t>(r->items.size(), 1) * sizeof(RunItem));
    *out = r;
    return PSGD_OK;
}

int psgd_runs_destroy(psgd_runs* r) {
    delete r;
    return PSGD_OK;
}

int psgd_runs_workspace_bytes(const psgd_runs* r, int64_t* bytes) {
    if (!r || !bytes) return fail(PSGD_ERR_VALUE, "null argument");
    *bytes = int64_t(r->ws_bytes);
    return PSGD_OK;
}

int psgd_runs_bind(psgd_runs* r, int32_t device, void* workspace) {
    if (!r || !workspace) return fail(PSGD_ERR_VALUE, "null argument");
    DevScope scope(device);
    r->device = device;
    r->ws = static_cast<char*>(workspace);
    r->tab.bind(r->ws + r->o_ptrs, size_t(r->ntensors));
    if (int st = upload(r->ws + r->o_items, r->items.data(), r->items.size() * sizeof(RunItem))) return st;
    r->bound = true;
    return PSGD_OK;
}

static int runs_launch(psgd_runs* r, const void* bucket, void* const* tensors, bool add, void* stream) {
    if (!r || (!bucket && !r->items.empty()) || (!tensors && r->ntensors > 0)) return fail(PSGD_ERR_VALUE, "null argument");
    if (!r->bound) return fail(PSGD_ERR_STATE, "run table is not bound");
    if (r->items.empty()) return PSGD_OK;
    DevScope scope(r->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    PSGD_HIP(r->tab.select(tensors, s));
    RunsArgs a{};
    a.items = reinterpret_cast<const RunItem*>(r->ws + r->o_items);
    a.bucket = const_cast<void*>(bucket);
    a.tensors = r->tab.table();
    a.nitems = int32_t(r->items.size());
    PSGD_HIP(launch_runs(r->dtype, add, a, s));
    return PSGD_OK;
}

int psgd_runs_add(psgd_runs* r, const void* bucket, void* const* tensors, void* stream) {
    return runs_launch(r, bucket, tensors, true, stream);
}

int psgd_runs_gather(psgd_runs* r, void* bucket, void* const* tensors, void* stream) {
    return runs_launch(r, bucket, tensors, false, stream);
}

// World-size-1 entry (psgd_aggregate / psgd_aggregate_flat): the pointer tables are selected
// (or uploaded) on the caller's stream, then the step's launches follow on it.
static int aggregate_entry(psgd_plan* p, void* const* grads, void* out, int64_t step, hipStream_t s,
                           const FlatArgs* fl, const psgd_flat*) {
    if (int st = refresh_pointers(p, grads, s)) return st;
    return aggregate_impl(p, grads, out, step, s, fl);
}

int psgd_aggregate_flat(psgd_plan* p, void* const* grads, void* out, int64_t step, psgd_flat* f,
                        void* const* unc, void* flat_out, void* stream) {
    if (!f || f->total == 0) return psgd_aggregate(p, grads, out, step, stream);
    if (!p || !grads || !out || !unc || !flat_out) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound || !f->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (step < 0) return fail(PSGD_ERR_VALUE, "step out of range");
    if (reinterpret_cast<uintptr_t>(out) % 16) return fail(PSGD_ERR_LAYOUT, "output buffer must be 16-byte aligned");
    if (f->dtype != p->dtype || f->device != p->device || p->f64()) {  // separate launches
        if (int st = psgd_aggregate(p, grads, out, step, stream)) return st;
        return psgd_flat_pack(f, unc, flat_out, 1, stream);
    }
    DevScope scope(p->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    FlatArgs a;
    if (int st = flat_args(f, unc, flat_out, 1, s, &a)) return st;
    return aggregate_entry(p, grads, out, step, s, &a, f);
}

static int aggregate_comm_body(psgd_plan* p, void* const* grads, void* out, int64_t step, psgd_flat* f,
                               void* const* unc, void* flat_out, psgd_comm* comm, hipStream_t s);

// World size W in one call (include/psgd.h): per iteration the kernels, then the in-place SUM
// all-reduce of the out-factor state on the same stream (the last grouped with the flat
// buffer of the uncompressed tensors), then the output pass. Same sequence as the building
// blocks psgd_compress / all_reduce / psgd_decompress (reference powersgd.py:172-230).
int psgd_aggregate_comm(psgd_plan* p, void* const* grads, void* out, int64_t step, psgd_flat* f, void* const* unc,
                        void* flat_out, psgd_comm* comm, void* stream) {
    if (!p || !grads || !out || !comm) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (step < 0) return fail(PSGD_ERR_VALUE, "step out of range");
    if (p->f64()) return fail(PSGD_ERR_DTYPE, "psgd_aggregate_comm takes fp32/bf16 plans (fp32 factors)");
    if (reinterpret_cast<uintptr_t>(out) % 16) return fail(PSGD_ERR_LAYOUT, "output buffer must be 16-byte aligned");
    const bool has_flat = f && f->total > 0;
    if (has_flat) {
        if (!unc || !flat_out) return fail(PSGD_ERR_VALUE, "null argument");
        if (!f->bound) return fail(PSGD_ERR_STATE, "flat plan is not bound");
        if (f->dtype != PSGD_F32) return fail(PSGD_ERR_DTYPE, "psgd_aggregate_comm packs fp32 uncompressed tensors");
    }
    // a poisoned communicator is refused before the step launches anything: the caller's
    // gradients and the P/Q state stay as they were
    std::string why;
    if (comm_poisoned(comm, &why))
        return fail(PSGD_ERR_STATE, ("communicator unusable after an earlier failure: " + why).c_str());
    DevScope scope(p->device);
    const int st = aggregate_comm_body(p, grads, out, step, has_flat ? f : nullptr, unc, flat_out, comm,
                                       static_cast<hipStream_t>(stream));
    // a failure past the argument checks can leave this rank's collective sequence short of its
    // peers': the communicator refuses every later call (psgd_comm.cpp, comm_poison)
    if (st) comm_poison(comm, psgd_last_error());
    return st;
}

static int aggregate_comm_body(psgd_plan* p, void* const* grads, void* out, int64_t step, psgd_flat* f,
                               void* const* unc, void* flat_out, psgd_comm* comm, hipStream_t s) {
    void* stream = s;
    const bool has_flat = f != nullptr;
    const int world = comm_world(comm);
    // x / W into the flat buffer, x = 0 (utils.py:43-47, powersgd.py:29-30): inside the first
    // even product's launch when the step starts even, else its own launch
    FlatArgs fa{};
    const bool fold = has_flat && p->even(step, 0);
    if (fold) {
        if (int st = flat_args(f, unc, flat_out, world, s, &fa)) return st;
    } else if (has_flat) {
        if (int st = psgd_flat_pack(f, unc, flat_out, world, stream)) return st;
    }
    for (int it = 0; it < p->iters; ++it) {
        if (int st = compress_impl(p, grads, step, it, s, false, false, fold ? &fa : nullptr)) return st;
        const bool e = p->even(step, it);
        const bool last = it == p->iters - 1;
        if (int st = comm_allreduce(comm, e ? p->Q : p->P, size_t(e ? p->qtot : p->ptot),
                                    last && has_flat ? static_cast<float*>(flat_out) : nullptr,
                                    last && has_flat ? size_t(f->total) : 0, s))
            return st;
    }
    return decompress_impl(p, grads, out, step, world, s, false);
}


// World size W over the IPC exchange (include/psgd.h): per iteration the codec kernels (the
// reduction or fused final pass also writes the local factor into this rank's exchange slot),
// then k_xchg (flag, bounded wait for the peers' flags, rank-order SUM into the state buffer; the
// last one also sums the uncompressed tensors packed /W into flat_out), then the output pass.
// Nothing leaves the stream: no host barrier, no host synchronisation.
int psgd_aggregate_ipc(psgd_plan* p, void* const* grads, void* out, int64_t step, psgd_flat* f, void* const* unc,
                       void* flat_out, void* stream) {
    if (!p || !grads || !out) return fail(PSGD_ERR_VALUE, "null argument");
    if (!p->bound) return fail(PSGD_ERR_STATE, "plan is not bound to device memory");
    if (p->ipc_peer.empty()) return fail(PSGD_ERR_STATE, "psgd_ipc_open first");
    // a wait of an earlier step gave up: that step's sums were invalid and the two-parity slot
    // reuse is no longer safe, so every later step is refused (the ranks have drifted apart)
    if (p->xerr_set())
        return fail(PSGD_ERR_STATE, "an earlier IPC exchange wait timed out (a peer did not arrive within "
                                    "PSGD_IPC_SPIN); the exchange is invalid until psgd_ipc_close");
    if (step < 0 || step >= 0xffffffffLL) return fail(PSGD_ERR_VALUE, "step out of range (epochs are 32-bit)");
    if (reinterpret_cast<uintptr_t>(out) % 16) return fail(PSGD_ERR_LAYOUT, "output buffer must be 16-byte aligned");
    const bool has_flat = f && f->total > 0;
    if (has_flat) {
        if (!unc || !flat_out) return fail(PSGD_ERR_VALUE, "null argument");
        if (!f->bound) return fail(PSGD_ERR_STATE, "flat plan is not bound");
        if (f->dtype != PSGD_F32) return fail(PSGD_ERR_DTYPE, "psgd_aggregate_ipc packs fp32 uncompressed tensors");
        if (f->total > p->ipc_flat_cap) return fail(PSGD_ERR_VALUE, "flat tensors exceed the exchange buffer (psgd_ipc_create)");
    }
    DevScope scope(p->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int world = p->ipc_world;
    const int last = p->iters - 1;
    static const uint32_t spin = uint32_t(std::min<int64_t>(env_int("PSGD_IPC_SPIN", int64_t(1) << 26), 0xffffffffLL));
    // x / W into this rank's last slot: inside the first even product's launch when the step
    // starts even, else its own launch
    FlatArgs fa{};
    const bool fold = has_flat && p->even(step, 0);
    float* flat_slot = p->xslot(step, last) + p->ipc_flat_off;
    if (has_flat) {
        if (int st = flat_args(f, unc, flat_slot, world, s, &fa)) return st;
        if (!fold) PSGD_HIP(launch_flat_pack(f->dtype, fa, s));
    }
    // rank 1: the joint group norm of every summed factor is folded as at world size 1 (no
    // k_orth_reg launch): k_xchg leaves per-item sums of squares and a raw copy (history slot 2)
    // that the next iteration's kernels normalise on the fly
    const bool nfold = p->rbucket == 1 && env_int("PSGD_IPC_NORM_FOLD", 1) != 0;
    // ranks 2/4, two iterations (every step starts even): the Q orthonormalisation from the
    // exchange's Gram partials of the summed Q (k_orth_chain instead of k_orth_chol)
    const bool gfold = p->qfold_ok && p->iters == 2 && p->even(step, 0) && env_int("PSGD_IPC_GRAM_FOLD", 1) != 0;
    for (int it = 0; it < p->iters; ++it) {
        p->xout_now = p->xslot(step, it);
        p->raw_slot = 2;
        p->xgram_now = gfold;
        const int st = compress_impl(p, grads, step, it, s, nfold, false, fold ? &fa : nullptr);
        p->xout_now = nullptr;
        p->raw_slot = 1;
        p->xgram_now = false;
        if (st) return st;
        const bool e = p->even(step, it);
        XchgArgs xa{};
        if (nfold && it + 1 < p->iters) {
            xa.items = p->dev<RedItem>(e ? p->o_red_even : p->o_red_odd);
            xa.nitems = int32_t(e ? p->red_even.size() : p->red_odd.size());
            xa.mats = p->dev<MatDesc>(p->o_mats);
            xa.even = e ? 1 : 0;
            xa.dst2 = p->hist(2, it);
            xa.ss_out = p->dev<float>(p->o_ss) + size_t(it & 1) * p->ss_stride;
        }
        if (gfold && it == 0) {  // even: the Q side; k_orth_chain of iteration 1 reads the Gram
            xa.items = p->dev<RedItem>(p->o_red_even);
            xa.nitems = int32_t(p->red_even.size());
            xa.mats = p->dev<MatDesc>(p->o_mats);
            xa.even = 1;
            xa.dst2 = p->hist(2, it);
            xa.gram = p->dev<double>(p->o_gram);
            xa.gram_r = p->rbucket;
        }
        xa.peers = p->dev<const char* const>(p->o_ipc_ptrs);
        xa.own_flag = reinterpret_cast<uint64_t*>(p->ipc_buf) + it;
        xa.flag_off = int64_t(it) * int64_t(sizeof(uint64_t));
        xa.slot_off = p->xslot_off(step, it);
        xa.dst = e ? p->Q : p->P;
        xa.n = e ? p->qtot : p->ptot;
        if (it == last && has_flat) {
            xa.flat_dst = static_cast<float*>(flat_out);
            xa.flat_off = p->ipc_flat_off;
            xa.nflat = f->total;
        }
        xa.epoch = uint64_t(step) + 1;
        xa.nonces = p->dev<const uint32_t>(p->o_ipc_nonce);
        xa.own_nonce = p->ipc_nonce;
        xa.spin_limit = spin;
        xa.world = world;
        xa.rank = p->ipc_rank;
        xa.err = p->xerr_dev;
        xa.err_dev = reinterpret_cast<int32_t*>(static_cast<char*>(p->ipc_buf) + kXchgErrOff);
        PSGD_HIP(launch_xchg(xa, s));
    }
    return decompress_impl(p, grads, out, step, world, s, false);
}

}  // extern "C"
