// Internal layout shared by the host plan (psgd_plan.cpp) and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <stdint.h>

struct psgd_comm;  // include/psgd.h (psgd_comm.cpp)

namespace psgd {

// host side of the RCCL communicator (psgd_comm.cpp): the error message goes to
// psgd_last_error (comm_fail, psgd_plan.cpp); comm_allreduce = a grouped in-place SUM of one or
// two fp32 buffers, stream-ordered on s
int comm_fail(int code, const char* msg);
int comm_world(const psgd_comm* c);
int comm_allreduce(psgd_comm* c, float* buf, size_t n, float* buf2, size_t n2, hipStream_t s);
void comm_poison(psgd_comm* c, const char* why);  // every later comm_allreduce fails (PSGD_ERR_STATE)
bool comm_poisoned(const psgd_comm* c, std::string* why);  // checked before a step launches anything

// Benchmark timing of the final pass (psgd_plan_set_timing): while set, the final-pass launch
// records these events from its own dispatch packet (hipExtLaunchKernel), so the measured span
// is the kernel alone, without the marker packets of separate hipEventRecord calls.
struct KernelTiming {
    hipEvent_t start, stop;
};
extern thread_local const KernelTiming* g_kernel_timing;

constexpr int kMaxTerms = 16;   // == PSGD_MAX_ITERS
constexpr int kBlock = 256;     // threads per workgroup for the streaming kernels
constexpr int kWaves = kBlock / 64;

// One compressed matrix (the [n, m] view of a tensor). Stored in GROUP order, so the
// P/Q offsets below are monotone and reproduce the reference's _ps/_qs_buffer layout.
struct MatDesc {
    int64_t n, m;
    int64_t poff, qoff;     // offsets (floats) of this matrix's P [n,r] / Q [m,r] panels
    int64_t out_off;        // element offset in the flat output buffer
    int64_t part_even;      // column partials [nchunk][m][r] (even iterations)
    int64_t part_odd;       // row partials    [nstrip][n][r] (odd iterations)
    int32_t r;
    int32_t tensor;         // index into the gradient pointer table
    int32_t group;
    int32_t vec;            // 1: 4-element vector loads/stores (m % 4 == 0, aligned)
    int32_t lanes;          // L: lanes sharing one row inside a wave (power of two <= 64)
    int32_t nstrip;         // column strips of L*V columns
    int32_t nchunk;         // row chunks
    int32_t chunk_rows;     // rows per chunk (multiple of the block's rows per pass)
    // odd iterations (P = G Q): MFMA tiles when odd_mfma, else the lane-column tiles above
    int32_t odd_mfma;
    int32_t odd_nstrip;     // column strips of the odd partials (reduce pass)
    int32_t odd_sw;         // MFMA strip width (columns, multiple of 16)
    int32_t odd_chunk_rows; // MFMA chunk rows (multiple of 16 * kWaves)
    // fused final odd iteration (k_final_odd): a row group of fin_T threads owns a row
    // (fin_S segments of 4*fin_T columns); a workgroup covers fin_rows rows in the projection
    // form, fin_rows_kt in the K-term form
    int32_t fin_T;
    int32_t fin_S;
    int32_t fin_rows;
    int32_t fin_rows_kt;
    // odd-even pass (k_final_oe, rank 1, world size 1): row block b (oe_rows rows, the K-term
    // row-group geometry) leaves its partial of the next even product at oe_part + b * m and its
    // sum of P^2 at oe_ss[oe_blk0 + b]
    int64_t oe_part;
    int32_t oe_blk0;
    int32_t oe_rows;
};

// Streaming tile: rows [chunk*chunk_rows, +chunk_rows) x columns of one strip.
struct Tile {
    int32_t mat, strip, chunk;
    int32_t tensor;  // fp32/bf16 streaming tiles: the matrix's gradient-table index (its pointer
                     // load goes out beside the MatDesc load instead of after it)
};

// Even-product work unit of the persistent k_even (psgd_even.cuh): rows [row0, row1) of one
// column strip (L lanes x V columns) of one matrix. Workgroup w walks segments
// [wg_seg[w], wg_seg[w + 1]) in order; segment boundaries split the plan (or a bucket of it)
// into equal gradient byte ranges, one per workgroup, so a strip is cut only where a
// workgroup's range ends: its column partials are few (one per segment, not one per small tile).
// The matrix fields the pass needs are copied in, so a segment start is one descriptor load
// and one gradient-pointer load (no MatDesc round trip in between).
struct Seg {
    int64_t m;           // columns of the matrix
    int64_t poff, qoff;  // its P / Q panel offsets (floats)
    int64_t part;        // float offset of this segment's partials [strip columns][r] in the workspace
    int32_t row0, row1, strip;
    int32_t tensor;      // gradient-table index of the matrix
    int32_t ss;          // rank-1 norm fold: sum-of-squares slot of a strip-0 segment, else -1
    int32_t r, lanes;
    int32_t vec;         // 0: scalar columns; 1: 4-column vectors; 2: full-width strip fast path
                         // (64 lanes x 4 columns, r == the plan's rank bucket, < 2^31 bytes)
};

// Reduction item for the partial-sum pass: up to 64 * per consecutive factor elements of one
// matrix that share their partial layout: partial k of element start + j lies at
// pbase + k * pstride + j (even: one column strip's segments; odd: the matrix's strips).
constexpr int kRedElems = 64;  // fp64 plans: factor elements per reduction item (one per lane)
constexpr int kRedItem = 256;  // fp32/bf16 plans: at most this many factor elements per reduction item
constexpr int kRedWide = 64;   // ... when an element has at most this many partials (else 64)

struct RedItem {
    int32_t mat, start;
    int32_t per;     // fp32/bf16 plans: elements per lane (4: 256-element item; 1: 64 elements,
                     // for factors with many partials, where 4 per lane is one CU's bandwidth)
    int32_t cnt;     // elements in the item (<= 64 * per)
    int64_t pbase;   // partial 0 of element `start` (floats from the partial workspace)
    int32_t pstride; // floats between consecutive partials of one element
    int32_t np;      // partials per element
};

// Orthonormalisation unit: rank 1 -> one shape GROUP (joint norm over count*k values);
// rank > 1 -> one matrix (Householder QR of a k x r panel).
struct OrthUnit {
    int64_t off;    // offset (floats) in the P- or Q-layout buffer
    int64_t k;      // rows of each panel
    int32_t r;
    int32_t count;  // panels in the unit (group size for rank 1, 1 otherwise)
};

// A list of rank-r terms  P_k Q_k^T : P-layout [n,r] and Q-layout [m,r] panel buffers.
struct Terms {
    const float* p[kMaxTerms];
    const float* q[kMaxTerms];
};

struct FlatEntry {
    int64_t off, numel;  // dense offset in the flat buffer (non-empty tensors only)
    int64_t tensor;      // index into the pointer table
    int64_t pad;
};

// Flat-pack work item: kFlatItem consecutive elements of one entry.
constexpr int kFlatItem = 8 * kBlock;
struct FlatItem {
    int32_t entry, pad;
    int64_t start;
};

struct FlatArgs {
    const FlatEntry* entries;
    const FlatItem* items;
    void* const* tensors;
    void* flat;
    int32_t nitems;
    int32_t world;
};

struct ProductArgs {
    const MatDesc* mats;
    const Tile* tiles;
    void* const* grads;
    const float* x;      // orthonormal in-factor: P-layout (even) / Q-layout (odd)
    float* part;         // partial-sum workspace
    Terms res;           // error-feedback terms applied on the fly
    int32_t nres;
    // rank-1 iteration 0 with the norm folded (even product on the RAW state P): strip-0
    // segments write sum_rows P^2 of their rows to ss0[seg.ss]
    float* ss0;
    // even product (k_even): segments and per-workgroup [begin, end) (wg_seg[blockIdx],
    // wg_seg[blockIdx + 1]) of its nwg workgroups; workgroups nwg .. nwg + flat.nitems - 1 pack
    // the uncompressed tensors (world size > 1: the first iteration's launch carries them)
    const Seg* segs;
    const int32_t* wg_seg;
    int32_t nwg;
    FlatArgs flat;
    // diagnostic builds only (-DPSGD_EVEN_STAMPS, tools/even_stamps.py): per workgroup of k_even
    // kEvenStamps 64-bit words (s_memrealtime at entry and after each segment, the XCC / HW ids)
    unsigned long long* stamps;
};
constexpr int kEvenStamps = 8;

struct ApplyArgs {
    const MatDesc* mats;
    const Tile* tiles;
    void* const* grads;  // in: G_0, out: residual
    void* out;           // flat output buffer
    Terms res;           // local terms (residual)
    Terms apx;           // all-reduced terms (approximation), scaled by alpha
    int32_t nterms;
    float alpha;         // 1 / world_size
    // blocks [0, flat.nitems) pack the uncompressed tensors (AllReduce at world size 1)
    // inside the same launch; the ntiles tiles follow
    int32_t ntiles;
    FlatArgs flat;
    // optional destination tables (device arrays of per-tensor pointers): the residual goes
    // to rdst[i] instead of back into grads[i], the output to odst[i] instead of the flat
    // buffer (psgd_reconstruct)
    void* const* rdst;
    void* const* odst;
    int32_t out_nt;      // world size 1 (shared terms): output stores nt only (large plans, as the
                         // fused final pass's FinalArgs::out_nt), a separate kernel instance
};

struct ReduceArgs {
    const MatDesc* mats;
    const RedItem* items;
    const float* part;
    float* yloc;         // history copy of the local factor
    float* state;        // reference-visible state buffer (the out-factor)
    int32_t even;
    int32_t nmain;       // items[0, nmain) reduce the out-factor
    // Rank-1 fused normalisation (world size 1, iteration >= 1): the product ran on the RAW
    // in-factor `raw` (the previous iteration's reduced out-factor); its group norm comes
    // from the previous reduction's sum-of-squares partials `ss_in` (per item, group g's
    // items are grng_in[g] = [begin, end)). The reduction divides by it, and the extra
    // items nitems[0, nnorm) write the normalised in-factor to `xstate` and `hx`.
    const float* ss_in;
    const int32_t* grng_in;
    const RedItem* nitems;
    int32_t nnorm;
    const float* raw;
    float* xstate;
    float* hx;
    float* ss_out;       // per-item sum of squares of this reduction's output (or null)
    // Folded orthonormalisation (projection form, k_orth_chain): per item the upper Gram of
    // its output rows (kGramStride fp64 entries, rank gram_r in {2, 4}), or null
    double* gram;
    int32_t gram_r;
    float* xout;         // one-shot exchange (psgd_aggregate_ipc): the local factor also goes to
                         // this rank's exchange slot (same offsets as `state`), or null
};

constexpr int kGramStride = 10;  // fp64 Gram entries per reduction item (rank <= 4)

// k_orth_chain: Cholesky-QR of each Q panel from the reduction's Gram partials (no Gram pass
// over the panel), the panel rows split over several workgroups that each run the r x r chain
// and apply X = raw M to their slice. Fallback panels (ill-conditioned, unreflected columns):
// the slice-0 workgroup runs the exact Householder recursion on the whole panel.
struct ChainArgs {
    const OrthUnit* units;
    const int32_t* uitems;  // per unit: [begin, end) of its reduction items
    const double* gram;     // kGramStride per item
    const float* raw;       // Q layout: the reduced (raw) factor
    float* state;           // Q state: X
    float* hx;              // X history
    float* rfac;            // Q layout: R' (r x r) at each unit's offset
};

// Fused LAST iteration when it is odd (P = G_k X): a row group holds whole rows in
// registers, so the reduction over columns completes inside the workgroup and the same
// registers produce the residual (and, at world size 1, the output) without re-reading G.
struct FinalArgs {
    const MatDesc* mats;
    const Tile* tiles;    // (mat, 0, row block)
    void* const* grads;   // in: G_0, out: residual
    void* out;            // flat output (written when write_out)
    const float* x;       // in-factor, Q layout (orthonormal, or raw when ss_in is set)
    Terms res;            // local terms of the earlier iterations (also the output terms at W = 1)
    int32_t nres;
    int32_t write_out;    // world size 1: output = sum of all terms
    float* yloc;          // P local -> history
    float* state;         // P local -> reference-visible state buffer
    // rank-1 fused normalisation of the raw in-factor (as ReduceArgs)
    const float* ss_in;
    const int32_t* grng_in;
    float* xstate;
    float* hx;
    int32_t ntiles;       // row blocks; flat pack items come first (as ApplyArgs)
    FlatArgs flat;
    // projection form (nres = kFinProj, see psgd_final.cuh): P_0 rows and R' per matrix
    const float* proj_p0;  // P layout
    const float* proj_r;   // Q layout: R' (r x r, row-major) at each matrix's qoff
    // rank-1 projection form: per matrix [begin, end) of the even reduction's sum-of-squares
    // items (ss_in), for ||Q_0,i||^2 of the matrix against the group norm
    const int32_t* mrng_in;
    float* xout;           // one-shot exchange: P local also to this rank's exchange slot, or null
    int32_t out_nt;        // output stores nt only (large plans), else write-through (psgd_stream.cuh)
    // odd-even pass (k_final_oe): no residual / output stores; per row block the next (even)
    // iteration's raw product sum_rows (g - P x^T) P and sum_rows P^2 (MatDesc::oe_part / oe_blk0)
    float* oe_part;
    float* oe_ss;
};
hipError_t launch_final_oe(int dtype, int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s, int* waves);
// nres value selecting the projection form of the fused final pass (I = 2, world size 1)
constexpr int kFinProj = 1000;
// rows per row block of the register-panel final pass (the projection form stages a block's
// P_0 rows in LDS)
constexpr int kFinRowsMax = 256;

struct OrthArgs {
    const OrthUnit* units;
    float* state;        // in-factor state buffer, orthonormalised in place
    float* hx;           // history copy of the orthonormal in-factor
    float* save;         // if non-null: copy of the pre-orthonormalisation values
    int32_t flags;       // diagnostics (PSGD_ORTH_DIAG): 1 = skip the Householder fallback
    // if non-null (Cholesky-QR kernels k_orth_chol<R>): the QR factor R' of each panel,
    // input panel = orthonormal output x R' (upper triangular r x r, row-major, written at the
    // unit's offset; rank-1 units: the joint-norm divisor at every panel's offset)
    float* rfac;
};

// ------------------------------------------------------------------ fp64 gradients
// The reference's own error-feedback test runs in float64 (tests/powersgd_test.py:38); its P/Q
// then follow the default dtype (powersgd.py:241-251), so gradients, factors and arithmetic are
// all fp64 (psgd_f64.hip). Same plan layout (MatDesc, OrthUnit, P/Q offsets) as fp32.
constexpr int kF64Cols = 64;    // even product: columns per tile (one per lane)
constexpr int kF64Rows = 256;   // even product: rows per chunk (partials per chunk)
constexpr int kF64OddRows = 16; // odd product: rows per workgroup (4 per wave)

struct TermsF64 {
    const double* p[kMaxTerms];
    const double* q[kMaxTerms];
};

struct F64Args {
    const MatDesc* mats;
    const Tile* tiles;
    void* const* grads;       // G_0 (in), residual (out, apply)
    const double* x;          // orthonormal in-factor (products)
    double* part;             // even partials [nchunk][m][r] per matrix at part_off[mat]
    const int64_t* part_off;
    double* y;                // out-factor state (reduce / odd product)
    double* yh;               // its history copy
    TermsF64 res;             // local terms (products: earlier iterations; apply: all)
    int32_t nres;
    TermsF64 apx;             // all-reduced terms (apply), scaled by alpha
    double alpha;
    void* out;                // flat output (apply)
    const RedItem* items;     // even reduction items
};

struct F64OrthArgs {
    const OrthUnit* units;
    double* state;            // in-factor, orthonormalised in place
    double* hx;               // history copy of the result
    double* save;             // if non-null: copy of the values before orthonormalisation
};

hipError_t launch_f64_product(bool even, int R, const F64Args& a, int ntiles, hipStream_t s);
hipError_t launch_f64_reduce(int R, const F64Args& a, int nitems, hipStream_t s);
hipError_t launch_f64_apply(int R, const F64Args& a, int ntiles, hipStream_t s);
hipError_t launch_f64_orth(int R, const F64OrthArgs& a, int nunits, hipStream_t s);

// Host-side launchers (psgd_kernels*.hip). Return hipError_t.
hipError_t launch_product(int dtype, int R, bool even, int nres, const ProductArgs& a,
                          int ntiles, hipStream_t s);
hipError_t launch_odd_mfma(int dtype, int R, int nres, const ProductArgs& a, int ntiles,
                           hipStream_t s);
hipError_t launch_apply(int dtype, int R, int nterms, bool shared, const ApplyArgs& a,
                        int ntiles, hipStream_t s);
// ntiles == 0: no launch, only the occupancy query (*waves = resident waves per SIMD)
hipError_t launch_final_odd(int dtype, int R, int nres, int smax, const FinalArgs& a, int ntiles,
                            hipStream_t s, int* waves = nullptr);
hipError_t launch_lowrank_out(int dtype, int R, int nterms, const ApplyArgs& a, int ntiles, hipStream_t s);
hipError_t launch_reduce(const ReduceArgs& a, int nitems, hipStream_t s);
hipError_t launch_orth(const OrthArgs& a, int nunits, int R, int64_t max_rows, bool chol, hipStream_t s);
hipError_t launch_orth_chain(const ChainArgs& a, int nunits, int64_t max_rows, int R, hipStream_t s);
// paper-code Gram-Schmidt (gradient_reducers.py:945-956) on one panel per unit, per matrix
hipError_t launch_orth_mgs(const OrthArgs& a, int nunits, int R, hipStream_t s);
hipError_t launch_flat_pack(int dtype, const FlatArgs& a, hipStream_t s);
hipError_t launch_flat_pack_f64(const FlatArgs& a, hipStream_t s);

// DDP bucket <-> parameter tensors (psgd_runs_*): one work item = up to kRunItem consecutive
// elements of one run; k_runs<ADD> adds the bucket into the tensors or gathers them into it.
constexpr int kRunItem = 16 * kBlock;
struct RunItem {
    int64_t boff, toff;  // element offsets in the bucket / in the tensor
    int32_t tensor, cnt; // tensor index, elements (<= kRunItem)
};
struct RunsArgs {
    const RunItem* items;
    void* bucket;
    void* const* tensors;
    int32_t nitems;
};
hipError_t launch_runs(int dtype, bool add, const RunsArgs& a, hipStream_t s);

// One-shot all-reduce over IPC-mapped exchange buffers (psgd_aggregate_ipc). Every rank's
// exchange buffer: kXchgHeader bytes of per-iteration epoch flags (uint64, one per iteration),
// then two parities x iterations slots of xchg_slot floats each; the producer kernels (k_reduce,
// k_final_odd, the flat pack) write the LOCAL factor into this rank's slot, and k_xchg raises
// this rank's flag, waits (bounded) for every peer's flag and sums the W slots in rank order.
constexpr int kMaxRanks = 64;
constexpr int64_t kXchgHeader = 256;
// byte offset, in the header, of the device copy of the sticky error word (XchgArgs::err_dev):
// past the flags of every iteration (num_iters_per_step <= kMaxTerms)
constexpr int64_t kXchgErrOff = 192;
// byte offset of this buffer's session nonce (uint32, written at psgd_ipc_create): peers check it
// through their mapping at psgd_ipc_open, and every epoch flag carries it in its high word, so a
// mapping that does not reach THIS session's buffer (a runtime that hands back a stale mapping
// of a freed buffer with an identical handle) fails loudly instead of summing stale slots
constexpr int64_t kXchgNonceOff = 200;
static_assert(kMaxTerms * 8 <= kXchgErrOff && kXchgErrOff + 4 <= kXchgNonceOff && kXchgNonceOff + 4 <= kXchgHeader,
              "exchange header layout");
struct XchgArgs {
    const char* const* peers;  // device array: the W exchange buffers (rank order, own included)
    uint64_t* own_flag;        // this rank's flag of this iteration (its own buffer)
    int64_t flag_off;          // byte offset of this iteration's flag in every buffer
    int64_t slot_off;          // byte offset of this step/iteration's slot in every buffer
    float* dst;                // SUM of the factors (the reference-visible state) ...
    int64_t n;                 // ... n floats
    float* flat_dst;           // SUM of the packed uncompressed tensors (last iteration) ...
    int64_t flat_off;          // ... at slot + flat_off floats
    int64_t nflat;
    uint64_t epoch;            // step + 1 (< 2^32)
    const uint32_t* nonces;    // device array: every rank's session nonce (flag = nonce << 32 | epoch)
    uint32_t own_nonce;
    uint32_t spin_limit;       // polls (~0.25 us apart) before a wait gives up
    int32_t world, rank;
    int32_t* err;              // set to 1 when a wait timed out (psgd_ipc_status; host-mapped)
    int32_t* err_dev;          // device copy of `err` (this rank's buffer header, kXchgErrOff):
                               // once set, later exchanges skip their waits and write NaN sums
    // rank-1 norm fold (non-last iterations): one workgroup per reduction item of this parity
    // (items, nitems, mats, even) writes the sum to dst and dst2 (the raw copy the next
    // iteration's kernels normalise on the fly) and the item's sum of squares to ss_out
    const RedItem* items;
    const MatDesc* mats;
    float* dst2;
    float* ss_out;
    int32_t nitems, even;
    // ranks 2/4, two iterations: the upper Gram of each item's rows of the SUMMED Q (fp64,
    // kGramStride per item) for k_orth_chain, as k_reduce leaves it at world size 1
    double* gram;
    int32_t gram_r;
};
hipError_t launch_xchg(const XchgArgs& a, hipStream_t s);

}  // namespace psgd
