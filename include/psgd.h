/*
 * psgd.h — C ABI of the MI355X-native PowerSGD codec (libpsgd.so).
 *
 * Drop-in boundary for the hot path of epfml/powersgd. Every entry point names the
 * reference interface it replaces (paths relative to the reference repository):
 *
 *   psgd_should_compress   powersgd/powersgd.py:101-105 (+ avg_compressed_size :292-294)
 *   psgd_plan_create       BasicPowerSGD.__init__       powersgd/powersgd.py:114-144, :253-263
 *   psgd_plan_* queries    _ps_buffer/_qs_buffer layout :130-144, compression_rate :265-275
 *   psgd_compress          one power iteration          powersgd/powersgd.py:172-202
 *                          (orthogonalize :188 -> orthogonalization.py:4-8; bmm :189-193;
 *                           local error-feedback update :195-202)
 *   psgd_decompress        approximation + un-batching  powersgd/powersgd.py:211-230
 *   psgd_plan_fused_final  (which final-pass form a step takes; no reference counterpart)
 *   psgd_*_bucket          the same per bucket of shape groups, for comm/compute overlap of the
 *                          factor all-reduce (powersgd.py:204-209 split into slices)
 *   psgd_aggregate         BasicPowerSGD.aggregate      powersgd/powersgd.py:146-235 (world size 1)
 *   psgd_flat_*            AllReduce.aggregate          powersgd/powersgd.py:22-31,
 *                          pack / allreduce_average      powersgd/utils.py:6-10, :43-49
 *   psgd_aggregate_flat    PowerSGD.aggregate           powersgd/powersgd.py:64-74 (world size 1)
 *   psgd_aggregate_comm    PowerSGD.aggregate at world size W over RCCL (:64-74, :204-209)
 *   psgd_aggregate_ipc     the same over IPC exchange buffers with device-side flags (one node)
 *   psgd_runs_*            DDP comm-hook plumbing: a DDP bucket's flat buffer
 *                          <-> the per-parameter tensors, by a run table; the error-feedback add
 *                          the reference gets from autograd's accumulation into p.grad
 *                          (README.md:39-42, powersgd/__init__.py:24-25) and the per-bucket
 *                          gather of the averaged gradients (paper-code/train_pytorch.py:106-131)
 *
 * Conventions
 *  - No torch types. Device buffers are plain pointers on the plan's device; `stream` is a
 *    hipStream_t passed as void*. All compute calls are stream-ordered and asynchronous, do no
 *    device allocation and no host synchronisation (except a one-off pointer-table upload when
 *    the set of gradient pointers changes).
 *  - Ownership: the caller owns gradients, outputs, the P/Q state buffers and the workspace;
 *    the plan owns host-side layout only.
 *  - Gradients are mutated in place into the error-feedback residual (reference :230).
 *  - P/Q factors are fp32 for fp32/bf16 gradients and fp64 for fp64 gradients (reference
 *    :241-251 allocates them in the default dtype, which must match the gradients' for its bmm).
 *  - The building blocks (psgd_product / psgd_orthogonalize / psgd_reconstruct) and the fused
 *    fp32 kernels take fp32/bf16 plans only (PSGD_ERR_DTYPE for an F64 plan).
 *  - Errors: every call returns a psgd_status; psgd_last_error() returns a thread-local message.
 *    PSGD_ERR_INDEX mirrors the reference's IndexError (no tensors, :118), PSGD_ERR_DTYPE its
 *    RuntimeError on unsupported dtypes (:189), PSGD_ERR_LAYOUT its RuntimeError on
 *    non-viewable tensors (:289).
 *  - Not re-entrant per plan; one plan per device/process (reference: single-threaded, :146).
 *  - Stream order: the calls of one plan must be ordered on ONE stream (as torch's current
 *    stream orders them). The plan's device pointer tables are re-uploaded on the launch stream
 *    when the gradient pointer set changes; a kernel of an earlier call still running on another
 *    stream could read a slot being rewritten.
 */
#ifndef PSGD_H
#define PSGD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct psgd_plan psgd_plan;
typedef struct psgd_flat psgd_flat;
typedef struct psgd_comm psgd_comm;
typedef struct psgd_runs psgd_runs;

enum psgd_status {
    PSGD_OK = 0,
    PSGD_ERR_INDEX = 1,   /* empty tensor list (reference IndexError)              */
    PSGD_ERR_VALUE = 2,   /* invalid argument (rank < 1, iterations out of range…) */
    PSGD_ERR_DTYPE = 3,   /* unsupported dtype                                      */
    PSGD_ERR_LAYOUT = 4,  /* unsupported layout / empty tensor                      */
    PSGD_ERR_DEVICE = 5,  /* HIP runtime error                                      */
    PSGD_ERR_STATE = 6    /* call order error (e.g. compute before psgd_plan_bind)  */
};

/* Gradient dtypes. F32 / BF16: factors (P/Q state) and arithmetic fp32. F64: the reference's
 * own test dtype (tests/powersgd_test.py:38): factors and arithmetic fp64, as the reference's
 * default-dtype P/Q (powersgd.py:241-251) are then. */
enum psgd_dtype { PSGD_F32 = 0, PSGD_BF16 = 1, PSGD_F64 = 2 };

/* Largest num_iters_per_step a plan accepts. */
#define PSGD_MAX_ITERS 16

int psgd_version(void);
const char* psgd_last_error(void);

/* Compression policy: numel / (0.5*iters*min(rank,min(shape))*sum(shape)) > min_rate,
 * evaluated on the ORIGINAL tensor shape (reference powersgd.py:101-105, :292-294). */
int psgd_should_compress(const int64_t* shape, int32_t ndim, int32_t rank,
                         int32_t num_iters_per_step, double min_compression_rate,
                         int32_t* out_flag);

/* ---------------------------------------------------------------- codec plan ------ */
/* `dims` holds the concatenated shapes of the `num_tensors` compressed tensors
 * (ndims[i] entries each). Matrices are the view [shape[0], numel/shape[0]]; they are
 * grouped by matrix shape in first-appearance order, and the P (resp. Q) state buffer
 * is the concatenation over groups of [count, n, r] (resp. [count, m, r]) fp32 arrays,
 * r = min(rank, n, m) — byte-for-byte the reference's _ps_buffer/_qs_buffer layout. */
int psgd_plan_create(const int64_t* dims, const int32_t* ndims, int32_t num_tensors,
                     int32_t rank, int32_t num_iters_per_step, int32_t dtype,
                     psgd_plan** out_plan);
int psgd_plan_destroy(psgd_plan* plan);

int psgd_plan_num_groups(const psgd_plan* plan, int32_t* out);
int psgd_plan_group(const psgd_plan* plan, int32_t g, int64_t* n, int64_t* m, int32_t* r,
                    int32_t* count);
int psgd_plan_factor_numel(const psgd_plan* plan, int64_t* p_numel, int64_t* q_numel);
/* Element offset of compressed tensor i inside the flat output buffer, and the total
 * number of elements that buffer needs. The layout is dense in tensor order (torch.cat). */
int psgd_plan_output_offset(const psgd_plan* plan, int32_t i, int64_t* offset);
int psgd_plan_output_numel(const psgd_plan* plan, int64_t* numel);
int psgd_plan_workspace_bytes(const psgd_plan* plan, int64_t* bytes);
/* reference compression_rate / uncompressed_num_floats / compressed_num_floats (:265-275) */
int psgd_plan_compression_rate(const psgd_plan* plan, double* rate, double* uncompressed,
                               double* compressed);

/* Bind caller-owned device memory: P state [p_numel] and Q state [q_numel] (fp32, or fp64
 * for a PSGD_F64 plan) and a workspace of psgd_plan_workspace_bytes() bytes (16-byte
 * aligned). Uploads the static layout tables (synchronous; call once). */
int psgd_plan_bind(psgd_plan* plan, int32_t device, void* p_state, void* q_state,
                   void* workspace);

/* Which state buffer iteration `it` of step `step` produces (and the caller must SUM-
 * all-reduce before the next call when world size > 1): 0 = Q (even), 1 = P (odd).
 * Parity = (step*num_iters_per_step + it) % 2 (reference :174). */
int psgd_out_factor(const psgd_plan* plan, int64_t step, int32_t it, int32_t* which);

/* One power iteration on every compressed matrix: orthonormalise the in-factor (rank 1:
 * one joint norm per shape group; rank > 1: Householder QR per matrix), then the
 * tall-skinny product with the error-feedback matrix G_it = G_0 - sum_{j<it} P_j Q_j^T
 * (formed on the fly). Leaves the LOCAL factor in the out-factor state buffer.
 * `grads[i]` = device pointer of compressed tensor i (contiguous).
 * Gradients are not written, EXCEPT by the last iteration of a step for which
 * psgd_plan_fused_final() reports 1: that iteration (odd, P = G X) is fused with the
 * final pass and leaves the error-feedback residual in `grads` (reference :195-202, :230);
 * psgd_decompress then only writes the output. */
int psgd_compress(psgd_plan* plan, void* const* grads, int64_t step, int32_t it, void* stream);

/* Fused final pass: grads[i] <- G_0 - sum_k P_k Q_k^T (local factors) and
 * out[i] <- (1/world_size) * sum_k P_k Qbar_k^T (all-reduced factors); `out` is the flat
 * output buffer (psgd_plan_output_offset). Call after the last psgd_compress (and its
 * all-reduce). */
int psgd_decompress(psgd_plan* plan, void* const* grads, void* out, int64_t step,
                    int32_t world_size, void* stream);

/* ------------------------------------------- buckets: comm/compute overlap (W > 1) ------ */
/* The reference all-reduces the whole out-factor buffer once per iteration (powersgd.py:
 * 204-209). With buckets, the shape groups are cut into `nbuckets` consecutive ranges
 * (group_end[b] = exclusive end group; the last must be psgd_plan_num_groups) and every launch of
 * an iteration can be issued per bucket: the caller all-reduces bucket b's slice of the factor
 * buffer (psgd_plan_bucket_range: element offset/length in the P and Q state buffers) as soon
 * as bucket b's kernels are queued, so that collective overlaps the next buckets' kernels. The
 * element-wise SUM over the slices equals the whole-buffer SUM. nbuckets = 0: one bucket (the
 * whole plan); at most 8 buckets. Synchronous (rewrites the tile tables): call between steps.
 * fp32/bf16 plans. */
int psgd_plan_set_buckets(psgd_plan* plan, int32_t nbuckets, const int32_t* group_end);
int psgd_plan_bucket_range(const psgd_plan* plan, int32_t bucket, int64_t* p_off, int64_t* p_len,
                           int64_t* q_off, int64_t* q_len);
/* psgd_compress / psgd_decompress restricted to one bucket's matrices (same semantics). */
int psgd_compress_bucket(psgd_plan* plan, void* const* grads, int64_t step, int32_t it, int32_t bucket,
                         void* stream);
int psgd_decompress_bucket(psgd_plan* plan, void* const* grads, void* out, int64_t step,
                           int32_t world_size, int32_t bucket, void* stream);

/* ------------------------- one-shot all-reduce over IPC, stream-ordered (W > 1, one node) ------ */
/* PowerSGD.aggregate at world size W (reference powersgd.py:64-74 with is_distributed(); the
 * factor all-reduce :204-209 and the uncompressed tensors' allreduce_average, utils.py:43-49)
 * without a collective library: one process per GPU, every rank reads all ranks' local factors
 * directly through IPC mappings (xGMI between GPUs) and sums them in rank order, so every rank
 * holds bitwise the same sum. Synchronisation is device-side: per iteration a kernel raises this
 * rank's epoch flag in its exchange buffer and polls the peers' flags (system scope, bounded: a
 * peer that never arrives sets the status word read by psgd_ipc_status instead of hanging).
 * No host barrier and no host synchronisation per step.
 * Exchange buffers are regions of a per-process, per-device arena that is allocated once and
 * never freed; every peer arena chunk is mapped once per process and never unmapped. A later
 * session of the same size gets the same region back: no free / malloc / re-map cycle between
 * sessions (a remapped, freed allocation can never alias a new session's buffer).
 *   psgd_ipc_create   takes this rank's exchange region (flags + two parities x iterations
 *                     slots, room for flat_numel uncompressed values), zeroes it, draws a fresh
 *                     session nonce into its header and exports arena handle + region offset +
 *                     nonce (psgd_ipc_handle_bytes bytes, the nonce last). Synchronous. Allowed
 *                     again after psgd_ipc_close (a new session on the same plan).
 *   psgd_ipc_open     the caller all-gathers the W handles (e.g. torch.distributed) and passes
 *                     them in rank order; maps each peer's arena chunk (first session only) and
 *                     reads each peer's nonce through the mapping: a mapping that does not reach
 *                     that session's region is PSGD_ERR_STATE, a list whose own entry is not this
 *                     rank's handle PSGD_ERR_VALUE. Every epoch flag carries its writer's nonce
 *                     in the high 32 bits and pollers accept only the nonce they opened with.
 *   psgd_aggregate_ipc the whole step on `stream` (same arguments as psgd_aggregate_comm).
 *   psgd_ipc_status   synchronous: 1 if a wait timed out since the last call (results invalid).
 *   psgd_ipc_close    synchronous: ends the session (mappings stay with the process). Teardown
 *                     is collective: every rank calls it, then the caller runs a cross-rank
 *                     barrier before any rank starts a new session or destroys the plan (its
 *                     region returns to the arena and a later session re-zeroes it).
 *   psgd_ipc_debug    diagnostics (tests): this process's arena counters, this session's region
 *                     address and nonce, and for peer w (open sessions) the mapped address and
 *                     the nonce read through the mapping. */
int psgd_ipc_handle_bytes(int64_t* bytes);
int psgd_ipc_create(psgd_plan* plan, int64_t flat_numel, void* handle_out);
int psgd_ipc_open(psgd_plan* plan, int32_t world_size, int32_t rank, const void* handles);
int psgd_aggregate_ipc(psgd_plan* plan, void* const* grads, void* out, int64_t step, psgd_flat* flat,
                       void* const* unc, void* flat_out, void* stream);
int psgd_ipc_status(psgd_plan* plan, int32_t* timed_out);
int psgd_ipc_close(psgd_plan* plan);
typedef struct psgd_ipc_info {
    int64_t arena_allocs;     /* arena chunks this process allocated (hipMalloc) */
    int64_t arena_opens;      /* peer chunks this process mapped (hipIpcOpenMemHandle) */
    int64_t arena_reuses;     /* regions served from chunks allocated earlier */
    int64_t arena_frees;      /* chunks freed: always 0 */
    uint64_t own_va;          /* this session's region */
    uint64_t peer_va;         /* peer w's region as mapped here (0 when no session is open) */
    uint32_t own_nonce;
    uint32_t peer_nonce_seen; /* the nonce in peer w's region header, read through the mapping */
} psgd_ipc_info;
int psgd_ipc_debug(psgd_plan* plan, int32_t peer, psgd_ipc_info* info);

/* Whole BasicPowerSGD.aggregate step for world size 1. */
int psgd_aggregate(psgd_plan* plan, void* const* grads, void* out, int64_t step, void* stream);

/* Nonzero when the last iteration of `step` is odd and every matrix fits the fused final
 * pass (row-resident product + residual, psgd_final.cuh). aggregate = 0: the building-block
 * path (psgd_compress of that iteration then writes the residual); aggregate = 1:
 * psgd_aggregate, which also fuses two-iteration rank-1/2/4 plans in the projection form
 * (output G X X^T, exact for I = 2 at world size 1): *fused = 2 for that
 * form (k_final_proj; ranks 1/2/4), 1 for the K-term form (k_final_odd), 0 unfused. */
int psgd_plan_fused_final(const psgd_plan* plan, int64_t step, int32_t aggregate, int32_t* fused);
/* Nonzero when iteration `it` of `step` (odd, followed by an even one) runs as ONE gradient pass
 * with the next iteration's product inside psgd_aggregate (rank 1, world size 1, I >= 3). */
int psgd_plan_odd_even(const psgd_plan* plan, int64_t step, int32_t it, int32_t* on);

/* Kernel timing for benchmarks: when enabled, every final pass launched by psgd_aggregate
 * (k_apply, or the fused final odd kernel) and by psgd_decompress (k_apply) is bracketed by HIP events recorded on its own stream.
 * psgd_plan_timing_read waits for the recorded events, returns the summed kernel time (ms)
 * and the number of launches, and clears the record. */
int psgd_plan_set_timing(psgd_plan* plan, int32_t enable);
int psgd_plan_timing_read(psgd_plan* plan, double* total_ms, int32_t* launches);

/* ------------------------------- building blocks (paper-code reducer variants) ------ */
/* The reference repository's paper code (paper-code/gradient_reducers.py) runs PowerSGD as
 * RankKReducer (:665-788) and HalfRankKReducer (:794-936) with a different call order. These
 * entry points expose the codec's kernels as steps so that such variants run on the same
 * plan, layout and kernels (powersgd_amd/reducers.py):
 *
 * psgd_product: y = G_k^T x (odd = 0; x P-layout, y Q-layout) or G_k x (odd = 1; x Q-layout,
 *   y P-layout) for every compressed matrix, G_k = G_0 - sum_{j<nterms} term_p[j] term_q[j]^T
 *   formed on the fly; no orthonormalisation (torch.matmul(matrix, q) :750 / matrix.t() @ p
 *   :770). y must not alias x or a term. */
int psgd_product(psgd_plan* plan, void* const* grads, int32_t odd, const float* x, float* y,
                 int32_t nterms, const float* const* term_p, const float* const* term_q, void* stream);
/* In-place orthonormalisation of every panel of a P-layout (which = 1) or Q-layout (0)
 * buffer. mode 0: the reference codec's (orthogonalization.py:4-8: joint rank-1 norm per
 * shape group, Householder QR above); mode 1: the paper code's Gram-Schmidt per matrix,
 * col /= sqrt(sum col^2) + 1e-8 (gradient_reducers.py:945-956). */
int psgd_orthogonalize(psgd_plan* plan, int32_t which, float* buf, int32_t mode, void* stream);
/* resid_out[i] <- G_0 - sum_k term_p[k] term_q[k]^T (null resid_out: back into grads[i]) and
 * out[i] <- alpha * sum_k avg_p[k] avg_q[k]^T, for the compressed tensors i (per-tensor
 * destination pointers; reference mem.data[:] = tensor - out, out.data[:] = p q^T). */
int psgd_reconstruct(psgd_plan* plan, void* const* grads, void* const* resid_out, void* const* out,
                     int32_t nterms, const float* const* term_p, const float* const* term_q,
                     const float* const* avg_p, const float* const* avg_q, float alpha, void* stream);

/* ------------------------------------ multi-GPU step with RCCL on the caller's stream ------ */
/* One process per GPU (reference: torch.distributed default group, powersgd.py:204-209 and
 * utils.py:43-49). The library drives RCCL itself, on the same stream as its kernels, so a
 * whole world-size-W step is ONE call with no host synchronisation and no per-collective
 * round trip through the host language. RCCL is resolved at run time (dlopen; an already loaded
 * librccl, e.g. PyTorch's, is reused): no link-time dependency.
 *   psgd_comm_unique_id  on rank 0: the communicator id (psgd_comm_id_bytes bytes), which the
 *                        caller broadcasts to every rank (e.g. torch.distributed);
 *   psgd_comm_init       on every rank, collectively: a communicator of `world` ranks on `device`.
 * psgd_aggregate_comm: PowerSGD.aggregate at world size W (reference :64-74 with
 * is_distributed()): for every power iteration the codec kernels and an in-place SUM all-reduce
 * of the out-factor state buffer (:204-209; the last iteration's collective grouped with the
 * SUM all-reduce of the uncompressed tensors packed /W into flat_out, utils.py:43-47), then the
 * output pass (alpha = 1/W). flat may be null (no uncompressed tensors). The whole plan is
 * one bucket here: a bucketed form (collectives on a second stream, event-ordered) was measured
 * host-enqueue-bound and removed. A poisoned communicator (an earlier failure)
 * is refused before anything is launched. */
int psgd_comm_id_bytes(int64_t* bytes);
int psgd_comm_unique_id(void* id_out);
int psgd_comm_init(int32_t world, int32_t rank, const void* id, int32_t device, psgd_comm** out);
int psgd_comm_destroy(psgd_comm* comm);
int psgd_aggregate_comm(psgd_plan* plan, void* const* grads, void* out, int64_t step, psgd_flat* flat,
                        void* const* unc, void* flat_out, psgd_comm* comm, void* stream);

/* ------------------------------------------ uncompressed tensors: flat average ------ */
/* AllReduce.aggregate minus the collective: flat[off_i + e] = x_i[e] / world_size (exact
 * copy when world_size == 1), then x_i[e] = 0. The caller SUM-all-reduces `flat` and
 * returns views of it (reference powersgd.py:22-31). Offsets are dense (torch.cat). */
int psgd_flat_create(const int64_t* numels, int32_t count, int32_t dtype, psgd_flat** out);
int psgd_flat_destroy(psgd_flat* flat);
int psgd_flat_workspace_bytes(const psgd_flat* flat, int64_t* bytes);
int psgd_flat_bind(psgd_flat* flat, int32_t device, void* workspace);
int psgd_flat_pack(psgd_flat* flat, void* const* tensors, void* flat_out, int32_t world_size,
                   void* stream);

/* PowerSGD.aggregate at world size 1 in one call (reference powersgd.py:64-74): the codec
 * step of psgd_aggregate on the compressed tensors `grads`, and the flat pack of the
 * uncompressed tensors `unc` into `flat_out` (psgd_flat_pack with world size 1) folded into
 * the codec's final-pass launch as extra workgroups (no launch of its own). Falls back to
 * two separate calls when the flat plan's dtype or device differs from the codec's. */
int psgd_aggregate_flat(psgd_plan* plan, void* const* grads, void* out, int64_t step, psgd_flat* flat,
                        void* const* unc, void* flat_out, void* stream);

/* ------------------------------------------ DDP bucket <-> parameter tensors ------ */
/* A run table maps a DDP bucket's flat buffer onto per-parameter tensors: run k covers
 * len[k] elements, bucket[bucket_off[k] + e] <-> tensors[tensor[k]][tensor_off[k] + e]. 64-bit
 * offsets throughout (no limit on the model's element count). `tensors` at call time is a host
 * array of ntensors device pointers (uploaded on the stream when it changes, like the codec's
 * gradient tables). psgd_runs_add: tensors += bucket (the error-feedback add, in the tensors'
 * dtype: fp32 / bf16 round to nearest even / fp64); psgd_runs_gather: bucket = tensors.
 * Runs must not overlap in the tensors (add) or in the bucket (gather). */
int psgd_runs_create(const int64_t* bucket_off, const int32_t* tensor, const int64_t* tensor_off,
                     const int64_t* len, int32_t nruns, int32_t ntensors, int32_t dtype, psgd_runs** out);
int psgd_runs_destroy(psgd_runs* runs);
int psgd_runs_workspace_bytes(const psgd_runs* runs, int64_t* bytes);
int psgd_runs_bind(psgd_runs* runs, int32_t device, void* workspace);
int psgd_runs_add(psgd_runs* runs, const void* bucket, void* const* tensors, void* stream);
int psgd_runs_gather(psgd_runs* runs, void* bucket, void* const* tensors, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PSGD_H */
