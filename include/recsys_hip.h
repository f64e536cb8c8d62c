/*
 * recsys_hip.h — C-ABI of librecsys_hip.so, the MI355X (gfx950) sparse-embedding and
 * feature-interaction engine.
 *
 * Every entry point replaces one stock TensorFlow / Keras / DGL kernel that the reference
 * (neoyinyao/Recommender, read-only at /root/reference) reaches through its Keras layers.
 * The reference has no native code of its own; the citation on each function names the
 * reference call site whose semantics it reproduces.
 *
 * Conventions:
 *   - return value: int32 status, 0 = RS_OK, < 0 = RS_E_*; rs_last_error() gives a
 *     thread-local message for the last failing call on the calling thread.
 *   - every buffer is a caller-owned DEVICE pointer; the library never allocates
 *     persistent memory. Scratch comes from a caller workspace sized by the matching
 *     rs_*_workspace_size() query.
 *   - every call takes a hipStream_t (passed as void*) and is stream-ordered and
 *     asynchronous: no host synchronisation inside, graph-capturable.
 *   - stateless and re-entrant. RNG state (Philox key, counter) is passed explicitly.
 *   - float tensors are fp32 row-major; ids are int32 or int64 (RS_ID_I32 / RS_ID_I64).
 *   - out-of-range ids (TF-GPU semantics): the row reads as zeros, its gradient is
 *     dropped and *err_flag (device int32, may be NULL) gets bit RS_ERRBIT_OOB set.
 */
#ifndef RECSYS_HIP_H
#define RECSYS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_OK 0
#define RS_E_INVALID (-1)     /* bad argument (shape, dtype, null pointer) */
#define RS_E_OOB (-2)         /* reserved: host-side id range violation */
#define RS_E_HIP (-3)         /* a HIP runtime call failed */
#define RS_E_WORKSPACE (-4)   /* workspace smaller than rs_*_workspace_size() */
#define RS_E_UNSUPPORTED (-5) /* shape outside what the kernels handle */

#define RS_ID_I32 0
#define RS_ID_I64 1

#define RS_ERRBIT_OOB 1
#define RS_ERRBIT_FORMAT 2  /* a malformed input record (rs_tfrecord_parse_criteo) */
#define RS_ERRBIT_RANGE 4   /* a size past what the caller declared (rs_sort_ids_slots: a slot
                               with more rows than max_slot_rows allows; the output is not sorted) */

/* optimizer kinds for rs_embedding_apply */
#define RS_OPT_SGD 0        /* var[u] -= lr * g_u                         (ctr/train.py:77-79) */
#define RS_OPT_LAZY_ADAM 1  /* Adam on touched rows only                   (SURVEY §8a-2 b)   */
#define RS_OPT_KERAS_ADAM 2 /* Keras OptimizerV2 Adam, dense decay of m/v/var (ctr/train.py:80) */
#define RS_OPT_ADAGRAD 3    /* reserved */

typedef struct rs_adam_params {
  float lr;        /* SGD: learning rate. Adam: lr_t = lr*sqrt(1-b2^t)/(1-b1^t), host-computed fp32 */
  float beta1;
  float beta2;
  float one_minus_beta1;
  float one_minus_beta2;
  float epsilon;
} rs_adam_params;

const char* rs_last_error(void);
int32_t rs_version(void);
/* sha256 prefix of the kernel sources + this header the library was built from (the host-side
 * loader compares it with the sources it ships beside: a stale build is refused) */
const char* rs_build_id(void);
/* number of gfx950 devices visible; 0 when no GPU (used by loaders to fail loudly) */
int32_t rs_device_count(void);
/* STREAM-style device copy (16-byte accesses): the measured HBM-bandwidth reference of the
 * bench's roofline; bytes a multiple of 16, both buffers 16-byte aligned. */
int32_t rs_stream_copy(const void* src, void* dst, size_t bytes, void* stream);
/* Device-scope stream ordering (no reference counterpart: engine plumbing between its own
 * streams). An event created with hipEventDisableSystemFence: its record is a device-scope
 * release, so one stream can wait for another without the system-scope cache write-back a
 * default event's record performs. Same-device ordering only. rs_event_create returns NULL on
 * failure (rs_last_error says why). */
void* rs_event_create(void);
int32_t rs_event_destroy(void* ev);
int32_t rs_event_record(void* ev, void* stream);
int32_t rs_stream_wait_event(void* stream, void* ev);

/* ------------------------------------------------------------------------------------
 * a-1  Embedding forward (multi-slot gather).
 * Replaces keras.layers.Embedding.call → ResourceGather:
 *   ctr/model.py:19 (DeepFM), ctr/model.py:49 (DLRM), esmm/esmm.py:16, esmm/mmoe.py:20,
 *   esmm/base.py:15, dien/model.py:16-17, eges/model.py:32-33, pinsage/train/layers.py:63-79.
 * ids: [n_ids] flattened [B, n_slots] (slot = position % n_slots).
 * slot_offsets: NULL (one shared table, ctr/model.py:10) or [n_slots+1] row offsets of
 *   per-slot tables packed in one slab (row = slot_offsets[s] + id, valid while
 *   id < slot_offsets[s+1]-slot_offsets[s]).
 * out: [n_ids, dim]. */
int32_t rs_embedding_fwd(const float* table, int64_t n_rows, int32_t dim, const void* ids,
                         int32_t id_dtype, int64_t n_ids, const int64_t* slot_offsets,
                         int32_t n_slots, float* out, int32_t* err_flag, void* stream);
/* rs_embedding_fwd with the rows written at a row stride out_ld >= dim (floats): a column block
 * of a wider row-major output. DIEN's flat embedding item ‖ category (dien/model.py:14-19,
 * tf.concat of the two lookups) is two of these into one [n, 36] tensor, no concat pass. */
int32_t rs_embedding_fwd_strided(const float* table, int64_t n_rows, int32_t dim, const void* ids,
                                 int32_t id_dtype, int64_t n_ids, const int64_t* slot_offsets,
                                 int32_t n_slots, float* out, int64_t out_ld, int32_t* err_flag,
                                 void* stream);

/* ------------------------------------------------------------------------------------
 * a-2 (part 1) Duplicate-index coalescing: the IndexedSlices gradient's `unique` +
 * `unsorted_segment_sum` (Keras OptimizerV2 _deduplicate_indexed_slices, reached from
 * apply_gradients at ctr/train.py:97, dien/train.py:22, esmm/train.py:104).
 * Stable LSD radix sort of the global row of every id; outputs
 *   sorted_rows[n_ids] (uint32, ascending; an OOB id gets the sentinel n_rows, sorting last),
 *   sorted_pos[n_ids]  (int32 original position, ascending inside a run of equal rows),
 *   n_unique[1]        (device int32: number of distinct valid rows).
 * Deterministic: identical inputs give identical outputs. */
size_t rs_sort_ids_workspace_size(int64_t n_ids);
int32_t rs_sort_ids(const void* ids, int32_t id_dtype, int64_t n_ids, const int64_t* slot_offsets,
                    int32_t n_slots, int64_t n_rows, uint32_t* sorted_rows, int32_t* sorted_pos,
                    int32_t* n_unique, int32_t* err_flag, void* workspace, size_t ws_bytes,
                    void* stream);

/* Masked variant: positions with valid[i] == 0 are excluded — they take the sentinel key (sorted
 * last, no segment, no OOB flag). For lookups whose masked positions carry no gradient by
 * construction (DIEN's padded history steps: dien/model.py mask_zero, dien/layers.py GRU / AUGRU
 * / aux loss all skip them), so the segmented sums below see only the steps that exist. */
int32_t rs_sort_ids_masked(const void* ids, int32_t id_dtype, int64_t n_ids, const uint8_t* valid,
                           const int64_t* slot_offsets, int32_t n_slots, int64_t n_rows,
                           uint32_t* sorted_rows, int32_t* sorted_pos, int32_t* n_unique,
                           int32_t* err_flag, void* workspace, size_t ws_bytes, void* stream);

/* The stable (row, position) sort of n_runs equal runs of n_ids / n_runs int32 rows, each
 * ascending with its padding (ids < 0) at the end — the row-sharded slab's owner side, one run
 * per source rank: a merge by binary searches, one launch; the output equals rs_sort_ids_masked's
 * with the padding masked (entries past a run's valid prefix take the sentinel n_rows, in
 * position order; rows >= n_rows among them set RS_ERRBIT_OOB). */
int32_t rs_sort_ids_runs(const int32_t* ids, int64_t n_ids, int32_t n_runs, int64_t n_rows,
                         uint32_t* sorted_rows, int32_t* sorted_pos, int32_t* err_flag,
                         void* stream);
/* rs_sort_ids_masked (valid may be NULL) with the largest slot's row count given: when the ids
 * are [B, n_slots] (B <= 131072, n_slots <= 64), one GPU, and every slot has < 2^24 rows, the
 * sort runs slot by slot (the slot of position p is p % n_slots: the order over slots is free) in
 * <= 2 passes of <= 12-bit digits, 4 launches; otherwise the LSD sort. The output is the same.
 * rs_sort_ids / rs_sort_ids_masked take that path when n_rows <= 2^24.
 * Sentinel order (every sort here): excluded / OOB positions follow all valid rows, grouped by
 * slot, each group in position order; their sorted_rows value is n_rows (key space). */
int32_t rs_sort_ids_slots(const void* ids, int32_t id_dtype, int64_t n_ids, const uint8_t* valid,
                          const int64_t* slot_offsets, int32_t n_slots, int64_t n_rows,
                          int64_t max_slot_rows, uint32_t* sorted_rows, int32_t* sorted_pos,
                          int32_t* n_unique, int32_t* err_flag, void* workspace, size_t ws_bytes,
                          void* stream);

/* Row-sharded variant: rows dealt cyclically over `world` ranks
 * (owner = row % world, local row = row / world). Keys are owner-major:
 * key = owner * ceil(n_rows/world) + local row, so the sorted unique keys are grouped by owner
 * rank with the owner's local rows ascending; the OOB sentinel is world * ceil(n_rows/world).
 * world = 1 is rs_sort_ids. */
int32_t rs_sort_ids_sharded(const void* ids, int32_t id_dtype, int64_t n_ids,
                            const int64_t* slot_offsets, int32_t n_slots, int64_t n_rows,
                            int32_t world, uint32_t* sorted_keys, int32_t* sorted_pos,
                            int32_t* n_unique, int32_t* err_flag, void* workspace, size_t ws_bytes,
                            void* stream);
/* From sorted keys: uniq_keys[u] (ascending), inverse[p] = u of position p (-1 for an OOB id),
 * n_unique[1], and owner_counts[world] (unique keys per owner rank; may be NULL).
 * Workspace: rs_unique_inverse_workspace_size(n_ids) bytes; it begins with int32 [n_ids], the
 * exclusive scan of the head flags — each sorted key's segment (unique) index — which
 * rs_embedding_dedup_grad_mapped_range takes as seg_excl for the same sorted keys. */
size_t rs_unique_inverse_workspace_size(int64_t n_ids);
int32_t rs_unique_inverse(const uint32_t* sorted_keys, const int32_t* sorted_pos, int64_t n_ids,
                          int64_t n_rows, int32_t world, uint32_t* uniq_keys, int32_t* inverse,
                          int32_t* n_unique, int32_t* owner_counts, void* workspace,
                          size_t ws_bytes, void* stream);

/* Capacity-bounded exchange of the row-sharded slab (recommender_amd/sharded.py; replaces the
 * MirroredStrategy replicas of ctr/train.py:71-97 with row sharding). Every rank
 * gives every owner `capacity` row slots: unique u (sorted owner-major, from rs_unique_inverse)
 * of owner o takes slot o*capacity + (u - first unique of o); send_ids[world*capacity] = the
 * owner-local rows (-1 = padding), slot_of_unique[u] = its slot (-1 past capacity: *overflow
 * is set), inverse_slot[p] = slot of position p's unique row (-1 for OOB ids / past capacity).
 * Both all-to-alls then move equal [world, capacity] blocks: no host sync on the counts. */
int32_t rs_exchange_pack(const uint32_t* uniq_keys, const int32_t* n_unique,
                         const int32_t* owner_counts, int32_t world, int64_t shard_stride,
                         int64_t capacity, const int32_t* inverse, int64_t n_ids,
                         int32_t* send_ids, int32_t* slot_of_unique, int32_t* inverse_slot,
                         int32_t* overflow, void* stream);
/* The spill round of the capacity-bounded exchange (a batch with more unique rows for some owner
 * than the capacity): rs_exchange_excess writes max_o max(0, owner_counts[o] - capacity) (int64,
 * device) — all-reduced (MAX) over the ranks it is the spill capacity C2; rs_exchange_pack_spill
 * then gives unique u of owner o with j = u - (first unique of o) >= capacity the slot
 * world·capacity + o·C2 + (j - capacity), its owner-local row to spill_ids[o·C2 + j - capacity]
 * (−1 = padding), and rewrites inverse_slot from slot_of_unique (rows within the capacity keep
 * the slots rs_exchange_pack gave them). *overflow is set only if C2 is below this rank's excess. */
int32_t rs_exchange_excess(const int32_t* owner_counts, int32_t world, int64_t capacity,
                           int64_t* excess, void* stream);
int32_t rs_exchange_pack_spill(const uint32_t* uniq_keys, const int32_t* n_unique,
                               const int32_t* owner_counts, int32_t world, int64_t shard_stride,
                               int64_t capacity, int64_t spill_capacity, const int32_t* inverse,
                               int64_t n_ids, int32_t* spill_ids, int32_t* slot_of_unique,
                               int32_t* inverse_slot, int32_t* overflow, void* stream);
/* The owner's side of the exchange: out[i] = shard[ids[i]], a zero row where ids[i] < 0
 * (padding) or out of range; no error flag (padding is expected). */
int32_t rs_gather_rows_padded(const float* shard, int64_t n_rows, int32_t dim, const int32_t* ids,
                              int64_t n, float* out, void* stream);
/* Rows a step ahead (recommender_amd/sharded.py): the next step's rows are gathered and sent
 * while the current step runs, and only the rows the current step updates are sent again after
 * its apply. rs_exchange_mark (owner): stamp[row] = seq for every requested row ids[i] >= 0
 * of the step now finishing. rs_exchange_classify (owner): of the next step's requested slots
 * recv_ids[world*capacity] (owner-local rows, -1 = padding), those with stamp[row] == pred_seq
 * are listed per requester r: late_rows[r*capacity + k] = the row, late_slot[r*capacity + k] =
 * its slot in r's block, late_count[r] = the count (the rest of late_rows / late_slot is -1;
 * list order is not fixed run to run). rs_exchange_scatter_late (requester): for the [world,
 * late_capacity] block of late rows received from the owners and each owner's late_slot block
 * recv_slot[world*capacity], rows[o*capacity + recv_slot[o*capacity + k]] =
 * recv_rows[o*late_capacity + k] (slot -1 skipped). dim % 4 == 0, 16-byte aligned rows. */
int32_t rs_exchange_mark(const int32_t* ids, int64_t n, int32_t* stamp, int64_t n_rows,
                         int32_t seq, void* stream);
int32_t rs_exchange_classify(const int32_t* recv_ids, int32_t world, int64_t capacity,
                             const int32_t* stamp, int64_t n_rows, int32_t pred_seq,
                             int32_t* late_rows, int32_t* late_slot, int32_t* late_count,
                             void* stream);
int32_t rs_exchange_scatter_late(const float* recv_rows, const int32_t* recv_slot, int32_t world,
                                 int64_t capacity, int64_t late_capacity, int32_t dim, float* rows,
                                 void* stream);

/* a-2 (part 2) deduplicated gradient: uniq_rows[u], uniq_grad[u, dim] for the n_unique
 * distinct valid rows (count from rs_sort_ids), uniq_grad[u] = Σ grad_out[p] over the
 * positions p of row u. Summation order: sequential over sorted positions inside tiles of
 * RS_DEDUP_TILE sorted entries, tile partials added in tile order
 * (oracle/embedding.py:segment_sum_tiled restates it). */
#define RS_DEDUP_TILE 32
size_t rs_dedup_workspace_size(int64_t n_ids, int32_t dim);
int32_t rs_embedding_dedup_grad(const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                int64_t n_ids, const float* grad_out, int32_t dim, int64_t n_rows,
                                uint32_t* uniq_rows, float* uniq_grad, void* workspace,
                                size_t ws_bytes, void* stream);
/* rs_embedding_dedup_grad with the gradient of position p read as row_scale[p / scale_group] *
 * grad_out[p] (one fmul_rn, as rs_embedding_apply_scaled): the row-sharded DLRM step's unit rows
 * and G[b] (rs_dlrm_train_step_fwd_unit). row_scale NULL = rs_embedding_dedup_grad. */
int32_t rs_embedding_dedup_grad_scaled(const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                       int64_t n_ids, const float* grad_out,
                                       const float* row_scale, int32_t scale_group, int32_t dim,
                                       int64_t n_rows, uint32_t* uniq_rows, float* uniq_grad,
                                       void* workspace, size_t ws_bytes, void* stream);
/* rs_embedding_dedup_grad_scaled writing segment s's sum to uniq_grad row seg_map[s] (skipped
 * when < 0): the row-sharded step's per-owner padded send buffer (rs_exchange_pack's
 * slot_of_unique). uniq_rows[s] as before. */
int32_t rs_embedding_dedup_grad_mapped(const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                       int64_t n_ids, const float* grad_out,
                                       const float* row_scale, int32_t scale_group, int32_t dim,
                                       int64_t n_rows, const int32_t* seg_map, uint32_t* uniq_rows,
                                       float* uniq_grad, void* workspace, size_t ws_bytes,
                                       void* stream);
/* rs_embedding_dedup_grad_mapped over the keys in [key_lo, key_hi) only (segments numbered over
 * the whole key space n_rows, so two calls over adjoining ranges emit exactly the segments one
 * call does, with the same sums); seg_ready 1: the workspace already holds the segment ids of a
 * previous call on the same sorted keys; seg_excl (may be NULL): those segment ids given (the
 * head of rs_unique_inverse's workspace over the same keys), seg_ready then ignored. D = 128
 * with 16-byte aligned rows (the group walk).
 * The row-sharded step deduplicates its two owner halves apart, so the first half's gradient
 * all-to-all runs while the second half is summed. */
int32_t rs_embedding_dedup_grad_mapped_range(const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                             int64_t n_ids, const float* grad_out,
                                             const float* row_scale, int32_t scale_group,
                                             int32_t dim, int64_t n_rows, uint32_t key_lo,
                                             uint32_t key_hi, int32_t seg_ready,
                                             const int32_t* seg_excl,
                                             const int32_t* seg_map, uint32_t* uniq_rows,
                                             float* uniq_grad, void* workspace, size_t ws_bytes,
                                             void* stream);

/* The deduplicated gradient as a dense [n_rows, dim] tensor: rows without ids 0, every other row
 * its segment sum (same additions, same order as rs_embedding_dedup_grad); dense is fully written.
 * workspace >= rs_apply_workspace_size(n_ids, dim) bytes. (The graph-captured Keras Adam steps'
 * densified table gradients: DIEN, EGES, PinSage.) */
int32_t rs_embedding_grad_dense(const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                int64_t n_ids, const float* grad_out, int32_t dim, int64_t n_rows,
                                float* dense, void* workspace, size_t ws_bytes, void* stream);

/* rs_embedding_grad_dense with the gradient rows in n_segs (1..4) host-listed segments instead of
 * one [n_ids, dim] array: position p of segment i (seg_n[i] rows, p counted from the segment's
 * start) is the row at seg_ptrs[i] + p * seg_ld[i] (seg_ld >= dim, e.g. a column block of a
 * wider row). Σ seg_n = n_ids; same additions in the same order as over the concatenation. The
 * host arrays are read during the call. (A table looked up several times in one step — DIEN's
 * item table: target, positive and negative histories — without a concatenation pass; replaces
 * the concat of the IndexedSlices parts Keras does in tf.IndexedSlices aggregation.) */
int32_t rs_embedding_grad_dense_segs(const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                     int64_t n_ids, int32_t n_segs, const float* const* seg_ptrs,
                                     const int64_t* seg_n, const int64_t* seg_ld, int32_t dim,
                                     int64_t n_rows, float* dense, void* workspace,
                                     size_t ws_bytes, void* stream);

/* Dense gradient of a small table, no sort: grad_dense [n_rows, dim] = Σ over entries n with
 * ids[n] = v of grad_rows[n, :] (Keras' IndexedSlices gradient densified for a dense Adam step,
 * pinsage/train/train.py:45-46 on the year / genre tables, layers.py:63-75). Fixed summation
 * order (per-block LDS lanes, then blocks in order): deterministic, not position order.
 * Limits: dim a power of two <= 256, n_rows * dim <= 16384. Ids outside [0, n_rows) are
 * skipped and set RS_ERRBIT_OOB in err_flag (may be NULL). */
size_t rs_embedding_grad_dense_small_workspace_size(int64_t n_ids, int64_t n_rows, int32_t dim);
int32_t rs_embedding_grad_dense_small(const void* ids, int32_t id_dtype, int64_t n_ids,
                                      const float* grad_rows, int32_t dim, int64_t n_rows,
                                      float* grad_dense, int32_t* err_flag, void* workspace,
                                      size_t ws_bytes, void* stream);

/* Keras Adam dense update (KerasAdam / [3p TF 2.2] _resource_apply_dense, as pinsage/train/
 * train.py:45-48 applies it to every variable) over one flat buffer of n floats (n % 4 == 0,
 * 16-byte aligned), with lr_t read from device memory: lr_t = lr_hist[*step_idx]
 * (params->lr ignored), so a captured HIP graph replays the right step. Same roundings as the
 * separate torch ops: m = m*b1 + g*(1-b1); v = v*b2 + (g*g)*(1-b2); var -= (m*lr_t)/(sqrt(v)+eps). */
int32_t rs_keras_adam_flat(float* var, float* m, float* v, const float* grad, int64_t n,
                           const float* lr_hist, const int64_t* step_idx,
                           const rs_adam_params* params, void* stream);

/* a-2 (part 3) fused segmented-sum + optimizer apply on the touched rows
 * (Keras Adam _resource_apply_sparse / SGD _resource_apply_sparse_duplicate_indices,
 * [3p] reached from ctr/train.py:80,84,97 and the commented SGD path ctr/train.py:77-79).
 * Same summation order as rs_embedding_dedup_grad. m, v: optimizer slots [n_rows, dim]
 * (NULL for SGD). For RS_OPT_KERAS_ADAM call rs_keras_adam_dense_sweep afterwards with the
 * same touched bitmap ([ceil(n_rows/32)] uint32, zero on entry): the pair reproduces Keras'
 * dense m/v decay and dense var update. */
size_t rs_apply_workspace_size(int64_t n_ids, int32_t dim);
int32_t rs_embedding_apply(int32_t opt, float* table, float* m, float* v, int64_t n_rows,
                           int32_t dim, const uint32_t* sorted_rows, const int32_t* sorted_pos,
                           int64_t n_ids, const float* grad_out, const rs_adam_params* params,
                           uint32_t* touched_bitmap, void* workspace, size_t ws_bytes,
                           void* stream);
/* rs_embedding_apply with the gradient of position p read as row_scale[p / scale_group] *
 * grad_out[p] (one fp32 multiply, rounded before the segmented sum). The fused DLRM step
 * (rs_dlrm_interaction_fwd_head_dx) hands its unit interaction gradient and the per-example
 * scale G[b] (scale_group = n_slots); row_scale NULL = rs_embedding_apply. */
int32_t rs_embedding_apply_scaled(int32_t opt, float* table, float* m, float* v, int64_t n_rows,
                                  int32_t dim, const uint32_t* sorted_rows,
                                  const int32_t* sorted_pos, int64_t n_ids, const float* grad_out,
                                  const float* row_scale, int32_t scale_group,
                                  const rs_adam_params* params, uint32_t* touched_bitmap,
                                  void* workspace, size_t ws_bytes, void* stream);
/* One-call forms (SURVEY §8(b) minimum exports): sort + dedup / sort + apply with one workspace of
 * rs_sparse_workspace_size(n_ids, dim) bytes; bit-identical to the two-call forms. ids[n_ids]
 * (id_dtype RS_ID_I32 / RS_ID_I64; slot = position % n_slots when slot_offsets is given);
 * grad_out[n_ids, dim] in position order. rs_embedding_bwd_dedup writes *n_unique (device). */
size_t rs_sparse_workspace_size(int64_t n_ids, int32_t dim);
int32_t rs_embedding_bwd_dedup(const void* ids, int32_t id_dtype, int64_t n_ids,
                               const int64_t* slot_offsets, int32_t n_slots, int64_t n_rows,
                               const float* grad_out, int32_t dim, uint32_t* uniq_rows,
                               float* uniq_grad, int32_t* n_unique, int32_t* err_flag,
                               void* workspace, size_t ws_bytes, void* stream);
int32_t rs_apply_sgd(float* table, int64_t n_rows, int32_t dim, const void* ids, int32_t id_dtype,
                     int64_t n_ids, const int64_t* slot_offsets, int32_t n_slots,
                     const float* grad_out, float lr, int32_t* err_flag, void* workspace,
                     size_t ws_bytes, void* stream);
int32_t rs_apply_lazy_adam(float* table, float* m, float* v, int64_t n_rows, int32_t dim,
                           const void* ids, int32_t id_dtype, int64_t n_ids,
                           const int64_t* slot_offsets, int32_t n_slots, const float* grad_out,
                           const rs_adam_params* params, int32_t* err_flag, void* workspace,
                           size_t ws_bytes, void* stream);
int32_t rs_apply_keras_dense_adam(float* table, float* m, float* v, int64_t n_rows, int32_t dim,
                                  const void* ids, int32_t id_dtype, int64_t n_ids,
                                  const int64_t* slot_offsets, int32_t n_slots,
                                  const float* grad_out, const rs_adam_params* params,
                                  uint32_t* touched_bitmap, int32_t* err_flag, void* workspace,
                                  size_t ws_bytes, void* stream);
/* dense sweep for RS_OPT_KERAS_ADAM: rows NOT marked in touched_bitmap get
 * m=b1*m, v=b2*v, var -= lr*m/(sqrt(v)+eps); the bitmap is cleared afterwards. */
int32_t rs_keras_adam_dense_sweep(float* table, float* m, float* v, int64_t n_rows, int32_t dim,
                                  const rs_adam_params* params, uint32_t* touched_bitmap,
                                  void* stream);
/* Deferred Keras decay (exact): the dense m/v decay + var update of rows without a gradient is
 * replayed per row on demand instead of swept over all V rows each step. last [n_rows] int32 =
 * the last step applied to each row (0 initially); lr_hist[s] = lr_t of step s (1-based, the
 * host's keras_adam_coefficients(s).lr); beta1 / beta2 / epsilon from params.
 * rs_keras_adam_catchup: before step `step` reads its rows, each unique row of sorted_rows
 *   (rs_sort_ids output; entries >= n_rows skipped) replays steps last+1 .. step-1 and is
 *   left at last = step - 1 (the step's sparse apply — rs_embedding_apply with
 *   RS_OPT_KERAS_ADAM, no dense sweep — updates it next, then rs_keras_adam_mark sets
 *   last = step; a presort whose apply never runs — a forward-only call, an exception —
 *   leaves that step to a later replay instead of losing it).
 * rs_keras_adam_materialize: every row replays last+1 .. step; afterwards table / m / v equal
 *   the per-step dense sweep's state bit for bit (same arithmetic per element and step). */
int32_t rs_keras_adam_catchup(float* table, float* m, float* v, int32_t* last, int64_t n_rows,
                              int32_t dim, const int32_t* sorted_rows, int64_t n,
                              const float* lr_hist, int32_t step, const rs_adam_params* params,
                              void* stream);
int32_t rs_keras_adam_materialize(float* table, float* m, float* v, int32_t* last, int64_t n_rows,
                                  int32_t dim, const float* lr_hist, int32_t step,
                                  const rs_adam_params* params, void* stream);
/* After step `step`'s sparse apply: its unique rows (the sorted rows the apply walked) are up
 * to date through that step, last[row] = step. */
int32_t rs_keras_adam_mark(int32_t* last, int64_t n_rows, const uint32_t* sorted_rows, int64_t n,
                           int32_t step, void* stream);

/* ------------------------------------------------------------------------------------
 * a-4 DotInteraction(self_interaction, skip_gather) — ctr/layers.py:17-43.
 * x: [B, F, D]. out row stride out_stride (>= output width):
 *   skip_gather: F*F values, (i,j) kept where included, zero elsewhere (ctr/layers.py:35-38);
 *   gather & !self: i<j row-major, F(F-1)/2 (ctr/layers.py:32-34,39-42);
 *   gather & self: i>=j row-major, F(F+1)/2 (ctr/layers.py:27-30,39-42). */
int32_t rs_dot_interaction_fwd(const float* x, int64_t batch, int32_t F, int32_t D,
                               int32_t self_interaction, int32_t skip_gather, float* out,
                               int64_t out_stride, void* stream);
int32_t rs_dot_interaction_bwd(const float* x, const float* grad_out, int64_t batch, int32_t F,
                               int32_t D, int32_t self_interaction, int32_t skip_gather,
                               int64_t grad_stride, float* grad_x, void* stream);

/* DLRM fused gather + interaction + concat (ctr/model.py:45-55 with
 * DotInteraction(False, True), ctr/model.py:43):
 *   X(b) = [ table[row(b,0)], ..., table[row(b,S-1)], dense[b] ]  (F = n_slots + 1 rows),
 *   compact = 0: out[b] = [ Z(b) (F*F, strict upper kept, zeros elsewhere), dense[b] ]
 *                (the reference's skip_gather layout, ctr/model.py:55),
 *   compact = 1: out[b] = [ Z(b) strict upper in row-major order (F(F-1)/2), dense[b] ]
 *                (the same values without the structural zeros; the caller drops the
 *                matching zero-input rows of the top-MLP kernel).
 * Columns [width, out_stride) of each output row are zero-filled (GEMM alignment padding).
 * bwd re-gathers X from the table and writes grad_emb[b*S+s] and grad_dense[b]. */
int32_t rs_dlrm_interaction_fwd(const float* table, int64_t n_rows, int32_t D, const void* ids,
                                int32_t id_dtype, int32_t n_slots, const int64_t* slot_offsets,
                                const float* dense, int64_t batch, int32_t compact, float* out,
                                int64_t out_stride, int32_t* err_flag, void* stream);
int32_t rs_dlrm_interaction_bwd(const float* table, int64_t n_rows, int32_t D, const void* ids,
                                int32_t id_dtype, int32_t n_slots, const int64_t* slot_offsets,
                                const float* dense, int64_t batch, int32_t compact,
                                const float* grad_out, int64_t grad_stride, float* grad_emb,
                                float* grad_dense, void* stream);

/* rs_dlrm_interaction_fwd (compact layout, D = 128, F <= 32) with the composed top MLP fused
 * (ctr/model.py:56 `self.top_mlp(...)` with linear hidden layers): besides writing out[b], the
 * kernel forms y[b] = act(out[b]·q + c[0]) (q [out_stride], from rs_chain3_vec_compose). */
int32_t rs_dlrm_interaction_fwd_head(const float* table, int64_t n_rows, int32_t D,
                                     const void* ids, int32_t id_dtype, int32_t n_slots,
                                     const int64_t* slot_offsets, const float* dense,
                                     int64_t batch, float* out, int64_t out_stride,
                                     const float* q, const float* c, int32_t act, float* y,
                                     int32_t* err_flag, void* stream);

/* rs_dlrm_interaction_fwd_head plus the example's UNIT interaction gradient, formed while the
 * gathered rows are in registers (ctr/model.py:49-57 forward; its backward for the rank-one
 * upstream gradient G[b] ⊗ q of the linear top chain, ctr/layers.py:8): with M the strict-upper
 * pairs of q, dxu_emb[b*S + i] = ((M + Mᵀ)·X[b])[i] for i < S and dxu_dense[b] = ((M + Mᵀ)·X[b])[S]
 * + q[F(F-1)/2 ..]. The embedding-row gradient is then G[b] * dxu_emb (rs_embedding_apply_scaled)
 * and the bottom-MLP gradient G[b] * dxu_dense: the backward needs no re-gather. D = 128, F <= 32. */
int32_t rs_dlrm_interaction_fwd_head_dx(const float* table, int64_t n_rows, int32_t D,
                                        const void* ids, int32_t id_dtype, int32_t n_slots,
                                        const int64_t* slot_offsets, const float* dense,
                                        int64_t batch, float* out, int64_t out_stride,
                                        const float* q, const float* c, int32_t act, float* y,
                                        float* dxu_emb, float* dxu_dense, int32_t* err_flag,
                                        void* stream);

/* Rank-one upstream gradient (the factored top-MLP backward, recommender_amd/nn.py
 * _LinearChainFn): grad row b = gscale[b] * grad_row[0..width), bit-identical to
 * rs_dlrm_interaction_bwd on the materialised rows; compact layout, D = 128, F <= 32 only
 * (RS_E_UNSUPPORTED otherwise). */
int32_t rs_dlrm_interaction_bwd_rank1(const float* table, int64_t n_rows, int32_t D,
                                      const void* ids, int32_t id_dtype, int32_t n_slots,
                                      const int64_t* slot_offsets, const float* dense,
                                      int64_t batch, const float* gscale, const float* grad_row,
                                      int64_t width, float* grad_emb, float* grad_dense,
                                      void* stream);

/* a-5 DeepFM second-order term — ctr/model.py:21-23:
 *   out[b] = 0.5 * Σ_d ((Σ_f e[b,f,d])^2 - Σ_f e[b,f,d]^2). */
int32_t rs_fm_fwd(const float* emb, int64_t batch, int32_t F, int32_t D, float* out, void* stream);
int32_t rs_fm_bwd(const float* emb, const float* grad_out, int64_t batch, int32_t F, int32_t D,
                  float* grad_emb, void* stream);

/* ------------------------------------------------------------------------------------
 * DIEN recurrences; one wave per example, H <= 64, uint8 mask [B, L]
 * (ids != 0, dien/model.py:68); masked steps carry the state. The input projections of all
 * steps (x·W + b) and all weight gradients are caller GEMMs.
 * a-9  keras GRU, reset_after (InterestExtract dien/layers.py:79,131):
 *      xw [B,L,3H] = [x_z,x_r,x_h]; U [H,3H] recurrent kernel; rb [3H] recurrent bias;
 *      out [B,L,H] state after every step; saved [B,L,4H] = [z, r, hh, inner_h] (may be NULL).
 *      bwd: dout [B,L,H] → dxw [B,L,3H] (grad of x·W+b), dinner [B,L,3H] (grad of h·U+rb).
 *      flags: RS_DIEN_SKIP_MASKED_ROWS leaves the masked steps' rows of dxw / dinner (and of the
 *      AUGRU's dxw and saved r·h_prev) unwritten — for callers that read only the valid rows
 *      (rs_masked_dx / rs_masked_wgrad); 0 writes them as 0. */
#define RS_DIEN_SKIP_MASKED_ROWS 1
int32_t rs_gru_fwd(const float* xw, const float* U, const float* rb, const uint8_t* mask,
                   int64_t B, int32_t L, int32_t H, float* out, float* saved, void* stream);
int32_t rs_gru_bwd(const float* dout, const float* out, const float* saved, const float* U,
                   const uint8_t* mask, int64_t B, int32_t L, int32_t H, float* dxw,
                   float* dinner, int32_t flags, void* stream);
/* a-11 AUGRUCell under keras RNN (dien/layers.py:161-204): xw = [x·Ku_x+bu, x·Kr_x+br,
 *      x·Kh_x+bh]; Kuh, Krh [H,H] = h rows of the update/reset kernels ([h, x] concat order),
 *      Khr [H,H] = r·h rows of the candidate kernel ([x, r·h] order); att [B,L].
 *      final_h [B,H]; states [B,L,H]; saved [B,L,4H] = [u, r, hh, r·h_prev].
 *      bwd: dfinal [B,H] → dxw [B,L,3H], datt [B,L]. */
int32_t rs_augru_fwd(const float* xw, const float* att, const float* Kuh, const float* Krh,
                     const float* Khr, const uint8_t* mask, int64_t B, int32_t L, int32_t H,
                     float* final_h, float* states, float* saved, int32_t flags, void* stream);
int32_t rs_augru_bwd(const float* dfinal, const float* att, const float* states,
                     const float* saved, const float* Kuh, const float* Krh, const float* Khr,
                     const uint8_t* mask, int64_t B, int32_t L, int32_t H, float* dxw,
                     float* datt, int32_t flags, void* stream);
/* a-10 DIENAttention (dien/layers.py:145-158): a = softmax_t(h_t·q + (1-m_t)(-1e9)),
 *      q = K·target [B,H] (caller); bwd: da → dhs [B,L,H] (= ds_t q, written), dq [B,H]. */
int32_t rs_dien_attention_fwd(const float* hs, const float* q, const uint8_t* mask, int64_t B,
                              int32_t L, int32_t H, float* a, void* stream);
int32_t rs_dien_attention_bwd(const float* hs, const float* q, const float* a, const float* da,
                              int64_t B, int32_t L, int32_t H, float* dhs, float* dq,
                              void* stream);
/* a-9  DIEN auxiliary loss (InterestExtract.compute_auxiliary_loss dien/layers.py:89-108 with
 *      AuxiliaryNet([80, 40, 1]) dien/layers.py:62-73), fused: x = [h_t, e_{t+1}] for
 *      e = pos / neg history embeddings, z = σ(σ(x·W1+b1)·W2+b2)·W3+b3,
 *      aux[b] = Σ_t m[b,t+1]·(ce(z_pos,1) + ce(z_neg,0)) / (2·Σ_t m[b,t+1]).
 *      hidden [B,L,H] (GRU states), pos/neg [B,L,E], mask [B,L] u8; W1 [H+E,80], b1 [80],
 *      W2 [80,40], b2 [40], W3 [40], b3 [1] (Keras [in, out] kernels). Rows with m = 0 add
 *      exactly 0 and are not evaluated. Built for (H, E) = (36, 36) and (16, 16); other widths
 *      return RS_E_UNSUPPORTED. bwd: daux [B] → dhidden [B,L,H], dpos / dneg [B,L,E] (every
 *      element written) and dparams = [dW1 | db1 | dW2 | db2 | dW3 | db3] (overwritten,
 *      deterministic); workspace ≥ rs_dien_aux_workspace_size(B, L, H, E) bytes. */
size_t rs_dien_aux_workspace_size(int64_t B, int32_t L, int32_t H, int32_t E);
/* a-9 / a-11 the B·L-row products around the recurrences, on the valid (mask != 0) rows only
 *      (replace the library GEMMs over all B·L rows: dien/layers.py:79,131,161-204 via
 *      keras GRU / RNN(AUGRUCell); a masked step carries the state, so its projection is never
 *      read and its gradient rows are 0).
 *      rs_valid_rows: idx [R] (the valid rows in order, first *count entries), count [1] int32
 *        on the device; workspace >= rs_valid_rows_workspace_size(R) bytes.
 *      rs_masked_proj: y[r, :N] = x[r, :K]·W [K,N] + bias[N] (bias may be NULL) for the listed
 *        rows; other rows of y untouched. K <= 64, N <= 192.
 *      rs_masked_dx: dx[r, :K] = d[r, :N]·Wᵀ (W [K,N]) for the listed rows (idx / count of
 *        rs_valid_rows over the same mask), 0 for the rows with mask == 0 (all R rows written).
 *      rs_masked_dx_acc: the same with an addend (add may be NULL): dx = add + d·Wᵀ on the listed
 *        rows, dx = add on the masked ones — a second consumer's gradient of the same input
 *        (the aux loss's of the positive history, dien/layers.py:89-108) summed in the kernel.
 *      rs_masked_wgrad: C [K,N] = Σ_listed A_rᵀ·D[r, :N] and sums [N] = Σ_listed D[r] (may be
 *        NULL); A_r = A row r, or with shift_L > 0 row r - 1 and zeros where r % shift_L == 0
 *        (the previous step's state). Fixed row chunks, folded in order: deterministic.
 *        workspace >= rs_masked_wgrad_workspace_size(K, N) bytes. */
size_t rs_valid_rows_workspace_size(int64_t R);
int32_t rs_valid_rows(const uint8_t* mask, int64_t R, int32_t* idx, int32_t* count,
                      void* workspace, size_t ws_bytes, void* stream);
int32_t rs_masked_proj(const float* x, int64_t ldx, const float* W, const float* bias,
                       const int32_t* idx, const int32_t* count, int64_t R, int32_t K, int32_t N,
                       float* y, int64_t ldy, void* stream);
int32_t rs_masked_dx(const float* d, int64_t ldd, const float* W, const uint8_t* mask,
                     const int32_t* idx, const int32_t* count, int64_t R, int32_t K, int32_t N,
                     float* dx, int64_t lddx, void* stream);
int32_t rs_masked_dx_acc(const float* d, int64_t ldd, const float* W, const uint8_t* mask,
                         const int32_t* idx, const int32_t* count, int64_t R, int32_t K, int32_t N,
                         const float* add, int64_t ldadd, float* dx, int64_t lddx, void* stream);
size_t rs_masked_wgrad_workspace_size(int32_t K, int32_t N);
int32_t rs_masked_wgrad(const float* A, int64_t lda, int32_t shift_L, const float* D, int64_t ldd,
                        const int32_t* idx, const int32_t* count, int32_t K, int32_t N, float* C,
                        float* sums, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * fp32 GEMM of the Keras Dense layers on the bf16 matrix cores at fp32 accuracy (split-bf16,
 * six part products; csrc/gemm.hip): C[b] = act(op(A[b])·op(B[b]) + bias[b]) for b < batch,
 * op(A)[m][k] = ta ? A[k*lda + m] : A[m*lda + k], op(B)[k][n] = tb ? B[n*ldb + k] : B[k*ldb + n],
 * per-batch strides sA / sB / sC / sbias (floats); act 0 none, 1 relu, 2 sigmoid; bias may be
 * NULL. Replaces the Dense layers' tf.matmul / BiasAdd / activation (esmm/layers.py:4-13,
 * esmm/mmoe.py:8-109, ctr/layers.py:5-14, dien/layers.py:20-31) forward (ta 0, tb 0), dgrad
 * (dz·Wᵀ: ta 0, tb 1) and wgrad (xᵀ·dz: ta 1, tb 0) products. splits > 1 divides K into that many
 * ranges (multiples of 32) whose partials are folded in order (deterministic);
 * workspace >= rs_gemm_x3_workspace_size(M, N, batch, splits). M, N, K, lda, ldb, sA, sB multiples
 * of 4; A, B 16-byte aligned. */
size_t rs_gemm_x3_workspace_size(int64_t M, int64_t N, int32_t batch, int32_t splits);
int32_t rs_gemm_x3(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, const float* A,
                   int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB, float* C,
                   int64_t ldc, int64_t sC, int32_t batch, const float* bias, int64_t sbias,
                   int32_t act, int32_t splits, void* workspace, size_t ws_bytes, void* stream);

int32_t rs_dien_aux_fwd(const float* hidden, const float* pos, const float* neg,
                        const uint8_t* mask, int64_t B, int32_t L, int32_t H, int32_t E,
                        const float* W1, const float* b1, const float* W2, const float* b2,
                        const float* W3, const float* b3, float* aux, void* stream);
int32_t rs_dien_aux_bwd(const float* hidden, const float* pos, const float* neg,
                        const uint8_t* mask, int64_t B, int32_t L, int32_t H, int32_t E,
                        const float* W1, const float* b1, const float* W2, const float* b2,
                        const float* W3, const float* b3, const float* daux, float* dhidden,
                        float* dpos, float* dneg, float* dparams, void* workspace,
                        size_t ws_bytes, void* stream);
/* rs_dien_aux_bwd with acc_hidden = 1: dhidden holds the hidden states' upstream gradient (the
 * attention's + the AUGRU's) and the aux loss's part is added in place (no fill, no add pass). */
int32_t rs_dien_aux_bwd_acc(const float* hidden, const float* pos, const float* neg,
                            const uint8_t* mask, int64_t B, int32_t L, int32_t H, int32_t E,
                            const float* W1, const float* b1, const float* W2, const float* b2,
                            const float* W3, const float* b3, const float* daux, float* dhidden,
                            int32_t acc_hidden, float* dpos, float* dneg, float* dparams,
                            void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * Keras binary_crossentropy on probabilities (ctr/train.py:85, dien/train.py:18,
 * esmm/train.py:101-102; [3p] TF 2.2 backend: clip to [eps, 1-eps], -(y log(p+eps) +
 * (1-y) log(1-p+eps))), fused. reduction 0 = none (out[n]), 1 = sum, 2 = mean (out[1]);
 * sums fold per-block partials in block order (deterministic). grad_out: [n] for
 * reduction 0, else [1]. */
size_t rs_bce_workspace_size(int64_t n);
int32_t rs_bce_fwd(const float* p, const float* y, int64_t n, float eps, int32_t reduction,
                   float* out, void* workspace, size_t ws_bytes, void* stream);
int32_t rs_bce_bwd(const float* p, const float* y, int64_t n, float eps, int32_t reduction,
                   const float* grad_out, float* grad_p, void* stream);

/* ------------------------------------------------------------------------------------
 * Dense-layer backward epilogue (Keras Dense with activation, ctr/layers.py:5-14,
 * esmm/layers.py:4-13): dz = act'(y) ⊙ dy (act 0 = linear: dz not written, 1 = relu,
 * 2 = sigmoid; y is the layer output) and db[n] = Σ_b dz[b, n] (deterministic fold). */
size_t rs_act_bwd_colsum_workspace_size(int64_t B, int32_t N);
int32_t rs_act_bwd_colsum(const float* dy, const float* y, int64_t B, int32_t N, int32_t act,
                          float* dz, float* db, void* workspace, size_t ws_bytes, void* stream);
/* The same over n_groups row groups of B / n_groups rows (a multiple of 512) in one pass:
 * db [n_groups, N] holds each group's column sums (act 1 or 2). MMOE's batched expert layer:
 * the [E, B, H] gradient masked at once, per-expert bias gradients. */
int32_t rs_act_bwd_colsum_groups(const float* dy, const float* y, int64_t B, int32_t N,
                                 int32_t act, int32_t n_groups, float* dz, float* db,
                                 void* workspace, size_t ws_bytes, void* stream);
/* The same on row-strided operands (ld_* >= N elements between rows): a column block of a
 * wider [B, ld] activation — the two ESMM towers' first layers evaluated as one GEMM over the
 * shared input (esmm/esmm.py:27-28), each tower's block masked from its own gradient. */
int32_t rs_act_bwd_colsum_ld(const float* dy, int64_t ld_dy, const float* y, int64_t ld_y,
                             int64_t B, int32_t N, int32_t act, float* dz, int64_t ld_dz, float* db,
                             void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * keras.layers.BatchNormalization on [B, C] rows (the DIEN / DIN / BASE MLP head's input,
 * dien/layers.py:20-31). training = 1: batch mean and population variance (tf.nn.moments),
 * y = ((x - mean)·rsqrt(var + epsilon))·gamma + beta, moving statistics updated in place by
 * Keras' m -= (m - value)·(1 - momentum); training = 0: the moving statistics, none updated.
 * save_mean / save_invstd [C] (the statistics used) feed the backward: dbeta = Σ dy,
 * dgamma = Σ dy·x̂, dx = gamma·r·(dy - dbeta/B - x̂·dgamma/B) (training) or gamma·r·dy.
 * Deterministic (fixed 64-row chunks merged in order). workspace >= rs_batch_norm_workspace_size
 * (unused by an inference forward). */
size_t rs_batch_norm_workspace_size(int64_t B, int32_t C);
int32_t rs_batch_norm_fwd(const float* x, int64_t B, int32_t C, const float* gamma,
                          const float* beta, float epsilon, float momentum, int32_t training,
                          float* moving_mean, float* moving_var, float* y, float* save_mean,
                          float* save_invstd, void* workspace, size_t ws_bytes, void* stream);
int32_t rs_batch_norm_bwd(const float* dy, const float* x, int64_t B, int32_t C,
                          const float* save_mean, const float* save_invstd, const float* gamma,
                          int32_t training, float* dx, float* dgamma, float* dbeta,
                          void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * Multi-hot mean lookup (PinSage FeatureProjector's genre, pinsage/train/layers.py:68-81):
 * out[n, :] = (Σ_g table[mh[items[n], g], :]) / G for the items' G-slot id rows of mh
 * [n_items, G] int32 (ids outside [0, V) read 0 and set RS_ERRBIT_OOB; items outside
 * [0, n_items) give a zero row forward, no gradient backward, and set RS_ERRBIT_OOB). Backward:
 * the dense [V, D] table gradient Σ_n Σ_{g: id = r} dout[n] / G (deterministic; V·D <= 256,
 * D <= 64, G <= 32). */
int32_t rs_multihot_mean_fwd(const float* table, int32_t V, int32_t D, const int32_t* mh, int32_t G,
                             int64_t n_items, const int64_t* items, int64_t N, float* out,
                             int32_t* err_flag, void* stream);
size_t rs_multihot_mean_bwd_workspace_size(int64_t N, int32_t V, int32_t D);
int32_t rs_multihot_mean_bwd(const int32_t* mh, int32_t G, int64_t n_items, const int64_t* items,
                             int64_t N, const float* dout, int32_t V, int32_t D, float* dtable,
                             int32_t* err_flag, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * Deterministic index_add of rows (the backward of a row gather h.index_select(0, ids), e.g.
 * PinSage's item2item scorer, pinsage/train/model.py:14-19): out [n_rows, dim] (contiguous) =
 * 0, then out[ids[p]] += rows[p] for every p with valid[p] != 0 (valid may be NULL = all). Each
 * row's terms are summed in position order inside tiles of RS_DEDUP_TILE sorted entries, tile
 * partials in tile order (rs_sort_ids + rs_embedding_grad_dense): run-to-run identical, unlike
 * float atomics. Ids outside [0, n_rows) are skipped and set RS_ERRBIT_OOB. */
size_t rs_index_add_rows_workspace_size(int64_t n, int32_t dim);
int32_t rs_index_add_rows(const void* ids, int32_t id_dtype, int64_t n, const uint8_t* valid,
                          const float* rows, int32_t dim, int64_t n_rows, float* out,
                          int32_t* err_flag, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * PinSage's item2item scores and margin loss in one pass (pinsage/train/model.py:14-19,
 * pinsage/train/train.py:17-20): pos_score[i] = h[pos_src[i]]·h[pos_dst[i]], neg_score likewise,
 * loss[0] = Σ_{live i} max((neg + delta) - pos, 0) / n_live (valid: uint8 per pair or null =
 * all live; n_live: device int32 [1] or null = n_pairs; -1 node ids score node 0, as padding;
 * ids >= n_rows read a zero row and set RS_ERRBIT_OOB in err_flag, which may be NULL).
 * Backward: dh [n_rows, D] contiguous = the loss's gradient (dloss: device float [1]); every
 * pair's four row terms are written as rows and folded per node by rs_index_add_rows (fixed
 * order: deterministic, no float atomics). D <= 64. */
size_t rs_pair_margin_workspace_size(int64_t n_pairs);
int32_t rs_pair_margin_fwd(const float* h, int64_t ld, int32_t D, int64_t n_rows,
                           const int32_t* pos_src, const int32_t* pos_dst, const int32_t* neg_src,
                           const int32_t* neg_dst, int64_t n_pairs, float delta,
                           const uint8_t* valid, const int32_t* n_live, float* pos_score,
                           float* neg_score, float* loss, int32_t* err_flag, void* workspace,
                           size_t ws_bytes, void* stream);
size_t rs_pair_margin_bwd_workspace_size(int64_t n_pairs, int32_t D);
int32_t rs_pair_margin_bwd(const float* h, int64_t ld, int32_t D, int64_t n_rows,
                           const int32_t* pos_src, const int32_t* pos_dst, const int32_t* neg_src,
                           const int32_t* neg_dst, int64_t n_pairs, float delta,
                           const uint8_t* valid, const int32_t* n_live, const float* pos_score,
                           const float* neg_score, const float* dloss, float* dh,
                           int32_t* err_flag, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * PinSage sampling + aggregation. The graph is the bipartite
 * item/user CSR in both directions: i2u_indptr [n_items+1] int64, i2u_idx int32 user ids,
 * u2i_indptr [n_users+1], u2i_idx item ids. Randomness is Philox4x32-10 keyed by `seed`
 * (64-bit) and a purpose word; counters (subject, walk | layer << 16, step, draw / 4), so
 * a draw depends only on (seed, step, subject): launch- and shard-invariant. Bounded ints
 * are (r * n) >> 32. oracle/pinsage.py restates every function bit for bit. */

/* Raw Philox4x32-10 (known-answer tests): out[4i..4i+3] = philox(ctr[4i..4i+3], (k0, k1)). */
int32_t rs_philox4x32_10(const uint32_t* ctr, int64_t n, uint32_t k0, uint32_t k1,
                         uint32_t* out, void* stream);

/* dgl.sampling.random_walk(g, seeds, metapath=[item→user, user→item] * n_traversals,
 * restart_prob) [3p DGL 0.6.1] as used by PinSAGESampler (pinsage/train/data_loader.py:26-27):
 * num_walks walks per seed; traces [n_seeds*num_walks, 2*n_traversals+1] int32 (row
 * s*num_walks + j = walk j of seed s), -1 after a dead end; with restart_prob > 0 a trace ends
 * after a transition whose stop draw falls below restart_prob. Uniform neighbour choice. */
int32_t rs_metapath_walk(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                         const int64_t* u2i_indptr, const int32_t* u2i_idx, const int32_t* seeds,
                         int64_t n_seeds, int32_t num_walks, int32_t n_traversals,
                         float restart_prob, uint64_t seed, uint32_t step, uint32_t layer,
                         int32_t* traces, void* stream);

/* a-14 item2item_batch_sampler (pinsage/train/data_loader.py:6-18): for pairs
 * i = pair_base .. pair_base+batch-1: head, neg ~ U[0, n_items), pos = item after one
 * item→user→item walk from head; pairs whose walk dead-ends are dropped (mask pos != -1,
 * :15-18), order kept. heads/pos_tails/neg_tails [batch] (first *n_valid written). */
size_t rs_item_pairs_workspace_size(int32_t batch);
int32_t rs_item_pairs(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                      const int64_t* u2i_indptr, const int32_t* u2i_idx, int32_t n_items,
                      int64_t pair_base, int32_t batch, uint64_t seed, uint32_t step,
                      int32_t* heads, int32_t* pos_tails, int32_t* neg_tails, int32_t* n_valid,
                      void* workspace, size_t ws_bytes, void* stream);

/* rs_item_pairs with the RNG step read from device memory (*step_ptr, uint32): a captured
 * HIP graph that advances the counter on the device samples the next step's pairs on replay. */
int32_t rs_item_pairs_at(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                         const int64_t* u2i_indptr, const int32_t* u2i_idx, int32_t n_items,
                         int64_t pair_base, int32_t batch, uint64_t seed, const uint32_t* step_ptr,
                         int32_t* heads, int32_t* pos_tails, int32_t* neg_tails, int32_t* n_valid,
                         void* workspace, size_t ws_bytes, void* stream);

/* Set of (dst, src) item pairs for the leak-edge removal of generate_blocks
 * (pinsage/train/data_loader.py:34-39): table [capacity] uint64, capacity a power of two > n,
 * filled with 0xFF bytes by the caller before the first build. */
int32_t rs_pair_set_build(const int32_t* src, const int32_t* dst, int64_t n, uint64_t* table,
                          int64_t capacity, void* stream);

/* a-15 dgl.sampling.PinSAGESampler(g, item, user, n_traversals, restart_prob, num_walks,
 * num_neighbors) [3p] (pinsage/train/data_loader.py:26-27) + remove_edges (:34-39): per seed,
 * num_walks walks of n_traversals item→user→item traversals; every item reached after a
 * traversal is one visit (self-visits count); the num_neighbors most visited (count desc,
 * item id asc — DGL's tie order is unspecified) become in-edges with weight = count; then
 * edges (src, dst=seed) in the exclusion set (excl_capacity 0 = none) are dropped without
 * back-filling. nbr/cnt [n_seeds, num_neighbors], -1/0 in empty slots; a seed < 0 (padding
 * of a capacity-shaped batch) gets k empty slots.
 * Limits: num_walks <= 64, n_traversals <= 8. */
int32_t rs_pinsage_neighbors(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                             const int64_t* u2i_indptr, const int32_t* u2i_idx,
                             const int32_t* seeds, int64_t n_seeds, int32_t num_walks,
                             int32_t n_traversals, float restart_prob, uint64_t seed,
                             uint32_t step, uint32_t layer, int32_t num_neighbors,
                             const uint64_t* excl_table, int64_t excl_capacity, int32_t* nbr,
                             int32_t* cnt, void* stream);

/* rs_pinsage_neighbors with the RNG step read from device memory (*step_ptr). */
int32_t rs_pinsage_neighbors_at(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                                const int64_t* u2i_indptr, const int32_t* u2i_idx,
                                const int32_t* seeds, int64_t n_seeds, int32_t num_walks,
                                int32_t n_traversals, float restart_prob, uint64_t seed,
                                const uint32_t* step_ptr, uint32_t layer, int32_t num_neighbors,
                                const uint64_t* excl_table, int64_t excl_capacity, int32_t* nbr,
                                int32_t* cnt, void* stream);

/* First-appearance unique (dgl.compact_graphs / dgl.to_block node order,
 * pinsage/train/data_loader.py:40,48): uniq = distinct ids >= 0 in order of first position,
 * local[i] = index of ids[i] in uniq (-1 for ids < 0; may be NULL). ids >= n_nodes set
 * RS_ERRBIT_OOB in err_flag (may be NULL) and count as -1. */
size_t rs_unique_first_workspace_size(int64_t n_nodes, int64_t n);
int32_t rs_unique_first(const int32_t* ids, int64_t n, int64_t n_nodes, int32_t* uniq,
                        int32_t* local, int32_t* n_unique, int32_t* err_flag, void* workspace,
                        size_t ws_bytes, void* stream);

/* dgl.to_block(frontier, dst_nodes) (pinsage/train/data_loader.py:40): from nbr_local
 * [n_dst, k] (src local ids, -1 = no edge) and cnt: CSR by dst (indptr [n_dst+1], edges in
 * slot order: edge_src, edge_dst, edge_w = (float)count), *n_edges, and the transpose
 * t_indptr [n_src+1] / t_edge [n_dst*k capacity] listing each src's edges in edge order. */
size_t rs_pinsage_block_workspace_size(int64_t n_dst, int32_t k);
int32_t rs_pinsage_block(const int32_t* nbr_local, const int32_t* cnt, int64_t n_dst, int32_t k,
                         int64_t n_src, int32_t* indptr, int32_t* edge_src, int32_t* edge_dst,
                         float* edge_w, int32_t* n_edges, int32_t* t_indptr, int32_t* t_edge,
                         void* workspace, size_t ws_bytes, void* stream);

/* a-18 Convolve weighted mean-pool (pinsage/train/layers.py:17-24: update_all(u_mul_e, sum),
 * update_all(copy_e, sum), clip ws >= 1, divide): nv[d] = Σ_e w_e u[src_e] / max(Σ_e w_e, 1)
 * over d's edges in CSR order; wsum[d] = Σ_e w_e (may be NULL). bwd: grad_u[s] =
 * Σ_{e of s} w_e / max(wsum[dst_e], 1) · grad_nv[dst_e] (transpose order; every src row
 * written). */
int32_t rs_weighted_mean_agg_fwd(const float* u, int64_t n_src, int32_t H, const int32_t* indptr,
                                 const int32_t* edge_src, const float* edge_w, int64_t n_dst,
                                 float* nv, float* wsum, void* stream);
int32_t rs_weighted_mean_agg_bwd(const float* grad_nv, int32_t H, const int32_t* t_indptr,
                                 const int32_t* t_edge, const int32_t* edge_dst,
                                 const float* edge_w, const float* wsum, int64_t n_src,
                                 float* grad_u, void* stream);

/* Global Frobenius normalisation y = x / ||x||_F (one scalar over the whole block,
 * pinsage/train/layers.py:28-29); norm [1] device. bwd: dx = (dy - y <dy, y>) / norm.
 * Fixed-partition reductions (deterministic). */
size_t rs_frobenius_workspace_size(int64_t n);
int32_t rs_frobenius_normalize_fwd(const float* x, int64_t n, float* y, float* norm,
                                   void* workspace, size_t ws_bytes, void* stream);
int32_t rs_frobenius_normalize_bwd(const float* dy, const float* y, const float* norm, int64_t n,
                                   float* dx, void* workspace, size_t ws_bytes, void* stream);
/* The same over a capacity-shaped [n_cap_rows, row_len] buffer whose first *n_rows (device
 * int32) rows are live (PinSageStep's sync-free batches): the norm / dot run over the live
 * rows only (bit-identical to the unpadded call), padding elements of y / dx are written 0.
 * Workspace: rs_frobenius_workspace_size(n_cap_rows * row_len). */
int32_t rs_frobenius_normalize_rows_fwd(const float* x, int64_t n_cap_rows, int32_t row_len,
                                        const int32_t* n_rows, float* y, float* norm,
                                        void* workspace, size_t ws_bytes, void* stream);
int32_t rs_frobenius_normalize_rows_bwd(const float* dy, const float* y, const float* norm,
                                        int64_t n_cap_rows, int32_t row_len,
                                        const int32_t* n_rows, float* dx, void* workspace,
                                        size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * EGES / GES / DeepWalk (eges/model.py).
 * Skip-gram logits, fused gather + dot (DeepWalk.call :26-36, GES.call :58-64):
 * logits[b, j] = out_table[match_ids[b, j]] · hidden[b] ([batch, n_match] ids, id_dtype as
 * rs_embedding_fwd; OOB ids read zero rows and set RS_ERRBIT_OOB). bwd: grad_rows
 * [batch*n_match, dim] = g[b, j] * hidden[b] (the output table's IndexedSlices values, position
 * order) and grad_hidden[b] = Σ_j g[b, j] * out_table[match_ids[b, j]]. */
int32_t rs_match_logits_fwd(const float* table, int64_t n_rows, int32_t dim,
                            const void* match_ids, int32_t id_dtype, int32_t n_match,
                            const float* hidden, int64_t batch, float* logits, int32_t* err_flag,
                            void* stream);
int32_t rs_match_logits_bwd(const float* table, int64_t n_rows, int32_t dim,
                            const void* match_ids, int32_t id_dtype, int32_t n_match,
                            const float* hidden, const float* grad_logits, int64_t batch,
                            float* grad_rows, float* grad_hidden, void* stream);
/* Side-information pooling over side [batch, n_side, dim]: weight_logits [batch, n_side] →
 * hidden = softmax(weight_logits) · side (EGES.get_hidden :92-102; attn [batch, n_side] saved,
 * may be NULL) or, with weight_logits NULL, hidden = (Σ_s side_s) / n_side (GES.get_hidden
 * :74-80). bwd: attn NULL selects the mean mode; grad_weight_logits is the softmax backward.
 * n_side <= 16. */
int32_t rs_side_pool_fwd(const float* side, const float* weight_logits, int64_t batch,
                         int32_t n_side, int32_t dim, float* hidden, float* attn, void* stream);
int32_t rs_side_pool_bwd(const float* side, const float* attn, const float* grad_hidden,
                         int64_t batch, int32_t n_side, int32_t dim, float* grad_side,
                         float* grad_weight_logits, void* stream);
/* The same over side rows at any layout: row s of example b at side + b*side_bstride +
 * s*side_sstride (floats; grad_side written at the same layout) — MMOE pools its experts' outputs
 * in the [E, B, H] order of the batched expert GEMMs (esmm/mmoe.py:88-96), no transpose pass.
 * A layout other than [batch, n_side, dim] needs dim % 4 == 0, dim <= 128, 16-byte rows. */
int32_t rs_side_pool_fwd_strided(const float* side, int64_t side_bstride, int64_t side_sstride,
                                 const float* weight_logits, int64_t batch, int32_t n_side,
                                 int32_t dim, float* hidden, float* attn, void* stream);
int32_t rs_side_pool_bwd_strided(const float* side, int64_t side_bstride, int64_t side_sstride,
                                 const float* attn, const float* grad_hidden, int64_t batch,
                                 int32_t n_side, int32_t dim, float* grad_side,
                                 float* grad_weight_logits, void* stream);
/* n_tasks (1..4) softmax poolings of the same side rows (MMOE: one gate per task over the same
 * expert outputs, esmm/mmoe.py:36-46), the side rows read once: hidden[t] [batch, dim] =
 * Σ_s softmax(weight_logits[t][b, :])[s] · side[b, s, :], attn[t] [batch, n_side] the weights
 * (logits rows logits_ld apart). Per task the same arithmetic as rs_side_pool_fwd. Side rows as
 * rs_side_pool_fwd_strided (16-byte aligned, dim % 4 == 0, dim <= 128). The task arrays are host
 * arrays read during the call. side_bias (optional, [n_side, dim], 16-byte aligned): the side rows
 * hold pre-activations z and are first replaced in place by relu(z + side_bias[s]) (MMOE's
 * batched expert layer's bias and relu), then pooled. */
int32_t rs_side_pool_fwd_multi(float* side, int64_t side_bstride, int64_t side_sstride,
                               int64_t batch, int32_t n_side, int32_t dim, int32_t n_tasks,
                               const float* const* weight_logits, int64_t logits_ld,
                               float* const* hidden, float* const* attn, const float* side_bias,
                               void* stream);
/* Backward of rs_side_pool_fwd_multi: grad_side = Σ_t attn[t][s] · grad_hidden[t] (task order,
 * each product rounded: the sum of n_tasks rs_side_pool_bwd results), grad_logits[t] as
 * rs_side_pool_bwd's (rows grad_logits_ld apart). One pass over the side rows. */
int32_t rs_side_pool_bwd_multi(const float* side, int64_t side_bstride, int64_t side_sstride,
                               int64_t batch, int32_t n_side, int32_t dim, int32_t n_tasks,
                               const float* const* attn, const float* const* grad_hidden,
                               float* grad_side, float* const* grad_logits,
                               int64_t grad_logits_ld, void* stream);

/* ------------------------------------------------------------------------------------
 * Factored linear-chain backward of a ctr MLP (hidden Dense layers linear, ctr/layers.py:8):
 * with G = act'(y) ⊙ dy (act 0 linear, 1 relu, 2 sigmoid on the output y [B, nl]),
 * out[0 .. n0*nl) = xᵀ·G (row-major [n0, nl]), out[n0*nl ..] = Σ_b G; x [B, n0] with row
 * stride ldx; g_out (may be NULL) receives G. Shapes: nl == 1 and n0 <= 1024, or nl <= 256
 * and n0 <= 32 (nl == 1 also needs n0, ldx multiples of 4 and a 16-B aligned x). Deterministic
 * (fixed row chunks folded in order). */
size_t rs_chain_reduce_workspace_size(int64_t B, int32_t n0, int32_t nl);
int32_t rs_chain_reduce(const float* x, int64_t ldx, int32_t n0, const float* dy, const float* y,
                        int32_t nl, int32_t act, int64_t B, float* out, float* g_out,
                        void* workspace, size_t ws_bytes, void* stream);

/* Parameter gradients of a 3-layer linear chain with a scalar output ([n1, n2, 1], e.g. the
 * DLRM / DeepFM top MLP) from A = xᵀ·G [n0] and s = Σ G [1] (rs_chain_reduce): kernels
 * K1 [n_full0, n1] (the input holds rows[n0] of it, inv[n_full0] = position in rows or -1;
 * both NULL: all rows), K2 [n1, n2], K3 [n2]; biases b1, b2 may be NULL. Writes dK1
 * [n_full0, n1] (zero rows outside `rows`), db1, dK2 [n1, n2], db2, dK3 [n2], db3 [1] and
 * p [n0] = K1[rows]·K2·K3 (the input gradient is G ⊗ p). Workspace >= 4·(2·n1 + 2·n2) bytes. */
int32_t rs_chain3_vec_grads(const float* K1, const int32_t* rows, const int32_t* inv,
                            int32_t n_full0, int32_t n0, const float* b1, const float* K2,
                            const float* b2, const float* K3, int32_t n1, int32_t n2,
                            const float* A, const float* s, float* dK1, float* db1, float* dK2,
                            float* db2, float* dK3, float* db3, float* p, void* workspace,
                            size_t ws_bytes, void* stream);

/* Composed forward of a ctr linear chain (hidden Dense layers linear, ctr/layers.py:8; replaces
 * the layer-by-layer Dense calls of ctr/layers.py:11-14): the chain is the one affine map
 * y = act(x·Q_0 + c_L).
 * rs_chain3_vec_compose: [n1, n2, 1] chain (the DLRM / DeepFM top MLP): q [n0] = K1[rows]·K2·K3
 *   (rows NULL: rows 0..n0) and c [1] = b3 + K3ᵀ·b2 + (K2·K3)ᵀ·b1 (biases may be NULL).
 *   Workspace >= 4·(n1 + 1) bytes.
 * rs_chain_aug_product: out [m+1, n] = [M; cin]·K + [0; b] with M [m, k] (row stride ldm, m < 33,
 *   (m+1)·k <= 16896), cin [k] and b [n] optional; two calls compose a narrow-input chain [K1; b1]·K2 + [0; b2],
 *   then ·K3 + [0; b3] = [Q_0; c_L].
 * rs_affine_narrow_fwd: y [B, n] (row stride ldy) = act(x·Qa[0:n0] + Qa[n0]) for x [B, n0]
 *   (n0 < 33, n <= 256, n % 4 == 0, Qa and y 16-B aligned).
 * rs_rowdot_act: y [B] = act(x·q + c[0]) for x [B, n0] (n0 <= 1024, n0 % 4 == 0, ldx % 4 == 0,
 *   x and q 16-B aligned). act: 0 linear, 1 relu, 2 sigmoid. */
int32_t rs_chain3_vec_compose(const float* K1, const int32_t* rows, int32_t n0, const float* b1,
                              const float* K2, const float* b2, const float* K3, const float* b3,
                              int32_t n1, int32_t n2, float* q, float* c, void* workspace,
                              size_t ws_bytes, void* stream);
int32_t rs_chain_aug_product(const float* M, int32_t ldm, int32_t m, const float* cin,
                             const float* K, int32_t k, int32_t n, const float* b, float* out,
                             void* stream);
int32_t rs_affine_narrow_fwd(const float* x, int64_t ldx, int64_t B, int32_t n0, const float* Qa,
                             int32_t n, int32_t act, float* y, int64_t ldy, void* stream);
int32_t rs_rowdot_act(const float* x, int64_t ldx, int64_t B, int32_t n0, const float* q,
                      const float* c, int32_t act, float* y, void* stream);

/* Parameter gradients of a narrow-input linear chain from Ã = [xᵀ·G; Σ G] ([n0+1, nL], the
 * rs_chain_reduce output): P_L = Ã, P_{j-1} = P_j·K_jᵀ, dK_j = R̃_{j-1}ᵀ·P_j, db_j = P_j[n0]
 * with R̃_j = [K_1···K_j; c_j] (rs_chain_aug_product's outputs; R̃_0 = [I; 0]).
 * rs_chain_rt_product: out [m+1, n] = P [m+1, k]·Kᵀ for K [n, k] row-major (m < 33,
 *   (m+1)·k <= 16896).
 * rs_chain_outer: out [na, nb] = R̃ᵀ·P with R̃ = [R (m rows, row stride ldr); rlast] (rlast
 *   NULL: zero row), P [m+1, nb] (nb % 4 == 0; P and out 16-B aligned). */
int32_t rs_chain_rt_product(const float* P, int32_t m, const float* K, int32_t k, int32_t n,
                            float* out, void* stream);
int32_t rs_chain_outer(const float* R, int32_t ldr, int32_t m, const float* rlast, int32_t na,
                       const float* P, int32_t nb, float* out, void* stream);

/* ------------------------------------------------------------------------------------
 * Keras thresholded AUC (keras.metrics.AUC in ctr/train.py:86,
 * dien/train.py:43-44, esmm/train.py:164). thresholds [n_thresholds] ascending float32 (the
 * Keras grid: -eps, i/(T-1) for i = 1..T-2, 1+eps); counts [2, n_thresholds+1] int64,
 * accumulated: counts[label != 0][#thresholds < pred] += 1 (a prediction outside [0, 1]
 * sets RS_ERRBIT_OOB, as Keras asserts). TP_i = Σ_{b > i} counts[1][b], FP_i likewise. */
int32_t rs_auc_update(const float* pred, const float* label, int64_t n, const float* thresholds,
                      int32_t n_thresholds, unsigned long long* counts, int32_t* err_flag,
                      void* stream);

/* ------------------------------------------------------------------------------------
 * Criteo TSV ingestion (ctr/tfrecord_io.py:15-96), text resident in HBM.
 * rs_line_index: line_starts [n_newlines + 1] int64 (line 0 at byte 0, line k after the k-th
 *   '\n'); *n_newlines device int32; line_starts NULL = count only.
 * rs_criteo_parse: per line "label \t n_int ints \t n_cat tokens": label [n_lines] f32,
 *   dense [n_lines, n_int] = logf(max(int, 0) + 1) (''/negative → 0, tfrecord_io.py:47-53),
 *   hashes [n_lines, n_cat] = FNV-1a 64 of each token (empty → the column's imputation token,
 *   :24-25; the last token keeps the line's '\n' as Python's split does); a line with the
 *   wrong field count sets RS_ERRBIT_OOB and yields zeros / imputation tokens.
 * rs_vocab_count: open-addressing table (capacity a power of two; keys filled with 0xFF,
 *   counts / first_pos with 0 / 0xFF by the caller): count += 1, first_pos = min(pos_base + i)
 *   (the reference dict's insertion order, :15-30).
 * rs_vocab_collect: slots with count > min_count (10, :33) → first_out / slot_out (slot
 *   order), *n_kept; the caller sorts them by first position and rs_vocab_assign gives slot
 *   sorted_slots[r] the id r (ids pre-filled with -1).
 * rs_vocab_lookup: id of every token, 0 when absent (OOV → 0, :64-67). */
size_t rs_line_index_workspace_size(int64_t n_bytes);
int32_t rs_line_index(const uint8_t* text, int64_t n_bytes, int64_t* line_starts,
                      int32_t* n_newlines, void* workspace, size_t ws_bytes, void* stream);
int32_t rs_criteo_parse(const uint8_t* text, int64_t n_bytes, const int64_t* line_starts,
                        int64_t n_lines, int32_t n_int, int32_t n_cat, float* label, float* dense,
                        uint64_t* hashes, int32_t* err_flag, void* stream);
int32_t rs_vocab_count(const uint64_t* hashes, int64_t n, int64_t pos_base, uint64_t* keys,
                       uint32_t* counts, uint64_t* first_pos, int64_t capacity, int32_t* err_flag,
                       void* stream);
size_t rs_vocab_collect_workspace_size(int64_t capacity);
int32_t rs_vocab_collect(const uint64_t* keys, const uint32_t* counts, const uint64_t* first_pos,
                         int64_t capacity, uint32_t min_count, uint64_t* first_out,
                         int32_t* slot_out, int32_t* n_kept, void* workspace, size_t ws_bytes,
                         void* stream);
int32_t rs_vocab_assign(const int32_t* sorted_slots, int64_t n_kept, int32_t* ids, void* stream);
int32_t rs_vocab_lookup(const uint64_t* hashes, int64_t n, const uint64_t* keys,
                        const int32_t* ids, int64_t capacity, int64_t* out, void* stream);

/* ------------------------------------------------------------------------------------
 * EGES training pairs (eges/data_loader.py:28-62), Philox-keyed draws.
 * rs_eges_walks: walk i (global walk_base + i) starts at 1 + U[0, n_items-1) and takes `length`
 *   weighted steps (dgl random_walk prob='weight': edge e of v with probability w_e / W_v;
 *   cumw = per-node inclusive float64 prefix of the CSR edge weights); traces
 *   [n_walks, length+1], -1 after a dead end.
 * rs_skipgram_pairs: keras skipgrams(window, negative_samples=0) over every trace (pairs of
 *   items > 0 in enumeration order, no shuffle): target / context [≤ n_traces*slots],
 *   *n_pairs.
 * rs_log_uniform_sample: log_uniform_candidate_sampler(num_sampled, unique=True, range_max):
 *   cdf [range_max] uint32 = floor(log(k+2)/log(range_max+1)·2^32); out [n_pairs, num_sampled].
 * rs_csr_weight_prefix: cumw[e] = Σ_{lo(v) ≤ f ≤ e} w[f] per node v (sequential float64). */
int32_t rs_csr_weight_prefix(const int64_t* indptr, const float* weights, int64_t n_nodes,
                             double* cumw, void* stream);
int32_t rs_eges_walks(const int64_t* indptr, const int32_t* indices, const double* cumw,
                      int32_t n_items, int64_t walk_base, int32_t n_walks, int32_t length,
                      uint64_t seed, uint32_t step, int32_t* traces, void* stream);
size_t rs_skipgram_workspace_size(int32_t n_traces, int32_t len, int32_t window);
int32_t rs_skipgram_pairs(const int32_t* traces, int32_t n_traces, int32_t len, int32_t window,
                          int32_t* target, int32_t* context, int32_t* n_pairs, void* workspace,
                          size_t ws_bytes, void* stream);
int32_t rs_log_uniform_sample(const uint32_t* cdf, int32_t range_max, int64_t pair_base,
                              int32_t n_pairs, int32_t num_sampled, uint64_t seed, uint32_t step,
                              int32_t* out, int32_t* err_flag, void* stream);

/* ------------------------------------------------------------------------------------
 * PinSage evaluation (pinsage/train/evaluation.py:27-65).
 * rs_latest_item: per user the item of its latest u2i edge by timestamp (select_topk(k=1),
 *   evaluation.py:33-34; ties → smaller item id); -1 and ++*n_missing for users without edges.
 * rs_masked_topk: rows r of scores [n_rows, ld] (user user_base + r) → the k best items
 *   (score desc, item asc) after setting the user's excl CSR items to -inf (:41-46); k ≤ 64,
 *   n_items ≤ 2^20. out_scores may be NULL.
 * rs_hit_flags: hit[r] = any(recs[r, :] ∈ truth CSR row of user user_base + r) (:54-65). */
int32_t rs_latest_item(const int64_t* u2i_indptr, const int32_t* u2i_items,
                       const int64_t* timestamps, int64_t n_users, int32_t* latest,
                       int32_t* n_missing, void* stream);
int32_t rs_masked_topk(const float* scores, int64_t ld, int32_t n_rows, int32_t n_items,
                       int64_t user_base, const int64_t* excl_indptr, const int32_t* excl_items,
                       int32_t k, int32_t* out_items, float* out_scores, void* stream);
int32_t rs_hit_flags(const int32_t* recs, int64_t n_rows, int32_t k, int64_t user_base,
                     const int64_t* truth_indptr, const int32_t* truth_items, int32_t* hit,
                     void* stream);

/* ------------------------------------------------------------------------------------
 * Ali-CCP and Amazon (DIEN) text → ids (esmm/process_public_dataset.py:40-153,
 * dien/util.py:4-37, dien/data_loader.py:27-63). Lines come from rs_line_index; each line is
 * str.strip()ped as the reference does.
 * rs_vocab_count_masked: rs_vocab_count over the entries with present[i] != 0.
 * rs_kv_parse: CSV line, field kv_field holds re.split('\x01|\x02|\x03') (field, value, weight)
 *   triples; vals [n_lines, n_cols] = FNV-1a 64 of the LAST value of field col_hashes[c]
 *   (dict(zip) semantics), present [n_lines, n_cols]; key_hash [n_lines] = hash of field
 *   key_field (may be NULL); with_labels: labels [n_lines, 2] = int fields 1, 2 and keep = not
 *   (field 1 == "0" and field 2 == "1") (:56). A line with too few fields sets RS_ERRBIT_OOB.
 * rs_map_insert: key_hash[i] → i in a (keys ~0, vals -1 filled) table; a later i wins.
 * rs_aliccp_join: kept skeleton lines compacted in order (*n_kept): out_keys [n_kept, n_cols] =
 *   (column, value) hash with the common line's value overriding (:60), '0' when absent;
 *   out_present; out_labels [n_kept, 2]. An unknown common id sets RS_ERRBIT_OOB (KeyError).
 * rs_vocab_regroup: sort_key = (first % n_groups) * per_group + first / n_groups, group.
 * rs_vocab_assign_grouped: ids[slots[order[r]]] = id_base + r - (first rank of r's group); order
 *   and group may be NULL (identity order, one group).
 * rs_vocab_lookup_i32: ids as int32, oov_id when absent (RS_ERRBIT_OOB too if err_on_oov).
 * rs_dien_parse: line "label\tuser\titem\tcat\this_items\this_cats", histories '\x02'-separated.
 *   Count pass (item_off NULL): n_hi, n_hc [n_lines] token counts, label. Fill pass: item_hash at
 *   item_off[l] (target) and item_off[l] + 1 + k (history k), cat_hash likewise at cat_off.
 * rs_dien_item_cat: cat_of_item[id] = cat id of the item's LAST (item, cat) pair in the stream
 *   (target pair, then zip(history)), -1 for an item without one.
 * rs_dien_encode: target_item / his_item ids (unknown → unk_item), target_cat / his_cat (unknown →
 *   0 + RS_ERRBIT_OOB, the reference's KeyError); histories keep the LAST maxlen tokens, zero-padded
 *   after (pad_sequences padding='post', truncating='pre'); neg_item (may be NULL) = 1 +
 *   U[0, n_item_ids - 1) by Philox (seed, line_base + l, position), neg_cat = cat_of_item. */
int32_t rs_vocab_count_masked(const uint64_t* hashes, const uint8_t* present, int64_t n,
                              int64_t pos_base, uint64_t* keys, uint32_t* counts,
                              uint64_t* first_pos, int64_t capacity, int32_t* err_flag,
                              void* stream);
int32_t rs_kv_parse(const uint8_t* text, int64_t n_bytes, const int64_t* line_starts,
                    int64_t n_lines, int32_t key_field, int32_t kv_field, int32_t with_labels,
                    const uint64_t* col_hashes, int32_t n_cols, uint64_t* key_hash, int32_t* keep,
                    int32_t* labels, uint64_t* vals, uint8_t* present, int32_t* err_flag,
                    void* stream);
int32_t rs_map_insert(const uint64_t* key_hash, int64_t n, uint64_t* keys, int32_t* vals,
                      int64_t capacity, int32_t* err_flag, void* stream);
size_t rs_aliccp_join_workspace_size(int64_t n_lines);
int32_t rs_aliccp_join(const int32_t* keep, int64_t n_lines, int32_t n_cols,
                       const uint64_t* common_id, const uint64_t* skel_vals,
                       const uint8_t* skel_present, const int32_t* skel_labels,
                       const uint64_t* map_keys, const int32_t* map_vals, int64_t map_capacity,
                       const uint64_t* common_vals, const uint8_t* common_present,
                       uint64_t* out_keys, uint8_t* out_present, int32_t* out_labels,
                       int32_t* n_kept, int32_t* err_flag, void* workspace, size_t ws_bytes,
                       void* stream);
int32_t rs_vocab_regroup(const uint64_t* first_pos, int64_t n, int32_t n_groups, int64_t per_group,
                         int64_t* sort_key, int32_t* group, void* stream);
int32_t rs_vocab_assign_grouped(const int32_t* order, const int32_t* slots, const int32_t* group,
                                int64_t n_kept, int32_t id_base, int32_t* ids, void* stream);
int32_t rs_vocab_lookup_i32(const uint64_t* hashes, int64_t n, const uint64_t* keys,
                            const int32_t* ids, int64_t capacity, int32_t oov_id,
                            int32_t err_on_oov, int32_t* out, int32_t* err_flag, void* stream);
int32_t rs_dien_parse(const uint8_t* text, int64_t n_bytes, const int64_t* line_starts,
                      int64_t n_lines, const int64_t* item_off, const int64_t* cat_off,
                      int32_t* n_hi, int32_t* n_hc, float* label, uint64_t* item_hash,
                      uint64_t* cat_hash, int32_t* err_flag, void* stream);
size_t rs_dien_item_cat_workspace_size(int64_t item_capacity);
int32_t rs_dien_item_cat(const uint64_t* item_hash, const uint64_t* cat_hash,
                         const int64_t* item_off, const int64_t* cat_off, const int32_t* n_hi,
                         const int32_t* n_hc, int64_t n_lines, const uint64_t* item_keys,
                         const int32_t* item_ids, int64_t item_capacity, const uint64_t* cat_keys,
                         const int32_t* cat_ids, int64_t cat_capacity, int32_t* cat_of_item,
                         void* workspace, size_t ws_bytes, void* stream);
int32_t rs_dien_encode(const uint64_t* item_hash, const uint64_t* cat_hash,
                       const int64_t* item_off, const int64_t* cat_off, const int32_t* n_hi,
                       const int32_t* n_hc, int64_t n_lines, const uint64_t* item_keys,
                       const int32_t* item_ids, int64_t item_capacity, int32_t unk_item,
                       const uint64_t* cat_keys, const int32_t* cat_ids, int64_t cat_capacity,
                       int32_t maxlen, const int32_t* cat_of_item, int32_t n_item_ids,
                       uint64_t seed, int64_t line_base, int32_t* target_item, int32_t* target_cat,
                       int32_t* his_item, int32_t* his_cat, int32_t* neg_item, int32_t* neg_cat,
                       int32_t* err_flag, void* stream);

/* ---- Criteo TFRecord reader (replaces ctr/tfrecord_io.py:78-96
 * read_tfrecord: tf.data.TFRecordDataset + parse_single_example + parse_tensor) ------------
 * rs_tfrecord_index (HOST memory, host code): walks the TFRecord framing of data[0, n_bytes)
 *   (uint64 length, masked CRC32C of it, payload, masked CRC32C of the payload), checking the
 *   length CRCs when verify_crc; writes up to `capacity` record offsets (of the length field)
 *   and payload lengths; *n_records = the count. Corrupt framing -> RS_E_INVALID.
 * rs_tfrecord_parse_criteo (DEVICE memory, stream-ordered): one tf.train.Example per record
 *   with 'int_features' / 'cat_features' = tf.io.serialize_tensor of float32 [n_int] / int64
 *   [n_cat] (tensor_content or packed float_val / int64_val) and 'label' = int64_list; any
 *   field order, unknown fields skipped. verify_crc: the payload CRC32C is checked too.
 *   Outputs int_features [n, n_int] f32, cat_features [n, n_cat] i64, label [n] i64; a
 *   malformed record (bad CRC, shape or dtype, missing key, payload > 4096 B) is zeroed and sets
 *   RS_ERRBIT_FORMAT in err_flag (may be NULL). */
/* rs_crc32c_masked (HOST memory): the TFRecord masked CRC32C of data[0, n_bytes) (writer side). */
int32_t rs_crc32c_masked(const uint8_t* data, int64_t n_bytes, uint32_t* out);
int32_t rs_tfrecord_index(const uint8_t* data, int64_t n_bytes, int32_t verify_crc,
                          int64_t* offsets, int32_t* lengths, int64_t capacity, int64_t* n_records);
int32_t rs_tfrecord_parse_criteo(const uint8_t* data, const int64_t* offsets,
                                 const int32_t* lengths, int64_t n_records, int32_t n_int,
                                 int32_t n_cat, int32_t verify_crc, float* int_features,
                                 int64_t* cat_features, int64_t* label, int32_t* err_flag,
                                 void* stream);

/* ---- the production DLRM training step's top half in one pass (D = 128, <= 27 slots, 13
 * dense inputs, sigmoid head, Keras BCE; ctr/model.py:45-57 + ctr/train.py:77-85) ------------
 * Gathers X = [emb(ids), dense], Z = X·Xᵀ, y = σ(Σ q·[Z_strict_upper, dense] + c) (q, c: the
 * composed top MLP, rs_chain3_vec_compose), the BCE loss against label (eps clip, scaled by
 * loss_scale), G_b = y(1-y)·dL/dy, the table gradient rows G_b·(M + Mᵀ)·X_b (M = the
 * strict-upper pair weights of q, written unit-scaled: below) in position order, y [B], and the
 * deterministic batch sums (fixed per-wave / per-block / two-level fold order) into
 * sums [rs_dlrm_train_sums()] = A_top [512] (Σ_b row_b·G_b over the compact row, zero padded)
 * | s_top = Σ G | loss sum | A_bot [13][128] = Σ_b x_bᵀ·g_b | s_bot [128] = Σ_b g_b, where
 * g_b = relu'(dense_b) ⊙ G_b·((M + Mᵀ)·X_b + q_dense)[row S] is the bottom MLP's last-layer
 * gradient and x = xin [B, 13] its input. */
size_t rs_dlrm_train_workspace_size(int64_t batch);
/* The table gradient rows are written UNIT-scaled: unit_rows[b, i] = U_b[i] (the interaction
 * backward's (M + Mᵀ)·X_b row) and g_rows[b] = G_b, so the gradient row of position p is
 * g_rows[p / n_slots] * unit_rows[p] — hand both to rs_embedding_apply_scaled (row_scale =
 * g_rows, scale_group = n_slots), which forms that product with one fmul_rn. The kernel computes
 * the interaction chunk by chunk (U written before the head's G is known), which is why the rows
 * leave it unscaled. loss_scale is dL/dl_b: 1/batch for the mean loss; a data-parallel rank
 * holding `batch` of a global batch of B examples passes 1/B, so G, the rows and every batch sum
 * are those of the global mean loss and the ranks' sums add up to the global ones. */
int32_t rs_dlrm_train_step_fwd_unit(const float* table, int64_t n_rows, int32_t D,
                                    const void* ids, int32_t id_dtype, int32_t n_slots,
                                    const int64_t* slot_offsets, const float* dense,
                                    const float* xin, int32_t n_in, const float* label,
                                    int64_t batch, const float* q, const float* c, float eps,
                                    float loss_scale, float* y, float* unit_rows, float* g_rows,
                                    float* sums, void* workspace, size_t ws_bytes,
                                    int32_t* err_flag, void* stream);
/* The same step in two calls (round 6): _nofold runs the kernel only (y, unit_rows and g_rows are
 * final after it; the per-block partial sums stay in the workspace), rs_dlrm_train_fold folds them
 * into sums — bit-identical to the one-call form. The production step orders its sparse update
 * after the kernel alone and folds on its own stream meanwhile. */
int32_t rs_dlrm_train_step_fwd_unit_nofold(const float* table, int64_t n_rows, int32_t D,
                                           const void* ids, int32_t id_dtype, int32_t n_slots,
                                           const int64_t* slot_offsets, const float* dense,
                                           const float* xin, int32_t n_in, const float* label,
                                           int64_t batch, const float* q, const float* c,
                                           float eps, float loss_scale, float* y,
                                           float* unit_rows, float* g_rows, void* workspace,
                                           size_t ws_bytes, int32_t* err_flag, void* stream);
int32_t rs_dlrm_train_fold(const void* workspace, size_t ws_bytes, int64_t batch, int32_t D,
                           int32_t id_dtype, float* sums, void* stream);

/* ---- the production DLRM step's dense tail (ctr/train.py:77-79 SGD of every MLP parameter;
 * ctr/layers.py:5-14 linear hidden layers) ------------------------------------------------
 * From the train step's sums: every kernel / bias gradient of the top chain [top_n0 rows of
 * top_k[0] (top_rows / top_inv as rs_chain3_vec_grads) -> n1 -> n2 -> 1] and of the narrow
 * bottom chain [bot_n0 -> n1 -> n2 -> n3] (P = [A_bot; s_bot], bot_comp2 = the current
 * [K1·K2; c2] of rs_chain_aug_product), then param -= lr·grad for all twelve parameters
 * (torch.optim.SGD's foreach update), then the next step's compositions from the updated
 * parameters: bot_comp2_next = [K1·K2; c2], bot_comp3_next = [K1·K2·K3; c3] (rs_chain_aug_product
 * x 2) and top_q [n0], top_c [1] (rs_chain3_vec_compose). Bottom gradients: dK3 -> bot_dk3,
 * dK2 -> bot_dk2, bot_P2 [n0+1, n2] (row n0 = db2), bot_P1 [n0+1, n1] (rows 0..n0-1 = dK1,
 * row n0 = db1), db3 = P row n0. Six stream-ordered launches; each value equals the separate
 * rs_chain3_vec_grads / rs_chain_outer / rs_chain_rt_product / rs_chain_aug_product /
 * rs_chain3_vec_compose calls bit for bit. */
typedef struct rs_dlrm_tail_args {
  float* top_k[3];
  float* top_b[3];
  const int32_t* top_rows;
  const int32_t* top_inv;
  int32_t top_n_full0, top_n0, top_n1, top_n2;
  const float* top_A; /* [top_n0] */
  const float* top_s; /* [1] */
  float* top_dk[3];
  float* top_db[3];
  float* top_q; /* [top_n0] next-step composition */
  float* top_c; /* [1] */
  float* bot_k[3];
  float* bot_b[3];
  int32_t bot_n0, bot_n1, bot_n2, bot_n3;
  const float* bot_P;     /* [bot_n0 + 1, bot_n3] */
  const float* bot_comp2; /* [bot_n0 + 1, bot_n2] */
  float* bot_dk2;         /* [bot_n1, bot_n2] */
  float* bot_dk3;         /* [bot_n2, bot_n3] */
  float* bot_P2;          /* [bot_n0 + 1, bot_n2] */
  float* bot_P1;          /* [bot_n0 + 1, bot_n1] */
  float* bot_comp2_next;  /* [bot_n0 + 1, bot_n2] */
  float* bot_comp3_next;  /* [bot_n0 + 1, bot_n3] */
  float lr;
} rs_dlrm_tail_args;
size_t rs_dlrm_dense_tail_workspace_size(int32_t top_n0, int32_t top_n1, int32_t top_n2);
int32_t rs_dlrm_dense_tail(const rs_dlrm_tail_args* args, void* workspace, size_t ws_bytes,
                           void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RECSYS_HIP_H */
