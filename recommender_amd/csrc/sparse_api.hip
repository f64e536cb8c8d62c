// sparse_api.hip — the one-call sparse-gradient entry points named in SURVEY §8(b):
//   rs_embedding_bwd_dedup   ids + grad rows -> (unique rows, summed grads, count)
//   rs_apply_sgd             var[u] -= lr * Σ g  (SGD _resource_apply_sparse_duplicate_indices)
//   rs_apply_lazy_adam       Keras Adam on the touched rows only
//   rs_apply_keras_dense_adam  exact Keras Adam (touched-row update + dense m/v decay sweep)
// Each is rs_sort_ids followed by rs_embedding_dedup_grad / rs_embedding_apply (and
// rs_keras_adam_dense_sweep) with one caller workspace (rs_sparse_workspace_size): the same
// kernels, the same summation order, so results are bit-identical to the two-call form.
#include "common.hpp"

extern "C" size_t rs_sort_ids_workspace_size(int64_t n_ids);
extern "C" size_t rs_dedup_workspace_size(int64_t n_ids, int32_t dim);
extern "C" size_t rs_apply_workspace_size(int64_t n_ids, int32_t dim);

namespace {

struct SortedScratch {
  uint32_t* rows;
  int32_t* pos;
  void* rest;
  size_t rest_bytes;
};

size_t sorted_head(int64_t n) {
  rs::Carver c(nullptr, 0);
  c.take<uint32_t>(n);
  c.take<int32_t>(n);
  return rs::align_up(c.off, 256);
}

bool carve(void* ws, size_t bytes, int64_t n, SortedScratch& s) {
  const size_t head = sorted_head(n);
  if (!ws || bytes < head) return false;
  rs::Carver c(ws, bytes);
  s.rows = c.take<uint32_t>(n);
  s.pos = c.take<int32_t>(n);
  s.rest = static_cast<char*>(ws) + head;
  s.rest_bytes = bytes - head;
  return true;
}

int32_t sort_into(const void* ids, int32_t id_dtype, int64_t n, const int64_t* slot_offsets,
                  int32_t n_slots, int64_t n_rows, SortedScratch& s, int32_t* n_unique,
                  int32_t* err_flag, void* stream) {
  return rs_sort_ids(ids, id_dtype, n, slot_offsets, n_slots, n_rows, s.rows, s.pos, n_unique,
                     err_flag, s.rest, s.rest_bytes, stream);
}

}  // namespace

extern "C" size_t rs_sparse_workspace_size(int64_t n_ids, int32_t dim) {
  size_t a = rs_sort_ids_workspace_size(n_ids), b = rs_dedup_workspace_size(n_ids, dim),
         c = rs_apply_workspace_size(n_ids, dim);
  size_t m = a > b ? a : b;
  m = m > c ? m : c;
  return sorted_head(n_ids) + m;
}

extern "C" int32_t rs_embedding_bwd_dedup(const void* ids, int32_t id_dtype, int64_t n_ids,
                                          const int64_t* slot_offsets, int32_t n_slots,
                                          int64_t n_rows, const float* grad_out, int32_t dim,
                                          uint32_t* uniq_rows, float* uniq_grad,
                                          int32_t* n_unique, int32_t* err_flag, void* workspace,
                                          size_t ws_bytes, void* stream) {
  SortedScratch s;
  RS_CHECK_ARG(carve(workspace, ws_bytes, n_ids, s), "rs_embedding_bwd_dedup: workspace too small");
  int32_t st = sort_into(ids, id_dtype, n_ids, slot_offsets, n_slots, n_rows, s, n_unique,
                         err_flag, stream);
  if (st) return st;
  return rs_embedding_dedup_grad(s.rows, s.pos, n_ids, grad_out, dim, n_rows, uniq_rows,
                                 uniq_grad, s.rest, s.rest_bytes, stream);
}

static int32_t apply_common(int32_t opt, float* table, float* m, float* v, int64_t n_rows,
                            int32_t dim, const void* ids, int32_t id_dtype, int64_t n_ids,
                            const int64_t* slot_offsets, int32_t n_slots, const float* grad_out,
                            const rs_adam_params* params, uint32_t* bitmap, int32_t* err_flag,
                            void* workspace, size_t ws_bytes, void* stream) {
  SortedScratch s;
  RS_CHECK_ARG(carve(workspace, ws_bytes, n_ids, s), "sparse apply: workspace too small");
  int32_t st = sort_into(ids, id_dtype, n_ids, slot_offsets, n_slots, n_rows, s, nullptr,
                         err_flag, stream);
  if (st) return st;
  return rs_embedding_apply(opt, table, m, v, n_rows, dim, s.rows, s.pos, n_ids, grad_out, params,
                            bitmap, s.rest, s.rest_bytes, stream);
}

extern "C" int32_t rs_apply_sgd(float* table, int64_t n_rows, int32_t dim, const void* ids,
                                int32_t id_dtype, int64_t n_ids, const int64_t* slot_offsets,
                                int32_t n_slots, const float* grad_out, float lr,
                                int32_t* err_flag, void* workspace, size_t ws_bytes,
                                void* stream) {
  rs_adam_params p{lr, 0.f, 0.f, 0.f, 0.f, 0.f};
  return apply_common(RS_OPT_SGD, table, nullptr, nullptr, n_rows, dim, ids, id_dtype, n_ids,
                      slot_offsets, n_slots, grad_out, &p, nullptr, err_flag, workspace, ws_bytes,
                      stream);
}

extern "C" int32_t rs_apply_lazy_adam(float* table, float* m, float* v, int64_t n_rows,
                                      int32_t dim, const void* ids, int32_t id_dtype,
                                      int64_t n_ids, const int64_t* slot_offsets, int32_t n_slots,
                                      const float* grad_out, const rs_adam_params* params,
                                      int32_t* err_flag, void* workspace, size_t ws_bytes,
                                      void* stream) {
  RS_CHECK_ARG(m && v && params, "rs_apply_lazy_adam: m, v and params are required");
  return apply_common(RS_OPT_LAZY_ADAM, table, m, v, n_rows, dim, ids, id_dtype, n_ids,
                      slot_offsets, n_slots, grad_out, params, nullptr, err_flag, workspace,
                      ws_bytes, stream);
}

extern "C" int32_t rs_apply_keras_dense_adam(float* table, float* m, float* v, int64_t n_rows,
                                             int32_t dim, const void* ids, int32_t id_dtype,
                                             int64_t n_ids, const int64_t* slot_offsets,
                                             int32_t n_slots, const float* grad_out,
                                             const rs_adam_params* params,
                                             uint32_t* touched_bitmap, int32_t* err_flag,
                                             void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(m && v && params && touched_bitmap,
               "rs_apply_keras_dense_adam: m, v, params and the touched bitmap are required");
  int32_t st = apply_common(RS_OPT_KERAS_ADAM, table, m, v, n_rows, dim, ids, id_dtype, n_ids,
                            slot_offsets, n_slots, grad_out, params, touched_bitmap, err_flag,
                            workspace, ws_bytes, stream);
  if (st) return st;
  return rs_keras_adam_dense_sweep(table, m, v, n_rows, dim, params, touched_bitmap, stream);
}

// Deterministic index_add (the backward of a row gather): rs_sort_ids_masked over the ids (one
// shared table of n_rows rows), then rs_embedding_grad_dense — out zeroed, each touched row the
// tiled fixed-order sum of its rows.
extern "C" size_t rs_index_add_rows_workspace_size(int64_t n, int32_t dim) {
  const int64_t m = n < 1 ? 1 : n;
  size_t a = rs_sort_ids_workspace_size(m), c = rs_apply_workspace_size(m, dim);
  return sorted_head(m) + (a > c ? a : c);
}

extern "C" int32_t rs_index_add_rows(const void* ids, int32_t id_dtype, int64_t n,
                                     const uint8_t* valid, const float* rows, int32_t dim,
                                     int64_t n_rows, float* out, int32_t* err_flag,
                                     void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(n >= 0 && dim >= 1 && n_rows >= 1, "rs_index_add_rows: bad sizes");
  RS_CHECK_ARG(out && (n == 0 || (ids && rows)), "rs_index_add_rows: null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_index_add_rows_workspace_size(n, dim),
               "rs_index_add_rows: workspace too small");
  SortedScratch s;
  RS_CHECK_ARG(carve(workspace, ws_bytes, n < 1 ? 1 : n, s), "rs_index_add_rows: workspace too small");
  if (n > 0) {
    const int32_t st = valid ? rs_sort_ids_masked(ids, id_dtype, n, valid, nullptr, 1, n_rows,
                                                  s.rows, s.pos, nullptr, err_flag, s.rest,
                                                  s.rest_bytes, stream)
                             : rs_sort_ids(ids, id_dtype, n, nullptr, 1, n_rows, s.rows, s.pos,
                                           nullptr, err_flag, s.rest, s.rest_bytes, stream);
    if (st) return st;
  }
  return rs_embedding_grad_dense(s.rows, s.pos, n, rows, dim, n_rows, out, s.rest, s.rest_bytes,
                                 stream);
}
