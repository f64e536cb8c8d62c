// metrics.hip — Keras thresholded AUC on device (keras.metrics.AUC used by
// ctr/train.py:86, dien/train.py:43-44, esmm/train.py:164, eges/train.py:91).
//
// [3p TF 2.2] metrics_utils.update_confusion_matrix_variables: for every threshold t_i,
// TP_i += Σ [y] [p > t_i], FP_i += Σ [!y] [p > t_i] (TN / FN the complements). Every
// prediction falls in ONE bucket = #{i : t_i < p} (the thresholds are sorted), so one pass
// builds per-label bucket histograms and TP_i = Σ_{b > i} pos[b]: O(n log T) instead of
// O(n T). Counts are exact int64 (Keras keeps float32 counts, which drift past 2^24).
#include "common.hpp"

namespace rs {

__global__ __launch_bounds__(256) void auc_update_kernel(const float* __restrict__ pred,
                                                         const float* __restrict__ label,
                                                         int64_t n,
                                                         const float* __restrict__ thr, int nthr,
                                                         unsigned long long* __restrict__ counts,
                                                         int32_t* __restrict__ err_flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float p = pred[i];
  if (!(p >= 0.f && p <= 1.f) && err_flag) atomicOr(err_flag, RS_ERRBIT_OOB);
  int lo = 0, hi = nthr;  // first threshold >= p  ==  #thresholds < p
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (thr[mid] < p) lo = mid + 1;
    else hi = mid;
  }
  const int bucket = lo;
  const bool pos = label[i] != 0.f;
  atomicAdd(counts + (pos ? (nthr + 1) : 0) + bucket, 1ull);
}

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_auc_update(const float* pred, const float* label, int64_t n,
                                 const float* thresholds, int32_t n_thresholds,
                                 unsigned long long* counts, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(n >= 0 && n_thresholds >= 2, "rs_auc_update: bad sizes");
  if (n == 0) return RS_OK;
  RS_CHECK_ARG(pred && label && thresholds && counts, "rs_auc_update: null pointer");
  auc_update_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, as_stream(stream)>>>(
      pred, label, n, thresholds, n_thresholds, counts, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
