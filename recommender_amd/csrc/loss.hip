// loss.hip — keras binary_crossentropy on probabilities, fused (ctr/train.py:85,
// dien/train.py:18, esmm/train.py:101-102; [3p] TF 2.2 backend.binary_crossentropy):
//   pc = clip(p, eps, 1-eps);  l_i = -(y log(pc + eps) + (1-y) log(1 - pc + eps))
// reduction: 0 = none (per example), 1 = sum, 2 = mean. Sums are deterministic: per-block
// partials in a fixed order, then one block folds the partials in block order.
#include "common.hpp"

namespace rs {

constexpr int kLossThreads = 256;
constexpr int kLossMaxBlocks = 1024;

__device__ __forceinline__ float bce_term(float p, float y, float eps) {
  float pc = fminf(fmaxf(p, eps), 1.f - eps);
  float a = y * logf(pc + eps);
  float b = (1.f - y) * logf((1.f - pc) + eps);
  return -(a + b);
}

__global__ __launch_bounds__(kLossThreads) void bce_fwd_kernel(const float* __restrict__ p,
                                                               const float* __restrict__ y, int64_t n,
                                                               float eps, int reduction,
                                                               float* __restrict__ out,
                                                               float* __restrict__ partial) {
  __shared__ float red[kLossThreads];
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float l = bce_term(p[i], y[i], eps);
    if (reduction == 0)
      out[i] = l;
    else
      acc += l;
  }
  if (reduction == 0) return;
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kLossThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void bce_fold_kernel(const float* __restrict__ partial, int nb, int64_t n, int reduction,
                                float* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += partial[b];
  out[0] = reduction == 2 ? s / (float)n : s;
}

__global__ __launch_bounds__(kLossThreads) void bce_bwd_kernel(const float* __restrict__ p,
                                                               const float* __restrict__ y, int64_t n,
                                                               float eps, int reduction,
                                                               const float* __restrict__ gout,
                                                               float* __restrict__ dp) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const float gscalar = reduction == 0 ? 0.f : gout[0] * (reduction == 2 ? 1.f / (float)n : 1.f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float pi = p[i], yi = y[i];
    const float g = reduction == 0 ? gout[i] : gscalar;
    const bool inside = pi >= eps && pi <= 1.f - eps;  // clip_by_value passes the gradient inside
    const float pc = fminf(fmaxf(pi, eps), 1.f - eps);
    const float d = -(yi / (pc + eps)) + (1.f - yi) / ((1.f - pc) + eps);
    dp[i] = inside ? g * d : 0.f;
  }
}

}  // namespace rs

using namespace rs;

extern "C" size_t rs_bce_workspace_size(int64_t n) { return kLossMaxBlocks * sizeof(float); }

extern "C" int32_t rs_bce_fwd(const float* p, const float* y, int64_t n, float eps, int32_t reduction,
                              float* out, void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(n >= 0 && reduction >= 0 && reduction <= 2, "bad arguments");
  RS_CHECK_ARG(reduction == 0 || ws_bytes >= rs_bce_workspace_size(n), "workspace too small");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    if (reduction) RS_CHECK_HIP(hipMemsetAsync(out, 0, 4, st));
    return RS_OK;
  }
  int nb = (int)std::min<int64_t>(ceil_div(n, kLossThreads * 4), kLossMaxBlocks);
  bce_fwd_kernel<<<nb, kLossThreads, 0, st>>>(p, y, n, eps, reduction, out,
                                              static_cast<float*>(workspace));
  RS_CHECK_LAUNCH();
  if (reduction) {
    bce_fold_kernel<<<1, 64, 0, st>>>(static_cast<float*>(workspace), nb, n, reduction, out);
    RS_CHECK_LAUNCH();
  }
  return RS_OK;
}

extern "C" int32_t rs_bce_bwd(const float* p, const float* y, int64_t n, float eps,
                              int32_t reduction, const float* grad_out, float* grad_p,
                              void* stream) {
  RS_CHECK_ARG(n >= 0 && reduction >= 0 && reduction <= 2, "bad arguments");
  if (n == 0) return RS_OK;
  int nb = (int)std::min<int64_t>(ceil_div(n, kLossThreads * 4), 2048);
  bce_bwd_kernel<<<nb, kLossThreads, 0, as_stream(stream)>>>(p, y, n, eps, reduction, grad_out,
                                                             grad_p);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
