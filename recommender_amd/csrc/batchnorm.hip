// batchnorm.hip — keras.layers.BatchNormalization on [B, C] rows (the DIEN / DIN / BASE MLP
// head, dien/layers.py:20-31: momentum 0.99, epsilon 1e-3) in two launches per direction instead
// of a dozen elementwise / reduction passes each.
//
// Forward, training (batch statistics): per column c, mean = Σ x / B and the population
// variance var = Σ (x - mean)² / B (tf.nn.moments), from per-chunk (count, mean, M2) partials
// merged in chunk order (Chan et al.); y = ((x - mean) · rsqrt(var + ε)) · γ + β; the moving
// statistics move by Keras' _assign_moving_average, m -= (m - value) · (1 - momentum).
// Inference: y from the moving statistics, nothing updated.
// Backward (training): with x̂ = (x - mean)·r, dβ = Σ dy, dγ = Σ dy·x̂,
// dx = γ·r·(dy - dβ/B - x̂·dγ/B); inference: dx = γ·r·dy.
// Deterministic: fixed chunking (kBnRows rows), every block of the second launch merges the
// chunk partials of its columns in chunk order itself.
#include "common.hpp"

namespace rs {
namespace {

constexpr int kBnRows = 64;   // rows per chunk
constexpr int kBnCols = 64;   // columns per block (one wave's lanes)
constexpr int kBnLanes = 4;   // row lanes per block (256 threads)

// partials: pa[chunk][c], pb[chunk][c] (forward: chunk mean, M2; backward: Σ dy, Σ dy·x̂)
__global__ __launch_bounds__(256) void bn_fwd_part_kernel(const float* __restrict__ x, int64_t B,
                                                          int C, float* __restrict__ pa,
                                                          float* __restrict__ pb) {
  __shared__ float red[kBnLanes][kBnCols];
  __shared__ float mean_s[kBnCols];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * kBnCols + cl;
  const int64_t r0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t r1 = r0 + kBnRows < B ? r0 + kBnRows : B;
  float s = 0.f;
  if (c < C)
    for (int64_t r = r0 + rl; r < r1; r += kBnLanes) s += x[r * C + c];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0) mean_s[cl] = (((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl]) / (float)(r1 - r0);
  __syncthreads();
  const float m = mean_s[cl];
  float q = 0.f;
  if (c < C)
    for (int64_t r = r0 + rl; r < r1; r += kBnLanes) {
      const float d = x[r * C + c] - m;
      q += d * d;
    }
  __syncthreads();
  red[rl][cl] = q;
  __syncthreads();
  if (rl == 0 && c < C) {
    pa[(int64_t)blockIdx.y * C + c] = m;
    pb[(int64_t)blockIdx.y * C + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
  }
}

// (mean, var) of column c from the chunk partials, merged in chunk order
__device__ __forceinline__ void bn_merge(const float* __restrict__ pa, const float* __restrict__ pb,
                                         int64_t B, int C, int c, float& mean, float& var) {
  const int nch = (int)((B + kBnRows - 1) / kBnRows);
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int k = 0; k < nch; ++k) {
    const float nb = (float)((int64_t)(k + 1) * kBnRows < B ? kBnRows : B - (int64_t)k * kBnRows);
    const float mb = pa[(int64_t)k * C + c], qb = pb[(int64_t)k * C + c];
    const float nn = n + nb;
    const float d = mb - mu;
    mu = mu + d * (nb / nn);
    m2 = (m2 + qb) + (d * d) * ((n * nb) / nn);
    n = nn;
  }
  mean = mu;
  var = m2 / (float)B;
}

__global__ __launch_bounds__(256) void bn_fwd_apply_kernel(
    const float* __restrict__ x, int64_t B, int C, const float* __restrict__ pa,
    const float* __restrict__ pb, const float* __restrict__ gamma, const float* __restrict__ beta,
    float eps, float decay, float* __restrict__ mmean, float* __restrict__ mvar, int training,
    float* __restrict__ y, float* __restrict__ save_mean, float* __restrict__ save_invstd) {
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * kBnCols + cl;
  if (c >= C) return;
  float mean, var;
  if (training) {
    bn_merge(pa, pb, B, C, c, mean, var);
  } else {
    mean = mmean[c];
    var = mvar[c];
  }
  const float r = rsqrtf(var + eps);
  const float g = gamma[c], bt = beta[c];
  const int64_t r0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t r1 = r0 + kBnRows < B ? r0 + kBnRows : B;
  for (int64_t row = r0 + rl; row < r1; row += kBnLanes)
    y[row * C + c] = ((x[row * C + c] - mean) * r) * g + bt;
  if (blockIdx.y == 0 && rl == 0) {
    save_mean[c] = mean;
    save_invstd[c] = r;
    if (training) {
      mmean[c] = mmean[c] - (mmean[c] - mean) * decay;
      mvar[c] = mvar[c] - (mvar[c] - var) * decay;
    }
  }
}

__global__ __launch_bounds__(256) void bn_bwd_part_kernel(const float* __restrict__ dy,
                                                          const float* __restrict__ x, int64_t B,
                                                          int C, const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          float* __restrict__ pa,
                                                          float* __restrict__ pb) {
  __shared__ float ra[kBnLanes][kBnCols];
  __shared__ float rb[kBnLanes][kBnCols];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * kBnCols + cl;
  const int64_t r0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t r1 = r0 + kBnRows < B ? r0 + kBnRows : B;
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    const float m = mean[c], r = invstd[c];
    for (int64_t row = r0 + rl; row < r1; row += kBnLanes) {
      const float g = dy[row * C + c];
      sa += g;
      sb += g * ((x[row * C + c] - m) * r);
    }
  }
  ra[rl][cl] = sa;
  rb[rl][cl] = sb;
  __syncthreads();
  if (rl == 0 && c < C) {
    pa[(int64_t)blockIdx.y * C + c] = ((ra[0][cl] + ra[1][cl]) + ra[2][cl]) + ra[3][cl];
    pb[(int64_t)blockIdx.y * C + c] = ((rb[0][cl] + rb[1][cl]) + rb[2][cl]) + rb[3][cl];
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int64_t B, int C,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ pa, const float* __restrict__ pb,
    int training, float* __restrict__ dx, float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * kBnCols + cl;
  if (c >= C) return;
  const int nch = (int)((B + kBnRows - 1) / kBnRows);
  float sa = 0.f, sb = 0.f;
  for (int k = 0; k < nch; ++k) {
    sa += pa[(int64_t)k * C + c];
    sb += pb[(int64_t)k * C + c];
  }
  const float m = mean[c], r = invstd[c], gr = gamma[c] * r;
  const float ma = sa / (float)B, mb = sb / (float)B;
  const int64_t r0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t r1 = r0 + kBnRows < B ? r0 + kBnRows : B;
  for (int64_t row = r0 + rl; row < r1; row += kBnLanes) {
    const float g = dy[row * C + c];
    if (training) {
      const float xh = (x[row * C + c] - m) * r;
      dx[row * C + c] = gr * ((g - ma) - xh * mb);
    } else {
      dx[row * C + c] = gr * g;
    }
  }
  if (blockIdx.y == 0 && rl == 0) {
    dbeta[c] = sa;
    dgamma[c] = sb;
  }
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" size_t rs_batch_norm_workspace_size(int64_t B, int32_t C) {
  return 2 * (size_t)ceil_div(B < 1 ? 1 : B, kBnRows) * (C < 1 ? 1 : C) * sizeof(float);
}

extern "C" int32_t rs_batch_norm_fwd(const float* x, int64_t B, int32_t C, const float* gamma,
                                     const float* beta, float epsilon, float momentum,
                                     int32_t training, float* moving_mean, float* moving_var,
                                     float* y, float* save_mean, float* save_invstd,
                                     void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(B >= 1 && C >= 1, "rs_batch_norm_fwd: B, C >= 1");
  RS_CHECK_ARG(x && gamma && beta && moving_mean && moving_var && y && save_mean && save_invstd,
               "rs_batch_norm_fwd: null pointer");
  RS_CHECK_ARG(!training || (workspace && ws_bytes >= rs_batch_norm_workspace_size(B, C)),
               "rs_batch_norm_fwd: workspace too small");
  hipStream_t st = as_stream(stream);
  const unsigned nch = (unsigned)ceil_div(B, kBnRows);
  const dim3 grid((unsigned)ceil_div(C, kBnCols), nch);
  float* pa = static_cast<float*>(workspace);
  float* pb = pa ? pa + (size_t)nch * C : nullptr;
  if (training) {
    bn_fwd_part_kernel<<<grid, 256, 0, st>>>(x, B, C, pa, pb);
    RS_CHECK_LAUNCH();
  }
  bn_fwd_apply_kernel<<<grid, 256, 0, st>>>(x, B, C, pa, pb, gamma, beta, epsilon,
                                            1.0f - momentum, moving_mean, moving_var, training, y,
                                            save_mean, save_invstd);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_batch_norm_bwd(const float* dy, const float* x, int64_t B, int32_t C,
                                     const float* save_mean, const float* save_invstd,
                                     const float* gamma, int32_t training, float* dx, float* dgamma,
                                     float* dbeta, void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(B >= 1 && C >= 1, "rs_batch_norm_bwd: B, C >= 1");
  RS_CHECK_ARG(dy && x && save_mean && save_invstd && gamma && dx && dgamma && dbeta && workspace,
               "rs_batch_norm_bwd: null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_batch_norm_workspace_size(B, C), "rs_batch_norm_bwd: workspace too small");
  hipStream_t st = as_stream(stream);
  const unsigned nch = (unsigned)ceil_div(B, kBnRows);
  const dim3 grid((unsigned)ceil_div(C, kBnCols), nch);
  float* pa = static_cast<float*>(workspace);
  float* pb = pa + (size_t)nch * C;
  bn_bwd_part_kernel<<<grid, 256, 0, st>>>(dy, x, B, C, save_mean, save_invstd, pa, pb);
  RS_CHECK_LAUNCH();
  bn_bwd_apply_kernel<<<grid, 256, 0, st>>>(dy, x, B, C, save_mean, save_invstd, gamma, pa, pb,
                                            training, dx, dgamma, dbeta);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
