// eges.hip — EGES / GES / DeepWalk surfaces (eges/model.py).
//
//   match logits  logits[b, j] = out_table[match[b, j]] · hidden[b]      (eges/model.py:33-35,
//                 fused gather + dot: the [B, 1+num_ns, D] match rows are never materialised
//                 in the forward; the backward writes them once as the sparse grad rows).
//   side pool     hidden[b] = Σ_s a[b, s] side[b, s]  with a = softmax(w[b]) (EGES :92-102) or
//                 a = 1/S as (Σ_s side) / S (GES :74-80).
// One wave per example, lanes over D (coalesced rows), xor-shuffle reductions (fixed order).
#include "common.hpp"

namespace rs {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

constexpr int kMaxSide = 16;
constexpr int kWavesPerBlock = 4;

// logits[b, j]; OOB ids read zero rows and set the error flag
__global__ __launch_bounds__(kWave * kWavesPerBlock) void match_fwd_kernel(
    const float* __restrict__ table, int64_t n_rows, int32_t D, const void* __restrict__ ids,
    int32_t dtype, int32_t M, const float* __restrict__ hidden, int64_t B,
    float* __restrict__ logits, int32_t* __restrict__ err_flag) {
  const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* h = hidden + b * D;
  for (int32_t j = 0; j < M; ++j) {
    const int64_t id = load_id(ids, dtype, b * M + j);
    const bool ok = id >= 0 && id < n_rows;
    if (!ok && lane == 0) flag_oob(err_flag);
    float acc = 0.f;
    if (ok) {
      const float* row = table + id * D;
      for (int32_t d = lane; d < D; d += kWave) acc += row[d] * h[d];
    }
    acc = wave_sum(acc);
    if (lane == 0) logits[b * M + j] = acc;
  }
}

// grad_rows[b*M + j] = g[b, j] * hidden[b]; grad_hidden[b] = Σ_j g[b, j] * row_j
__global__ __launch_bounds__(kWave * kWavesPerBlock) void match_bwd_kernel(
    const float* __restrict__ table, int64_t n_rows, int32_t D, const void* __restrict__ ids,
    int32_t dtype, int32_t M, const float* __restrict__ hidden, const float* __restrict__ g,
    int64_t B, float* __restrict__ grad_rows, float* __restrict__ grad_hidden) {
  const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* h = hidden + b * D;
  for (int32_t d = lane; d < D; d += kWave) {
    const float hd = h[d];
    float acc = 0.f;
    for (int32_t j = 0; j < M; ++j) {
      const float gj = g[b * M + j];
      const int64_t id = load_id(ids, dtype, b * M + j);
      const float r = (id >= 0 && id < n_rows) ? table[id * D + d] : 0.f;
      acc += gj * r;
      grad_rows[(b * M + j) * D + d] = gj * hd;
    }
    grad_hidden[b * D + d] = acc;
  }
}

__global__ __launch_bounds__(kWave * kWavesPerBlock) void pool_fwd_kernel(
    const float* __restrict__ side, const float* __restrict__ wlogits, int64_t B, int32_t S,
    int32_t D, float* __restrict__ hidden, float* __restrict__ attn) {
  const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  float a[kMaxSide];
  if (wlogits) {
    float mx = -INFINITY;
    for (int s = 0; s < S; ++s) mx = fmaxf(mx, wlogits[b * S + s]);
    float sum = 0.f;
    for (int s = 0; s < S; ++s) {
      a[s] = expf(wlogits[b * S + s] - mx);
      sum += a[s];
    }
    for (int s = 0; s < S; ++s) a[s] = a[s] / sum;
    if (attn && lane < S) {
      for (int s = 0; s < S; ++s)
        if (s == lane) attn[b * S + s] = a[s];
    }
  }
  const float* x = side + b * S * D;
  for (int32_t d = lane; d < D; d += kWave) {
    float acc = 0.f;
    if (wlogits) {
      for (int s = 0; s < S; ++s) acc += a[s] * x[s * D + d];
    } else {
      for (int s = 0; s < S; ++s) acc += x[s * D + d];
      acc = acc / (float)S;
    }
    hidden[b * D + d] = acc;
  }
}

// softmax mode: grad_side[b,s] = a_s g; ga_s = <g, side_s>; grad_w[b,s] = a_s (ga_s - Σ_t a_t ga_t)
// mean mode (attn == NULL): grad_side[b,s] = g / S
__global__ __launch_bounds__(kWave * kWavesPerBlock) void pool_bwd_kernel(
    const float* __restrict__ side, const float* __restrict__ attn, const float* __restrict__ g,
    int64_t B, int32_t S, int32_t D, float* __restrict__ grad_side,
    float* __restrict__ grad_w) {
  const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* x = side + b * S * D;
  const float* gb = g + b * D;
  float* gs = grad_side + b * S * D;
  if (!attn) {
    for (int32_t d = lane; d < D; d += kWave) {
      const float v = gb[d] / (float)S;
      for (int s = 0; s < S; ++s) gs[s * D + d] = v;
    }
    return;
  }
  float a[kMaxSide], ga[kMaxSide];
  for (int s = 0; s < S; ++s) a[s] = attn[b * S + s];
  for (int s = 0; s < S; ++s) ga[s] = 0.f;
  for (int32_t d = lane; d < D; d += kWave) {
    const float gd = gb[d];
    for (int s = 0; s < S; ++s) {
      gs[s * D + d] = a[s] * gd;
      ga[s] += gd * x[s * D + d];
    }
  }
  float dot = 0.f;
  for (int s = 0; s < S; ++s) {
    ga[s] = wave_sum(ga[s]);
    dot += a[s] * ga[s];
  }
  if (grad_w && lane == 0)
    for (int s = 0; s < S; ++s) grad_w[b * S + s] = a[s] * (ga[s] - dot);
}

inline unsigned waves_grid(int64_t B) { return (unsigned)ceil_div(B < 1 ? 1 : B, kWavesPerBlock); }

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_match_logits_fwd(const float* table, int64_t n_rows, int32_t dim,
                                       const void* match_ids, int32_t id_dtype, int32_t n_match,
                                       const float* hidden, int64_t batch, float* logits,
                                       int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(dim >= 1 && n_match >= 1 && batch >= 0 && n_rows >= 1,
               "rs_match_logits_fwd: bad sizes");
  if (batch == 0) return RS_OK;
  match_fwd_kernel<<<waves_grid(batch), kWave * kWavesPerBlock, 0, as_stream(stream)>>>(
      table, n_rows, dim, match_ids, id_dtype, n_match, hidden, batch, logits, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_match_logits_bwd(const float* table, int64_t n_rows, int32_t dim,
                                       const void* match_ids, int32_t id_dtype, int32_t n_match,
                                       const float* hidden, const float* grad_logits,
                                       int64_t batch, float* grad_rows, float* grad_hidden,
                                       void* stream) {
  RS_CHECK_ARG(dim >= 1 && n_match >= 1 && batch >= 0 && n_rows >= 1,
               "rs_match_logits_bwd: bad sizes");
  if (batch == 0) return RS_OK;
  match_bwd_kernel<<<waves_grid(batch), kWave * kWavesPerBlock, 0, as_stream(stream)>>>(
      table, n_rows, dim, match_ids, id_dtype, n_match, hidden, grad_logits, batch, grad_rows,
      grad_hidden);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_side_pool_fwd(const float* side, const float* weight_logits, int64_t batch,
                                    int32_t n_side, int32_t dim, float* hidden, float* attn,
                                    void* stream) {
  RS_CHECK_ARG(n_side >= 1 && n_side <= kMaxSide && dim >= 1 && batch >= 0,
               "rs_side_pool_fwd: need 1 <= n_side <= %d", kMaxSide);
  if (batch == 0) return RS_OK;
  pool_fwd_kernel<<<waves_grid(batch), kWave * kWavesPerBlock, 0, as_stream(stream)>>>(
      side, weight_logits, batch, n_side, dim, hidden, attn);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_side_pool_bwd(const float* side, const float* attn, const float* grad_hidden,
                                    int64_t batch, int32_t n_side, int32_t dim, float* grad_side,
                                    float* grad_weight_logits, void* stream) {
  RS_CHECK_ARG(n_side >= 1 && n_side <= kMaxSide && dim >= 1 && batch >= 0,
               "rs_side_pool_bwd: need 1 <= n_side <= %d", kMaxSide);
  if (batch == 0) return RS_OK;
  pool_bwd_kernel<<<waves_grid(batch), kWave * kWavesPerBlock, 0, as_stream(stream)>>>(
      side, attn, grad_hidden, batch, n_side, dim, grad_side, grad_weight_logits);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
