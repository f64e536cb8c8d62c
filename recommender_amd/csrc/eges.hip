// eges.hip — EGES / GES / DeepWalk surfaces (eges/model.py).
//
//   match logits  logits[b, j] = out_table[match[b, j]] · hidden[b]      (eges/model.py:33-35,
//                 fused gather + dot: the [B, 1+num_ns, D] match rows are never materialised
//                 in the forward; the backward writes them once as the sparse grad rows).
//   side pool     hidden[b] = Σ_s a[b, s] side[b, s]  with a = softmax(w[b]) (EGES :92-102) or
//                 a = 1/S as (Σ_s side) / S (GES :74-80).
// One wave per example, lanes over D (coalesced rows), xor-shuffle reductions (fixed order).
#include "common.hpp"
#include "rng.hpp"

namespace rs {

int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* total, void* ws,
                           size_t ws_bytes, hipStream_t st);
size_t exclusive_scan_ws_size(int64_t n);

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

// Row widths D = 4k <= 128: a 32-lane half-wave per example, lane c on the float4 column c, the
// S side rows' loads in flight together (the one-float-per-lane form above left lanes 16-63 idle
// on the second pass at D = 80 and ran at 1.5 TB/s: MMOE's gate pooling, 4 launches per step).
// Any layout: side row s of example b at side + b * sb + s * ss (MMOE pools its experts' outputs
// in the [E, B, H] order the batched expert GEMMs leave them). The forward sums in the same order
// as the scalar kernel (bit-identical); the backward's <g, side_s> folds over the half-wave.
typedef float pf4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 32);
  return v;
}

__global__ __launch_bounds__(kWave * kWavesPerBlock) void pool_fwd_vec_kernel(
    const float* __restrict__ side, int64_t sb, int64_t ss, const float* __restrict__ wlogits,
    int64_t B, int32_t S, int32_t D, float* __restrict__ hidden, float* __restrict__ attn) {
  const int lane = threadIdx.x & 63, c = lane & 31;
  const int64_t b = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 2 + (lane >> 5);
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
    if (attn && c < S) {
      for (int s = 0; s < S; ++s)
        if (s == c) attn[b * S + s] = a[s];
    }
  }
  if (4 * c >= D) return;
  const float* x = side + b * sb + 4 * c;
  pf4 v[kMaxSide];
#pragma unroll
  for (int s = 0; s < kMaxSide; ++s)
    if (s < S) v[s] = *reinterpret_cast<const pf4*>(x + s * ss);
  pf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < kMaxSide; ++s) {
    if (s < S) {
      if (wlogits) acc += a[s] * v[s];
      else acc += v[s];
    }
  }
  if (!wlogits) acc = acc / (float)S;
  *reinterpret_cast<pf4*>(hidden + b * D + 4 * c) = acc;
}

__global__ __launch_bounds__(kWave * kWavesPerBlock) void pool_bwd_vec_kernel(
    const float* __restrict__ side, int64_t sb, int64_t ss, const float* __restrict__ attn,
    const float* __restrict__ g, int64_t B, int32_t S, int32_t D, float* __restrict__ grad_side,
    float* __restrict__ grad_w) {
  const int lane = threadIdx.x & 63, c = lane & 31;
  const int64_t b = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  if (b >= B) return;  // a whole half-wave: its shuffles below stay within its own 32 lanes
  const bool on = 4 * c < D;
  const pf4 gd = on ? *reinterpret_cast<const pf4*>(g + b * D + 4 * c) : pf4{0.f, 0.f, 0.f, 0.f};
  if (!attn) {
    if (on)
      for (int s = 0; s < S; ++s)
        *reinterpret_cast<pf4*>(grad_side + b * sb + s * ss + 4 * c) = gd / (float)S;
    return;
  }
  float a[kMaxSide], ga[kMaxSide];
  for (int s = 0; s < S; ++s) a[s] = attn[b * S + s];
  pf4 v[kMaxSide];
#pragma unroll
  for (int s = 0; s < kMaxSide; ++s)
    if (s < S) v[s] = on ? *reinterpret_cast<const pf4*>(side + b * sb + s * ss + 4 * c)
                         : pf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < kMaxSide; ++s) {
    if (s < S) {
      if (on) *reinterpret_cast<pf4*>(grad_side + b * sb + s * ss + 4 * c) = a[s] * gd;
      const pf4 p = gd * v[s];
      ga[s] = half_sum((p[0] + p[1]) + (p[2] + p[3]));
    }
  }
  float dot = 0.f;
  for (int s = 0; s < S; ++s) dot += a[s] * ga[s];
  if (grad_w && c == 0)
    for (int s = 0; s < S; ++s) grad_w[b * S + s] = a[s] * (ga[s] - dot);
}

// ---- several softmax poolings of the same side rows (MMOE: one gate per task over the same
// expert outputs, esmm/mmoe.py:36-46) ---------------------------------------------------------
// The side rows are read once for all T tasks; per task the arithmetic is pool_*_vec_kernel's
// (same order), and the backward's side gradient is Σ_t attn_t[s]·g_t summed in task order,
// each product rounded (contraction is off) — the sum autograd forms over T separate poolings.
constexpr int kMaxPoolTasks = 4;
struct PoolTasks {
  const float* wl[kMaxPoolTasks];  // [B, S] gate logits of task t, row stride wl_ld
  float* hidden[kMaxPoolTasks];    // forward: [B, D] pooled rows
  float* attn[kMaxPoolTasks];      // [B, S] softmax weights (forward out, backward in)
  const float* g[kMaxPoolTasks];   // backward: [B, D] upstream gradient of hidden
  float* gw[kMaxPoolTasks];        // backward: [B, S] logit gradient, row stride gw_ld
  int64_t wl_ld, gw_ld;
  int T;
};

// sbias (optional, [S, D]): the side rows arrive as pre-activations z and become
// relu(z + sbias[s]) — written back in place (the rows the backward reads) before pooling:
// MMOE's batched expert layer's bias and relu taken here instead of a bias broadcast into the
// GEMM output and a relu pass over it.
__global__ __launch_bounds__(kWave * kWavesPerBlock) void pool_fwd_multi_kernel(
    float* __restrict__ side, int64_t sb, int64_t ss, int64_t B, int32_t S, int32_t D,
    const float* __restrict__ sbias, PoolTasks pt) {
  const int lane = threadIdx.x & 63, c = lane & 31;
  const int64_t b = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  if (b >= B) return;
  const bool on = 4 * c < D;
  // Round 6: every load unguarded from an in-bounds address (side s < S, column 4c < D, else
  // side 0 / column 0) and masked where used; guarded per element, the compiler waited for each
  // (tools/isa_wait_audit.py)
  const int cc = on ? 4 * c : 0;
  pf4 v[kMaxSide], bb[kMaxSide];
#pragma unroll
  for (int s = 0; s < kMaxSide; ++s)
    v[s] = *reinterpret_cast<const pf4*>(side + b * sb + (s < S ? s : 0) * ss + cc);
  if (sbias) {
#pragma unroll
    for (int s = 0; s < kMaxSide; ++s)
      bb[s] = *reinterpret_cast<const pf4*>(sbias + (s < S ? s : 0) * D + cc);
  }
#pragma unroll
  for (int s = 0; s < kMaxSide; ++s)
    if (!(s < S && on)) v[s] = pf4{0.f, 0.f, 0.f, 0.f};
  if (sbias && on) {
#pragma unroll
    for (int s = 0; s < kMaxSide; ++s) {
      if (s < S) {
        const pf4 z = v[s] + bb[s];
        v[s] = pf4{fmaxf(z[0], 0.f), fmaxf(z[1], 0.f), fmaxf(z[2], 0.f), fmaxf(z[3], 0.f)};
        *reinterpret_cast<pf4*>(side + b * sb + s * ss + 4 * c) = v[s];
      }
    }
  }
  for (int t = 0; t < pt.T; ++t) {
    const float* wl = pt.wl[t] + b * pt.wl_ld;
    float a[kMaxSide], wv[kMaxSide];
#pragma unroll
    for (int s = 0; s < kMaxSide; ++s) wv[s] = wl[s < S ? s : 0];
    float mx = -INFINITY;
    for (int s = 0; s < S; ++s) mx = fmaxf(mx, wv[s]);
    float sum = 0.f;
    for (int s = 0; s < S; ++s) {
      a[s] = expf(wv[s] - mx);
      sum += a[s];
    }
    for (int s = 0; s < S; ++s) a[s] = a[s] / sum;
    if (c < S) {
      for (int s = 0; s < S; ++s)
        if (s == c) pt.attn[t][b * S + s] = a[s];
    }
    pf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kMaxSide; ++s)
      if (s < S) acc += a[s] * v[s];
    if (on) *reinterpret_cast<pf4*>(pt.hidden[t] + b * D + 4 * c) = acc;
  }
}

__global__ __launch_bounds__(kWave * kWavesPerBlock) void pool_bwd_multi_kernel(
    const float* __restrict__ side, int64_t sb, int64_t ss, int64_t B, int32_t S, int32_t D,
    float* __restrict__ grad_side, PoolTasks pt) {
  const int lane = threadIdx.x & 63, c = lane & 31;
  const int64_t b = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  if (b >= B) return;  // a whole half-wave: its shuffles stay within its own 32 lanes
  const bool on = 4 * c < D;
  pf4 v[kMaxSide], gs[kMaxSide];
#pragma unroll
  for (int s = 0; s < kMaxSide; ++s)
    if (s < S) v[s] = on ? *reinterpret_cast<const pf4*>(side + b * sb + s * ss + 4 * c)
                         : pf4{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < pt.T; ++t) {
    const pf4 gd = on ? *reinterpret_cast<const pf4*>(pt.g[t] + b * D + 4 * c)
                      : pf4{0.f, 0.f, 0.f, 0.f};
    float a[kMaxSide], ga[kMaxSide];
    for (int s = 0; s < S; ++s) a[s] = pt.attn[t][b * S + s];
#pragma unroll
    for (int s = 0; s < kMaxSide; ++s) {
      if (s < S) {
        const pf4 q = a[s] * gd;
        gs[s] = t == 0 ? q : gs[s] + q;
        const pf4 p = gd * v[s];
        ga[s] = half_sum((p[0] + p[1]) + (p[2] + p[3]));
      }
    }
    float dot = 0.f;
    for (int s = 0; s < S; ++s) dot += a[s] * ga[s];
    if (c == 0)
      for (int s = 0; s < S; ++s) pt.gw[t][b * pt.gw_ld + s] = a[s] * (ga[s] - dot);
  }
  if (on) {
#pragma unroll
    for (int s = 0; s < kMaxSide; ++s)
      if (s < S) *reinterpret_cast<pf4*>(grad_side + b * sb + s * ss + 4 * c) = gs[s];
  }
}

// ---- training-pair sampler (eges/data_loader.py:28-62) -------------
// walk i (global index walk_base + i) starts at 1 + U[0, n_items - 1) (:30, item 0 is OOV) and
// takes `length` weighted steps (dgl.sampling.random_walk(prob='weight') [3p]: out-edge e of
// node v with probability w_e / Σ w): draw r, target = (r + 0.5) / 2^32 · W_v, first edge whose
// inclusive prefix weight (float64, per node) exceeds it. -1 after a dead end.
constexpr uint32_t kPurposeEgesSeed = 0x400;
constexpr uint32_t kPurposeEgesWalk = 0x500;
constexpr uint32_t kPurposeEgesNeg = 0x600;

__global__ __launch_bounds__(256) void eges_walk_kernel(const int64_t* __restrict__ indptr,
                                                        const int32_t* __restrict__ indices,
                                                        const double* __restrict__ cumw,
                                                        int32_t n_items, int64_t walk_base,
                                                        int32_t n_walks, int32_t length,
                                                        uint64_t seed, uint32_t step,
                                                        int32_t* __restrict__ traces) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_walks) return;
  const uint32_t gi = (uint32_t)(walk_base + i);
  int32_t node = 1 + (int32_t)bounded(draw(seed, kPurposeEgesSeed, gi, 0u, step, 0u),
                                      (uint32_t)(n_items - 1));
  int32_t* out = traces + (int64_t)i * (length + 1);
  out[0] = node;
  DrawStream ds(seed, kPurposeEgesWalk, gi, 0u, step);
  for (int32_t h = 0; h < length; ++h) {
    if (node >= 0) {
      const int64_t lo = indptr[node], hi = indptr[node + 1];
      if (hi <= lo || !(cumw[hi - 1] > 0.0)) {
        node = -1;
      } else {
        const uint32_t r = ds.at((uint32_t)h);
        const double target = ((double)r + 0.5) * 2.3283064365386963e-10 * cumw[hi - 1];
        int64_t a = lo, b = hi - 1;  // first e in [lo, hi) with cumw[e] > target
        while (a < b) {
          const int64_t m = (a + b) >> 1;
          if (cumw[m] > target) b = m;
          else a = m + 1;
        }
        node = indices[a];
      }
    }
    out[h + 1] = node;
  }
}

// per-node inclusive prefix of the CSR edge weights, sequential float64 sum (one thread per
// node; built once per graph)
__global__ __launch_bounds__(256) void weight_prefix_kernel(const int64_t* __restrict__ indptr,
                                                            const float* __restrict__ w,
                                                            int64_t n_nodes,
                                                            double* __restrict__ cumw) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_nodes) return;
  double acc = 0.0;
  for (int64_t e = indptr[v]; e < indptr[v + 1]; ++e) {
    acc += (double)w[e];
    cumw[e] = acc;
  }
}

// keras.preprocessing.sequence.skipgrams(seq, window_size, negative_samples=0) [3p]: for every
// position i with w_i != 0, every j != i within the window with w_j != 0 gives (w_i, w_j); the
// reference's shuffle only reorders. A slot per (trace, i, j) in enumeration order; items
// <= 0 (OOV 0, dead end -1) are skipped.
// slot k of a trace → (i, j): slots enumerate i ascending, then j ascending over the window
__device__ __forceinline__ void skipgram_slot(int32_t k, int32_t len, int32_t window, int32_t& i,
                                              int32_t& j) {
  for (i = 0; i < len; ++i) {
    const int32_t j0 = i - window < 0 ? 0 : i - window;
    const int32_t j1 = i + window + 1 > len ? len : i + window + 1;
    const int32_t c = j1 - j0 - 1;
    if (k < c) {
      j = j0 + k;
      if (j >= i) ++j;
      return;
    }
    k -= c;
  }
}

// one thread per (trace, slot): coalesced flag / offset traffic
__global__ __launch_bounds__(256) void skipgram_flag_kernel(const int32_t* __restrict__ traces,
                                                            int64_t n_slots, int32_t len,
                                                            int32_t window, int32_t slots,
                                                            int32_t* __restrict__ flag) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slots) return;
  const int64_t t = s / slots;
  int32_t i, j;
  skipgram_slot((int32_t)(s - t * slots), len, window, i, j);
  const int32_t* tr = traces + t * len;
  flag[s] = tr[i] > 0 && tr[j] > 0;
}

__global__ __launch_bounds__(256) void skipgram_emit_kernel(const int32_t* __restrict__ traces,
                                                            int64_t n_slots, int32_t len,
                                                            int32_t window, int32_t slots,
                                                            const int32_t* __restrict__ flag,
                                                            const int32_t* __restrict__ offs,
                                                            int32_t* __restrict__ target,
                                                            int32_t* __restrict__ context) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slots || !flag[s]) return;
  const int64_t t = s / slots;
  int32_t i, j;
  skipgram_slot((int32_t)(s - t * slots), len, window, i, j);
  const int32_t* tr = traces + t * len;
  target[offs[s]] = tr[i];
  context[offs[s]] = tr[j];
}

// tf.random.log_uniform_candidate_sampler(num_sampled, unique=True, range_max) [3p]:
// P(k) = log((k+2)/(k+1)) / log(range_max+1), sampled without repeats. Draw r → the first k with
// cdf[k] > r (cdf[k] = floor(log(k+2)/log(range_max+1) · 2^32), built on the host), rejecting
// classes already taken for this pair.
__global__ __launch_bounds__(256) void log_uniform_kernel(const uint32_t* __restrict__ cdf,
                                                          int32_t range_max, int64_t pair_base,
                                                          int32_t n_pairs, int32_t num_sampled,
                                                          uint64_t seed, uint32_t step,
                                                          int32_t* __restrict__ out,
                                                          int32_t* __restrict__ err_flag) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const uint32_t gp = (uint32_t)(pair_base + p);
  int32_t* o = out + (int64_t)p * num_sampled;
  int32_t got = 0;
  DrawStream ds(seed, kPurposeEgesNeg, gp, 0u, step);
  const float l2r = log2f((float)range_max + 1.0f) * 2.3283064365386963e-10f;
  for (uint32_t d = 0; got < num_sampled; ++d) {
    if (d >= 4096u * (uint32_t)num_sampled) {  // degenerate range: stop, flag
      for (; got < num_sampled; ++got) o[got] = 0;
      flag_oob(err_flag);
      break;
    }
    const uint32_t r = ds.at(d);
    // first k with cdf[k] > r (range_max - 1 if none): start at the float inverse-CDF guess
    // (off by at most a step or two) and walk to the exact answer on the table
    int32_t a = (int32_t)exp2f((float)r * l2r) - 1;
    a = a < 0 ? 0 : a > range_max - 1 ? range_max - 1 : a;
    while (a < range_max - 1 && cdf[a] <= r) ++a;
    while (a > 0 && cdf[a - 1] > r) --a;
    bool dup = false;
    for (int32_t q = 0; q < got; ++q) dup |= o[q] == a;
    if (!dup) o[got++] = a;
  }
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

static bool pool_vec_ok(const void* side, const void* a, const void* b, int32_t dim, int64_t sb,
                        int64_t ss) {
  return dim % 4 == 0 && dim <= 128 && sb % 4 == 0 && ss % 4 == 0 &&
         ((reinterpret_cast<uintptr_t>(side) | reinterpret_cast<uintptr_t>(a) |
           reinterpret_cast<uintptr_t>(b)) & 15) == 0;
}

extern "C" int32_t rs_side_pool_fwd_strided(const float* side, int64_t side_bstride,
                                            int64_t side_sstride, const float* weight_logits,
                                            int64_t batch, int32_t n_side, int32_t dim,
                                            float* hidden, float* attn, void* stream) {
  RS_CHECK_ARG(n_side >= 1 && n_side <= kMaxSide && dim >= 1 && batch >= 0,
               "rs_side_pool_fwd: need 1 <= n_side <= %d", kMaxSide);
  if (batch == 0) return RS_OK;
  RS_CHECK_ARG(side && hidden, "null pointer");
  const bool dense = side_bstride == (int64_t)n_side * dim && side_sstride == dim;
  if (pool_vec_ok(side, hidden, side, dim, side_bstride, side_sstride)) {
    pool_fwd_vec_kernel<<<waves_grid(ceil_div(batch, 2)), kWave * kWavesPerBlock, 0,
                          as_stream(stream)>>>(side, side_bstride, side_sstride, weight_logits,
                                               batch, n_side, dim, hidden, attn);
  } else {
    RS_CHECK_ARG(dense, "rs_side_pool_fwd: strided side rows need dim % 4 == 0, dim <= 128");
    pool_fwd_kernel<<<waves_grid(batch), kWave * kWavesPerBlock, 0, as_stream(stream)>>>(
        side, weight_logits, batch, n_side, dim, hidden, attn);
  }
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_side_pool_bwd_strided(const float* side, int64_t side_bstride,
                                            int64_t side_sstride, const float* attn,
                                            const float* grad_hidden, int64_t batch,
                                            int32_t n_side, int32_t dim, float* grad_side,
                                            float* grad_weight_logits, void* stream) {
  RS_CHECK_ARG(n_side >= 1 && n_side <= kMaxSide && dim >= 1 && batch >= 0,
               "rs_side_pool_bwd: need 1 <= n_side <= %d", kMaxSide);
  if (batch == 0) return RS_OK;
  RS_CHECK_ARG(side && grad_hidden && grad_side, "null pointer");
  const bool dense = side_bstride == (int64_t)n_side * dim && side_sstride == dim;
  if (pool_vec_ok(side, grad_hidden, grad_side, dim, side_bstride, side_sstride)) {
    pool_bwd_vec_kernel<<<waves_grid(ceil_div(batch, 2)), kWave * kWavesPerBlock, 0,
                          as_stream(stream)>>>(side, side_bstride, side_sstride, attn, grad_hidden,
                                               batch, n_side, dim, grad_side, grad_weight_logits);
  } else {
    RS_CHECK_ARG(dense, "rs_side_pool_bwd: strided side rows need dim % 4 == 0, dim <= 128");
    pool_bwd_kernel<<<waves_grid(batch), kWave * kWavesPerBlock, 0, as_stream(stream)>>>(
        side, attn, grad_hidden, batch, n_side, dim, grad_side, grad_weight_logits);
  }
  RS_CHECK_LAUNCH();
  return RS_OK;
}

static int32_t check_pool_multi(const float* side, int64_t sb, int64_t ss, int64_t batch,
                                int32_t n_side, int32_t dim, int32_t n_tasks) {
  RS_CHECK_ARG(n_side >= 1 && n_side <= kMaxSide && dim >= 1 && dim <= 128 && dim % 4 == 0 &&
                   batch >= 0 && n_tasks >= 1 && n_tasks <= kMaxPoolTasks,
               "rs_side_pool_multi: need 1 <= n_side <= %d, dim % 4 == 0 and <= 128, 1 <= tasks "
               "<= %d", kMaxSide, kMaxPoolTasks);
  RS_CHECK_ARG(side && (reinterpret_cast<uintptr_t>(side) & 15) == 0 && sb % 4 == 0 && ss % 4 == 0,
               "rs_side_pool_multi: side rows must be 16-byte aligned");
  return RS_OK;
}

extern "C" int32_t rs_side_pool_fwd_multi(float* side, int64_t side_bstride,
                                          int64_t side_sstride, int64_t batch, int32_t n_side,
                                          int32_t dim, int32_t n_tasks,
                                          const float* const* weight_logits, int64_t logits_ld,
                                          float* const* hidden, float* const* attn,
                                          const float* side_bias, void* stream) {
  if (int32_t e = check_pool_multi(side, side_bstride, side_sstride, batch, n_side, dim, n_tasks))
    return e;
  RS_CHECK_ARG(weight_logits && hidden && attn && logits_ld >= n_side, "bad task arrays");
  if (batch == 0) return RS_OK;
  PoolTasks pt{};
  pt.T = n_tasks;
  pt.wl_ld = logits_ld;
  for (int t = 0; t < n_tasks; ++t) {
    RS_CHECK_ARG(weight_logits[t] && hidden[t] && attn[t] &&
                     (reinterpret_cast<uintptr_t>(hidden[t]) & 15) == 0,
                 "task %d: null or unaligned pointer", t);
    pt.wl[t] = weight_logits[t];
    pt.hidden[t] = hidden[t];
    pt.attn[t] = attn[t];
  }
  RS_CHECK_ARG(!side_bias || (reinterpret_cast<uintptr_t>(side_bias) & 15) == 0,
               "rs_side_pool_fwd_multi: side_bias must be 16-byte aligned");
  pool_fwd_multi_kernel<<<waves_grid(ceil_div(batch, 2)), kWave * kWavesPerBlock, 0,
                          as_stream(stream)>>>(side, side_bstride, side_sstride, batch, n_side,
                                               dim, side_bias, pt);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_side_pool_bwd_multi(const float* side, int64_t side_bstride,
                                          int64_t side_sstride, int64_t batch, int32_t n_side,
                                          int32_t dim, int32_t n_tasks, const float* const* attn,
                                          const float* const* grad_hidden, float* grad_side,
                                          float* const* grad_logits, int64_t grad_logits_ld,
                                          void* stream) {
  if (int32_t e = check_pool_multi(side, side_bstride, side_sstride, batch, n_side, dim, n_tasks))
    return e;
  RS_CHECK_ARG(attn && grad_hidden && grad_side && grad_logits && grad_logits_ld >= n_side &&
                   (reinterpret_cast<uintptr_t>(grad_side) & 15) == 0,
               "bad task arrays");
  if (batch == 0) return RS_OK;
  PoolTasks pt{};
  pt.T = n_tasks;
  pt.gw_ld = grad_logits_ld;
  for (int t = 0; t < n_tasks; ++t) {
    RS_CHECK_ARG(attn[t] && grad_hidden[t] && grad_logits[t] &&
                     (reinterpret_cast<uintptr_t>(grad_hidden[t]) & 15) == 0,
                 "task %d: null or unaligned pointer", t);
    pt.attn[t] = const_cast<float*>(attn[t]);
    pt.g[t] = grad_hidden[t];
    pt.gw[t] = grad_logits[t];
  }
  pool_bwd_multi_kernel<<<waves_grid(ceil_div(batch, 2)), kWave * kWavesPerBlock, 0,
                          as_stream(stream)>>>(side, side_bstride, side_sstride, batch, n_side,
                                               dim, grad_side, pt);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_side_pool_fwd(const float* side, const float* weight_logits, int64_t batch,
                                    int32_t n_side, int32_t dim, float* hidden, float* attn,
                                    void* stream) {
  return rs_side_pool_fwd_strided(side, (int64_t)n_side * dim, dim, weight_logits, batch, n_side,
                                  dim, hidden, attn, stream);
}

extern "C" int32_t rs_side_pool_bwd(const float* side, const float* attn, const float* grad_hidden,
                                    int64_t batch, int32_t n_side, int32_t dim, float* grad_side,
                                    float* grad_weight_logits, void* stream) {
  return rs_side_pool_bwd_strided(side, (int64_t)n_side * dim, dim, attn, grad_hidden, batch,
                                  n_side, dim, grad_side, grad_weight_logits, stream);
}

extern "C" int32_t rs_eges_walks(const int64_t* indptr, const int32_t* indices, const double* cumw,
                                 int32_t n_items, int64_t walk_base, int32_t n_walks,
                                 int32_t length, uint64_t seed, uint32_t step, int32_t* traces,
                                 void* stream) {
  RS_CHECK_ARG(n_items >= 2 && n_walks >= 0 && length >= 0, "rs_eges_walks: bad sizes");
  if (n_walks == 0) return RS_OK;
  eges_walk_kernel<<<(unsigned)ceil_div(n_walks, 256), 256, 0, as_stream(stream)>>>(
      indptr, indices, cumw, n_items, walk_base, n_walks, length, seed, step, traces);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

static int32_t skipgram_slots(int32_t len, int32_t window) {
  int32_t k = 0;
  for (int32_t i = 0; i < len; ++i) {
    const int32_t j0 = i - window < 0 ? 0 : i - window;
    const int32_t j1 = i + window + 1 > len ? len : i + window + 1;
    k += j1 - j0 - 1;
  }
  return k;
}

extern "C" size_t rs_skipgram_workspace_size(int32_t n_traces, int32_t len, int32_t window) {
  const int64_t n = (int64_t)n_traces * skipgram_slots(len, window);
  Carver c(nullptr, 0);
  c.take<int32_t>(n);
  c.take<int32_t>(n);
  c.take<char>(exclusive_scan_ws_size(n < 1 ? 1 : n));
  return c.off + 256;
}

extern "C" int32_t rs_skipgram_pairs(const int32_t* traces, int32_t n_traces, int32_t len,
                                     int32_t window, int32_t* target, int32_t* context,
                                     int32_t* n_pairs, void* workspace, size_t ws_bytes,
                                     void* stream) {
  RS_CHECK_ARG(n_traces >= 0 && len >= 1 && window >= 1, "rs_skipgram_pairs: bad sizes");
  hipStream_t st = as_stream(stream);
  const int32_t slots = skipgram_slots(len, window);
  const int64_t n = (int64_t)n_traces * slots;
  if (n == 0) {
    RS_CHECK_HIP(hipMemsetAsync(n_pairs, 0, 4, st));
    return RS_OK;
  }
  Carver c(workspace, ws_bytes);
  int32_t* flag = c.take<int32_t>(n);
  int32_t* offs = c.take<int32_t>(n);
  void* sws = c.take<char>(exclusive_scan_ws_size(n));
  if (!c.ok()) {
    set_error("rs_skipgram_pairs: workspace too small");
    return RS_E_WORKSPACE;
  }
  const unsigned g = (unsigned)ceil_div(n, 256);
  skipgram_flag_kernel<<<g, 256, 0, st>>>(traces, n, len, window, slots, flag);
  RS_CHECK_LAUNCH();
  int32_t s = exclusive_scan_i32(flag, offs, n, n_pairs, sws, exclusive_scan_ws_size(n), st);
  if (s) return s;
  skipgram_emit_kernel<<<g, 256, 0, st>>>(traces, n, len, window, slots, flag, offs, target,
                                          context);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_log_uniform_sample(const uint32_t* cdf, int32_t range_max, int64_t pair_base,
                                         int32_t n_pairs, int32_t num_sampled, uint64_t seed,
                                         uint32_t step, int32_t* out, int32_t* err_flag,
                                         void* stream) {
  RS_CHECK_ARG(range_max >= 1 && num_sampled >= 1 && num_sampled <= range_max && n_pairs >= 0,
               "rs_log_uniform_sample: bad sizes");
  if (n_pairs == 0) return RS_OK;
  log_uniform_kernel<<<(unsigned)ceil_div(n_pairs, 256), 256, 0, as_stream(stream)>>>(
      cdf, range_max, pair_base, n_pairs, num_sampled, seed, step, out, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_csr_weight_prefix(const int64_t* indptr, const float* weights,
                                        int64_t n_nodes, double* cumw, void* stream) {
  RS_CHECK_ARG(n_nodes >= 0, "rs_csr_weight_prefix: bad sizes");
  if (n_nodes == 0) return RS_OK;
  weight_prefix_kernel<<<(unsigned)ceil_div(n_nodes, 256), 256, 0, as_stream(stream)>>>(
      indptr, weights, n_nodes, cumw);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
