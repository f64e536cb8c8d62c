// dense.hip — fused epilogues around the dense (hipBLASLt) MLP GEMMs of the reference's
// Keras Dense layers (ctr/layers.py:5-14, esmm/layers.py:4-13, dien/layers.py:20-31):
//   rs_act_bwd_colsum: dz = act'(y) * dy and db = Σ_b dz (the bias gradient), one pass over
//   dy instead of an activation-backward kernel plus a two-stage torch reduction.
// Deterministic: each block folds a fixed 512-row range of its columns (a fixed row-lane
// assignment, row lanes folded in order), partials are folded in chunk order by a second kernel.
#include "common.hpp"

namespace rs {

constexpr int kColRows = 512;  // rows per chunk

// 256 threads = 16 row lanes x 16 column lanes; a column lane owns VEC consecutive columns, so
// a block covers 16*VEC columns and every wave-instruction moves 4 rows x 16*VEC*4 bytes.
template <int ACT, int VEC>
__global__ __launch_bounds__(256) void act_bwd_colsum_kernel(const float* __restrict__ dy,
                                                             const float* __restrict__ y, int64_t B,
                                                             int N, float* __restrict__ dz,
                                                             float* __restrict__ part,
                                                             int64_t ldg, int64_t ldy,
                                                             int64_t ldz) {
  __shared__ float red[16][16 * VEC + 1];
  const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col0 = (blockIdx.x * 16 + cl) * VEC;
  const int64_t r0 = (int64_t)blockIdx.y * kColRows;
  const int64_t r1 = r0 + kColRows < B ? r0 + kColRows : B;
  float acc[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
  if (col0 < N) {
#pragma unroll 4
    for (int64_t r = r0 + rl; r < r1; r += 16) {
      const int64_t og = r * ldg + col0, oy = r * ldy + col0, o = r * ldz + col0;
      float g[VEC], yy[VEC];
      if constexpr (VEC == 4) {
        float4 t = *reinterpret_cast<const float4*>(dy + og);
        g[0] = t.x; g[1] = t.y; g[2] = t.z; g[3] = t.w;
        if constexpr (ACT != 0) {
          float4 u = *reinterpret_cast<const float4*>(y + oy);
          yy[0] = u.x; yy[1] = u.y; yy[2] = u.z; yy[3] = u.w;
        }
      } else {
        g[0] = dy[og];
        if constexpr (ACT != 0) yy[0] = y[oy];
      }
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        if constexpr (ACT == 1) g[e] = yy[e] > 0.f ? g[e] : 0.f;
        if constexpr (ACT == 2) g[e] = g[e] * (yy[e] * (1.f - yy[e]));
        acc[e] += g[e];
      }
      if constexpr (ACT != 0) {
        if constexpr (VEC == 4)
          *reinterpret_cast<float4*>(dz + o) = make_float4(g[0], g[1], g[2], g[3]);
        else
          dz[o] = g[0];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) red[rl][cl * VEC + e] = acc[e];
  __syncthreads();
  if (threadIdx.x < 16 * VEC) {
    const int c = blockIdx.x * 16 * VEC + threadIdx.x;
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += red[i][threadIdx.x];
    if (c < N) part[(int64_t)blockIdx.y * N + c] = s;
  }
}

// 4 waves per 64 columns: wave w folds chunks w, w+4, ... in order; the 4 wave sums are then
// folded in wave order (fixed tree → deterministic)
__global__ __launch_bounds__(256) void fold_chunks_kernel(const float* __restrict__ part, int nchunks,
                                                          int N, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < N) {
#pragma unroll 8
    for (int c = w; c < nchunks; c += 4) s += part[(int64_t)c * N + col];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < N) out[col] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}


// fold_chunks_kernel per group of chunks: group g folds chunks [g·cpg, (g+1)·cpg) into out[g]
__global__ __launch_bounds__(256) void fold_chunk_groups_kernel(const float* __restrict__ part,
                                                                int cpg, int N,
                                                                float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const float* p = part + (int64_t)blockIdx.y * cpg * N;
  float s = 0.f;
  if (col < N) {
#pragma unroll 8
    for (int c = w; c < cpg; c += 4) s += p[(int64_t)c * N + col];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < N)
    out[(int64_t)blockIdx.y * N + col] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// ---- factored linear-chain backward: A = xᵀ·G and s = Σ_b G in one pass ----------------
// G = act'(y) ⊙ dy is formed on the fly (the formula of act_bwd_colsum_kernel) and optionally
// written out. Rows are cut into fixed chunks of kChainRows; each block folds its chunk in row
// order, the chunk partials [n0*nl + nl] are folded in chunk order by fold_chunks_kernel:
// deterministic.
constexpr int kChainRows = 128;

template <int ACT>
__device__ __forceinline__ float act_grad(float g, float y) {
  if constexpr (ACT == 1) return y > 0.f ? g : 0.f;
  if constexpr (ACT == 2) return g * (y * (1.f - y));
  return g;
}

// nl == 1: thread (phase, column group) moves 4 consecutive columns per row (float4); the
// 256/cgp row phases of a block are folded in phase order through LDS. Every thread forms g_b
// itself (broadcast loads); the phase's group-0 thread accumulates Σ g and writes g_out.
constexpr int kVecRows = 128;

template <int ACT>
__global__ __launch_bounds__(256) void chain_reduce_vec_kernel(
    const float* __restrict__ x, int64_t ldx, int n0, int cgp, const float* __restrict__ dy,
    const float* __restrict__ y, int64_t B, float* __restrict__ gout, float* __restrict__ part) {
  constexpr int U = 8;
  __shared__ float4 red[256];
  __shared__ float sred[256];
  const int t = threadIdx.x;
  const int P = 256 / cgp;
  const int cg = t % cgp, ph = t / cgp;
  const int c0 = 4 * cg;
  const bool live = c0 < n0;
  const int64_t r0 = (int64_t)blockIdx.x * kVecRows;
  const int64_t r1 = r0 + kVecRows < B ? r0 + kVecRows : B;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float sacc = 0.f;
  for (int64_t b0 = r0 + ph; b0 < r1; b0 += (int64_t)U * P) {
    float4 v[U];
    float g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // all U rows' loads in flight before any use
      const int64_t b = b0 + (int64_t)u * P;
      const bool in = b < r1;
      const int64_t bb = in ? b : r0;
      g[u] = in ? act_grad<ACT>(dy[bb], ACT ? y[bb] : 0.f) : 0.f;
      v[u] = (live && in) ? *reinterpret_cast<const float4*>(x + bb * ldx + c0)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += v[u].x * g[u];
      acc.y += v[u].y * g[u];
      acc.z += v[u].z * g[u];
      acc.w += v[u].w * g[u];
      const int64_t b = b0 + (int64_t)u * P;
      if (cg == 0 && b < r1) {
        sacc += g[u];
        if (gout) gout[b] = g[u];
      }
    }
  }
  red[t] = acc;
  sred[t] = sacc;
  __syncthreads();
  float* pp = part + (int64_t)blockIdx.x * (n0 + 1);
  if (t < cgp && live) {
    float4 v = red[t];
    for (int q = 1; q < P; ++q) {
      const float4 w = red[q * cgp + t];
      v.x += w.x;
      v.y += w.y;
      v.z += w.z;
      v.w += w.w;
    }
    pp[c0] = v.x;
    if (c0 + 1 < n0) pp[c0 + 1] = v.y;
    if (c0 + 2 < n0) pp[c0 + 2] = v.z;
    if (c0 + 3 < n0) pp[c0 + 3] = v.w;
  }
  if (t == 0) {
    float v = sred[0];
    for (int q = 1; q < P; ++q) v += sred[q * cgp];
    pp[n0] = v;
  }
}

// n0 <= N0MAX, nl <= 256: thread (phase, j) walks rows r0 + phase, r0 + phase + P, ...; the
// chunk's x rows are staged in LDS; the P phase sums are folded in phase order
template <int ACT, int N0MAX>
__global__ __launch_bounds__(256) void chain_reduce_outer_kernel(
    const float* __restrict__ x, int64_t ldx, int n0, const float* __restrict__ dy,
    const float* __restrict__ y, int nl, int nlp, int64_t B, float* __restrict__ gout,
    float* __restrict__ part) {
  __shared__ float xs[kChainRows * N0MAX];
  __shared__ float red[256 * (N0MAX + 1)];
  const int t = threadIdx.x;
  const int P = 256 / nlp;
  const int j = t % nlp, ph = t / nlp;
  const int64_t r0 = (int64_t)blockIdx.x * kChainRows;
  const int64_t r1 = r0 + kChainRows < B ? r0 + kChainRows : B;
  const int nr = (int)(r1 - r0);
  for (int e = t; e < nr * n0; e += 256) xs[e] = x[(r0 + e / n0) * ldx + e % n0];
  __syncthreads();
  float acc[N0MAX];
#pragma unroll
  for (int i = 0; i < N0MAX; ++i) acc[i] = 0.f;
  float sacc = 0.f;
  constexpr int U = 8;
  if (j < nl) {
    for (int r0b = ph; r0b < nr; r0b += U * P) {
      float g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // U rows' loads in flight before any use
        const int r = r0b + u * P;
        const int64_t o = (r0 + (r < nr ? r : 0)) * nl + j;
        g[u] = r < nr ? act_grad<ACT>(dy[o], ACT ? y[o] : 0.f) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0b + u * P;
        if (r < nr) {
#pragma unroll
          for (int i = 0; i < N0MAX; ++i)
            if (i < n0) acc[i] += xs[r * n0 + i] * g[u];
          sacc += g[u];
          if (gout) gout[(r0 + r) * nl + j] = g[u];
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < N0MAX; ++i) red[t * (N0MAX + 1) + i] = acc[i];
  red[t * (N0MAX + 1) + N0MAX] = sacc;
  __syncthreads();
  float* pp = part + (int64_t)blockIdx.x * ((int64_t)n0 * nl + nl);
  for (int e = t; e < (n0 + 1) * nlp; e += 256) {
    const int i = e / nlp, jj = e % nlp;  // i == n0: the column sum
    if (jj >= nl) continue;
    const int slot = i == n0 ? N0MAX : i;
    float v = 0.f;
    for (int q = 0; q < P; ++q) v += red[(q * nlp + jj) * (N0MAX + 1) + slot];
    pp[(int64_t)i * nl + jj] = v;
  }
}

// nl % 4 == 0, nl <= 256, n0 <= N0MAX: thread (phase, column quad) moves 16 B of dy and of y
// per row; 256 / (nl / 4) row phases walk the chunk's rows interleaved, 4 rows in flight; the
// phases are folded in phase order through LDS (one phase per round: deterministic)
constexpr int kQuadRows = 128;

template <int ACT, int N0MAX>
__global__ __launch_bounds__(256) void chain_reduce_quad_kernel(
    const float* __restrict__ x, int64_t ldx, int n0, const float* __restrict__ dy,
    const float* __restrict__ y, int nl, int64_t B, float* __restrict__ gout,
    float* __restrict__ part) {
  __shared__ float xs[kQuadRows * N0MAX];
  __shared__ float red[(N0MAX + 1) * 256];
  const int t = threadIdx.x;
  const int nq = nl / 4;
  const int P = 256 / nq;
  const int q = t % nq, ph = t / nq;
  const int j0 = 4 * q;
  const int64_t r0 = (int64_t)blockIdx.x * kQuadRows;
  const int64_t r1 = r0 + kQuadRows < B ? r0 + kQuadRows : B;
  const int nr = (int)(r1 - r0);
  for (int e = t; e < nr * n0; e += 256) {
    const int rr = e / n0;
    xs[e] = x[(r0 + rr) * ldx + (e - rr * n0)];
  }
  __syncthreads();
  float4 acc[N0MAX];
#pragma unroll
  for (int i = 0; i < N0MAX; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sacc = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int U = 4;
  if (ph < P) {
    for (int rb = ph; rb < nr; rb += U * P) {
      float4 g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = rb + u * P;
        const int64_t o = (r0 + (r < nr ? r : 0)) * nl + j0;
        const float4 d = *reinterpret_cast<const float4*>(dy + o);
        float4 yy = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ACT) yy = *reinterpret_cast<const float4*>(y + o);
        g[u] = r < nr ? make_float4(act_grad<ACT>(d.x, yy.x), act_grad<ACT>(d.y, yy.y),
                                    act_grad<ACT>(d.z, yy.z), act_grad<ACT>(d.w, yy.w))
                      : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = rb + u * P;
        if (r < nr) {
#pragma unroll
          for (int i = 0; i < N0MAX; ++i) {
            if (i < n0) {
              const float xv = xs[r * n0 + i];
              acc[i].x += xv * g[u].x;
              acc[i].y += xv * g[u].y;
              acc[i].z += xv * g[u].z;
              acc[i].w += xv * g[u].w;
            }
          }
          sacc.x += g[u].x;
          sacc.y += g[u].y;
          sacc.z += g[u].z;
          sacc.w += g[u].w;
          if (gout)
            *reinterpret_cast<float4*>(gout + (r0 + r) * nl + j0) = g[u];
        }
      }
    }
  }
  // fold the phases in order: red[i][column] (i == N0MAX: the column sum)
  for (int p = 0; p < P; ++p) {
    if (ph == p) {
#pragma unroll
      for (int i = 0; i <= N0MAX; ++i) {
        if (i < n0 || i == N0MAX) {
          const float4 v = i == N0MAX ? sacc : acc[i];
          float* dst = red + i * 256 + j0;
          if (p == 0) {
            dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
          } else {
            dst[0] += v.x; dst[1] += v.y; dst[2] += v.z; dst[3] += v.w;
          }
        }
      }
    }
    __syncthreads();
  }
  float* pp = part + (int64_t)blockIdx.x * ((int64_t)n0 * nl + nl);
  for (int e = t; e < (n0 + 1) * nl; e += 256) {
    const int i = e / nl, j = e - i * nl;
    pp[(int64_t)i * nl + j] = red[(i == n0 ? N0MAX : i) * 256 + j];
  }
}

// ---- parameter gradients of a 3-layer linear chain with a scalar output --------------------
// (the DLRM / DeepFM top MLP [n1, n2, 1]; see recommender_amd/nn.py chain_param_grads). With
// q2 = K3, q1 = K2·q2, T2 = K1[r]ᵀ·A, c2 = K2ᵀ·b1 + b2, T3 = K2ᵀ·T2, p = K1[r]·q1:
//   dK1[r[a], :] = A[a]·q1 (other rows 0), dK2 = (T2 + b1·s) ⊗ q2, dK3 = T3 + c2·s,
//   db1 = q1·s, db2 = q2·s, db3 = s, and p = Q_0 (the rank-one input gradient's row).
// Three launches of fixed-order dot products (deterministic).
struct Chain3Args {
  const float* K1;    // [n_full0, n1]
  const int32_t* r;   // [n0] rows of K1 the input holds (nullptr: identity, n_full0 == n0)
  const int32_t* inv; // [n_full0] position of each K1 row in r, -1 if absent (nullptr: identity)
  const float* b1;    // [n1] (nullable)
  const float* K2;    // [n1, n2]
  const float* b2;    // [n2] (nullable)
  const float* K3;    // [n2]
  const float* A;     // [n0]
  const float* s;     // [1]
  int n_full0, n0, n1, n2;
  float* q1;          // [n1] scratch
  float* T2;          // [n1] scratch
  float* c2;          // [n2] scratch
  float* T3;          // [n2] scratch
  float* dK1;         // [n_full0, n1]
  float* db1;         // [n1]
  float* dK2;         // [n1, n2]
  float* db2;         // [n2]
  float* dK3;         // [n2]
  float* db3;         // [1]
  float* p;           // [n0]
};

__device__ __forceinline__ float wave_sum(float v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// out[i] = Σ_k M[row(i), k] · v[k] (one wave per output, lanes stride k, fixed butterfly)
__device__ __forceinline__ void rowdot_wave(const float* M, int ld, int i_row, int n,
                                            const float* v, float* out_i, int lane) {
  float acc = 0.f;
#pragma unroll 4  // (four trips' loads in flight: one trip waited for its loads before the next)
  for (int k = lane; k < n; k += 64) acc += M[(int64_t)i_row * ld + k] * v[k];
  acc = wave_sum(acc);
  if (lane == 0) *out_i = acc;
}

// The weight-sized matrix-vector products of the chain: blocks of kC3Waves waves, so the
// column sums (k up to a few hundred deep) run 16-wide in k with four loads in flight per wave
// (they are latency-bound, not bandwidth-bound: 4 waves striding k one load at a time took
// 60 us for K1ᵀ·A at 480 x 512).
constexpr int kC3Waves = 16;

// out[c] = Σ_k M[row(k), c] · v[k] (+ add[c]) for a 64-column tile: kC3Waves waves stride k,
// folded in wave order
__device__ __forceinline__ void coldot_tile(const float* M, int ld, const int32_t* rowmap, int n,
                                            int ncol, int c0, const float* v, const float* add,
                                            float* out) {
  __shared__ float red[kC3Waves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = c0 + lane;
  float acc = 0.f;
  if (c < ncol) {
#pragma unroll 4
    for (int k = w; k < n; k += kC3Waves) acc += M[(int64_t)(rowmap ? rowmap[k] : k) * ld + c] * v[k];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < ncol) {
    float t = red[0][lane];
#pragma unroll
    for (int j = 1; j < kC3Waves; ++j) t += red[j][lane];
    out[c] = add ? t + add[c] : t;
  }
  __syncthreads();
}

// Bodies take the (virtual) block index so the grouped dense-tail launches (rs_dlrm_dense_tail)
// run exactly the arithmetic of the standalone kernels.
__device__ __forceinline__ void chain3_stage1_body(const Chain3Args& a, int blk) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nq = (a.n1 + kC3Waves - 1) / kC3Waves;  // q1 blocks (one wave per output)
  const int nt = (a.n1 + 63) / 64;                   // T2 column tiles
  if (blk < nq) {
    const int i = blk * kC3Waves + w;
    if (i < a.n1) rowdot_wave(a.K2, a.n2, i, a.n2, a.K3, a.q1 + i, lane);
    return;
  }
  blk -= nq;
  if (blk < nt) {
    coldot_tile(a.K1, a.n1, a.r, a.n0, a.n1, blk * 64, a.A, nullptr, a.T2);
    return;
  }
  blk -= nt;
  // c2 = K2ᵀ·b1 + b2
  if (a.b1) {
    coldot_tile(a.K2, a.n2, nullptr, a.n1, a.n2, blk * 64, a.b1, a.b2, a.c2);
  } else if (threadIdx.x < 64) {
    const int c = blk * 64 + threadIdx.x;
    if (c < a.n2) a.c2[c] = a.b2 ? a.b2[c] : 0.f;
  }
}
__global__ __launch_bounds__(kC3Waves * 64) void chain3_stage1(Chain3Args a) {
  chain3_stage1_body(a, blockIdx.x);
}

__device__ __forceinline__ void chain3_stage2_body(const Chain3Args& a, int blk) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int npb = (a.n0 + kC3Waves - 1) / kC3Waves;
  if (blk < npb) {
    const int i = blk * kC3Waves + w;
    if (i < a.n0) rowdot_wave(a.K1, a.n1, a.r ? a.r[i] : i, a.n1, a.q1, a.p + i, lane);
    return;
  }
  coldot_tile(a.K2, a.n2, nullptr, a.n1, a.n2, (blk - npb) * 64, a.T2, nullptr, a.T3);
}
__global__ __launch_bounds__(kC3Waves * 64) void chain3_stage2(Chain3Args a) {
  chain3_stage2_body(a, blockIdx.x);
}

__device__ __forceinline__ void chain3_stage3_body(const Chain3Args& a, int64_t e) {
  const float s = a.s[0];
  const int64_t n_k1 = (int64_t)a.n_full0 * a.n1, n_k2 = (int64_t)a.n1 * a.n2;
  if (e < n_k1) {
    const int row = (int)(e / a.n1), col = (int)(e - (int64_t)row * a.n1);
    const int ai = a.inv ? a.inv[row] : row;
    a.dK1[e] = ai >= 0 ? a.A[ai] * a.q1[col] : 0.f;
    return;
  }
  int64_t f = e - n_k1;
  if (f < n_k2) {
    const int b = (int)(f / a.n2), d = (int)(f - (int64_t)b * a.n2);
    const float m2 = a.b1 ? a.T2[b] + a.b1[b] * s : a.T2[b];
    a.dK2[f] = m2 * a.K3[d];
    return;
  }
  f -= n_k2;
  if (f < a.n2) {
    a.dK3[f] = a.T3[f] + a.c2[f] * s;
    a.db2[f] = a.K3[f] * s;
    return;
  }
  f -= a.n2;
  if (f < a.n1) {
    a.db1[f] = a.q1[f] * s;
    return;
  }
  if (f == a.n1) a.db3[0] = s;
}
__global__ __launch_bounds__(256) void chain3_stage3(Chain3Args a) {
  chain3_stage3_body(a, (int64_t)blockIdx.x * 256 + threadIdx.x);
}

// first level of a two-level fold for many chunks of a narrow row: block (cx, seg) folds the
// chunks of its segment (4 waves interleaved, then in wave order) into part2[seg][col]
__global__ __launch_bounds__(256) void fold_segments_kernel(const float* __restrict__ part,
                                                            int nchunks, int per_seg, int N,
                                                            float* __restrict__ part2) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int c0 = blockIdx.y * per_seg;
  const int c1 = min(c0 + per_seg, nchunks);
  float s = 0.f;
  if (col < N) {
#pragma unroll 4
    for (int c = c0 + w; c < c1; c += 4) s += part[(int64_t)c * N + col];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < N)
    part2[(int64_t)blockIdx.y * N + col] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// fixed two-level fold of nchunks partial rows [N] (deterministic for given nchunks)
int32_t fold_two_level(const float* part, int nchunks, int N, float* part2, float* out,
                       hipStream_t st) {
  constexpr int kSeg = 32;
  const int per = (int)ceil_div(nchunks, kSeg);
  const int nseg = (int)ceil_div(nchunks, per);
  fold_segments_kernel<<<dim3((unsigned)ceil_div(N, 64), (unsigned)nseg), 256, 0, st>>>(
      part, nchunks, per, N, part2);
  RS_CHECK_LAUNCH();
  fold_chunks_kernel<<<(unsigned)ceil_div(N, 64), 256, 0, st>>>(part2, nseg, N, out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}


// ---------------------------------------------------------------------------------------
// Composed forward of the ctr linear chains (nn.chain_forward, composed=True): the chain's
// hidden layers are linear (ctr/layers.py:8), so y = act(x·Q_0 + c_L). The weight-sized
// composition runs in one or two launches; the batch-deep evaluation is one memory-bound pass.
// ---------------------------------------------------------------------------------------
struct VecComposeArgs {
  const float* K1;   // [n_full0, n1]
  const int32_t* r;  // [n0] rows of K1 the input holds (nullptr: rows 0..n0)
  const float* b1;   // [n1] or nullptr
  const float* K2;   // [n1, n2]
  const float* b2;   // [n2] or nullptr
  const float* K3;   // [n2] (one output)
  const float* b3;   // [1] or nullptr
  int n0, n1, n2;
  float* q1;  // [n1] scratch: K2·K3
  float* cb;  // [1] scratch: K3ᵀ·b2 + b3
  float* q;   // [n0] out: K1[r]·q1 (= Q_0)
  float* c;   // [1] out: c_L = b3 + K3ᵀ·b2 + q1ᵀ·b1
};

__device__ __forceinline__ void vcompose_stage1_body(const VecComposeArgs& a, int blk) {
  const int lane = threadIdx.x & 63;
  const int i = blk * kC3Waves + (threadIdx.x >> 6);
  if (i < a.n1) {
    rowdot_wave(a.K2, a.n2, i, a.n2, a.K3, a.q1 + i, lane);
  } else if (i == a.n1) {
    float acc = 0.f;
    if (a.b2)
      for (int k = lane; k < a.n2; k += 64) acc += a.b2[k] * a.K3[k];
    acc = wave_sum(acc);
    if (lane == 0) a.cb[0] = a.b3 ? acc + a.b3[0] : acc;
  }
}
__global__ __launch_bounds__(kC3Waves * 64) void vcompose_stage1(VecComposeArgs a) {
  vcompose_stage1_body(a, blockIdx.x);
}

__device__ __forceinline__ void vcompose_stage2_body(const VecComposeArgs& a, int blk) {
  const int lane = threadIdx.x & 63;
  const int i = blk * kC3Waves + (threadIdx.x >> 6);
  if (i < a.n0) {
    rowdot_wave(a.K1, a.n1, a.r ? a.r[i] : i, a.n1, a.q1, a.q + i, lane);
  } else if (i == a.n0) {
    float acc = 0.f;
    if (a.b1)
      for (int k = lane; k < a.n1; k += 64) acc += a.b1[k] * a.q1[k];
    acc = wave_sum(acc);
    if (lane == 0) a.c[0] = acc + a.cb[0];
  }
}
__global__ __launch_bounds__(kC3Waves * 64) void vcompose_stage2(VecComposeArgs a) {
  vcompose_stage2_body(a, blockIdx.x);
}

// Narrow-input product with a bias row: out[i, c] = Σ_k M̃[i, k]·K[k, c] (+ b[c] on row m),
// M̃ = [M; cin] ([m + 1, k], m < kAugRows). Chained twice it composes [K1; b1]·K2 + [0; b2]
// and then ·K3 + [0; b3]: rows 0..m-1 of the result are Q = K1·K2·K3, row m is c_L. M̃ is
// staged in LDS (one coalesced pass, every load in flight at once); a block covers 64 columns,
// its kC3Waves waves stride k eight loads of K at a time, and are folded in wave order.
constexpr int kAugRows = 33;
constexpr int kAugLds = 16896;  // floats of M̃ staged in LDS: (m + 1)·k <= kAugLds

template <int MR>
__device__ __forceinline__ void aug_product_body(
    const float* __restrict__ M, int ldm, int m, const float* __restrict__ cin,
    const float* __restrict__ K, int k, int n, const float* __restrict__ b,
    float* __restrict__ out, int bx) {
  extern __shared__ float ms[];  // max((m + 1)·k, 8·MR·64) floats (aug_lds_bytes)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  {  // staged 8 passes' loads at a time, unguarded (guarded, each pass waited for its load)
    constexpr int kSB = 8, kT = kC3Waves * 64;
    const int tot = (m + 1) * k;
    for (int e0 = threadIdx.x; e0 < tot; e0 += kSB * kT) {
      float v[kSB];
#pragma unroll
      for (int j = 0; j < kSB; ++j) {
        const int e = e0 + j * kT < tot ? e0 + j * kT : e0;
        const int i = e / k, kk = e - i * k;
        v[j] = *(i < m ? M + (int64_t)i * ldm + kk : (cin ? cin + kk : M));
      }
#pragma unroll
      for (int j = 0; j < kSB; ++j) {
        const int e = e0 + j * kT;
        if (e < tot) ms[e] = (e / k < m || cin) ? v[j] : 0.f;
      }
    }
  }
  __syncthreads();
  const int c = bx * 64 + lane;
  float acc[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i) acc[i] = 0.f;
  if (c < n) {
    constexpr int U = 8;
    int kk = w;
    for (; kk + (U - 1) * kC3Waves < k; kk += U * kC3Waves) {
      float kv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) kv[u] = K[(int64_t)(kk + u * kC3Waves) * n + c];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float* mr = ms + kk + u * kC3Waves;
#pragma unroll
        for (int i = 0; i < MR; ++i)
          if (i <= m) acc[i] += mr[i * k] * kv[u];
      }
    }
    for (; kk < k; kk += kC3Waves) {
      const float kv = K[(int64_t)kk * n + c];
#pragma unroll
      for (int i = 0; i < MR; ++i)
        if (i <= m) acc[i] += ms[i * k + kk] * kv;
    }
  }
  // fold: waves [8, 16) park their partials in the (consumed) staging buffer, waves [0, 8)
  // add them (wave w + w), then every partial row is folded in wave order by output
  static_assert(kC3Waves == 16 && 8 * MR * 64 <= kAugLds, "fold layout");
  __syncthreads();
  float* part = ms;  // [8][MR][64]
  if (w >= 8) {
#pragma unroll
    for (int i = 0; i < MR; ++i) part[((w - 8) * MR + i) * 64 + lane] = acc[i];
  }
  __syncthreads();
  if (w < 8) {
#pragma unroll
    for (int i = 0; i < MR; ++i) acc[i] += part[(w * MR + i) * 64 + lane];
  }
  __syncthreads();
  if (w < 8) {
#pragma unroll
    for (int i = 0; i < MR; ++i) part[(w * MR + i) * 64 + lane] = acc[i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < (m + 1) * 64; e += kC3Waves * 64) {
    const int i = e >> 6, cl = e & 63, cc = bx * 64 + cl;
    if (cc >= n) continue;
    float t = part[i * 64 + cl];
#pragma unroll
    for (int j = 1; j < 8; ++j) t += part[(j * MR + i) * 64 + cl];
    if (i == m && b) t += b[cc];
    out[(int64_t)i * n + cc] = t;
  }
}
template <int MR>
__global__ __launch_bounds__(kC3Waves * 64) void aug_product_kernel(
    const float* __restrict__ M, int ldm, int m, const float* __restrict__ cin,
    const float* __restrict__ K, int k, int n, const float* __restrict__ b,
    float* __restrict__ out) {
  aug_product_body<MR>(M, ldm, m, cin, K, k, n, b, out, blockIdx.x);
}

template <int ACT>
__device__ __forceinline__ float act_fwd(float v) {
  if constexpr (ACT == 1) return v > 0.f ? v : 0.f;
  if constexpr (ACT == 2) return 1.f / (1.f + expf(-v));
  return v;
}

// y[b, :] = act(x[b, :n0]·Q + c) for a narrow input (n0 < kAugRows): Q̃ = [Q; c] and a tile of
// kNarrowRows input rows are staged in LDS; the block's lanes each own one float4 column and
// walk the tile's rows (16-byte stores, consecutive lanes consecutive columns).
constexpr int kNarrowRows = 64;

template <int ACT, int N0MAX>
__global__ __launch_bounds__(256) void affine_narrow_fwd_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t B, int n0, const float* __restrict__ Qa,
    int n, float* __restrict__ y, int64_t ldy) {
  __shared__ float xs[kNarrowRows * N0MAX];
  const int nq = n >> 2;  // float4 columns (<= 64)
  const int rpb = 256 / nq;  // rows in flight per pass
  const int t = threadIdx.x % nq, rl = threadIdx.x / nq;
  // this lane's column of Q̃ = [Q; c] in registers (the loop below is unrolled over N0MAX).
  // Round 6: the first tile's x rows, then Q̃'s column, are loaded unguarded and together, so a
  // block waits one round trip for both (guarded per element, the staging loop waited for each
  // of its passes and for the column before it); the next tile's rows are loaded while this one
  // is computed
  constexpr int kPer = kNarrowRows * N0MAX / 256;
  const int64_t stride = (int64_t)gridDim.x * kNarrowRows;
  int64_t r0 = (int64_t)blockIdx.x * kNarrowRows;
  float xv[kPer];
  auto load_x = [&](int64_t rb) {
    const int nrb = B - rb < kNarrowRows ? (int)(B - rb) : kNarrowRows;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = threadIdx.x + i * 256;
      const int rr = e / n0, k = e - rr * n0;
      xv[i] = x[e < nrb * n0 ? (rb + rr) * ldx + k : rb * ldx];
    }
  };
  if (r0 < B) load_x(r0);
  float4 qr[N0MAX + 1];
#pragma unroll
  for (int k = 0; k <= N0MAX; ++k)
    qr[k] = reinterpret_cast<const float4*>(Qa)[(k <= n0 ? k : 0) * nq + t];
  float4 cc = qr[0];
#pragma unroll
  for (int k = 0; k <= N0MAX; ++k) {
    if (k == n0) cc = qr[k];
    if (k >= n0) qr[k] = make_float4(0.f, 0.f, 0.f, 0.f);  // (the rows loop stops at n0 anyway)
  }
  for (; r0 < B; r0 += stride) {
    const int nr = B - r0 < kNarrowRows ? (int)(B - r0) : kNarrowRows;
    __syncthreads();  // previous tile consumed
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = threadIdx.x + i * 256;
      if (e < nr * n0) xs[e] = xv[i];
    }
    __syncthreads();
    if (r0 + stride < B) load_x(r0 + stride);
    if (rl >= rpb) continue;
    for (int rr = rl; rr < nr; rr += rpb) {
      const float* xr = xs + rr * n0;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < N0MAX; ++k) {
        if (k < n0) {
          const float xk = xr[k];
          acc.x += xk * qr[k].x;
          acc.y += xk * qr[k].y;
          acc.z += xk * qr[k].z;
          acc.w += xk * qr[k].w;
        }
      }
      float4 o;
      o.x = act_fwd<ACT>(acc.x + cc.x);
      o.y = act_fwd<ACT>(acc.y + cc.y);
      o.z = act_fwd<ACT>(acc.z + cc.z);
      o.w = act_fwd<ACT>(acc.w + cc.w);
      reinterpret_cast<float4*>(y + (r0 + rr) * ldy)[t] = o;
    }
  }
}

// Backward of a narrow-input chain (nn._narrow_chain_grads): with Ã = [xᵀ·G; Σ G] and
// P_L = Ã, P_{j-1} = P_j·K_jᵀ, every gradient is dK_j = R̃_{j-1}ᵀ·P_j, db_j = P_j[n0]
// (R̃_j = [K_1···K_j; c_j], the forward composition's rows; R̃_0 = [I; 0]).
// rt_product: out [m+1, n] = P [m+1, k]·Kᵀ, K [n, k] row-major: P staged in LDS, one wave per
// output column (lanes stride the contiguous row of K), fixed butterfly per row.
template <int MR>
__device__ __forceinline__ void rt_product_body(const float* __restrict__ P, int m,
                                                const float* __restrict__ K, int k, int n,
                                                float* __restrict__ out, int bx) {
  extern __shared__ float ps[];  // (m + 1)·k floats
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  {  // staged 8 passes' loads at a time (one pass per trip waited for its load)
    constexpr int kSB = 8, kT = kC3Waves * 64;
    const int tot = (m + 1) * k;
    for (int e0 = threadIdx.x; e0 < tot; e0 += kSB * kT) {
      float v[kSB];
#pragma unroll
      for (int j = 0; j < kSB; ++j) v[j] = P[e0 + j * kT < tot ? e0 + j * kT : e0];
#pragma unroll
      for (int j = 0; j < kSB; ++j)
        if (e0 + j * kT < tot) ps[e0 + j * kT] = v[j];
    }
  }
  __syncthreads();
  const int c = bx * kC3Waves + w;
  if (c >= n) return;
  float acc[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i) acc[i] = 0.f;
  const float* kr = K + (int64_t)c * k;
#pragma unroll 4
  for (int kk = lane; kk < k; kk += 64) {
    const float kv = kr[kk];
#pragma unroll
    for (int i = 0; i < MR; ++i)
      if (i <= m) acc[i] += ps[i * k + kk] * kv;
  }
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    if (i > m) break;
    const float v = wave_sum(acc[i]);
    if (lane == 0) out[(int64_t)i * n + c] = v;
  }
}
template <int MR>
__global__ __launch_bounds__(kC3Waves * 64) void rt_product_kernel(
    const float* __restrict__ P, int m, const float* __restrict__ K, int k, int n,
    float* __restrict__ out) {
  rt_product_body<MR>(P, m, K, k, n, out, blockIdx.x);
}

// out [na, nb] = R̃ᵀ·P: R̃ = [R (m rows, stride ldr); rlast] ([m+1, na], rlast NULL: a zero
// row), P [m+1, nb] contiguous; four output columns per thread, r ascending.
// P4: P is 16-byte aligned (one float4 load per row); else four scalar loads, same arithmetic
template <bool P4 = true>
__device__ __forceinline__ void outer_sum_body(const float* __restrict__ R, int ldr, int m,
                                               const float* __restrict__ rlast, int na,
                                               const float* __restrict__ P, int nb,
                                               float* __restrict__ out, int64_t e) {
  const int nbq = nb >> 2;
  if (e >= (int64_t)na * nbq) return;
  const int a = (int)(e / nbq), bq = (int)(e - (int64_t)a * nbq);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // rows loaded 8 at a time, unguarded (a row past the last reads row 0 and is not added):
  // one row per trip with the rlast / break branches waited for each load in turn (round 6)
  const int rows = rlast ? m + 1 : m;
  constexpr int kB = 8;
  for (int r0 = 0; r0 < rows; r0 += kB) {
    float rv[kB];
    float4 pv[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const int r = r0 + j < rows ? r0 + j : 0;
      rv[j] = (r < m || !rlast) ? R[(int64_t)r * ldr + a] : rlast[a];
      if constexpr (P4) {
        pv[j] = reinterpret_cast<const float4*>(P)[(int64_t)r * nbq + bq];
      } else {
        const float* pp = P + ((int64_t)r * nbq + bq) * 4;
        pv[j] = make_float4(pp[0], pp[1], pp[2], pp[3]);
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      if (r0 + j < rows) {
        acc.x += rv[j] * pv[j].x;
        acc.y += rv[j] * pv[j].y;
        acc.z += rv[j] * pv[j].z;
        acc.w += rv[j] * pv[j].w;
      }
    }
  }
  reinterpret_cast<float4*>(out)[e] = acc;
}
__global__ __launch_bounds__(256) void outer_sum_kernel(const float* __restrict__ R, int ldr, int m,
                                                        const float* __restrict__ rlast, int na,
                                                        const float* __restrict__ P, int nb,
                                                        float* __restrict__ out) {
  outer_sum_body(R, ldr, m, rlast, na, P, nb, out, (int64_t)blockIdx.x * 256 + threadIdx.x);
}

// y[b] = act(x[b, :n0]·q + c[0]): one wave per row (16-byte loads, q held in registers),
// rows grid-strided over the waves, fixed butterfly fold.
template <int ACT>
__global__ __launch_bounds__(256) void rowdot_act_kernel(const float* __restrict__ x, int64_t ldx,
                                                         int64_t B, int n0,
                                                         const float* __restrict__ q,
                                                         const float* __restrict__ c,
                                                         float* __restrict__ y) {
  constexpr int kMaxQ = 4;  // float4 chunks per lane: n0 <= 1024
  const int lane = threadIdx.x & 63;
  const int nq = n0 >> 2;
  float4 qv[kMaxQ];
#pragma unroll
  for (int j = 0; j < kMaxQ; ++j) {
    const int e = lane + 64 * j;
    qv[j] = e < nq ? reinterpret_cast<const float4*>(q)[e] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float cc = c[0];
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < B; row += nw) {
    const float4* xr = reinterpret_cast<const float4*>(x + row * ldx);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxQ; ++j) {
      const int e = lane + 64 * j;
      if (e < nq) {
        const float4 v = xr[e];
        acc += v.x * qv[j].x + v.y * qv[j].y + v.z * qv[j].z + v.w * qv[j].w;
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) y[row] = act_fwd<ACT>(acc + cc);
  }
}

// ---------------------------------------------------------------------------------------
// The production DLRM step's dense tail (rs_dlrm_dense_tail): every MLP parameter gradient of
// the [n0 -> n1 -> n2 -> 1] top chain (rs_chain3_vec_grads) and the narrow [m -> n1 -> n2 -> n3]
// bottom chain (nn._narrow_chain_grads_hip), the SGD update of all twelve parameters, and the
// next step's compositions (rs_chain_aug_product x 2, rs_chain3_vec_compose) in six launches
// instead of sixteen. Independent products share a launch (block ranges select the body); the
// bodies are the standalone kernels' own, so every value is bit-identical to the separate calls.
// Launch boundaries stay where a product reads another's output (no in-launch grid sync: these
// launches run beside the HBM-bound sparse-update walk, which holds most CU slots).
// ---------------------------------------------------------------------------------------
struct TailOuter {
  const float* R;
  int ldr, m;
  const float* rlast;
  int na;
  const float* P;
  int nb;
  float* out;
  int64_t units() const { return (int64_t)na * (nb >> 2); }
};
struct TailRt {
  const float* P;
  int m;
  const float* K;
  int k, n;
  float* out;
};
struct TailAug {
  const float* M;
  int ldm, m;
  const float* cin;
  const float* K;
  int k, n;
  const float* b;
  float* out;
};
constexpr int kTailParams = 12;
struct TailSgd {
  float* p[kTailParams];
  const float* g[kTailParams];
  int64_t off[kTailParams + 1];  // element offsets of the concatenated parameter space
  float lr;
};

// outer units -> 1024-thread blocks (4 virtual 256-thread blocks each)
template <bool P4>
__device__ __forceinline__ void tail_outer(const TailOuter& o, int bx) {
  outer_sum_body<P4>(o.R, o.ldr, o.m, o.rlast, o.na, o.P, o.nb, o.out, (int64_t)bx * 1024 + threadIdx.x);
}

// grads 1: top stage 1 | bottom dK3 = R~2ᵀ·P | bottom P2 = P·K3ᵀ
__global__ __launch_bounds__(kC3Waves * 64) void tail_grads1(Chain3Args top, int nb_top, TailOuter o,
                                                             int nb_o, TailRt r) {
  int bx = blockIdx.x;
  if (bx < nb_top) { chain3_stage1_body(top, bx); return; }
  bx -= nb_top;
  if (bx < nb_o) { tail_outer<false>(o, bx); return; }
  rt_product_body<16>(r.P, r.m, r.K, r.k, r.n, r.out, bx - nb_o);
}
// grads 2: top stage 2 | bottom dK2 = [K1; b1]ᵀ·P2 | bottom P1 = P2·K2ᵀ (= [dK1; db1])
__global__ __launch_bounds__(kC3Waves * 64) void tail_grads2(Chain3Args top, int nb_top, TailOuter o,
                                                             int nb_o, TailRt r) {
  int bx = blockIdx.x;
  if (bx < nb_top) { chain3_stage2_body(top, bx); return; }
  bx -= nb_top;
  if (bx < nb_o) { tail_outer<true>(o, bx); return; }
  rt_product_body<16>(r.P, r.m, r.K, r.k, r.n, r.out, bx - nb_o);
}
// grads 3: the top chain's elementwise gradients
__global__ __launch_bounds__(kC3Waves * 64) void tail_grads3(Chain3Args top) {
  chain3_stage3_body(top, (int64_t)blockIdx.x * 1024 + threadIdx.x);
}
// SGD over the concatenated parameters: p = p + (-lr)·g, the update of torch.optim.SGD's
// foreach path (_foreach_add_(params, grads, alpha=-lr)) with its fused multiply-add
__global__ __launch_bounds__(256) void tail_sgd(TailSgd a) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= a.off[kTailParams]) return;
  int j = 0;
#pragma unroll
  for (int i = 1; i < kTailParams; ++i) j += e >= a.off[i] ? 1 : 0;
  const int64_t o = e - a.off[j];
#ifndef RS_SGD_UNFUSED
  a.p[j][o] = fmaf(-a.lr, a.g[j][o], a.p[j][o]);
#else
  a.p[j][o] = a.p[j][o] + (-a.lr) * a.g[j][o];
#endif
}
// compose 1: bottom R~2' = [K1; b1]·K2 + [0; b2] | top q1 = K2·K3, cb
__global__ __launch_bounds__(kC3Waves * 64) void tail_compose1(TailAug g, int nb_aug, VecComposeArgs v) {
  if ((int)blockIdx.x < nb_aug) {
    aug_product_body<16>(g.M, g.ldm, g.m, g.cin, g.K, g.k, g.n, g.b, g.out, blockIdx.x);
    return;
  }
  vcompose_stage1_body(v, blockIdx.x - nb_aug);
}
// compose 2: bottom R~3' = R~2'·K3 + [0; b3] | top q = K1[rows]·q1, c
__global__ __launch_bounds__(kC3Waves * 64) void tail_compose2(TailAug g, int nb_aug, VecComposeArgs v) {
  if ((int)blockIdx.x < nb_aug) {
    aug_product_body<16>(g.M, g.ldm, g.m, g.cin, g.K, g.k, g.n, g.b, g.out, blockIdx.x);
    return;
  }
  vcompose_stage2_body(v, blockIdx.x - nb_aug);
}

}  // namespace rs

using namespace rs;

extern "C" size_t rs_act_bwd_colsum_workspace_size(int64_t B, int32_t N) {
  return (size_t)ceil_div(B, kColRows) * N * sizeof(float);
}

extern "C" int32_t rs_act_bwd_colsum_ld(const float* dy, int64_t ld_dy, const float* y,
                                        int64_t ld_y, int64_t B, int32_t N, int32_t act, float* dz,
                                        int64_t ld_dz, float* db, void* workspace, size_t ws_bytes,
                                        void* stream) {
  RS_CHECK_ARG(B >= 0 && N >= 1 && act >= 0 && act <= 2, "bad arguments");
  RS_CHECK_ARG(act == 0 || (y && dz), "activation backward needs y and dz");
  RS_CHECK_ARG(ld_dy >= N && (act == 0 || (ld_y >= N && ld_dz >= N)), "row strides must be >= N");
  RS_CHECK_ARG(ws_bytes >= rs_act_bwd_colsum_workspace_size(B, N), "workspace too small");
  hipStream_t st = as_stream(stream);
  if (B == 0) {
    RS_CHECK_HIP(hipMemsetAsync(db, 0, (size_t)N * 4, st));
    return RS_OK;
  }
  const int nchunks = (int)ceil_div(B, kColRows);
  float* part = static_cast<float*>(workspace);
  auto al16 = [](const void* p, int64_t ld) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 4 == 0;
  };
  const bool v4 = N % 4 == 0 && al16(dy, ld_dy) && (act == 0 || (al16(y, ld_y) && al16(dz, ld_dz)));
  if (act == 0) ld_y = ld_dz = N;  // y / dz unread
  if (v4) {
    dim3 grid((unsigned)ceil_div(N, 64), (unsigned)nchunks);
    switch (act) {
      case 0: act_bwd_colsum_kernel<0, 4><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, ld_dy, ld_y, ld_dz); break;
      case 1: act_bwd_colsum_kernel<1, 4><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, ld_dy, ld_y, ld_dz); break;
      default: act_bwd_colsum_kernel<2, 4><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, ld_dy, ld_y, ld_dz); break;
    }
  } else {
    dim3 grid((unsigned)ceil_div(N, 16), (unsigned)nchunks);
    switch (act) {
      case 0: act_bwd_colsum_kernel<0, 1><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, ld_dy, ld_y, ld_dz); break;
      case 1: act_bwd_colsum_kernel<1, 1><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, ld_dy, ld_y, ld_dz); break;
      default: act_bwd_colsum_kernel<2, 1><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, ld_dy, ld_y, ld_dz); break;
    }
  }
  RS_CHECK_LAUNCH();
  fold_chunks_kernel<<<(unsigned)ceil_div(N, 64), 256, 0, st>>>(part, nchunks, N, db);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

// n_groups row groups of B / n_groups rows each (a whole number of 512-row chunks): one masking
// pass over all rows, then each group's column sums folded apart — db [n_groups, N]. MMOE's
// batched expert layer: the [E, B, H] gradient masked in one launch, per-expert bias sums.
extern "C" int32_t rs_act_bwd_colsum_groups(const float* dy, const float* y, int64_t B, int32_t N,
                                            int32_t act, int32_t n_groups, float* dz, float* db,
                                            void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(B >= 1 && N >= 1 && act >= 1 && act <= 2 && n_groups >= 1 && B % n_groups == 0 &&
                   (B / n_groups) % kColRows == 0,
               "rs_act_bwd_colsum_groups: act 1 / 2 and groups of whole %d-row chunks", kColRows);
  RS_CHECK_ARG(dy && y && dz && db, "null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_act_bwd_colsum_workspace_size(B, N), "workspace too small");
  hipStream_t st = as_stream(stream);
  const int nchunks = (int)ceil_div(B, kColRows);
  float* part = static_cast<float*>(workspace);
  const bool v4 = N % 4 == 0 && ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(y) |
                                  reinterpret_cast<uintptr_t>(dz)) & 15) == 0;
  if (v4) {
    dim3 grid((unsigned)ceil_div(N, 64), (unsigned)nchunks);
    if (act == 1) act_bwd_colsum_kernel<1, 4><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, N, N, N);
    else act_bwd_colsum_kernel<2, 4><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, N, N, N);
  } else {
    dim3 grid((unsigned)ceil_div(N, 16), (unsigned)nchunks);
    if (act == 1) act_bwd_colsum_kernel<1, 1><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, N, N, N);
    else act_bwd_colsum_kernel<2, 1><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part, N, N, N);
  }
  RS_CHECK_LAUNCH();
  fold_chunk_groups_kernel<<<dim3((unsigned)ceil_div(N, 64), (unsigned)n_groups), 256, 0, st>>>(
      part, nchunks / n_groups, N, db);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_act_bwd_colsum(const float* dy, const float* y, int64_t B, int32_t N,
                                     int32_t act, float* dz, float* db, void* workspace,
                                     size_t ws_bytes, void* stream) {
  return rs_act_bwd_colsum_ld(dy, N, y, N, B, N, act, dz, N, db, workspace, ws_bytes, stream);
}

extern "C" size_t rs_chain_reduce_workspace_size(int64_t B, int32_t n0, int32_t nl) {
  const int rows = nl == 1 ? kVecRows : kChainRows;
  // chunk partials + 32 segment partials of the two-level fold
  return ((size_t)ceil_div(B < 1 ? 1 : B, rows) + 32) * ((size_t)n0 * nl + nl) * sizeof(float) + 256;
}

extern "C" int32_t rs_chain_reduce(const float* x, int64_t ldx, int32_t n0, const float* dy,
                                   const float* y, int32_t nl, int32_t act, int64_t B, float* out,
                                   float* g_out, void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(B >= 0 && n0 >= 1 && nl >= 1 && ldx >= n0 && act >= 0 && act <= 2,
               "rs_chain_reduce: bad arguments");
  RS_CHECK_ARG(act == 0 || y, "rs_chain_reduce: activation backward needs y");
  RS_CHECK_ARG((nl == 1 && n0 <= 1024) || (nl <= 256 && n0 <= 32),
               "rs_chain_reduce: shape outside the kernels (nl == 1 and n0 <= 1024, or nl <= 256 "
               "and n0 <= 32)");
  RS_CHECK_ARG(ws_bytes >= rs_chain_reduce_workspace_size(B, n0, nl),
               "rs_chain_reduce: workspace too small");
  hipStream_t st = as_stream(stream);
  const int M = n0 * nl + nl;
  if (B == 0) {
    RS_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)M * 4, st));
    return RS_OK;
  }
  float* part = static_cast<float*>(workspace);
  int nchunks = (int)ceil_div(B, kChainRows);
  if (nl == 1) {
    RS_CHECK_ARG(n0 % 4 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
                 "rs_chain_reduce: nl == 1 needs n0, ldx multiples of 4 and a 16-B aligned x");
    nchunks = (int)ceil_div(B, kVecRows);
    int cgp = 1;
    while (cgp < n0 / 4) cgp <<= 1;
    switch (act) {
      case 0: chain_reduce_vec_kernel<0><<<nchunks, 256, 0, st>>>(x, ldx, n0, cgp, dy, y, B, g_out, part); break;
      case 1: chain_reduce_vec_kernel<1><<<nchunks, 256, 0, st>>>(x, ldx, n0, cgp, dy, y, B, g_out, part); break;
      default: chain_reduce_vec_kernel<2><<<nchunks, 256, 0, st>>>(x, ldx, n0, cgp, dy, y, B, g_out, part); break;
    }
  } else if (nl % 4 == 0 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0 &&
             (!y || (reinterpret_cast<uintptr_t>(y) & 15) == 0) &&
             (!g_out || (reinterpret_cast<uintptr_t>(g_out) & 15) == 0)) {
    nchunks = (int)ceil_div(B, kQuadRows);
    auto go = [&](auto kern) { kern<<<nchunks, 256, 0, st>>>(x, ldx, n0, dy, y, nl, B, g_out, part); };
    if (n0 <= 16) {
      switch (act) {
        case 0: go(chain_reduce_quad_kernel<0, 16>); break;
        case 1: go(chain_reduce_quad_kernel<1, 16>); break;
        default: go(chain_reduce_quad_kernel<2, 16>); break;
      }
    } else {
      switch (act) {
        case 0: go(chain_reduce_quad_kernel<0, 32>); break;
        case 1: go(chain_reduce_quad_kernel<1, 32>); break;
        default: go(chain_reduce_quad_kernel<2, 32>); break;
      }
    }
  } else {
    int nlp = 1;
    while (nlp < nl) nlp <<= 1;
    auto go = [&](auto kern) { kern<<<nchunks, 256, 0, st>>>(x, ldx, n0, dy, y, nl, nlp, B, g_out, part); };
    if (n0 <= 16) {
      switch (act) {
        case 0: go(chain_reduce_outer_kernel<0, 16>); break;
        case 1: go(chain_reduce_outer_kernel<1, 16>); break;
        default: go(chain_reduce_outer_kernel<2, 16>); break;
      }
    } else {
      switch (act) {
        case 0: go(chain_reduce_outer_kernel<0, 32>); break;
        case 1: go(chain_reduce_outer_kernel<1, 32>); break;
        default: go(chain_reduce_outer_kernel<2, 32>); break;
      }
    }
  }
  RS_CHECK_LAUNCH();
  return fold_two_level(part, nchunks, M, part + (size_t)nchunks * M, out, st);
}

extern "C" int32_t rs_chain3_vec_grads(const float* K1, const int32_t* rows, const int32_t* inv,
                                       int32_t n_full0, int32_t n0, const float* b1,
                                       const float* K2, const float* b2, const float* K3,
                                       int32_t n1, int32_t n2, const float* A, const float* s,
                                       float* dK1, float* db1, float* dK2, float* db2, float* dK3,
                                       float* db3, float* p, void* workspace, size_t ws_bytes,
                                       void* stream) {
  RS_CHECK_ARG(n0 >= 1 && n1 >= 1 && n2 >= 1 && n_full0 >= n0 && (rows != nullptr) == (inv != nullptr) &&
                   (rows || n_full0 == n0),
               "rs_chain3_vec_grads: bad sizes");
  RS_CHECK_ARG(ws_bytes >= (size_t)(2 * n1 + 2 * n2) * sizeof(float), "workspace too small");
  hipStream_t st = as_stream(stream);
  float* w = static_cast<float*>(workspace);
  Chain3Args a{K1, rows, inv, b1, K2, b2, K3, A, s, n_full0, n0, n1, n2,
               w, w + n1, w + 2 * n1, w + 2 * n1 + n2, dK1, db1, dK2, db2, dK3, db3, p};
  const unsigned g1 = (unsigned)(ceil_div(n1, kC3Waves) + ceil_div(n1, 64) + ceil_div(n2, 64));
  chain3_stage1<<<g1, kC3Waves * 64, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  const unsigned g2 = (unsigned)(ceil_div(n0, kC3Waves) + ceil_div(n2, 64));
  chain3_stage2<<<g2, kC3Waves * 64, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  const int64_t tot = (int64_t)n_full0 * n1 + (int64_t)n1 * n2 + n2 + n1 + 1;
  chain3_stage3<<<(unsigned)ceil_div(tot, 256), 256, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_chain3_vec_compose(const float* K1, const int32_t* rows, int32_t n0,
                                         const float* b1, const float* K2, const float* b2,
                                         const float* K3, const float* b3, int32_t n1,
                                         int32_t n2, float* q, float* c, void* workspace,
                                         size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(n0 >= 1 && n1 >= 1 && n2 >= 1 && K1 && K2 && K3 && q && c,
               "rs_chain3_vec_compose: bad arguments");
  RS_CHECK_ARG(ws_bytes >= (size_t)(n1 + 1) * sizeof(float), "workspace too small");
  hipStream_t st = as_stream(stream);
  float* w = static_cast<float*>(workspace);
  VecComposeArgs a{K1, rows, b1, K2, b2, K3, b3, n0, n1, n2, w, w + n1, q, c};
  vcompose_stage1<<<(unsigned)ceil_div(n1 + 1, kC3Waves), kC3Waves * 64, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  vcompose_stage2<<<(unsigned)ceil_div(n0 + 1, kC3Waves), kC3Waves * 64, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_chain_aug_product(const float* M, int32_t ldm, int32_t m, const float* cin,
                                        const float* K, int32_t k, int32_t n, const float* b,
                                        float* out, void* stream) {
  RS_CHECK_ARG(m >= 0 && m < kAugRows && k >= 1 && n >= 1 && ldm >= k && K && out &&
                   (m == 0 || M) && (int64_t)(m + 1) * k <= kAugLds,
               "rs_chain_aug_product: bad arguments");
  const unsigned g = (unsigned)ceil_div(n, 64);
  hipStream_t st = as_stream(stream);
  // LDS sized to the product (not the kAugLds maximum): a small block footprint lets these
  // latency-bound launches find room beside the co-running sparse-update walk
  const int mr = m < 16 ? 16 : kAugRows;
  const size_t lds = (size_t)std::max<int64_t>((int64_t)(m + 1) * k, (int64_t)8 * mr * 64) * 4;
  if (m < 16)
    aug_product_kernel<16><<<g, kC3Waves * 64, lds, st>>>(M, ldm, m, cin, K, k, n, b, out);
  else
    aug_product_kernel<kAugRows><<<g, kC3Waves * 64, lds, st>>>(M, ldm, m, cin, K, k, n, b, out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

static int fwd_blocks(int64_t units, int64_t per_block) {
  const int64_t b = ceil_div(units, per_block);
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

extern "C" int32_t rs_affine_narrow_fwd(const float* x, int64_t ldx, int64_t B, int32_t n0,
                                        const float* Qa, int32_t n, int32_t act, float* y,
                                        int64_t ldy, void* stream) {
  RS_CHECK_ARG(B >= 0 && n0 >= 1 && n0 < kAugRows && n >= 4 && n <= 256 && n % 4 == 0 &&
                   ldx >= n0 && ldy >= n && ldy % 4 == 0 && act >= 0 && act <= 2,
               "rs_affine_narrow_fwd: bad sizes");
  RS_CHECK_ARG(B == 0 || (x && Qa && y), "null pointer");
  RS_CHECK_ARG((reinterpret_cast<uintptr_t>(Qa) | reinterpret_cast<uintptr_t>(y)) % 16 == 0,
               "rs_affine_narrow_fwd: Qa and y must be 16-byte aligned");
  if (B == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  const int g = fwd_blocks(B, kNarrowRows);
#define RS_NARROW(A, M) affine_narrow_fwd_kernel<A, M><<<g, 256, 0, st>>>(x, ldx, B, n0, Qa, n, y, ldy)
  if (n0 < 16) {
    if (act == 0) RS_NARROW(0, 16); else if (act == 1) RS_NARROW(1, 16); else RS_NARROW(2, 16);
  } else {
    if (act == 0) RS_NARROW(0, 32); else if (act == 1) RS_NARROW(1, 32); else RS_NARROW(2, 32);
  }
#undef RS_NARROW
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_rowdot_act(const float* x, int64_t ldx, int64_t B, int32_t n0,
                                 const float* q, const float* c, int32_t act, float* y,
                                 void* stream) {
  RS_CHECK_ARG(B >= 0 && n0 >= 4 && n0 <= 1024 && n0 % 4 == 0 && ldx >= n0 && ldx % 4 == 0 &&
                   act >= 0 && act <= 2,
               "rs_rowdot_act: bad sizes");
  RS_CHECK_ARG(B == 0 || (x && q && c && y), "null pointer");
  RS_CHECK_ARG((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(q)) % 16 == 0,
               "rs_rowdot_act: x and q must be 16-byte aligned");
  if (B == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  const int g = fwd_blocks(B, 4 * 4);  // 4 rows per wave on average
  switch (act) {
    case 0: rowdot_act_kernel<0><<<g, 256, 0, st>>>(x, ldx, B, n0, q, c, y); break;
    case 1: rowdot_act_kernel<1><<<g, 256, 0, st>>>(x, ldx, B, n0, q, c, y); break;
    default: rowdot_act_kernel<2><<<g, 256, 0, st>>>(x, ldx, B, n0, q, c, y); break;
  }
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_chain_rt_product(const float* P, int32_t m, const float* K, int32_t k,
                                       int32_t n, float* out, void* stream) {
  RS_CHECK_ARG(m >= 0 && m < kAugRows && k >= 1 && n >= 1 && P && K && out &&
                   (int64_t)(m + 1) * k <= kAugLds,
               "rs_chain_rt_product: bad arguments");
  const unsigned g = (unsigned)ceil_div(n, kC3Waves);
  hipStream_t st = as_stream(stream);
  const size_t lds = (size_t)(m + 1) * k * 4;
  if (m < 16)
    rt_product_kernel<16><<<g, kC3Waves * 64, lds, st>>>(P, m, K, k, n, out);
  else
    rt_product_kernel<kAugRows><<<g, kC3Waves * 64, lds, st>>>(P, m, K, k, n, out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_chain_outer(const float* R, int32_t ldr, int32_t m, const float* rlast,
                                  int32_t na, const float* P, int32_t nb, float* out,
                                  void* stream) {
  RS_CHECK_ARG(m >= 0 && na >= 1 && nb >= 4 && nb % 4 == 0 && ldr >= na && P && out &&
                   (m == 0 || R),
               "rs_chain_outer: bad arguments");
  RS_CHECK_ARG((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(out)) % 16 == 0,
               "rs_chain_outer: P and out must be 16-byte aligned");
  const int64_t tot = (int64_t)na * (nb / 4);
  outer_sum_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, as_stream(stream)>>>(
      R, ldr, m, rlast, na, P, nb, out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_dlrm_dense_tail_workspace_size(int32_t n0, int32_t n1, int32_t n2) {
  return (size_t)(2 * n1 + 2 * n2 + std::max(n0, n1 + 1)) * sizeof(float);
}

extern "C" int32_t rs_dlrm_dense_tail(const rs_dlrm_tail_args* t, void* workspace, size_t ws_bytes,
                                      void* stream) {
  RS_CHECK_ARG(t, "rs_dlrm_dense_tail: null args");
  const int n0 = t->top_n0, n1 = t->top_n1, n2 = t->top_n2, nf = t->top_n_full0;
  const int m = t->bot_n0, b1 = t->bot_n1, b2 = t->bot_n2, b3 = t->bot_n3;
  RS_CHECK_ARG(n0 >= 1 && n1 >= 1 && n2 >= 1 && nf >= n0 && (t->top_rows != nullptr) == (t->top_inv != nullptr) &&
                   (t->top_rows || nf == n0),
               "rs_dlrm_dense_tail: bad top chain sizes");
  RS_CHECK_ARG(m >= 1 && m < 16 && b1 >= 4 && b2 >= 4 && b3 >= 4 && b1 % 4 == 0 && b2 % 4 == 0 &&
                   b3 % 4 == 0 && (int64_t)(m + 1) * b1 <= kAugLds && (int64_t)(m + 1) * b2 <= kAugLds &&
                   (int64_t)(m + 1) * b3 <= kAugLds,
               "rs_dlrm_dense_tail: bad bottom chain sizes");
  for (int i = 0; i < 3; ++i)
    RS_CHECK_ARG(t->top_k[i] && t->top_b[i] && t->top_dk[i] && t->top_db[i] && t->bot_k[i] && t->bot_b[i],
                 "rs_dlrm_dense_tail: null parameter / gradient");
  RS_CHECK_ARG(t->top_A && t->top_s && t->top_q && t->top_c && t->bot_P && t->bot_comp2 && t->bot_dk2 &&
                   t->bot_dk3 && t->bot_P2 && t->bot_P1 && t->bot_comp2_next && t->bot_comp3_next,
               "rs_dlrm_dense_tail: null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_dlrm_dense_tail_workspace_size(n0, n1, n2), "workspace too small");
  const uintptr_t al = reinterpret_cast<uintptr_t>(t->bot_P2) |
                       reinterpret_cast<uintptr_t>(t->bot_dk2) | reinterpret_cast<uintptr_t>(t->bot_dk3);
  RS_CHECK_ARG(al % 16 == 0 && reinterpret_cast<uintptr_t>(t->bot_P) % 4 == 0,
               "rs_dlrm_dense_tail: bot_P2 / dk2 / dk3 must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  float* w = static_cast<float*>(workspace);
  // top chain gradients (rs_chain3_vec_grads' stages); p (the input gradient) is not needed
  Chain3Args top{t->top_k[0], t->top_rows, t->top_inv, t->top_b[0], t->top_k[1], t->top_b[1],
                 t->top_k[2], t->top_A, t->top_s, nf, n0, n1, n2, w, w + n1, w + 2 * n1,
                 w + 2 * n1 + n2, t->top_dk[0], t->top_db[0], t->top_dk[1], t->top_db[1],
                 t->top_dk[2], t->top_db[2], w + 2 * n1 + 2 * n2};
  // stage 2's p[i] rows (the top chain's input gradient) are a by-product the tail does not
  // keep: they land in scratch
  const int g1_top = (int)(ceil_div(n1, kC3Waves) + ceil_div(n1, 64) + ceil_div(n2, 64));
  const int g2_top = (int)(ceil_div(n0, kC3Waves) + ceil_div(n2, 64));
  // bottom: P = [A; s] [m+1, b3]; dK3 = R~2ᵀ·P; P2 = P·K3ᵀ [m+1, b2]; dK2 = [K1; b1]ᵀ·P2;
  // P1 = P2·K2ᵀ [m+1, b1] = [dK1; db1]; db2 = P2[m]; db3 = P[m]
  TailOuter o1{t->bot_comp2, b2, m, t->bot_comp2 + (size_t)m * b2, b2, t->bot_P, b3, t->bot_dk3};
  TailRt r1{t->bot_P, m, t->bot_k[2], b3, b2, t->bot_P2};
  TailOuter o2{t->bot_k[0], b1, m, t->bot_b[0], b1, t->bot_P2, b2, t->bot_dk2};
  TailRt r2{t->bot_P2, m, t->bot_k[1], b2, b1, t->bot_P1};
  const int nb_o1 = (int)ceil_div(o1.units(), 1024), nb_o2 = (int)ceil_div(o2.units(), 1024);
  const int nb_r1 = (int)ceil_div(b2, kC3Waves), nb_r2 = (int)ceil_div(b1, kC3Waves);
  tail_grads1<<<g1_top + nb_o1 + nb_r1, kC3Waves * 64, (size_t)(m + 1) * b3 * 4, st>>>(top, g1_top, o1, nb_o1, r1);
  RS_CHECK_LAUNCH();
  tail_grads2<<<g2_top + nb_o2 + nb_r2, kC3Waves * 64, (size_t)(m + 1) * b2 * 4, st>>>(top, g2_top, o2, nb_o2, r2);
  RS_CHECK_LAUNCH();
  const int64_t tot3 = (int64_t)nf * n1 + (int64_t)n1 * n2 + n2 + n1 + 1;
  tail_grads3<<<(unsigned)ceil_div(tot3, 1024), kC3Waves * 64, 0, st>>>(top);
  RS_CHECK_LAUNCH();
  // SGD, parameter order: top K1 b1 K2 b2 K3 b3, bottom K1 b1 K2 b2 K3 b3
  TailSgd sg{};
  const int64_t sz[kTailParams] = {(int64_t)nf * n1, n1, (int64_t)n1 * n2, n2, n2, 1,
                                   (int64_t)m * b1, b1, (int64_t)b1 * b2, b2, (int64_t)b2 * b3, b3};
  float* ps[kTailParams] = {t->top_k[0], t->top_b[0], t->top_k[1], t->top_b[1], t->top_k[2], t->top_b[2],
                            t->bot_k[0], t->bot_b[0], t->bot_k[1], t->bot_b[1], t->bot_k[2], t->bot_b[2]};
  const float* gs[kTailParams] = {t->top_dk[0], t->top_db[0], t->top_dk[1], t->top_db[1], t->top_dk[2],
                                  t->top_db[2], t->bot_P1, t->bot_P1 + (size_t)m * b1, t->bot_dk2,
                                  t->bot_P2 + (size_t)m * b2, t->bot_dk3, t->bot_P + (size_t)m * b3};
  sg.off[0] = 0;
  for (int i = 0; i < kTailParams; ++i) {
    sg.p[i] = ps[i];
    sg.g[i] = gs[i];
    sg.off[i + 1] = sg.off[i] + sz[i];
  }
  sg.lr = t->lr;
  tail_sgd<<<(unsigned)ceil_div(sg.off[kTailParams], 256), 256, 0, st>>>(sg);
  RS_CHECK_LAUNCH();
  // next step's compositions from the updated parameters
  TailAug a1{t->bot_k[0], b1, m, t->bot_b[0], t->bot_k[1], b1, b2, t->bot_b[1], t->bot_comp2_next};
  TailAug a2{t->bot_comp2_next, b2, m, t->bot_comp2_next + (size_t)m * b2, t->bot_k[2], b2, b3,
             t->bot_b[2], t->bot_comp3_next};
  VecComposeArgs v{t->top_k[0], t->top_rows, t->top_b[0], t->top_k[1], t->top_b[1], t->top_k[2],
                   t->top_b[2], n0, n1, n2, w, w + n1, t->top_q, t->top_c};
  const size_t lds1 = (size_t)std::max<int64_t>((int64_t)(m + 1) * b1, 8 * 16 * 64) * 4;
  const size_t lds2 = (size_t)std::max<int64_t>((int64_t)(m + 1) * b2, 8 * 16 * 64) * 4;
  const int nb_a1 = (int)ceil_div(b2, 64), nb_a2 = (int)ceil_div(b3, 64);
  tail_compose1<<<nb_a1 + (int)ceil_div(n1 + 1, kC3Waves), kC3Waves * 64, lds1, st>>>(a1, nb_a1, v);
  RS_CHECK_LAUNCH();
  tail_compose2<<<nb_a2 + (int)ceil_div(n0 + 1, kC3Waves), kC3Waves * 64, lds2, st>>>(a2, nb_a2, v);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
