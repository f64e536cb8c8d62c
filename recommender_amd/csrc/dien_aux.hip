// dien_aux.hip — DIEN auxiliary loss (a-9: InterestExtract.compute_auxiliary_loss,
// dien/layers.py:89-108, with AuxiliaryNet dien/layers.py:62-73) as two fused kernels.
//
// Per example b and history step t < L-1, with x = [h_t (H), e_{t+1} (E)] for the positive
// (e = pos_his) and negative (e = neg_his) next item:
//   z = σ(σ(x·W1 + b1)·W2 + b2)·W3 + b3          (Dense 80 σ → Dense 40 σ → Dense 1)
//   aux_b = Σ_t m[b,t+1]·(ce(z_pos, 1) + ce(z_neg, 0)) / (2·Σ_t m[b,t+1])
// ce = tf.nn.sigmoid_cross_entropy_with_logits. The reference evaluates the net on all B·(L-1)
// rows of both sets (two [2B(L-1), 72] GEMM chains + their backward). A row with m[b,t+1] = 0
// contributes exactly 0 to the loss and to every gradient (its factor is 0 and the net is
// finite), so these kernels evaluate only the 16-row tiles that hold a valid row — with
// post-padded histories that is ≈1/8 of the rows at L = 100 — and write the zero input
// gradients of the others. Same values, a fraction of the work, no [rows, 80] activations in
// HBM (the backward recomputes the forward of the tiles it visits).
//
// MFMA layout (v_mfma_f32_16x16x4_f32, exact f32): activations are kept TRANSPOSED — a 16-row
// tile is the N side, units the M side — so the C layout of one layer (lane = (row j, unit
// group kq), 4 consecutive units per lane) is directly the B operand of the next layer when the
// K axis is walked as (tile u, register r): no transposes between layers. Weights sit in LDS and
// are read as A operands with the matching permutation. The weight gradients (K = rows) need the
// row axis on lane>>4, so h1 / dz2 / dz1 go through a wave-private LDS tile for them.
// Determinism: the backward is a persistent grid with a static item → wave assignment; each wave
// accumulates its weight gradients in registers (MFMA C tiles), writes one partial row, and the
// partials are folded in a fixed order (fold_two_level).
#include <algorithm>

#include "common.hpp"

namespace rs {

int32_t fold_two_level(const float* part, int nchunks, int N, float* part2, float* out,
                       hipStream_t st);
int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* total, void* ws,
                           size_t ws_bytes, hipStream_t st);
size_t exclusive_scan_ws_size(int64_t n);

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kN1 = 80, kN2 = 40;  // AuxiliaryNet([80, 40, 1])
constexpr int kT1 = 5, kT2 = 3;    // 16-unit tiles of the two hidden layers (40 padded to 48)
constexpr int kMaxIn = 80, kMaxKS = kMaxIn / 4;
constexpr int kW1S = 81, kW2S = 49;  // LDS row strides: W1 [In][80], W2 [80][48] (bank spread)
constexpr int kS1 = 81, kS2 = 49;    // wave scratch strides: [16 rows][80] and [16 rows][48]
constexpr int kWaves = 4;
constexpr int kBwdBlocksPerCU = 1;

struct AuxArgs {
  const float* hidden;  // [B, L, H]
  const float* pos;     // [B, L, E]
  const float* neg;     // [B, L, E]
  const uint8_t* mask;  // [B, L]
  int64_t B;
  int L, H, E;
  const float *W1, *b1, *W2, *b2, *W3, *b3;  // [H+E, 80], [80], [80, 40], [40], [40], [1]
};

struct AuxLds {
  float w1[kMaxIn * kW1S];
  float w2[kN1 * kW2S];
  float b1[kN1], b2[48], w3[48];
};

// σ with the hardware exp2 / reciprocal (≈1-2 ulp; the parity tests bound the net at 1e-5)
__device__ __forceinline__ float aux_sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ void stage_weights(const AuxArgs& a, AuxLds& s) {
  const int In = a.H + a.E;
  for (int i = threadIdx.x; i < kMaxIn * kN1; i += blockDim.x) {
    const int f = i / kN1, u = i % kN1;
    s.w1[f * kW1S + u] = f < In ? a.W1[f * kN1 + u] : 0.f;
  }
  for (int i = threadIdx.x; i < kN1 * 48; i += blockDim.x) {
    const int u = i / 48, v = i % 48;
    s.w2[u * kW2S + v] = v < kN2 ? a.W2[u * kN2 + v] : 0.f;
  }
  for (int i = threadIdx.x; i < kN1; i += blockDim.x) s.b1[i] = a.b1[i];
  for (int i = threadIdx.x; i < 48; i += blockDim.x) {
    s.b2[i] = i < kN2 ? a.b2[i] : 0.f;
    s.w3[i] = i < kN2 ? a.W3[i] : 0.f;
  }
}

// Number of valid aux rows of example b: Σ_{t=1}^{L-1} mask[b, t] (wave-uniform).
__device__ __forceinline__ int aux_count(const AuxArgs& a, int64_t b, int lane) {
  int c = 0;
  for (int t = 1 + lane; t < a.L; t += 64) c += a.mask[b * a.L + t] != 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  return c;
}

// B operands of layer 1 for the tile's row j = lane & 15 (history step t): feature 4s + kq of
// x = [h_t, e_{t+1}]; zero for rows past L-2 and for padding features. load_x_raw issues the
// loads unguarded (a row past L-2 reads step 0's, always in bounds) and zero_x applies the row
// mask where the values are used: guarded per element, the compiler waited for each load in turn
// (round 6, gfx950 ISA), and the backward's one-round-ahead fetch was drained at once.
template <int H, int E>
__device__ __forceinline__ void load_x_raw(const AuxArgs& a, const float* e, int64_t b, int t,
                                           int kq, float (&xv)[(H + E) / 4]) {
  const bool ok = t <= a.L - 2;
  const float* hr = a.hidden + (b * a.L + (ok ? t : 0)) * (int64_t)H + kq;
  const float* er = e + (b * a.L + (ok ? t + 1 : 0)) * (int64_t)E + kq;
#pragma unroll
  for (int s = 0; s < H / 4; ++s) xv[s] = hr[4 * s];
#pragma unroll
  for (int s = 0; s < E / 4; ++s) xv[H / 4 + s] = er[4 * s];
}
template <int H, int E>
__device__ __forceinline__ void zero_x(const AuxArgs& a, int t, float (&xv)[(H + E) / 4]) {
  const bool ok = t <= a.L - 2;
#pragma unroll
  for (int s = 0; s < (H + E) / 4; ++s) xv[s] = ok ? xv[s] : 0.f;
}
template <int H, int E>
__device__ __forceinline__ void load_x(const AuxArgs& a, const float* e, int64_t b, int t,
                                       int kq, float (&xv)[(H + E) / 4]) {
  load_x_raw<H, E>(a, e, b, t, kq, xv);
  zero_x<H, E>(a, t, xv);
}

// Forward of one 16-row set: h1 (C layout, 5 tiles), h2 (3 tiles) and the logit of row j
// (identical in the four kq lanes of the row).
template <int H, int E>
__device__ __forceinline__ float aux_forward(const AuxArgs& a, const AuxLds& s,
                                             const float (&xv)[(H + E) / 4], int j, int kq,
                                             f4 (&h1)[kT1], f4 (&h2)[kT2]) {
#pragma unroll
  for (int u = 0; u < kT1; ++u) h1[u] = f4{0.f, 0.f, 0.f, 0.f};
  const float* w1 = s.w1 + kq * kW1S + j;
#pragma unroll
  for (int k = 0; k < (H + E) / 4; ++k) {
    const float* w = w1 + 4 * k * kW1S;  // A: W1[4k + kq][16u + j]
#pragma unroll
    for (int u = 0; u < kT1; ++u) h1[u] = mfma4(w[16 * u], xv[k], h1[u]);
  }
#pragma unroll
  for (int u = 0; u < kT1; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) h1[u][r] = aux_sigm(h1[u][r] + s.b1[16 * u + 4 * kq + r]);
#pragma unroll
  for (int m = 0; m < kT2; ++m) h2[m] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < kT1; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* w = s.w2 + (16 * u + 4 * kq + r) * kW2S + j;  // A: W2[16u+4kq+r][16m + j]
#pragma unroll
      for (int m = 0; m < kT2; ++m) h2[m] = mfma4(w[16 * m], h1[u][r], h2[m]);
    }
  float p = 0.f;
#pragma unroll
  for (int m = 0; m < kT2; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = 16 * m + 4 * kq + r;
      h2[m][r] = aux_sigm(h2[m][r] + s.b2[v]);
      p = fmaf(h2[m][r], s.w3[v], p);
    }
  p += __shfl_xor(p, 16);
  p += __shfl_xor(p, 32);
  return p + a.b3[0];
}

// tf.nn.sigmoid_cross_entropy_with_logits(labels = y, logits = z)
__device__ __forceinline__ float sig_ce(float z, float y) {
  return fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z)));
}

// ---------------------------------------------------------------------------------------
// forward: persistent blocks (the 42 KB of weights staged once per block, not once per two
// examples: staging was most of the kernel's time); each round the block's waves are 2 examples
// × {pos, neg}, summed in LDS; aux[b] as dien/layers.py:105-108
// ---------------------------------------------------------------------------------------
template <int H, int E>
__global__ __launch_bounds__(256) void aux_fwd_kernel(AuxArgs a, float* __restrict__ aux) {
  __shared__ AuxLds s;
  __shared__ float sums[kWaves];
  stage_weights(a, s);
  __syncthreads();
  const int lane = threadIdx.x & 63, j = lane & 15, kq = lane >> 4, wave = threadIdx.x >> 6;
  const int set = wave & 1;
  const int NT = (a.L - 1 + 15) / 16;
  const float* e = set == 0 ? a.pos : a.neg;
  const int64_t n_rounds = (a.B + kWaves / 2 - 1) / (kWaves / 2);
  for (int64_t rd = blockIdx.x; rd < n_rounds; rd += gridDim.x) {
    const int64_t b = rd * (kWaves / 2) + (wave >> 1);
    float total = 0.f;
    int cnt = 1;
    if (b < a.B) {
      cnt = aux_count(a, b, lane);
      for (int tile = 0; tile < NT; ++tile) {
        const int t = 16 * tile + j;
        const bool m = t <= a.L - 2 && a.mask[b * a.L + t + 1] != 0;
        if (__ballot(m) == 0) continue;  // no valid row: the tile adds exactly 0
        float xv[(H + E) / 4];
        load_x<H, E>(a, e, b, t, kq, xv);
        f4 h1[kT1], h2[kT2];
        const float z = aux_forward<H, E>(a, s, xv, j, kq, h1, h2);
        float tl = m ? sig_ce(z, set == 0 ? 1.f : 0.f) : 0.f;
        // row sum of the tile (rows j of each kq lane group, fixed butterfly order)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) tl += __shfl_xor(tl, off);
        total += tl;
      }
    }
    if (lane == 0) sums[wave] = total;
    __syncthreads();
    if (b < a.B && set == 0 && lane == 0)
      aux[b] = (sums[wave] + sums[wave + 1]) / ((float)cnt * 2.f);
    __syncthreads();  // sums is rewritten next round
  }
}

// ---------------------------------------------------------------------------------------
// backward: persistent blocks over pairs of items (tile, b). In a round the block's four waves
// each take one set (item i or i+1, pos or neg): recompute the forward, G = dL/dz, dz2, dz1 and
// the input gradients (MFMA, C layout, no weight gradients). They publish h1 / dz1 / dz2 / h2 /
// d3 of their 16 rows in LDS; then every wave accumulates ITS share of the weight-gradient
// tiles (K = rows) over the round's four sets. Static item → block assignment and a fixed
// accumulation order make the per-block partials, and their fold, deterministic.
// ---------------------------------------------------------------------------------------
struct AuxGrad {
  const float* daux;       // [B]
  float* dhidden;          // [B, L, H]
  float* dpos;             // [B, L, E]
  float* dneg;             // [B, L, E]
  float* part;             // [n_blocks, n_param]
  const int32_t* items;    // live items (tile-major index tile·B + b), in order
  const int32_t* n_items;  // [1] their count
  const int32_t* cnt;      // [B] Σ_t m[b, t+1]
  int acc_hidden;          // 1: dhidden += this loss's part (the caller's upstream gradient kept)
};

// live items: tile·B + b holds a valid row, or example b has none (0/0: NaN, as the reference)
__global__ __launch_bounds__(256) void aux_live_kernel(AuxArgs a, int NT, int32_t* __restrict__ flag,
                                                       int32_t* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (b >= a.B) return;
  const int c = aux_count(a, b, lane);
  if (lane == 0) cnt[b] = c;
  for (int tile = 0; tile < NT; ++tile) {
    const int t = 16 * tile + (lane & 15);
    const bool m = t <= a.L - 2 && a.mask[b * a.L + t + 1] != 0;
    const bool live = c == 0 || __ballot(m) != 0;
    if (lane == 0) flag[(int64_t)tile * a.B + b] = live ? 1 : 0;
  }
}

__global__ void aux_compact_kernel(const int32_t* __restrict__ flag, const int32_t* __restrict__ pos,
                                   int64_t n, int32_t* __restrict__ items) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    if (flag[i]) items[pos[i]] = (int32_t)i;
}

__host__ __device__ inline int aux_n_param(int In) {
  return In * kN1 + kN1 + kN1 * kN2 + kN2 + kN2 + 1;
}

constexpr int kSets = 4;        // sets per round: items (2) × {pos, neg}
constexpr int kTilesW1 = 25;    // dW1 (+ db1 as the ones feature): 5 feature × 5 unit tiles
constexpr int kTilesW2 = 15;    // dW2: 5 × 3 tiles
constexpr int kTilesPerWave = (kTilesW1 + kTilesW2) / kWaves;  // 10
constexpr int kMaxH = 76;

struct SetTile {
  float x[16 * kS1];  // [row][feature]: x = [h, e], 1 at feature In (db1), 0 after
  float h1[16 * kS1];
  float dz1[16 * kS1];
  float dz2[16 * kS2];
  float h2[16 * kS2];
  float d3[16];
};

struct BwdLds {
  AuxLds w;
  SetTile st[kSets];
  float dxh[2][16 * kMaxH];  // the neg set's h-part input gradient, per item of the round
  int live[kSets];           // the set was computed this round
};

__device__ __forceinline__ void store4(float* p, f4 v) {  // 16-byte aligned global rows
  *reinterpret_cast<f4*>(p) = v;
}
__device__ __forceinline__ void lds4(float* p, f4 v) {  // odd-stride LDS tile: 4 dword writes
  p[0] = v[0];
  p[1] = v[1];
  p[2] = v[2];
  p[3] = v[3];
}

template <int H, int E>
__global__ __launch_bounds__(256) void aux_bwd_kernel(AuxArgs a, AuxGrad g) {
  extern __shared__ float dyn[];
  BwdLds& S = *reinterpret_cast<BwdLds*>(dyn);
  stage_weights(a, S.w);
  const int lane = threadIdx.x & 63, j = lane & 15, kq = lane >> 4, wave = threadIdx.x >> 6;
  constexpr int In = H + E;
  const int L = a.L;
  const int io = wave >> 1, set = wave & 1;  // this wave's item of the pair, pos / neg
  SetTile& T = S.st[wave];

  f4 acc[kTilesPerWave];
#pragma unroll
  for (int q = 0; q < kTilesPerWave; ++q) acc[q] = f4{0.f, 0.f, 0.f, 0.f};
  float vacc = 0.f;  // thread q < 81: dW3[q] (q < 40), db2[q-40] (q < 80), db3 (q = 80)
  __syncthreads();

  const int64_t n_live = *g.n_items;
  const int64_t n_pairs_live = (n_live + 1) / 2;
  const float* e = set == 0 ? a.pos : a.neg;
  float* de = set == 0 ? g.dpos : g.dneg;
  // Round 6: a round's global inputs are loaded one round ahead (at one wave per SIMD nothing
  // else hides their latency): the item of the round after next (stage A), and for the next
  // round its example's count, mask bit, upstream daux, the 16 rows' x = [h, e] and — for the
  // pos waves — the dL/dh rows the h part is added to (stage B). Same values, same arithmetic.
  struct RoundIn {
    int64_t b;
    int t;
    bool live, m;
    float sb;
    int cnt;
    uint8_t mraw;
    float daux;
    float xv[In / 4];
    f4 dh[kT1];
  };
  auto item_of = [&](int64_t p, bool& lv) -> int64_t {
    const int64_t li = 2 * p + io;
    lv = p < n_pairs_live && li < n_live;
    const int32_t v = g.items[lv ? li : 0];  // unguarded (items holds >= 1 entry)
    return lv ? v : 0;
  };
  // fetch issues every load unguarded from an in-bounds address (an item that is not live reads
  // item 0's); finish applies the masks and the arithmetic when the round starts, so the loads
  // stay in flight under the current round
  auto fetch = [&](int64_t it, bool lv, RoundIn& r) {
    r.live = lv;
    r.b = it % a.B;
    r.t = 16 * (int)(it / a.B) + j;
    const int tc = r.t <= L - 2 ? r.t : 0;
    r.cnt = g.cnt[r.b];
    r.mraw = a.mask[r.b * L + tc + 1];
    r.daux = g.daux[r.b];
    load_x_raw<H, E>(a, e, r.b, r.t, kq, r.xv);
    const int tt = r.t < L ? r.t : 0;
#pragma unroll
    for (int x = 0; x < kT1; ++x) {
      const int f0 = 16 * x + 4 * kq;
      r.dh[x] = *reinterpret_cast<const f4*>(g.dhidden + (r.b * L + tt) * (int64_t)H +
                                             (f0 < H ? f0 : 0));
    }
  };
  auto finish = [&](RoundIn& r) {
    r.m = r.live && r.t <= L - 2 && r.mraw != 0;
    // dL/d(loss sum of b) = daux_b / (2·cnt)  (0 rows → inf·0 = NaN, as the reference)
    r.sb = r.daux / ((float)r.cnt * 2.f);
    zero_x<H, E>(a, r.t, r.xv);
    const bool dh_ok = set == 0 && g.acc_hidden && r.live && r.t < L;
#pragma unroll
    for (int x = 0; x < kT1; ++x)
      if (!(dh_ok && 16 * x + 4 * kq < H)) r.dh[x] = f4{0.f, 0.f, 0.f, 0.f};
  };
  RoundIn cur;
  {
    bool lv0;
    const int64_t it0 = item_of(blockIdx.x, lv0);
    fetch(it0, lv0, cur);
  }
  bool lv1;
  int64_t it1 = item_of((int64_t)blockIdx.x + gridDim.x, lv1);
  for (int64_t pr = blockIdx.x; pr < n_pairs_live; pr += gridDim.x) {
    RoundIn nxt;
    fetch(it1, lv1, nxt);  // stage B of the next round
    bool lv2;
    const int64_t it2 = item_of(pr + 2 * (int64_t)gridDim.x, lv2);  // stage A of the one after
    finish(cur);
    const bool live = cur.live;
    const int64_t b = cur.b;
    const int t = cur.t;
    const bool m = cur.m;
    f4 dxh[kT1];
    if (live) {
      const float sb = cur.sb;
      const float (&xv)[In / 4] = cur.xv;
#pragma unroll
      for (int k = 0; k < In / 4; ++k) T.x[j * kS1 + 4 * k + kq] = xv[k];
      for (int f = In + kq; f < kMaxIn; f += 4) T.x[j * kS1 + f] = f == In ? 1.f : 0.f;
      f4 h1[kT1], h2[kT2];
      const float z = aux_forward<H, E>(a, S.w, xv, j, kq, h1, h2);
      const float d3 = (sb * (m ? 1.f : 0.f)) * (aux_sigm(z) - (set == 0 ? 1.f : 0.f));
      f4 dz2[kT2];
#pragma unroll
      for (int mm = 0; mm < kT2; ++mm)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = 16 * mm + 4 * kq + r;
          dz2[mm][r] = d3 * S.w.w3[v] * (h2[mm][r] * (1.f - h2[mm][r]));
        }
#pragma unroll
      for (int mm = 0; mm < kT2; ++mm) {
        lds4(T.dz2 + j * kS2 + 16 * mm + 4 * kq, dz2[mm]);
        lds4(T.h2 + j * kS2 + 16 * mm + 4 * kq, h2[mm]);
      }
      if (kq == 0) T.d3[j] = d3;
      // dh1ᵀ = W2 · dz2ᵀ, then dz1 = dh1 ⊙ h1(1 − h1)
      f4 dz1[kT1];
#pragma unroll
      for (int u = 0; u < kT1; ++u) {
        f4 c = f4{0.f, 0.f, 0.f, 0.f};
        const float* w = S.w.w2 + (16 * u + j) * kW2S + 4 * kq;  // A: W2[16u + j][16m + 4kq + r]
#pragma unroll
        for (int mm = 0; mm < kT2; ++mm)
#pragma unroll
          for (int r = 0; r < 4; ++r) c = mfma4(w[16 * mm + r], dz2[mm][r], c);
#pragma unroll
        for (int r = 0; r < 4; ++r) dz1[u][r] = c[r] * (h1[u][r] * (1.f - h1[u][r]));
        lds4(T.h1 + j * kS1 + 16 * u + 4 * kq, h1[u]);
        lds4(T.dz1 + j * kS1 + 16 * u + 4 * kq, dz1[u]);
      }
      // dXᵀ = W1 · dz1ᵀ: e part stored for this set; h part kept (summed with the other set)
#pragma unroll
      for (int x = 0; x < kT1; ++x) {
        dxh[x] = f4{0.f, 0.f, 0.f, 0.f};
        if (16 * x >= In) continue;
        f4 c = f4{0.f, 0.f, 0.f, 0.f};
        const float* w = S.w.w1 + (16 * x + j) * kW1S + 4 * kq;  // A: W1[16x + j][16u + 4kq + r]
#pragma unroll
        for (int u = 0; u < kT1; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) c = mfma4(w[16 * u + r], dz1[u][r], c);
        const int f0 = 16 * x + 4 * kq;
        if (f0 < H) {
          dxh[x] = c;
          if (set == 1) lds4(S.dxh[io] + j * kMaxH + f0, c);
        } else if (f0 < In && t <= L - 2) {
          store4(de + (b * L + t + 1) * (int64_t)E + (f0 - H), c);
        }
      }
    }
    if (lane == 0) S.live[wave] = live ? 1 : 0;
    __syncthreads();
    if (live && set == 0 && t < L) {  // h part: pos set + neg set of the same item
#pragma unroll
      for (int x = 0; x < kT1; ++x) {
        const int f0 = 16 * x + 4 * kq;
        if (f0 < H) {
          const float* o = S.dxh[io] + j * kMaxH + f0;
          float* dst = g.dhidden + (b * L + t) * (int64_t)H + f0;
          const f4 v = dxh[x] + f4{o[0], o[1], o[2], o[3]};
          store4(dst, g.acc_hidden ? cur.dh[x] + v : v);  // dh: the upstream rows, prefetched
        }
      }
    }
    // this wave's weight-gradient tiles over the round's live sets (K = rows)
#pragma unroll
    for (int q = 0; q < kTilesPerWave; ++q) {
      const int tq = wave * kTilesPerWave + q;
#pragma unroll 1
      for (int sidx = 0; sidx < kSets; ++sidx) {
        if (!S.live[sidx]) continue;
        const SetTile& U = S.st[sidx];
        if (tq < kTilesW1) {  // dW1[16x + i][16u + n] += Σ_rows xaug[row][16x + i]·dz1[row][16u + n]
          const int x = tq / kT1, u = tq % kT1;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int row = 4 * k + kq;
            acc[q] = mfma4(U.x[row * kS1 + 16 * x + j], U.dz1[row * kS1 + 16 * u + j], acc[q]);
          }
        } else {  // dW2[16u + i][16m + n] += Σ_rows h1[row][16u + i]·dz2[row][16m + n]
          const int t2 = tq - kTilesW1;
          const int u = t2 / kT2, mm = t2 % kT2;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int row = 4 * k + kq;
            acc[q] = mfma4(U.h1[row * kS1 + 16 * u + j], U.dz2[row * kS2 + 16 * mm + j], acc[q]);
          }
        }
      }
    }
    {  // dW3 / db2 / db3 on the vector unit: one output per thread
      const int q = threadIdx.x;
      if (q <= 2 * kN2) {
        for (int sidx = 0; sidx < kSets; ++sidx) {
          if (!S.live[sidx]) continue;
          const SetTile& U = S.st[sidx];
          float va[16], vb[16];
#pragma unroll
          for (int row = 0; row < 16; ++row) {  // all 32 reads in flight, then the chain
            va[row] = q < kN2 ? U.h2[row * kS2 + q] : q < 2 * kN2 ? U.dz2[row * kS2 + (q - kN2)] : 1.f;
            vb[row] = q < kN2 || q == 2 * kN2 ? U.d3[row] : 1.f;
          }
#pragma unroll
          for (int row = 0; row < 16; ++row) vacc = fmaf(va[row], vb[row], vacc);
        }
      }
    }
    __syncthreads();  // the set tiles are rewritten next round
    cur = nxt;
    it1 = it2;
    lv1 = lv2;
  }

  // this block's partial gradients: [dW1 In×80 | db1 80 | dW2 80×40 | db2 40 | dW3 40 | db3 1]
  float* out = g.part + (int64_t)blockIdx.x * aux_n_param(In);
  float* o_b1 = out + In * kN1;
  float* o_w2 = o_b1 + kN1;
  float* o_b2 = o_w2 + kN1 * kN2;
  float* o_w3 = o_b2 + kN2;
#pragma unroll
  for (int q = 0; q < kTilesPerWave; ++q) {
    const int tq = wave * kTilesPerWave + q;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (tq < kTilesW1) {
        const int x = tq / kT1, u = tq % kT1;
        const int f = 16 * x + 4 * kq + r, un = 16 * u + j;
        if (f < In) out[f * kN1 + un] = acc[q][r];
        else if (f == In) o_b1[un] = acc[q][r];
      } else {
        const int t2 = tq - kTilesW1;
        const int u = t2 / kT2, mm = t2 % kT2;
        const int un = 16 * u + 4 * kq + r, v = 16 * mm + j;
        if (v < kN2) o_w2[un * kN2 + v] = acc[q][r];
      }
    }
  }
  const int q = threadIdx.x;
  if (q < kN2) o_w3[q] = vacc;
  else if (q < 2 * kN2) o_b2[q - kN2] = vacc;
  else if (q == 2 * kN2) o_w3[kN2] = vacc;  // db3 follows dW3
}

size_t bwd_lds_bytes() { return sizeof(BwdLds); }

int bwd_blocks(int dev_cus) { return dev_cus * kBwdBlocksPerCU; }

int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

int32_t check_aux(const AuxArgs& a) {
  RS_CHECK_ARG(a.B >= 0 && a.L >= 2 && a.L <= 4096, "bad sizes (L >= 2)");
  RS_CHECK_ARG(a.H > 0 && a.E > 0 && a.H % 4 == 0 && a.E % 4 == 0 && a.H + a.E < kMaxIn,
               "hidden / embedding widths must be multiples of 4 with H + E <= 76");
  RS_CHECK_ARG(a.hidden && a.pos && a.neg && a.mask && a.W1 && a.b1 && a.W2 && a.b2 && a.W3 &&
                   a.b3,
               "null pointer");
  return RS_OK;
}

}  // namespace
}  // namespace rs

using namespace rs;

namespace rs {
namespace {
struct AuxWs {  // workspace carve: partials | fold scratch | flags | positions | items | cnt | n | scan
  size_t part, part2, flag, pos, items, cnt, n, scan, total;
};
AuxWs aux_ws_layout(int64_t B, int32_t L, int32_t H, int32_t E) {
  const size_t np = (size_t)aux_n_param(H + E);
  const int64_t ni = (int64_t)((L + 15) / 16) * B;
  AuxWs w;
  w.part = 0;
  w.part2 = align_up(w.part + (size_t)bwd_blocks(device_cus()) * np * 4, 256);
  w.flag = align_up(w.part2 + 32 * np * 4, 256);
  w.pos = align_up(w.flag + (size_t)ni * 4, 256);
  w.items = align_up(w.pos + (size_t)ni * 4, 256);
  w.cnt = align_up(w.items + (size_t)ni * 4, 256);
  w.n = align_up(w.cnt + (size_t)B * 4, 256);
  w.scan = align_up(w.n + 4, 256);
  w.total = w.scan + exclusive_scan_ws_size(ni);
  return w;
}
}  // namespace
}  // namespace rs

extern "C" size_t rs_dien_aux_workspace_size(int64_t B, int32_t L, int32_t H, int32_t E) {
  return aux_ws_layout(B, L, H, E).total;
}

extern "C" int32_t rs_dien_aux_fwd(const float* hidden, const float* pos, const float* neg,
                                   const uint8_t* mask, int64_t B, int32_t L, int32_t H, int32_t E,
                                   const float* W1, const float* b1, const float* W2,
                                   const float* b2, const float* W3, const float* b3, float* aux,
                                   void* stream) {
  AuxArgs a{hidden, pos, neg, mask, B, L, H, E, W1, b1, W2, b2, W3, b3};
  if (int32_t e = check_aux(a)) return e;
  RS_CHECK_ARG(aux, "null pointer");
  if (B == 0) return RS_OK;
  // 3 resident blocks per CU (42 KB of LDS each), persistent over the example pairs
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(B, kWaves / 2), 3 * device_cus());
  hipStream_t st = as_stream(stream);
  if (H == 36 && E == 36) aux_fwd_kernel<36, 36><<<grid, 64 * kWaves, 0, st>>>(a, aux);
  else if (H == 16 && E == 16) aux_fwd_kernel<16, 16><<<grid, 64 * kWaves, 0, st>>>(a, aux);
  else { set_error("dien aux: (H, E) = (%d, %d) not built (36/36, 16/16)", H, E); return RS_E_UNSUPPORTED; }
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_dien_aux_bwd_acc(const float* hidden, const float* pos, const float* neg,
                                       const uint8_t* mask, int64_t B, int32_t L, int32_t H,
                                       int32_t E, const float* W1, const float* b1, const float* W2,
                                       const float* b2, const float* W3, const float* b3,
                                       const float* daux, float* dhidden, int32_t acc_hidden,
                                       float* dpos, float* dneg, float* dparams, void* workspace,
                                       size_t ws_bytes, void* stream);

extern "C" int32_t rs_dien_aux_bwd(const float* hidden, const float* pos, const float* neg,
                                   const uint8_t* mask, int64_t B, int32_t L, int32_t H, int32_t E,
                                   const float* W1, const float* b1, const float* W2,
                                   const float* b2, const float* W3, const float* b3,
                                   const float* daux, float* dhidden, float* dpos, float* dneg,
                                   float* dparams, void* workspace, size_t ws_bytes,
                                   void* stream) {
  return rs_dien_aux_bwd_acc(hidden, pos, neg, mask, B, L, H, E, W1, b1, W2, b2, W3, b3, daux,
                             dhidden, 0, dpos, dneg, dparams, workspace, ws_bytes, stream);
}

// acc_hidden = 1: dhidden holds the upstream gradient of the hidden states (attention + AUGRU)
// and this loss's part is added to it in place (rows of tiles without a valid step untouched):
// no zero fill and no separate add pass
extern "C" int32_t rs_dien_aux_bwd_acc(const float* hidden, const float* pos, const float* neg,
                                       const uint8_t* mask, int64_t B, int32_t L, int32_t H,
                                       int32_t E, const float* W1, const float* b1, const float* W2,
                                       const float* b2, const float* W3, const float* b3,
                                       const float* daux, float* dhidden, int32_t acc_hidden,
                                       float* dpos, float* dneg, float* dparams, void* workspace,
                                       size_t ws_bytes, void* stream) {
  AuxArgs a{hidden, pos, neg, mask, B, L, H, E, W1, b1, W2, b2, W3, b3};
  if (int32_t e = check_aux(a)) return e;
  RS_CHECK_ARG(daux && dhidden && dpos && dneg && dparams && workspace, "null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_dien_aux_workspace_size(B, L, H, E), "workspace too small");
  hipStream_t st = as_stream(stream);
  const int np = aux_n_param(H + E);
  if (B == 0) {
    RS_CHECK_HIP(hipMemsetAsync(dparams, 0, (size_t)np * 4, st));
    return RS_OK;
  }
  const int nb = bwd_blocks(device_cus());
  const AuxWs wl = aux_ws_layout(B, L, H, E);
  char* wsb = static_cast<char*>(workspace);
  float* part = reinterpret_cast<float*>(wsb + wl.part);
  float* part2 = reinterpret_cast<float*>(wsb + wl.part2);
  int32_t* flag = reinterpret_cast<int32_t*>(wsb + wl.flag);
  int32_t* ipos = reinterpret_cast<int32_t*>(wsb + wl.pos);
  int32_t* items = reinterpret_cast<int32_t*>(wsb + wl.items);
  int32_t* cnt = reinterpret_cast<int32_t*>(wsb + wl.cnt);
  int32_t* n_live = reinterpret_cast<int32_t*>(wsb + wl.n);
  const int NT = (L + 15) / 16;  // tiles over every hidden row t < L
  const int64_t ni = (int64_t)NT * B;
  RS_CHECK_ARG(ni < (1LL << 31), "too many (tile, example) items");
  aux_live_kernel<<<(unsigned)ceil_div(B, kWaves), 64 * kWaves, 0, st>>>(a, NT, flag, cnt);
  RS_CHECK_LAUNCH();
  if (int32_t e = exclusive_scan_i32(flag, ipos, ni, n_live, wsb + wl.scan,
                                     exclusive_scan_ws_size(ni), st))
    return e;
  aux_compact_kernel<<<(unsigned)std::min<int64_t>(ceil_div(ni, 256), 4096), 256, 0, st>>>(
      flag, ipos, ni, items);
  RS_CHECK_LAUNCH();
  const size_t lds = bwd_lds_bytes();
  // input gradients start at 0: the kernel writes only the rows of tiles that hold a valid row
  if (!acc_hidden) RS_CHECK_HIP(hipMemsetAsync(dhidden, 0, (size_t)B * L * H * 4, st));
  RS_CHECK_HIP(hipMemsetAsync(dpos, 0, (size_t)B * L * E * 4, st));
  RS_CHECK_HIP(hipMemsetAsync(dneg, 0, (size_t)B * L * E * 4, st));
  AuxGrad g{daux, dhidden, dpos, dneg, part, items, n_live, cnt, acc_hidden ? 1 : 0};
  auto run = [&](auto kern) -> int32_t {
    RS_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    kern<<<(unsigned)nb, 64 * kWaves, lds, st>>>(a, g);
    RS_CHECK_LAUNCH();
    return RS_OK;
  };
  int32_t rc;
  if (H == 36 && E == 36) rc = run(aux_bwd_kernel<36, 36>);
  else if (H == 16 && E == 16) rc = run(aux_bwd_kernel<16, 16>);
  else { set_error("dien aux: (H, E) = (%d, %d) not built (36/36, 16/16)", H, E); return RS_E_UNSUPPORTED; }
  if (rc) return rc;
  return fold_two_level(part, nb, np, part2, dparams, st);
}
