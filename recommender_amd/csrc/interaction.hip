// interaction.hip — DLRM DotInteraction (a-4, ctr/layers.py:17-43) and the DeepFM
// second-order FM term (a-5, ctr/model.py:21-23).
//
// Fast path (F <= 32, D % 16 == 0 fwd / D % 32 == 0 bwd): one wave per sample on the exact-fp32
// MFMA (gfx950 has no xf32; v_mfma_f32_*_f32 is an fma chain at the f32 vector rate).
//   fwd  Z = X·Xᵀ as three 16x16 blocks (0,0), (0,1), (1,1) of v_mfma_f32_16x16x4_f32 — the
//        (1,0) block is the mirror and is never computed. The K (= D) axis is permuted so that
//        lane group g = lane>>4 reads 16 contiguous bytes per row per instruction straight from
//        the table into VGPRs (no LDS staging of X); the same register is both the A and the B
//        operand of the diagonal blocks.
//   bwd  dX = S·X with S = M + Mᵀ (M = dZ on the kept pairs) on v_mfma_f32_32x32x2_f32, D
//        permuted so that every lane loads / stores NTILE = D/32 contiguous floats: a
//        half-wave moves one whole row per instruction, so the re-gather of X and the
//        grad-row stores are fully coalesced.
// DLRM variant (rs_dlrm_interaction_*): X rows come straight from the embedding table by id
// (fused gather), row F-1 is the bottom-MLP output, and the output row is the top-MLP input
// [Z (F*F, skip_gather), dense (D)] (ctr/model.py:51-55), so the [B,S,D] embedding tensor
// is never materialised in HBM; the backward re-gathers the rows instead of re-reading a
// saved copy (one 512-B read instead of a write + a read per row).
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

#include "common.hpp"

namespace rs {

// fixed two-level fold of nchunks partial rows [N] into out[N] (csrc/dense.hip); part2 holds
// 32 x N floats of scratch
int32_t fold_two_level(const float* part, int nchunks, int N, float* part2, float* out,
                       hipStream_t st);

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

struct InterMode {
  int self_interaction;
  int skip_gather;
};

__device__ __forceinline__ bool keep_pair(int i, int j, int self_i) {
  return self_i ? (i >= j) : (i < j);
}
// compact output index of kept pair (i,j) (row-major boolean_mask order, ctr/layers.py:39-42)
__device__ __forceinline__ int compact_index(int i, int j, int F, int self_i) {
  return self_i ? (i * (i + 1) / 2 + j) : (i * F - i * (i + 1) / 2 + (j - i - 1));
}
__host__ __device__ inline int out_width(int F, int self_i, int skip_gather) {
  return skip_gather ? F * F : (self_i ? F * (F + 1) / 2 : F * (F - 1) / 2);
}

// X row source: embedding rows by id (DLRM) or a dense [B, F, D] tensor
struct GatherSrc {
  const float* table;
  int64_t n_rows;
  const void* ids;
  int32_t id_dtype;
  int32_t n_slots;
  const int64_t* slot_offsets;
  const float* dense;  // [B, D], row F-1
  int32_t* err_flag;
  // pointer to X[b][i] (nullptr = zero row)
  __device__ __forceinline__ const float* row(int64_t b, int i, int D, bool& oob) const {
    if (i < n_slots) {
      int64_t r = global_row(ids, id_dtype, b * n_slots + i, slot_offsets, n_slots, n_rows);
      if (r < 0) {
        oob = true;
        return nullptr;
      }
      return table + r * D;
    }
    if (i == n_slots) return dense + b * D;
    return nullptr;
  }
};
struct DenseSrc {
  const float* x;
  int F;
  __device__ __forceinline__ const float* row(int64_t b, int i, int D, bool&) const {
    return i < F ? x + (b * F + i) * (int64_t)D : nullptr;
  }
};

// invert compact_index for the non-self (i < j) layout: row i starts at i*F - i(i+1)/2
__device__ __forceinline__ void compact_pair(int o, int F, int self_i, int& i, int& j) {
  if (self_i) {  // o = i(i+1)/2 + j, j <= i
    int ii = (int)((sqrtf(8.f * o + 1.f) - 1.f) * 0.5f);
    while (ii * (ii + 1) / 2 > o) --ii;
    while ((ii + 1) * (ii + 2) / 2 <= o) ++ii;
    i = ii;
    j = o - ii * (ii + 1) / 2;
  } else {
    const float b = 2.f * F - 1.f;
    int ii = (int)((b - sqrtf(b * b - 8.f * o)) * 0.5f);
    if (ii < 0) ii = 0;
    while (ii > 0 && ii * F - ii * (ii + 1) / 2 > o) --ii;
    while ((ii + 1) * F - (ii + 1) * (ii + 2) / 2 <= o) ++ii;
    i = ii;
    j = o - (ii * F - ii * (ii + 1) / 2) + ii + 1;
  }
}

__device__ __forceinline__ const float* shfl_ptr(const float* p, int src) {
  return reinterpret_cast<const float*>(__shfl(reinterpret_cast<long long>(p), src));
}

// ---------------------------------------------------------------------------------------
// forward, MFMA: one wave per sample, 4 waves per block
// ---------------------------------------------------------------------------------------
// HEAD (DLRM, composed top MLP): the top MLP is one affine map of the row (its hidden layers
// are linear, ctr/layers.py:8), so the wave also forms y[b] = act(row·q + c) from the values it
// writes (row order, fixed butterfly), and the top MLP's batch-deep GEMM disappears.
struct FwdHead {
  const float* q;  // [out_stride] Q_0 over the written row (padding entries multiply zeros)
  const float* c;  // [1]
  float* y;        // [batch]
  int act;         // 0 linear, 1 relu, 2 sigmoid
  // DX: the unit interaction backward of the fused step (see below)
  float* dxu_emb;    // [batch * n_slots, D]
  float* dxu_dense;  // [batch, D]
};

// DX (production DLRM step, D = 128): the top MLP is one linear chain into a sigmoid, so the
// upstream gradient of the interaction row is rank one, G[b] ⊗ Q_0 (G[b] = σ'(y)·dL/dy, a
// per-example scalar known only after the loss). dX[b] = G[b] · (M + Mᵀ)·X[b] with M the
// strict-upper Q_0 pairs, a matrix shared by every example. While X[b] is still in registers
// the wave also forms the UNIT gradient U[b] = (M + Mᵀ)·X[b] (and U[b, S] + Q_0's dense part for
// the bottom-MLP row); the sparse apply scales each row by G[b] as it reads it. The backward
// then never re-gathers the 27 table rows of an example (the 872 MB re-read of the separate
// backward at the north star). (M + Mᵀ)·X runs on v_mfma_f32_16x16x4_f32 per 16-column tile:
// the X tile is transposed through 2 KB of LDS (the gather layout puts rows on lane % 16, the
// B operand wants them on lane / 16).

template <int D, class Src, bool DLRM_OUT, bool HEAD = false, bool DX = false>
__global__ __launch_bounds__(256) void inter_fwd_mfma(Src src, int64_t batch, int F, InterMode md,
                                                      float* __restrict__ out, int64_t out_stride,
                                                      FwdHead hd = {}) {
  constexpr int NT = D / 16;  // float4 loads per lane per block-row
  static_assert(!DX || (HEAD && DLRM_OUT && D == 128), "DX is the fused DLRM head path");
  __shared__ float zt[4][32][33];
  __shared__ __attribute__((aligned(16))) float xtile[DX ? 4 : 1][32][16];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  if (b >= batch) return;
  const int r = lane & 15, g = lane >> 4;
  bool oob = false;
  // HEAD: this lane's q entries (compact row: pair o = lane + 64t, dense d = lane + 64t), loaded
  // ahead of the gathers so their latency hides behind the row loads
  // Every global load of the example is issued before its first store: vmcnt counts loads and
  // stores in one in-order counter, so a load issued after the row stores would make its wait
  // drain those stores too.
  constexpr int kHz = HEAD ? 8 : 1, kHd = HEAD ? (D + 63) / 64 : 1;
  float qz[kHz], qd[kHd], dnv[kHd], cc = 0.f;
  if constexpr (HEAD) {
    const int nzc = F * (F - 1) / 2;
#pragma unroll
    for (int t = 0; t < kHz; ++t) qz[t] = lane + 64 * t < nzc ? hd.q[lane + 64 * t] : 0.f;
#pragma unroll
    for (int t = 0; t < kHd; ++t) {
      const bool in = lane + 64 * t < D;
      qd[t] = in ? hd.q[nzc + lane + 64 * t] : 0.f;
      dnv[t] = in ? src.dense[b * D + lane + 64 * t] : 0.f;
    }
    cc = hd.c[0];
  }
  // DX: the A operand (M + Mᵀ)[m = 16 ib + r][k = 4 kk + g] of the unit backward, and this
  // lane's q dense entries for the bottom row's pass-through (column 16 t + r)
  constexpr int kSa = DX ? 8 : 1, kQn = DX ? NT : 1;
  float sa[2][kSa], qdn[kQn];
  if constexpr (DX) {
    const int nzc = F * (F - 1) / 2;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int kk = 0; kk < kSa; ++kk) {
        const int m = 16 * ib + r, k = 4 * kk + g;
        const bool in = m < F && k < F && m != k;
        const int o = in ? compact_index(m < k ? m : k, m < k ? k : m, F, 0) : 0;
        const float v = hd.q[o];  // unconditional (clamped) load, then select
        sa[ib][kk] = in ? v : 0.f;
      }
#pragma unroll
    for (int t = 0; t < kQn; ++t) qdn[t] = hd.q[nzc + 16 * t + r];
  }
  // lane k < F resolves row k once; the MFMA lanes fetch the pointers by shuffle
  const float* mine = lane < F ? src.row(b, lane, D, oob) : nullptr;
  const float* p0 = shfl_ptr(mine, r);
  const float* p1 = shfl_ptr(mine, 16 + r);
  if (r >= F) p0 = nullptr;
  if (16 + r >= F) p1 = nullptr;
  float4 a0[NT], a1[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int col = g * 4 + 16 * t;
    a0[t] = p0 ? *reinterpret_cast<const float4*>(p0 + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    a1[t] = p1 ? *reinterpret_cast<const float4*>(p1 + col) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  floatx4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c11 = c00;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float x0[4] = {a0[t].x, a0[t].y, a0[t].z, a0[t].w};
    const float x1[4] = {a1[t].x, a1[t].y, a1[t].z, a1[t].w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      c00 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[c], x0[c], c00, 0, 0, 0);
      c01 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[c], x1[c], c01, 0, 0, 0);
      c11 = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[c], x1[c], c11, 0, 0, 0);
    }
  }
  // C layout: lane holds G[4g + reg][r] of each block; mirror into a full 32x32 tile
  float(*z)[33] = zt[wave];
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    int i = 4 * g + reg;
    z[i][r] = c00[reg];
    z[i][16 + r] = c01[reg];
    z[16 + r][i] = c01[reg];
    z[16 + i][16 + r] = c11[reg];
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  float* orow = out + b * out_stride;
  const int nz = out_width(F, md.self_interaction, md.skip_gather);
  float hacc = 0.f;  // HEAD: this lane's share of row·q
  if constexpr (HEAD) {  // compact row only (F <= 32: nz <= 465 < 64·kHz)
#pragma unroll
    for (int t = 0; t < kHz; ++t) {
      const int o = lane + 64 * t;
      if (o < nz) {
        int i, j;
        compact_pair(o, F, false, i, j);
        const float v = z[i][j];
        orow[o] = v;
        hacc += v * qz[t];
      }
    }
  } else if (md.skip_gather) {
    for (int o = lane; o < nz; o += 64) {
      int i = o / F, j = o - i * F;
      orow[o] = keep_pair(i, j, md.self_interaction) ? z[i][j] : 0.f;
    }
  } else {
    for (int o = lane; o < nz; o += 64) {
      int i, j;
      compact_pair(o, F, md.self_interaction, i, j);
      orow[o] = z[i][j];
    }
  }
  if constexpr (DLRM_OUT) {
    // concat the bottom-MLP output behind Z (ctr/model.py:54)
    const float* dn = src.dense + b * D;
    float* od = orow + nz;
    if constexpr (HEAD) {
#pragma unroll
      for (int t = 0; t < kHd; ++t) {
        const int d = lane + 64 * t;
        if (d < D) {
          const float v = dnv[t];
          od[d] = v;
          hacc += v * qd[t];
        }
      }
    } else {
      for (int d = lane; d < D; d += 64) od[d] = dn[d];
    }
    if constexpr (HEAD) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) hacc += __shfl_xor(hacc, off);
      if (lane == 0) {
        const float v = hacc + cc;
        hd.y[b] = hd.act == 2 ? 1.f / (1.f + expf(-v)) : (hd.act == 1 ? fmaxf(v, 0.f) : v);
      }
    }
    // zero the alignment padding of the row (compact layout padded for the GEMM tiles)
    for (int64_t o = nz + D + lane; o < out_stride; o += 64) orow[o] = 0.f;
    if (__any(oob) && lane == 0) flag_oob(src.err_flag);
  }
  if constexpr (DX) {
    const int S = src.n_slots;
    float(*xt)[16] = xtile[wave];
    float* de = hd.dxu_emb + b * S * (int64_t)D;
    float* dd = hd.dxu_dense + b * D;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      // X[:, 16t .. 16t+15] → LDS as [row][col]; read back with the row on lane / 16
      *reinterpret_cast<float4*>(&xt[r][4 * g]) = a0[t];
      *reinterpret_cast<float4*>(&xt[16 + r][4 * g]) = a1[t];
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      float bv[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) bv[kk] = xt[4 * kk + g][r];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // every read done before the next tile's writes
      __builtin_amdgcn_wave_barrier();
      floatx4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(sa[0][kk], bv[kk], d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(sa[1][kk], bv[kk], d1, 0, 0, 0);
      }
      // C layout: lane holds U[4g + reg (+16)][16t + r]
      const int col = 16 * t + r;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int i0 = 4 * g + reg, i1 = 16 + 4 * g + reg;
        if (i0 < S) de[i0 * D + col] = d0[reg];
        else if (i0 == S) dd[col] = d0[reg] + qdn[t];  // + the concat pass-through
        if (i1 < S) de[i1 * D + col] = d1[reg];
        else if (i1 == S) dd[col] = d1[reg] + qdn[t];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// backward, MFMA: dX = S · X, one wave per sample
// ---------------------------------------------------------------------------------------
constexpr int kMaxGradRow = 32 * 32 + 256;

template <int D, class Src, bool DLRM_OUT>
__global__ __launch_bounds__(256) void inter_bwd_mfma(Src src, int64_t batch, int F, InterMode md,
                                                      const float* __restrict__ gout, int64_t gstride,
                                                      float* __restrict__ gx,      // dense: [B,F,D]
                                                      float* __restrict__ gemb,    // DLRM: [B*S, D]
                                                      float* __restrict__ gdense)  // DLRM: [B, D]
{
  constexpr int NTILE = D / 32;
  constexpr int KS = 16;  // up to 32 k-rows in steps of 2
  __shared__ float gsm[4][kMaxGradRow];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  if (b >= batch) return;
  const int r = lane & 31, h = lane >> 5;
  const int ks = (F + 1) >> 1;
  const int nz = out_width(F, md.self_interaction, md.skip_gather);
  bool oob = false;

  // (1) row pointers: lane k < F resolves row k
  const float* mine = lane < F ? src.row(b, lane, D, oob) : nullptr;
  // (2) stage the incoming gradient row (coalesced)
  float* gs = gsm[wave];
  const float* grow = gout + b * gstride;
  const int gw = nz + (DLRM_OUT ? D : 0);
  for (int o = lane; o < gw; o += 64) gs[o] = grow[o];
  // (3) every X row this lane feeds to the MFMA: rows k = 2s + h, NTILE floats at NTILE*r
  float xv[KS][NTILE];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + h;
    const float* xr = shfl_ptr(mine, k < 64 ? k : 0);
    if (k >= F) xr = nullptr;
    if (xr) {
      if constexpr (NTILE == 4) {
        float4 t = *reinterpret_cast<const float4*>(xr + NTILE * r);
        xv[s][0] = t.x; xv[s][1] = t.y; xv[s][2] = t.z; xv[s][3] = t.w;
      } else if constexpr (NTILE == 2) {
        float2 t = *reinterpret_cast<const float2*>(xr + NTILE * r);
        xv[s][0] = t.x; xv[s][1] = t.y;
      } else {
#pragma unroll
        for (int c = 0; c < NTILE; ++c) xv[s][c] = xr[NTILE * r + c];
      }
    } else {
#pragma unroll
      for (int c = 0; c < NTILE; ++c) xv[s][c] = 0.f;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  // (4) S[r][k] = M[r][k] + M[k][r] from the staged gradient
  auto m_at = [&](int i, int k) -> float {
    if (!keep_pair(i, k, md.self_interaction)) return 0.f;
    return md.skip_gather ? gs[i * F + k] : gs[compact_index(i, k, F, md.self_interaction)];
  };
  float sa[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + h;
    sa[s] = (r < F && k < F) ? m_at(r, k) + m_at(k, r) : 0.f;
  }
  floatx16 acc[NTILE];
#pragma unroll
  for (int c = 0; c < NTILE; ++c)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[c][e] = 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s < ks) {
#pragma unroll
      for (int c = 0; c < NTILE; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(sa[s], xv[s][c], acc[c], 0, 0, 0);
    }
  }
  // D layout: acc[c][reg] = dX[i = (reg&3) + 8*(reg>>2) + 4*h][d = NTILE*r + c]
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int i = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    if (i >= F) continue;
    float v[NTILE];
#pragma unroll
    for (int c = 0; c < NTILE; ++c) v[c] = acc[c][reg];
    float* dst;
    if constexpr (DLRM_OUT) {
      if (i < src.n_slots) {
        dst = gemb + (b * src.n_slots + i) * (int64_t)D;
      } else {
        // bottom-MLP row: interaction grad + the concat pass-through (ctr/model.py:54)
#pragma unroll
        for (int c = 0; c < NTILE; ++c) v[c] += gs[nz + NTILE * r + c];
        dst = gdense + b * D;
      }
    } else {
      dst = gx + (b * F + i) * (int64_t)D;
    }
    if constexpr (NTILE == 4) {
      *reinterpret_cast<float4*>(dst + NTILE * r) = make_float4(v[0], v[1], v[2], v[3]);
    } else if constexpr (NTILE == 2) {
      *reinterpret_cast<float2*>(dst + NTILE * r) = make_float2(v[0], v[1]);
    } else {
#pragma unroll
      for (int c = 0; c < NTILE; ++c) dst[NTILE * r + c] = v[c];
    }
  }
}

// ---------------------------------------------------------------------------------------
// DLRM backward, software-pipelined (the production path for D = 128): each wave walks
// kPipeEPW consecutive examples. The ids of b+2 are loaded while b is processed, the row
// pointers of b+1 are resolved before b's MFMAs, and b+1's rows are gathered into the operand
// registers as soon as b's MFMA chain has read them — overlapping b's MFMA drain, its grad-row
// stores and the staging of the next grad row. Every wait is a counted in-order vmcnt (plain
// global loads, no LDS-DMA), so b's stores never hold up b+1's loads. Per-example arithmetic
// is that of inter_bwd_mfma (same MFMA order): bit-identical results.
// Measured (1x MI355X, north-star batch): 393 us → 298-320 us at 2 waves/SIMD (186 VGPR + 64
// AGPR); forcing 3 waves spills and is slower (385 us); 64 examples per wave loses to the tail.
// The same pipelining of the forward (3 waves/SIMD) measured 277-280 us against 244 us for
// the 5-wave inter_fwd_mfma, so the forward keeps the one-example-per-wave kernel.
// ---------------------------------------------------------------------------------------
constexpr int kPipeEPW = 16;  // upper bound; the launch sizes it to the occupancy (pipe_epw)

// Examples per wave so that the grid is exactly kPipeRounds full rounds of resident waves
// (a partial last round idles most SIMDs: 16 examples/wave at 3 waves/SIMD is 1.33 rounds).
#ifndef RS_PIPE_ROUNDS
#define RS_PIPE_ROUNDS 2
#endif
constexpr int kPipeRounds = RS_PIPE_ROUNDS;
static int pipe_epw_uncached(const void* kernel, int dev, int64_t batch, int rounds) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus < 1)
    cus = 256;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t slots = (int64_t)cus * per_cu * 4 * rounds;  // waves over all rounds
  const int64_t e = ceil_div(batch, slots);
  return (int)(e < 1 ? 1 : (e > 64 ? 64 : e));
}

// cached per (device, kernel, batch, rounds): occupancy depends on the device, and several host
// threads may launch at once (one per GPU), so the cache is shared and locked
static int pipe_epw(const void* kernel, int64_t batch, int rounds = kPipeRounds) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, int64_t, int>, int> cache;
  const auto key = std::make_tuple(dev, kernel, batch, rounds);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  const int e = pipe_epw_uncached(kernel, dev, batch, rounds);
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = e;
  return e;
}

typedef __attribute__((address_space(1))) const floatx4 gfloatx4;
typedef __attribute__((address_space(1))) const float gfloat;

// a zero row in global memory: absent / out-of-table rows are gathered from here, so the
// pipelined gathers need no per-row select (a select would keep a lane mask live per row)
__device__ const float kZeroRow[256] = {};

// RANK1: the upstream gradient is rank one, grad row b = gscale[b] * gout[0..gstride) (the
// factored top-MLP backward's dZ = G ⊗ Q_0): each staged value is the same single fp32 product
// the materialised dZ would hold, so the results are bit-identical to that path, without the
// [B, width] write and read.
template <int D, int GREG, int KS, bool SELF, bool SKIP, bool ID64, bool RANK1 = false>
__global__ __launch_bounds__(256) void dlrm_bwd_pipe(GatherSrc src, int64_t batch, int F,
                                                     const float* __restrict__ gout,
                                                     int64_t gstride, float* __restrict__ gemb,
                                                     float* __restrict__ gdense, int epw,
                                                     const float* __restrict__ gscale = nullptr) {
  static_assert(D == 128, "pipelined backward is laid out for D = 128 (4 floats per lane)");
  constexpr int NTILE = 4;
  // per wave: the staged grad row + one zero slot (index ZS) that dropped pairs read
  constexpr int ZS = GREG * 64;
  __shared__ float gsm[4][ZS + 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t first = ((int64_t)blockIdx.x * 4 + wave) * epw;
  if (first >= batch) return;
  const int64_t last = first + epw < batch ? first + epw : batch;
  const int r = lane & 31, h = lane >> 5;
  const int nz = out_width(F, SELF, SKIP);
  const int S = src.n_slots;
  // lane i < S owns slot i: its table range is loaded once
  int64_t lo = 0, n_ok = src.n_rows;
  if (lane < S && src.slot_offsets) {
    lo = src.slot_offsets[lane];
    n_ok = src.slot_offsets[lane + 1] - lo;
  }
  bool oob = false;
  auto raw_id = [&](int64_t b) -> int64_t {
    const int64_t bb = b < last ? b : first;  // past the end: a valid, unused load
    if (lane >= S) return 0;
    return ID64 ? static_cast<const int64_t*>(src.ids)[bb * S + lane]
                : static_cast<int64_t>(static_cast<const int32_t*>(src.ids)[bb * S + lane]);
  };
  // lane k's row of example b (kZeroRow for absent / OOB rows and for k >= F)
  auto row_of = [&](int64_t b, int64_t id) -> const float* {
    const bool live = b < last;
    const bool id_ok = id >= 0 && id < n_ok;
    if (lane < S && !id_ok && live) oob = true;
    if (lane < S) return id_ok ? src.table + (lo + id) * D : kZeroRow;
    return (lane == S && live) ? src.dense + b * D : kZeroRow;
  };
  float xv[KS][NTILE];
  auto load_rows = [&](const float* mine, int s) {
    const float* xr = shfl_ptr(mine, 2 * s + h);
    const floatx4 t = *(gfloatx4*)(xr + NTILE * r);  // global_load_dwordx4 (not flat)
    xv[s][0] = t[0];
    xv[s][1] = t[1];
    xv[s][2] = t[2];
    xv[s][3] = t[3];
  };
  float gnx[GREG];
  const int glast = (int)gstride - 1;  // reads past the row end are clamped (the values there
                                       // are never used: every index read is < gw)
  float pv[RANK1 ? GREG : 1];
  if constexpr (RANK1) {
#pragma unroll
    for (int j = 0; j < GREG; ++j) pv[j] = gout[min(lane + 64 * j, glast)];
  }
  auto load_g = [&](int64_t b, int ln) {  // ln: a lane id (the loop passes the opaque one)
    const int64_t bb = b < last ? b : first;
    if constexpr (RANK1) {
      const float gsc = gscale[bb];
#pragma unroll
      for (int j = 0; j < GREG; ++j) gnx[j] = gsc * pv[j];
    } else {
      gfloat* grow = (gfloat*)(gout + bb * gstride);
#pragma unroll
      for (int j = 0; j < GREG; ++j) gnx[j] = grow[min(ln + 64 * j, glast)];
    }
  };
  // prologue: example `first` in flight, ids of first+1 in flight
  const float* cur = row_of(first, raw_id(first));
  int64_t id_next = raw_id(first + 1);
#pragma unroll
  for (int s = 0; s < KS; ++s) load_rows(cur, s);
  load_g(first, lane);
  float* gs = gsm[wave];
  if (lane == 0) gs[ZS] = 0.f;
  for (int64_t b = first; b < last; ++b) {
    // lane-derived values recomputed per example from an opaque lane id: hoisted out of the
    // loop they would pin ~70 VGPRs (LDS indices, store offsets) for the whole loop
    int lanev;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lanev));
    const int r = lanev & 31, h = lanev >> 5;
    // (1) stage this example's grad row; resolve b+1's rows; put b+2's ids in flight
#pragma unroll
    for (int j = 0; j < GREG; ++j) gs[lane + 64 * j] = gnx[j];
    const float* nxt = row_of(b + 1, id_next);
    id_next = raw_id(b + 2);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the staged row is visible to the wave
    __builtin_amdgcn_wave_barrier();
    float sa[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 2 * s + h;
      const bool in = r < F && k < F;
      const bool p1 = in && keep_pair(r, k, SELF);
      const bool p2 = in && keep_pair(k, r, SELF);
      const int j1 = p1 ? (SKIP ? r * F + k : compact_index(r, k, F, SELF)) : ZS;
      const int j2 = p2 ? (SKIP ? k * F + r : compact_index(k, r, F, SELF)) : ZS;
      sa[s] = gs[j1] + gs[j2];
    }
    // (2) dX = S·X; each k-step's registers are refilled with b+1's rows right behind it
    floatx16 acc[NTILE];
#pragma unroll
    for (int c = 0; c < NTILE; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[c][e] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int c = 0; c < NTILE; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(sa[s], xv[s][c], acc[c], 0, 0, 0);
    }
    // every operand register has been read by its MFMA: refill them with b+1's rows while the
    // MFMA chain drains and this example's grad rows are stored
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < KS; ++s) load_rows(nxt, s);
    __builtin_amdgcn_sched_barrier(0);
    // bottom-MLP pass-through of this example (read before the LDS row is restaged)
    float dpass[NTILE];
#pragma unroll
    for (int c = 0; c < NTILE; ++c) dpass[c] = gs[nz + NTILE * r + c];
    load_g(b + 1, lanev);
    // (3) grad rows (position order) + bottom grad
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int i = (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (i < F) {
        float v[NTILE];
#pragma unroll
        for (int c = 0; c < NTILE; ++c) v[c] = acc[c][reg] + (i == S ? dpass[c] : 0.f);
        float* dst = (i < S ? gemb + (b * S + i) * (int64_t)D : gdense + b * D) + NTILE * r;
        *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
  if (__any(oob) && lane == 0) flag_oob(src.err_flag);
}

// ---------------------------------------------------------------------------------------
// Fused forward + unit backward, software-pipelined (the production DLRM step at D = 128,
// F <= 28): each wave walks `epw` consecutive examples. Per example b:
//   Z = X·Xᵀ from the gather registers (as inter_fwd_mfma) → X(b) copied to the wave's LDS
//   region → the registers are refilled with X(b+1) (its loads fly behind everything below)
//   → z row + fused head y → U = (M + Mᵀ)·X per 16-column tile from LDS on
//   v_mfma_f32_16x16x4_f32, written back over the tile → U rows stored whole (a half-wave per
//   512-B row, as the re-gathering backward stored its grad rows).
// Per-example arithmetic is that of inter_fwd_mfma<…, HEAD, DX> (same MFMA order, same head
// butterfly): bit-identical z, y, U. Every global load of an iteration is issued before its
// stores except X(b+1)'s, which only the next iteration waits for (in-order vmcnt).
// ---------------------------------------------------------------------------------------
constexpr int kDxLdx = 136;               // X / U row stride in LDS (floats): every LDS
                                          // access pattern of the loop is at most 2-way
                                          // bank-conflicted
constexpr int kDxRows = 28;               // LDS rows per wave: F <= 28 (a multiple of 4)
constexpr int kDxZt = 32 * 33;            // Z staging

template <bool ID64>
__global__ __launch_bounds__(256) void dlrm_fwd_dx_pipe(GatherSrc src, int64_t batch, int F,
                                                        float* __restrict__ out,
                                                        int64_t out_stride, FwdHead hd, int epw) {
  constexpr int D = 128, NT = 8;
  __shared__ __attribute__((aligned(16))) float lds[4][kDxRows * kDxLdx + kDxZt];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t first = ((int64_t)blockIdx.x * 4 + wave) * epw;
  if (first >= batch) return;
  const int64_t last = first + epw < batch ? first + epw : batch;
  const int r = lane & 15, g = lane >> 4;
  const int r32 = lane & 31, h = lane >> 5;
  const int S = src.n_slots;
  const int nzc = F * (F - 1) / 2;
  float* X = lds[wave];                       // [kDxRows][kDxLdx]: X, then U in place
  float(*z)[33] = reinterpret_cast<float(*)[33]>(lds[wave] + kDxRows * kDxLdx);
  // per-wave constants: head q entries, (M + Mᵀ) operand, q's dense part for the bottom row
  float qz[8], qd[2], sa[2][8], qdn[4];
#pragma unroll
  for (int t = 0; t < 8; ++t) qz[t] = lane + 64 * t < nzc ? hd.q[lane + 64 * t] : 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) qd[t] = hd.q[nzc + lane + 64 * t];
  const float cc = hd.c[0];
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int m = 16 * ib + r, k = 4 * kk + g;
      const bool in = m < F && k < F && m != k;
      const float v = hd.q[in ? compact_index(m < k ? m : k, m < k ? k : m, F, 0) : 0];
      sa[ib][kk] = in ? v : 0.f;
    }
#pragma unroll
  for (int c = 0; c < 4; ++c) qdn[c] = hd.q[nzc + 4 * r32 + c];
  // this lane's compact outputs o = lane + 64 t read Z[i][j]: the LDS offsets are the same for
  // every example (computed once; inverting the pair index costs a sqrt and two loops)
  int zoff[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int o = lane + 64 * t;
    int i = 0, j = 0;
    if (o < nzc) compact_pair(o, F, false, i, j);
    zoff[t] = o < nzc ? i * 33 + j : -1;
  }
  // lane i < S owns slot i: its table range is loaded once
  int64_t lo = 0, n_ok = src.n_rows;
  if (lane < S && src.slot_offsets) {
    lo = src.slot_offsets[lane];
    n_ok = src.slot_offsets[lane + 1] - lo;
  }
  bool oob = false;
  // every memory op of the loop is issued unconditionally (lanes that have nothing to do load
  // or store a harmless duplicate), so the compiler can count vmcnt exactly across iterations
  // instead of draining all stores before each example's MFMAs
  auto raw_id = [&](int64_t b) -> int64_t {
    const int64_t bb = b < last ? b : first;
    const int ln = lane < S ? lane : S - 1;
    const int64_t v = ID64 ? static_cast<const int64_t*>(src.ids)[bb * S + ln]
                           : static_cast<int64_t>(static_cast<const int32_t*>(src.ids)[bb * S + ln]);
    return lane < S ? v : 0;
  };
  auto row_of = [&](int64_t b, int64_t id) -> const float* {
    const bool live = b < last;
    const bool id_ok = id >= 0 && id < n_ok;
    if (lane < S && !id_ok && live) oob = true;
    if (lane < S) return id_ok ? src.table + (lo + id) * D : kZeroRow;
    return (lane == S && live) ? src.dense + (b < last ? b : first) * D : kZeroRow;
  };
  floatx4 a0[NT], a1[NT];
  float dnv[2];
  auto gather = [&](const float* mine, int64_t b) {
    const float* p0 = shfl_ptr(mine, r);
    const float* p1 = shfl_ptr(mine, 16 + r);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      a0[t] = *(gfloatx4*)(p0 + 4 * g + 16 * t);
      a1[t] = *(gfloatx4*)(p1 + 4 * g + 16 * t);
    }
    const int64_t bb = b < last ? b : first;
#pragma unroll
    for (int t = 0; t < 2; ++t) dnv[t] = *(gfloat*)(src.dense + bb * D + lane + 64 * t);
  };
  // prologue: X(first) in flight, ids of first+1 in flight
  gather(row_of(first, raw_id(first)), first);
  int64_t id_next = raw_id(first + 1);
  for (int64_t b = first; b < last; ++b) {
    // lane-derived values are recomputed per example from an opaque lane id: hoisted out of
    // the loop, the LDS / store offsets would pin ~100 VGPRs for the whole loop
    int lanev;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lanev));
    const int r = lanev & 15, g = (lanev >> 4) & 3;
    const int r32 = lanev & 31, h = (lanev >> 5) & 1;
    const float* nxt = row_of(b + 1, id_next);
    id_next = raw_id(b + 2);
    // (1) Z = X·Xᵀ (three 16x16 blocks), as inter_fwd_mfma
    floatx4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c11 = c00;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        c00 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[t][c], a0[t][c], c00, 0, 0, 0);
        c01 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[t][c], a1[t][c], c01, 0, 0, 0);
        c11 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[t][c], a1[t][c], c11, 0, 0, 0);
      }
    }
    // (2) X(b) → LDS rows 0..27 (rows >= F are zeros and never read back as U)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      *reinterpret_cast<floatx4*>(&X[r * kDxLdx + 16 * t + 4 * g]) = a0[t];
      if (16 + r < kDxRows) *reinterpret_cast<floatx4*>(&X[(16 + r) * kDxLdx + 16 * t + 4 * g]) = a1[t];
    }
    float dn_cur[2] = {dnv[0], dnv[1]};
    // (3) the registers are free: X(b+1) loads fly behind the rest of this example
    __builtin_amdgcn_sched_barrier(0);
    gather(nxt, b + 1);
    __builtin_amdgcn_sched_barrier(0);
    // (4) z row + head, as inter_fwd_mfma<…, HEAD>
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int i = 4 * g + reg;
      z[i][r] = c00[reg];
      z[i][16 + r] = c01[reg];
      z[16 + r][i] = c01[reg];
      z[16 + i][16 + r] = c11[reg];
    }
    __builtin_amdgcn_wave_barrier();  // Z staging: the reads below follow the writes in issue order
    float* orow = out + b * out_stride;
    float hacc = 0.f;
    const int pad = nzc + D;  // first padding column (zero): lanes past the row write it
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int o = lanev + 64 * t;
      const bool in = zoff[t] >= 0;
      const float v = in ? (&z[0][0])[zoff[t]] : 0.f;
      orow[in ? o : pad] = v;
      hacc += v * qz[t];
    }
    float* od = orow + nzc;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int d = lanev + 64 * t;
      od[d] = dn_cur[t];
      hacc += dn_cur[t] * qd[t];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) hacc += __shfl_xor(hacc, off);
    {  // every lane holds the same sum: all store the same y[b]
      const float v = hacc + cc;
      hd.y[b] = hd.act == 2 ? 1.f / (1.f + expf(-v)) : (hd.act == 1 ? fmaxf(v, 0.f) : v);
    }
    {  // zero padding (out_stride - pad <= 64, checked by the launcher)
      const int o = pad + lanev;
      orow[o < out_stride ? o : pad] = 0.f;
    }
    // (5) U = (M + Mᵀ)·X per 16-column tile, written back over the tile
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      // K = the kDxRows = 28 LDS rows (rows >= F are zeros meeting a zero A operand): 7 k-steps
      constexpr int KK = kDxRows / 4;
      float bv[KK];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) bv[kk] = X[(4 * kk + g) * kDxLdx + 16 * t + r];
      floatx4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(sa[0][kk], bv[kk], d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(sa[1][kk], bv[kk], d1, 0, 0, 0);
      }
      // the U tile overwrites the X tile it was computed from: its values depend on every
      // lane's reads of that tile (through the MFMA), and one wave's LDS operations execute in
      // issue order, so no wait is needed; the next tile's reads touch other columns
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int i0 = 4 * g + reg, i1 = 16 + 4 * g + reg;
        X[i0 * kDxLdx + 16 * t + r] = d0[reg];
        if (i1 < kDxRows) X[i1 * kDxLdx + 16 * t + r] = d1[reg];
      }
    }
    __builtin_amdgcn_wave_barrier();  // keep the row reads after the U writes (program order)
    // (6) U rows: a half-wave per 512-B row
    float* de = hd.dxu_emb + b * S * (int64_t)D;
#pragma unroll
    for (int s2 = 0; s2 < kDxRows / 2; ++s2) {
      // rows past S are clamped to S: both halves then store the same bottom row
      const int i = 2 * s2 + h < S ? 2 * s2 + h : S;
      floatx4 v = *reinterpret_cast<const floatx4*>(&X[i * kDxLdx + 4 * r32]);
      const bool emb = i < S;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = emb ? v[c] : v[c] + qdn[c];  // + the concat pass-through
      float* dst = emb ? de + i * D : hd.dxu_dense + b * D;
      *reinterpret_cast<floatx4*>(dst + 4 * r32) = v;
    }
    __builtin_amdgcn_wave_barrier();  // the next example's LDS writes follow these reads
  }
  if (__any(oob) && lane == 0) flag_oob(src.err_flag);
}

// ---------------------------------------------------------------------------------------
// The whole top half of the production DLRM training step in one pipelined pass (D = 128,
// F <= 28, sigmoid head, mean / sum Keras BCE). Per example b, as dlrm_fwd_dx_pipe (Z = X·Xᵀ on
// MFMA, X(b) to LDS, X(b+1) loads in flight, U = (M + Mᵀ)·X per 16-column tile), plus:
//   head     y = σ(Σ q·z + Σ q_d·dense + c) straight from the MFMA accumulators (no Z staging:
//            each lane owns 12 Z entries, their q weights are lane constants);
//   loss     l_b = keras BCE(label_b, y) (clip to [eps, 1-eps], log(p + eps)), summed;
//   G        G_b = σ'(y)·dL/dy = y(1-y)·g·d(label, y) (g = 1/B for the mean) — the top MLP
//            chain's last-layer gradient, known here, so the backward needs no second pass:
//   A_top    Σ_b z_b·G_b and Σ_b G_b (the factored top-MLP backward's reduction,
//            nn.chain_reduce) accumulated per lane from the same registers;
//   rows     the table gradient rows G_b·U_b written whole (position order), ready for the
//            segmented-sum apply (no row_scale);
//   bottom   the bottom-MLP row's gradient G_b·(U_b,S + q_d) through the bottom chain's relu
//            (h > 0), reduced on the spot: A_bot = Σ_b x_bᵀ·G_bot,b ([13, 128]) and Σ_b G_bot,b
//            (x = the 13 dense input features) — the bottom MLP's factored backward reduction.
// The z row, the [B, 128] bottom gradient and the BCE / chain-reduce passes are never
// materialised. Per-wave sums (examples in order) are folded per block in wave order and written
// as one partial row [kTrainM] per block; rs_dlrm_train_fold folds the blocks in a fixed order.
// ---------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// x = h + m + l with h, m, l bf16 (v_cvt_pk_bf16_f32, round to nearest): the two residuals are
// exact in fp32 and l carries x's bits below 2^-16 |x| to 2^-24 |x|. lo / hi: elements 0-3 / 4-7.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split3(const floatx4& lo, const floatx4& hi, bf16x8& h, bf16x8& m,
                                       bf16x8& l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // in pairs: one v_cvt_pk_bf16_f32 and one v_pk_add_f32 each
    const floatx2 x = j < 2 ? floatx2{lo[2 * j], lo[2 * j + 1]} : floatx2{hi[2 * j - 4], hi[2 * j - 3]};
    const bf16x2 hp = __builtin_convertvector(x, bf16x2);
    const floatx2 r1 = x - __builtin_convertvector(hp, floatx2);
    const bf16x2 mp = __builtin_convertvector(r1, bf16x2);
    const bf16x2 lp = __builtin_convertvector(r1 - __builtin_convertvector(mp, floatx2), bf16x2);
    h[2 * j] = hp[0];
    h[2 * j + 1] = hp[1];
    m[2 * j] = mp[0];
    m[2 * j + 1] = mp[1];
    l[2 * j] = lp[0];
    l[2 * j + 1] = lp[1];
  }
}

// c + A·B from the split operands: the six products down to 2^-16 |a||b|, smallest first
__device__ __forceinline__ floatx4 mfma6(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                         const bf16x8& bh, const bf16x8& bm, const bf16x8& bl,
                                         floatx4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

constexpr int kTrainAtop = 512;                       // A_top (compact row, zero padding)
constexpr int kTrainNI = 13;                          // bottom-MLP inputs (Criteo dense)
// the per-block partial row: A_top | s_top | loss | A_bot [13][D] | s_bot [D]
template <int D>
constexpr int train_m() { return kTrainAtop + 2 + kTrainNI * D + D; }
constexpr int kTrainM = train_m<128>();  // the largest (workspace sizing)

struct TrainArgs {
  const float* q;      // [nzc + D] Q_0 over the compact row
  const float* c;      // [1]
  const float* label;  // [B]
  const float* xin;    // [B, 13] bottom-MLP input
  float eps;           // BCE clip
  float gscale;        // dL/dl_b: 1/B (mean) or 1 (sum)
  float* y;            // [B] prediction
  float* grad_emb;     // [B * S, D] table gradient rows
  float* part;         // [gridDim.x, kTrainM]
};

// ---------------------------------------------------------------------------------------
// The train step with the interaction computed chunk by chunk (round 3): per 32-column chunk s
// of X(b) (rows r / 16 + r of the bf16 MFMA operand layout, already in registers),
//   split   x = h + m + l (split3), once — the same three parts feed both products;
//   Z       the chunk's k-step of Z = X·Xᵀ (three 16x16 blocks, mfma6);
//   loads   X(b+1)'s chunk s is issued into the registers just freed, so every chunk's loads
//           have a whole example of latency cover (no second register set);
//   image   the six bf16x8 parts go to a 6 KB per-wave LDS image [part][32 rows][32 columns]
//           (chunk-swizzled, ch_off: conflict-free writes and transposed reads), read back
//           column-major with ds_read_b64_tr_b16 as the A operand of
//   Uᵀ      Uᵀ = Xᵀ·(M + Mᵀ) for the chunk's two 16-column tiles: the MFMA result puts four
//           consecutive columns of one U row in each lane; a 4.5 KB staging tile turns them
//           into 128-B row segments for the stores (64-B segments measured half the rate).
// U is written UNSCALED (the head's G needs all of Z, known only after the last chunk) and G[b]
// goes to g_rows: the apply multiplies each gradient row by its example's G
// (rs_embedding_apply_scaled, row_scale = g_rows, scale_group = n_slots) with the same fmul_rn,
// so the table update is the one the G·U rows would give. Against round 3's first form (one
// kernel writing G·U rows, X staged in LDS as fp32 rows for U's transposed operand): no second
// split of X for U (≈0.3 k VALU per example), no fp32 X / U round trip through LDS, 6 KB
// instead of 17 KB of LDS per wave.
// ---------------------------------------------------------------------------------------
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) shortx4 lds_shortx4;

// the Uᵀ product: c + Xᵀ·S from the split operands, the six products smallest first
// (X as A, S as B: m·m, l·h, h·l, m·h, h·m, h·h)
__device__ __forceinline__ floatx4 mfma6_xs(const bf16x8& xh, const bf16x8& xm, const bf16x8& xl,
                                            const bf16x8& sh, const bf16x8& sm, const bf16x8& sl,
                                            floatx4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xm, sm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xl, sh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, sl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xm, sh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, sm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, sh, c, 0, 0, 0);
}

constexpr int kChPlane = 32 * 32 * 2;  // one part of the chunk image: 32 rows x 32 bf16
constexpr int kChImage = 3 * kChPlane;  // bytes
// byte offset of (row, column) in a plane: 64-B rows of four 16-B chunks (8 columns each), the
// chunk index XOR-swizzled by row bits 1-2 and 3. Conflict-free both ways (MI355X_MICROARCH
// §LDS): a ds_write_b128 group (8 lanes = 8 consecutive rows, one logical chunk) covers 32
// distinct banks mod 32, and a ds_read_b64_tr_b16 half-wave (rows 4h + q and 8 + 4h + q, one
// 16-column tile) gets rows 8 apart on the other chunk pair: 64 distinct banks mod 64
__device__ __forceinline__ int ch_off(int row, int col) {
  const int chunk = (col >> 3) ^ ((row >> 1) & 3) ^ (((row >> 3) & 1) << 1);
  return row * 64 + 16 * chunk + 2 * (col & 7);
}
constexpr int kChStageLd = 36;  // fp32 U staging rows [32][36]: 32 columns + 4 of padding
template <int D>
constexpr int chunk_region_floats() {
  return (kChImage / 4 + 32 * kChStageLd + D) > train_m<D>() ? (kChImage / 4 + 32 * kChStageLd + D)
                                                             : train_m<D>();
}

template <int D, bool ID64>
__global__ __launch_bounds__(256, 2) void dlrm_train_chunk(GatherSrc src, int64_t batch, int F,
                                                        TrainArgs ta, float* g_rows, int epw) {
  static_assert(D == 64 || D == 128, "train kernel laid out for D = 64 or 128");
  constexpr int NT = D / 16, NC = D / 32, DL = D / 4, RPI = 64 / DL, DPL = D / 64;
  constexpr int TM = train_m<D>();
  constexpr int RW = chunk_region_floats<D>();
  // per wave: the chunk image (kChImage bytes) + U's bottom row [D]; the partial row at the end
  __shared__ __attribute__((aligned(16))) float lds[4][RW];
  __shared__ __attribute__((aligned(16))) float qlane[64][12];
  __shared__ __attribute__((aligned(16))) float qsh[kTrainAtop];
  // S's split parts (the Uᵀ product's B operands), read per chunk: 24 VGPRs the loop needs more
  __shared__ __attribute__((aligned(16))) bf16x8 sash[2][3][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t first = ((int64_t)blockIdx.x * 4 + wave) * epw;
  const int64_t last = first + epw < batch ? first + epw : batch;
  const bool active = first < batch;
  const int r = lane & 15, g = lane >> 4;
  const int S = src.n_slots;
  const int nzc = F * (F - 1) / 2;
  char* img = reinterpret_cast<char*>(lds[wave]);
  float* stg = lds[wave] + kChImage / 4;          // the chunk's U columns, row-major
  float* ubot = stg + 32 * kChStageLd;
  // The prologue's loads are unguarded (index 0 where a weight does not exist, zeroed after):
  // guarded, the compiler waited for each of wave 0's twelve q loads in turn before the block
  // barrier every wave waits at (round 6, gfx950 ISA)
  for (int e = threadIdx.x; e < kTrainAtop; e += 256) {
    const float v = ta.q[e < nzc + D ? e : 0];
    qsh[e] = e < nzc + D ? v : 0.f;
  }
  if (wave == 0) {
    float qv[12];
    bool qk[12];
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int i0 = 4 * g + reg, j0 = r;
      const int i1 = 4 * g + reg, j1 = 16 + r;
      const int i2 = 16 + 4 * g + reg, j2 = 16 + r;
      qk[reg] = i0 < j0 && j0 < F;
      qk[4 + reg] = j1 < F;
      qk[8 + reg] = i2 < j2 && j2 < F;
      qv[reg] = ta.q[qk[reg] ? compact_index(i0, j0, F, 0) : 0];
      qv[4 + reg] = ta.q[qk[4 + reg] ? compact_index(i1, j1, F, 0) : 0];
      qv[8 + reg] = ta.q[qk[8 + reg] ? compact_index(i2, j2, F, 0) : 0];
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) qlane[lane][k] = qk[k] ? qv[k] : 0.f;
  }
  // S = M + Mᵀ as the B operand of Uᵀ = Xᵀ·S: lane (r, g) holds S[8g + j][16 ib + r], which by
  // symmetry is S[16 ib + r][8g + j]
  if (wave == 1) {
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      floatx4 v[2];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = 16 * ib + r, kk = 8 * g + j;
        const bool in = m < F && kk < F && m != kk;
        const float q = ta.q[in ? compact_index(m < kk ? m : kk, m < kk ? kk : m, F, 0) : 0];
        v[j >> 2][j & 3] = in ? q : 0.f;
      }
      split3(v[0], v[1], sash[ib][0][lane], sash[ib][1][lane], sash[ib][2][lane]);
    }
  }
  __syncthreads();
  const float cc = ta.c[0];
  float az[12], ad[4], abot[DPL][kTrainNI], sbot[DPL];
  float s_top = 0.f, loss = 0.f;
#pragma unroll
  for (int k = 0; k < 12; ++k) az[k] = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) ad[k] = 0.f;
#pragma unroll
  for (int k = 0; k < DPL; ++k) {
    sbot[k] = 0.f;
#pragma unroll
    for (int i = 0; i < kTrainNI; ++i) abot[k][i] = 0.f;
  }
  int64_t lo = 0, n_ok = src.n_rows;
  if (lane < S && src.slot_offsets) {
    lo = src.slot_offsets[lane];
    n_ok = src.slot_offsets[lane + 1] - lo;
  }
  bool oob = false;
  auto raw_id = [&](int64_t b) -> int64_t {
    const int64_t bb = b < last ? b : first;
    const int ln = lane < S ? lane : S - 1;
    const int64_t v = ID64 ? static_cast<const int64_t*>(src.ids)[bb * S + ln]
                           : static_cast<int64_t>(static_cast<const int32_t*>(src.ids)[bb * S + ln]);
    return lane < S ? v : 0;
  };
  auto row_of = [&](int64_t b, int64_t id) -> const float* {
    const bool live = b < last;
    const bool id_ok = id >= 0 && id < n_ok;
    if (lane < S && !id_ok && live) oob = true;
    if (lane < S) return id_ok ? src.table + (lo + id) * D : kZeroRow;
    return (lane == S && live) ? src.dense + (b < last ? b : first) * D : kZeroRow;
  };
  floatx4 a0[NT], a1[NT];
  floatx4 dn4;
  const float* p0 = nullptr;
  const float* p1 = nullptr;
  auto load_chunk = [&](int s) {
    a0[2 * s] = *(gfloatx4*)(p0 + 32 * s + 8 * g);
    a0[2 * s + 1] = *(gfloatx4*)(p0 + 32 * s + 8 * g + 4);
    a1[2 * s] = *(gfloatx4*)(p1 + 32 * s + 8 * g);
    a1[2 * s + 1] = *(gfloatx4*)(p1 + 32 * s + 8 * g + 4);
  };
  auto load_side = [&](int64_t b) {
    const int cl = lane & (DL - 1);
    const int64_t bb = b < last ? b : first;
    dn4 = *(gfloatx4*)(src.dense + bb * D + 4 * cl);
  };
  if (active) {
    {
      const float* mine = row_of(first, raw_id(first));
      p0 = shfl_ptr(mine, r);
      p1 = shfl_ptr(mine, 16 + r);
      load_side(first);
#pragma unroll
      for (int s = 0; s < NC; ++s) load_chunk(s);
    }
    int64_t id_next = raw_id(first + 1);
    for (int64_t b = first; b < last; ++b) {
      int lanev;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lanev));
      const int r = lanev & 15, g = (lanev >> 4) & 3;
      // X(b+1)'s rows: the chunk loads below go there
      {
        const float* nxt = row_of(b + 1, id_next);
        p0 = shfl_ptr(nxt, r);
        p1 = shfl_ptr(nxt, 16 + r);
      }
      id_next = raw_id(b + 2);
      const floatx4 dn = dn4;
      float xb[kTrainNI];
      // x_b (13 inputs) and label_b are wave-uniform: scalar loads, counted by lgkmcnt, so
      // reading them waits on nothing in the vector memory queue (a vector load + readlane
      // waited for the previous example's row stores: vmcnt(2) in the ISA; -3 % measured)
      typedef __attribute__((address_space(4))) const float cfloat;
      const int bq = __builtin_amdgcn_readfirstlane((int)b);
      const cfloat* xr = (const cfloat*)(ta.xin + (int64_t)bq * kTrainNI);
#pragma unroll
      for (int i = 0; i < kTrainNI; ++i) xb[i] = xr[i];
      const float lb = ((const cfloat*)ta.label)[bq];
      load_side(b + 1);
      float* de = ta.grad_emb + b * S * (int64_t)D;
      floatx4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c11 = c00;
      // transposed-read addresses (lane 4q + p of group g: row 8g + 4h + q, columns 4p.. of
      // 16-column tile tt, through ch_off's swizzle)
      const int q = (lanev >> 2) & 3, p4 = lanev & 3;
#pragma unroll
      for (int s = 0; s < NC; ++s) {
        bf16x8 sa[2][3];
#pragma unroll
        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
          for (int pt = 0; pt < 3; ++pt) sa[ib][pt] = sash[ib][pt][lanev & 63];
        bf16x8 h0, m0, l0, h1, m1, l1;
        split3(a0[2 * s], a0[2 * s + 1], h0, m0, l0);
        split3(a1[2 * s], a1[2 * s + 1], h1, m1, l1);
        __builtin_amdgcn_sched_barrier(0);
        load_chunk(s);  // X(b+1), chunk s: in flight for a whole example
        __builtin_amdgcn_sched_barrier(0);
        c00 = mfma6(h0, m0, l0, h0, m0, l0, c00);
        c01 = mfma6(h0, m0, l0, h1, m1, l1, c01);
        c11 = mfma6(h1, m1, l1, h1, m1, l1, c11);
        // the parts → the chunk image (rows r and 16 + r, columns 8g .. 8g + 7)
        *reinterpret_cast<bf16x8*>(img + 0 * kChPlane + ch_off(r, 8 * g)) = h0;
        *reinterpret_cast<bf16x8*>(img + 1 * kChPlane + ch_off(r, 8 * g)) = m0;
        *reinterpret_cast<bf16x8*>(img + 2 * kChPlane + ch_off(r, 8 * g)) = l0;
        *reinterpret_cast<bf16x8*>(img + 0 * kChPlane + ch_off(16 + r, 8 * g)) = h1;
        *reinterpret_cast<bf16x8*>(img + 1 * kChPlane + ch_off(16 + r, 8 * g)) = m1;
        *reinterpret_cast<bf16x8*>(img + 2 * kChPlane + ch_off(16 + r, 8 * g)) = l1;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          bf16x8 xp[3];
#pragma unroll
          for (int pt = 0; pt < 3; ++pt) {
            const int o0 = pt * kChPlane + ch_off(8 * g + q, 16 * tt + 4 * p4);
            const int o1 = pt * kChPlane + ch_off(8 * g + 4 + q, 16 * tt + 4 * p4);
            const shortx4 lo4 =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4*)(img + o0));
            const shortx4 hi4 =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4*)(img + o1));
            const shortx8 v8 = __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7);
            xp[pt] = __builtin_bit_cast(bf16x8, v8);
          }
          floatx4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0;
          d0 = mfma6_xs(xp[0], xp[1], xp[2], sa[0][0], sa[0][1], sa[0][2], d0);
          d1 = mfma6_xs(xp[0], xp[1], xp[2], sa[1][0], sa[1][1], sa[1][2], d1);
          // lane (r, g): U[16 ib + r][32 s + 16 tt + 4g ..+3] → the staging rows (and U's row S,
          // the bottom-MLP row, to ubot)
          const int col = 16 * tt + 4 * g;
          *reinterpret_cast<floatx4*>(stg + r * kChStageLd + col) = d0;
          *reinterpret_cast<floatx4*>(stg + (16 + r) * kChStageLd + col) = d1;
          if (r == S) *reinterpret_cast<floatx4*>(ubot + 32 * s + col) = d0;
          if (16 + r == S) *reinterpret_cast<floatx4*>(ubot + 32 * s + col) = d1;
        }
        __builtin_amdgcn_wave_barrier();
        // the chunk's 128-B row segments to HBM: 8 rows per store, 8 lanes per row (a 64-B
        // segment per row and store measured half the rate: tools/microbench_gather.hip)
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
          const int i = 8 * pp + (lanev >> 3), c8 = lanev & 7;
          const floatx4 v = *reinterpret_cast<const floatx4*>(stg + i * kChStageLd + 4 * c8);
          if (i < S)
            __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(de + i * D + 32 * s + 4 * c8));
        }
        __builtin_amdgcn_wave_barrier();  // the next chunk's image / staging writes follow
      }
      // head, loss, G
      const int cl = lanev & (DL - 1), rg = (lanev / DL) & (RPI - 1);
      float zr[12];
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        zr[reg] = c00[reg];
        zr[4 + reg] = c01[reg];
        zr[8 + reg] = c11[reg];
      }
      float hacc = 0.f;
      {
        const floatx4* ql = reinterpret_cast<const floatx4*>(&qlane[lanev & 63][0]);
#pragma unroll
        for (int q4 = 0; q4 < 3; ++q4) {
          const floatx4 qv = ql[q4];
#pragma unroll
          for (int k = 0; k < 4; ++k) hacc += zr[4 * q4 + k] * qv[k];
        }
        const floatx4 qd = *reinterpret_cast<const floatx4*>(&qsh[nzc + 4 * cl]);
        if (rg == 0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) hacc += dn[k] * qd[k];
        }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) hacc += __shfl_xor(hacc, off);
      const float p = 1.f / (1.f + expf(-(hacc + cc)));
      {
        const float pc = fminf(fmaxf(p, ta.eps), 1.f - ta.eps);
        loss += -(lb * logf(pc + ta.eps) + (1.f - lb) * logf((1.f - pc) + ta.eps));
      }
      const bool inside = p >= ta.eps && p <= 1.f - ta.eps;
      const float pcg = fminf(fmaxf(p, ta.eps), 1.f - ta.eps);
      const float dbce = -(lb / (pcg + ta.eps)) + (1.f - lb) / ((1.f - pcg) + ta.eps);
      const float dp = inside ? ta.gscale * dbce : 0.f;
      const float G = dp * (p * (1.f - p));
      if (lanev == 0) {
        ta.y[b] = p;
        g_rows[b] = G;
      }
      s_top += G;
#pragma unroll
      for (int k = 0; k < 12; ++k) az[k] += zr[k] * G;
#pragma unroll
      for (int k = 0; k < 4; ++k) ad[k] += dn[k] * G;
      {  // the bottom-MLP row from U's row S
        const floatx4 v = *reinterpret_cast<const floatx4*>(ubot + 4 * cl);
        const floatx4 qdn = *reinterpret_cast<const floatx4*>(&qsh[nzc + 4 * cl]);
#pragma unroll
        for (int k = 0; k < DPL; ++k) {
          const int c = DPL * rg + k;
          const float gd = __fmul_rn(G, v[c] + qdn[c]);
          const float gb = dn[c] > 0.f ? gd : 0.f;
          sbot[k] += gb;
#pragma unroll
          for (int ii = 0; ii < kTrainNI; ++ii) abot[k][ii] += xb[ii] * gb;
        }
      }
      __builtin_amdgcn_wave_barrier();  // the next example's ubot writes follow these reads
    }
  }
  // the wave's partial row → its LDS region, then the block folds its four waves in order
  __syncthreads();
  float* X = lds[wave];
  for (int e = lane; e < TM; e += 64) X[e] = 0.f;
  __builtin_amdgcn_wave_barrier();
  if (active) {
    const int cl = lane & (DL - 1), rg = lane / DL;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int i0 = 4 * g + reg, j0 = r, i1 = 4 * g + reg, j1 = 16 + r, i2 = 16 + 4 * g + reg, j2 = 16 + r;
      if (i0 < j0 && j0 < F) X[compact_index(i0, j0, F, 0)] = az[reg];
      if (j1 < F) X[compact_index(i1, j1, F, 0)] = az[4 + reg];
      if (i2 < j2 && j2 < F) X[compact_index(i2, j2, F, 0)] = az[8 + reg];
    }
    if (rg == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) X[nzc + 4 * cl + k] = ad[k];
    }
    if (lane == 0) {
      X[kTrainAtop] = s_top;
      X[kTrainAtop + 1] = loss;
    }
#pragma unroll
    for (int k = 0; k < DPL; ++k) {
      const int d = 4 * cl + DPL * rg + k;
#pragma unroll
      for (int ii = 0; ii < kTrainNI; ++ii) X[kTrainAtop + 2 + ii * D + d] = abot[k][ii];
      X[kTrainAtop + 2 + kTrainNI * D + d] = sbot[k];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < TM; e += 256) {
    float v = lds[0][e];
    v += lds[1][e];
    v += lds[2][e];
    v += lds[3][e];
    ta.part[(int64_t)blockIdx.x * TM + e] = v;
  }
  if (__any(oob) && lane == 0) flag_oob(src.err_flag);
}

// (Round 5 built a three-waves-per-SIMD form of this kernel, RS_TRAIN3: 433-450 us against
// 318-334, profiles/r05_train_kernel_pmc_2wave_vs_3wave.txt; removed in round 6.)

template <int GREG, int KS, bool ID64>
static void launch_pipe_t(const GatherSrc& src, int64_t batch, int F, InterMode md,
                          const float* gout, int64_t gstride, float* gemb, float* gdense, int,
                          hipStream_t st, const float* gscale = nullptr) {
  auto go = [&](auto kern) {
    const int epw = pipe_epw(reinterpret_cast<const void*>(kern), batch);
    kern<<<ceil_div(batch, 4 * (int64_t)epw), 256, 0, st>>>(src, batch, F, gout, gstride, gemb,
                                                           gdense, epw, gscale);
  };
  if (gscale) {  // rank-one upstream gradient: the DLRM layout only (non-self, compact)
    go(dlrm_bwd_pipe<128, GREG, KS, false, false, ID64, true>);
    return;
  }
  if (md.self_interaction) {
    if (md.skip_gather) go(dlrm_bwd_pipe<128, GREG, KS, true, true, ID64>);
    else go(dlrm_bwd_pipe<128, GREG, KS, true, false, ID64>);
  } else {
    if (md.skip_gather) go(dlrm_bwd_pipe<128, GREG, KS, false, true, ID64>);
    else go(dlrm_bwd_pipe<128, GREG, KS, false, false, ID64>);
  }
}

template <int GREG, int KS>
static void launch_pipe(const GatherSrc& src, int64_t batch, int F, InterMode md,
                        const float* gout, int64_t gstride, float* gemb, float* gdense, int epw,
                        hipStream_t st, const float* gscale = nullptr) {
  if (src.id_dtype == RS_ID_I64)
    launch_pipe_t<GREG, KS, true>(src, batch, F, md, gout, gstride, gemb, gdense, epw, st, gscale);
  else
    launch_pipe_t<GREG, KS, false>(src, batch, F, md, gout, gstride, gemb, gdense, epw, st, gscale);
}

// ---------------------------------------------------------------------------------------
// generic (any F, D): one wave per sample, X staged in LDS
// ---------------------------------------------------------------------------------------
template <class Src, bool DLRM_OUT>
__global__ __launch_bounds__(64) void inter_fwd_generic(Src src, int64_t batch, int F, int D,
                                                        InterMode md, float* __restrict__ out,
                                                        int64_t out_stride) {
  extern __shared__ __attribute__((aligned(16))) float xs[];  // [F][D+1]
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int ld = D + 1;
  bool oob = false;
  for (int i = 0; i < F; ++i) {
    const float* xr = src.row(b, i, D, oob);
    for (int d = lane; d < D; d += 64) xs[i * ld + d] = xr ? xr[d] : 0.f;
  }
  __syncthreads();
  float* orow = out + b * out_stride;
  for (int o = lane; o < F * F; o += 64) {
    int i = o / F, j = o - i * F;
    bool keep = keep_pair(i, j, md.self_interaction);
    if (!keep && !md.skip_gather) continue;
    float s = 0.f;
    if (keep)
      for (int d = 0; d < D; ++d) s = fmaf(xs[i * ld + d], xs[j * ld + d], s);
    if (md.skip_gather)
      orow[o] = s;
    else
      orow[compact_index(i, j, F, md.self_interaction)] = s;
  }
  if constexpr (DLRM_OUT) {
    const int nz = out_width(F, md.self_interaction, md.skip_gather);
    float* od = orow + nz;
    for (int d = lane; d < D; d += 64) od[d] = src.dense[b * D + d];
    for (int64_t o = nz + D + lane; o < out_stride; o += 64) orow[o] = 0.f;
    if (__any(oob) && lane == 0) flag_oob(src.err_flag);
  }
}

template <class Src, bool DLRM_OUT>
__global__ __launch_bounds__(64) void inter_bwd_generic(Src src, int64_t batch, int F, int D,
                                                        InterMode md, const float* __restrict__ gout,
                                                        int64_t gstride, float* __restrict__ gx,
                                                        float* __restrict__ gemb,
                                                        float* __restrict__ gdense) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;                 // [F][D+1]
  float* ss = sm + F * (D + 1);   // [F][F+1]
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int ld = D + 1, ls = F + 1;
  bool oob = false;
  const float* grow = gout + b * gstride;
  for (int i = 0; i < F; ++i) {
    const float* xr = src.row(b, i, D, oob);
    for (int d = lane; d < D; d += 64) xs[i * ld + d] = xr ? xr[d] : 0.f;
  }
  for (int o = lane; o < F * F; o += 64) {
    int i = o / F, k = o - i * F;
    float v = 0.f;
    if (keep_pair(i, k, md.self_interaction))
      v += md.skip_gather ? grow[i * F + k] : grow[compact_index(i, k, F, md.self_interaction)];
    if (keep_pair(k, i, md.self_interaction))
      v += md.skip_gather ? grow[k * F + i] : grow[compact_index(k, i, F, md.self_interaction)];
    ss[i * ls + k] = v;
  }
  __syncthreads();
  for (int o = lane; o < F * D; o += 64) {
    int i = o / D, d = o - i * D;
    float s = 0.f;
    for (int k = 0; k < F; ++k) s = fmaf(ss[i * ls + k], xs[k * ld + d], s);
    if constexpr (DLRM_OUT) {
      if (i < src.n_slots) {
        gemb[(b * src.n_slots + i) * (int64_t)D + d] = s;
      } else {
        gdense[b * D + d] = s + grow[out_width(F, md.self_interaction, md.skip_gather) + d];
      }
    } else {
      gx[(b * F + i) * (int64_t)D + d] = s;
    }
  }
}

// ---------------------------------------------------------------------------------------
// FM (DeepFM second order): out[b] = 0.5 * Σ_d (sum_f e)^2 - Σ_f e^2
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fm_fwd_kernel(const float* __restrict__ emb, int64_t batch,
                                                     int F, int D, float* __restrict__ out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  if (b >= batch) return;
  const float* e = emb + b * F * (int64_t)D;
  float part = 0.f;
  for (int d = lane; d < D; d += 64) {
    float s = 0.f, q = 0.f;
    for (int f = 0; f < F; ++f) {
      float x = e[f * D + d];
      s += x;
      q += x * x;
    }
    part += s * s - q;
  }
  for (int off = 32; off > 0; off >>= 1) part += __shfl_down(part, off);
  if (lane == 0) out[b] = 0.5f * part;
}

__global__ __launch_bounds__(256) void fm_bwd_kernel(const float* __restrict__ emb,
                                                     const float* __restrict__ gout, int64_t batch,
                                                     int F, int D, float* __restrict__ gemb) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  if (b >= batch) return;
  const float* e = emb + b * F * (int64_t)D;
  float* ge = gemb + b * F * (int64_t)D;
  const float g = gout[b];
  for (int d = lane; d < D; d += 64) {
    float s = 0.f;
    for (int f = 0; f < F; ++f) s += e[f * D + d];
    // d/de_fd of 0.5*((Σe)^2 - Σe^2) = Σe - e_fd
    for (int f = 0; f < F; ++f) ge[f * D + d] = g * (s - e[f * D + d]);
  }
}

// ---------------------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------------------
template <class Src, bool DLRM_OUT>
static int32_t launch_fwd(const Src& src, int64_t batch, int F, int D, InterMode md, float* out,
                          int64_t out_stride, bool aligned16, hipStream_t st) {
  if (batch == 0) return RS_OK;
  if (F <= 32 && aligned16) {
    int64_t blocks = ceil_div(batch, 4);
    switch (D) {
      case 16: inter_fwd_mfma<16, Src, DLRM_OUT><<<blocks, 256, 0, st>>>(src, batch, F, md, out, out_stride); RS_CHECK_LAUNCH(); return RS_OK;
      case 32: inter_fwd_mfma<32, Src, DLRM_OUT><<<blocks, 256, 0, st>>>(src, batch, F, md, out, out_stride); RS_CHECK_LAUNCH(); return RS_OK;
      case 64: inter_fwd_mfma<64, Src, DLRM_OUT><<<blocks, 256, 0, st>>>(src, batch, F, md, out, out_stride); RS_CHECK_LAUNCH(); return RS_OK;
      case 128: inter_fwd_mfma<128, Src, DLRM_OUT><<<blocks, 256, 0, st>>>(src, batch, F, md, out, out_stride); RS_CHECK_LAUNCH(); return RS_OK;
      case 256: inter_fwd_mfma<256, Src, DLRM_OUT><<<blocks, 256, 0, st>>>(src, batch, F, md, out, out_stride); RS_CHECK_LAUNCH(); return RS_OK;
      default: break;
    }
  }
  size_t lds = (size_t)F * (D + 1) * 4;
  if (lds > 64 * 1024) {
    set_error("interaction F=%d D=%d too large for the generic kernel", F, D);
    return RS_E_UNSUPPORTED;
  }
  inter_fwd_generic<Src, DLRM_OUT><<<batch, 64, lds, st>>>(src, batch, F, D, md, out, out_stride);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

template <class Src, bool DLRM_OUT>
static int32_t launch_bwd(const Src& src, int64_t batch, int F, int D, InterMode md,
                          const float* gout, int64_t gstride, float* gx, float* gemb, float* gdense,
                          bool aligned16, hipStream_t st) {
  if (batch == 0) return RS_OK;
  if constexpr (DLRM_OUT && std::is_same<Src, GatherSrc>::value) {
    const int epw = kPipeEPW;
    const int gw = out_width(F, md.self_interaction, md.skip_gather) + D;
    if (F <= 32 && aligned16 && D == 128 && gw <= 20 * 64) {
      const bool k14 = F <= 28;
      if (gw <= 8 * 64) {
        if (k14) launch_pipe<8, 14>(src, batch, F, md, gout, gstride, gemb, gdense, epw, st);
        else launch_pipe<8, 16>(src, batch, F, md, gout, gstride, gemb, gdense, epw, st);
        RS_CHECK_LAUNCH();
        return RS_OK;
      }
      {
        if (k14) launch_pipe<20, 14>(src, batch, F, md, gout, gstride, gemb, gdense, epw, st);
        else launch_pipe<20, 16>(src, batch, F, md, gout, gstride, gemb, gdense, epw, st);
        RS_CHECK_LAUNCH();
        return RS_OK;
      }
    }
  }
  if (F <= 32 && aligned16) {
    int64_t blocks = ceil_div(batch, 4);
    switch (D) {
      case 32: inter_bwd_mfma<32, Src, DLRM_OUT><<<blocks, 256, 0, st>>>(src, batch, F, md, gout, gstride, gx, gemb, gdense); RS_CHECK_LAUNCH(); return RS_OK;
      case 64: inter_bwd_mfma<64, Src, DLRM_OUT><<<blocks, 256, 0, st>>>(src, batch, F, md, gout, gstride, gx, gemb, gdense); RS_CHECK_LAUNCH(); return RS_OK;
      case 128: inter_bwd_mfma<128, Src, DLRM_OUT><<<blocks, 256, 0, st>>>(src, batch, F, md, gout, gstride, gx, gemb, gdense); RS_CHECK_LAUNCH(); return RS_OK;
      default: break;
    }
  }
  size_t lds = ((size_t)F * (D + 1) + (size_t)F * (F + 1)) * 4;
  if (lds > 64 * 1024) {
    set_error("interaction F=%d D=%d too large for the generic kernel", F, D);
    return RS_E_UNSUPPORTED;
  }
  inter_bwd_generic<Src, DLRM_OUT><<<batch, 64, lds, st>>>(src, batch, F, D, md, gout, gstride, gx,
                                                           gemb, gdense);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_dot_interaction_fwd(const float* x, int64_t batch, int32_t F, int32_t D,
                                          int32_t self_interaction, int32_t skip_gather, float* out,
                                          int64_t out_stride, void* stream) {
  RS_CHECK_ARG(F >= 1 && D >= 1 && batch >= 0, "bad sizes");
  RS_CHECK_ARG(out_stride >= out_width(F, self_interaction, skip_gather), "out_stride too small");
  RS_CHECK_ARG(batch == 0 || (x && out), "null pointer");
  DenseSrc src{x, F};
  return launch_fwd<DenseSrc, false>(src, batch, F, D, {self_interaction, skip_gather}, out,
                                     out_stride, al16(x), as_stream(stream));
}

extern "C" int32_t rs_dot_interaction_bwd(const float* x, const float* grad_out, int64_t batch,
                                          int32_t F, int32_t D, int32_t self_interaction,
                                          int32_t skip_gather, int64_t grad_stride, float* grad_x,
                                          void* stream) {
  RS_CHECK_ARG(F >= 1 && D >= 1 && batch >= 0, "bad sizes");
  RS_CHECK_ARG(grad_stride >= out_width(F, self_interaction, skip_gather), "grad_stride too small");
  RS_CHECK_ARG(batch == 0 || (x && grad_out && grad_x), "null pointer");
  DenseSrc src{x, F};
  return launch_bwd<DenseSrc, false>(src, batch, F, D, {self_interaction, skip_gather}, grad_out,
                                     grad_stride, grad_x, nullptr, nullptr, al16(x) && al16(grad_x),
                                     as_stream(stream));
}

extern "C" int32_t rs_dlrm_interaction_fwd(const float* table, int64_t n_rows, int32_t D,
                                           const void* ids, int32_t id_dtype, int32_t n_slots,
                                           const int64_t* slot_offsets, const float* dense,
                                           int64_t batch, int32_t compact, float* out,
                                           int64_t out_stride, int32_t* err_flag, void* stream) {
  const int F = n_slots + 1;
  const InterMode md{0, compact ? 0 : 1};
  RS_CHECK_ARG(n_slots >= 1 && D >= 1 && batch >= 0, "bad sizes");
  RS_CHECK_ARG(id_dtype == RS_ID_I32 || id_dtype == RS_ID_I64, "bad id dtype");
  RS_CHECK_ARG(out_stride >= out_width(F, 0, md.skip_gather) + D, "out_stride too small");
  RS_CHECK_ARG(batch == 0 || (table && ids && dense && out), "null pointer");
  GatherSrc src{table, n_rows, ids, id_dtype, n_slots, slot_offsets, dense, err_flag};
  return launch_fwd<GatherSrc, true>(src, batch, F, D, md, out, out_stride,
                                     al16(table) && al16(dense), as_stream(stream));
}

extern "C" int32_t rs_dlrm_interaction_bwd(const float* table, int64_t n_rows, int32_t D,
                                           const void* ids, int32_t id_dtype, int32_t n_slots,
                                           const int64_t* slot_offsets, const float* dense,
                                           int64_t batch, int32_t compact, const float* grad_out,
                                           int64_t grad_stride, float* grad_emb, float* grad_dense,
                                           void* stream) {
  const int F = n_slots + 1;
  const InterMode md{0, compact ? 0 : 1};
  RS_CHECK_ARG(n_slots >= 1 && D >= 1 && batch >= 0, "bad sizes");
  RS_CHECK_ARG(grad_stride >= out_width(F, 0, md.skip_gather) + D, "grad_stride too small");
  RS_CHECK_ARG(batch == 0 || (table && ids && dense && grad_out && grad_emb && grad_dense),
               "null pointer");
  GatherSrc src{table, n_rows, ids, id_dtype, n_slots, slot_offsets, dense, nullptr};
  return launch_bwd<GatherSrc, true>(src, batch, F, D, md, grad_out, grad_stride, nullptr,
                                     grad_emb, grad_dense,
                                     al16(table) && al16(dense) && al16(grad_emb) && al16(grad_dense),
                                     as_stream(stream));
}

extern "C" int32_t rs_dlrm_interaction_bwd_rank1(const float* table, int64_t n_rows, int32_t D,
                                                 const void* ids, int32_t id_dtype,
                                                 int32_t n_slots, const int64_t* slot_offsets,
                                                 const float* dense, int64_t batch,
                                                 const float* gscale, const float* grad_row,
                                                 int64_t width, float* grad_emb,
                                                 float* grad_dense, void* stream) {
  const int F = n_slots + 1;
  const InterMode md{0, 0};
  const int gw = out_width(F, 0, 0) + D;
  RS_CHECK_ARG(n_slots >= 1 && D >= 1 && batch >= 0, "bad sizes");
  RS_CHECK_ARG(width >= gw, "width too small");
  if (batch == 0) return RS_OK;
  RS_CHECK_ARG(table && ids && dense && gscale && grad_row && grad_emb && grad_dense,
               "null pointer");
  if (!(F <= 32 && D == 128 && gw <= 20 * 64 && al16(table) && al16(dense) && al16(grad_emb) &&
        al16(grad_dense))) {
    set_error("rs_dlrm_interaction_bwd_rank1: needs D = 128, F <= 32, 16-B aligned buffers");
    return RS_E_UNSUPPORTED;
  }
  GatherSrc src{table, n_rows, ids, id_dtype, n_slots, slot_offsets, dense, nullptr};
  hipStream_t st = as_stream(stream);
  const bool k14 = F <= 28;
  if (gw <= 8 * 64) {
    if (k14) launch_pipe<8, 14>(src, batch, F, md, grad_row, width, grad_emb, grad_dense, 0, st, gscale);
    else launch_pipe<8, 16>(src, batch, F, md, grad_row, width, grad_emb, grad_dense, 0, st, gscale);
  } else {
    if (k14) launch_pipe<20, 14>(src, batch, F, md, grad_row, width, grad_emb, grad_dense, 0, st, gscale);
    else launch_pipe<20, 16>(src, batch, F, md, grad_row, width, grad_emb, grad_dense, 0, st, gscale);
  }
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_fm_fwd(const float* emb, int64_t batch, int32_t F, int32_t D, float* out,
                             void* stream) {
  RS_CHECK_ARG(F >= 1 && D >= 1 && batch >= 0, "bad sizes");
  if (batch == 0) return RS_OK;
  RS_CHECK_ARG(emb && out, "null pointer");
  fm_fwd_kernel<<<ceil_div(batch, 4), 256, 0, as_stream(stream)>>>(emb, batch, F, D, out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_fm_bwd(const float* emb, const float* grad_out, int64_t batch, int32_t F,
                             int32_t D, float* grad_emb, void* stream) {
  RS_CHECK_ARG(F >= 1 && D >= 1 && batch >= 0, "bad sizes");
  if (batch == 0) return RS_OK;
  RS_CHECK_ARG(emb && grad_out && grad_emb, "null pointer");
  fm_bwd_kernel<<<ceil_div(batch, 4), 256, 0, as_stream(stream)>>>(emb, grad_out, batch, F, D,
                                                                   grad_emb);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_dlrm_interaction_fwd_head(const float* table, int64_t n_rows, int32_t D,
                                                const void* ids, int32_t id_dtype,
                                                int32_t n_slots, const int64_t* slot_offsets,
                                                const float* dense, int64_t batch, float* out,
                                                int64_t out_stride, const float* q,
                                                const float* c, int32_t act, float* y,
                                                int32_t* err_flag, void* stream) {
  const int F = n_slots + 1;
  const InterMode md{0, 0};  // compact row
  RS_CHECK_ARG(n_slots >= 1 && F <= 32 && D == 128 && batch >= 0,
               "rs_dlrm_interaction_fwd_head: needs D = 128 and at most 31 slots");
  RS_CHECK_ARG(id_dtype == RS_ID_I32 || id_dtype == RS_ID_I64, "bad id dtype");
  RS_CHECK_ARG(out_stride >= out_width(F, 0, 0) + D, "out_stride too small");
  RS_CHECK_ARG(act >= 0 && act <= 2, "bad activation");
  RS_CHECK_ARG(batch == 0 || (table && ids && dense && out && q && c && y), "null pointer");
  RS_CHECK_ARG(al16(table) && al16(dense), "table and dense must be 16-byte aligned");
  if (batch == 0) return RS_OK;
  GatherSrc src{table, n_rows, ids, id_dtype, n_slots, slot_offsets, dense, err_flag};
  FwdHead hd{q, c, y, act};
  inter_fwd_mfma<128, GatherSrc, true, true>
      <<<ceil_div(batch, 4), 256, 0, as_stream(stream)>>>(src, batch, F, md, out, out_stride, hd);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_dlrm_interaction_fwd_head_dx(const float* table, int64_t n_rows, int32_t D,
                                                   const void* ids, int32_t id_dtype,
                                                   int32_t n_slots, const int64_t* slot_offsets,
                                                   const float* dense, int64_t batch, float* out,
                                                   int64_t out_stride, const float* q,
                                                   const float* c, int32_t act, float* y,
                                                   float* dxu_emb, float* dxu_dense,
                                                   int32_t* err_flag, void* stream) {
  const int F = n_slots + 1;
  const InterMode md{0, 0};  // compact row
  RS_CHECK_ARG(n_slots >= 1 && F <= 32 && D == 128 && batch >= 0,
               "rs_dlrm_interaction_fwd_head_dx: needs D = 128 and at most 31 slots");
  RS_CHECK_ARG(id_dtype == RS_ID_I32 || id_dtype == RS_ID_I64, "bad id dtype");
  RS_CHECK_ARG(out_stride >= out_width(F, 0, 0) + D, "out_stride too small");
  RS_CHECK_ARG(act >= 0 && act <= 2, "bad activation");
  RS_CHECK_ARG(batch == 0 || (table && ids && dense && out && q && c && y && dxu_emb && dxu_dense),
               "null pointer");
  RS_CHECK_ARG(al16(table) && al16(dense), "table and dense must be 16-byte aligned");
  if (batch == 0) return RS_OK;
  GatherSrc src{table, n_rows, ids, id_dtype, n_slots, slot_offsets, dense, err_flag};
  FwdHead hd{q, c, y, act, dxu_emb, dxu_dense};
  hipStream_t st = as_stream(stream);
  if (F <= kDxRows && out_stride > out_width(F, 0, 0) + D &&
      out_stride <= out_width(F, 0, 0) + D + 64) {
    auto go = [&](auto kern) {
      const int epw = pipe_epw(reinterpret_cast<const void*>(kern), batch);
      kern<<<ceil_div(batch, 4 * (int64_t)epw), 256, 0, st>>>(src, batch, F, out, out_stride, hd, epw);
    };
    if (id_dtype == RS_ID_I64) go(dlrm_fwd_dx_pipe<true>);
    else go(dlrm_fwd_dx_pipe<false>);
  } else {
    inter_fwd_mfma<128, GatherSrc, true, true, true>
        <<<ceil_div(batch, 4), 256, 0, st>>>(src, batch, F, md, out, out_stride, hd);
  }
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_dlrm_train_workspace_size(int64_t batch) {
  // one partial row per block (at most ceil(batch / 4) blocks) + the fold's 32 segment rows
  return (size_t)(ceil_div(batch, 4) + 32) * kTrainM * sizeof(float) + 256;
}

// the train kernel's grid for (batch, D): one round of resident blocks (the fold needs it too)
static int64_t train_blocks(int64_t batch, int32_t D, int id_dtype) {
  const void* k = D == 128 ? (id_dtype == RS_ID_I64 ? reinterpret_cast<const void*>(dlrm_train_chunk<128, true>)
                                                    : reinterpret_cast<const void*>(dlrm_train_chunk<128, false>))
                           : (id_dtype == RS_ID_I64 ? reinterpret_cast<const void*>(dlrm_train_chunk<64, true>)
                                                    : reinterpret_cast<const void*>(dlrm_train_chunk<64, false>));
  return ceil_div(batch, 4 * (int64_t)pipe_epw(k, batch, 1));
}

static int32_t train_step_launch(
    const float* table, int64_t n_rows, int32_t D, const void* ids, int32_t id_dtype,
    int32_t n_slots, const int64_t* slot_offsets, const float* dense, const float* xin,
    int32_t n_in, const float* label, int64_t batch, const float* q, const float* c, float eps,
    float loss_scale, float* y, float* grad_emb, float* sums, void* workspace, size_t ws_bytes,
    int32_t* err_flag, void* stream, float* g_rows, bool fold = true) {
  const int F = n_slots + 1;
  RS_CHECK_ARG((D == 128 || D == 64) && n_slots >= 1 && F <= kDxRows && n_in == kTrainNI &&
                   batch >= 1,
               "rs_dlrm_train_step_fwd_unit: needs D = 128 or 64, at most %d slots, %d dense inputs",
               kDxRows - 1, kTrainNI);
  RS_CHECK_ARG(id_dtype == RS_ID_I32 || id_dtype == RS_ID_I64, "bad id dtype");
  RS_CHECK_ARG(loss_scale > 0.f, "loss_scale must be positive");
  RS_CHECK_ARG(table && ids && dense && xin && label && q && c && y && grad_emb && sums && workspace,
               "null pointer");
  RS_CHECK_ARG(al16(table) && al16(dense) && al16(grad_emb), "table, dense and grad rows must be 16-byte aligned");
  RS_CHECK_ARG(ws_bytes >= rs_dlrm_train_workspace_size(batch), "workspace too small");
  hipStream_t st = as_stream(stream);
  GatherSrc src{table, n_rows, ids, id_dtype, n_slots, slot_offsets, dense, err_flag};
  float* part = static_cast<float*>(workspace);
  TrainArgs ta{q, c, label, xin, eps, loss_scale, y, grad_emb, part};
  int64_t blocks = 0;
  auto go = [&](auto kern) {
    // ONE round of resident blocks: the side-stream sort then only fills the resources the
    // kernel leaves free instead of taking CU slots between rounds (A/B on one box: kernel
    // 458 -> 448 us alone, step 0.878 -> 0.848 ms; four rounds 0.912)
    const int epw = pipe_epw(reinterpret_cast<const void*>(kern), batch, 1);
    blocks = ceil_div(batch, 4 * (int64_t)epw);
    kern<<<blocks, 256, 0, st>>>(src, batch, F, ta, g_rows, epw);
  };
  if (D == 128) {
    if (id_dtype == RS_ID_I64) go(dlrm_train_chunk<128, true>);
    else go(dlrm_train_chunk<128, false>);
  } else {
    if (id_dtype == RS_ID_I64) go(dlrm_train_chunk<64, true>);
    else go(dlrm_train_chunk<64, false>);
  }
  RS_CHECK_LAUNCH();
  if (!fold) return RS_OK;
  const int tm = D == 128 ? train_m<128>() : train_m<64>();
  return fold_two_level(part, (int)blocks, tm, part + (size_t)blocks * tm, sums, st);
}

extern "C" int32_t rs_dlrm_train_step_fwd_unit(
    const float* table, int64_t n_rows, int32_t D, const void* ids, int32_t id_dtype,
    int32_t n_slots, const int64_t* slot_offsets, const float* dense, const float* xin,
    int32_t n_in, const float* label, int64_t batch, const float* q, const float* c, float eps,
    float loss_scale, float* y, float* unit_rows, float* g_rows, float* sums, void* workspace,
    size_t ws_bytes, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(g_rows, "null pointer");
  return train_step_launch(table, n_rows, D, ids, id_dtype, n_slots, slot_offsets, dense, xin,
                           n_in, label, batch, q, c, eps, loss_scale, y, unit_rows, sums,
                           workspace, ws_bytes, err_flag, stream, g_rows);
}

// The same step as two calls: the kernel alone (its per-block partial rows left in the workspace),
// then rs_dlrm_train_fold for the batch sums. The gradient rows, G and y are final after the
// first call, so the sparse update can be ordered after the kernel alone (not after the fold too).
extern "C" int32_t rs_dlrm_train_step_fwd_unit_nofold(
    const float* table, int64_t n_rows, int32_t D, const void* ids, int32_t id_dtype,
    int32_t n_slots, const int64_t* slot_offsets, const float* dense, const float* xin,
    int32_t n_in, const float* label, int64_t batch, const float* q, const float* c, float eps,
    float loss_scale, float* y, float* unit_rows, float* g_rows, void* workspace,
    size_t ws_bytes, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(g_rows, "null pointer");
  float dummy_sums[1];
  return train_step_launch(table, n_rows, D, ids, id_dtype, n_slots, slot_offsets, dense, xin,
                           n_in, label, batch, q, c, eps, loss_scale, y, unit_rows, dummy_sums,
                           workspace, ws_bytes, err_flag, stream, g_rows, false);
}

extern "C" int32_t rs_dlrm_train_fold(const void* workspace, size_t ws_bytes, int64_t batch,
                                      int32_t D, int32_t id_dtype, float* sums, void* stream) {
  RS_CHECK_ARG((D == 128 || D == 64) && batch >= 1, "rs_dlrm_train_fold: D = 128 or 64, batch >= 1");
  RS_CHECK_ARG(id_dtype == RS_ID_I32 || id_dtype == RS_ID_I64, "bad id dtype");
  RS_CHECK_ARG(workspace && sums, "null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_dlrm_train_workspace_size(batch), "workspace too small");
  const int64_t blocks = train_blocks(batch, D, id_dtype);
  const int tm = D == 128 ? train_m<128>() : train_m<64>();
  float* part = static_cast<float*>(const_cast<void*>(workspace));
  return fold_two_level(part, (int)blocks, tm, part + (size_t)blocks * tm, sums, as_stream(stream));
}
