// dien.hip — DIEN interest extraction / evolution recurrences (a-9..a-11):
//   GRU      keras.layers.GRU(units, return_sequences=True) [3p TF 2.2, reset_after=True]
//            (InterestExtract, dien/layers.py:79,131), masked steps carry the state;
//   AUGRU    AUGRUCell under keras.layers.RNN (dien/layers.py:161-204): u = a·σ(·), opposite
//            update convention to the GRU, masked steps carry the state, output = last state;
//   ATTN     DIENAttention (dien/layers.py:145-158): softmax_L(h_t·(K t) + (1-m_t)(-1e9)).
// Design (MI355X): the recurrence is latency-bound (100 dependent steps, [B,H]x[H,3H] per step),
// so one wave owns one example for the whole sequence: lane j < H keeps unit j's state and the
// j-th column (fwd) or row (bwd) of every recurrent weight in VGPRs, and the state vector is
// broadcast by v_readlane (scalar operand of the FMA) — no LDS, no barriers, no per-step launch.
// The input projections x·W (+bias) of all steps and all weight gradients are plain GEMMs done
// by the caller (hipBLASLt); the kernels only do what is inherently sequential.
#include "common.hpp"

namespace rs {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
// two gates' recurrent sums as one packed pair: v_pk_fma_f32 does both fused multiply-adds in one
// instruction (each element rounded once, as two fmaf)
typedef float pk2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pk2 pk_fma(float a, pk2 b, pk2 c) {
  return __builtin_elementwise_fma(pk2{a, a}, b, c);
}
__device__ __forceinline__ float bcast(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

// One gate's recurrent weights in LDS (w(k, j) for lane j, row k; 0 outside H x H) instead of
// VGPRs: with two gates' columns in registers the kernels fit 4 waves per SIMD (<= 128 VGPRs),
// so the whole batch's waves are resident in one round (at 3 waves per SIMD, B = 4096 examples
// took 1.33 rounds: the last third of the waves ran a second full recurrence behind the rest).
// Called by every thread of the block before any wave returns.
template <int HM, class F>
__device__ __forceinline__ void stage_gate(float* ws, int H, F w) {
  for (int e = threadIdx.x; e < HM * 64; e += blockDim.x) {
    const int k = e >> 6, jj = e & 63;
    ws[e] = (k < H && jj < H) ? w(k, jj) : 0.f;
  }
  __syncthreads();
}

// An example's mask row as wave-uniform bit words (L <= 256); longer rows read the byte.
struct MaskBits {
  uint64_t w[4];
  int L;
  __device__ __forceinline__ MaskBits(const uint8_t* mb, int L_, int lane) : L(L_) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int t = 64 * q + lane;
      w[q] = __ballot(t < L && t < 256 && mb[t] != 0);
    }
  }
  __device__ __forceinline__ bool test(const uint8_t* mb, int t) const {
    return t < 256 ? ((w[t >> 6] >> (t & 63)) & 1ull) != 0 : mb[t] != 0;
  }
};

// ---------------------------------------------------------------------------------------
// GRU (Keras reset_after): xw[b,t] = [x_z, x_r, x_h] = x·W + b_in (caller),
// inner = h·U + rb; z = σ(x_z+inner_z); r = σ(x_r+inner_r); hh = tanh(x_h + r·inner_h);
// h = z·h_prev + (1-z)·hh.  saved[b,t] = [z, r, hh, inner_h].
// ---------------------------------------------------------------------------------------
template <int HM>
__global__ __launch_bounds__(256) void gru_fwd_kernel(const float* __restrict__ xw,
                                                      const float* __restrict__ U,
                                                      const float* __restrict__ rb,
                                                      const uint8_t* __restrict__ mask, int64_t B,
                                                      int L, int H, float* __restrict__ out,
                                                      float* __restrict__ saved) {
  const int wave = threadIdx.x >> 6, j = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  const int H3 = 3 * H;
  __shared__ float uh_s[HM * 64];
  stage_gate<HM>(uh_s, H, [&](int k, int jj) { return U[k * H3 + 2 * H + jj]; });
  if (b >= B) return;
  const bool act = j < H;
  pk2 uzr[HM];  // (update, reset) recurrent weights of unit j
#pragma unroll
  for (int k = 0; k < HM; ++k) {
    const bool ok = act && k < H;
    uzr[k] = pk2{ok ? U[k * H3 + j] : 0.f, ok ? U[k * H3 + H + j] : 0.f};
  }
  const float rbz = act ? rb[j] : 0.f, rbr = act ? rb[H + j] : 0.f, rbh = act ? rb[2 * H + j] : 0.f;
  const float* xb = xw + b * (int64_t)L * H3;
  const uint8_t* mb = mask + b * L;
  // the mask row as wave-uniform bits: a step's branch waits on no load (a per-step mask load
  // put one memory latency on every one of the L steps, masked or not)
  const MaskBits mbits(mb, L, j);
  float h = 0.f;
  const bool v0 = mbits.test(mb, 0);
  float nz = act && v0 ? xb[j] : 0.f, nr = act && v0 ? xb[H + j] : 0.f,
        nh = act && v0 ? xb[2 * H + j] : 0.f;
  for (int t = 0; t < L; ++t) {
    const float xz = nz, xr = nr, xh = nh;
    if (t + 1 < L && act && mbits.test(mb, t + 1)) {  // prefetch the next valid step's x·W
      const float* xn = xb + (int64_t)(t + 1) * H3;
      nz = xn[j];
      nr = xn[H + j];
      nh = xn[2 * H + j];
    }
    if (!mbits.test(mb, t)) {
      // masked step (wave-uniform: one example per wave): the state is carried, so the step's
      // arithmetic is skipped — its result would be discarded; the backward never reads its
      // saved row (post-padded histories make most of the L steps such steps)
      if (act) out[(b * L + t) * H + j] = h;
      continue;
    }
    pk2 izr = pk2{0.f, 0.f};
    float ih = 0.f;
#pragma unroll
    for (int k = 0; k < HM; ++k) {
      const float hk = bcast(h, k);
      izr = pk_fma(hk, uzr[k], izr);
      ih = fmaf(hk, uh_s[k * 64 + j], ih);
    }
    float iz = izr.x, ir = izr.y;
    iz += rbz;
    ir += rbr;
    ih += rbh;
    const float z = sigm(xz + iz), r = sigm(xr + ir);
    const float hh = tanhf(xh + r * ih);
    const float hn = z * h + (1.f - z) * hh;
    h = act ? hn : 0.f;
    if (act) {
      const int64_t o = b * L + t;
      out[o * H + j] = h;
      if (saved) {
        float* s = saved + o * 4 * H;
        s[j] = z;
        s[H + j] = r;
        s[2 * H + j] = hh;
        s[3 * H + j] = ih;
      }
    }
  }
}

// dout[b,t] = dL/dh_t (every step); writes dxw = [dpre_z, dpre_r, dpre_h] (grad of x·W + b_in)
// and dinner = [dpre_z, dpre_r, r·dpre_h] (grad of h·U + rb); dU / dW / biases are GEMMs.
template <int HM>
__global__ __launch_bounds__(256) void gru_bwd_kernel(const float* __restrict__ dout,
                                                      const float* __restrict__ out,
                                                      const float* __restrict__ saved,
                                                      const float* __restrict__ U,
                                                      const uint8_t* __restrict__ mask, int64_t B,
                                                      int L, int H, float* __restrict__ dxw,
                                                      float* __restrict__ dinner, bool zero_masked) {
  const int wave = threadIdx.x >> 6, j = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  const int H3 = 3 * H;
  __shared__ float wh_s[HM * 64];
  stage_gate<HM>(wh_s, H, [&](int k, int jj) { return U[jj * H3 + 2 * H + k]; });
  if (b >= B) return;
  const bool act = j < H;
  pk2 wzr[HM];  // row j of U: (U[j][k], U[j][H + k])
#pragma unroll
  for (int k = 0; k < HM; ++k) {
    const bool ok = act && k < H;
    wzr[k] = pk2{ok ? U[j * H3 + k] : 0.f, ok ? U[j * H3 + H + k] : 0.f};
  }
  const uint8_t* mb = mask + b * L;
  const MaskBits mbits(mb, L, j);
  float dh = 0.f;
  // step t's operands are loaded one step ahead (t-1's loads are in flight while t computes);
  // the mask lives in registers (one ballot per 64 steps)
  float nd = 0.f, nz = 0.f, nr = 0.f, nhh = 0.f, nih = 0.f, nhp = 0.f;
  auto fetch = [&](int t) {
    const int64_t o = b * L + t;
    if (act) nd = dout[o * H + j];
    if (act && mbits.test(mb, t)) {
      const float* s = saved + o * 4 * H;
      nz = s[j];
      nr = s[H + j];
      nhh = s[2 * H + j];
      nih = s[3 * H + j];
      nhp = t > 0 ? out[(o - 1) * H + j] : 0.f;
    }
  };
  fetch(L - 1);
  for (int t = L - 1; t >= 0; --t) {
    const int64_t o = b * L + t;
    const float dcur = nd, z = nz, r = nr, hh = nhh, ih = nih, hp = nhp;
    const bool valid = mbits.test(mb, t);
    if (t > 0) fetch(t - 1);
    if (act) dh += dcur;
    float* dx = dxw + o * H3;
    float* di = dinner + o * H3;
    if (!valid) {  // state carried: the gradient passes through unchanged
      if (act && zero_masked) {
        dx[j] = dx[H + j] = dx[2 * H + j] = 0.f;
        di[j] = di[H + j] = di[2 * H + j] = 0.f;
      }
      continue;
    }
    const float dz = dh * (hp - hh);
    const float dph = dh * (1.f - z) * (1.f - hh * hh);
    const float dih = dph * r;
    const float dr = dph * ih;
    const float dpz = act ? dz * z * (1.f - z) : 0.f;
    const float dpr = act ? dr * r * (1.f - r) : 0.f;
    const float dihm = act ? dih : 0.f;
    if (act) {
      dx[j] = dpz;
      dx[H + j] = dpr;
      dx[2 * H + j] = dph;
      di[j] = dpz;
      di[H + j] = dpr;
      di[2 * H + j] = dih;
    }
    // three independent 36-deep chains (update / reset gates as one packed pair, candidate)
    // summed at the end, instead of one 108-deep chain: the step's latency in the tail of long
    // histories, where few waves are left to hide it
    pk2 azr = pk2{0.f, 0.f};
    float ahh = 0.f;
#pragma unroll
    for (int k = 0; k < HM; ++k) {
      azr = __builtin_elementwise_fma(pk2{bcast(dpz, k), bcast(dpr, k)}, wzr[k], azr);
      ahh = fmaf(bcast(dihm, k), wh_s[k * 64 + j], ahh);
    }
    const float acc = dh * z + ((azr.x + azr.y) + ahh);
    dh = act ? acc : 0.f;
  }
}

// ---------------------------------------------------------------------------------------
// AUGRU: xw[b,t] = [x·Ku_x + bu, x·Kr_x + br, x·Kh_x + bh]; Kuh/Krh = the h rows of the update
// and reset kernels ([prev, x] concat order), Khr = the r·h rows of the candidate kernel
// ([x, r·h] order). u = σ(xu + h·Kuh), r = σ(xr + h·Krh), hh = tanh(xh + (r⊙h)·Khr),
// u' = a_t·u, h = u'·hh + (1-u')·h_prev. saved[b,t] = [u, r, hh, r⊙h_prev].
// ---------------------------------------------------------------------------------------
template <int HM>
__global__ __launch_bounds__(256) void augru_fwd_kernel(const float* __restrict__ xw,
                                                        const float* __restrict__ att,
                                                        const float* __restrict__ Kuh,
                                                        const float* __restrict__ Krh,
                                                        const float* __restrict__ Khr,
                                                        const uint8_t* __restrict__ mask, int64_t B,
                                                        int L, int H, float* __restrict__ final_h,
                                                        float* __restrict__ states,
                                                        float* __restrict__ saved, bool zero_masked) {
  const int wave = threadIdx.x >> 6, j = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  __shared__ float kh_s[HM * 64];
  stage_gate<HM>(kh_s, H, [&](int k, int jj) { return Khr[k * H + jj]; });
  if (b >= B) return;
  const bool act = j < H;
  const int H3 = 3 * H;
  float ku[HM], kr[HM];
#pragma unroll
  for (int k = 0; k < HM; ++k) {
    const bool ok = act && k < H;
    ku[k] = ok ? Kuh[k * H + j] : 0.f;
    kr[k] = ok ? Krh[k * H + j] : 0.f;
  }
  const float* xb = xw + b * (int64_t)L * H3;
  const uint8_t* mb = mask + b * L;
  const float* ab = att + b * L;
  float h = 0.f;
  for (int t = 0; t < L; ++t) {
    if (!mb[t]) {  // masked step: state carried, arithmetic skipped (as in gru_fwd_kernel)
      if (act) {
        const int64_t o = b * L + t;
        if (states) states[o * H + j] = h;
        // r⊙h_prev feeds the caller's candidate-kernel gradient GEMM, whose dxw row is 0 here:
        // a defined 0 keeps that product exactly 0
        if (saved && zero_masked) saved[o * 4 * H + 3 * H + j] = 0.f;
      }
      continue;
    }
    const float* x = xb + (int64_t)t * H3;
    const float xu = act ? x[j] : 0.f, xr = act ? x[H + j] : 0.f, xh = act ? x[2 * H + j] : 0.f;
    const float a = ab[t];
    float iu = 0.f, ir = 0.f;
#pragma unroll
    for (int k = 0; k < HM; ++k) {
      const float hk = bcast(h, k);
      iu = fmaf(hk, ku[k], iu);
      ir = fmaf(hk, kr[k], ir);
    }
    const float u = sigm(xu + iu), r = sigm(xr + ir);
    const float rh = act ? r * h : 0.f;
    float ihh = 0.f;
#pragma unroll
    for (int k = 0; k < HM; ++k) ihh = fmaf(bcast(rh, k), kh_s[k * 64 + j], ihh);
    const float hh = tanhf(xh + ihh);
    const float ua = u * a;
    const float hn = ua * hh + (1.f - ua) * h;
    h = act ? hn : 0.f;
    if (act) {
      const int64_t o = b * L + t;
      if (states) states[o * H + j] = h;
      if (saved) {
        float* s = saved + o * 4 * H;
        s[j] = u;
        s[H + j] = r;
        s[2 * H + j] = hh;
        s[3 * H + j] = rh;
      }
    }
  }
  if (act) final_h[b * H + j] = h;
}

// dfinal[b] = dL/d(last state); writes dxw = [dpre_u, dpre_r, dpre_hh] and datt[b,t].
template <int HM>
__global__ __launch_bounds__(256) void augru_bwd_kernel(const float* __restrict__ dfinal,
                                                        const float* __restrict__ att,
                                                        const float* __restrict__ states,
                                                        const float* __restrict__ saved,
                                                        const float* __restrict__ Kuh,
                                                        const float* __restrict__ Krh,
                                                        const float* __restrict__ Khr,
                                                        const uint8_t* __restrict__ mask, int64_t B,
                                                        int L, int H, float* __restrict__ dxw,
                                                        float* __restrict__ datt, bool zero_masked) {
  const int wave = threadIdx.x >> 6, j = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  __shared__ float kh_s[HM * 64];
  stage_gate<HM>(kh_s, H, [&](int k, int jj) { return Khr[jj * H + k]; });
  if (b >= B) return;
  const bool act = j < H;
  const int H3 = 3 * H;
  pk2 kur[HM];  // rows j: (Kuh[j][k], Krh[j][k])
#pragma unroll
  for (int k = 0; k < HM; ++k) {
    const bool ok = act && k < H;
    kur[k] = pk2{ok ? Kuh[j * H + k] : 0.f, ok ? Krh[j * H + k] : 0.f};
  }
  const uint8_t* mb = mask + b * L;
  const MaskBits mbits(mb, L, j);
  const float* ab = att + b * L;
  float dh = act ? dfinal[b * H + j] : 0.f;
  // the next valid step's operands are loaded while the current one computes
  float nu = 0.f, nr = 0.f, nhh = 0.f, nhp = 0.f, na = 0.f;
  auto fetch = [&](int t) {
    if (!mbits.test(mb, t)) return;
    const int64_t o = b * L + t;
    na = ab[t];
    if (act) {
      const float* s = saved + o * 4 * H;
      nu = s[j];
      nr = s[H + j];
      nhh = s[2 * H + j];
      nhp = t > 0 ? states[(o - 1) * H + j] : 0.f;
    }
  };
  fetch(L - 1);
  for (int t = L - 1; t >= 0; --t) {
    const int64_t o = b * L + t;
    float* dx = dxw + o * H3;
    if (!mbits.test(mb, t)) {
      if (act && zero_masked) dx[j] = dx[H + j] = dx[2 * H + j] = 0.f;
      if (j == 0) datt[o] = 0.f;
      if (t > 0) fetch(t - 1);
      continue;
    }
    const float u = nu, r = nr, hh = nhh, hp = nhp, a = na;
    if (t > 0) fetch(t - 1);
    const float ua = u * a;
    const float dua = dh * (hh - hp);
    float dhp = dh * (1.f - ua);
    // attention-score gradient: Σ_j dua_j · u_j
    float ds = act ? dua * u : 0.f;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ds += __shfl_xor(ds, off);
    if (j == 0) datt[o] = ds;
    const float dpu = act ? dua * a * u * (1.f - u) : 0.f;
    const float dph = act ? dh * ua * (1.f - hh * hh) : 0.f;
    float drh = 0.f;
#pragma unroll
    for (int k = 0; k < HM; ++k) drh = fmaf(bcast(dph, k), kh_s[k * 64 + j], drh);
    const float dr = drh * hp;
    dhp = fmaf(drh, r, dhp);
    const float dpr = act ? dr * r * (1.f - r) : 0.f;
    // update / reset contributions as one packed pair of 36-deep chains (not one 72-deep chain)
    pk2 aur = pk2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < HM; ++k)
      aur = __builtin_elementwise_fma(pk2{bcast(dpu, k), bcast(dpr, k)}, kur[k], aur);
    dhp = dhp + (aur.x + aur.y);
    if (act) {
      dx[j] = dpu;
      dx[H + j] = dpr;
      dx[2 * H + j] = dph;
    }
    dh = act ? dhp : 0.f;
  }
}

// ---------------------------------------------------------------------------------------
// DIENAttention: s_t = h_t·q + (1-m_t)(-1e9), q = K·target (caller); a = softmax over t.
// One wave per example, lanes over time steps.
// ---------------------------------------------------------------------------------------
constexpr int kAttMaxT = 4;  // L <= 256

// One wave (one block) per example: the example's [L, H] block of hidden states is contiguous,
// so it is staged into LDS with coalesced loads (row stride H+1: conflict-free row reads), then
// lane t computes s_t from LDS. (Lanes walking their own 4H-byte row straight from HBM made
// every load instruction touch 64 rows: 85% of wave cycles waiting on memory.)
__global__ __launch_bounds__(64) void att_fwd_kernel(const float* __restrict__ hs,
                                                     const float* __restrict__ q,
                                                     const uint8_t* __restrict__ mask, int64_t B,
                                                     int L, int H, float* __restrict__ a) {
  extern __shared__ float hsm[];  // [L][H + 1]
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int ld = H + 1;
  const float* hb = hs + b * (int64_t)L * H;
  const int n = L * H;
  for (int o = lane; o < n; o += 64) {
    const int t = o / H, i = o - t * H;
    hsm[t * ld + i] = hb[o];
  }
  __syncthreads();
  const float* qb = q + b * H;  // uniform loads: every lane reads the same q_i
  float s[kAttMaxT];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < kAttMaxT; ++c) {
    const int t = lane + 64 * c;
    s[c] = -INFINITY;
    if (t < L) {
      const float* hr = hsm + t * ld;
      float acc = 0.f;
      for (int i = 0; i < H; ++i) acc = fmaf(hr[i], qb[i], acc);
      const float m = mask[b * L + t] ? 1.f : 0.f;
      acc = acc + (1.f - m) * -1e9f;
      s[c] = acc;
      mx = fmaxf(mx, acc);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < kAttMaxT; ++c) {
    const int t = lane + 64 * c;
    s[c] = t < L ? expf(s[c] - mx) : 0.f;
    sum += s[c];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
#pragma unroll
  for (int c = 0; c < kAttMaxT; ++c) {
    const int t = lane + 64 * c;
    if (t < L) a[b * L + t] = s[c] / sum;
  }
}

// ds_t = a_t (da_t - Σ a·da); dhs[b,t,:] = ds_t·q (written, not accumulated); dq = Σ_t ds_t h_t
__global__ __launch_bounds__(256) void att_bwd_kernel(const float* __restrict__ hs,
                                                      const float* __restrict__ q,
                                                      const float* __restrict__ a,
                                                      const float* __restrict__ da, int64_t B, int L,
                                                      int H, float* __restrict__ dhs,
                                                      float* __restrict__ dq) {
  __shared__ float dsm[4][64 * kAttMaxT];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  if (b >= B) return;
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < kAttMaxT; ++c) {
    const int t = lane + 64 * c;
    if (t < L) dot += a[b * L + t] * da[b * L + t];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dot += __shfl_xor(dot, off);
#pragma unroll
  for (int c = 0; c < kAttMaxT; ++c) {
    const int t = lane + 64 * c;
    if (t < L) dsm[wave][t] = a[b * L + t] * (da[b * L + t] - dot);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  // lane i < H: dq_i = Σ_t ds_t h_{t,i}; dhs rows: lane i writes column i of every step
  const float qi = lane < H ? q[b * H + lane] : 0.f;
  float acc = 0.f;
  for (int t = 0; t < L; ++t) {
    const float ds = dsm[wave][t];
    if (lane < H) {
      const int64_t o = (b * L + t) * (int64_t)H + lane;
      acc = fmaf(ds, hs[o], acc);
      dhs[o] = ds * qi;
    }
  }
  if (lane < H) dq[b * H + lane] = acc;
}

static int hm_for(int H) {
  if (H <= 8) return 8;
  if (H <= 16) return 16;
  if (H <= 24) return 24;
  if (H <= 32) return 32;
  if (H <= 36) return 36;
  if (H <= 40) return 40;
  if (H <= 48) return 48;
  if (H <= 64) return 64;
  return 0;
}

#define RS_HM_DISPATCH(H, CALL)                                       \
  switch (hm_for(H)) {                                                \
    case 8: { constexpr int HM = 8; CALL; } break;                   \
    case 16: { constexpr int HM = 16; CALL; } break;                 \
    case 24: { constexpr int HM = 24; CALL; } break;                 \
    case 32: { constexpr int HM = 32; CALL; } break;                 \
    case 36: { constexpr int HM = 36; CALL; } break;                 \
    case 40: { constexpr int HM = 40; CALL; } break;                 \
    case 48: { constexpr int HM = 48; CALL; } break;                 \
    case 64: { constexpr int HM = 64; CALL; } break;                 \
    default: set_error("recurrent units %d > 64 unsupported", H); return RS_E_UNSUPPORTED; \
  }

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_gru_fwd(const float* xw, const float* U, const float* rb, const uint8_t* mask,
                              int64_t B, int32_t L, int32_t H, float* out, float* saved,
                              void* stream) {
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1, "bad sizes");
  if (B == 0) return RS_OK;
  RS_CHECK_ARG(xw && U && rb && mask && out, "null pointer");
  hipStream_t st = as_stream(stream);
  RS_HM_DISPATCH(H, ({ gru_fwd_kernel<HM><<<ceil_div(B, 4), 256, 0, st>>>(xw, U, rb, mask, B, L, H, out, saved); }));
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_gru_bwd(const float* dout, const float* out, const float* saved, const float* U,
                              const uint8_t* mask, int64_t B, int32_t L, int32_t H, float* dxw,
                              float* dinner, int32_t flags, void* stream) {
  const bool zm = !(flags & RS_DIEN_SKIP_MASKED_ROWS);
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1, "bad sizes");
  if (B == 0) return RS_OK;
  RS_CHECK_ARG(dout && out && saved && U && mask && dxw && dinner, "null pointer");
  hipStream_t st = as_stream(stream);
  RS_HM_DISPATCH(H, ({ gru_bwd_kernel<HM><<<ceil_div(B, 4), 256, 0, st>>>(dout, out, saved, U, mask, B, L, H, dxw, dinner, zm); }));
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_augru_fwd(const float* xw, const float* att, const float* Kuh, const float* Krh,
                                const float* Khr, const uint8_t* mask, int64_t B, int32_t L,
                                int32_t H, float* final_h, float* states, float* saved,
                                int32_t flags, void* stream) {
  const bool zm = !(flags & RS_DIEN_SKIP_MASKED_ROWS);
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1, "bad sizes");
  if (B == 0) return RS_OK;
  RS_CHECK_ARG(xw && att && Kuh && Krh && Khr && mask && final_h, "null pointer");
  hipStream_t st = as_stream(stream);
  RS_HM_DISPATCH(H, ({ augru_fwd_kernel<HM><<<ceil_div(B, 4), 256, 0, st>>>(xw, att, Kuh, Krh, Khr, mask, B, L, H, final_h, states, saved, zm); }));
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_augru_bwd(const float* dfinal, const float* att, const float* states,
                                const float* saved, const float* Kuh, const float* Krh,
                                const float* Khr, const uint8_t* mask, int64_t B, int32_t L,
                                int32_t H, float* dxw, float* datt, int32_t flags, void* stream) {
  const bool zm = !(flags & RS_DIEN_SKIP_MASKED_ROWS);
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1, "bad sizes");
  if (B == 0) return RS_OK;
  RS_CHECK_ARG(dfinal && att && states && saved && Kuh && Krh && Khr && mask && dxw && datt,
               "null pointer");
  hipStream_t st = as_stream(stream);
  RS_HM_DISPATCH(H, ({ augru_bwd_kernel<HM><<<ceil_div(B, 4), 256, 0, st>>>(dfinal, att, states, saved, Kuh, Krh, Khr, mask, B, L, H, dxw, datt, zm); }));
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_dien_attention_fwd(const float* hs, const float* q, const uint8_t* mask,
                                         int64_t B, int32_t L, int32_t H, float* a, void* stream) {
  RS_CHECK_ARG(B >= 0 && L >= 1 && L <= 64 * kAttMaxT && H >= 1 && H <= 64, "bad sizes");
  if (B == 0) return RS_OK;
  RS_CHECK_ARG(hs && q && mask && a, "null pointer");
  const size_t lds = (size_t)L * (H + 1) * sizeof(float);
  if (lds > 64 * 1024)
    RS_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(att_fwd_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  att_fwd_kernel<<<(unsigned)B, 64, lds, as_stream(stream)>>>(hs, q, mask, B, L, H, a);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_dien_attention_bwd(const float* hs, const float* q, const float* a,
                                         const float* da, int64_t B, int32_t L, int32_t H,
                                         float* dhs, float* dq, void* stream) {
  RS_CHECK_ARG(B >= 0 && L >= 1 && L <= 64 * kAttMaxT && H >= 1 && H <= 64, "bad sizes");
  if (B == 0) return RS_OK;
  RS_CHECK_ARG(hs && q && a && da && dhs && dq, "null pointer");
  att_bwd_kernel<<<ceil_div(B, 4), 256, 0, as_stream(stream)>>>(hs, q, a, da, B, L, H, dhs, dq);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
