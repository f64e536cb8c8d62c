// dien_proj.hip — the B·L-row products around the DIEN recurrences (a-9 / a-11),
// restricted to the steps that exist. With post-padded histories (cfg3: lengths 2 + Geometric,
// clipped to L = 100) ≈ 1 step in 8 is valid; a masked step carries the recurrent state, so its
// input projection is never read and its gradient rows are exactly 0. The library GEMMs these
// replace ran over all B·L rows (x·W + b, dxw·Wᵀ, xᵀ·dxw and the bias column sums: ≈1 ms of the
// 3.45 ms cfg3 step); here every kernel reads and writes only the valid rows (the dx kernel also
// writes the masked rows' zeros its consumers expect).
//   rs_valid_rows    the valid rows of a [R] mask, in order (two launches, graph-safe: the count
//                    stays on the device and sizes nothing on the host);
//   rs_masked_proj   y = x·W + b on those rows — one wave per 16 rows, lane = output column, W's
//                    column in VGPRs, x broadcast by v_readlane;
//   rs_masked_dx     dx = d·Wᵀ on every row (0 on masked ones) — lane = output column, W's row in
//                    VGPRs, the d rows staged through the wave's LDS and read as broadcasts;
//   rs_masked_wgrad  C = Σ_valid A_rᵀ·D_r (+ the column sums of D) — fixed row chunks per block,
//                    rows staged in LDS, per-block partials folded in block order (deterministic).
// The products are tiny next to their traffic (K = 36, N = 108): HBM-bound work, kept on VALU.
#include "common.hpp"

namespace rs {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kVrTile = 4096;  // mask rows per block of the valid-row list

__global__ __launch_bounds__(256) void vr_count_kernel(const uint8_t* __restrict__ mask, int64_t R,
                                                       int32_t* __restrict__ blk) {
  __shared__ int32_t red[4];
  const int64_t base = (int64_t)blockIdx.x * kVrTile;
  int c = 0;
  for (int i = threadIdx.x; i < kVrTile; i += 256) {
    const int64_t r = base + i;
    c += (r < R && mask[r]) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) blk[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// wave w of a block lists rows base + 1024 w .. + 1023 in 64-row chunks (ballot order = row order)
__global__ __launch_bounds__(256) void vr_write_kernel(const uint8_t* __restrict__ mask, int64_t R,
                                                       const int32_t* __restrict__ blk,
                                                       int32_t* __restrict__ idx,
                                                       int32_t* __restrict__ count) {
  __shared__ int32_t off_s;
  __shared__ int32_t wsum[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave == 0) {
    int s = 0;
    for (int i = lane; i < (int)blockIdx.x; i += 64) s += blk[i];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
    if (lane == 0) off_s = s;
  }
  const int64_t base = (int64_t)blockIdx.x * kVrTile + (int64_t)wave * 1024;
  int wc = 0;
  for (int ch = 0; ch < 16; ++ch) {
    const int64_t r = base + ch * 64 + lane;
    wc += __popcll(__ballot(r < R && mask[r]));
  }
  if (lane == 0) wsum[wave] = wc;
  __syncthreads();
  int o = off_s;
  for (int w = 0; w < wave; ++w) o += wsum[w];
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int ch = 0; ch < 16; ++ch) {
    const int64_t r = base + ch * 64 + lane;
    const bool v = r < R && mask[r];
    const uint64_t m = __ballot(v);
    if (v) idx[o + __popcll(m & lt)] = static_cast<int32_t>(r);
    o += __popcll(m);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
    *count = off_s + wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__device__ __forceinline__ float rdlane(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

// y[r, n] = b[n] + Σ_k x[r, k]·W[k, n] for the listed rows; K <= KM <= 64, N <= 64·NB.
// One wave per 32 listed rows (the grid is sized for the capacity R; waves past the count leave
// before loading anything): W's columns in VGPRs, the rows' x loaded together, x[k] broadcast
// by v_readlane into the FMAs.
constexpr int kProjRows = 32;
template <int KM, int NB>
__global__ __launch_bounds__(256) void masked_proj_kernel(const float* __restrict__ x, int64_t ldx,
                                                          const float* __restrict__ W,
                                                          const float* __restrict__ bias,
                                                          const int32_t* __restrict__ idx,
                                                          const int32_t* __restrict__ count, int K,
                                                          int N, float* __restrict__ y, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t g = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kProjRows;
  const int64_t cnt = *count;
  if (g >= cnt) return;
  const int64_t gi = g + (lane & (kProjRows - 1));
  const int rr = (lane < kProjRows && gi < cnt) ? idx[gi] : -1;
  float xr[kProjRows];
#pragma unroll
  for (int i = 0; i < kProjRows; ++i) {
    const int row = __builtin_amdgcn_readlane(rr, i);
    xr[i] = (row >= 0 && lane < K) ? x[(int64_t)row * ldx + lane] : 0.f;
  }
  float w[NB][KM], bb[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = 64 * nb + lane;
    bb[nb] = (bias && n < N) ? bias[n] : 0.f;
#pragma unroll
    for (int k = 0; k < KM; ++k) w[nb][k] = (k < K && n < N) ? W[(int64_t)k * N + n] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < kProjRows; ++i) {
    const int row = __builtin_amdgcn_readlane(rr, i);
    if (row < 0) break;  // wave-uniform: the list's tail
    float acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb] = bb[nb];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const float xk = rdlane(xr[i], k);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[nb] = fmaf(xk, w[nb][k], acc[nb]);
    }
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int n = 64 * nb + lane;
      if (n < N) y[(int64_t)row * ldy + n] = acc[nb];
    }
  }
}

// The masked rows' dx: 0, or the addend (its loads issued together). Wave gw takes rows
// [16 gw, 16 gw + 16). No LDS: full occupancy for what is a copy / fill of most of the B·L rows
// (it shared the listed-row kernel's 57 KB of LDS per block before, at 2 blocks per CU).
__global__ __launch_bounds__(256) void masked_fill_kernel(const uint8_t* __restrict__ mask,
                                                          int64_t R, int K,
                                                          float* __restrict__ dx, int64_t lddx,
                                                          const float* __restrict__ add,
                                                          int64_t ldadd) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t r0 = gw * 16;
  const int64_t rl = r0 + (lane & 15);
  const uint64_t zm = __ballot(lane < 16 && rl < R && mask[rl] == 0);
  if (!zm) return;
  float v[16];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int e = lane + 64 * it;
    const int i = e / K, k = e - i * K;
    v[it] = (add && e < 16 * K && ((zm >> i) & 1ull)) ? add[(r0 + i) * ldadd + k] : 0.f;
  }
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int e = lane + 64 * it;
    const int i = e / K, k = e - i * K;
    if (e < 16 * K && ((zm >> i) & 1ull)) dx[(r0 + i) * lddx + k] = v[it];
  }
}

// dx[r, k] = Σ_n d[r, n]·W[k, n] (+ add[r, k]) for the listed rows; K <= 64, N <= NM (the masked
// rows are masked_fill_kernel's). Wave gw computes listed rows [16 gw, 16 gw + 16): the d rows'
// loads issued together and staged in the wave's LDS (read back as broadcasts), W's row k in lane
// k's VGPRs (staged once per block through LDS, and only by blocks that have listed rows).
template <int NM>
__global__ __launch_bounds__(256) void masked_dx_kernel(const float* __restrict__ d, int64_t ldd,
                                                        const float* __restrict__ W,
                                                        const int32_t* __restrict__ idx,
                                                        const int32_t* __restrict__ count,
                                                        int K, int N, float* __restrict__ dx,
                                                        int64_t lddx, const float* __restrict__ add,
                                                        int64_t ldadd) {
  constexpr int NQ = (NM + 63) / 64;  // d elements per lane per row
  __shared__ __attribute__((aligned(16))) float ds[4][16][NM];
  __shared__ float wsh[64 * NM];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t cnt = *count;
  if ((int64_t)blockIdx.x * 64 >= cnt) return;  // block-uniform: no listed rows here
  for (int e = threadIdx.x; e < K * N; e += 256) wsh[e] = W[e];
  __syncthreads();
  const int64_t g = gw * 16;
  if (g >= cnt) return;
  const int64_t gi = g + (lane & 15);
  const int rr = (lane < 16 && gi < cnt) ? idx[gi] : -1;
  float t[16][NQ];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = __builtin_amdgcn_readlane(rr, i);
    const float* src = d + (int64_t)(row >= 0 ? row : 0) * ldd;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int n = lane + 64 * q;
      t[i][q] = (row >= 0 && n < N) ? src[n] : 0.f;
    }
  }
  // the addend of the listed rows (lane = output column), loaded with the d rows
  float av[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = __builtin_amdgcn_readlane(rr, i);
    av[i] = (add && row >= 0 && lane < K) ? add[(int64_t)row * ldadd + lane] : 0.f;
  }
  float w[NM];
#pragma unroll
  for (int n = 0; n < NM; ++n) w[n] = (lane < K && n < N) ? wsh[lane * N + n] : 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (lane + 64 * q < NM) ds[wave][i][lane + 64 * q] = t[i][q];
  __builtin_amdgcn_wave_barrier();  // one wave's LDS writes and reads run in issue order
#pragma unroll 2
  for (int i = 0; i < 16; ++i) {
    const int row = __builtin_amdgcn_readlane(rr, i);
    if (row < 0) break;
    const floatx4* rowp = reinterpret_cast<const floatx4*>(&ds[wave][i][0]);
    float acc = 0.f;
#pragma unroll
    for (int n4 = 0; n4 < NM / 4; ++n4) {
      const floatx4 v = rowp[n4];
      acc = fmaf(v[0], w[4 * n4], acc);
      acc = fmaf(v[1], w[4 * n4 + 1], acc);
      acc = fmaf(v[2], w[4 * n4 + 2], acc);
      acc = fmaf(v[3], w[4 * n4 + 3], acc);
    }
    if (lane < K) dx[(int64_t)row * lddx + lane] = add ? av[i] + acc : acc;
  }
}

constexpr int kWgBlocks = 512;  // row chunks (partials) of a weight gradient
constexpr int kWgRows = 64;     // rows staged per round
constexpr int kWgK = 68;        // A row stride in LDS (K <= 64, + the ones column)
constexpr int kWgN = 192;       // D row stride in LDS (N <= 192)

// part[blk][k][n] = Σ_{rows of blk} A_r[k]·D_r[n], k = K the ones column (→ column sums).
// Each round stages 64 listed rows: a wave's rows' indices come in one load, then every A / D
// element of them is loaded before any is stored to LDS (one memory round trip per round).
template <int RPW>  // rows per wave per round (= kWgRows / waves)
__global__ __launch_bounds__(1024) void masked_wgrad_kernel(const float* __restrict__ A, int64_t lda,
                                                            int shift_L, const float* __restrict__ D,
                                                            int64_t ldd,
                                                            const int32_t* __restrict__ idx,
                                                            const int32_t* __restrict__ count,
                                                            int K, int N, float* __restrict__ part) {
  __shared__ float As[kWgRows][kWgK];
  __shared__ __attribute__((aligned(16))) float Ds[kWgRows][kWgN];
  const int nth = blockDim.x, tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int KR = K + 1, NC = (N + 3) >> 2, items = KR * NC;
  int kk[4], cq[4];
  float acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int it = tid + j * nth;
    kk[j] = it < items ? it / NC : -1;
    cq[j] = it < items ? it % NC : 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[j][c] = 0.f;
  }
  const int64_t cnt = *count;
  const int64_t per = ((cnt + gridDim.x - 1) / gridDim.x + 15) / 16 * 16;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < cnt ? lo + per : cnt;
  for (int64_t s = lo; s < hi; s += kWgRows) {
    const int nr = hi - s < kWgRows ? (int)(hi - s) : kWgRows;
    const int i0 = wave * RPW;
    const int rl = (lane < RPW && i0 + lane < nr) ? idx[s + i0 + lane] : -1;
    float av[RPW], dv[RPW][3];
    int rj[RPW];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int r = __builtin_amdgcn_readlane(rl, j);
      rj[j] = r;
      const float* ar = nullptr;
      if (r >= 0) {
        if (shift_L > 0) ar = (r % shift_L) > 0 ? A + (int64_t)(r - 1) * lda : nullptr;
        else ar = A + (int64_t)r * lda;
      }
      av[j] = lane < K ? (ar ? ar[lane] : 0.f) : (lane == K && r >= 0 ? 1.f : 0.f);
      const float* dr = D + (int64_t)(r >= 0 ? r : 0) * ldd;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int n = lane + 64 * q;
        dv[j][q] = (r >= 0 && n < N) ? dr[n] : 0.f;
      }
    }
    __syncthreads();  // the previous round's rows are consumed
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      As[i0 + j][lane] = av[j];
      if (lane < kWgK - 64) As[i0 + j][64 + lane] = (64 + lane == K && rj[j] >= 0) ? 1.f : 0.f;
#pragma unroll
      for (int q = 0; q < 3; ++q) Ds[i0 + j][lane + 64 * q] = dv[j][q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (kk[j] < 0) continue;
      for (int i = 0; i < nr; ++i) {
        const float a = As[i][kk[j]];
        const floatx4 v = *reinterpret_cast<const floatx4*>(&Ds[i][4 * cq[j]]);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[j][c] = fmaf(a, v[c], acc[j][c]);
      }
    }
  }
  float* pb = part + (int64_t)blockIdx.x * KR * N;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (kk[j] < 0) continue;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int n = 4 * cq[j] + c;
      if (n < N) pb[kk[j] * N + n] = acc[j][c];
    }
  }
}

// C / sums = Σ_blk part[blk] in a fixed order: a block folds 64 outputs, its four waves take
// every fourth partial, then wave 0 adds the four in order
__global__ __launch_bounds__(256) void masked_wgrad_fold_kernel(const float* __restrict__ part,
                                                                int nblk, int K, int N,
                                                                float* __restrict__ C,
                                                                float* __restrict__ sums) {
  __shared__ float red[4][64];
  const int total = (K + 1) * N;
  const int q = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int e = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (e < total) {
#pragma unroll 8
    for (int b = q; b < nblk; b += 4) s += part[(int64_t)b * total + e];
  }
  red[q][lane] = s;
  __syncthreads();
  if (q == 0 && e < total) {
    const float v = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    if (e < K * N) C[e] = v;
    else if (sums) sums[e - K * N] = v;
  }
}

}  // namespace rs

using namespace rs;

extern "C" size_t rs_valid_rows_workspace_size(int64_t R) {
  return align_up((size_t)(ceil_div(R > 0 ? R : 1, kVrTile) + 1) * 4, 256);
}

extern "C" int32_t rs_valid_rows(const uint8_t* mask, int64_t R, int32_t* idx, int32_t* count,
                                 void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(R >= 0 && R < (int64_t(1) << 31), "R out of range");
  RS_CHECK_ARG(count && (R == 0 || (mask && idx)), "null pointer");
  hipStream_t st = as_stream(stream);
  if (R == 0) {
    RS_CHECK_HIP(hipMemsetAsync(count, 0, 4, st));
    return RS_OK;
  }
  RS_CHECK_ARG(workspace && ws_bytes >= rs_valid_rows_workspace_size(R), "workspace too small");
  const int nblk = (int)ceil_div(R, kVrTile);
  int32_t* blk = static_cast<int32_t*>(workspace);
  vr_count_kernel<<<nblk, 256, 0, st>>>(mask, R, blk);
  RS_CHECK_LAUNCH();
  vr_write_kernel<<<nblk, 256, 0, st>>>(mask, R, blk, idx, count);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_masked_proj(const float* x, int64_t ldx, const float* W, const float* bias,
                                  const int32_t* idx, const int32_t* count, int64_t R, int32_t K,
                                  int32_t N, float* y, int64_t ldy, void* stream) {
  RS_CHECK_ARG(R >= 0 && K >= 1 && K <= 64 && N >= 1 && N <= 192, "bad sizes (K <= 64, N <= 192)");
  RS_CHECK_ARG(ldx >= K && ldy >= N, "bad leading dimensions");
  if (R == 0) return RS_OK;
  RS_CHECK_ARG(x && W && idx && count && y, "null pointer");
  hipStream_t st = as_stream(stream);
  const int grid = (int)ceil_div(R, 4 * kProjRows);  // capacity: one wave per 32 listed rows
#define RS_PROJ(KM, NB) masked_proj_kernel<KM, NB><<<grid, 256, 0, st>>>(x, ldx, W, bias, idx, count, K, N, y, ldy)
  const int nb = (N + 63) / 64;
  if (K <= 16) {
    if (nb == 1) RS_PROJ(16, 1); else if (nb == 2) RS_PROJ(16, 2); else RS_PROJ(16, 3);
  } else if (K <= 36) {
    if (nb == 1) RS_PROJ(36, 1); else if (nb == 2) RS_PROJ(36, 2); else RS_PROJ(36, 3);
  } else {
    if (nb == 1) RS_PROJ(64, 1); else if (nb == 2) RS_PROJ(64, 2); else RS_PROJ(64, 3);
  }
#undef RS_PROJ
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_masked_dx_acc(const float* d, int64_t ldd, const float* W, const uint8_t* mask,
                                    const int32_t* idx, const int32_t* count, int64_t R, int32_t K,
                                    int32_t N, const float* add, int64_t ldadd, float* dx,
                                    int64_t lddx, void* stream) {
  RS_CHECK_ARG(R >= 0 && K >= 1 && K <= 64 && N >= 1 && N <= 192, "bad sizes (K <= 64, N <= 192)");
  RS_CHECK_ARG(ldd >= N && lddx >= K && (!add || ldadd >= K), "bad leading dimensions");
  if (R == 0) return RS_OK;
  RS_CHECK_ARG(d && W && mask && idx && count && dx, "null pointer");
  hipStream_t st = as_stream(stream);
  const int grid = (int)ceil_div(R, 64);  // one wave per 16 rows (and per 16 listed rows)
  masked_fill_kernel<<<grid, 256, 0, st>>>(mask, R, K, dx, lddx, add, ldadd);
  RS_CHECK_LAUNCH();
#define RS_DX(NM) masked_dx_kernel<NM><<<grid, 256, 0, st>>>(d, ldd, W, idx, count, K, N, dx, lddx, add, ldadd)
  if (N <= 64) RS_DX(64);
  else if (N <= 112) RS_DX(112);
  else if (N <= 128) RS_DX(128);
  else RS_DX(192);
#undef RS_DX
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_masked_dx(const float* d, int64_t ldd, const float* W, const uint8_t* mask,
                                const int32_t* idx, const int32_t* count, int64_t R, int32_t K,
                                int32_t N, float* dx, int64_t lddx, void* stream) {
  return rs_masked_dx_acc(d, ldd, W, mask, idx, count, R, K, N, nullptr, 0, dx, lddx, stream);
}

extern "C" size_t rs_masked_wgrad_workspace_size(int32_t K, int32_t N) {
  return align_up((size_t)kWgBlocks * (K + 1) * N * 4, 256);
}

extern "C" int32_t rs_masked_wgrad(const float* A, int64_t lda, int32_t shift_L, const float* D,
                                   int64_t ldd, const int32_t* idx, const int32_t* count, int32_t K,
                                   int32_t N, float* C, float* sums, void* workspace,
                                   size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(K >= 1 && K <= 64 && N >= 1 && N <= kWgN && shift_L >= 0, "bad sizes (K <= 64, N <= 192)");
  RS_CHECK_ARG(lda >= K && ldd >= N, "bad leading dimensions");
  RS_CHECK_ARG(A && D && idx && count && C, "null pointer");
  RS_CHECK_ARG(workspace && ws_bytes >= rs_masked_wgrad_workspace_size(K, N), "workspace too small");
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  const int items = (K + 1) * ((N + 3) / 4);
  if (items <= 1024)
    masked_wgrad_kernel<kWgRows / 4><<<kWgBlocks, 256, 0, st>>>(A, lda, shift_L, D, ldd, idx, count, K, N, part);
  else
    masked_wgrad_kernel<kWgRows / 16><<<kWgBlocks, 1024, 0, st>>>(A, lda, shift_L, D, ldd, idx, count, K, N, part);
  RS_CHECK_LAUNCH();
  const int total = (K + 1) * N;
  masked_wgrad_fold_kernel<<<(int)ceil_div(total, 64), 256, 0, st>>>(part, kWgBlocks, K, N, C, sums);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
