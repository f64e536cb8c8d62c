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
                                                             float* __restrict__ part) {
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
      const int64_t o = r * N + col0;
      float g[VEC], yy[VEC];
      if constexpr (VEC == 4) {
        float4 t = *reinterpret_cast<const float4*>(dy + o);
        g[0] = t.x; g[1] = t.y; g[2] = t.z; g[3] = t.w;
        if constexpr (ACT != 0) {
          float4 u = *reinterpret_cast<const float4*>(y + o);
          yy[0] = u.x; yy[1] = u.y; yy[2] = u.z; yy[3] = u.w;
        }
      } else {
        g[0] = dy[o];
        if constexpr (ACT != 0) yy[0] = y[o];
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

}  // namespace rs

using namespace rs;

extern "C" size_t rs_act_bwd_colsum_workspace_size(int64_t B, int32_t N) {
  return (size_t)ceil_div(B, kColRows) * N * sizeof(float);
}

extern "C" int32_t rs_act_bwd_colsum(const float* dy, const float* y, int64_t B, int32_t N,
                                     int32_t act, float* dz, float* db, void* workspace,
                                     size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(B >= 0 && N >= 1 && act >= 0 && act <= 2, "bad arguments");
  RS_CHECK_ARG(act == 0 || (y && dz), "activation backward needs y and dz");
  RS_CHECK_ARG(ws_bytes >= rs_act_bwd_colsum_workspace_size(B, N), "workspace too small");
  hipStream_t st = as_stream(stream);
  if (B == 0) {
    RS_CHECK_HIP(hipMemsetAsync(db, 0, (size_t)N * 4, st));
    return RS_OK;
  }
  const int nchunks = (int)ceil_div(B, kColRows);
  float* part = static_cast<float*>(workspace);
  const bool v4 = N % 4 == 0 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0 &&
                  (!y || (reinterpret_cast<uintptr_t>(y) & 15) == 0) &&
                  (!dz || (reinterpret_cast<uintptr_t>(dz) & 15) == 0);
  if (v4) {
    dim3 grid((unsigned)ceil_div(N, 64), (unsigned)nchunks);
    switch (act) {
      case 0: act_bwd_colsum_kernel<0, 4><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part); break;
      case 1: act_bwd_colsum_kernel<1, 4><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part); break;
      default: act_bwd_colsum_kernel<2, 4><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part); break;
    }
  } else {
    dim3 grid((unsigned)ceil_div(N, 16), (unsigned)nchunks);
    switch (act) {
      case 0: act_bwd_colsum_kernel<0, 1><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part); break;
      case 1: act_bwd_colsum_kernel<1, 1><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part); break;
      default: act_bwd_colsum_kernel<2, 1><<<grid, 256, 0, st>>>(dy, y, B, N, dz, part); break;
    }
  }
  RS_CHECK_LAUNCH();
  fold_chunks_kernel<<<(unsigned)ceil_div(N, 64), 256, 0, st>>>(part, nchunks, N, db);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
