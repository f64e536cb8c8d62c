// gemm.hip — fp32 GEMMs of the Keras Dense layers (esmm/layers.py:4-13, esmm/mmoe.py:8-109, the
// ctr / dien MLPs: y = act(x·W + b) and its two backward products) on the bf16 matrix cores at
// fp32 accuracy.
//
// gfx950 has no xf32 and runs fp32-input MFMA at 1/16 of the bf16 rate (MI355X_MICROARCH: 155 TF
// measured vs ~2.5 PF). Every fp32 operand is split into three bf16 parts x = h + m + l (h, m, l
// round-to-nearest; the residuals are exact in fp32, so the parts carry x's 24 bits), and each
// product a·b is formed from the six part products down to 2^-16 |a||b| (mfma6: m·m, h·l, l·h,
// h·m, m·h, h·h, smallest first, fp32 accumulation). The three dropped products are below
// 2^-24 |a||b|: the same error class as an fp32 fma chain, at 6/16 of the fp32-MFMA cycles per
// K element.
//
// Tiling: a 256-thread block computes a 128x128 tile of C with four waves of 64x64 (4x4 MFMA
// 16x16x32 tiles, 64 fp32 accumulators per lane); K advances 32 at a time. Each K-step the block
// loads its A and B slices from global memory into registers (issued before the previous step's
// products, so they fly under them), splits them, and stores the parts to LDS as [row][k] bf16
// planes, 64 B per row, the four 16-B chunks of a row XOR-swizzled by row bits 2-3 so that a
// ds_read_b128 group of 16 lanes (rows i, chunk g) covers all 64 banks. A fragment = 8
// consecutive k of one row = one ds_read_b128 per part.
//
// Operand access: op(A)[m][k] = ta ? A[k·lda + m] : A[m·lda + k]; op(B)[k][n] = tb ? B[n·ldb + k]
// : B[k·ldb + n]. A k-contiguous operand is read as float4 along k; an m/n-contiguous one as four
// float4 rows of a 4x4 block transposed in registers. The three Dense products:
//   forward  y = x·W        ta 0, tb 0 (x [B, in], W [in, out])
//   dgrad    dx = dz·Wᵀ     ta 0, tb 1
//   wgrad    dW = xᵀ·dz     ta 1, tb 0, K = the batch: split into `splits` K ranges written as
//            partials and folded in split order (deterministic).
// Batched (MMOE's experts): blockIdx.z = batch · splits + split, with per-batch strides.
#include "common.hpp"

namespace rs {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));

constexpr int kBM = 128, kBN = 128, kBK = 32;
constexpr int kPlane = 128 * kBK * 2;  // bytes of one part plane of a 128-row tile

// 16-B chunk c (0..3) of row r inside a plane: XOR-swizzled by row bits 2-3 with the
// permutation (0, 2, 3, 1), so each ds_read_b128 lane group (MI355X_MICROARCH §LDS: lanes
// {0-3, 12-15, 20-27}, ...) reads 16 distinct 16-B bank quads
__device__ __forceinline__ int swz_off(int row, int chunk) {
  const int q = (row >> 2) & 3;
  const int h = (0x78 >> (2 * q)) & 3;  // q -> 0, 2, 3, 1
  return row * 64 + 16 * (chunk ^ h);
}

// four fp32 values -> their three bf16 parts (v_cvt_pk_bf16_f32 pairs)
__device__ __forceinline__ void split4(const f4& x, bf4& h, bf4& m, bf4& l) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f2 v = f2{x[2 * j], x[2 * j + 1]};
    const bf2 hp = __builtin_convertvector(v, bf2);
    const f2 r1 = v - __builtin_convertvector(hp, f2);
    const bf2 mp = __builtin_convertvector(r1, bf2);
    const bf2 lp = __builtin_convertvector(r1 - __builtin_convertvector(mp, f2), bf2);
    h[2 * j] = hp[0];
    h[2 * j + 1] = hp[1];
    m[2 * j] = mp[0];
    m[2 * j + 1] = mp[1];
    l[2 * j] = lp[0];
    l[2 * j + 1] = lp[1];
  }
}

__device__ __forceinline__ f4 mfma6(const bf8& ah, const bf8& am, const bf8& al, const bf8& bh,
                                    const bf8& bm, const bf8& bl, f4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

// One operand's 128 x 32 slice for this K-step, 4 float4 per thread.
//   KC (k-contiguous): thread t -> row t / 8 + 32 i (i = 0..3), k4 = t % 8
//   !KC (row-contiguous): thread t -> 4x4 block (rows 4 (t / 8) .., k 4 (t % 8) ..): the
//   four float4 are the block's k rows, transposed at the store
template <bool KC>
struct Slice {
  f4 v[4];
  __device__ __forceinline__ void load(const float* __restrict__ base, int64_t ld, int64_t r0,
                                       int64_t rows, int64_t k0, int64_t K) {
    const int t = threadIdx.x;
    if (KC) {
      const int64_t k = k0 + 4 * (t & 7);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t r = r0 + (t >> 3) + 32 * i;
        v[i] = (r < rows && k < K) ? *reinterpret_cast<const f4*>(base + r * ld + k)
                                   : f4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      const int64_t r = r0 + 4 * (t >> 3);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t k = k0 + 4 * (t & 7) + i;
        v[i] = (r < rows && k < K) ? *reinterpret_cast<const f4*>(base + k * ld + r)
                                   : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  // the three parts to the planes [row][k]
  __device__ __forceinline__ void store(char* planes) const {
    const int t = threadIdx.x;
    if (KC) {
      const int kk = 4 * (t & 7);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (t >> 3) + 32 * i;
        bf4 h, m, l;
        split4(v[i], h, m, l);
        const int off = swz_off(row, kk >> 3) + 2 * (kk & 7);
        *reinterpret_cast<bf4*>(planes + off) = h;
        *reinterpret_cast<bf4*>(planes + kPlane + off) = m;
        *reinterpret_cast<bf4*>(planes + 2 * kPlane + off) = l;
      }
    } else {
      const int kk = 4 * (t & 7);
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // row 4 (t / 8) + j holds element j of each k row
        const f4 x = f4{v[0][j], v[1][j], v[2][j], v[3][j]};
        bf4 h, m, l;
        split4(x, h, m, l);
        const int row = 4 * (t >> 3) + j;
        const int off = swz_off(row, kk >> 3) + 2 * (kk & 7);
        *reinterpret_cast<bf4*>(planes + off) = h;
        *reinterpret_cast<bf4*>(planes + kPlane + off) = m;
        *reinterpret_cast<bf4*>(planes + 2 * kPlane + off) = l;
      }
    }
  }
};

struct GemmArgs {
  const float* A;
  int64_t lda, sA;
  const float* B;
  int64_t ldb, sB;
  float* C;  // the output, or the split partials [batch * splits][M][N] when splits > 1
  int64_t ldc, sC;
  const float* bias;  // [N] per batch (stride sbias), may be null
  int64_t sbias;
  int64_t M, N, K;
  int64_t k_per_split;
  int splits;
  int act;  // 0 none, 1 relu, 2 sigmoid
};

// two blocks per CU (210 VGPRs, 48 KB LDS each): one block's split-and-store phase runs under the
// other's products (a two-stage register prefetch at one block per CU measured 1.3-1.9x slower)
template <bool TA, bool TB>
__global__ __launch_bounds__(256, 2) void gemm_x3_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char lds[6 * kPlane];  // A parts | B parts (48 KB)
  char* la = lds;
  char* lb = lds + 3 * kPlane;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int z = blockIdx.z;
  const int batch = z / g.splits, split = z - batch * g.splits;
  const float* A = g.A + batch * g.sA;
  const float* B = g.B + batch * g.sB;
  const int64_t m0 = (int64_t)blockIdx.y * kBM, n0 = (int64_t)blockIdx.x * kBN;
  const int64_t kb = split * g.k_per_split;
  const int64_t ke = kb + g.k_per_split < g.K ? kb + g.k_per_split : g.K;

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  Slice<!TA> sa;  // op(A) rows = m: k-contiguous unless A is given transposed
  Slice<TB> sb;   // op(B) rows = n: k-contiguous when B is given as [n][k]
  sa.load(A, g.lda, m0, g.M, kb, ke);
  sb.load(B, g.ldb, n0, g.N, kb, ke);
  const int r = lane & 15, kg = lane >> 4;
  auto products = [&]() {
    bf8 bh[4], bm[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int off = swz_off(wn * 64 + 16 * j + r, kg);
      bh[j] = *reinterpret_cast<const bf8*>(lb + off);
      bm[j] = *reinterpret_cast<const bf8*>(lb + kPlane + off);
      bl[j] = *reinterpret_cast<const bf8*>(lb + 2 * kPlane + off);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = swz_off(wm * 64 + 16 * i + r, kg);
      const bf8 ah = *reinterpret_cast<const bf8*>(la + off);
      const bf8 am = *reinterpret_cast<const bf8*>(la + kPlane + off);
      const bf8 al = *reinterpret_cast<const bf8*>(la + 2 * kPlane + off);
      // each K-step's six products summed from zero, then added to the running sum on the VALU
      // (round to nearest): summed straight into the long accumulator the result drifted
      // one-signed (tools/gemm_bias_probe.py: mean signed error 10 % of the mean |error| on
      // one-signed data; the library GEMM's 0.01 %); re-accumulated, the mean |error| is 4x
      // below the library's
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] += mfma6(ah, am, al, bh[j], bm[j], bl[j], f4{0.f, 0.f, 0.f, 0.f});
    }
  };
  for (int64_t k0 = kb; k0 < ke; k0 += kBK) {
    __syncthreads();  // the previous step's fragments are read
    sa.store(la);
    sb.store(lb);
    __syncthreads();
    if (k0 + kBK < ke) {  // the next slice flies under this step's products
      sa.load(A, g.lda, m0, g.M, k0 + kBK, ke);
      sb.load(B, g.ldb, n0, g.N, k0 + kBK, ke);
    }
    products();
  }
  // C[m][n]: lane (r, kg) of tile (i, j) holds rows 4 kg + q, column r
  float* C = g.C + (g.splits > 1 ? (int64_t)z * g.M * g.N : batch * g.sC);
  const int64_t ldc = g.splits > 1 ? g.N : g.ldc;
  const float* bias = g.bias ? g.bias + batch * g.sbias : nullptr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = n0 + wn * 64 + 16 * j + r;
    const float bv = (bias && n < g.N && g.splits == 1) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * kg + q;
        if (m < g.M && n < g.N) {
          float v = acc[i][j][q];
          if (g.splits == 1) {
            v += bv;
            if (g.act == 1) v = fmaxf(v, 0.f);
            else if (g.act == 2) v = 1.f / (1.f + expf(-v));
          }
          C[m * ldc + n] = v;
        }
      }
    }
  }
}

// out[b][m][n] = act(Σ_s part[b][s][m][n] + bias[b][n]), the splits summed in order
__global__ __launch_bounds__(256) void gemm_fold_kernel(const float* __restrict__ part, int splits,
                                                        int64_t M, int64_t N, int batch,
                                                        float* __restrict__ C, int64_t ldc,
                                                        int64_t sC, const float* __restrict__ bias,
                                                        int64_t sbias, int act) {
  const int64_t MN = M * N;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < MN * batch;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / MN, mn = e - b * MN;
    const int64_t m = mn / N, n = mn - m * N;
    const float* p = part + b * splits * MN + mn;
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += p[s * MN];
    if (bias) v += bias[b * sbias + n];
    if (act == 1) v = fmaxf(v, 0.f);
    else if (act == 2) v = 1.f / (1.f + expf(-v));
    C[b * sC + m * ldc + n] = v;
  }
}

}  // namespace rs

using namespace rs;

extern "C" size_t rs_gemm_x3_workspace_size(int64_t M, int64_t N, int32_t batch, int32_t splits) {
  return splits > 1 ? align_up((size_t)M * N * batch * splits * sizeof(float), 256) : 0;
}

extern "C" int32_t rs_gemm_x3(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K,
                              const float* A, int64_t lda, int64_t sA, const float* B, int64_t ldb,
                              int64_t sB, float* C, int64_t ldc, int64_t sC, int32_t batch,
                              const float* bias, int64_t sbias, int32_t act, int32_t splits,
                              void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && batch >= 1 && splits >= 1, "rs_gemm_x3: bad sizes");
  RS_CHECK_ARG(act >= 0 && act <= 2, "rs_gemm_x3: act must be 0 (none), 1 (relu) or 2 (sigmoid)");
  RS_CHECK_ARG(M % 4 == 0 && N % 4 == 0 && K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 &&
                   sA % 4 == 0 && sB % 4 == 0,
               "rs_gemm_x3: M, N, K, lda, ldb and the batch strides must be multiples of 4");
  RS_CHECK_ARG(((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0,
               "rs_gemm_x3: A and B must be 16-byte aligned");
  RS_CHECK_ARG(lda >= (ta ? M : K) && ldb >= (tb ? K : N) && ldc >= N, "rs_gemm_x3: bad leading dimensions");
  if (M == 0 || N == 0) return RS_OK;
  RS_CHECK_ARG(A && B && C, "rs_gemm_x3: null pointer");
  hipStream_t st = as_stream(stream);
  if (K == 0) splits = 1;
  // K ranges of the splits: multiples of the 32-deep step
  const int64_t kps = splits > 1 ? align_up((size_t)ceil_div(K, splits), kBK) : (K > 0 ? K : 1);
  const int eff = splits > 1 ? (int)ceil_div(K, kps) : 1;
  float* out = C;
  if (eff > 1) {
    RS_CHECK_ARG(workspace && ws_bytes >= rs_gemm_x3_workspace_size(M, N, batch, eff),
                 "rs_gemm_x3: workspace too small for the split-K partials");
    out = static_cast<float*>(workspace);
  }
  GemmArgs g{A, lda, sA, B, ldb, sB, out, ldc, sC, bias, sbias, M, N, K, kps, eff, act};
  RS_CHECK_ARG((int64_t)batch * eff < 65536, "rs_gemm_x3: batch x splits too large");
  dim3 grid((unsigned)ceil_div(N, kBN), (unsigned)ceil_div(M, kBM), (unsigned)(batch * eff));
  RS_CHECK_ARG(grid.y < 65536, "rs_gemm_x3: M too large");
  if (ta == 0 && tb == 0) gemm_x3_kernel<false, false><<<grid, 256, 0, st>>>(g);
  else if (ta == 0 && tb != 0) gemm_x3_kernel<false, true><<<grid, 256, 0, st>>>(g);
  else if (ta != 0 && tb == 0) gemm_x3_kernel<true, false><<<grid, 256, 0, st>>>(g);
  else gemm_x3_kernel<true, true><<<grid, 256, 0, st>>>(g);
  RS_CHECK_LAUNCH();
  if (eff > 1) {
    const int64_t total = M * N * batch;
    const int blocks = (int)std::min<int64_t>(ceil_div(total, 256), 8192);
    gemm_fold_kernel<<<blocks, 256, 0, st>>>(out, eff, M, N, batch, C, ldc, sC, bias, sbias, act);
    RS_CHECK_LAUNCH();
  }
  return RS_OK;
}
