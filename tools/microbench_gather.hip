// Microbenchmark: what rate does the north-star train kernel's memory pattern reach, without its
// arithmetic? One wave per example gathers the example's 26 slab rows + its dense row (512 B each,
// lane (r, g) holds row r / 16 + r, 16-B chunks 4g + 16t as in dlrm_train_pipe), keeps DEPTH
// examples in flight in registers, optionally burns MF dependent-free v_mfma_f32_16x16x4_f32 per
// example (the kernel's 208) and optionally writes the 26 gradient rows (position order).
// Ids: the bench's synthetic batch (Criteo-skewed slot cardinalities over 40M rows, bounded
// Zipf(1.05) per slot, the same spread permutation), or uniform rows; the slab is 20.5 GB.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_gather.hip -o /tmp/mbg && /tmp/mbg
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                      \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4 gf4;
__device__ const float kZero[128] = {};

constexpr int S = 26, D = 128;

template <int DEPTH, int MF, int WRITE, bool READ = true, int VALU = 0>
__global__ __launch_bounds__(256) void pattern_k(const float* __restrict__ table,
                                                 const int* __restrict__ rows,
                                                 const float* __restrict__ dense, long batch,
                                                 int epw, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const long first = ((long)blockIdx.x * 4 + wave) * epw;
  const long last = first + epw < batch ? first + epw : batch;
  if (first >= batch) return;
  auto rowp = [&](long b, int i) -> const float* {
    if (b >= last) return kZero;
    if (i < S) return table + (long)rows[b * S + i] * D;
    if (i == S) return dense + b * D;
    return kZero;
  };
  f4 x[DEPTH][16];
  auto issue = [&](int slot, long b) {
    const float* p0 = READ ? rowp(b, r) : kZero;
    const float* p1 = READ ? rowp(b, 16 + r) : kZero;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      x[slot][t] = *(gf4*)(p0 + 4 * g + 16 * t);
      x[slot][8 + t] = *(gf4*)(p1 + 4 * g + 16 * t);
    }
  };
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) issue(k, first + k);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long b = first; b < last; b += DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      const long bb = b + k;
      f4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 16; ++t) c += x[k][t];
      if constexpr (MF > 0) {
        f4 m0 = c, m1 = c;
#pragma unroll
        for (int j = 0; j < MF / 2; ++j) {
          m0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[k][j & 15][0], x[k][j & 15][1], m0, 0, 0, 0);
          m1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[k][j & 15][2], x[k][j & 15][3], m1, 0, 0, 0);
        }
        c += m0 + m1;
      }
      if constexpr (VALU > 0) {  // the bf16 split's conversion work: VALU ops per lane
        uint32_t u = __float_as_uint(c[0]);
#pragma unroll
        for (int j = 0; j < VALU / 2; ++j) {
          u = (u & 0xFFFF0000u) ^ (uint32_t)j;
          u = __float_as_uint(__uint_as_float(u) - c[1]);
        }
        c[2] += __uint_as_float(u);
      }
      if constexpr (WRITE == 2 || WRITE == 3) {  // half-wave per 512-B row, 1 KB per store
        if (bb < last) {
          float* o = out + bb * S * (long)D;
          const int r32 = lane & 31, h = lane >> 5;
#pragma unroll
          for (int s2 = 0; s2 < S / 2; ++s2) {
            f4 v = x[k][s2 & 15] + c;
            float* dst = o + (2 * s2 + h) * D + 4 * r32;
            if constexpr (WRITE == 3) __builtin_nontemporal_store(v, (f4*)dst);
            else *(f4*)dst = v;
          }
        }
      }
      if constexpr (WRITE == 1) {
        if (bb < last) {
          float* o = out + bb * S * (long)D;
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            *(f4*)(o + r * D + 4 * g + 16 * t) = x[k][t];
            if (16 + r < S) *(f4*)(o + (16 + r) * D + 4 * g + 16 * t) = x[k][8 + t];
          }
        }
      }
      acc += c;
      issue(k, bb + DEPTH);
    }
  }
  if (acc[0] == 1234.5f) out[0] = acc[1];
}

static std::vector<long> criteo_cards(long total) {
  const double base[26] = {1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683,
                           8351593, 3194, 27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15,
                           286181, 105, 142572};
  double small = 0, big = 0;
  for (double b : base) (b < 100000 ? small : big) += b;
  std::vector<long> out(26);
  long sum = 0;
  for (int i = 0; i < 26; ++i) {
    out[i] = base[i] < 100000 ? (long)base[i] : (long)std::floor(base[i] * (total - small) / big);
    sum += out[i];
  }
  *std::max_element(out.begin(), out.end()) += total - sum;
  return out;
}

int main(int argc, char** argv) {
  const long V = 40000000, B = 65536;
  const size_t tbytes = (size_t)V * D * 4;
  float *table, *dense, *out;
  int* rows;
  CK(hipMalloc(&table, tbytes));
  CK(hipMalloc(&dense, B * D * 4));
  CK(hipMalloc(&out, (size_t)B * S * D * 4));
  CK(hipMalloc(&rows, B * S * 4));
  CK(hipMemset(table, 0, tbytes));
  CK(hipMemset(dense, 0, B * D * 4));
  CK(hipMemset(out, 0, (size_t)B * S * D * 4));
  auto cards = criteo_cards(V);
  std::vector<long> off(27, 0);
  for (int i = 0; i < 26; ++i) off[i + 1] = off[i] + cards[i];
  std::mt19937_64 rng(4);
  std::uniform_real_distribution<double> U01(0.0, 1.0);
  std::vector<int> zipf(B * S), unif(B * S), small(B * S);
  for (long b = 0; b < B; ++b)
    for (int s = 0; s < S; ++s) {
      const long c = cards[s];
      long k = 0;
      if (c > 1) {
        const double a1 = 1.0 - 1.05, u = U01(rng);
        k = (long)std::floor(std::pow((std::pow((double)c, a1) - 1.0) * u + 1.0, 1.0 / a1)) - 1;
        k = std::min(std::max(k, 0L), c - 1);
      }
      long mult = c > 2 ? 2654435761L % c : 1;
      while (std::gcd(mult, c) != 1) ++mult;
      const long id = (long)((__int128)k * mult % c);
      zipf[b * S + s] = (int)(off[s] + id);
      unif[b * S + s] = (int)(rng() % V);
      small[b * S + s] = (int)(rng() % 2000000);  // a 1 GB table: TLB reach / MALL check
    }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto kern, const std::vector<int>& ids, int blocks_per_cu,
                 bool write, bool read = true) {
    CK(hipMemcpy(rows, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
    const int nb = 256 * blocks_per_cu;
    const int epw = (int)((B + nb * 4 - 1) / (nb * 4));
    for (int w = 0; w < 2; ++w) kern<<<nb, 256>>>(table, rows, dense, B, epw, out);
    CK(hipDeviceSynchronize());
    const int it = 10;
    CK(hipEventRecord(e0));
    for (int w = 0; w < it; ++w) kern<<<nb, 256>>>(table, rows, dense, B, epw, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000.0 / it;
    const double by = (read ? (double)B * (S * 4 + 27 * 512.0) : 0) + (write ? (double)B * S * 512 : 0);
    printf("%-44s blocks/CU %d  %7.1f us  %5.2f TB/s\n", name, blocks_per_cu, us, by / us / 1e6);
  };
  for (int bpc : {1, 2, 3, 4}) {
    run("zipf  d1 rd only", pattern_k<1, 0, 0>, zipf, bpc, false);
    run("zipf  d2 rd only", pattern_k<2, 0, 0>, zipf, bpc, false);
    run("zipf  d1 rd+wr nt", pattern_k<1, 0, 3>, zipf, bpc, true);
    run("zipf  d2 rd+wr nt", pattern_k<2, 0, 3>, zipf, bpc, true);
    run("zipf  d1 rd+wr 64B rows", pattern_k<1, 0, 1>, zipf, bpc, true);
    run("zipf  d1 rd+wr nt +84mfma +300valu", pattern_k<1, 84, 3, true, 300>, zipf, bpc, true);
  }
  return 0;
}
