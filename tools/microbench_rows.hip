// Microbenchmark: what HBM rate do random whole-row reads / writes reach on this MI355X?
// (guides the embedding-path kernels: 512-B rows at D = 128 fp32). Standalone:
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_rows.hip -o /tmp/mbr && /tmp/mbr
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// copy: n float4
__global__ void copy_k(const f4* __restrict__ a, f4* __restrict__ b, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x, s = (long)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = a[i];
}

// gather rows: row r = idx[k]; LPR lanes per row (LPR*16 B = row bytes), ROWS rows in flight
// per lane group; MODE 0: read only (sum, store if impossible), 1: read + write dst row k
template <int LPR, int INFL, int MODE>
__global__ __launch_bounds__(256) void gather_k(const f4* __restrict__ src, const int* __restrict__ idx,
                                                long n_rows, f4* __restrict__ dst) {
  const int gl = threadIdx.x % LPR;
  const long grp = (blockIdx.x * (long)blockDim.x + threadIdx.x) / LPR;
  const long ngrp = (long)gridDim.x * blockDim.x / LPR;
  f4 acc = {0, 0, 0, 0};
  for (long k0 = grp * INFL; k0 < n_rows; k0 += ngrp * INFL) {
    f4 v[INFL];
#pragma unroll
    for (int u = 0; u < INFL; ++u) {
      long k = k0 + u;
      int r = k < n_rows ? idx[k] : 0;
      v[u] = src[(long)r * LPR + gl];
    }
#pragma unroll
    for (int u = 0; u < INFL; ++u) {
      long k = k0 + u;
      if (MODE == 1) { if (k < n_rows) dst[k * LPR + gl] = v[u]; }
      else acc += v[u];
    }
  }
  if (MODE == 0 && acc[0] == 1234.5f) dst[0] = acc;
}

// scatter rows: dst row idx[k] = src row k
template <int LPR, int INFL>
__global__ __launch_bounds__(256) void scatter_k(const f4* __restrict__ src, const int* __restrict__ idx,
                                                 long n_rows, f4* __restrict__ dst) {
  const int gl = threadIdx.x % LPR;
  const long grp = (blockIdx.x * (long)blockDim.x + threadIdx.x) / LPR;
  const long ngrp = (long)gridDim.x * blockDim.x / LPR;
  for (long k0 = grp * INFL; k0 < n_rows; k0 += ngrp * INFL) {
    f4 v[INFL];
    int r[INFL];
#pragma unroll
    for (int u = 0; u < INFL; ++u) {
      long k = k0 + u;
      r[u] = k < n_rows ? idx[k] : -1;
      v[u] = src[(k < n_rows ? k : 0) * LPR + gl];
    }
#pragma unroll
    for (int u = 0; u < INFL; ++u) if (r[u] >= 0) dst[(long)r[u] * LPR + gl] = v[u];
  }
}

template <class F>
float timeit(F f, int iters = 10) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / iters;
}

int main() {
  const long n_rows = 1703936;           // 65536 * 26 rows of 512 B = 872 MB
  const long bytes = n_rows * 512;
  f4 *a, *b;
  int* idx;
  CK(hipMalloc(&a, bytes * 2));          // room for 1-KB rows at half the count
  CK(hipMalloc(&b, bytes * 2));
  CK(hipMalloc(&idx, n_rows * 4));
  CK(hipMemset(a, 0, bytes * 2));
  CK(hipMemset(b, 0, bytes * 2));
  std::vector<int> perm(n_rows);
  for (long i = 0; i < n_rows; ++i) perm[i] = (int)i;
  std::mt19937 rng(4);
  std::shuffle(perm.begin(), perm.end(), rng);
  CK(hipMemcpy(idx, perm.data(), n_rows * 4, hipMemcpyHostToDevice));
  const int blocks = 256 * 8;
  {
    long n4 = bytes / 16;
    float us = timeit([&] { copy_k<<<4096, 256>>>(a, b, n4); });
    printf("copy 872 MB (r+w)            %8.1f us  %6.2f TB/s\n", us, 2.0 * bytes / us / 1e6);
  }
#define G(LPR, INFL, MODE, NAME)                                                                    \
  {                                                                                                \
    long nr = bytes / (LPR * 16);                                                                  \
    float us = timeit([&] { gather_k<LPR, INFL, MODE><<<blocks, 256>>>(a, idx, nr, b); });         \
    double by = (double)nr * LPR * 16 * (MODE ? 2 : 1);                                            \
    printf("%-28s %8.1f us  %6.2f TB/s\n", NAME, us, by / us / 1e6);                               \
  }
  // (the 1-KB case reuses the first half of the permutation: its indices stay < nr)
  G(32, 4, 0, "gather 512B rd INFL4");
  G(32, 8, 0, "gather 512B rd INFL8");
  G(32, 16, 0, "gather 512B rd INFL16");
  G(32, 8, 1, "gather 512B rd+wr INFL8");
  {
    long nr = n_rows;
    float us = timeit([&] { scatter_k<32, 8><<<blocks, 256>>>(a, idx, nr, b); });
    printf("%-28s %8.1f us  %6.2f TB/s\n", "scatter 512B INFL8", us, 2.0 * bytes / us / 1e6);
  }
  {  // sequential index = in-order rows
    std::vector<int> seq(n_rows);
    for (long i = 0; i < n_rows; ++i) seq[i] = (int)i;
    CK(hipMemcpy(idx, seq.data(), n_rows * 4, hipMemcpyHostToDevice));
    G(32, 8, 0, "in-order 512B rd INFL8");
    CK(hipMemcpy(idx, perm.data(), n_rows * 4, hipMemcpyHostToDevice));
  }
  return 0;
}
