// STREAM-copy variants on one MI355X (tools/, not the product): which 16-byte copy shape reaches
// the guide's ~6.3 TB/s. hipcc --offload-arch=gfx950 -O3 tools/microbench_copy.hip -o tools/microbench_copy.bin
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void copy_flat(const float4* __restrict__ s, float4* __restrict__ d, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) d[i] = s[i];
}
template <int U>
__global__ void copy_unroll(const float4* __restrict__ s, float4* __restrict__ d, long n) {
  long base = (long)blockIdx.x * blockDim.x * U + threadIdx.x;
  float4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; if (i < n) v[u] = s[i]; }
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; if (i < n) d[i] = v[u]; }
}
typedef float f4 __attribute__((ext_vector_type(4)));
template <int U>
__global__ void copy_nt(const f4* __restrict__ s, f4* __restrict__ d, long n) {
  long base = (long)blockIdx.x * blockDim.x * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; if (i < n) v[u] = __builtin_nontemporal_load(s + i); }
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; if (i < n) __builtin_nontemporal_store(v[u], d + i); }
}
__global__ void copy_gs(const float4* __restrict__ s, float4* __restrict__ d, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) d[i] = s[i];
}

int main() {
  const long bytes = 4L << 30, n = bytes / 16;
  float4 *s, *d;
  (void)hipMalloc(&s, bytes); (void)hipMalloc(&d, bytes);
  (void)hipMemset(s, 0, bytes); (void)hipMemset(d, 0, bytes);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) launch();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.1f GB/s\n", name, 2.0 * bytes * 10 / (ms * 1e-3) / 1e9);
  };
  run("flat 256", [&] { copy_flat<<<(n + 255) / 256, 256>>>(s, d, n); });
  run("flat 1024", [&] { copy_flat<<<(n + 1023) / 1024, 1024>>>(s, d, n); });
  run("unroll4 256", [&] { copy_unroll<4><<<(n + 1023) / 1024, 256>>>(s, d, n); });
  run("unroll8 256", [&] { copy_unroll<8><<<(n + 2047) / 2048, 256>>>(s, d, n); });
  run("unroll16 256", [&] { copy_unroll<16><<<(n + 4095) / 4096, 256>>>(s, d, n); });
  run("nt unroll4 256", [&] { copy_nt<4><<<(n + 1023) / 1024, 256>>>((const f4*)s, (f4*)d, n); });
  run("nt unroll8 256", [&] { copy_nt<8><<<(n + 2047) / 2048, 256>>>((const f4*)s, (f4*)d, n); });
  run("gridstride 2048x256", [&] { copy_gs<<<2048, 256>>>(s, d, n); });
  run("gridstride 8192x256", [&] { copy_gs<<<8192, 256>>>(s, d, n); });
  run("hipMemcpy D2D", [&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice); });
  return 0;
}
