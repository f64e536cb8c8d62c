// rng.hpp — Philox4x32-10 (Salmon et al., SC'11) and the engine's draw scheme, shared by the
// PinSage and EGES samplers: key (seed_lo, seed_hi ^ purpose), counter (a, b, c, idx / 4),
// word idx % 4; bounded ints by multiply-high. oracle/pinsage.py restates it.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rs {

struct U4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
           (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ uint32_t draw(uint64_t seed, uint32_t purpose, uint32_t a, uint32_t b,
                                         uint32_t c, uint32_t idx) {
  U4 r = philox4x32_10(U4{a, b, c, idx >> 2}, (uint32_t)seed, (uint32_t)(seed >> 32) ^ purpose);
  switch (idx & 3) {
    case 0: return r.x;
    case 1: return r.y;
    case 2: return r.z;
    default: return r.w;
  }
}

// draw(seed, purpose, a, b, c, idx) for a run of idx, one Philox block per 4 draws
struct DrawStream {
  uint32_t k0, k1, a, b, c, blk;
  U4 r;
  __device__ __forceinline__ DrawStream(uint64_t seed, uint32_t purpose, uint32_t a_, uint32_t b_,
                                        uint32_t c_)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32) ^ purpose), a(a_), b(b_), c(c_),
        blk(0xFFFFFFFFu), r{0, 0, 0, 0} {}
  __device__ __forceinline__ uint32_t at(uint32_t idx) {
    if ((idx >> 2) != blk) {
      blk = idx >> 2;
      r = philox4x32_10(U4{a, b, c, blk}, k0, k1);
    }
    const uint32_t q = idx & 3;
    return q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
  }
};

__device__ __forceinline__ uint32_t bounded(uint32_t r, uint32_t n) {
  return (uint32_t)(((uint64_t)r * n) >> 32);
}

}  // namespace rs
