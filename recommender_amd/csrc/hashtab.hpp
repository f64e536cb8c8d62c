// hashtab.hpp — token hashing and the open-addressing tables shared by the text ingestion
// kernels (criteo.hip, textpipe.hip): FNV-1a 64 token identity, linear probing over a
// power-of-two table whose empty slots hold ~0.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rs {

constexpr uint64_t kFnvBasis = 1469598103934665603ull;
constexpr uint64_t kFnvPrime = 1099511628211ull;
constexpr uint64_t kEmptySlot = ~0ull;

__device__ __forceinline__ uint64_t fnv1a(const uint8_t* p, int n) {
  uint64_t h = kFnvBasis;
  for (int i = 0; i < n; ++i) h = (h ^ p[i]) * kFnvPrime;
  return h;
}

__device__ __forceinline__ uint32_t vslot(uint64_t key, uint32_t mask) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32) & mask;
}

// a stored key never equals the empty marker
__device__ __forceinline__ uint64_t table_key(uint64_t h) { return h == kEmptySlot ? kEmptySlot - 1 : h; }

// slot of `key` or -1 when absent
__device__ __forceinline__ int64_t table_find(const uint64_t* __restrict__ keys, uint32_t mask,
                                              uint64_t key) {
  key = table_key(key);
  uint32_t h = vslot(key, mask);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const uint64_t k = keys[h];
    if (k == key) return h;
    if (k == kEmptySlot) return -1;
    h = (h + 1) & mask;
  }
  return -1;
}

// slot of `key`, inserting it when absent; -1 when the table is full
__device__ __forceinline__ int64_t table_insert(uint64_t* keys, uint32_t mask, uint64_t key) {
  key = table_key(key);
  uint32_t h = vslot(key, mask);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long prev =
        atomicCAS(reinterpret_cast<unsigned long long*>(keys + h), kEmptySlot, key);
    if (prev == kEmptySlot || prev == key) return h;
    h = (h + 1) & mask;
  }
  return -1;
}

}  // namespace rs

namespace rs {

// Lanes of the wave grouped by equal key (active lanes only): the mask of this lane's group.
// One iteration per distinct key in the wave; lets one lane per group do the table atomics, so a
// hot key (Zipf head) costs one atomic per wave instead of one per occurrence. Call with every
// lane of the wave present.
__device__ __forceinline__ uint64_t wave_key_group(uint64_t key, bool active) {
  const int lane = __lane_id();
  uint64_t remaining = __ballot(active);
  uint64_t mine = 0;
  while (remaining) {
    const int leader = __builtin_ctzll(remaining);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)key, leader);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(key >> 32), leader);
    const uint64_t k = ((uint64_t)hi << 32) | lo;
    const uint64_t same = __ballot(active && key == k) & remaining;
    if ((same >> lane) & 1) mine = same;
    remaining &= ~same;
  }
  return mine;
}

}  // namespace rs
