// sort.hip — stable LSD radix sort of embedding rows (the `unique` half of Keras'
// _deduplicate_indexed_slices, SURVEY §2.3 row "Gather-gradient + Unique + UnsortedSegmentSum"),
// plus the device-wide scans the dedup and sharding passes use.
//
// Design (MI355X): keys are global table rows (uint32, < 2^31), values are the original
// flattened positions p = b*S + s. Only ceil(log2(n_rows+1)) key bits are sorted, split evenly
// into passes of <= 8 bits. Each pass = per-tile digit histogram → one-block exclusive scan
// over [digit][tile] → stable scatter. Inside a tile each wave owns a contiguous 64*K-key
// stretch; a key's rank among equal digits in its wave comes from a 64-lane ballot match
// (RADIX_BITS ballots, popcount below the lane), so order is exactly the input order.
#include "common.hpp"

namespace rs {

constexpr int kSortThreads = 256;         // 4 waves
constexpr int kSortKeysPerLane = 16;      // K: keys per lane per tile (large sorts)
constexpr int kSortTile = kSortThreads * kSortKeysPerLane;  // 4096 keys per tile
// small sorts (cfg2's 213k ids, DeepFM's 27k, DIEN's tables) take 1024-key tiles: 4x the blocks
// per launch for a latency-bound pass that would otherwise run on a few dozen CUs
// and sorts under 2^17 ids (DeepFM's, EGES' and PinSage's tables) 512-key tiles
constexpr int kSortKeysPerLaneSmall = 4;
constexpr int kSortKeysPerLaneTiny = 2;
constexpr int64_t kSortSmallN = 1 << 20;
constexpr int64_t kSortTinyN = 1 << 17;
static inline int sort_kpl(int64_t n) {
  return n < kSortTinyN ? kSortKeysPerLaneTiny : (n < kSortSmallN ? kSortKeysPerLaneSmall : kSortKeysPerLane);
}
constexpr int kMaxBins = 512;

// match mask: lanes of this wave whose digit equals mine. Lanes whose bit b differs from mine
// are collected as mismatches — ballot(bit) XOR my bit's sign mask, OR-ed per 32-lane half — and
// the match is the valid lanes outside them (≈ 5 VALU per bit, against 9 for a per-lane select
// of the ballot or its complement: the one-workgroup sort is VALU-bound on its single CU)
template <int BITS>
__device__ __forceinline__ uint64_t match_digit(uint32_t digit, bool valid) {
  uint32_t mis_lo = 0u, mis_hi = 0u;
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const uint32_t sgn = (uint32_t)(-(int32_t)((digit >> b) & 1u));  // all ones if my bit is set
    const uint64_t bb = __ballot(sgn != 0u);
    mis_lo |= (uint32_t)bb ^ sgn;
    mis_hi |= (uint32_t)(bb >> 32) ^ sgn;
  }
  return __ballot(valid) & ~(((uint64_t)mis_hi << 32) | mis_lo);
}

// the same over the low nb <= MAXB bits (nb wave-uniform: a skipped bit costs a scalar branch)
template <int MAXB>
__device__ __forceinline__ uint64_t match_digit_n(uint32_t digit, bool valid, int nb) {
  uint32_t mis_lo = 0u, mis_hi = 0u;
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    if (b < nb) {
      const uint32_t sgn = (uint32_t)(-(int32_t)((digit >> b) & 1u));
      const uint64_t bb = __ballot(sgn != 0u);
      mis_lo |= (uint32_t)bb ^ sgn;
      mis_hi |= (uint32_t)(bb >> 32) ^ sgn;
    }
  }
  return __ballot(valid) & ~(((uint64_t)mis_hi << 32) | mis_lo);
}

__device__ __forceinline__ uint64_t lanemask_lt64() {
  int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Key source of pass 0: either a key array or the ids themselves (key = slot offset + id, made
// on the fly by the histogram pass, which also stores it for the later passes).
struct KeyGen {
  const void* ids;
  int32_t dtype;
  const int64_t* slot_offsets;
  int32_t n_slots;
  int64_t n_rows;
  int32_t world;
  int64_t shard_stride;
  int64_t key_space;
  int32_t* err_flag;
  const uint8_t* valid;  // optional: positions with valid[i] == 0 take the sentinel key, unflagged
};

// Sentinel of position i: key_space + its slot, so excluded / OOB positions sort after every
// valid row grouped by slot, each group in position order (the last pass writes them all as
// key_space: the outputs' sentinel value is unchanged). The slot-segmented sort (below) gives the
// same order.
__device__ __forceinline__ uint32_t sentinel_key(const KeyGen& g, int64_t i) {
  const int64_t sl = g.slot_offsets ? i % g.n_slots : 0;
  return static_cast<uint32_t>(g.key_space + sl);
}

__device__ __forceinline__ uint32_t make_key(const KeyGen& g, int64_t i, bool& oob) {
  if (g.valid && !g.valid[i]) return sentinel_key(g, i);  // excluded position
  const int64_t r = global_row(g.ids, g.dtype, i, g.slot_offsets, g.n_slots, g.n_rows);
  if (r < 0) {
    oob = true;
    return sentinel_key(g, i);  // sentinel: sorts after every valid row
  }
  return static_cast<uint32_t>(g.world == 1 ? r : (r % g.world) * g.shard_stride + r / g.world);
}

// histogram: hist[digit * n_tiles + tile]. Equal digits inside a wave are aggregated by a
// ballot match so skewed (Zipf) keys do not serialise on one LDS counter. FROM_IDS: pass 0 of
// an id sort — the keys are made from the ids here and stored to `keys` for the later passes.
template <int BITS, bool FROM_IDS, int KPL = kSortKeysPerLane>
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(
    uint32_t* __restrict__ keys, KeyGen kg, int64_t n, int shift, int32_t* __restrict__ hist,
    int n_tiles) {
  constexpr int BINS = 1 << BITS;
  constexpr int kMaxLdsSlots = 128;
  __shared__ int32_t cnt[BINS];
  __shared__ int64_t offs[FROM_IDS ? kMaxLdsSlots + 1 : 1];
  for (int d = threadIdx.x; d < BINS; d += blockDim.x) cnt[d] = 0;
  // pass 0 of an id sort: the slot offsets in LDS and the slot from a 32-bit modulo (n < 2^31)
  // instead of a 64-bit one and two global loads per key
  const bool lds_slots = FROM_IDS && kg.slot_offsets && kg.n_slots <= kMaxLdsSlots;
  if (lds_slots)
    for (int e = threadIdx.x; e <= kg.n_slots; e += blockDim.x) offs[e] = kg.slot_offsets[e];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t base = (int64_t)blockIdx.x * (kSortThreads * KPL);
  uint32_t kv[KPL];
  bool oob = false;
  // Round 6: the tile's ids (and valid flags) are loaded unguarded, all before any is used (a
  // position past n reads position 0 and is dropped); per element, the compiler waited for each
  // guarded load in turn (tools/isa_wait_audit.py)
  int64_t idv[KPL];
  uint32_t excl = 0u;
  // the batched path: slot offsets in LDS, or no slots at all (one range [0, n_rows))
  const bool batched = FROM_IDS && (lds_slots || !kg.slot_offsets);
  if (batched) {
    if (kg.dtype == RS_ID_I64) {
#pragma unroll
      for (int k = 0; k < KPL; ++k) {
        const int64_t i = base + (int64_t)k * kSortThreads + threadIdx.x;
        idv[k] = static_cast<const int64_t*>(kg.ids)[i < n ? i : 0];
      }
    } else {
#pragma unroll
      for (int k = 0; k < KPL; ++k) {
        const int64_t i = base + (int64_t)k * kSortThreads + threadIdx.x;
        idv[k] = static_cast<const int32_t*>(kg.ids)[i < n ? i : 0];
      }
    }
    if (kg.valid) {
      uint8_t f[KPL];
#pragma unroll
      for (int k = 0; k < KPL; ++k) {
        const int64_t i = base + (int64_t)k * kSortThreads + threadIdx.x;
        f[k] = kg.valid[i < n ? i : 0];
      }
#pragma unroll
      for (int k = 0; k < KPL; ++k) excl |= (uint32_t)(f[k] == 0) << k;
    }
  } else if (!FROM_IDS) {
#pragma unroll
    for (int k = 0; k < KPL; ++k) {
      const int64_t i = base + (int64_t)k * kSortThreads + threadIdx.x;
      kv[k] = keys[i < n ? i : 0];
    }
  }
#pragma unroll
  for (int k = 0; k < KPL; ++k) {
    const int64_t i = base + (int64_t)k * kSortThreads + threadIdx.x;
    if (FROM_IDS) {
      if (batched) {
        uint32_t key = 0u;
        const int sl = lds_slots ? (int)((uint32_t)i % (uint32_t)kg.n_slots) : 0;
        if (i < n && ((excl >> k) & 1u)) {
          key = static_cast<uint32_t>(kg.key_space + sl);  // excluded position: sentinel, unflagged
          keys[i] = key;
        } else if (i < n) {
          const int64_t id = idv[k];
          const int64_t lo = lds_slots ? offs[sl] : 0, hi = lds_slots ? offs[sl + 1] : kg.n_rows;
          if (id < 0 || id >= hi - lo) {
            oob = true;
            key = static_cast<uint32_t>(kg.key_space + sl);  // sentinel: sorts after every valid row
          } else {
            const int64_t r = lo + id;
            key = static_cast<uint32_t>(kg.world == 1 ? r
                                                       : (r % kg.world) * kg.shard_stride + r / kg.world);
          }
          keys[i] = key;
        }
        kv[k] = key;
      } else {
        kv[k] = i < n ? make_key(kg, i, oob) : 0u;
        if (i < n) keys[i] = kv[k];
      }
    } else {
      kv[k] = i < n ? kv[k] : 0u;
    }
  }
#pragma unroll
  for (int k = 0; k < KPL; ++k) {
    const int64_t i = base + (int64_t)k * kSortThreads + threadIdx.x;
    const bool valid = i < n;
    const uint32_t d = (kv[k] >> shift) & (BINS - 1);
    const uint64_t m = match_digit<BITS>(d, valid);
    // lowest lane of each match group adds the group size
    if (valid && (m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane)))) == 0)
      atomicAdd(&cnt[d], __popcll(m));
  }
  if (FROM_IDS && __any(oob) && lane == 0) flag_oob(kg.err_flag);
  __syncthreads();
  for (int d = threadIdx.x; d < BINS; d += blockDim.x) hist[(int64_t)d * n_tiles + blockIdx.x] = cnt[d];
}

// per-digit scan over the tiles: one wave per digit turns hist[d][*] into its exclusive
// prefix in place and writes the digit's total (the scatter adds the digit bases itself)
constexpr int kColChunks = 8;  // tiles per lane per round: 512 tiles in one round
__global__ __launch_bounds__(256) void radix_colscan_kernel(int32_t* __restrict__ hist, int n_tiles,
                                                            int bins, int32_t* __restrict__ totals) {
  const int d = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (d >= bins) return;
  int32_t* row = hist + (int64_t)d * n_tiles;
  int32_t carry = 0;
  for (int base = 0; base < n_tiles; base += 64 * kColChunks) {
    int32_t v[kColChunks];
    // lane owns kColChunks consecutive tiles: the loads of a round are issued together
#pragma unroll
    for (int c = 0; c < kColChunks; ++c) {
      const int t = base + lane * kColChunks + c;
      v[c] = t < n_tiles ? row[t] : 0;
    }
    int32_t s = 0;
#pragma unroll
    for (int c = 0; c < kColChunks; ++c) s += v[c];
    int32_t x = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    int32_t run = carry + x - s;
#pragma unroll
    for (int c = 0; c < kColChunks; ++c) {
      const int t = base + lane * kColChunks + c;
      if (t < n_tiles) row[t] = run;
      run += v[c];
    }
    carry += __shfl(x, 63);
  }
  if (lane == 0) totals[d] = carry;
}

// stable scatter. The digit bases (exclusive scan of the digit totals) are formed per block
// in LDS. IOTA_VALS: pass 0 of an id sort — the value of key i is its position i.
// The tile is first reordered by digit in LDS (stable: digit, then input order), then written
// out in that order: consecutive lanes store consecutive addresses of one digit's run instead of
// each lane storing to its own bin (measured before the reorder: pass 0, whose low digits are
// spread over all 512 bins, 31 us; the same pass as direct per-lane stores).
template <int BITS, bool IOTA_VALS, int KPL = kSortKeysPerLane>
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(
    const uint32_t* __restrict__ keys_in, const int32_t* __restrict__ vals_in, int64_t n, int shift,
    const int32_t* __restrict__ hist_scanned, const int32_t* __restrict__ totals, int n_tiles,
    uint32_t* __restrict__ keys_out, int32_t* __restrict__ vals_out, uint32_t clamp_key) {
  constexpr int BINS = 1 << BITS;
  constexpr int WAVES = kSortThreads / 64;
  constexpr int PER = (BINS + kSortThreads - 1) / kSortThreads;  // digits per thread
  __shared__ int32_t wcnt[WAVES][BINS];  // per-wave running counts, then per-wave offsets in digit
  __shared__ int32_t lstart[BINS];       // digit start inside the tile's reordered keys
  __shared__ int32_t doff[BINS];         // global destination of reordered slot j = doff[d] + j
  __shared__ int32_t wsum[2][WAVES];
  __shared__ uint32_t sk[kSortThreads * KPL];
  __shared__ int32_t sv[kSortThreads * KPL];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int d = threadIdx.x; d < WAVES * BINS; d += blockDim.x) (&wcnt[0][0])[d] = 0;

  const int64_t tile0 = (int64_t)blockIdx.x * (kSortThreads * KPL);
  const int64_t base = tile0 + (int64_t)wave * 64 * KPL;
  uint32_t key[KPL];
  int32_t val[KPL];
  int32_t rank[KPL];
#pragma unroll
  for (int k = 0; k < KPL; ++k) {
    int64_t i = base + k * 64 + lane;
    bool valid = i < n;
    key[k] = valid ? keys_in[i] : 0u;
    val[k] = IOTA_VALS ? static_cast<int32_t>(i) : (valid ? vals_in[i] : 0);
  }
  // per-thread digit totals and tile counts are scanned below over digits d = tid*PER + c
  int32_t tot[PER];
#pragma unroll
  for (int c = 0; c < PER; ++c) {
    const int d = threadIdx.x * PER + c;
    tot[c] = d < BINS ? totals[d] : 0;
  }
  __syncthreads();  // wcnt zeroed
  const uint64_t lt = lanemask_lt64();
#pragma unroll
  for (int k = 0; k < KPL; ++k) {
    int64_t i = base + k * 64 + lane;
    bool valid = i < n;
    uint32_t d = (key[k] >> shift) & (BINS - 1);
    uint64_t m = match_digit<BITS>(d, valid);
    int32_t before = __popcll(m & lt);
    int32_t prev = valid ? wcnt[wave][d] : 0;
    rank[k] = prev + before;
    // the highest lane of each match group publishes the new count (after all lanes read)
    __builtin_amdgcn_wave_barrier();
    if (valid && (m >> lane) == 1ull) wcnt[wave][d] = prev + before + 1;
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // per digit: tile count (per-wave counts -> offsets inside the digit's run), then one block
  // scan over the digits of both the global totals and the tile counts
  int32_t cnt[PER];
  int32_t s_tot = 0, s_cnt = 0;
#pragma unroll
  for (int c = 0; c < PER; ++c) {
    const int d = threadIdx.x * PER + c;
    int32_t run = 0;
    if (d < BINS) {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) {
        const int32_t t = wcnt[w][d];
        wcnt[w][d] = run;
        run += t;
      }
    }
    cnt[c] = run;
    s_tot += tot[c];
    s_cnt += run;
  }
  int32_t x_tot = s_tot, x_cnt = s_cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t a = __shfl_up(x_tot, off), b = __shfl_up(x_cnt, off);
    if (lane >= off) {
      x_tot += a;
      x_cnt += b;
    }
  }
  if (lane == 63) {
    wsum[0][wave] = x_tot;
    wsum[1][wave] = x_cnt;
  }
  __syncthreads();
  int32_t run_tot = x_tot - s_tot, run_cnt = x_cnt - s_cnt;
  for (int w = 0; w < wave; ++w) {
    run_tot += wsum[0][w];
    run_cnt += wsum[1][w];
  }
#pragma unroll
  for (int c = 0; c < PER; ++c) {
    const int d = threadIdx.x * PER + c;
    if (d < BINS) {
      lstart[d] = run_cnt;
      doff[d] = run_tot + hist_scanned[(int64_t)d * n_tiles + blockIdx.x] - run_cnt;
    }
    run_tot += tot[c];
    run_cnt += cnt[c];
  }
  __syncthreads();
  // reorder the tile by digit in LDS (stable)
#pragma unroll
  for (int k = 0; k < KPL; ++k) {
    int64_t i = base + k * 64 + lane;
    if (i < n) {
      const uint32_t d = (key[k] >> shift) & (BINS - 1);
      const int32_t j = lstart[d] + wcnt[wave][d] + rank[k];
      sk[j] = key[k];
      sv[j] = val[k];
    }
  }
  __syncthreads();
  const int tile_n = (int)(n - tile0 < kSortThreads * KPL ? n - tile0 : kSortThreads * KPL);
  for (int j = threadIdx.x; j < tile_n; j += kSortThreads) {
    const uint32_t k = sk[j];
    const int32_t dst = doff[(k >> shift) & (BINS - 1)] + j;
    keys_out[dst] = k < clamp_key ? k : clamp_key;  // the last pass folds the slot sentinels
    vals_out[dst] = sv[j];
  }
}

// count distinct valid rows in a sorted key array (one atomic per block). Each thread takes 4
// consecutive keys in one 16-byte load (the key before them from the previous thread's group, an
// L1 hit), grid-strided: the whole array is in flight at once (the one-key-per-iteration loop it
// replaces walked 13 dependent loads per thread: 12.7 us at the north star's 1.7 M keys)
__global__ __launch_bounds__(256) void count_unique_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                           uint32_t n_rows, int32_t* __restrict__ n_unique) {
  __shared__ int32_t red[4];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int32_t c = 0;
  const bool vec = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
  const int64_t n4 = vec ? n / 4 : 0;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n4; q += stride) {
    const uint4 k = reinterpret_cast<const uint4*>(keys)[q];
    const uint32_t prev = q > 0 ? keys[4 * q - 1] : ~0u;
    c += (k.x < n_rows && (q == 0 || k.x != prev)) ? 1 : 0;
    c += (k.y < n_rows && k.y != k.x) ? 1 : 0;
    c += (k.z < n_rows && k.z != k.y) ? 1 : 0;
    c += (k.w < n_rows && k.w != k.z) ? 1 : 0;
  }
  for (int64_t i = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t k = keys[i];
    c += (k < n_rows && (i == 0 || keys[i - 1] != k)) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t t = red[0] + red[1] + red[2] + red[3];
    if (t) atomicAdd(n_unique, t);
  }
}

__global__ void head_flags_u32_kernel(const uint32_t* __restrict__ keys, int64_t n, uint32_t key_space,
                                      int32_t* __restrict__ flags) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t k = keys[i];
    flags[i] = (k < key_space && (i == 0 || keys[i - 1] != k)) ? 1 : 0;
  }
}

// unique keys, inverse map and per-owner counts from the sorted keys (excl = exclusive scan of
// the head flags): uniq[seg] = key, inverse[pos[k]] = seg for valid keys, -1 for OOB ones.
__global__ void unique_inverse_kernel(const uint32_t* __restrict__ keys, const int32_t* __restrict__ pos,
                                      const int32_t* __restrict__ excl, int64_t n, uint32_t key_space,
                                      uint32_t* __restrict__ uniq, int32_t* __restrict__ inverse) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    const uint32_t k = keys[i];
    const bool valid = k < key_space;
    const bool head = valid && (i == 0 || keys[i - 1] != k);
    const int32_t seg = excl[i] + (head ? 1 : 0) - 1;
    if (head) uniq[seg] = k;
    inverse[pos[i]] = valid ? seg : -1;
  }
}

// owner_counts[o] = #unique keys in [o*stride, (o+1)*stride) (uniq sorted ascending)
__global__ void owner_counts_kernel(const uint32_t* __restrict__ uniq, const int32_t* __restrict__ n_unique,
                                    int64_t shard_stride, int32_t world, int32_t* __restrict__ counts) {
  const int o = threadIdx.x;
  if (o >= world) return;
  const int32_t nu = *n_unique;
  auto lb = [&](int64_t v) {
    int32_t lo = 0, hi = nu;
    while (lo < hi) {
      int32_t mid = (lo + hi) >> 1;
      if ((int64_t)uniq[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  counts[o] = lb((int64_t)(o + 1) * shard_stride) - lb((int64_t)o * shard_stride);
}

static int key_bits_for(int64_t n_rows) {
  // keys are in [0, n_rows] (n_rows = OOB sentinel)
  int b = 1;
  while (b < 32 && ((int64_t)1 << b) <= n_rows) ++b;
  return b;
}

struct SortPlan {
  int passes;
  int bits;   // per pass
  int kpl;    // keys per lane per tile
  int n_tiles;
};

static SortPlan plan_sort(int64_t n_ids, int64_t n_rows) {
  SortPlan p;
  int kb = key_bits_for(n_rows);
  p.passes = (kb + 8) / 9;  // digits of <= 9 bits (512 bins): 3 passes for 40M rows
  p.bits = (kb + p.passes - 1) / p.passes;
  p.kpl = sort_kpl(n_ids);
  p.n_tiles = (int)ceil_div(n_ids, (int64_t)kSortThreads * p.kpl);
  return p;
}

int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* total, void* ws,
                           size_t ws_bytes, hipStream_t st);
size_t exclusive_scan_ws_size(int64_t n);

// workspace: keys_alt[n], vals_alt[n], hist[BINS * n_tiles], digit totals[BINS]
static size_t sort_ws_layout(int64_t n_ids, Carver& c, uint32_t** keys_alt, int32_t** vals_alt,
                             int32_t** hist, int32_t** totals) {
  int n_tiles = (int)ceil_div(n_ids, (int64_t)kSortThreads * sort_kpl(n_ids));
  *keys_alt = c.take<uint32_t>(n_ids);
  *vals_alt = c.take<int32_t>(n_ids);
  *hist = c.take<int32_t>((size_t)kMaxBins * n_tiles + 1);
  *totals = c.take<int32_t>(kMaxBins);
  return c.off;
}

// one LSD pass = 3 launches: tile histograms, per-digit scan over tiles, stable scatter
template <int BITS, bool FIRST_FROM_IDS, int KPL>
static int32_t launch_pass_k(uint32_t* kin, const int32_t* vin, uint32_t* kout, int32_t* vout,
                             int64_t n, int shift, int32_t* hist, int32_t* totals, int n_tiles,
                             const KeyGen& kg, hipStream_t st, uint32_t clamp_key) {
  radix_hist_kernel<BITS, FIRST_FROM_IDS, KPL><<<n_tiles, kSortThreads, 0, st>>>(kin, kg, n, shift,
                                                                                 hist, n_tiles);
  RS_CHECK_LAUNCH();
  constexpr int BINS = 1 << BITS;
  radix_colscan_kernel<<<(BINS + 3) / 4, 256, 0, st>>>(hist, n_tiles, BINS, totals);
  RS_CHECK_LAUNCH();
  radix_scatter_kernel<BITS, FIRST_FROM_IDS, KPL><<<n_tiles, kSortThreads, 0, st>>>(
      kin, vin, n, shift, hist, totals, n_tiles, kout, vout, clamp_key);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

template <int BITS, bool FIRST_FROM_IDS>
static int32_t launch_pass(uint32_t* kin, const int32_t* vin, uint32_t* kout, int32_t* vout,
                           int64_t n, int shift, int32_t* hist, int32_t* totals, int n_tiles,
                           const KeyGen& kg, hipStream_t st, uint32_t clamp_key) {
  if (sort_kpl(n) == kSortKeysPerLaneTiny)
    return launch_pass_k<BITS, FIRST_FROM_IDS, kSortKeysPerLaneTiny>(kin, vin, kout, vout, n, shift,
                                                                     hist, totals, n_tiles, kg, st,
                                                                     clamp_key);
  if (sort_kpl(n) == kSortKeysPerLaneSmall)
    return launch_pass_k<BITS, FIRST_FROM_IDS, kSortKeysPerLaneSmall>(kin, vin, kout, vout, n, shift,
                                                                      hist, totals, n_tiles, kg, st,
                                                                      clamp_key);
  return launch_pass_k<BITS, FIRST_FROM_IDS, kSortKeysPerLane>(kin, vin, kout, vout, n, shift, hist,
                                                               totals, n_tiles, kg, st, clamp_key);
}

template <bool FIRST_FROM_IDS>
static int32_t dispatch_pass(int bits, uint32_t* kin, const int32_t* vin, uint32_t* kout,
                             int32_t* vout, int64_t n, int shift, int32_t* hist, int32_t* totals,
                             int n_tiles, const KeyGen& kg, hipStream_t st, uint32_t clamp_key) {
#define RS_PASS(B) \
  case B: return launch_pass<B, FIRST_FROM_IDS>(kin, vin, kout, vout, n, shift, hist, totals, n_tiles, kg, st, clamp_key);
  switch (bits) {
    RS_PASS(1) RS_PASS(2) RS_PASS(3) RS_PASS(4) RS_PASS(5) RS_PASS(6) RS_PASS(7) RS_PASS(8) RS_PASS(9)
  }
#undef RS_PASS
  set_error("radix pass bits %d unsupported", bits);
  return RS_E_UNSUPPORTED;
}

// Sort (keys, vals) ascending by key (stable); result ends in keys_out/vals_out.
// keys_in/vals_in are clobbered. kg != null: the keys are made from ids in pass 0 (keys_in is
// then only scratch and vals are the positions 0..n-1; vals_in is not read), sentinels are
// kg->key_space + slot and the output keys are clamped to kg->key_space. Keys are <= max_key.
static int32_t radix_sort_impl(uint32_t* keys_in, int32_t* vals_in, uint32_t* keys_out,
                               int32_t* vals_out, int64_t n, int64_t max_key, void* ws,
                               size_t ws_bytes, const KeyGen* kg, hipStream_t st) {
  SortPlan p = plan_sort(n, max_key);
  Carver c(ws, ws_bytes);
  uint32_t* kalt;
  int32_t* valt;
  int32_t* hist;
  int32_t* totals;
  sort_ws_layout(n, c, &kalt, &valt, &hist, &totals);
  if (!c.ok()) {
    set_error("sort workspace too small: need %zu have %zu", c.off, ws_bytes);
    return RS_E_WORKSPACE;
  }
  // A = (keys_in, vals_in), B = (kalt, valt): A→B→A… and the last pass writes the output
  uint32_t* ka = keys_in;
  int32_t* va = vals_in;
  const KeyGen none{};
  for (int pass = 0; pass < p.passes; ++pass) {
    bool last = pass == p.passes - 1;
    uint32_t* kb = last ? keys_out : (ka == keys_in ? kalt : keys_in);
    int32_t* vb = last ? vals_out : (va == vals_in ? valt : vals_in);
    const uint32_t clamp = (last && kg) ? static_cast<uint32_t>(kg->key_space) : 0xFFFFFFFFu;
    int32_t s = (pass == 0 && kg)
                    ? dispatch_pass<true>(p.bits, ka, va, kb, vb, n, 0, hist, totals, p.n_tiles, *kg, st,
                                          clamp)
                    : dispatch_pass<false>(p.bits, ka, va, kb, vb, n, pass * p.bits, hist, totals,
                                           p.n_tiles, none, st, clamp);
    if (s) return s;
    ka = kb;
    va = vb;
  }
  return RS_OK;
}

int32_t radix_sort_pairs(uint32_t* keys_in, int32_t* vals_in, uint32_t* keys_out,
                         int32_t* vals_out, int64_t n, int64_t n_rows, void* ws, size_t ws_bytes,
                         hipStream_t st) {
  return radix_sort_impl(keys_in, vals_in, keys_out, vals_out, n, n_rows, ws, ws_bytes, nullptr, st);
}

size_t radix_sort_ws_size(int64_t n) {
  Carver c(nullptr, 0);
  uint32_t* a;
  int32_t* b;
  int32_t* h;
  int32_t* t;
  return sort_ws_layout(n, c, &a, &b, &h, &t) + 256;
}

// single-block exclusive scan, in place (n up to a few 100k): the 1024 threads sweep the
// array in coalesced 4096-element stripes; a stripe is scanned in LDS and carried forward.
__global__ __launch_bounds__(1024) void scan_single_block_kernel(int32_t* __restrict__ a, int64_t n,
                                                                 int32_t* __restrict__ total) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry_s;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) carry_s = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += 4096) {
    // each thread owns 4 consecutive elements of the stripe
    int32_t v[4];
    int64_t i0 = base + (int64_t)t * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (i0 + k < n) ? a[i0 + k] : 0;
    int32_t s = v[0] + v[1] + v[2] + v[3];
    // inclusive wave scan
    int32_t x = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      int32_t y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (t < 16) {
      int32_t ws = wsum[t];
      int32_t xs = ws;
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        int32_t y = __shfl_up(xs, off, 16);
        if ((t & 15) >= off) xs += y;
      }
      wsum[t] = xs - ws;  // exclusive over waves
    }
    __syncthreads();
    int32_t run = carry_s + wsum[w] + x - s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < n) a[i0 + k] = run;
      run += v[k];
    }
    __syncthreads();
    if (t == 1023) carry_s = run;
    __syncthreads();
  }
  if (t == 0 && total) *total = carry_s;
}

// ---- device-wide exclusive scan of int32 (3-phase) -----------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanPerThread = 16;
constexpr int kScanTile = kScanThreads * kScanPerThread;

__global__ __launch_bounds__(kScanThreads) void scan_tile_sums_kernel(const int32_t* __restrict__ in,
                                                                      int64_t n,
                                                                      int32_t* __restrict__ sums) {
  __shared__ int32_t red[kScanThreads / 64];
  int64_t base = (int64_t)blockIdx.x * kScanTile;
  int32_t s = 0;
  int32_t v[kScanPerThread];  // every load issued first (guarded, each was waited for in turn)
#pragma unroll
  for (int k = 0; k < kScanPerThread; ++k) {
    const int64_t i = base + (int64_t)k * kScanThreads + threadIdx.x;
    v[k] = in[i < n ? i : 0];
  }
#pragma unroll
  for (int k = 0; k < kScanPerThread; ++k)
    if (base + (int64_t)k * kScanThreads + threadIdx.x < n) s += v[k];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t t = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) t += red[w];
    sums[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kScanThreads) void scan_tile_apply_kernel(const int32_t* __restrict__ in,
                                                                       int64_t n,
                                                                       const int32_t* __restrict__ sums,
                                                                       int32_t* __restrict__ out) {
  // each thread scans a contiguous run of kScanPerThread elements
  __shared__ int32_t part[kScanThreads];
  int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPerThread;
  int32_t v[kScanPerThread];
  int32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPerThread; ++k) {
    int64_t i = base + k;
    v[k] = i < n ? in[i] : 0;
    s += v[k];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < kScanThreads; off <<= 1) {
    int32_t t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += t;
    __syncthreads();
  }
  int32_t run = sums[blockIdx.x] + (threadIdx.x ? part[threadIdx.x - 1] : 0);
#pragma unroll
  for (int k = 0; k < kScanPerThread; ++k) {
    int64_t i = base + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
}

size_t exclusive_scan_ws_size(int64_t n) { return align_up((ceil_div(n, kScanTile) + 1) * 4, 256); }

// out may alias in. total (device, may be null) receives the sum.
int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* total, void* ws,
                           size_t ws_bytes, hipStream_t st) {
  int64_t tiles = ceil_div(n, kScanTile);
  if (ws_bytes < exclusive_scan_ws_size(n)) {
    set_error("scan workspace too small");
    return RS_E_WORKSPACE;
  }
  int32_t* sums = static_cast<int32_t*>(ws);
  if (n == 0) {
    if (total) RS_CHECK_HIP(hipMemsetAsync(total, 0, 4, st));
    return RS_OK;
  }
  scan_tile_sums_kernel<<<tiles, kScanThreads, 0, st>>>(in, n, sums);
  RS_CHECK_LAUNCH();
  scan_single_block_kernel<<<1, 1024, 0, st>>>(sums, tiles, total);
  RS_CHECK_LAUNCH();
  scan_tile_apply_kernel<<<tiles, kScanThreads, 0, st>>>(in, n, sums, out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

// ---- slot-segmented sort (one GPU; BASELINE north star: 26 slots x 65 536 examples) ---------
// The sorted order is (slot, id) for valid positions, then the sentinels grouped by slot (each
// in position order): the slot of position p = b·S + s is known from p, so the order over slots
// needs no sorting pass. Inside a slot, its B ids (rows_s < 2^24) are sorted stably in at most
// two LSD passes of <= 12-bit digits (w0 = min(bits_s, 12) low bits, then the rest), per
// (slot, tile of 4096 examples) block:
//   hist    the tile's digit counts (uint16 [4096], ballot-aggregated in LDS), its valid and
//           sentinel counts;
//   scatter the block re-reads its slot's tile histograms (<= 32 x 8 KB, L2), forms the digit
//           bases and its own tile prefix in place (no column-scan launch), ranks its keys with
//           per-wave running counts (stable), and writes each key to its final (single-pass
//           slot) or temporary (two-pass slot) place; sentinels go to the end.
// Four launches for the north star's 1.7 M ids (hist, scatter per pass; the second pass only
// over the slots wider than 12 bits), against nine for the three-pass LSD sort. Blocks are
// placed XCD-aware: pass 0 puts the 26 slots' tiles of one example range on one XCD (their ids
// share cache lines), pass 1 puts one slot's tiles on one XCD (its histograms and output stay in
// that XCD's L2).
constexpr int kSegThreads = 256;
#ifndef RS_SEG_KPL
#define RS_SEG_KPL 16
#endif
constexpr int kSegKPL = RS_SEG_KPL;              // keys per thread (A/B builds: 8)
constexpr int kSegTile = kSegThreads * kSegKPL;  // 4096 examples of one slot
constexpr int kSegBits = 12;
constexpr int kSegBins = 1 << kSegBits;
constexpr int kSegMaxTiles = 32 * 16 / kSegKPL;  // tiles per slot: B <= 131 072
constexpr int kSegMaxSlots = 64;
constexpr int kSegMaxBits = 2 * kSegBits;  // slot ids < 2^24
constexpr int kNumXcd = 8;

struct SegArgs {
  const void* ids;
  int32_t dtype;
  const uint8_t* valid;         // optional: 0 = excluded (sentinel, unflagged)
  const int64_t* slot_offsets;  // null: one slot of n_rows rows
  int n_slots;
  int64_t B;                    // examples (ids per slot)
  int tiles;                    // tiles per slot
  int64_t n_rows;
  uint16_t* hist0;              // [n_slots][tiles][4096]
  uint16_t* hist1;
  int32_t* vcnt;                // [n_slots][tiles] valid ids per tile (pass-0 tiles)
  int32_t* scnt;                // [n_slots][tiles] sentinels per tile
  uint2* tmp;                   // [n] (id, position) after pass 0 of a two-pass slot
  uint32_t* keys0;              // [n_slots][tiles][4096] pass-0 keys in tile order (bit 31: sentinel)
  int32_t* starts;              // [2][kSegMaxSlots + 1] valid / sentinel starts per slot (+ totals)
  uint32_t* rows_out;
  int32_t* pos_out;
  int32_t* err_flag;
};

__device__ __forceinline__ int seg_bits(int64_t rows) {  // ids in [0, rows) fit in this many bits
  int b = 0;
  while (b < 31 && ((int64_t)1 << b) < rows) ++b;
  return b;
}

struct SegSlot {
  int64_t lo, rows;
  int w0, w1;
};

// The host picks this form from max_slot_rows (<= 2^24); the widths come from the device
// offsets. A slot wider than 2^24 rows (offsets that disagree with the host's bound) would need
// w1 > 12 and overrun the 4096-bin LDS arrays: the widths are clamped to 12 (no overrun), the
// output is not sorted, and RS_ERRBIT_RANGE is raised instead.
__device__ __forceinline__ SegSlot seg_slot(const SegArgs& a, int s) {
  SegSlot r;
  r.lo = a.slot_offsets ? a.slot_offsets[s] : 0;
  r.rows = a.slot_offsets ? a.slot_offsets[s + 1] - r.lo : a.n_rows;
  const int bits = seg_bits(r.rows);
  r.w0 = bits < kSegBits ? bits : kSegBits;
  r.w1 = bits - r.w0;
  if (r.w1 > kSegBits) {
    r.w1 = kSegBits;
    if (threadIdx.x == 0 && a.err_flag) atomicOr(a.err_flag, RS_ERRBIT_RANGE);
  }
  return r;
}

// pass 0 block → (slot, tile): the slots' tiles of one example range share an XCD
__device__ __forceinline__ void seg_tile0(const SegArgs& a, int& s, int& t) {
  const int x = blockIdx.x % kNumXcd, rest = blockIdx.x / kNumXcd;
  s = rest % a.n_slots;
  t = (rest / a.n_slots) * kNumXcd + x;
}
// pass 1 block → (slot, tile): one slot's tiles share an XCD
__device__ __forceinline__ void seg_tile1(const SegArgs& a, int& s, int& t) {
  const int x = blockIdx.x % kNumXcd, rest = blockIdx.x / kNumXcd;
  const int spx = (a.n_slots + kNumXcd - 1) / kNumXcd;
  s = x + kNumXcd * (rest % spx);
  t = rest / spx;
}

// the tile's keys of pass 0: id (local to the slot) per lane and k; live = a valid id, sent = a
// sentinel (excluded or out of range); wave w owns tile entries [w·64·KPL, (w+1)·64·KPL)
template <bool ID64>
__device__ __forceinline__ void seg_load0(const SegArgs& a, const SegSlot& sl, int s, int t,
                                          uint32_t (&id)[kSegKPL], uint32_t& live,
                                          uint32_t& sent, bool& oob) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // Every load of the tile is issued before any is used: a load guarded per element (b < B,
  // then the valid flag) made the compiler wait for each one in turn (round 6, gfx950 ISA: 16
  // dependent round trips per thread). Positions past B read position 0 and are dropped below.
  int64_t v[kSegKPL];
  int64_t pp[kSegKPL];
  uint32_t inb = 0u;
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) {
    const int64_t b = (int64_t)t * kSegTile + wave * 64 * kSegKPL + k * 64 + lane;
    const bool in = b < a.B;
    inb |= (uint32_t)in << k;
    pp[k] = in ? b * a.n_slots + s : 0;
    v[k] = ID64 ? static_cast<const int64_t*>(a.ids)[pp[k]]
                : static_cast<int64_t>(static_cast<const int32_t*>(a.ids)[pp[k]]);
  }
  uint32_t excl = 0u;
  if (a.valid) {  // uniform: the flags' loads issued together too
    uint8_t f[kSegKPL];
#pragma unroll
    for (int k = 0; k < kSegKPL; ++k) f[k] = a.valid[pp[k]];
#pragma unroll
    for (int k = 0; k < kSegKPL; ++k) excl |= (uint32_t)(f[k] == 0) << k;
  }
  live = 0u;
  sent = 0u;
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) {
    id[k] = 0u;
    if ((inb >> k) & 1u) {
      if ((excl >> k) & 1u) {
        sent |= 1u << k;
      } else if (v[k] < 0 || v[k] >= sl.rows) {
        sent |= 1u << k;
        oob = true;
      } else {
        id[k] = static_cast<uint32_t>(v[k]);
        live |= 1u << k;
      }
    }
  }
}

// the tile's counts as uint16
__device__ __forceinline__ void seg_store_hist(uint16_t* __restrict__ h, const int32_t* cnt, int bins) {
  for (int d = threadIdx.x; d < bins; d += blockDim.x) h[d] = static_cast<uint16_t>(cnt[d]);
}

template <bool ID64>
__global__ __launch_bounds__(kSegThreads) void slot_sort_hist0_kernel(SegArgs a) {
  __shared__ int32_t cnt[kSegBins];
  __shared__ int32_t nsent;
  int s, t;
  seg_tile0(a, s, t);
  if (s >= a.n_slots || t >= a.tiles) return;
  const SegSlot sl = seg_slot(a, s);
  const int bins = 1 << sl.w0;
  for (int d = threadIdx.x; d < bins; d += blockDim.x) cnt[d] = 0;
  if (threadIdx.x == 0) nsent = 0;
  __syncthreads();
  uint32_t id[kSegKPL], live, sent;
  bool oob = false;
  seg_load0<ID64>(a, sl, s, t, id, live, sent, oob);
  const int lane = threadIdx.x & 63;
  const uint32_t mask = (uint32_t)bins - 1u;
  int ns = 0;
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) {
    // one LDS atomic per key: the LDS unit serialises a hot digit's lanes, which costs less
    // than the 12-ballot match that would aggregate them on the VALU
    if ((live >> k) & 1u) atomicAdd(&cnt[id[k] & mask], 1);
    ns += __popcll(__ballot((sent >> k) & 1u));
  }
  if (lane == 0 && ns) atomicAdd(&nsent, ns);
  if (__any(oob) && lane == 0) flag_oob(a.err_flag);
  const int64_t tile = (int64_t)s * a.tiles + t;
  {  // the keys in tile order for the scatter (contiguous; the ids were strided by n_slots)
    const int wave = threadIdx.x >> 6;
    uint32_t* kt = a.keys0 + tile * kSegTile + wave * 64 * kSegKPL + lane;
#pragma unroll
    for (int k = 0; k < kSegKPL; ++k) kt[k * 64] = ((sent >> k) & 1u) ? 0x80000000u : id[k];
  }
  __syncthreads();
  seg_store_hist(a.hist0 + tile * kSegBins, cnt, bins);
  if (threadIdx.x == 0) {
    const int64_t b0 = (int64_t)t * kSegTile;
    const int64_t tn = a.B - b0 < kSegTile ? a.B - b0 : kSegTile;
    a.vcnt[tile] = (int32_t)tn - nsent;
    a.scnt[tile] = nsent;
  }
}

// slot starts: vstart[s] = valid ids of slots < s, sstart[s] = sentinels of slots < s (index
// n_slots: the totals), from the pass-0 tile counts (n_slots x tiles ints, L2 / MALL): every count
// loaded by its own lane in one round trip, summed per slot in LDS, the slot prefix by one wave
__device__ __forceinline__ void seg_slot_starts(const SegArgs& a, int32_t* vstart, int32_t* sstart,
                                                int s, int t, int32_t* spre) {
  if (threadIdx.x <= a.n_slots) {
    vstart[threadIdx.x] = 0;
    sstart[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) *spre = 0;
  __syncthreads();
  // every count's load issued before any is summed (at most kSegMaxSlots x kSegMaxTiles counts:
  // 8 per thread); the sentinels of slot s in tiles before t (this block's sentinel base) summed
  // on the way, instead of a serial loop of dependent loads
  constexpr int kPer = kSegMaxSlots * kSegMaxTiles / kSegThreads;
  const int total = a.n_slots * a.tiles;
  int32_t cv[kPer], cz[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int e = threadIdx.x + i * kSegThreads;
    const int ec = e < total ? e : 0;
    cv[i] = a.vcnt[ec];
    cz[i] = a.scnt[ec];
  }
  int32_t mine = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int e = threadIdx.x + i * kSegThreads;
    if (e < total) {
      const int sl = e / a.tiles;
      if (cv[i]) atomicAdd(&vstart[sl], cv[i]);
      if (cz[i]) atomicAdd(&sstart[sl], cz[i]);
      if (sl == s && e - sl * a.tiles < t) mine += cz[i];
    }
  }
  if (mine) atomicAdd(spre, mine);
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan over the slots (n_slots <= 64), totals at n_slots
    const int lane = threadIdx.x;
    const int32_t v = lane < a.n_slots ? vstart[lane] : 0, z = lane < a.n_slots ? sstart[lane] : 0;
    int32_t xv = v, xz = z;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t yv = __shfl_up(xv, off), yz = __shfl_up(xz, off);
      if (lane >= off) {
        xv += yv;
        xz += yz;
      }
    }
    if (lane < a.n_slots) {
      vstart[lane] = xv - v;
      sstart[lane] = xz - z;
    }
    if (lane == 63) {
      vstart[a.n_slots] = xv;
      sstart[a.n_slots] = xz;
    }
  }
  __syncthreads();
}

// stable in-tile ranks: rank[k] = position of key k among the tile's keys of its digit that
// precede it (waves own consecutive stretches; per-wave running counts, then each digit's
// counts turned into wave offsets). wcnt: [4][kSegBins] uint16 in LDS.
__device__ __forceinline__ void seg_rank(const uint32_t (&dig)[kSegKPL], uint32_t live,
                                         uint16_t (*wcnt)[kSegBins], int bins,
                                         int32_t (&rank)[kSegKPL]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt64();
  for (int e = threadIdx.x; e < 4 * bins; e += blockDim.x) wcnt[e / bins][e % bins] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) {
    const bool lv = (live >> k) & 1u;
    const uint32_t d = dig[k];
    const uint64_t m = match_digit<kSegBits>(d, lv);
    const int32_t before = __popcll(m & lt);
    const int32_t prev = lv ? wcnt[wave][d] : 0;
    rank[k] = prev + before;
    __builtin_amdgcn_wave_barrier();
    if (lv && (m >> lane) == 1ull) wcnt[wave][d] = (uint16_t)(prev + before + 1);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  for (int d = threadIdx.x; d < bins; d += blockDim.x) {
    int32_t run = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int32_t c = wcnt[w][d];
      wcnt[w][d] = (uint16_t)run;
      run += c;
    }
  }
  __syncthreads();
}

// Round 6: the column scan done inside the scatter block (no scan launch, no offs round trip):
// doff[d] = base + (keys of the slot's digits < d) + (keys of digit d in the slot's tiles < t).
// Thread j owns digits [16 j, 16 j + 16): it reads its 32-byte slice of every tile's histogram
// row (the slot's n_tiles rows, L2 / MALL resident: hist0 / hist1 are a few MB), sums them for
// the digit totals and the tiles before t for the column prefix; one block scan of the 256
// thread totals orders the digits. The same sums round 5's separate scan launch formed, so the
// same offsets. wsum: 4 ints of LDS. Ends with a block barrier (doff published).
__device__ __forceinline__ void seg_offsets_inblock(const uint16_t* __restrict__ hist, int n_tiles,
                                                    int t, int bins, int32_t base,
                                                    int32_t* __restrict__ doff, int32_t* wsum) {
  constexpr int PER = kSegBins / kSegThreads;  // 16
  const int d0 = threadIdx.x * PER;
  int32_t tot[PER], pre[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) tot[i] = pre[i] = 0;
  if (d0 < bins) {  // bins >= 16 or a single thread (bins < 16: the first thread alone)
    // eight tiles' rows in flight at a time (one row per loop trip waited for each load in turn:
    // 16 dependent L2 round trips at the north star's 16 tiles per slot)
    constexpr int kBatch = 8;
    for (int u0 = 0; u0 < n_tiles; u0 += kBatch) {
      uint4 q[kBatch][2];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int u = u0 + j < n_tiles ? u0 + j : 0;
        const uint4* row = reinterpret_cast<const uint4*>(hist + (int64_t)u * kSegBins + d0);
        q[j][0] = row[0];
        q[j][1] = row[1];
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int u = u0 + j;
        if (u < n_tiles) {
          const uint32_t w[8] = {q[j][0].x, q[j][0].y, q[j][0].z, q[j][0].w,
                                 q[j][1].x, q[j][1].y, q[j][1].z, q[j][1].w};
#pragma unroll
          for (int i = 0; i < PER; ++i) {
            const int32_t c = d0 + i < bins ? (int32_t)((w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) : 0;
            tot[i] += c;
            if (u < t) pre[i] += c;
          }
        }
      }
    }
  }
  int32_t mine = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) mine += tot[i];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int32_t x = mine;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int32_t run = base + x - mine;
  for (int w = 0; w < wave; ++w) run += wsum[w];
  if (d0 < bins) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (d0 + i < bins) doff[d0 + i] = run + pre[i];
      run += tot[i];
    }
  }
  __syncthreads();
}

template <bool ID64>
__global__ __launch_bounds__(kSegThreads) void slot_sort_scatter0_kernel(SegArgs a) {
  __shared__ uint16_t wcnt[4][kSegBins];
  __shared__ int32_t doff[kSegBins];
  __shared__ int32_t wsent[4];
  int s, t;
  seg_tile0(a, s, t);
  if (s >= a.n_slots || t >= a.tiles) return;
  const SegSlot sl = seg_slot(a, s);
  const int bins = 1 << sl.w0;
  uint32_t id[kSegKPL], live = 0u, sent = 0u;
  {  // the histogram pass's keys (bit 31: sentinel), past the tile's end neither
    const int64_t b0 = (int64_t)t * kSegTile;
    const int tn = (int)(a.B - b0 < kSegTile ? a.B - b0 : kSegTile);
    const int w0 = (threadIdx.x >> 6) * 64 * kSegKPL + (threadIdx.x & 63);
    const uint32_t* kt = a.keys0 + ((int64_t)s * a.tiles + t) * kSegTile + w0;
    uint32_t raw[kSegKPL];  // the whole tile is allocated (and written by hist0): load it all first
#pragma unroll
    for (int k = 0; k < kSegKPL; ++k) raw[k] = kt[k * 64];
#pragma unroll
    for (int k = 0; k < kSegKPL; ++k) {
      const bool in = w0 + k * 64 < tn;
      const uint32_t v = in ? raw[k] : 0u;
      id[k] = v & 0x7FFFFFFFu;
      if (in && (v >> 31)) sent |= 1u << k;
      else if (in) live |= 1u << k;
    }
  }
  // slot starts (valid / sentinel ids of the slots before s) from the pass-0 tile counts, this
  // slot's sentinels in tiles before t, then the digit offsets — all in the block (round 6)
  __shared__ int32_t vstart[kSegMaxSlots + 1], sstart[kSegMaxSlots + 1], wsc[4], spre_sh;
  seg_slot_starts(a, vstart, sstart, s, t, &spre_sh);
  if (s == 0 && t == 0)  // for pass 1 (later launches)
    for (int q = threadIdx.x; q <= a.n_slots; q += blockDim.x) {
      a.starts[q] = vstart[q];
      a.starts[kSegMaxSlots + 1 + q] = sstart[q];
    }
  const int32_t spre = spre_sh;
  seg_offsets_inblock(a.hist0 + (int64_t)s * a.tiles * kSegBins, a.tiles, t, bins, vstart[s], doff,
                      wsc);
  const int32_t n_valid = vstart[a.n_slots];
  const int32_t sent_base = n_valid + sstart[s] + spre;
  uint32_t dig[kSegKPL];
  const uint32_t mask = (uint32_t)bins - 1u;
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) dig[k] = id[k] & mask;
  int32_t rank[kSegKPL];
  seg_rank(dig, live, wcnt, bins, rank);  // its block barriers also publish doff
  // sentinel ranks: waves in order, lanes in order
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt64();
  int32_t srank[kSegKPL];
  int32_t srun = 0;
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) {
    const uint64_t m = __ballot((sent >> k) & 1u);
    srank[k] = srun + __popcll(m & lt);
    srun += __popcll(m);
  }
  if (lane == 0) wsent[wave] = srun;
  __syncthreads();
  int32_t sbase = sent_base;
  for (int w = 0; w < wave; ++w) sbase += wsent[w];
  const bool final_pass = sl.w1 == 0;
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) {
    const int64_t b = (int64_t)t * kSegTile + wave * 64 * kSegKPL + k * 64 + lane;
    const int32_t p = (int32_t)(b * a.n_slots + s);
    if ((live >> k) & 1u) {
      const int32_t dst = doff[dig[k]] + wcnt[wave][dig[k]] + rank[k];
      if (final_pass) {
        a.rows_out[dst] = static_cast<uint32_t>(sl.lo + id[k]);
        a.pos_out[dst] = p;
      } else {
        a.tmp[dst] = make_uint2(id[k], static_cast<uint32_t>(p));
      }
    } else if ((sent >> k) & 1u) {
      const int32_t dst = sbase + srank[k];
      a.rows_out[dst] = static_cast<uint32_t>(a.n_rows);
      a.pos_out[dst] = p;
    }
  }
}

// pass 1 (slots wider than 12 bits): tile t of slot s = tmp[start + 4096 t ..) (its valid ids in
// pass-0 order), digit = id >> w0
__device__ __forceinline__ void seg_load1(const SegArgs& a, int32_t start, int32_t n_s, int t,
                                          uint32_t (&id)[kSegKPL], int32_t (&pos)[kSegKPL],
                                          uint32_t& live) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  live = 0u;
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) {
    const int32_t j = t * kSegTile + wave * 64 * kSegKPL + k * 64 + lane;
    id[k] = 0u;
    pos[k] = 0;
    if (j < n_s) {
      const uint2 e = a.tmp[start + j];
      id[k] = e.x;
      pos[k] = static_cast<int32_t>(e.y);
      live |= 1u << k;
    }
  }
}

__global__ __launch_bounds__(kSegThreads) void slot_sort_hist1_kernel(SegArgs a) {
  __shared__ int32_t cnt[kSegBins];
  int s, t;
  seg_tile1(a, s, t);
  if (s >= a.n_slots || t >= a.tiles) return;
  const SegSlot sl = seg_slot(a, s);
  if (sl.w1 == 0) return;
  const int32_t start = a.starts[s], n_s = a.starts[s + 1] - start;
  if (t * kSegTile >= n_s) return;
  const int bins = 1 << sl.w1;
  uint32_t id[kSegKPL], live;
  int32_t pos[kSegKPL];
  seg_load1(a, start, n_s, t, id, pos, live);
  for (int d = threadIdx.x; d < bins; d += blockDim.x) cnt[d] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k)
    if ((live >> k) & 1u) atomicAdd(&cnt[id[k] >> sl.w0], 1);
  __syncthreads();
  seg_store_hist(a.hist1 + ((int64_t)s * a.tiles + t) * kSegBins, cnt, bins);
}

__global__ __launch_bounds__(kSegThreads) void slot_sort_scatter1_kernel(SegArgs a) {
  __shared__ uint16_t wcnt[4][kSegBins];
  __shared__ int32_t doff[kSegBins];
  int s, t;
  seg_tile1(a, s, t);
  if (s >= a.n_slots || t >= a.tiles) return;
  const SegSlot sl = seg_slot(a, s);
  if (sl.w1 == 0) return;
  const int32_t start = a.starts[s], n_s = a.starts[s + 1] - start;
  if (t * kSegTile >= n_s) return;
  const int bins = 1 << sl.w1;
  uint32_t id[kSegKPL], live;
  int32_t pos[kSegKPL];
  seg_load1(a, start, n_s, t, id, pos, live);
  __shared__ int32_t wsc[4];
  seg_offsets_inblock(a.hist1 + (int64_t)s * a.tiles * kSegBins, (n_s + kSegTile - 1) / kSegTile,
                      t, bins, start, doff, wsc);
  uint32_t dig[kSegKPL];
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) dig[k] = id[k] >> sl.w0;
  int32_t rank[kSegKPL];
  seg_rank(dig, live, wcnt, bins, rank);
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kSegKPL; ++k) {
    if ((live >> k) & 1u) {
      const int32_t dst = doff[dig[k]] + wcnt[wave][dig[k]] + rank[k];
      a.rows_out[dst] = static_cast<uint32_t>(sl.lo + id[k]);
      a.pos_out[dst] = pos[k];
    }
  }
}

// ---------------------------------------------------------------------------------------
// Small sorts in one workgroup (round 5): a one-slot id sort of n <= 16 384 ids over fewer than
// 2^18 - 2 rows (the PinSage pair-term fold, small densifies) as one launch. Entry = key << 14 |
// position in a uint32 (key: the row, or the sentinel n_rows for an excluded / OOB id; entries
// past n: all ones). Wave w owns positions [1024 w, 1024 w + 1024), lane-strided, so (wave,
// round, lane) order is position order. Per digit pass (the key bits in the fewest passes of
// <= 9 bits, split evenly), between two 64 KB LDS buffers:
// counts per (wave, digit) and each entry's rank in its wave from one wave match, per-wave digit
// offsets, then every entry placed (digit base + wave offset + rank in the wave). Output identical to the
// multi-launch forms (stable by position, sentinels after every row).
// ---------------------------------------------------------------------------------------
constexpr int kSmallThreads = 1024, kSmallWaves = kSmallThreads / 64;
constexpr int kSmallMax = 16384, kSmallKPT = kSmallMax / kSmallThreads;  // 16 entries per lane
constexpr int kSmallPosBits = 14;
constexpr int64_t kSmallMaxRows = (int64_t(1) << (32 - kSmallPosBits)) - 2;
constexpr int kSmallDigitMax = 9, kSmallBins = 1 << kSmallDigitMax;  // digits of <= 9 bits

// BOUNDED: only the positions below n take part (sorts well under the capacity); otherwise every
// position does (near the capacity the bounds tests cost more than the few padding entries)
template <bool BOUNDED>
__global__ __launch_bounds__(kSmallThreads) void small_sort_kernel(
    const void* __restrict__ ids, int32_t dtype, int64_t n, const uint8_t* __restrict__ valid,
    const int64_t* __restrict__ slot_offsets, int64_t n_rows, int key_bits,
    uint32_t* __restrict__ rows_out, int32_t* __restrict__ pos_out, int32_t* __restrict__ n_unique,
    int32_t* __restrict__ err_flag) {
  __shared__ uint32_t bufs[2][kSmallMax];
  __shared__ uint16_t wcnt[kSmallWaves][kSmallBins];
  __shared__ int32_t dbase[kSmallBins];
  __shared__ int32_t heads[kSmallWaves];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt64();
  const int64_t lo = slot_offsets ? slot_offsets[0] : 0;
  const int64_t span = slot_offsets ? slot_offsets[1] - lo : n_rows;
  const int own = wave * (kSmallKPT * 64) + lane;  // this lane's first entry; then + 64 per round
  bool oob = false;
#pragma unroll 4
  for (int r = 0; r < kSmallKPT; ++r) {
    const int i = own + r * 64;
    uint32_t e = 0xFFFFFFFFu;
    if (i < n) {
      uint32_t key = (uint32_t)n_rows;  // sentinel
      if (!valid || valid[i]) {
        const int64_t id = load_id(ids, dtype, i);
        if (id >= 0 && id < span) key = (uint32_t)(lo + id);
        else oob = true;
      }
      e = key << kSmallPosBits | (uint32_t)i;
    }
    bufs[0][i] = e;
  }
  if (__any(oob) && lane == 0) flag_oob(err_flag);
  // the key bits in as few passes of <= 9 bits as possible, split evenly (18 bits: 9 + 9)
  const int passes = (key_bits + kSmallDigitMax - 1) / kSmallDigitMax;
  const int per = (key_bits + passes - 1) / passes;
  int cur = 0;
  for (int shift = kSmallPosBits; shift < kSmallPosBits + key_bits; shift += per) {
    const int nb = kSmallPosBits + key_bits - shift < per ? kSmallPosBits + key_bits - shift : per;
    const int bins = 1 << nb;
    const uint32_t dmask = (uint32_t)bins - 1u;
    const uint32_t* src = bufs[cur];
    uint32_t* dst = bufs[cur ^ 1];
    for (int e = threadIdx.x; e < kSmallWaves * kSmallBins; e += kSmallThreads) (&wcnt[0][0])[e] = 0;
    __syncthreads();
    // counts per (wave, digit): each match group's last lane adds the group's size; every
    // entry's rank among its wave's entries of the digit before it is kept for the placing loop
    uint32_t ent[kSmallKPT];
    int32_t rank[kSmallKPT];
    // only positions < n take part (rounds wholly past n are skipped, wave-uniformly): the
    // work scales with n, not with the 16 384-entry capacity
#pragma unroll
    for (int r = 0; r < kSmallKPT; ++r) {
      ent[r] = 0u;
      rank[r] = 0;
      if (!BOUNDED || wave * (kSmallKPT * 64) + r * 64 < n) {
        const bool in = !BOUNDED || own + r * 64 < n;
        ent[r] = src[own + r * 64];
        const uint32_t d = (ent[r] >> shift) & dmask;
        const uint64_t m = match_digit_n<kSmallDigitMax>(d, in, nb);
        const int32_t prev = in ? wcnt[wave][d] : 0;
        rank[r] = prev + __popcll(m & lt);
        __builtin_amdgcn_wave_barrier();
        if (in && (m >> lane) == 1ull) wcnt[wave][d] = (uint16_t)(prev + __popcll(m));
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    if (threadIdx.x < bins) {  // per digit: the waves' counts -> wave offsets, the digit total
      const int d = threadIdx.x;
      int32_t run = 0;
#pragma unroll
      for (int w = 0; w < kSmallWaves; ++w) {
        const int32_t c = wcnt[w][d];
        wcnt[w][d] = (uint16_t)run;
        run += c;
      }
      dbase[d] = run;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the digit totals, bins / 64 per lane
      constexpr int Q = kSmallBins / 64;
      int32_t t[Q], sum = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        t[q] = Q * lane + q < bins ? dbase[Q * lane + q] : 0;
        sum += t[q];
      }
      int32_t x = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
      }
      int32_t run = x - sum;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (Q * lane + q < bins) dbase[Q * lane + q] = run;
        run += t[q];
      }
    }
    __syncthreads();
    // placed: digit base + this wave's offset + the rank in the wave (no second match)
#pragma unroll
    for (int r = 0; r < kSmallKPT; ++r) {
      if (!BOUNDED || own + r * 64 < n) {
        const uint32_t d = (ent[r] >> shift) & dmask;
        dst[dbase[d] + wcnt[wave][d] + rank[r]] = ent[r];
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  // sorted entries out; the heads of distinct rows counted
  const uint32_t* out = bufs[cur];
  int32_t h = 0;
  for (int i = threadIdx.x; i < n; i += kSmallThreads) {
    const uint32_t e = out[i];
    const uint32_t key = e >> kSmallPosBits;
    rows_out[i] = key;
    pos_out[i] = (int32_t)(e & ((1u << kSmallPosBits) - 1u));
    if (key < (uint32_t)n_rows && (i == 0 || (out[i - 1] >> kSmallPosBits) != key)) ++h;
  }
  if (n_unique) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) h += __shfl_xor(h, off);
    if (lane == 0) heads[wave] = h;
    __syncthreads();
    if (threadIdx.x == 0) {
      int32_t t = 0;
      for (int w = 0; w < kSmallWaves; ++w) t += heads[w];
      *n_unique = t;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Sorted runs merged (round 5): the row-sharded slab's owner receives n_runs blocks of run_len
// owner-local rows, each ascending (its source's unique rows in key order) with its padding
// (ids < 0) at the end; the stable sort of all of them by (row, position) is a merge. Element j
// of run s lands at j + Σ_{s' < s} #{run s' rows <= its row} + Σ_{s' > s} #{run s' rows < its
// row} (binary searches of the other runs' valid prefixes); entries past a run's valid prefix
// (padding, rows >= n_rows: flagged) take the sentinel n_rows after every valid row, in position
// order — the masked radix sort's output, in one launch instead of nine.
// ---------------------------------------------------------------------------------------
constexpr int kMaxRuns = 1024;

__global__ __launch_bounds__(256) void runs_merge_kernel(const int32_t* __restrict__ ids, int64_t n,
                                                         int n_runs, int64_t run_len,
                                                         int64_t n_rows, uint32_t* __restrict__ rows_out,
                                                         int32_t* __restrict__ pos_out,
                                                         int32_t* __restrict__ err_flag) {
  __shared__ int64_t vl[kMaxRuns];    // valid prefix length of each run
  __shared__ int64_t padb[kMaxRuns];  // entries past the valid prefixes of the runs before
  __shared__ int64_t nvalid;
  for (int r = threadIdx.x; r < n_runs; r += blockDim.x) {
    const int32_t* run = ids + (int64_t)r * run_len;
    int64_t lo = 0, hi = run_len;  // first index whose id is not a row (monotone predicate)
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      const int32_t v = run[mid];
      if (v >= 0 && v < n_rows) lo = mid + 1;
      else hi = mid;
    }
    vl[r] = lo;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t acc = 0, pad = 0;
    for (int r = 0; r < n_runs; ++r) {
      padb[r] = pad;
      acc += vl[r];
      pad += run_len - vl[r];
    }
    nvalid = acc;
  }
  __syncthreads();
  bool oob = false;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int s = (int)(e / run_len);
    const int64_t j = e - (int64_t)s * run_len;
    const int32_t key = ids[e];
    int64_t out;
    uint32_t kout;
    if (j < vl[s]) {
      out = j;
      for (int r = 0; r < n_runs; ++r) {
        if (r == s) continue;
        const int32_t* run = ids + (int64_t)r * run_len;
        int64_t lo = 0, hi = vl[r];
        if (r < s) {  // upper bound: equal rows of earlier runs come first
          while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (run[mid] <= key) lo = mid + 1; else hi = mid;
          }
        } else {      // lower bound
          while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (run[mid] < key) lo = mid + 1; else hi = mid;
          }
        }
        out += lo;
      }
      kout = (uint32_t)key;
    } else {
      out = nvalid + padb[s] + (j - vl[s]);
      kout = (uint32_t)n_rows;
      if (key >= n_rows) oob = true;
    }
    rows_out[out] = kout;
    pos_out[out] = (int32_t)e;
  }
  if (__any(oob) && (threadIdx.x & 63) == 0) flag_oob(err_flag);
}

static bool small_eligible(int64_t n_ids, int n_slots, int world, int64_t n_rows) {
  return world == 1 && n_slots == 1 && n_ids >= 1 && n_ids <= kSmallMax && n_rows <= kSmallMaxRows;
}

static int32_t small_sort(const void* ids, int32_t id_dtype, int64_t n_ids, const uint8_t* valid,
                          const int64_t* slot_offsets, int64_t n_rows, uint32_t* sorted_rows,
                          int32_t* sorted_pos, int32_t* n_unique, int32_t* err_flag, hipStream_t st) {
  int key_bits = 1;
  while (key_bits < 32 - kSmallPosBits && (int64_t(1) << key_bits) <= n_rows) ++key_bits;  // keys <= n_rows
  if (n_ids <= kSmallMax * 3 / 4)
    small_sort_kernel<true><<<1, kSmallThreads, 0, st>>>(ids, id_dtype, n_ids, valid, slot_offsets,
                                                          n_rows, key_bits, sorted_rows, sorted_pos,
                                                          n_unique, err_flag);
  else
    small_sort_kernel<false><<<1, kSmallThreads, 0, st>>>(ids, id_dtype, n_ids, valid, slot_offsets, n_rows,
                                                 key_bits, sorted_rows, sorted_pos, n_unique,
                                                 err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

static size_t seg_ws_layout(int64_t n, int n_slots, int tiles, Carver& c, SegArgs* a) {
  const size_t nt = (size_t)n_slots * tiles;
  uint32_t* k0 = c.take<uint32_t>(nt * kSegTile);
  uint16_t* h0 = c.take<uint16_t>(nt * kSegBins);
  uint16_t* h1 = c.take<uint16_t>(nt * kSegBins);
  int32_t* v = c.take<int32_t>(nt);
  int32_t* z = c.take<int32_t>(nt);
  int32_t* st = c.take<int32_t>(2 * (kSegMaxSlots + 1));
  uint2* tmp = c.take<uint2>(n);
  if (a) {
    a->keys0 = k0;
    a->hist0 = h0;
    a->hist1 = h1;
    a->vcnt = v;
    a->scnt = z;
    a->starts = st;
    a->tmp = tmp;
  }
  return c.off;
}

// the slot-segmented sort fits: one GPU, ids [B, n_slots], B <= 32 tiles, every slot < 2^24 rows
static bool seg_eligible(int64_t n_ids, int n_slots, int world, int64_t max_slot_rows) {
  if (world != 1 || n_slots < 1 || n_slots > kSegMaxSlots || n_ids < 1) return false;
  if (n_ids % n_slots) return false;
  const int64_t B = n_ids / n_slots;
  return B <= (int64_t)kSegMaxTiles * kSegTile && max_slot_rows >= 1 &&
         max_slot_rows <= ((int64_t)1 << kSegMaxBits);
}

size_t seg_ws_size(int64_t n_ids) {
  // tiles over all slots <= n/4096 + n_slots (each slot rounds up once)
  const int64_t tiles_total = n_ids / kSegTile + kSegMaxSlots;
  Carver c(nullptr, 0);
  return seg_ws_layout(n_ids, 1, (int)tiles_total, c, nullptr) + 1024;
}

static int32_t seg_sort(const void* ids, int32_t id_dtype, int64_t n_ids, const uint8_t* valid,
                        const int64_t* slot_offsets, int n_slots, int64_t n_rows,
                        uint32_t* sorted_rows, int32_t* sorted_pos, int32_t* err_flag,
                        void* workspace, size_t ws_bytes, hipStream_t st) {
  SegArgs a{};
  a.ids = ids;
  a.dtype = id_dtype;
  a.valid = valid;
  a.slot_offsets = slot_offsets;
  a.n_slots = n_slots;
  a.B = n_ids / n_slots;
  a.tiles = (int)ceil_div(a.B, kSegTile);
  a.n_rows = n_rows;
  a.rows_out = sorted_rows;
  a.pos_out = sorted_pos;
  a.err_flag = err_flag;
  Carver c(workspace, ws_bytes);
  seg_ws_layout(n_ids, n_slots, a.tiles, c, &a);
  if (!c.ok()) {
    set_error("sort workspace too small: need %zu have %zu", c.off, ws_bytes);
    return RS_E_WORKSPACE;
  }
  const int tiles_pad = (int)ceil_div(a.tiles, kNumXcd) * kNumXcd;
  const int grid0 = tiles_pad * n_slots;
  const int spx = (int)ceil_div(n_slots, kNumXcd);
  const int grid1 = kNumXcd * spx * a.tiles;
  if (id_dtype == RS_ID_I64) slot_sort_hist0_kernel<true><<<grid0, kSegThreads, 0, st>>>(a);
  else slot_sort_hist0_kernel<false><<<grid0, kSegThreads, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  if (id_dtype == RS_ID_I64) slot_sort_scatter0_kernel<true><<<grid0, kSegThreads, 0, st>>>(a);
  else slot_sort_scatter0_kernel<false><<<grid0, kSegThreads, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  // pass 1 only matters for slots wider than 12 bits; its blocks of narrower slots exit at once
  slot_sort_hist1_kernel<<<grid1, kSegThreads, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  slot_sort_scatter1_kernel<<<grid1, kSegThreads, 0, st>>>(a);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

}  // namespace rs

using namespace rs;

static int32_t sort_ids_impl(const void* ids, int32_t id_dtype, int64_t n_ids,
                             const int64_t* slot_offsets, int32_t n_slots, int64_t n_rows,
                             int32_t world, uint32_t* sorted_keys, int32_t* sorted_pos,
                             int32_t* n_unique, int32_t* err_flag, void* workspace, size_t ws_bytes,
                             hipStream_t st, const uint8_t* valid, int64_t max_slot_rows);

extern "C" size_t rs_sort_ids_workspace_size(int64_t n_ids) {
  Carver c(nullptr, 0);
  c.take<uint32_t>(n_ids);
  c.take<int32_t>(n_ids);
  const size_t lsd = c.off + radix_sort_ws_size(n_ids) + exclusive_scan_ws_size(n_ids) + 1024;
  const size_t seg = seg_ws_size(n_ids);
  return lsd > seg ? lsd : seg;
}

extern "C" int32_t rs_sort_ids(const void* ids, int32_t id_dtype, int64_t n_ids,
                               const int64_t* slot_offsets, int32_t n_slots, int64_t n_rows,
                               uint32_t* sorted_rows, int32_t* sorted_pos, int32_t* n_unique,
                               int32_t* err_flag, void* workspace, size_t ws_bytes, void* stream) {
  return sort_ids_impl(ids, id_dtype, n_ids, slot_offsets, n_slots, n_rows, 1, sorted_rows,
                       sorted_pos, n_unique, err_flag, workspace, ws_bytes, as_stream(stream), nullptr,
                       n_rows);
}

extern "C" int32_t rs_sort_ids_masked(const void* ids, int32_t id_dtype, int64_t n_ids,
                                      const uint8_t* valid, const int64_t* slot_offsets,
                                      int32_t n_slots, int64_t n_rows, uint32_t* sorted_rows,
                                      int32_t* sorted_pos, int32_t* n_unique, int32_t* err_flag,
                                      void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(valid || n_ids == 0, "valid is null");
  return sort_ids_impl(ids, id_dtype, n_ids, slot_offsets, n_slots, n_rows, 1, sorted_rows,
                       sorted_pos, n_unique, err_flag, workspace, ws_bytes, as_stream(stream), valid,
                       n_rows);
}

extern "C" int32_t rs_sort_ids_slots(const void* ids, int32_t id_dtype, int64_t n_ids,
                                     const uint8_t* valid, const int64_t* slot_offsets,
                                     int32_t n_slots, int64_t n_rows, int64_t max_slot_rows,
                                     uint32_t* sorted_rows, int32_t* sorted_pos, int32_t* n_unique,
                                     int32_t* err_flag, void* workspace, size_t ws_bytes,
                                     void* stream) {
  RS_CHECK_ARG(max_slot_rows >= 1 && max_slot_rows <= n_rows, "max_slot_rows out of range");
  return sort_ids_impl(ids, id_dtype, n_ids, slot_offsets, n_slots, n_rows, 1, sorted_rows,
                       sorted_pos, n_unique, err_flag, workspace, ws_bytes, as_stream(stream), valid,
                       max_slot_rows);
}

extern "C" int32_t rs_sort_ids_sharded(const void* ids, int32_t id_dtype, int64_t n_ids,
                                       const int64_t* slot_offsets, int32_t n_slots, int64_t n_rows,
                                       int32_t world, uint32_t* sorted_keys, int32_t* sorted_pos,
                                       int32_t* n_unique, int32_t* err_flag, void* workspace,
                                       size_t ws_bytes, void* stream) {
  return sort_ids_impl(ids, id_dtype, n_ids, slot_offsets, n_slots, n_rows, world, sorted_keys,
                       sorted_pos, n_unique, err_flag, workspace, ws_bytes, as_stream(stream), nullptr,
                       n_rows);
}

extern "C" size_t rs_unique_inverse_workspace_size(int64_t n_ids) {
  Carver c(nullptr, 0);
  c.take<int32_t>(n_ids > 0 ? n_ids : 1);
  c.take<char>(exclusive_scan_ws_size(n_ids > 0 ? n_ids : 1));
  return c.off + 256;
}

extern "C" int32_t rs_unique_inverse(const uint32_t* sorted_keys, const int32_t* sorted_pos,
                                     int64_t n_ids, int64_t n_rows, int32_t world,
                                     uint32_t* uniq_keys, int32_t* inverse, int32_t* n_unique,
                                     int32_t* owner_counts, void* workspace, size_t ws_bytes,
                                     void* stream) {
  RS_CHECK_ARG(world >= 1 && n_rows > 0 && n_ids >= 0, "bad sizes");
  RS_CHECK_ARG(n_ids == 0 || (sorted_keys && sorted_pos && uniq_keys && inverse && n_unique),
               "null pointer");
  hipStream_t st = as_stream(stream);
  const int64_t stride = ceil_div(n_rows, world);
  const int64_t key_space = world == 1 ? n_rows : stride * world;
  RS_CHECK_HIP(hipMemsetAsync(n_unique, 0, 4, st));
  if (n_ids == 0) {
    if (owner_counts) RS_CHECK_HIP(hipMemsetAsync(owner_counts, 0, 4 * (size_t)world, st));
    return RS_OK;
  }
  Carver c(workspace, ws_bytes);
  int32_t* excl = c.take<int32_t>(n_ids);
  void* scan_ws = c.take<char>(exclusive_scan_ws_size(n_ids));
  if (!c.ok()) {
    set_error("unique workspace too small");
    return RS_E_WORKSPACE;
  }
  int blocks = (int)std::min<int64_t>(ceil_div(n_ids, 256), 4096);
  head_flags_u32_kernel<<<blocks, 256, 0, st>>>(sorted_keys, n_ids, (uint32_t)key_space, excl);
  RS_CHECK_LAUNCH();
  int32_t s = exclusive_scan_i32(excl, excl, n_ids, n_unique, scan_ws, exclusive_scan_ws_size(n_ids), st);
  if (s) return s;
  unique_inverse_kernel<<<blocks, 256, 0, st>>>(sorted_keys, sorted_pos, excl, n_ids,
                                                (uint32_t)key_space, uniq_keys, inverse);
  RS_CHECK_LAUNCH();
  if (owner_counts) {
    owner_counts_kernel<<<1, 64 * ((world + 63) / 64), 0, st>>>(uniq_keys, n_unique, stride, world,
                                                                owner_counts);
    RS_CHECK_LAUNCH();
  }
  return RS_OK;
}

static int32_t sort_ids_impl(const void* ids, int32_t id_dtype, int64_t n_ids,
                             const int64_t* slot_offsets, int32_t n_slots, int64_t n_rows,
                             int32_t world, uint32_t* sorted_rows, int32_t* sorted_pos,
                             int32_t* n_unique, int32_t* err_flag, void* workspace, size_t ws_bytes,
                             hipStream_t st, const uint8_t* valid, int64_t max_slot_rows) {
  RS_CHECK_ARG(n_ids >= 0 && n_ids < (int64_t(1) << 31), "n_ids out of range");
  RS_CHECK_ARG(n_rows > 0 && n_rows < (int64_t(1) << 31) - 1, "n_rows out of range");
  RS_CHECK_ARG(id_dtype == RS_ID_I32 || id_dtype == RS_ID_I64, "bad id dtype");
  RS_CHECK_ARG(n_slots >= 1, "n_slots must be >= 1");
  RS_CHECK_ARG(world >= 1 && world <= 1024, "world out of range");
  RS_CHECK_ARG(ids || n_ids == 0, "ids is null");
  const int64_t shard_stride = ceil_div(n_rows, world);
  const int64_t key_space = world == 1 ? n_rows : shard_stride * world;
  RS_CHECK_ARG(key_space < (int64_t(1) << 31) - 1, "key space out of range");
  if (n_unique) RS_CHECK_HIP(hipMemsetAsync(n_unique, 0, sizeof(int32_t), st));
  if (n_ids == 0) return RS_OK;
  if (small_eligible(n_ids, n_slots, world, n_rows))
    // one workgroup, one launch
    return small_sort(ids, id_dtype, n_ids, valid, slot_offsets, n_rows, sorted_rows, sorted_pos,
                      n_unique, err_flag, st);
  if ((slot_offsets || n_slots == 1) && seg_eligible(n_ids, n_slots, world, max_slot_rows)) {
    // the slot-segmented sort: same output as the LSD form below, six launches
    int32_t s = seg_sort(ids, id_dtype, n_ids, valid, slot_offsets, n_slots, n_rows, sorted_rows,
                         sorted_pos, err_flag, workspace, ws_bytes, st);
    if (s) return s;
    if (n_unique) {
      const int cblocks = (int)std::min<int64_t>(ceil_div(ceil_div(n_ids, 4), 256), 2048);
      count_unique_kernel<<<cblocks, 256, 0, st>>>(sorted_rows, n_ids, (uint32_t)key_space, n_unique);
      RS_CHECK_LAUNCH();
    }
    return RS_OK;
  }
  Carver c(workspace, ws_bytes);
  uint32_t* keys = c.take<uint32_t>(n_ids);
  int32_t* vals = c.take<int32_t>(n_ids);
  size_t rest_off = align_up(c.off, 256);
  if (rest_off > ws_bytes) {
    set_error("sort workspace too small");
    return RS_E_WORKSPACE;
  }
  int blocks = (int)std::min<int64_t>(ceil_div(n_ids, 256), 4096);
  // pass 0 makes the keys from the ids (slot offset + id; owner-major when world > 1)
  const KeyGen kg{ids, id_dtype, slot_offsets, n_slots, n_rows, world, shard_stride, key_space, err_flag,
                  valid};
  const int64_t max_key = key_space + (slot_offsets ? n_slots - 1 : 0);  // slot sentinels
  RS_CHECK_ARG(max_key < (int64_t(1) << 31) - 1, "key space out of range");
  int32_t s = radix_sort_impl(keys, vals, sorted_rows, sorted_pos, n_ids, max_key,
                              static_cast<char*>(workspace) + rest_off, ws_bytes - rest_off, &kg, st);
  if (s) return s;
  if (n_unique) {
    const int cblocks = (int)std::min<int64_t>(ceil_div(ceil_div(n_ids, 4), 256), 2048);
    count_unique_kernel<<<cblocks, 256, 0, st>>>(sorted_rows, n_ids, (uint32_t)key_space, n_unique);
    RS_CHECK_LAUNCH();
  }
  return RS_OK;
}

extern "C" int32_t rs_sort_ids_runs(const int32_t* ids, int64_t n_ids, int32_t n_runs,
                                    int64_t n_rows, uint32_t* sorted_rows, int32_t* sorted_pos,
                                    int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(n_ids >= 0 && n_ids < (int64_t(1) << 31), "n_ids out of range");
  RS_CHECK_ARG(n_runs >= 1 && n_runs <= kMaxRuns && n_ids % n_runs == 0, "n_runs must divide n_ids");
  RS_CHECK_ARG(n_rows > 0 && n_rows < (int64_t(1) << 31) - 1, "n_rows out of range");
  if (n_ids == 0) return RS_OK;
  RS_CHECK_ARG(ids && sorted_rows && sorted_pos, "null pointer");
  const int blocks = (int)std::min<int64_t>(ceil_div(n_ids, 256), 4096);
  runs_merge_kernel<<<blocks, 256, 0, as_stream(stream)>>>(ids, n_ids, n_runs, n_ids / n_runs,
                                                           n_rows, sorted_rows, sorted_pos, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
