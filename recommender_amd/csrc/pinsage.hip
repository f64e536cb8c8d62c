// pinsage.hip — PinSage sampling + aggregation on gfx950.
//
// Graph: bipartite item/user CSR in both directions (int64 indptr, int32 neighbour ids), HBM
// resident (ML-20M: 2 x 20M x 4 B + indptrs ≈ 161 MB, fits the 256 MB Infinity Cache).
//
// Randomness: Philox4x32-10 (Salmon et al., SC'11) keyed by the caller's 64-bit seed and a
// purpose word; counters are (subject id, walk index | layer << 16, step, draw index / 4), so
// every draw is a pure function of (seed, step, subject) — results do not depend on the launch
// shape or on how seeds are sharded over ranks. Bounded ints are the multiply-high
// (r * n) >> 32, so the numpy oracle reproduces them bit for bit.
//
// Kernels:
//   walk / pairs / neighbours : one thread per (seed, walk); 2 dependent loads per hop
//                               (indptr then neighbour) → latency bound, many waves in flight.
//   unique_first              : first-appearance compaction (DGL compact_graphs / to_block
//                               src order) via atomicMin marks + a device scan: deterministic.
//   block                     : CSR by dst + a stable radix-sorted transpose (CSR by src) so the
//                               aggregation backward is a gather, not a float atomic scatter.
//   agg fwd / bwd             : one thread per (row, column), rows coalesced.
//   frobenius                 : fixed-partition two-level reduction, then an elementwise pass.
#include <cmath>

#include "common.hpp"
#include "rng.hpp"

namespace rs {

int32_t radix_sort_pairs(uint32_t* keys_in, int32_t* vals_in, uint32_t* keys_out,
                         int32_t* vals_out, int64_t n, int64_t n_rows, void* ws, size_t ws_bytes,
                         hipStream_t st);
size_t radix_sort_ws_size(int64_t n);
int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* total, void* ws,
                           size_t ws_bytes, hipStream_t st);
size_t exclusive_scan_ws_size(int64_t n);

struct Graph {
  const int64_t* i2u_ptr;
  const int32_t* i2u;
  const int64_t* u2i_ptr;
  const int32_t* u2i;
};

// One uniform transition (DGL random_walk without `prob`): -1 at a dead end.
__device__ __forceinline__ int32_t hop(const int64_t* __restrict__ ptr,
                                       const int32_t* __restrict__ nbr, int32_t node,
                                       uint32_t r) {
  const int64_t lo = ptr[node];
  const int64_t deg = ptr[node + 1] - lo;
  if (deg <= 0) return -1;
  return nbr[lo + bounded(r, (uint32_t)deg)];
}

// Walk item → user → item ... for 2*T hops; visit(t, item) gets the item after traversal t.
// A trace ends at a dead end, or (stop_thr > 0) after a transition whose stop draw < stop_thr.
template <typename F>
__device__ __forceinline__ void metapath(const Graph& g, int32_t start, int32_t T,
                                         uint32_t stop_thr, uint64_t seed, uint32_t purpose,
                                         uint32_t a, uint32_t b, uint32_t step, F&& visit) {
  int32_t node = start;
  bool alive = start >= 0;
  for (int32_t h = 0; h < 2 * T; ++h) {
    if (alive) {
      const uint32_t r = draw(seed, purpose, a, b, step, (uint32_t)h);
      node = (h & 1) ? hop(g.u2i_ptr, g.u2i, node, r) : hop(g.i2u_ptr, g.i2u, node, r);
      alive = node >= 0;
      visit(h, node);
      if (alive && stop_thr && draw(seed, purpose + 1, a, b, step, (uint32_t)h) < stop_thr) {
        alive = false;  // the trace ends after the node just reached
        node = -1;
      }
    } else {
      visit(h, -1);
    }
  }
}

constexpr uint32_t kPurposeWalk = 0x100;  // +1: stop draws
constexpr uint32_t kPurposePair = 0x200;
constexpr uint32_t kPurposePairWalk = 0x300;

__global__ __launch_bounds__(256) void philox_kernel(const uint32_t* __restrict__ ctr, int64_t n,
                                                     uint32_t k0, uint32_t k1,
                                                     uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  U4 r = philox4x32_10(U4{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]}, k0, k1);
  out[4 * i] = r.x;
  out[4 * i + 1] = r.y;
  out[4 * i + 2] = r.z;
  out[4 * i + 3] = r.w;
}

__global__ __launch_bounds__(256) void walk_kernel(Graph g, const int32_t* __restrict__ seeds,
                                                   int64_t n_seeds, int32_t num_walks, int32_t T,
                                                   uint32_t stop_thr, uint64_t seed,
                                                   uint32_t step, uint32_t layer,
                                                   int32_t* __restrict__ traces) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_seeds * num_walks) return;
  const int64_t s = t / num_walks;
  const int32_t j = (int32_t)(t - s * num_walks);
  const int32_t start = seeds[s];
  int32_t* out = traces + t * (2 * T + 1);
  out[0] = start;
  metapath(g, start, T, stop_thr, seed, kPurposeWalk, (uint32_t)start,
           (uint32_t)j | (layer << 16), step, [&](int32_t h, int32_t node) { out[h + 1] = node; });
}

// item2item_batch_sampler (pinsage/train/data_loader.py:6-18): pair i (global index
// pair_base + i) draws head, neg ~ U[0, n_items) and pos = item after one item→user→item walk.
__global__ __launch_bounds__(256) void pairs_gen_kernel(Graph g, int32_t n_items,
                                                        int64_t pair_base, int32_t batch,
                                                        uint64_t seed, uint32_t step_add,
                                                        const uint32_t* __restrict__ step_ptr,
                                                        int32_t* __restrict__ tmp,
                                                        int32_t* __restrict__ flag) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  const uint32_t step = step_add + (step_ptr ? *step_ptr : 0u);
  const uint32_t gi = (uint32_t)(pair_base + i);
  const U4 r = philox4x32_10(U4{gi, 0u, step, 0u}, (uint32_t)seed,
                             (uint32_t)(seed >> 32) ^ kPurposePair);
  const int32_t head = (int32_t)bounded(r.x, (uint32_t)n_items);
  const int32_t neg = (int32_t)bounded(r.y, (uint32_t)n_items);
  int32_t pos = -1;
  metapath(g, head, 1, 0u, seed, kPurposePairWalk, gi, 0u, step,
           [&](int32_t h, int32_t node) { if (h == 1) pos = node; });
  tmp[i] = head;
  tmp[batch + i] = pos;
  tmp[2 * batch + i] = neg;
  flag[i] = pos >= 0;
}

__global__ __launch_bounds__(256) void pairs_compact_kernel(const int32_t* __restrict__ tmp,
                                                            const int32_t* __restrict__ flag,
                                                            const int32_t* __restrict__ offs,
                                                            int32_t batch,
                                                            int32_t* __restrict__ heads,
                                                            int32_t* __restrict__ pos,
                                                            int32_t* __restrict__ neg) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch || !flag[i]) return;
  const int32_t o = offs[i];
  heads[o] = tmp[i];
  pos[o] = tmp[batch + i];
  neg[o] = tmp[2 * batch + i];
}

// ---- (dst, src) pair set: open addressing, linear probing -------------------------------
constexpr uint64_t kEmpty = ~0ull;

__device__ __forceinline__ uint32_t slot_of(uint64_t key, uint32_t mask) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32) & mask;
}

__device__ __forceinline__ uint64_t pair_key(int32_t dst, int32_t src) {
  return ((uint64_t)(uint32_t)dst << 32) | (uint32_t)src;
}

__global__ __launch_bounds__(256) void pair_set_build_kernel(const int32_t* __restrict__ src,
                                                             const int32_t* __restrict__ dst,
                                                             int64_t n, uint64_t* table,
                                                             uint32_t mask) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t s = src[i], d = dst[i];
  if (s < 0 || d < 0) return;
  const uint64_t key = pair_key(d, s);
  uint32_t h = slot_of(key, mask);
  for (;;) {
    const unsigned long long prev =
        atomicCAS(reinterpret_cast<unsigned long long*>(table + h), kEmpty, key);
    if (prev == kEmpty || prev == key) return;
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ bool pair_set_has(const uint64_t* __restrict__ table, uint32_t mask,
                                             uint64_t key) {
  uint32_t h = slot_of(key, mask);
  for (;;) {
    const uint64_t v = table[h];
    if (v == key) return true;
    if (v == kEmpty) return false;
    h = (h + 1) & mask;
  }
}

// ---- PinSAGESampler (a-15): walks + visit counts + top-k + leak-edge removal -------------
// Block = 256 threads = (256 >> wshift) seeds x (1 << wshift) walk lanes. Each lane walks and
// writes its T visited items to LDS, counts them against the seed's C = num_walks*T visits,
// then lane 0 selects the k most visited (count desc, item id asc), drops edges in the
// exclusion set and writes nbr/cnt [n_seeds, k] (-1 / 0 in empty slots).
__global__ __launch_bounds__(256) void neighbors_kernel(
    Graph g, const int32_t* __restrict__ seeds, int64_t n_seeds, int32_t num_walks,
    int32_t wshift, int32_t T, uint32_t stop_thr, uint64_t seed, uint32_t step_add,
    const uint32_t* __restrict__ step_ptr, uint32_t layer, int32_t k,
    const uint64_t* __restrict__ excl, uint32_t excl_mask, int32_t* __restrict__ nbr,
    int32_t* __restrict__ cnt) {
  const uint32_t step = step_add + (step_ptr ? *step_ptr : 0u);
  extern __shared__ int32_t lds[];
  int32_t* cand = lds;                    // [256 * T]
  int32_t* ccount = lds + 256 * T;        // [256 * T]: count at first occurrence, else 0
  const int32_t tid = threadIdx.x;
  const int32_t wp = 1 << wshift;
  const int32_t grp = tid >> wshift;
  const int32_t j = tid & (wp - 1);
  const int64_t s = (int64_t)blockIdx.x * (256 >> wshift) + grp;
  const int32_t start = s < n_seeds ? seeds[s] : -1;
  // a padding seed (< 0, capacity-shaped batches) walks nowhere and gets k empty slots
  const bool live = s < n_seeds && j < num_walks && start >= 0;
  int32_t* mine = cand + tid * T;
  for (int32_t t = 0; t < T; ++t) mine[t] = -1;
  if (live)
    metapath(g, start, T, stop_thr, seed, kPurposeWalk, (uint32_t)start,
             (uint32_t)j | (layer << 16), step, [&](int32_t h, int32_t node) {
               if (h & 1) mine[h >> 1] = node;
             });
  __syncthreads();
  const int32_t C = num_walks * T;
  const int32_t* gc = cand + (grp << wshift) * T;
  int32_t* gcc = ccount + (grp << wshift) * T;
  if (live) {
    for (int32_t t = 0; t < T; ++t) {
      const int32_t me = j * T + t;
      const int32_t v = gc[me];
      int32_t c = 0;
      bool first = v >= 0;
      for (int32_t m = 0; m < C && first; ++m) {
        if (gc[m] == v) {
          if (m < me) first = false;
          ++c;
        }
      }
      gcc[me] = first ? c : 0;
    }
  } else if (j < num_walks) {
    for (int32_t t = 0; t < T; ++t) gcc[j * T + t] = 0;
  }
  __syncthreads();
  if (s >= n_seeds || j != 0) return;
  int32_t prev_c = 0x7fffffff, prev_id = -1;
  for (int32_t r = 0; r < k; ++r) {
    int32_t best_c = 0, best_id = -1;
    for (int32_t m = 0; m < C; ++m) {
      const int32_t c = gcc[m];
      if (c == 0) continue;
      const int32_t v = gc[m];
      // strictly after the previous pick in (count desc, id asc) order
      const bool after = c < prev_c || (c == prev_c && v > prev_id);
      if (!after) continue;
      if (c > best_c || (c == best_c && v < best_id)) best_c = c, best_id = v;
    }
    int32_t out_id = best_id, out_c = best_c;
    if (best_id >= 0) {
      prev_c = best_c, prev_id = best_id;
      if (excl_mask != 0u && pair_set_has(excl, excl_mask, pair_key(start, best_id)))
        out_id = -1, out_c = 0;
    }
    nbr[s * k + r] = out_id;
    cnt[s * k + r] = out_c;
  }
}

// ---- first-appearance unique (compact_graphs / to_block src order) -----------------------
__global__ __launch_bounds__(256) void fill_i32_kernel(int32_t* __restrict__ a, int64_t n,
                                                       int32_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = v;
}

__global__ __launch_bounds__(256) void first_mark_kernel(const int32_t* __restrict__ ids,
                                                         int64_t n, int64_t n_nodes,
                                                         int32_t* __restrict__ mark,
                                                         int32_t* __restrict__ err_flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t v = ids[i];
  if (v < 0) return;
  if (v >= n_nodes) {
    flag_oob(err_flag);
    return;
  }
  atomicMin(mark + v, (int32_t)i);
}

__global__ __launch_bounds__(256) void first_flag_kernel(const int32_t* __restrict__ ids,
                                                         int64_t n, int64_t n_nodes,
                                                         const int32_t* __restrict__ mark,
                                                         int32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t v = ids[i];
  flag[i] = (v >= 0 && v < n_nodes && mark[v] == (int32_t)i) ? 1 : 0;
}

__global__ __launch_bounds__(256) void first_emit_kernel(const int32_t* __restrict__ ids,
                                                         int64_t n, int64_t n_nodes,
                                                         const int32_t* __restrict__ mark,
                                                         const int32_t* __restrict__ flag,
                                                         const int32_t* __restrict__ pos,
                                                         int32_t* __restrict__ uniq,
                                                         int32_t* __restrict__ local) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t v = ids[i];
  const bool ok = v >= 0 && v < n_nodes;
  if (local) local[i] = ok ? pos[mark[v]] : -1;
  if (flag[i]) uniq[pos[i]] = v;
}

// ---- block (to_block): CSR by dst + stable transpose ----------------------------------------
__global__ __launch_bounds__(256) void block_valid_kernel(const int32_t* __restrict__ nbr_local,
                                                          int64_t cap,
                                                          int32_t* __restrict__ valid) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) valid[i] = nbr_local[i] >= 0;
}

__global__ __launch_bounds__(256) void block_emit_kernel(
    const int32_t* __restrict__ nbr_local, const int32_t* __restrict__ cnt, int64_t n_dst,
    int32_t k, int64_t n_src, const int32_t* __restrict__ epos, const int32_t* __restrict__ total,
    int32_t* __restrict__ indptr, int32_t* __restrict__ edge_src, int32_t* __restrict__ edge_dst,
    float* __restrict__ edge_w, uint32_t* __restrict__ keys, int32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t cap = n_dst * k;
  if (i > cap) return;
  if (i == cap) {
    indptr[n_dst] = *total;
    return;
  }
  const int64_t d = i / k;
  const int32_t e = epos[i];
  if (i - d * k == 0) indptr[d] = e;
  const int32_t s = nbr_local[i];
  if (s >= 0) {
    edge_src[e] = s;
    edge_dst[e] = (int32_t)d;
    edge_w[e] = (float)cnt[i];
    keys[i] = (uint32_t)s;
    vals[i] = e;
  } else {
    keys[i] = (uint32_t)n_src;  // sentinel: sorts after every real src
    vals[i] = -1;
  }
}

__global__ __launch_bounds__(256) void lower_bound_kernel(const uint32_t* __restrict__ sorted,
                                                          int64_t n, int64_t n_keys,
                                                          int32_t* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n_keys) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)sorted[mid] < s) lo = mid + 1;
    else hi = mid;
  }
  out[s] = (int32_t)lo;
}

// ---- weighted mean-pool (Convolve update_all u_mul_e/sum, copy_e/sum, clip, divide) -----
__global__ __launch_bounds__(256) void agg_fwd_kernel(const float* __restrict__ u, int32_t H,
                                                      const int32_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ edge_src,
                                                      const float* __restrict__ edge_w,
                                                      int64_t n_dst, float* __restrict__ nv,
                                                      float* __restrict__ wsum) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_dst * H) return;
  const int64_t d = i / H;
  const int32_t c = (int32_t)(i - d * H);
  float acc = 0.f, ws = 0.f;
  // the in-edges' loads issued 4 at a time, summed in edge order (bit-identical to one by one)
  int32_t e = indptr[d];
  const int32_t end = indptr[d + 1];
  for (; e + 4 <= end; e += 4) {
    float w[4], x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[k] = edge_w[e + k];
      x[k] = u[(int64_t)edge_src[e + k] * H + c];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc += w[k] * x[k];
      ws += w[k];
    }
  }
  for (; e < end; ++e) {
    const float w = edge_w[e];
    acc += w * u[(int64_t)edge_src[e] * H + c];
    ws += w;
  }
  nv[i] = acc / fmaxf(ws, 1.f);
  if (c == 0 && wsum) wsum[d] = ws;
}

__global__ __launch_bounds__(256) void agg_bwd_kernel(const float* __restrict__ gnv, int32_t H,
                                                      const int32_t* __restrict__ t_indptr,
                                                      const int32_t* __restrict__ t_edge,
                                                      const int32_t* __restrict__ edge_dst,
                                                      const float* __restrict__ edge_w,
                                                      const float* __restrict__ wsum,
                                                      int64_t n_src, float* __restrict__ gu) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_src * H) return;
  const int64_t s = i / H;
  const int32_t c = (int32_t)(i - s * H);
  float acc = 0.f;
  // a hub source (an item many sampled destinations pooled) walks a long in-edge list: its three
  // dependent loads per edge (slot -> edge -> destination row) are issued for 8 edges at a time,
  // then summed in edge order (the same sum, bit for bit, as one edge at a time; measured: the
  // one-edge loop ran 41.6 us per launch at cfg5, 0.035 of HBM — latency chains, not bytes)
  constexpr int U = 8;
  int32_t j = t_indptr[s];
  const int32_t end = t_indptr[s + 1];
  for (; j + U <= end; j += U) {
    int32_t e[U], d[U];
    float w[U], ws[U], g[U];
#pragma unroll
    for (int k = 0; k < U; ++k) e[k] = t_edge[j + k];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      d[k] = edge_dst[e[k]];
      w[k] = edge_w[e[k]];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      ws[k] = wsum[d[k]];
      g[k] = gnv[(int64_t)d[k] * H + c];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) acc += w[k] / fmaxf(ws[k], 1.f) * g[k];
  }
  for (; j < end; ++j) {
    const int32_t e = t_edge[j];
    const int32_t d = edge_dst[e];
    acc += edge_w[e] / fmaxf(wsum[d], 1.f) * gnv[(int64_t)d * H + c];
  }
  gu[i] = acc;
}

// ---- global Frobenius normalisation (Convolve :28-29) -----------------------------------
constexpr int kRedThreads = 256;
constexpr int kRedChunk = kRedThreads * 16;

__device__ __forceinline__ float block_sum(float v, float* sm) {
  sm[threadIdx.x] = v;
  __syncthreads();
  for (int w = kRedThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sm[threadIdx.x] += sm[threadIdx.x + w];
    __syncthreads();
  }
  return sm[0];
}

// partial[b] = Σ a[i] * b[i] over chunk b (b == nullptr: Σ a[i]^2)
// live length of a capacity-shaped [rows, row_len] buffer: the first *n_rows rows
// (n_rows == nullptr: all n elements). Elements past it are padding: excluded from the
// reduction and written as 0.
__device__ __forceinline__ int64_t live_len(int64_t n, const int32_t* n_rows, int32_t row_len) {
  if (!n_rows) return n;
  const int64_t m = (int64_t)*n_rows * row_len;
  return m < n ? m : n;
}

__global__ __launch_bounds__(kRedThreads) void dot_partial_kernel(const float* __restrict__ a,
                                                                  const float* __restrict__ b,
                                                                  int64_t n_cap,
                                                                  const int32_t* __restrict__ n_rows,
                                                                  int32_t row_len,
                                                                  float* __restrict__ partial) {
  __shared__ float sm[kRedThreads];
  const int64_t n = live_len(n_cap, n_rows, row_len);
  const int64_t base = (int64_t)blockIdx.x * kRedChunk;
  float acc = 0.f;
  for (int64_t i = base + threadIdx.x; i < base + kRedChunk && i < n; i += kRedThreads) {
    const float x = a[i];
    acc += x * (b ? b[i] : x);
  }
  const float t = block_sum(acc, sm);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// total = Σ partial (fixed order); mode 0: out = sqrt(total) (the norm), 1: out = total
__global__ __launch_bounds__(kRedThreads) void fold_partial_kernel(const float* __restrict__ partial,
                                                                   int64_t n, int32_t mode,
                                                                   float* __restrict__ out) {
  __shared__ float sm[kRedThreads];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += kRedThreads) acc += partial[i];
  const float t = block_sum(acc, sm);
  if (threadIdx.x == 0) *out = mode == 0 ? sqrtf(t) : t;
}

__global__ __launch_bounds__(256) void scale_div_kernel(const float* __restrict__ x, int64_t n,
                                                        const int32_t* __restrict__ n_rows,
                                                        int32_t row_len,
                                                        const float* __restrict__ norm,
                                                        float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  y[i] = i < live_len(n, n_rows, row_len) ? x[i] / *norm : 0.f;
}

__global__ __launch_bounds__(256) void frob_bwd_kernel(const float* __restrict__ dy,
                                                       const float* __restrict__ y, int64_t n,
                                                       const int32_t* __restrict__ n_rows,
                                                       int32_t row_len,
                                                       const float* __restrict__ norm,
                                                       const float* __restrict__ dot,
                                                       float* __restrict__ dx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dx[i] = i < live_len(n, n_rows, row_len) ? (dy[i] - y[i] * *dot) / *norm : 0.f;
}

inline unsigned grid_for(int64_t n, int threads = 256) {
  return (unsigned)ceil_div(n < 1 ? 1 : n, threads);
}

inline uint32_t stop_threshold(float p) {
  if (!(p > 0.f)) return 0u;
  const double t = std::floor((double)p * 4294967296.0);
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// ---- item2item scores + margin loss (pinsage/train/model.py:14-19, train.py:17-20) -------
// score(u, v) = h[u]·h[v] for the positive and the negative pair of each example, hinge =
// max((neg + delta) - pos, 0) over the live pairs, loss = Σ hinge / n_live. One thread per pair
// (D <= 64 row elements, products rounded then summed in order, as the mul + sum it replaces);
// the block sums folded in block order (deterministic). Padding pairs (src or dst -1) score
// node 0 and carry no weight, as the capacity-shaped batch's clamp + mask did; a node id >= n_rows
// reads a zero row and flags RS_ERRBIT_OOB.
constexpr int kPairThreads = 256;

// the row a pair endpoint reads: -1 (padding) -> node 0, >= n_rows -> none (oob)
__device__ __forceinline__ int pair_row(int32_t r, int64_t n_rows, bool& oob) {
  if (r < 0) return 0;
  if (r >= n_rows) {
    oob = true;
    return -1;
  }
  return r;
}

__device__ __forceinline__ float row_dot(const float* __restrict__ h, int64_t ld, int D, int u,
                                         int v) {
  if (u < 0 || v < 0) return 0.f;
  const float* a = h + (int64_t)u * ld;
  const float* b = h + (int64_t)v * ld;
  float s = 0.f;
  for (int d = 0; d < D; ++d) s += a[d] * b[d];
  return s;
}

__global__ __launch_bounds__(kPairThreads) void pair_margin_fwd_kernel(
    const float* __restrict__ h, int64_t ld, int D, int64_t n_rows, const int32_t* __restrict__ ps,
    const int32_t* __restrict__ pd, const int32_t* __restrict__ ns, const int32_t* __restrict__ nd,
    int64_t P, float delta, const uint8_t* __restrict__ valid, float* __restrict__ pos,
    float* __restrict__ neg, float* __restrict__ part, int32_t* err_flag) {
  __shared__ float red[kPairThreads];
  const int64_t i = (int64_t)blockIdx.x * kPairThreads + threadIdx.x;
  float w = 0.f;
  bool oob = false;
  if (i < P) {
    const int a = pair_row(ps[i], n_rows, oob), b = pair_row(pd[i], n_rows, oob);
    const int c = pair_row(ns[i], n_rows, oob), e = pair_row(nd[i], n_rows, oob);
    const float p = row_dot(h, ld, D, a, b);
    const float q = row_dot(h, ld, D, c, e);
    pos[i] = p;
    neg[i] = q;
    const float hinge = fmaxf((q + delta) - p, 0.f);
    w = (valid == nullptr || valid[i]) ? hinge : 0.f;
  }
  if (oob) flag_oob(err_flag);
  red[threadIdx.x] = w;
  __syncthreads();
  for (int o = kPairThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(64) void pair_margin_fold_kernel(const float* __restrict__ part,
                                                             int nb, const int32_t* __restrict__ n_live,
                                                             int64_t P, float* __restrict__ loss) {
  if (threadIdx.x != 0) return;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += part[b];
  loss[0] = s / (float)(n_live ? n_live[0] : P);
}

// The backward's row terms: the hinge's gradient g = dloss / n_live on live pairs with
// (neg + delta) - pos >= 0 (clamp's backward passes at the boundary), -g to the positive score,
// +g to the negative one; each score's two rows take the other row times it. Endpoint
// e = role·P + i (roles: pos src, pos dst, neg src, neg dst) gets the row terms[e] = coef · h[other]
// (one fmul_rn, the product the gathers' backward formed), key[e] = its node and live[e] = 1 when
// it carries a gradient; rs_index_add_rows then folds them per node in a fixed order. One thread
// per (pair, element).
__global__ __launch_bounds__(kPairThreads) void pair_margin_terms_kernel(
    const float* __restrict__ h, int64_t ld, int D, int64_t n_rows, const int32_t* __restrict__ ps,
    const int32_t* __restrict__ pd, const int32_t* __restrict__ ns, const int32_t* __restrict__ nd,
    int64_t P, float delta, const uint8_t* __restrict__ valid, const float* __restrict__ pos,
    const float* __restrict__ neg, const float* __restrict__ dloss,
    const int32_t* __restrict__ n_live, float* __restrict__ terms, int32_t* __restrict__ key,
    uint8_t* __restrict__ live) {
  const int64_t k = (int64_t)blockIdx.x * kPairThreads + threadIdx.x;
  if (k >= P * D) return;
  const int64_t i = k / D;
  const int d = (int)(k - i * D);
  bool oob = false;
  const int a = pair_row(ps[i], n_rows, oob), b = pair_row(pd[i], n_rows, oob);
  const int c = pair_row(ns[i], n_rows, oob), e = pair_row(nd[i], n_rows, oob);
  const bool on = (valid == nullptr || valid[i]) && ((neg[i] + delta) - pos[i] >= 0.f);
  const float g = on ? dloss[0] / (float)(n_live ? n_live[0] : P) : 0.f;
  const float ha = a >= 0 ? h[(int64_t)a * ld + d] : 0.f, hb = b >= 0 ? h[(int64_t)b * ld + d] : 0.f;
  const float hc = c >= 0 ? h[(int64_t)c * ld + d] : 0.f, he = e >= 0 ? h[(int64_t)e * ld + d] : 0.f;
  terms[(0 * P + i) * D + d] = -g * hb;
  terms[(1 * P + i) * D + d] = -g * ha;
  terms[(2 * P + i) * D + d] = g * he;
  terms[(3 * P + i) * D + d] = g * hc;
  if (d == 0) {
    const int rows[4] = {a, b, c, e};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      key[r * P + i] = rows[r] < 0 ? 0 : rows[r];
      live[r * P + i] = (on && rows[r] >= 0) ? 1 : 0;
    }
  }
}

// ---- multi-hot mean lookup (FeatureProjector's genre, pinsage/train/layers.py:68-81) --------
// out[n] = mean_g table[mh[item[n], g]] over the item's G multi-hot slots: the item's id row is
// read in place (no gathered [N, G] id tensor, no [N, G, D] rows) — a sequential sum over g,
// then / G. Ids outside [0, V) read 0 and flag RS_ERRBIT_OOB.
__global__ __launch_bounds__(256) void multihot_mean_fwd_kernel(
    const float* __restrict__ table, int V, int D, const int32_t* __restrict__ mh, int G,
    int64_t n_items, const int64_t* __restrict__ items, int64_t N, float* __restrict__ out,
    int32_t* err_flag) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * D) return;
  const int64_t n = e / D;
  const int d = (int)(e - n * D);
  const int64_t item = items[n];
  if (item < 0 || item >= n_items) {  // no id row to read: a zero row
    out[e] = 0.f;
    if (d == 0) flag_oob(err_flag);
    return;
  }
  const int32_t* row = mh + item * G;
  float s = 0.f;
  bool oob = false;
  for (int g = 0; g < G; ++g) {
    const int r = row[g];
    if (r >= 0 && r < V) s += table[(int64_t)r * D + d];
    else oob = true;
  }
  out[e] = s / (float)G;
  if (oob && err_flag) atomicOr(err_flag, RS_ERRBIT_OOB);
}

// dtable[r][d] = Σ_n Σ_{g: mh[item[n], g] = r} dout[n][d] / G: a block per 32 items stages their
// id rows and dout rows in LDS (coalesced), thread (r, d) sums its entries in (n, g) order into
// the block's partial; the partials are folded per (r, d) by a block of 256 lanes (lane j the
// blocks j, j + 256, ... in order, then a fixed tree): deterministic. V·D <= 256, G <= 32, D <= 64.
constexpr int kMhRows = 32;
__global__ __launch_bounds__(256) void multihot_mean_bwd_part_kernel(
    const int32_t* __restrict__ mh, int G, int64_t n_items, const int64_t* __restrict__ items,
    int64_t N, const float* __restrict__ dout, int V, int D, float* __restrict__ part,
    int32_t* err_flag) {
  __shared__ int32_t ids[kMhRows * 32];
  __shared__ float gs[kMhRows * 64];
  const int64_t n0 = (int64_t)blockIdx.x * kMhRows;
  const int rows = (int)(N - n0 < kMhRows ? N - n0 : kMhRows);
  for (int e = threadIdx.x; e < rows * G; e += blockDim.x) {
    const int i = e / G, g = e - i * G;
    const int64_t item = items[n0 + i];
    const bool ok = item >= 0 && item < n_items;  // an out-of-range item adds nothing
    ids[i * G + g] = ok ? mh[item * G + g] : -1;
    if (!ok && g == 0) flag_oob(err_flag);
  }
  for (int e = threadIdx.x; e < rows * D; e += blockDim.x) gs[e] = dout[n0 * D + e] / (float)G;
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= V * D) return;
  const int r = t / D, d = t - r * D;
  float acc = 0.f;
  for (int i = 0; i < rows; ++i) {
    const float x = gs[i * D + d];
    for (int g = 0; g < G; ++g)
      if (ids[i * G + g] == r) acc += x;
  }
  part[(int64_t)blockIdx.x * V * D + t] = acc;
}

__global__ __launch_bounds__(256) void multihot_mean_bwd_fold_kernel(const float* __restrict__ part,
                                                                    int nb, int VD,
                                                                    float* __restrict__ dtable) {
  __shared__ float red[256];
  const int t = blockIdx.x, j = threadIdx.x;
  float s = 0.f;
  for (int b = j; b < nb; b += 256) s += part[(int64_t)b * VD + t];
  red[j] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (j < o) red[j] += red[j + o];
    __syncthreads();
  }
  if (j == 0) dtable[t] = red[0];
}

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_multihot_mean_fwd(const float* table, int32_t V, int32_t D, const int32_t* mh,
                                        int32_t G, int64_t n_items, const int64_t* items, int64_t N,
                                        float* out, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(V >= 1 && D >= 1 && G >= 1 && N >= 0 && n_items >= 0, "rs_multihot_mean_fwd: bad sizes");
  if (N == 0) return RS_OK;
  RS_CHECK_ARG(table && mh && items && out, "rs_multihot_mean_fwd: null pointer");
  multihot_mean_fwd_kernel<<<(unsigned)ceil_div(N * D, 256), 256, 0, as_stream(stream)>>>(
      table, V, D, mh, G, n_items, items, N, out, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_multihot_mean_bwd_workspace_size(int64_t N, int32_t V, int32_t D) {
  return (size_t)ceil_div(N < 1 ? 1 : N, kMhRows) * V * D * sizeof(float) + 256;
}

extern "C" int32_t rs_multihot_mean_bwd(const int32_t* mh, int32_t G, int64_t n_items,
                                        const int64_t* items, int64_t N, const float* dout,
                                        int32_t V, int32_t D, float* dtable, int32_t* err_flag,
                                        void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(V >= 1 && D >= 1 && D <= 64 && V * D <= 256 && G >= 1 && G <= 32 && N >= 1 &&
                   n_items >= 0,
               "rs_multihot_mean_bwd: V·D <= 256, D <= 64, 1 <= G <= 32, N >= 1");
  RS_CHECK_ARG(mh && items && dout && dtable && workspace, "rs_multihot_mean_bwd: null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_multihot_mean_bwd_workspace_size(N, V, D), "workspace too small");
  hipStream_t st = as_stream(stream);
  const int nb = (int)ceil_div(N, kMhRows);
  float* part = static_cast<float*>(workspace);
  multihot_mean_bwd_part_kernel<<<nb, 256, 0, st>>>(mh, G, n_items, items, N, dout, V, D, part,
                                                    err_flag);
  RS_CHECK_LAUNCH();
  multihot_mean_bwd_fold_kernel<<<V * D, 256, 0, st>>>(part, nb, V * D, dtable);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_pair_margin_workspace_size(int64_t n_pairs) {
  return (size_t)(ceil_div(n_pairs < 1 ? 1 : n_pairs, kPairThreads)) * sizeof(float) + 256;
}

extern "C" int32_t rs_pair_margin_fwd(const float* h, int64_t ld, int32_t D, int64_t n_rows,
                                      const int32_t* pos_src, const int32_t* pos_dst,
                                      const int32_t* neg_src, const int32_t* neg_dst,
                                      int64_t n_pairs, float delta, const uint8_t* valid,
                                      const int32_t* n_live, float* pos_score, float* neg_score,
                                      float* loss, int32_t* err_flag, void* workspace,
                                      size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(n_pairs >= 1 && D >= 1 && D <= 64 && ld >= D && n_rows >= 1,
               "rs_pair_margin_fwd: bad sizes");
  RS_CHECK_ARG(h && pos_src && pos_dst && neg_src && neg_dst && pos_score && neg_score && loss &&
                   workspace,
               "rs_pair_margin_fwd: null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_pair_margin_workspace_size(n_pairs), "workspace too small");
  hipStream_t st = as_stream(stream);
  const int nb = (int)ceil_div(n_pairs, kPairThreads);
  float* part = static_cast<float*>(workspace);
  pair_margin_fwd_kernel<<<nb, kPairThreads, 0, st>>>(h, ld, D, n_rows, pos_src, pos_dst, neg_src,
                                                      neg_dst, n_pairs, delta, valid, pos_score,
                                                      neg_score, part, err_flag);
  RS_CHECK_LAUNCH();
  pair_margin_fold_kernel<<<1, 64, 0, st>>>(part, nb, n_live, n_pairs, loss);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

// workspace: terms [4P, D] fp32, keys [4P] int32, live [4P] uint8, then rs_index_add_rows' own
static size_t pair_terms_bytes(int64_t P, int32_t D, float** terms, int32_t** key, uint8_t** live,
                               void* ws) {
  Carver c(ws, ~(size_t)0);
  *terms = c.take<float>((size_t)4 * P * D);
  *key = c.take<int32_t>((size_t)4 * P);
  *live = c.take<uint8_t>((size_t)4 * P);
  return align_up(c.off, 256);
}

extern "C" size_t rs_pair_margin_bwd_workspace_size(int64_t n_pairs, int32_t D) {
  float* t;
  int32_t* k;
  uint8_t* l;
  const int64_t P = n_pairs < 1 ? 1 : n_pairs;
  return pair_terms_bytes(P, D, &t, &k, &l, nullptr) + rs_index_add_rows_workspace_size(4 * P, D);
}

extern "C" int32_t rs_pair_margin_bwd(const float* h, int64_t ld, int32_t D, int64_t n_rows,
                                      const int32_t* pos_src, const int32_t* pos_dst,
                                      const int32_t* neg_src, const int32_t* neg_dst,
                                      int64_t n_pairs, float delta, const uint8_t* valid,
                                      const int32_t* n_live, const float* pos_score,
                                      const float* neg_score, const float* dloss, float* dh,
                                      int32_t* err_flag, void* workspace, size_t ws_bytes,
                                      void* stream) {
  RS_CHECK_ARG(n_pairs >= 1 && D >= 1 && D <= 64 && ld >= D && n_rows >= 1,
               "rs_pair_margin_bwd: bad sizes");
  RS_CHECK_ARG(h && pos_src && pos_dst && neg_src && neg_dst && pos_score && neg_score && dloss &&
                   dh && workspace,
               "rs_pair_margin_bwd: null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_pair_margin_bwd_workspace_size(n_pairs, D), "workspace too small");
  float* terms;
  int32_t* key;
  uint8_t* live;
  const size_t head = pair_terms_bytes(n_pairs, D, &terms, &key, &live, workspace);
  hipStream_t st = as_stream(stream);
  pair_margin_terms_kernel<<<(unsigned)ceil_div(n_pairs * D, kPairThreads), kPairThreads, 0, st>>>(
      h, ld, D, n_rows, pos_src, pos_dst, neg_src, neg_dst, n_pairs, delta, valid, pos_score,
      neg_score, dloss, n_live, terms, key, live);
  RS_CHECK_LAUNCH();
  return rs_index_add_rows(key, RS_ID_I32, 4 * n_pairs, live, terms, D, n_rows, dh, err_flag,
                           static_cast<char*>(workspace) + head, ws_bytes - head, stream);
}

static Graph make_graph(const int64_t* a, const int32_t* b, const int64_t* c, const int32_t* d) {
  return Graph{a, b, c, d};
}

extern "C" int32_t rs_philox4x32_10(const uint32_t* ctr, int64_t n, uint32_t k0, uint32_t k1,
                                    uint32_t* out, void* stream) {
  RS_CHECK_ARG(n >= 0 && (n == 0 || (ctr && out)), "rs_philox4x32_10: bad args");
  if (n == 0) return RS_OK;
  philox_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(ctr, n, k0, k1, out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_metapath_walk(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                                    const int64_t* u2i_indptr, const int32_t* u2i_idx,
                                    const int32_t* seeds, int64_t n_seeds, int32_t num_walks,
                                    int32_t n_traversals, float restart_prob, uint64_t seed,
                                    uint32_t step, uint32_t layer, int32_t* traces,
                                    void* stream) {
  RS_CHECK_ARG(num_walks >= 1 && n_traversals >= 1 && n_seeds >= 0 && layer < 65536 &&
                   num_walks < 65536,
               "rs_metapath_walk: bad sizes");
  RS_CHECK_ARG(i2u_indptr && i2u_idx && u2i_indptr && u2i_idx, "rs_metapath_walk: null graph");
  const int64_t n = n_seeds * num_walks;
  if (n == 0) return RS_OK;
  walk_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(
      make_graph(i2u_indptr, i2u_idx, u2i_indptr, u2i_idx), seeds, n_seeds, num_walks,
      n_traversals, stop_threshold(restart_prob), seed, step, layer, traces);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_item_pairs_workspace_size(int32_t batch) {
  Carver c(nullptr, 0);
  c.take<int32_t>((size_t)3 * batch);
  c.take<int32_t>(batch);
  c.take<int32_t>(batch);
  c.take<char>(exclusive_scan_ws_size(batch));
  return c.off + 256;
}

static int32_t item_pairs(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                          const int64_t* u2i_indptr, const int32_t* u2i_idx, int32_t n_items,
                          int64_t pair_base, int32_t batch, uint64_t seed, uint32_t step,
                          const uint32_t* step_ptr, int32_t* heads, int32_t* pos_tails,
                          int32_t* neg_tails, int32_t* n_valid, void* workspace, size_t ws_bytes,
                          void* stream) {
  RS_CHECK_ARG(n_items >= 1 && batch >= 0, "rs_item_pairs: bad sizes");
  RS_CHECK_ARG(i2u_indptr && i2u_idx && u2i_indptr && u2i_idx, "rs_item_pairs: null graph");
  hipStream_t st = as_stream(stream);
  if (batch == 0) {
    RS_CHECK_HIP(hipMemsetAsync(n_valid, 0, 4, st));
    return RS_OK;
  }
  Carver c(workspace, ws_bytes);
  int32_t* tmp = c.take<int32_t>((size_t)3 * batch);
  int32_t* flag = c.take<int32_t>(batch);
  int32_t* offs = c.take<int32_t>(batch);
  void* sws = c.take<char>(exclusive_scan_ws_size(batch));
  if (!c.ok()) {
    set_error("rs_item_pairs: workspace too small (%zu > %zu)", c.off, ws_bytes);
    return RS_E_WORKSPACE;
  }
  pairs_gen_kernel<<<grid_for(batch), 256, 0, st>>>(
      make_graph(i2u_indptr, i2u_idx, u2i_indptr, u2i_idx), n_items, pair_base, batch, seed, step,
      step_ptr, tmp, flag);
  RS_CHECK_LAUNCH();
  int32_t s = exclusive_scan_i32(flag, offs, batch, n_valid, sws, exclusive_scan_ws_size(batch), st);
  if (s) return s;
  pairs_compact_kernel<<<grid_for(batch), 256, 0, st>>>(tmp, flag, offs, batch, heads, pos_tails,
                                                        neg_tails);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_item_pairs(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                                 const int64_t* u2i_indptr, const int32_t* u2i_idx,
                                 int32_t n_items, int64_t pair_base, int32_t batch, uint64_t seed,
                                 uint32_t step, int32_t* heads, int32_t* pos_tails,
                                 int32_t* neg_tails, int32_t* n_valid, void* workspace,
                                 size_t ws_bytes, void* stream) {
  return item_pairs(i2u_indptr, i2u_idx, u2i_indptr, u2i_idx, n_items, pair_base, batch, seed,
                    step, nullptr, heads, pos_tails, neg_tails, n_valid, workspace, ws_bytes,
                    stream);
}

extern "C" int32_t rs_item_pairs_at(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                                    const int64_t* u2i_indptr, const int32_t* u2i_idx,
                                    int32_t n_items, int64_t pair_base, int32_t batch,
                                    uint64_t seed, const uint32_t* step_ptr, int32_t* heads,
                                    int32_t* pos_tails, int32_t* neg_tails, int32_t* n_valid,
                                    void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(step_ptr != nullptr, "rs_item_pairs_at: null step pointer");
  return item_pairs(i2u_indptr, i2u_idx, u2i_indptr, u2i_idx, n_items, pair_base, batch, seed, 0u,
                    step_ptr, heads, pos_tails, neg_tails, n_valid, workspace, ws_bytes, stream);
}

extern "C" int32_t rs_pair_set_build(const int32_t* src, const int32_t* dst, int64_t n,
                                     uint64_t* table, int64_t capacity, void* stream) {
  RS_CHECK_ARG(capacity > n && capacity <= ((int64_t)1 << 31) &&
                   (capacity & (capacity - 1)) == 0,
               "rs_pair_set_build: capacity %lld must be a power of two > n (%lld)",
               (long long)capacity, (long long)n);
  if (n == 0) return RS_OK;
  pair_set_build_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(src, dst, n, table,
                                                                    (uint32_t)(capacity - 1));
  RS_CHECK_LAUNCH();
  return RS_OK;
}

static int32_t pinsage_neighbors(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                                 const int64_t* u2i_indptr, const int32_t* u2i_idx,
                                 const int32_t* seeds, int64_t n_seeds, int32_t num_walks,
                                 int32_t n_traversals, float restart_prob, uint64_t seed,
                                 uint32_t step, const uint32_t* step_ptr, uint32_t layer,
                                 int32_t num_neighbors, const uint64_t* excl_table,
                                 int64_t excl_capacity, int32_t* nbr, int32_t* cnt, void* stream) {
  RS_CHECK_ARG(num_walks >= 1 && num_walks <= 64 && n_traversals >= 1 && n_traversals <= 8 &&
                   num_neighbors >= 1 && layer < 65536 && n_seeds >= 0,
               "rs_pinsage_neighbors: need 1<=num_walks<=64, 1<=n_traversals<=8, k>=1");
  RS_CHECK_ARG(excl_capacity == 0 ||
                   (excl_table && (excl_capacity & (excl_capacity - 1)) == 0 &&
                    excl_capacity <= ((int64_t)1 << 31)),
               "rs_pinsage_neighbors: exclusion capacity must be 0 or a power of two");
  if (n_seeds == 0) return RS_OK;
  int32_t wshift = 0;
  while ((1 << wshift) < num_walks) ++wshift;
  const int64_t per_block = 256 >> wshift;
  const size_t lds = (size_t)2 * 256 * n_traversals * sizeof(int32_t);
  neighbors_kernel<<<(unsigned)ceil_div(n_seeds, per_block), 256, lds, as_stream(stream)>>>(
      make_graph(i2u_indptr, i2u_idx, u2i_indptr, u2i_idx), seeds, n_seeds, num_walks, wshift,
      n_traversals, stop_threshold(restart_prob), seed, step, step_ptr, layer, num_neighbors,
      excl_table, excl_capacity ? (uint32_t)(excl_capacity - 1) : 0u, nbr, cnt);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_pinsage_neighbors(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                                        const int64_t* u2i_indptr, const int32_t* u2i_idx,
                                        const int32_t* seeds, int64_t n_seeds,
                                        int32_t num_walks, int32_t n_traversals,
                                        float restart_prob, uint64_t seed, uint32_t step,
                                        uint32_t layer, int32_t num_neighbors,
                                        const uint64_t* excl_table, int64_t excl_capacity,
                                        int32_t* nbr, int32_t* cnt, void* stream) {
  return pinsage_neighbors(i2u_indptr, i2u_idx, u2i_indptr, u2i_idx, seeds, n_seeds, num_walks,
                           n_traversals, restart_prob, seed, step, nullptr, layer, num_neighbors,
                           excl_table, excl_capacity, nbr, cnt, stream);
}

extern "C" int32_t rs_pinsage_neighbors_at(const int64_t* i2u_indptr, const int32_t* i2u_idx,
                                           const int64_t* u2i_indptr, const int32_t* u2i_idx,
                                           const int32_t* seeds, int64_t n_seeds,
                                           int32_t num_walks, int32_t n_traversals,
                                           float restart_prob, uint64_t seed,
                                           const uint32_t* step_ptr, uint32_t layer,
                                           int32_t num_neighbors, const uint64_t* excl_table,
                                           int64_t excl_capacity, int32_t* nbr, int32_t* cnt,
                                           void* stream) {
  RS_CHECK_ARG(step_ptr != nullptr, "rs_pinsage_neighbors_at: null step pointer");
  return pinsage_neighbors(i2u_indptr, i2u_idx, u2i_indptr, u2i_idx, seeds, n_seeds, num_walks,
                           n_traversals, restart_prob, seed, 0u, step_ptr, layer, num_neighbors,
                           excl_table, excl_capacity, nbr, cnt, stream);
}

extern "C" size_t rs_unique_first_workspace_size(int64_t n_nodes, int64_t n) {
  Carver c(nullptr, 0);
  c.take<int32_t>(n_nodes);
  c.take<int32_t>(n);
  c.take<int32_t>(n);
  c.take<char>(exclusive_scan_ws_size(n));
  return c.off + 256;
}

extern "C" int32_t rs_unique_first(const int32_t* ids, int64_t n, int64_t n_nodes,
                                   int32_t* uniq, int32_t* local, int32_t* n_unique,
                                   int32_t* err_flag, void* workspace, size_t ws_bytes,
                                   void* stream) {
  RS_CHECK_ARG(n >= 0 && n < ((int64_t)1 << 31) && n_nodes >= 1 && n_nodes < ((int64_t)1 << 31),
               "rs_unique_first: bad sizes");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    RS_CHECK_HIP(hipMemsetAsync(n_unique, 0, 4, st));
    return RS_OK;
  }
  Carver c(workspace, ws_bytes);
  int32_t* mark = c.take<int32_t>(n_nodes);
  int32_t* flag = c.take<int32_t>(n);
  int32_t* pos = c.take<int32_t>(n);
  void* sws = c.take<char>(exclusive_scan_ws_size(n));
  if (!c.ok()) {
    set_error("rs_unique_first: workspace too small (%zu > %zu)", c.off, ws_bytes);
    return RS_E_WORKSPACE;
  }
  fill_i32_kernel<<<grid_for(n_nodes), 256, 0, st>>>(mark, n_nodes, 0x7fffffff);
  RS_CHECK_LAUNCH();
  first_mark_kernel<<<grid_for(n), 256, 0, st>>>(ids, n, n_nodes, mark, err_flag);
  RS_CHECK_LAUNCH();
  first_flag_kernel<<<grid_for(n), 256, 0, st>>>(ids, n, n_nodes, mark, flag);
  RS_CHECK_LAUNCH();
  int32_t s = exclusive_scan_i32(flag, pos, n, n_unique, sws, exclusive_scan_ws_size(n), st);
  if (s) return s;
  first_emit_kernel<<<grid_for(n), 256, 0, st>>>(ids, n, n_nodes, mark, flag, pos, uniq, local);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_pinsage_block_workspace_size(int64_t n_dst, int32_t k) {
  const int64_t cap = n_dst * k;
  Carver c(nullptr, 0);
  c.take<int32_t>(cap);             // valid
  c.take<int32_t>(cap);             // epos
  c.take<int32_t>(1);               // total
  c.take<uint32_t>(cap);            // keys
  c.take<int32_t>(cap);             // vals
  c.take<uint32_t>(cap);            // sorted keys
  c.take<char>(exclusive_scan_ws_size(cap));
  c.take<char>(radix_sort_ws_size(cap));
  return c.off + 256;
}

extern "C" int32_t rs_pinsage_block(const int32_t* nbr_local, const int32_t* cnt, int64_t n_dst,
                                    int32_t k, int64_t n_src, int32_t* indptr, int32_t* edge_src,
                                    int32_t* edge_dst, float* edge_w, int32_t* n_edges,
                                    int32_t* t_indptr, int32_t* t_edge, void* workspace,
                                    size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(n_dst >= 0 && k >= 1 && n_src >= n_dst && n_dst * k < ((int64_t)1 << 31),
               "rs_pinsage_block: bad sizes");
  hipStream_t st = as_stream(stream);
  const int64_t cap = n_dst * k;
  if (cap == 0) {
    RS_CHECK_HIP(hipMemsetAsync(n_edges, 0, 4, st));
    RS_CHECK_HIP(hipMemsetAsync(indptr, 0, (n_dst + 1) * 4, st));
    RS_CHECK_HIP(hipMemsetAsync(t_indptr, 0, (n_src + 1) * 4, st));
    return RS_OK;
  }
  Carver c(workspace, ws_bytes);
  int32_t* valid = c.take<int32_t>(cap);
  int32_t* epos = c.take<int32_t>(cap);
  int32_t* total = c.take<int32_t>(1);
  uint32_t* keys = c.take<uint32_t>(cap);
  int32_t* vals = c.take<int32_t>(cap);
  uint32_t* skeys = c.take<uint32_t>(cap);
  void* sws = c.take<char>(exclusive_scan_ws_size(cap));
  void* rws = c.take<char>(radix_sort_ws_size(cap));
  if (!c.ok()) {
    set_error("rs_pinsage_block: workspace too small (%zu > %zu)", c.off, ws_bytes);
    return RS_E_WORKSPACE;
  }
  block_valid_kernel<<<grid_for(cap), 256, 0, st>>>(nbr_local, cap, valid);
  RS_CHECK_LAUNCH();
  int32_t s = exclusive_scan_i32(valid, epos, cap, total, sws, exclusive_scan_ws_size(cap), st);
  if (s) return s;
  block_emit_kernel<<<grid_for(cap + 1), 256, 0, st>>>(nbr_local, cnt, n_dst, k, n_src, epos,
                                                       total, indptr, edge_src, edge_dst, edge_w,
                                                       keys, vals);
  RS_CHECK_LAUNCH();
  RS_CHECK_HIP(hipMemcpyAsync(n_edges, total, 4, hipMemcpyDeviceToDevice, st));
  // stable sort of slots by src: valid edges first, in (src, edge id) order
  s = radix_sort_pairs(keys, vals, skeys, t_edge, cap, n_src + 1, rws, radix_sort_ws_size(cap), st);
  if (s) return s;
  lower_bound_kernel<<<grid_for(n_src + 1), 256, 0, st>>>(skeys, cap, n_src, t_indptr);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_weighted_mean_agg_fwd(const float* u, int64_t n_src, int32_t H,
                                            const int32_t* indptr, const int32_t* edge_src,
                                            const float* edge_w, int64_t n_dst, float* nv,
                                            float* wsum, void* stream) {
  RS_CHECK_ARG(H >= 1 && n_dst >= 0 && n_src >= 0, "rs_weighted_mean_agg_fwd: bad sizes");
  if (n_dst == 0) return RS_OK;
  agg_fwd_kernel<<<grid_for(n_dst * H), 256, 0, as_stream(stream)>>>(u, H, indptr, edge_src,
                                                                     edge_w, n_dst, nv, wsum);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_weighted_mean_agg_bwd(const float* grad_nv, int32_t H,
                                            const int32_t* t_indptr, const int32_t* t_edge,
                                            const int32_t* edge_dst, const float* edge_w,
                                            const float* wsum, int64_t n_src, float* grad_u,
                                            void* stream) {
  RS_CHECK_ARG(H >= 1 && n_src >= 0, "rs_weighted_mean_agg_bwd: bad sizes");
  if (n_src == 0) return RS_OK;
  agg_bwd_kernel<<<grid_for(n_src * H), 256, 0, as_stream(stream)>>>(
      grad_nv, H, t_indptr, t_edge, edge_dst, edge_w, wsum, n_src, grad_u);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_frobenius_workspace_size(int64_t n) {
  return align_up((size_t)(ceil_div(n < 1 ? 1 : n, kRedChunk) + 2) * 4, 256);
}

static int32_t frobenius_fwd(const float* x, int64_t n, const int32_t* n_rows, int32_t row_len,
                             float* y, float* norm, void* workspace, size_t ws_bytes,
                             void* stream) {
  RS_CHECK_ARG(n >= 1, "rs_frobenius_normalize_fwd: empty input");
  RS_CHECK_ARG(ws_bytes >= rs_frobenius_workspace_size(n), "rs_frobenius: workspace too small");
  hipStream_t st = as_stream(stream);
  const int64_t nb = ceil_div(n, kRedChunk);
  float* partial = static_cast<float*>(workspace);
  dot_partial_kernel<<<(unsigned)nb, kRedThreads, 0, st>>>(x, nullptr, n, n_rows, row_len,
                                                           partial);
  RS_CHECK_LAUNCH();
  fold_partial_kernel<<<1, kRedThreads, 0, st>>>(partial, nb, 0, norm);
  RS_CHECK_LAUNCH();
  scale_div_kernel<<<grid_for(n), 256, 0, st>>>(x, n, n_rows, row_len, norm, y);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

static int32_t frobenius_bwd(const float* dy, const float* y, const float* norm, int64_t n,
                             const int32_t* n_rows, int32_t row_len, float* dx, void* workspace,
                             size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(n >= 1, "rs_frobenius_normalize_bwd: empty input");
  RS_CHECK_ARG(ws_bytes >= rs_frobenius_workspace_size(n), "rs_frobenius: workspace too small");
  hipStream_t st = as_stream(stream);
  const int64_t nb = ceil_div(n, kRedChunk);
  float* partial = static_cast<float*>(workspace);
  float* dot = partial + nb;
  dot_partial_kernel<<<(unsigned)nb, kRedThreads, 0, st>>>(dy, y, n, n_rows, row_len, partial);
  RS_CHECK_LAUNCH();
  fold_partial_kernel<<<1, kRedThreads, 0, st>>>(partial, nb, 1, dot);
  RS_CHECK_LAUNCH();
  frob_bwd_kernel<<<grid_for(n), 256, 0, st>>>(dy, y, n, n_rows, row_len, norm, dot, dx);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_frobenius_normalize_fwd(const float* x, int64_t n, float* y, float* norm,
                                              void* workspace, size_t ws_bytes, void* stream) {
  return frobenius_fwd(x, n, nullptr, 1, y, norm, workspace, ws_bytes, stream);
}

extern "C" int32_t rs_frobenius_normalize_bwd(const float* dy, const float* y, const float* norm,
                                              int64_t n, float* dx, void* workspace,
                                              size_t ws_bytes, void* stream) {
  return frobenius_bwd(dy, y, norm, n, nullptr, 1, dx, workspace, ws_bytes, stream);
}

extern "C" int32_t rs_frobenius_normalize_rows_fwd(const float* x, int64_t n_cap_rows,
                                                   int32_t row_len, const int32_t* n_rows,
                                                   float* y, float* norm, void* workspace,
                                                   size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(row_len >= 1 && n_rows != nullptr, "rs_frobenius_normalize_rows_fwd: bad args");
  return frobenius_fwd(x, n_cap_rows * row_len, n_rows, row_len, y, norm, workspace, ws_bytes,
                       stream);
}

extern "C" int32_t rs_frobenius_normalize_rows_bwd(const float* dy, const float* y,
                                                   const float* norm, int64_t n_cap_rows,
                                                   int32_t row_len, const int32_t* n_rows,
                                                   float* dx, void* workspace, size_t ws_bytes,
                                                   void* stream) {
  RS_CHECK_ARG(row_len >= 1 && n_rows != nullptr, "rs_frobenius_normalize_rows_bwd: bad args");
  return frobenius_bwd(dy, y, norm, n_cap_rows * row_len, n_rows, row_len, dx, workspace,
                       ws_bytes, stream);
}
