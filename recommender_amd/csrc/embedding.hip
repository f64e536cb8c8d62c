// embedding.hip — multi-slot embedding gather (a-1) and the deterministic sparse-gradient
// apply (a-2): segmented sum over the radix-sorted ids fused with the optimizer update.
//
// Row layout: a row of `dim` fp32 is covered by a lane group of LPR lanes (LPR = power of two
// <= 64), each lane moving VEC floats (16 B when dim % 4 == 0) per chunk, CPL chunks per lane.
// At dim = 128 a half-wave moves one 512-B row per instruction, so a wave issues two
// independent rows per load instruction and every load is a full 512-B contiguous segment.
//
// Segmented sum (SURVEY §7 "Bit-exact duplicate reduction"): the sorted entries are cut into
// tiles of RS_DEDUP_TILE; one lane group walks a tile in order, summing consecutive equal rows.
// A run that is a whole segment is finalised in place (optimizer applied to the table row);
// a run cut by a tile edge stores a partial ([tile][0] = continuation, [tile][1] = head part),
// and a fix-up pass folds the partials of each spanning segment in tile order. The order is
// therefore fixed by the sorted order alone (oracle/embedding.py:segment_sum_tiled).
#include <cstdlib>

#include "common.hpp"

namespace rs {

int32_t radix_sort_pairs(uint32_t*, int32_t*, uint32_t*, int32_t*, int64_t, int64_t, void*, size_t,
                         hipStream_t);
size_t radix_sort_ws_size(int64_t);
int32_t exclusive_scan_i32(const int32_t*, int32_t*, int64_t, int32_t*, void*, size_t, hipStream_t);
size_t exclusive_scan_ws_size(int64_t);

// ---- vector row I/O ------------------------------------------------------------------
template <int VEC>
struct RowIO;
template <>
struct RowIO<4> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[4]) {
    float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
// a read-once stream (the walk's gradient rows): non-temporal, so it does not evict the
// table rows and tile partials that are read again
template <int VEC>
__device__ __forceinline__ void load_stream(const float* p, float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    RowIO<VEC>::load(p, v);
  }
}
template <>
struct RowIO<2> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[2]) {
    float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x; v[1] = t.y;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[2]) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  }
};
template <>
struct RowIO<1> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[1]) { v[0] = *p; }
  static __device__ __forceinline__ void store(float* p, const float (&v)[1]) { *p = v[0]; }
};

struct RowGeom {
  int vec, lpr_log2, cpl;
};

static RowGeom row_geom(int dim, const void* const* ptrs, int nptr) {
  int vec = (dim % 4 == 0) ? 4 : (dim % 2 == 0 ? 2 : 1);
  // downgrade the vector width if any base pointer is not aligned for it
  for (int i = 0; i < nptr; ++i) {
    uintptr_t a = reinterpret_cast<uintptr_t>(ptrs[i]);
    while (vec > 1 && (a % (vec * 4)) != 0) vec >>= 1;
  }
  int chunks = dim / vec;
  int lpr = 1, l2 = 0;
  while (lpr < chunks && lpr < 64) { lpr <<= 1; ++l2; }
  int cpl = (chunks + lpr - 1) / lpr;
  int c = 1;
  while (c < cpl) c <<= 1;
  return {vec, l2, c};
}

// ---- a-1: gather ----------------------------------------------------------------------
template <int VEC, int CPL>
__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ table, int64_t n_rows,
                                                     int dim, const void* __restrict__ ids,
                                                     int32_t dtype, int64_t n_ids,
                                                     const int64_t* __restrict__ slot_offsets,
                                                     int32_t n_slots, float* __restrict__ out,
                                                     int32_t* err_flag, int lpr_log2, int64_t out_ld) {
  constexpr int U = 4;
  const int lpr = 1 << lpr_log2;
  const int gl = threadIdx.x & (lpr - 1);
  const int64_t gpb = blockDim.x >> lpr_log2;
  const int64_t groups = (int64_t)gridDim.x * gpb;
  const int64_t g = (int64_t)blockIdx.x * gpb + (threadIdx.x >> lpr_log2);
  bool oob = false;
  for (int64_t base = g; base < n_ids; base += groups * U) {
    float v[U][CPL][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t p = base + u * groups;
      int64_t r = -2;
      if (p < n_ids) {
        r = global_row(ids, dtype, p, slot_offsets, n_slots, n_rows);
        oob |= (r == -1);
      }
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        int col = (gl + c * lpr) * VEC;
        if (r >= 0 && col < dim) {
          RowIO<VEC>::load(table + r * dim + col, v[u][c]);
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e) v[u][c][e] = 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t p = base + u * groups;
      if (p < n_ids) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          int col = (gl + c * lpr) * VEC;
          if (col < dim) RowIO<VEC>::store(out + p * out_ld + col, v[u][c]);
        }
      }
    }
  }
  if (__any(oob) && (threadIdx.x & 63) == 0) flag_oob(err_flag);
}

// Narrow rows whose width is not a multiple of 4 floats (ESMM / MMOE's D = 18: 72-B rows, 8-B
// aligned): the output is a flat [n_ids · dim] array of float2 pairs, one pair per lane, so every
// lane stores and every store instruction writes 512 contiguous bytes (the row-group kernel above
// left 7 of 16 lanes idle per row at D = 18 and ran at 0.27 of HBM)
__global__ __launch_bounds__(256) void gather_flat2_kernel(const float* __restrict__ table,
                                                           int64_t n_rows, int dim,
                                                           const void* __restrict__ ids,
                                                           int32_t dtype, int64_t n_ids,
                                                           const int64_t* __restrict__ slot_offsets,
                                                           int32_t n_slots, float* __restrict__ out,
                                                           int32_t* err_flag) {
  const int64_t pairs = n_ids * dim / 2;
  const int half = dim / 2;
  bool oob = false;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < pairs;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = q / half;
    const int c = 2 * (int)(q - p * half);
    const int64_t r = global_row(ids, dtype, p, slot_offsets, n_slots, n_rows);
    oob |= r == -1;
    const float2 v = r >= 0 ? *reinterpret_cast<const float2*>(table + r * dim + c)
                            : make_float2(0.f, 0.f);
    *reinterpret_cast<float2*>(out + 2 * q) = v;
  }
  if (__any(oob) && (threadIdx.x & 63) == 0) flag_oob(err_flag);
}

// ---- a-2: segmented sum + apply -------------------------------------------------------
// OPT_EMIT: segment sums to (uniq_rows, uniq_grad) in segment order; OPT_DENSE: each segment sum
// stored as row `row` of a dense [n_rows, dim] gradient (a.table)
enum { OPT_SGD = RS_OPT_SGD, OPT_LAZY = RS_OPT_LAZY_ADAM, OPT_KERAS = RS_OPT_KERAS_ADAM, OPT_EMIT = 100,
       OPT_DENSE = 101 };

struct ApplyArgs {
  float* table;
  float* m;
  float* v;
  int dim;
  rs_adam_params p;
  uint32_t* bitmap;       // keras: touched rows
  float* partial;         // [n_tiles][2][dim]
  float* chunk;           // [n_tiles][2][dim] level-1 chunk sums of spanning segments
  uint8_t* tile_flags;    // [n_tiles] bit0: head of a spanning segment, bit1: aligned-group lead
  // grad row of position p = row_scale[p / scale_group] * grad[p] (null: unscaled). The fused
  // DLRM step hands the UNIT interaction gradient and the per-example scale G[b]; the product is
  // one rounded fp32 multiply (__fmul_rn, never contracted into the sum), as if materialised.
  const float* row_scale;
  int32_t scale_group;
  // OPT_EMIT (dedup output)
  float* uniq_grad;
  uint32_t* uniq_rows;
  const int32_t* seg_excl;  // exclusive scan of head flags
  // OPT_EMIT: segment s's sum goes to uniq_grad row seg_map[s] (skipped when < 0) instead of
  // row s (the row-sharded exchange's padded per-owner send buffer, rs_exchange_pack)
  const int32_t* seg_map;
  // the D = 128 walk (tile32_walk) takes only keys in [key_lo, n_rows) as rows; the others are
  // treated as the OOB sentinel (dropped). 0 = every key below n_rows (the row-sharded exchange
  // deduplicates its two owner halves in two launches, rs_embedding_dedup_grad_mapped_range)
  uint32_t key_lo;
  // a key-range walk over part of the key space (the owner halves): groups with no key in range
  // exit before walking (seg_group32_kernel); 0 for full-range walks
  int ranged;
  // OPT_DENSE: the gradient rows in up to 4 segments — position p in [gstart[i], gstart[i+1])
  // reads gseg[i] + (p - gstart[i]) * gld[i] (a table looked up several times hands each
  // lookup's upstream rows, strided column blocks included, without concatenating them);
  // n_gseg 0: grad + p * dim
  const float* gseg[4];
  int64_t gstart[4];
  int64_t gld[4];
  int32_t n_gseg;
};

__device__ __forceinline__ const float* dense_grad_row(const ApplyArgs& a,
                                                       const float* __restrict__ grad, int64_t p,
                                                       int dim) {
  if (a.n_gseg == 0) return grad + p * dim;
  const float* b = a.gseg[0];
  int64_t s0 = 0, ld = a.gld[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    if (i < a.n_gseg && p >= a.gstart[i]) {
      b = a.gseg[i];
      s0 = a.gstart[i];
      ld = a.gld[i];
    }
  }
  return b + (p - s0) * ld;
}

template <int OPT, int VEC>
__device__ __forceinline__ void finalize_chunk(const ApplyArgs& a, uint32_t row, int col,
                                               const float (&g)[VEC], int32_t seg_id) {
  if constexpr (OPT == OPT_EMIT) {
    const int32_t dst = a.seg_map ? a.seg_map[seg_id] : seg_id;
    if (dst >= 0) RowIO<VEC>::store(a.uniq_grad + (int64_t)dst * a.dim + col, g);
  } else if constexpr (OPT == OPT_DENSE) {
    RowIO<VEC>::store(a.table + (int64_t)row * a.dim + col, g);
  } else if constexpr (OPT == OPT_SGD) {
    float* t = a.table + (int64_t)row * a.dim + col;
    float w[VEC];
    RowIO<VEC>::load(t, w);
#pragma unroll
    for (int e = 0; e < VEC; ++e) w[e] = w[e] - a.p.lr * g[e];
    RowIO<VEC>::store(t, w);
  } else {  // lazy / keras Adam on a touched row (Keras _resource_apply_sparse op order)
    int64_t off = (int64_t)row * a.dim + col;
    float w[VEC], m[VEC], v[VEC];
    RowIO<VEC>::load(a.table + off, w);
    RowIO<VEC>::load(a.m + off, m);
    RowIO<VEC>::load(a.v + off, v);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      float mm = m[e] * a.p.beta1;
      mm = mm + g[e] * a.p.one_minus_beta1;
      float gg = g[e] * g[e];
      float vv = v[e] * a.p.beta2;
      vv = vv + gg * a.p.one_minus_beta2;
      float upd = (a.p.lr * mm) / (sqrtf(vv) + a.p.epsilon);
      m[e] = mm;
      v[e] = vv;
      w[e] = w[e] - upd;
    }
    RowIO<VEC>::store(a.table + off, w);
    RowIO<VEC>::store(a.m + off, m);
    RowIO<VEC>::store(a.v + off, v);
  }
}

template <int OPT, int VEC, int CPL>
__device__ __forceinline__ void finalize_row(const ApplyArgs& a, uint32_t row, int gl, int lpr,
                                             const float (&acc)[CPL][VEC], int32_t seg_id) {
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    int col = (gl + c * lpr) * VEC;
    if (col < a.dim) finalize_chunk<OPT, VEC>(a, row, col, acc[c], seg_id);
  }
  // (Keras' touched-row bitmap is marked by keras_bitmap_mark_kernel after the walk: an atomic
  // here, inlined into every emit of the unrolled walk, took the Keras walk past 128 VGPRs —
  // 495 spilled registers, 1.6 ms per apply instead of ≈0.3)
  if constexpr (OPT == OPT_EMIT) {
    if (gl == 0) a.uniq_rows[seg_id] = row;
  }
}

__device__ __forceinline__ int32_t seg_id_of(const ApplyArgs& a, const uint32_t* keys, int64_t k) {
  bool head = (k == 0) || keys[k - 1] != keys[k];
  return a.seg_excl ? a.seg_excl[k] + (head ? 1 : 0) - 1 : 0;
}

// Persistent over the tiles: the grid is a few blocks per CU (kApplyBlocksPerCU) and each lane
// group walks tiles t, t + groups, ... — the walk is bandwidth-bound, and a grid of thousands of
// blocks would hold every CU slot, starving the latency-bound kernels the step runs beside it.
#ifndef RS_APPLY_BLOCKS_PER_CU
#define RS_APPLY_BLOCKS_PER_CU (1 << 20)  // effectively one lane group per tile (A/B: 2-64 per CU were slower)
#endif
constexpr int kApplyBlocksPerCU = RS_APPLY_BLOCKS_PER_CU;

template <int OPT, int VEC, int CPL>
__device__ __forceinline__ void seg_tile_one(const uint32_t* __restrict__ keys,
                                             const int32_t* __restrict__ pos, int64_t n,
                                             uint32_t n_rows, const float* __restrict__ grad,
                                             const ApplyArgs& a, int lpr_log2, int64_t t);

template <int OPT, int VEC, int CPL>
__global__ __launch_bounds__(256) void seg_tile_kernel(const uint32_t* __restrict__ keys,
                                                       const int32_t* __restrict__ pos, int64_t n,
                                                       uint32_t n_rows, const float* __restrict__ grad,
                                                       ApplyArgs a, int lpr_log2, int64_t n_tiles) {
  const int gpb = blockDim.x >> lpr_log2;
  const int64_t groups = (int64_t)gridDim.x * gpb;
  for (int64_t t = (int64_t)blockIdx.x * gpb + (threadIdx.x >> lpr_log2); t < n_tiles; t += groups)
    seg_tile_one<OPT, VEC, CPL>(keys, pos, n, n_rows, grad, a, lpr_log2, t);
}

template <int OPT, int VEC, int CPL>
__device__ __forceinline__ void seg_tile_one(const uint32_t* __restrict__ keys,
                                             const int32_t* __restrict__ pos, int64_t n,
                                             uint32_t n_rows, const float* __restrict__ grad,
                                             const ApplyArgs& a, int lpr_log2, int64_t t) {
  constexpr int T = RS_DEDUP_TILE;
  constexpr int U = 8;
  const int lpr = 1 << lpr_log2;
  const int gl = threadIdx.x & (lpr - 1);
  const int64_t k0 = t * T;
  const int64_t k1 = k0 + T < n ? k0 + T : n;
  const int dim = a.dim;

  uint32_t run_row = keys[k0];
  int64_t run_start = k0;
  bool run_starts = (k0 == 0) || keys[k0 - 1] != run_row;
  // an always-valid gradient address for entries that carry no gradient (loaded, never used)
  const float* grad0 = (OPT == OPT_DENSE && a.n_gseg > 0) ? a.gseg[0] : grad;
  float acc[CPL][VEC];
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[c][e] = 0.f;

  auto emit = [&](uint32_t row, bool starts, bool ends, int64_t head_k) {
    if (row >= n_rows) return;  // OOB sentinel run: gradient dropped
    if (starts && ends) {
      finalize_row<OPT, VEC, CPL>(a, row, gl, lpr, acc, OPT == OPT_EMIT ? seg_id_of(a, keys, head_k) : 0);
    } else {
      float* dst = a.partial + ((t * 2) + (starts ? 1 : 0)) * (int64_t)dim;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        int col = (gl + c * lpr) * VEC;
        if (col < dim) RowIO<VEC>::store(dst + col, acc[c]);
      }
    }
  };

  for (int64_t kb = k0; kb < k1; kb += U) {
    float r[U][CPL][VEC];
    float sc[U];  // applied at the sum: a multiply right behind each load would serialise them
    uint32_t kk[U];
    // Round 6: unguarded loads from always-valid addresses (guarded, the compiler waited for
    // each batch entry's loads in turn). An entry past the tile reads entry k0 (never consumed);
    // an OOB key's rows are read from row 0 (its run is never emitted); lanes past dim read
    // column 0 (never stored).
    uint32_t kr[U];
    int32_t pr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = kb + u < k1 ? kb + u : k0;
      kr[u] = keys[k];
      pr[u] = pos[k];
    }
    const float* rsp = a.row_scale ? a.row_scale : grad0;
    float sr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool valid = kb + u < k1;
      kk[u] = valid ? kr[u] : 0xFFFFFFFFu;
      const int64_t p = valid ? pr[u] : 0;
      const bool live = valid && kk[u] < n_rows;
      sr[u] = rsp[a.row_scale && live ? p / a.scale_group : 0];
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        int col = (gl + c * lpr) * VEC;
        const bool ok = live && col < dim;
        if constexpr (OPT == OPT_DENSE)
          load_stream<VEC>(ok ? dense_grad_row(a, grad, p, dim) + col : grad0, r[u][c]);
        else
          load_stream<VEC>(ok ? grad + p * dim + col : grad0, r[u][c]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) sc[u] = a.row_scale ? sr[u] : 1.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t k = kb + u;
      if (k < k1) {
        if (kk[u] != run_row) {
          emit(run_row, run_starts, true, run_start);
#pragma unroll
          for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[c][e] = 0.f;
          run_row = kk[u];
          run_starts = true;
          run_start = k;
        }
        if (a.row_scale) {
#pragma unroll
          for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[c][e] += __fmul_rn(sc[u], r[u][c][e]);
        } else {
#pragma unroll
          for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[c][e] += r[u][c][e];
        }
      }
    }
  }
  bool ends = (k1 >= n) || keys[k1] != run_row;
  emit(run_row, run_starts, ends, run_start);
  // fix-up roles of this tile (consumed by seg_chunk_kernel / seg_fixup_kernel)
  if (gl == 0) {
    uint8_t f = 0;
    if (!ends && run_starts && run_row < n_rows) f |= 1;  // last run opens a spanning segment
    const uint32_t fk = keys[k0];
    if ((t % 32) == 0 && k0 > 0 && fk < n_rows && keys[k0 - 1] == fk) f |= 2;
    a.tile_flags[t] = f;
  }
}

// D = 128 (a half-wave of 32 lanes x float4 per row, RS_DEDUP_TILE = 32): the same walk with
// the tile's 32 keys / positions / row scales loaded lane-parallel in one instruction each (lane
// gl holds entry gl; entry u's values come by a width-32 shuffle) instead of per entry, and the
// gradient rows of the next 8 entries in flight while the current 8 are summed. Same order of
// additions as seg_tile_kernel: bit-identical results. The walk of one tile by one half-wave;
// a run cut by a tile edge leaves its partial at pbase[(starts ? 1 : 0) * 128 ..] (global tile
// partials or the group kernel's LDS), and the returned edges say how the tile's runs continue.
struct Tile32Edges {
  uint32_t last_row;  // row of the tile's last run
  bool last_open;     // that run started in this tile and continues into the next (valid row)
  bool first_cont;    // the tile's first run continues from the previous tile (valid row)
  uint32_t first_key;
};

// Q > 0 (SGD only): the table read-modify-writes of the runs that end inside the tile are queued
// (Q run sums in registers) and done Q at a time — their Q table-row loads issued together —
// instead of one per run: a table load waits for every load issued before it (vmcnt counts in
// order), so an inline update drains the in-flight gradient rows at each run end. Same
// arithmetic, each row written once: bit-identical.
// (Round 5 also built row preloads at the tile start, RS_APPLY_PRE: measured 249-261 us against
// 232-238 and removed in round 6.)
template <int OPT, int Q = 0>
__device__ __forceinline__ Tile32Edges tile32_walk(const uint32_t* __restrict__ keys,
                                                   const int32_t* __restrict__ pos, int64_t n,
                                                   uint32_t n_rows, const float* __restrict__ grad,
                                                   const ApplyArgs& a, int64_t t, float* pbase) {
  constexpr int T = 32, VEC = 4, CPL = 1, U = 8;
  constexpr bool kQueue = Q > 0 && OPT == OPT_SGD;
  constexpr int QN = Q > 0 ? Q : 1;
  const int gl = threadIdx.x & 31;
  const int64_t k0 = t * T;
  const int64_t k1 = k0 + T < n ? k0 + T : n;
  const int ne = (int)(k1 - k0);
  const int dim = a.dim;  // 128
  const int col = gl * VEC;
  // lane-parallel tile metadata
  const bool mine = gl < ne;
  // a row of this walk: below n_rows and at or past a.key_lo (one unsigned compare)
  const uint32_t klo = a.key_lo, kspan = n_rows - a.key_lo;
  auto key_ok = [&](uint32_t k) { return k - klo < kspan; };
  // Round 6: every load below is issued unguarded from an address that is always valid (the
  // guarded forms made the compiler branch around each load and wait for all of them at every
  // join — gfx950 ISA: the two gradient batches and the queued table rows were each drained
  // with vmcnt(0), so the next batch never flew under the current one). The tile's keys and
  // positions and its two neighbour keys go out in one round trip.
  const int64_t ki = k0 + (mine ? gl : 0);
  const uint32_t kraw = keys[ki];
  const int32_t praw = pos[ki];
  const uint32_t kbraw = keys[k0 > 0 ? k0 - 1 : 0];
  const uint32_t karaw = keys[k1 < n ? k1 : n - 1];
  const uint32_t kv = mine ? kraw : 0xFFFFFFFFu;
  const int32_t pv = mine ? praw : 0;
  const bool lv = mine && key_ok(kv);
  const uint32_t key_before = k0 > 0 ? kbraw : 0xFFFFFFFFu;
  const uint32_t key_after = k1 < n ? karaw : 0xFFFFFFFEu;
  float sv = 1.f;
  if (a.row_scale) sv = a.row_scale[(lv ? pv : 0) / a.scale_group];  // used at lv lanes only
  auto key_of = [&](int u) { return (uint32_t)__shfl((int)kv, u, 32); };
  // the row scale multiplies at the sum (consume), not here: a multiply right behind each load
  // would wait for it and serialise the batch's loads (measured: apply 215 -> 272 us alone).
  // An entry that is not a row of this walk (past the tile, out of range) reads gradient row 0
  // instead: its run is never emitted (emit drops rows that fail key_ok; consume stops at ne).
  auto load_batch = [&](int b0, float (&r)[U][VEC]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = b0 + u;
      const int32_t p = __shfl(pv, e, 32);
      const bool live = e < ne && key_ok(key_of(e));
      load_stream<VEC>(grad + (live ? (int64_t)p * dim : 0) + col, r[u]);
    }
  };
  uint32_t run_row = key_of(0);
  int run_start = 0;
  bool run_starts = run_row != key_before;
  float acc[CPL][VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) acc[0][c] = 0.f;
  uint32_t qrow[QN];
  float qacc[QN][VEC];
  int qn = 0;
  auto flush = [&]() {
    if constexpr (kQueue) {
      float tr[QN][VEC];
#pragma unroll
      for (int i = 0; i < QN; ++i) {  // unguarded (a free slot re-reads row qrow[0] or row 0)
        const uint32_t rr = i < qn ? qrow[i] : (qn > 0 ? qrow[0] : 0u);
        RowIO<VEC>::load(a.table + (int64_t)rr * dim + col, tr[i]);
      }
#pragma unroll
      for (int i = 0; i < QN; ++i) {
        if (i < qn) {
#pragma unroll
          for (int c = 0; c < VEC; ++c) tr[i][c] = tr[i][c] - a.p.lr * qacc[i][c];
          RowIO<VEC>::store(a.table + (int64_t)qrow[i] * dim + col, tr[i]);
        }
      }
      qn = 0;
    }
  };
  auto emit = [&](uint32_t row, bool starts, bool ends, int head_e) {
    if (!key_ok(row)) return;  // OOB sentinel (or out-of-range) run: gradient dropped
    if (starts && ends) {
      if constexpr (kQueue) {
        if (qn == QN) flush();
#pragma unroll
        for (int i = 0; i < QN; ++i) {
          if (i == qn) {
            qrow[i] = row;
#pragma unroll
            for (int c = 0; c < VEC; ++c) qacc[i][c] = acc[0][c];
          }
        }
        ++qn;
      } else {
        finalize_row<OPT, VEC, CPL>(a, row, gl, 32, acc, OPT == OPT_EMIT ? seg_id_of(a, keys, k0 + head_e) : 0);
      }
    } else {
      RowIO<VEC>::store(pbase + (starts ? 1 : 0) * dim + col, acc[0]);
    }
  };
  float rA[U][VEC], rB[U][VEC];
  load_batch(0, rA);
  auto consume = [&](int b0, float (&r)[U][VEC]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = b0 + u;
      if (e < ne) {
        const uint32_t ku = key_of(e);
        if (ku != run_row) {
          emit(run_row, run_starts, true, run_start);
#pragma unroll
          for (int c = 0; c < VEC; ++c) acc[0][c] = 0.f;
          run_row = ku;
          run_starts = true;
          run_start = e;
        }
        if (a.row_scale) {
          const float sc = __shfl(sv, e, 32);
#pragma unroll
          for (int c = 0; c < VEC; ++c) acc[0][c] += __fmul_rn(sc, r[u][c]);
        } else {
#pragma unroll
          for (int c = 0; c < VEC; ++c) acc[0][c] += r[u][c];
        }
      }
    }
  };
#ifndef RS_T32_SINGLE
  // four batches of 8, the next batch's rows in flight while the current one is summed
  load_batch(U, rB);
  consume(0, rA);
  if (ne > 2 * U) load_batch(2 * U, rA);
  consume(U, rB);
  if (ne > 3 * U) load_batch(3 * U, rB);
  if (ne > 2 * U) consume(2 * U, rA);
  if (ne > 3 * U) consume(3 * U, rB);
#else
  consume(0, rA);
  for (int b0 = U; b0 < ne; b0 += U) {
    load_batch(b0, rA);
    consume(b0, rA);
  }
#endif
  const bool ends = key_after != run_row;
  emit(run_row, run_starts, ends, run_start);
  flush();
  Tile32Edges ed;
  ed.last_row = run_row;
  ed.last_open = !ends && run_starts && key_ok(run_row);
  ed.first_key = key_of(0);
  ed.first_cont = k0 > 0 && key_ok(ed.first_key) && key_before == ed.first_key;
  return ed;
}

template <int OPT>
__global__ __launch_bounds__(256) void seg_tile32_kernel(const uint32_t* __restrict__ keys,
                                                         const int32_t* __restrict__ pos, int64_t n,
                                                         uint32_t n_rows,
                                                         const float* __restrict__ grad,
                                                         ApplyArgs a, int64_t n_tiles) {
  const int64_t t = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  if (t >= n_tiles) return;
  const Tile32Edges e = tile32_walk<OPT>(keys, pos, n, n_rows, grad, a, t,
                                         a.partial + t * 2 * (int64_t)a.dim);
  if ((threadIdx.x & 31) == 0) {
    uint8_t f = 0;
    if (e.last_open) f |= 1;  // last run opens a spanning segment
    if ((t % 32) == 0 && e.first_cont) f |= 2;
    a.tile_flags[t] = f;
  }
}

// The D = 128 walk with the first fix-up level folded in: a block of 32 half-waves walks one
// ALIGNED group of 32 tiles (= kFixChunk), its cut runs' partials kept in LDS. After a block
// barrier each segment that spans tiles of the group is folded in tile order from LDS — the
// level-1 sum of seg_chunk_kernel, same additions in the same order — and finalised on the spot
// when it also ends inside the group (the level-2 fold of a single group sum is that sum).
// Only segments that cross a group edge leave global state: the head's group sum
// (chunk[t][1], tile flag bit 0) and, at a group's first tile, the continuation's group sum
// (chunk[t][0]); seg_fixup_kernel folds those (level 2). Bit-identical to seg_tile32 + seg_chunk
// + seg_fixup, one launch fewer and no global partials.
template <int OPT, int Q = 0>
__global__ __launch_bounds__(1024) void seg_group32_kernel(const uint32_t* __restrict__ keys,
                                                           const int32_t* __restrict__ pos,
                                                           int64_t n, uint32_t n_rows,
                                                           const float* __restrict__ grad,
                                                           ApplyArgs a, int64_t n_tiles) {
  constexpr int G = 32, D = 128, T = 32;
  __shared__ __attribute__((aligned(16))) float ps[G][2][D];
  __shared__ uint32_t fkey[G];
  __shared__ int skip;
  const int gi = threadIdx.x >> 5, gl = threadIdx.x & 31;
  const int64_t t = (int64_t)blockIdx.x * G + gi;
  const bool live = t < n_tiles;
  // Key-range walks only (the row-sharded dedup's owner halves: a.ranged, a kernel argument,
  // so the branch is uniform): a group with no key in [key_lo, n_rows) has nothing to sum or
  // write. The full-range walk (the production apply) skips the check (two dependent key loads
  // and a block barrier per group; interleaved A/B, round 6: no measurable cost either way).
  if (a.ranged) {
    if (threadIdx.x == 0) {
      const int64_t f = (int64_t)blockIdx.x * G * T;
      const int64_t l = (f + (int64_t)G * T < n ? f + (int64_t)G * T : n) - 1;
      skip = f < n && (keys[l] < a.key_lo || keys[f] >= n_rows);
    }
    __syncthreads();
    if (skip) {  // the walk would find no run in range: the same (empty) tile flags
      if (gl == 0 && live) a.tile_flags[t] = 0;
      return;
    }
  }
  Tile32Edges e{};
  if (live) e = tile32_walk<OPT, Q>(keys, pos, n, n_rows, grad, a, t, &ps[gi][0][0]);
  if (gl == 0) fkey[gi] = live ? e.first_key : 0xFFFFFFFFu;
  __syncthreads();
  if (!live) return;
  const int col = gl * 4;
  uint8_t gflag = 0;
  if (e.last_open) {  // head of a spanning segment: its level-1 sum inside this group
    const uint32_t row = e.last_row;
    float acc[1][4];
    {
      const float4 h = *reinterpret_cast<const float4*>(&ps[gi][1][col]);
      acc[0][0] = h.x; acc[0][1] = h.y; acc[0][2] = h.z; acc[0][3] = h.w;
    }
    int u = gi + 1;
    for (; u < G && fkey[u] == row; ++u) {
      const float4 c = *reinterpret_cast<const float4*>(&ps[u][0][col]);
      acc[0][0] += c.x; acc[0][1] += c.y; acc[0][2] += c.z; acc[0][3] += c.w;
    }
    const int64_t tn = ((int64_t)blockIdx.x + 1) * G;  // first tile of the next group
    const bool crosses = u == G && tn < n_tiles && keys[tn * T] == row;
    if (crosses) {
      RowIO<4>::store(a.chunk + (t * 2 + 1) * (int64_t)D + col, acc[0]);
      gflag = 1;
    } else {
      finalize_row<OPT, 4, 1>(a, row, gl, 32, acc,
                              OPT == OPT_EMIT ? seg_id_of(a, keys, t * T + T - 1) : 0);
    }
  }
  if (gi == 0 && e.first_cont) {  // the group's first tile continues a segment from before
    const uint32_t fk = e.first_key;
    float acc[4];
    {
      const float4 h = *reinterpret_cast<const float4*>(&ps[0][0][col]);
      acc[0] = h.x; acc[1] = h.y; acc[2] = h.z; acc[3] = h.w;
    }
    for (int u = 1; u < G && fkey[u] == fk; ++u) {
      const float4 c = *reinterpret_cast<const float4*>(&ps[u][0][col]);
      acc[0] += c.x; acc[1] += c.y; acc[2] += c.z; acc[3] += c.w;
    }
    RowIO<4>::store(a.chunk + (t * 2) * (int64_t)D + col, acc);
  }
  if (gl == 0) a.tile_flags[t] = gflag;
}

// ---- fix-up of segments that span tiles ----------------------------------------------
// A spanning segment with head tile h and last tile e has one partial per tile:
//   P(h) = partial[h][1] (head part), P(t) = partial[t][0] for t = h+1..e.
// Level 1: inside each ALIGNED group of kFixChunk tiles, the segment's partials are folded in
// tile order by one lane group (the head tile for the head's group, else the group's first
// tile) into chunk[leader][role] (role 1 = head group, 0 = continuation group).
// Level 2: one lane group per head tile folds the group sums in order and finalises the row.
// No search is needed: every boundary test is a load of the first key of a tile.
constexpr int kFixChunk = 32;

template <int VEC, int CPL>
__device__ __forceinline__ void load_or_zero(const float* p, int dim, int gl, int lpr,
                                             float (&acc)[CPL][VEC]) {
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    int col = (gl + c * lpr) * VEC;
    if (col < dim) {
      RowIO<VEC>::load(p + col, acc[c]);
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[c][e] = 0.f;
    }
  }
}

template <int VEC, int CPL>
__device__ __forceinline__ void store_row(float* p, int dim, int gl, int lpr,
                                          const float (&acc)[CPL][VEC]) {
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    int col = (gl + c * lpr) * VEC;
    if (col < dim) RowIO<VEC>::store(p + col, acc[c]);
  }
}

// acc += partial[t][0] for t = t1, t1+1, ... while tile t's first key == key, t < t_end
template <int VEC, int CPL>
__device__ __forceinline__ void fold_group(const uint32_t* keys, int64_t n, uint32_t key,
                                           const float* part, int64_t t1, int64_t t_end, int dim,
                                           int gl, int lpr, float (&acc)[CPL][VEC]) {
  constexpr int T = RS_DEDUP_TILE;
  constexpr int U = 8;
  for (int64_t t = t1; t < t_end; t += U) {
    bool in[U];
    float r[U][CPL][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t tt = t + u;
      in[u] = tt < t_end && tt * T < n && keys[tt * T] == key;
    }
    bool more = true;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      more = more && in[u];
      in[u] = more;  // the segment is contiguous: stop at the first tile it does not reach
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (in[u]) {
        load_or_zero<VEC, CPL>(part + ((t + u) * 2) * (int64_t)dim, dim, gl, lpr, r[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (in[u])
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[c][e] += r[u][c][e];
    if (!more) return;
  }
}

// level 1: one lane group per tile, in up to two roles
template <int VEC, int CPL>
__global__ __launch_bounds__(256) void seg_chunk_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                        uint32_t n_rows, ApplyArgs a, int lpr_log2,
                                                        int64_t n_tiles, float* __restrict__ chunk) {
  constexpr int T = RS_DEDUP_TILE;
  const int lpr = 1 << lpr_log2;
  const int gl = threadIdx.x & (lpr - 1);
  const int64_t t = (int64_t)blockIdx.x * (blockDim.x >> lpr_log2) + (threadIdx.x >> lpr_log2);
  if (t >= n_tiles) return;
  const uint8_t flags = a.tile_flags[t];
  if (flags == 0) return;
  const int dim = a.dim;
  const int64_t k0 = t * T;
  const int64_t klast = (k0 + T < n ? k0 + T : n) - 1;
  const int64_t group_end = (t / kFixChunk + 1) * kFixChunk;  // first tile of the next group
  float acc[CPL][VEC];
  // role 1: head tile of a segment that continues into tile t+1
  if (flags & 1) {
    const uint32_t lk = keys[klast];
    load_or_zero<VEC, CPL>(a.partial + (t * 2 + 1) * (int64_t)dim, dim, gl, lpr, acc);
    fold_group<VEC, CPL>(keys, n, lk, a.partial, t + 1, group_end, dim, gl, lpr, acc);
    store_row<VEC, CPL>(chunk + (t * 2 + 1) * (int64_t)dim, dim, gl, lpr, acc);
  }
  // role 0: first tile of an aligned group, continuing a segment from the previous group
  if (flags & 2) {
    const uint32_t fk = keys[k0];
    load_or_zero<VEC, CPL>(a.partial + (t * 2) * (int64_t)dim, dim, gl, lpr, acc);
    fold_group<VEC, CPL>(keys, n, fk, a.partial, t + 1, group_end, dim, gl, lpr, acc);
    store_row<VEC, CPL>(chunk + (t * 2) * (int64_t)dim, dim, gl, lpr, acc);
  }
}

// level 2: one lane group per head tile of a spanning segment
template <int OPT, int VEC, int CPL>
__device__ __forceinline__ void fixup_one(const uint32_t* __restrict__ keys, const ApplyArgs& a,
                                          int lpr_log2, int64_t n_tiles,
                                          const float* __restrict__ chunk, int64_t t);

template <int OPT, int VEC, int CPL>
__global__ __launch_bounds__(256) void seg_fixup_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                        uint32_t n_rows, ApplyArgs a, int lpr_log2,
                                                        int64_t n_tiles,
                                                        const float* __restrict__ chunk) {
  const int64_t t = (int64_t)blockIdx.x * (blockDim.x >> lpr_log2) + (threadIdx.x >> lpr_log2);
  if (t >= n_tiles - 1) return;
  if (!(a.tile_flags[t] & 1)) return;  // not the head tile of a spanning segment
  fixup_one<OPT, VEC, CPL>(keys, a, lpr_log2, n_tiles, chunk, t);
}

// Level 2 with the whole wave on one head tile (the generic-D path): each of the wave's
// 64/lpr lane groups loads 16 following groups' leader keys and sums, so a hot row spanning
// hundreds of groups (DIEN's padding id: ~350 groups) costs one load latency per 64 groups
// instead of per 16; the group sums are then added in group order by shuffling each lane
// group's values across, so the additions are those of fixup_one, in the same order.
template <int OPT, int VEC, int CPL>
__global__ __launch_bounds__(256) void seg_fixup_wave_kernel(const uint32_t* __restrict__ keys,
                                                             ApplyArgs a, int lpr_log2,
                                                             int64_t n_tiles,
                                                             const float* __restrict__ chunk) {
  constexpr int T = RS_DEDUP_TILE;
  constexpr int U = 16;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n_tiles - 1) return;             // wave-uniform
  if (!(a.tile_flags[t] & 1)) return;       // not the head tile of a spanning segment
  const int lane = threadIdx.x & 63;
  const int lpr = 1 << lpr_log2;
  const int nlg = 64 >> lpr_log2;           // lane groups per wave (1..64)
  const int lg = lane >> lpr_log2, gl = lane & (lpr - 1);
  const int64_t klast = t * T + T - 1;
  const uint32_t row = keys[klast];
  const int dim = a.dim;
  float acc[CPL][VEC];
  load_or_zero<VEC, CPL>(chunk + (t * 2 + 1) * (int64_t)dim, dim, gl, lpr, acc);
  const int span = nlg * U < 64 ? nlg * U : 64;  // groups per round (<= 64 continuation bits)
  for (int64_t g = t / kFixChunk + 1;; g += span) {
    uint32_t k[U];
    float r[U][CPL][VEC];
    uint32_t mine = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t gg = g + (int64_t)lg * U + u;
      const int64_t tt = gg * kFixChunk;
      const bool in = lg * U + u < span && tt < n_tiles;
      k[u] = in ? keys[tt * T] : ~row;
      if (in)
        load_or_zero<VEC, CPL>(chunk + (tt * 2) * (int64_t)dim, dim, gl, lpr, r[u]);
      else
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
          for (int e = 0; e < VEC; ++e) r[u][c][e] = 0.f;
      mine |= (k[u] == row ? 1u : 0u) << u;
    }
    // continuation bits of all lane groups, in group order; the segment covers the leading ones
    uint64_t w = 0;
    for (int src = 0; src < nlg && src * U < span; ++src)
      w |= (uint64_t)(uint32_t)__shfl((int)mine, src * lpr) << (src * U);
    const int nrun = ~w == 0ull ? 64 : (int)__builtin_ctzll(~w);  // bits >= span are 0
    for (int src = 0; src < nlg && src * U < nrun; ++src) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float v[CPL][VEC];
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
          for (int e = 0; e < VEC; ++e) v[c][e] = __shfl(r[u][c][e], src * lpr + gl);
        if (src * U + u < nrun)
#pragma unroll
          for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[c][e] += v[c][e];
      }
    }
    if (nrun < span) break;
  }
  if (lg == 0) finalize_row<OPT, VEC, CPL>(a, row, gl, lpr, acc, OPT == OPT_EMIT ? seg_id_of(a, keys, klast) : 0);
}

// The level-2 pass after seg_group32_kernel: few tiles head a segment that crosses a group edge,
// so a small grid sweeps the tile flags instead of one lane group per tile — each half-wave
// loads the flags of 32 tiles at once and folds the flagged ones (same fold as seg_fixup_kernel).
template <int OPT>
__global__ __launch_bounds__(256) void seg_fixup_sweep_kernel(const uint32_t* __restrict__ keys,
                                                              ApplyArgs a, int64_t n_tiles,
                                                              const float* __restrict__ chunk) {
  const int gl = threadIdx.x & 31;
  const int64_t groups = (int64_t)gridDim.x * 8;
  for (int64_t t0 = ((int64_t)blockIdx.x * 8 + (threadIdx.x >> 5)) * 32; t0 < n_tiles - 1;
       t0 += groups * 32) {
    const int64_t tl = t0 + gl;
    const bool head = tl < n_tiles - 1 && (a.tile_flags[tl] & 1);
    uint32_t bits = (uint32_t)(__ballot(head) >> (threadIdx.x & 32));
    while (bits) {
      const int u = __builtin_ctz(bits);
      bits &= bits - 1;
      fixup_one<OPT, 4, 1>(keys, a, 5, n_tiles, chunk, t0 + u);
    }
  }
}

template <int OPT, int VEC, int CPL>
__device__ __forceinline__ void fixup_one(const uint32_t* __restrict__ keys, const ApplyArgs& a,
                                          int lpr_log2, int64_t n_tiles,
                                          const float* __restrict__ chunk, int64_t t) {
  constexpr int T = RS_DEDUP_TILE;
  // 16 groups per round trip: the group-leader keys and the group sums are loaded together
  // (speculatively past the segment's end, discarded there), then added in group order — a hot
  // row spanning hundreds of groups (e.g. a padding id) costs one load latency per 16 groups
  constexpr int U = 16;
  const int lpr = 1 << lpr_log2;
  const int gl = threadIdx.x & (lpr - 1);
  const int64_t klast = t * T + T - 1;
  const uint32_t row = keys[klast];
  const int dim = a.dim;
  float acc[CPL][VEC];
  load_or_zero<VEC, CPL>(chunk + (t * 2 + 1) * (int64_t)dim, dim, gl, lpr, acc);
  // following groups: leader tile g*32 continues the segment iff its first key == row
  for (int64_t g = t / kFixChunk + 1;; g += U) {
    bool in[U];
    float r[U][CPL][VEC];
    bool more = true;
    uint32_t k[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t tt = (g + u) * kFixChunk;
      k[u] = tt < n_tiles ? keys[tt * T] : ~row;
      if (tt < n_tiles)
        load_or_zero<VEC, CPL>(chunk + ((g + u) * kFixChunk * 2) * (int64_t)dim, dim, gl, lpr, r[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      in[u] = more && k[u] == row;
      more = in[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (in[u])
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[c][e] += r[u][c][e];
    if (!more) break;
  }
  finalize_row<OPT, VEC, CPL>(a, row, gl, lpr, acc, OPT == OPT_EMIT ? seg_id_of(a, keys, klast) : 0);
}

__global__ void head_flags_kernel(const uint32_t* __restrict__ keys, int64_t n, uint32_t n_rows,
                                  int32_t* __restrict__ flags) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t k = keys[i];
    flags[i] = (k < n_rows && (i == 0 || keys[i - 1] != k)) ? 1 : 0;
  }
}

// One Keras dense-Adam step of an element whose slice holds no gradient (g = 0): m·β1, v·β2,
// var -= lr_t·m/(√v + ε) [3p TF 2.2 _resource_apply_sparse, untouched rows]. Shared by the dense
// sweep and the deferred replay below so that both round identically.
__device__ __forceinline__ void keras_decay(float& w, float& m, float& v, float lr, float b1,
                                            float b2, float eps) {
  const float m1 = m * b1;
  const float v1 = v * b2;
  const float upd = (lr * m1) / (sqrtf(v1) + eps);
  m = m1;
  v = v1;
  w = w - upd;
}

// A (m, v) chunk whose m is +0 and v is ±0 in every element decays to itself and moves no
// weight: m·β1 = +0, v·β2 = ±0, lr·(+0) / (√v + ε) = +0 and w − (+0) = w for every w (−0
// included). Any number of such steps is the identity, so the sweep and the replay skip the
// chunk — bit for bit the same state — without loading its weights or storing anything (the
// rows Keras' dense decay walks but that no gradient has reached yet). A −0 in m is not skipped
// (w = −0 would become +0).
template <int VEC>
__device__ __forceinline__ bool keras_state_zero(const float (&mm)[VEC], const float (&vv)[VEC]) {
  bool z = true;
#pragma unroll
  for (int e = 0; e < VEC; ++e) z &= (__float_as_uint(mm[e]) == 0u) & (vv[e] == 0.0f);
  return z;
}

// Keras dense sweep over untouched rows (touched rows were fully updated by the sparse pass)
template <int VEC>
__global__ __launch_bounds__(256) void keras_dense_sweep_kernel(float* __restrict__ w,
                                                                float* __restrict__ m,
                                                                float* __restrict__ v, int64_t n_rows,
                                                                int dim, rs_adam_params p,
                                                                const uint32_t* __restrict__ bitmap) {
  const int64_t chunks_per_row = dim / VEC;
  const int64_t total = n_rows * chunks_per_row;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < total; i += stride) {
    int64_t row = i / chunks_per_row;
    if ((bitmap[row >> 5] >> (row & 31)) & 1u) continue;
    int64_t off = i * VEC;
    float ww[VEC], mm[VEC], vv[VEC];
    RowIO<VEC>::load(m + off, mm);
    RowIO<VEC>::load(v + off, vv);
    if (keras_state_zero<VEC>(mm, vv)) continue;
    RowIO<VEC>::load(w + off, ww);
#pragma unroll
    for (int e = 0; e < VEC; ++e) keras_decay(ww[e], mm[e], vv[e], p.lr, p.beta1, p.beta2, p.epsilon);
    RowIO<VEC>::store(w + off, ww);
    RowIO<VEC>::store(m + off, mm);
    RowIO<VEC>::store(v + off, vv);
  }
}

// Deferred Keras decay (SparseAdam(mode='keras', defer_decay=True)): instead of sweeping all V
// rows every step, row r records last[r], the last step applied to it. Before a step s reads
// its rows, the step's unique rows replay the skipped steps last[r]+1 .. s-1 with the very
// arithmetic of the sweep (keras_decay, lr_t of each step from lr_hist[step]) and claim step s
// (its sparse apply follows); materialize replays every row up to the current step. The state
// after materialize equals the dense-sweep state bit for bit.
template <int VEC>
__device__ __forceinline__ void keras_replay_row(float* w, float* m, float* v, int64_t r, int dim,
                                                 int gl, int lpr, int32_t from, int32_t to,
                                                 const float* lr_hist, float b1, float b2,
                                                 float eps) {
  for (int col = gl * VEC; col < dim; col += lpr * VEC) {
    const int64_t off = r * dim + col;
    float ww[VEC], mm[VEC], vv[VEC];
    RowIO<VEC>::load(m + off, mm);
    RowIO<VEC>::load(v + off, vv);
    if (keras_state_zero<VEC>(mm, vv)) continue;  // every replayed step is the identity
    RowIO<VEC>::load(w + off, ww);
    for (int32_t st = from; st <= to; ++st) {
      const float lr = lr_hist[st];
#pragma unroll
      for (int e = 0; e < VEC; ++e) keras_decay(ww[e], mm[e], vv[e], lr, b1, b2, eps);
    }
    RowIO<VEC>::store(w + off, ww);
    RowIO<VEC>::store(m + off, mm);
    RowIO<VEC>::store(v + off, vv);
  }
}

template <int VEC>
__global__ __launch_bounds__(256) void keras_catchup_kernel(
    float* __restrict__ w, float* __restrict__ m, float* __restrict__ v, int32_t* __restrict__ last,
    uint32_t n_rows, int dim, const uint32_t* __restrict__ rows, int64_t n,
    const float* __restrict__ lr_hist, int32_t step, float b1, float b2, float eps, int lpr_log2) {
  const int lpr = 1 << lpr_log2;
  const int gl = threadIdx.x & (lpr - 1);
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> lpr_log2;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> lpr_log2; i < n; i += stride) {
    const uint32_t r = rows[i];
    if (r >= n_rows || (i > 0 && rows[i - 1] == r)) continue;  // one lane group per unique row
    const int32_t l0 = last[r];
    if (l0 + 1 <= step - 1)
      keras_replay_row<VEC>(w, m, v, r, dim, gl, lpr, l0 + 1, step - 1, lr_hist, b1, b2, eps);
    // caught up through step - 1; the step's sparse apply marks it step once it ran
    // (rs_keras_adam_mark), so a presort whose apply never runs leaves the step to a replay
    if (gl == 0) last[r] = step - 1;
  }
}

// after the sparse apply of step s: its unique rows are now up to date through s
__global__ __launch_bounds__(256) void keras_mark_kernel(int32_t* __restrict__ last, uint32_t n_rows,
                                                          const uint32_t* __restrict__ rows,
                                                          int64_t n, int32_t step) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = rows[i];
    if (r < n_rows && (i == 0 || rows[i - 1] != r)) last[r] = step;
  }
}

template <int VEC>
__global__ __launch_bounds__(256) void keras_materialize_kernel(
    float* __restrict__ w, float* __restrict__ m, float* __restrict__ v, int32_t* __restrict__ last,
    int64_t n_rows, int dim, const float* __restrict__ lr_hist, int32_t step, float b1, float b2,
    float eps, int lpr_log2) {
  const int lpr = 1 << lpr_log2;
  const int gl = threadIdx.x & (lpr - 1);
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> lpr_log2;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> lpr_log2; r < n_rows; r += stride) {
    const int32_t l0 = last[r];
    if (l0 + 1 <= step)
      keras_replay_row<VEC>(w, m, v, r, dim, gl, lpr, l0 + 1, step, lr_hist, b1, b2, eps);
    if (gl == 0) last[r] = step;
  }
}

// ---- host launchers -------------------------------------------------------------------
template <template <int, int> class K>
struct Noop {};

#define RS_DISPATCH_VEC_CPL(geom, CALL)                                   \
  do {                                                                    \
    switch ((geom).vec * 100 + (geom).cpl) {                              \
      case 401: { constexpr int VEC = 4, CPL = 1; CALL; } break;          \
      case 402: { constexpr int VEC = 4, CPL = 2; CALL; } break;          \
      case 404: { constexpr int VEC = 4, CPL = 4; CALL; } break;          \
      case 408: { constexpr int VEC = 4, CPL = 8; CALL; } break;          \
      case 201: { constexpr int VEC = 2, CPL = 1; CALL; } break;          \
      case 202: { constexpr int VEC = 2, CPL = 2; CALL; } break;          \
      case 204: { constexpr int VEC = 2, CPL = 4; CALL; } break;          \
      case 101: { constexpr int VEC = 1, CPL = 1; CALL; } break;          \
      case 102: { constexpr int VEC = 1, CPL = 2; CALL; } break;          \
      case 104: { constexpr int VEC = 1, CPL = 4; CALL; } break;          \
      default:                                                            \
        set_error("row geometry vec=%d cpl=%d unsupported (dim too large)", (geom).vec, (geom).cpl); \
        return RS_E_UNSUPPORTED;                                          \
    }                                                                     \
  } while (0)

// Keras Adam's touched-row bitmap: every distinct valid row of the sorted keys (the rows the
// walk finalised), one atomicOr per segment head; OR is order-free, so the bitmap is exact
__global__ __launch_bounds__(256) void keras_bitmap_mark_kernel(const uint32_t* __restrict__ keys,
                                                               int64_t n, uint32_t n_rows,
                                                               uint32_t* __restrict__ bitmap) {
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
    const uint32_t row = keys[k];
    if (row < n_rows && (k == 0 || keys[k - 1] != row)) atomicOr(bitmap + (row >> 5), 1u << (row & 31));
  }
}

// The D = 128 SGD walk queues its table updates 2 runs at a time (tile32_walk<OPT_SGD, 2>; Q = 3
// and 4 spill at 128 VGPRs): round 4's A/B against the one-run-at-a-time walk, 200 steps each,
// interleaved: step 0.685-0.688 -> 0.671-0.674 ms, apply alone 238 -> 230 us, bit-identical.

static int32_t launch_segments(int opt, const uint32_t* keys, const int32_t* pos, int64_t n,
                               int64_t n_rows, const float* grad, const ApplyArgs& a,
                               const RowGeom& geom, hipStream_t st) {
  const int64_t n_tiles = ceil_div(n, RS_DEDUP_TILE);
  const int gpb = 256 >> geom.lpr_log2;
  const int64_t blocks = ceil_div(n_tiles, gpb);
  if (blocks == 0) return RS_OK;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int64_t walk_blocks = std::min<int64_t>(blocks, (int64_t)cus * kApplyBlocksPerCU);
#ifndef RS_NO_T32
  const bool t32 = geom.vec == 4 && geom.cpl == 1 && geom.lpr_log2 == 5 && RS_DEDUP_TILE == 32;
#else
  const bool t32 = false;
#endif
#ifndef RS_NO_G32
  const bool g32 = t32;
#else
  const bool g32 = false;
#endif
  if (a.key_lo && !g32) {
    set_error("a key range needs the D = 128 group walk (16-byte aligned rows)");
    return RS_E_UNSUPPORTED;
  }
#define RS_SEG_LAUNCH(OPTV)                                                                     \
  RS_DISPATCH_VEC_CPL(geom, ({                                                                  \
    if (g32) {                                                                                  \
      if (OPTV == OPT_SGD)                                                                      \
        seg_group32_kernel<OPTV, 2><<<ceil_div(n_tiles, 32), 1024, 0, st>>>(                    \
            keys, pos, n, (uint32_t)n_rows, grad, a, n_tiles);                                  \
      else                                                                                      \
        seg_group32_kernel<OPTV><<<ceil_div(n_tiles, 32), 1024, 0, st>>>(keys, pos, n,          \
                                                                     (uint32_t)n_rows, grad, a, \
                                                                     n_tiles);                  \
    } else {                                                                                    \
      if (t32)                                                                                  \
        seg_tile32_kernel<OPTV><<<ceil_div(n_tiles, 8), 256, 0, st>>>(       \
            keys, pos, n, (uint32_t)n_rows, grad, a, n_tiles);                                  \
      else                                                                                      \
        seg_tile_kernel<OPTV, VEC, CPL><<<walk_blocks, 256, 0, st>>>(                           \
            keys, pos, n, (uint32_t)n_rows, grad, a, geom.lpr_log2, n_tiles);                   \
      seg_chunk_kernel<VEC, CPL><<<blocks, 256, 0, st>>>(keys, n, (uint32_t)n_rows, a,          \
                                                         geom.lpr_log2, n_tiles, a.chunk);      \
    }                                                                                           \
    if (g32)                                                                                    \
      seg_fixup_sweep_kernel<OPTV><<<(unsigned)std::min<int64_t>(ceil_div(n_tiles, 256), 1024),  \
                                     256, 0, st>>>(keys, a, n_tiles, a.chunk);                  \
    else                                                                                        \
      seg_fixup_wave_kernel<OPTV, VEC, CPL><<<(unsigned)ceil_div(n_tiles, 4), 256, 0, st>>>(    \
          keys, a, geom.lpr_log2, n_tiles, a.chunk);                                            \
  }))
  switch (opt) {
    case OPT_SGD: RS_SEG_LAUNCH(OPT_SGD); break;
    case OPT_LAZY: RS_SEG_LAUNCH(OPT_LAZY); break;
    case OPT_KERAS:
      RS_SEG_LAUNCH(OPT_KERAS);
      keras_bitmap_mark_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 2048), 256, 0, st>>>(
          keys, n, (uint32_t)n_rows, a.bitmap);
      break;
    case OPT_EMIT: RS_SEG_LAUNCH(OPT_EMIT); break;
    case OPT_DENSE: RS_SEG_LAUNCH(OPT_DENSE); break;
    default: set_error("unknown optimizer %d", opt); return RS_E_INVALID;
  }
#undef RS_SEG_LAUNCH
  RS_CHECK_LAUNCH();
  return RS_OK;
}

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_embedding_fwd_strided(const float* table, int64_t n_rows, int32_t dim,
                                            const void* ids, int32_t id_dtype, int64_t n_ids,
                                            const int64_t* slot_offsets, int32_t n_slots, float* out,
                                            int64_t out_ld, int32_t* err_flag, void* stream);

extern "C" int32_t rs_embedding_fwd(const float* table, int64_t n_rows, int32_t dim, const void* ids,
                                    int32_t id_dtype, int64_t n_ids, const int64_t* slot_offsets,
                                    int32_t n_slots, float* out, int32_t* err_flag, void* stream) {
  return rs_embedding_fwd_strided(table, n_rows, dim, ids, id_dtype, n_ids, slot_offsets, n_slots,
                                  out, dim, err_flag, stream);
}

// the gathered rows written at a row stride: out[p * out_ld + c] (a column block of a wider
// row-major tensor, e.g. the item ‖ category halves of DIEN's flat embedding, no concat)
extern "C" int32_t rs_embedding_fwd_strided(const float* table, int64_t n_rows, int32_t dim,
                                            const void* ids, int32_t id_dtype, int64_t n_ids,
                                            const int64_t* slot_offsets, int32_t n_slots, float* out,
                                            int64_t out_ld, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(dim > 0, "dim must be > 0");
  RS_CHECK_ARG(out_ld >= dim, "out_ld must be >= dim");
  RS_CHECK_ARG(n_ids >= 0, "n_ids must be >= 0");
  RS_CHECK_ARG(n_slots >= 1, "n_slots must be >= 1");
  RS_CHECK_ARG(id_dtype == RS_ID_I32 || id_dtype == RS_ID_I64, "bad id dtype");
  RS_CHECK_ARG(n_ids == 0 || (table && ids && out), "null pointer");
  if (n_ids == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  if (out_ld == dim && dim % 4 != 0 && dim % 2 == 0 && dim <= 64 &&
      ((reinterpret_cast<uintptr_t>(table) | reinterpret_cast<uintptr_t>(out)) & 7) == 0) {
    const int64_t pairs = n_ids * dim / 2;
    const int blocks = (int)std::min<int64_t>(ceil_div(pairs, 256), 256 * 32);
    gather_flat2_kernel<<<blocks, 256, 0, st>>>(table, n_rows, dim, ids, id_dtype, n_ids,
                                                slot_offsets, n_slots, out, err_flag);
    RS_CHECK_LAUNCH();
    return RS_OK;
  }
  // a row stride that breaks the vector width's alignment downgrades it like a base pointer
  const void* ptrs[3] = {table, out, reinterpret_cast<const void*>((uintptr_t)(out_ld * 4))};
  RowGeom geom = row_geom(dim, ptrs, 3);
  const int gpb = 256 >> geom.lpr_log2;
  int64_t blocks = std::min<int64_t>(ceil_div(n_ids, gpb * 4), 256 * 16);
  RS_DISPATCH_VEC_CPL(geom, ({
    gather_kernel<VEC, CPL><<<blocks, 256, 0, st>>>(table, n_rows, dim, ids, id_dtype, n_ids,
                                                    slot_offsets, n_slots, out, err_flag,
                                                    geom.lpr_log2, out_ld);
  }));
  RS_CHECK_LAUNCH();
  return RS_OK;
}

static size_t partial_bytes(int64_t n_ids, int32_t dim) {
  // tile partials + level-1 chunk sums, each [n_tiles][2][dim], + one flag byte per tile
  return 2 * align_up((size_t)ceil_div(n_ids, RS_DEDUP_TILE) * 2 * dim * sizeof(float), 256) +
         align_up((size_t)ceil_div(n_ids, RS_DEDUP_TILE), 256);
}
static uint8_t* flags_of(float* partial, int64_t n_ids, int32_t dim) {
  return reinterpret_cast<uint8_t*>(partial) +
         2 * align_up((size_t)ceil_div(n_ids, RS_DEDUP_TILE) * 2 * dim * sizeof(float), 256);
}
static float* chunk_of(float* partial, int64_t n_ids, int32_t dim) {
  return partial + align_up((size_t)ceil_div(n_ids, RS_DEDUP_TILE) * 2 * dim * sizeof(float), 256) / 4;
}

extern "C" size_t rs_dedup_workspace_size(int64_t n_ids, int32_t dim) {
  return align_up(partial_bytes(n_ids, dim), 256) + align_up((size_t)n_ids * 4, 256) +
         exclusive_scan_ws_size(n_ids) + 256;
}

extern "C" int32_t rs_embedding_dedup_grad_scaled(const uint32_t* sorted_rows,
                                                  const int32_t* sorted_pos, int64_t n_ids,
                                                  const float* grad_out, const float* row_scale,
                                                  int32_t scale_group, int32_t dim, int64_t n_rows,
                                                  uint32_t* uniq_rows, float* uniq_grad,
                                                  void* workspace, size_t ws_bytes, void* stream);

extern "C" int32_t rs_embedding_dedup_grad(const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                           int64_t n_ids, const float* grad_out, int32_t dim,
                                           int64_t n_rows, uint32_t* uniq_rows, float* uniq_grad,
                                           void* workspace, size_t ws_bytes, void* stream) {
  return rs_embedding_dedup_grad_scaled(sorted_rows, sorted_pos, n_ids, grad_out, nullptr, 1, dim,
                                        n_rows, uniq_rows, uniq_grad, workspace, ws_bytes, stream);
}

extern "C" int32_t rs_embedding_dedup_grad_mapped(const uint32_t* sorted_rows,
                                                  const int32_t* sorted_pos, int64_t n_ids,
                                                  const float* grad_out, const float* row_scale,
                                                  int32_t scale_group, int32_t dim, int64_t n_rows,
                                                  const int32_t* seg_map, uint32_t* uniq_rows,
                                                  float* uniq_grad, void* workspace,
                                                  size_t ws_bytes, void* stream);

extern "C" int32_t rs_embedding_dedup_grad_scaled(const uint32_t* sorted_rows,
                                                  const int32_t* sorted_pos, int64_t n_ids,
                                                  const float* grad_out, const float* row_scale,
                                                  int32_t scale_group, int32_t dim, int64_t n_rows,
                                                  uint32_t* uniq_rows, float* uniq_grad,
                                                  void* workspace, size_t ws_bytes, void* stream) {
  return rs_embedding_dedup_grad_mapped(sorted_rows, sorted_pos, n_ids, grad_out, row_scale,
                                        scale_group, dim, n_rows, nullptr, uniq_rows, uniq_grad,
                                        workspace, ws_bytes, stream);
}

extern "C" int32_t rs_embedding_dedup_grad_mapped_range(
    const uint32_t* sorted_rows, const int32_t* sorted_pos, int64_t n_ids, const float* grad_out,
    const float* row_scale, int32_t scale_group, int32_t dim, int64_t n_rows, uint32_t key_lo,
    uint32_t key_hi, int32_t seg_ready, const int32_t* seg_excl, const int32_t* seg_map,
    uint32_t* uniq_rows,
    float* uniq_grad, void* workspace, size_t ws_bytes, void* stream);

extern "C" int32_t rs_embedding_dedup_grad_mapped(const uint32_t* sorted_rows,
                                                  const int32_t* sorted_pos, int64_t n_ids,
                                                  const float* grad_out, const float* row_scale,
                                                  int32_t scale_group, int32_t dim, int64_t n_rows,
                                                  const int32_t* seg_map, uint32_t* uniq_rows,
                                                  float* uniq_grad, void* workspace,
                                                  size_t ws_bytes, void* stream) {
  return rs_embedding_dedup_grad_mapped_range(sorted_rows, sorted_pos, n_ids, grad_out, row_scale,
                                              scale_group, dim, n_rows, 0u, (uint32_t)n_rows, 0,
                                              nullptr, seg_map, uniq_rows, uniq_grad, workspace,
                                              ws_bytes, stream);
}

extern "C" int32_t rs_embedding_dedup_grad_mapped_range(
    const uint32_t* sorted_rows, const int32_t* sorted_pos, int64_t n_ids, const float* grad_out,
    const float* row_scale, int32_t scale_group, int32_t dim, int64_t n_rows, uint32_t key_lo,
    uint32_t key_hi, int32_t seg_ready, const int32_t* seg_excl, const int32_t* seg_map,
    uint32_t* uniq_rows,
    float* uniq_grad, void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(dim > 0 && n_ids >= 0 && n_rows > 0, "bad sizes");
  RS_CHECK_ARG(key_lo < key_hi && (int64_t)key_hi <= n_rows, "key range outside [0, n_rows)");
  RS_CHECK_ARG(!row_scale || scale_group >= 1, "scale_group must be >= 1");
  if (n_ids == 0) return RS_OK;
  RS_CHECK_ARG(sorted_rows && sorted_pos && grad_out && uniq_rows && uniq_grad, "null pointer");
  if (ws_bytes < rs_dedup_workspace_size(n_ids, dim)) {
    set_error("dedup workspace too small");
    return RS_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  Carver c(workspace, ws_bytes);
  float* partial = c.take<float>(partial_bytes(n_ids, dim) / 4);
  int32_t* seg = c.take<int32_t>(n_ids);
  void* scan_ws = c.take<char>(exclusive_scan_ws_size(n_ids));
  int blocks = (int)std::min<int64_t>(ceil_div(n_ids, 256), 4096);
  if (seg_excl) {
    seg = const_cast<int32_t*>(seg_excl);  // given (rs_unique_inverse's, same sorted keys)
  } else if (!seg_ready) {  // segment ids over the whole key space (a second range call reuses them)
    head_flags_kernel<<<blocks, 256, 0, st>>>(sorted_rows, n_ids, (uint32_t)n_rows, seg);
    RS_CHECK_LAUNCH();
    int32_t s = exclusive_scan_i32(seg, seg, n_ids, nullptr, scan_ws, exclusive_scan_ws_size(n_ids), st);
    if (s) return s;
  }
  ApplyArgs a{};
  a.dim = dim;
  a.partial = partial;
  a.chunk = chunk_of(partial, n_ids, dim);
  a.tile_flags = flags_of(partial, n_ids, dim);
  a.uniq_grad = uniq_grad;
  a.uniq_rows = uniq_rows;
  a.seg_excl = seg;
  a.row_scale = row_scale;
  a.scale_group = scale_group;
  a.seg_map = seg_map;
  a.key_lo = key_lo;
  a.ranged = key_lo != 0 || (int64_t)key_hi < n_rows;
  const void* ptrs[2] = {grad_out, uniq_grad};
  RowGeom geom = row_geom(dim, ptrs, 2);
  return launch_segments(OPT_EMIT, sorted_rows, sorted_pos, n_ids, key_hi, grad_out, a, geom, st);
}

extern "C" int32_t rs_embedding_grad_dense(const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                           int64_t n_ids, const float* grad_out, int32_t dim,
                                           int64_t n_rows, float* dense, void* workspace,
                                           size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(dim > 0 && n_ids >= 0 && n_rows > 0, "bad sizes");
  RS_CHECK_ARG(dense, "null pointer");
  hipStream_t st = as_stream(stream);
  RS_CHECK_HIP(hipMemsetAsync(dense, 0, (size_t)n_rows * dim * sizeof(float), st));
  if (n_ids == 0) return RS_OK;
  RS_CHECK_ARG(sorted_rows && sorted_pos && grad_out, "null pointer");
  if (ws_bytes < partial_bytes(n_ids, dim)) {
    set_error("dense-gradient workspace too small");
    return RS_E_WORKSPACE;
  }
  ApplyArgs a{};
  a.table = dense;
  a.dim = dim;
  a.partial = static_cast<float*>(workspace);
  a.chunk = chunk_of(a.partial, n_ids, dim);
  a.tile_flags = flags_of(a.partial, n_ids, dim);
  const void* ptrs[2] = {grad_out, dense};
  RowGeom geom = row_geom(dim, ptrs, 2);
  return launch_segments(OPT_DENSE, sorted_rows, sorted_pos, n_ids, n_rows, grad_out, a, geom, st);
}

extern "C" int32_t rs_embedding_grad_dense_segs(const uint32_t* sorted_rows,
                                                const int32_t* sorted_pos, int64_t n_ids,
                                                int32_t n_segs, const float* const* seg_ptrs,
                                                const int64_t* seg_n, const int64_t* seg_ld,
                                                int32_t dim, int64_t n_rows, float* dense,
                                                void* workspace, size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(dim > 0 && n_ids >= 0 && n_rows > 0, "bad sizes");
  RS_CHECK_ARG(n_segs >= 1 && n_segs <= 4, "1..4 gradient segments");
  RS_CHECK_ARG(dense && seg_ptrs && seg_n && seg_ld, "null pointer");
  ApplyArgs a{};
  int64_t total = 0;
  // the vector width must suit every segment's base and row stride: a stride is checked as a
  // byte offset (ld * 4 aligned to VEC * 4 <=> ld % VEC == 0)
  const void* ptrs[9];
  int np = 0;
  for (int i = 0; i < n_segs; ++i) {
    RS_CHECK_ARG(seg_n[i] >= 0 && seg_ld[i] >= dim, "segment rows >= 0, row stride >= dim");
    RS_CHECK_ARG(seg_n[i] == 0 || seg_ptrs[i], "null segment pointer");
    a.gseg[i] = seg_ptrs[i];
    a.gstart[i] = total;
    a.gld[i] = seg_ld[i];
    total += seg_n[i];
    ptrs[np++] = seg_ptrs[i];
    ptrs[np++] = reinterpret_cast<const void*>((uintptr_t)seg_ld[i] * 4);
  }
  RS_CHECK_ARG(total == n_ids, "segment rows must sum to n_ids");
  a.n_gseg = n_segs;
  hipStream_t st = as_stream(stream);
  RS_CHECK_HIP(hipMemsetAsync(dense, 0, (size_t)n_rows * dim * sizeof(float), st));
  if (n_ids == 0) return RS_OK;
  RS_CHECK_ARG(sorted_rows && sorted_pos, "null pointer");
  if (ws_bytes < partial_bytes(n_ids, dim)) {
    set_error("dense-gradient workspace too small");
    return RS_E_WORKSPACE;
  }
  a.table = dense;
  a.dim = dim;
  a.partial = static_cast<float*>(workspace);
  a.chunk = chunk_of(a.partial, n_ids, dim);
  a.tile_flags = flags_of(a.partial, n_ids, dim);
  ptrs[np++] = dense;
  RowGeom geom = row_geom(dim, ptrs, np);
  // the 128-wide group / tile32 walks address rows as grad + p * dim: keep them off this path
  if (geom.vec == 4 && geom.cpl == 1 && geom.lpr_log2 == 5) geom.vec = 2, geom.lpr_log2 = 6;
  return launch_segments(OPT_DENSE, sorted_rows, sorted_pos, n_ids, n_rows, a.gseg[0], a, geom, st);
}

extern "C" size_t rs_apply_workspace_size(int64_t n_ids, int32_t dim) {
  return align_up(partial_bytes(n_ids, dim), 256) + 256;
}

extern "C" int32_t rs_embedding_apply_scaled(int32_t opt, float* table, float* m, float* v,
                                             int64_t n_rows, int32_t dim,
                                             const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                             int64_t n_ids, const float* grad_out,
                                             const float* row_scale, int32_t scale_group,
                                             const rs_adam_params* params,
                                             uint32_t* touched_bitmap, void* workspace,
                                             size_t ws_bytes, void* stream);

extern "C" int32_t rs_embedding_apply(int32_t opt, float* table, float* m, float* v, int64_t n_rows,
                                      int32_t dim, const uint32_t* sorted_rows,
                                      const int32_t* sorted_pos, int64_t n_ids,
                                      const float* grad_out, const rs_adam_params* params,
                                      uint32_t* touched_bitmap, void* workspace, size_t ws_bytes,
                                      void* stream) {
  return rs_embedding_apply_scaled(opt, table, m, v, n_rows, dim, sorted_rows, sorted_pos, n_ids,
                                   grad_out, nullptr, 1, params, touched_bitmap, workspace,
                                   ws_bytes, stream);
}

extern "C" int32_t rs_embedding_apply_scaled(int32_t opt, float* table, float* m, float* v,
                                             int64_t n_rows, int32_t dim,
                                             const uint32_t* sorted_rows, const int32_t* sorted_pos,
                                             int64_t n_ids, const float* grad_out,
                                             const float* row_scale, int32_t scale_group,
                                             const rs_adam_params* params,
                                             uint32_t* touched_bitmap, void* workspace,
                                             size_t ws_bytes, void* stream) {
  RS_CHECK_ARG(dim > 0 && n_ids >= 0 && n_rows > 0, "bad sizes");
  RS_CHECK_ARG(!row_scale || scale_group >= 1, "scale_group must be >= 1");
  RS_CHECK_ARG(params, "params is null");
  RS_CHECK_ARG(opt == RS_OPT_SGD || opt == RS_OPT_LAZY_ADAM || opt == RS_OPT_KERAS_ADAM,
               "unknown optimizer %d", opt);
  RS_CHECK_ARG(opt == RS_OPT_SGD || (m && v), "Adam needs m and v slots");
  RS_CHECK_ARG(opt != RS_OPT_KERAS_ADAM || touched_bitmap, "Keras Adam needs the touched bitmap");
  if (n_ids == 0) return RS_OK;
  RS_CHECK_ARG(table && sorted_rows && sorted_pos && grad_out, "null pointer");
  if (ws_bytes < rs_apply_workspace_size(n_ids, dim)) {
    set_error("apply workspace too small: need %zu", rs_apply_workspace_size(n_ids, dim));
    return RS_E_WORKSPACE;
  }
  ApplyArgs a{};
  a.table = table;
  a.m = m;
  a.v = v;
  a.dim = dim;
  a.p = *params;
  a.bitmap = touched_bitmap;
  a.row_scale = row_scale;
  a.scale_group = scale_group;
  a.partial = static_cast<float*>(workspace);
  a.chunk = chunk_of(a.partial, n_ids, dim);
  a.tile_flags = flags_of(a.partial, n_ids, dim);
  const void* ptrs[4] = {table, grad_out, m ? m : table, v ? v : table};
  RowGeom geom = row_geom(dim, ptrs, 4);
  return launch_segments(opt, sorted_rows, sorted_pos, n_ids, n_rows, grad_out, a, geom,
                         as_stream(stream));
}

static void replay_geom(int dim, const void* const* ptrs, int np, int* vec, int* lpr_log2) {
  RowGeom g = row_geom(dim, ptrs, np);
  *vec = g.vec;
  int lanes = dim / g.vec, l2 = 0;
  while ((1 << l2) < lanes && l2 < 6) ++l2;
  *lpr_log2 = l2;
}

extern "C" int32_t rs_keras_adam_catchup(float* table, float* m, float* v, int32_t* last,
                                         int64_t n_rows, int32_t dim, const int32_t* sorted_rows,
                                         int64_t n, const float* lr_hist, int32_t step,
                                         const rs_adam_params* params, void* stream) {
  RS_CHECK_ARG(table && m && v && last && lr_hist && params && (n == 0 || sorted_rows),
               "null pointer");
  RS_CHECK_ARG(dim > 0 && n_rows > 0 && n_rows <= 0xFFFFFFFFll && n >= 0 && step >= 1,
               "bad sizes");
  if (n == 0) return RS_OK;
  const void* ptrs[3] = {table, m, v};
  int vec, l2;
  replay_geom(dim, ptrs, 3, &vec, &l2);
  const int64_t groups = n, per_block = 256 >> l2;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(groups, per_block), 4096);
  hipStream_t st = as_stream(stream);
  const uint32_t* rows = reinterpret_cast<const uint32_t*>(sorted_rows);
  const rs_adam_params p = *params;
  switch (vec) {
    case 4: keras_catchup_kernel<4><<<blocks, 256, 0, st>>>(table, m, v, last, (uint32_t)n_rows, dim, rows, n, lr_hist, step, p.beta1, p.beta2, p.epsilon, l2); break;
    case 2: keras_catchup_kernel<2><<<blocks, 256, 0, st>>>(table, m, v, last, (uint32_t)n_rows, dim, rows, n, lr_hist, step, p.beta1, p.beta2, p.epsilon, l2); break;
    default: keras_catchup_kernel<1><<<blocks, 256, 0, st>>>(table, m, v, last, (uint32_t)n_rows, dim, rows, n, lr_hist, step, p.beta1, p.beta2, p.epsilon, l2); break;
  }
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_keras_adam_mark(int32_t* last, int64_t n_rows, const uint32_t* sorted_rows,
                                      int64_t n, int32_t step, void* stream) {
  RS_CHECK_ARG(last && (n == 0 || sorted_rows) && n >= 0 && n_rows > 0, "bad arguments");
  if (n == 0) return RS_OK;
  const int blocks = (int)std::min<int64_t>(ceil_div(n, 256), 2048);
  keras_mark_kernel<<<blocks, 256, 0, as_stream(stream)>>>(last, (uint32_t)n_rows, sorted_rows, n, step);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_keras_adam_materialize(float* table, float* m, float* v, int32_t* last,
                                             int64_t n_rows, int32_t dim, const float* lr_hist,
                                             int32_t step, const rs_adam_params* params,
                                             void* stream) {
  RS_CHECK_ARG(table && m && v && last && lr_hist && params, "null pointer");
  RS_CHECK_ARG(dim > 0 && n_rows > 0 && step >= 0, "bad sizes");
  if (step == 0) return RS_OK;
  const void* ptrs[3] = {table, m, v};
  int vec, l2;
  replay_geom(dim, ptrs, 3, &vec, &l2);
  const int64_t per_block = 256 >> l2;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n_rows, per_block), 256 * 64);
  hipStream_t st = as_stream(stream);
  const rs_adam_params p = *params;
  switch (vec) {
    case 4: keras_materialize_kernel<4><<<blocks, 256, 0, st>>>(table, m, v, last, n_rows, dim, lr_hist, step, p.beta1, p.beta2, p.epsilon, l2); break;
    case 2: keras_materialize_kernel<2><<<blocks, 256, 0, st>>>(table, m, v, last, n_rows, dim, lr_hist, step, p.beta1, p.beta2, p.epsilon, l2); break;
    default: keras_materialize_kernel<1><<<blocks, 256, 0, st>>>(table, m, v, last, n_rows, dim, lr_hist, step, p.beta1, p.beta2, p.epsilon, l2); break;
  }
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_keras_adam_dense_sweep(float* table, float* m, float* v, int64_t n_rows,
                                             int32_t dim, const rs_adam_params* params,
                                             uint32_t* touched_bitmap, void* stream) {
  RS_CHECK_ARG(table && m && v && params && touched_bitmap, "null pointer");
  RS_CHECK_ARG(dim > 0 && n_rows > 0, "bad sizes");
  hipStream_t st = as_stream(stream);
  const void* ptrs[3] = {table, m, v};
  RowGeom geom = row_geom(dim, ptrs, 3);
  int64_t total = n_rows * (dim / geom.vec);
  int64_t blocks = std::min<int64_t>(ceil_div(total, 256), 256 * 32);
  switch (geom.vec) {
    case 4: keras_dense_sweep_kernel<4><<<blocks, 256, 0, st>>>(table, m, v, n_rows, dim, *params, touched_bitmap); break;
    case 2: keras_dense_sweep_kernel<2><<<blocks, 256, 0, st>>>(table, m, v, n_rows, dim, *params, touched_bitmap); break;
    default: keras_dense_sweep_kernel<1><<<blocks, 256, 0, st>>>(table, m, v, n_rows, dim, *params, touched_bitmap); break;
  }
  RS_CHECK_LAUNCH();
  RS_CHECK_HIP(hipMemsetAsync(touched_bitmap, 0, (size_t)ceil_div(n_rows, 32) * 4, st));
  return RS_OK;
}

// ---- small-table dense gradient (no sort) ---------------------------------------------------
// grad_dense[v, :] = Σ_{n: ids[n] = v} grad_rows[n, :] for a table of V·dim ≤ kSmallVD floats
// (PinSage's year / genre tables: Keras' IndexedSlices gradient densified, pinsage/train/
// train.py:45-46). Block b sums entries [b·chunk, (b+1)·chunk): thread (e, d) of E entry lanes
// × dim columns adds column d of entries e, e+E, … into its own LDS copy of the table, the E
// copies are folded in lane order and the block partials in block order — a fixed summation
// order, independent of timing. One pass over the entries, no radix sort, no hot-row fix-up
// (the genre table's 2 live rows take every entry).
namespace rs {
constexpr int64_t kSmallVD = 16384;  // 64 KiB of LDS at E = 1

template <typename Id>
__global__ __launch_bounds__(256) void dense_small_partial_kernel(
    const Id* __restrict__ ids, int64_t n, const float* __restrict__ rows, int32_t dim,
    int32_t dshift, int32_t E, int64_t V, int64_t chunk, float* __restrict__ partial,
    int32_t* __restrict__ err_flag) {
  extern __shared__ float acc[];  // [E][V * dim]
  const int32_t t = threadIdx.x, d = t & (dim - 1), e = t >> dshift;
  const int64_t VD = V * dim;
  for (int64_t i = t; i < (int64_t)E * VD; i += blockDim.x) acc[i] = 0.f;
  __syncthreads();
  float* mine = acc + (int64_t)e * VD;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  // 4 entries' ids and gradient values loaded before their 4 read-modify-writes (same order)
  int64_t k = lo + e;
  for (; k + 3 * E < hi; k += 4 * E) {
    int64_t r[4];
    float x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = (int64_t)ids[k + u * E];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = rows[(k + u * E) * dim + d];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (r[u] < 0 || r[u] >= V) {
        if (d == 0) flag_oob(err_flag);
        continue;
      }
      mine[r[u] * dim + d] += x[u];
    }
  }
  for (; k < hi; k += E) {
    const int64_t r = (int64_t)ids[k];
    if (r < 0 || r >= V) {
      if (d == 0) flag_oob(err_flag);
      continue;
    }
    mine[r * dim + d] += rows[k * dim + d];
  }
  __syncthreads();
  for (int64_t i = t; i < VD; i += blockDim.x) {
    float s = 0.f;
    for (int32_t q = 0; q < E; ++q) s += acc[(int64_t)q * VD + i];
    partial[(int64_t)blockIdx.x * VD + i] = s;
  }
}

// 64 outputs per block x 4 lanes: lane q sums blocks q, q+4, … (8 loads in flight), then the
// 4 lane sums are added in lane order.
__global__ __launch_bounds__(256) void dense_small_fold_kernel(const float* __restrict__ partial,
                                                               int32_t nb, int64_t VD,
                                                               float* __restrict__ out) {
  __shared__ float lane_sum[4][64];
  const int32_t c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + c;
  float s = 0.f;
  if (i < VD) {
    int32_t b = q;
    for (; b + 28 < nb; b += 32) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = partial[(int64_t)(b + 4 * u) * VD + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += x[u];
    }
    for (; b < nb; b += 4) s += partial[(int64_t)b * VD + i];
  }
  lane_sum[q][c] = s;
  __syncthreads();
  if (q == 0 && i < VD) out[i] = ((lane_sum[0][c] + lane_sum[1][c]) + lane_sum[2][c]) + lane_sum[3][c];
}

struct SmallGeom {
  int32_t E, nb;
  int64_t chunk;
};

inline SmallGeom small_geom(int64_t n_ids, int64_t n_rows, int32_t dim) {
  const int64_t VD = n_rows * dim;
  int32_t E = 256 / dim;
  while (E > 1 && (int64_t)E * VD > kSmallVD) E >>= 1;
  SmallGeom g;
  g.E = E;
  g.nb = (int32_t)std::min<int64_t>(1024, std::max<int64_t>(1, ceil_div(n_ids, 512)));
  g.chunk = ceil_div(n_ids < 1 ? 1 : n_ids, g.nb);
  return g;
}
}  // namespace rs

extern "C" size_t rs_embedding_grad_dense_small_workspace_size(int64_t n_ids, int64_t n_rows,
                                                                int32_t dim) {
  using namespace rs;
  if (dim <= 0 || n_rows <= 0) return 256;
  return align_up((size_t)small_geom(n_ids, n_rows, dim).nb * n_rows * dim * 4, 256);
}

extern "C" int32_t rs_embedding_grad_dense_small(const void* ids, int32_t id_dtype, int64_t n_ids,
                                                 const float* grad_rows, int32_t dim,
                                                 int64_t n_rows, float* grad_dense,
                                                 int32_t* err_flag, void* workspace,
                                                 size_t ws_bytes, void* stream) {
  using namespace rs;
  RS_CHECK_ARG(dim > 0 && dim <= 256 && (dim & (dim - 1)) == 0,
               "rs_embedding_grad_dense_small: dim must be a power of two <= 256");
  RS_CHECK_ARG(n_rows > 0 && n_rows * dim <= kSmallVD,
               "rs_embedding_grad_dense_small: n_rows * dim must be <= 16384");
  RS_CHECK_ARG(n_ids >= 0 && id_dtype >= RS_ID_I32 && id_dtype <= RS_ID_I64, "bad ids");
  RS_CHECK_ARG(grad_dense && (n_ids == 0 || (ids && grad_rows)), "null pointer");
  RS_CHECK_ARG(ws_bytes >= rs_embedding_grad_dense_small_workspace_size(n_ids, n_rows, dim),
               "rs_embedding_grad_dense_small: workspace too small");
  hipStream_t st = as_stream(stream);
  const int64_t VD = n_rows * dim;
  if (n_ids == 0) {
    RS_CHECK_HIP(hipMemsetAsync(grad_dense, 0, (size_t)VD * 4, st));
    return RS_OK;
  }
  const SmallGeom g = small_geom(n_ids, n_rows, dim);
  int32_t dshift = 0;
  while ((1 << dshift) < dim) ++dshift;
  float* partial = static_cast<float*>(workspace);
  const size_t lds = (size_t)g.E * VD * 4;
  const int threads = g.E * dim;
  if (id_dtype == RS_ID_I32)
    dense_small_partial_kernel<int32_t><<<g.nb, threads, lds, st>>>(
        static_cast<const int32_t*>(ids), n_ids, grad_rows, dim, dshift, g.E, n_rows, g.chunk,
        partial, err_flag);
  else
    dense_small_partial_kernel<int64_t><<<g.nb, threads, lds, st>>>(
        static_cast<const int64_t*>(ids), n_ids, grad_rows, dim, dshift, g.E, n_rows, g.chunk,
        partial, err_flag);
  RS_CHECK_LAUNCH();
  dense_small_fold_kernel<<<(unsigned)ceil_div(VD, 64), 256, 0, st>>>(partial, g.nb, VD,
                                                                      grad_dense);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

// ---- Keras Adam over one flat buffer, lr_t from device memory ---------------------------------
// The dense update of KerasAdam (m = m·b1 + g·(1-b1); v = v·b2 + g²·(1-b2);
// var -= m·lr_t / (√v + eps), each product / sum rounded as the separate torch ops round) for
// every parameter of a model at once (parameters as views of one buffer), with lr_t =
// lr_hist[*step_idx]: a HIP graph holding this launch replays the right step each time.
namespace rs {
__global__ __launch_bounds__(256) void keras_adam_flat_kernel(
    float4* __restrict__ var, float4* __restrict__ m, float4* __restrict__ v,
    const float4* __restrict__ g, int64_t n4, const float* __restrict__ lr_hist,
    const int64_t* __restrict__ step_idx, rs_adam_params p) {
  const float lr = lr_hist[*step_idx];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 gi = g[i];
    float4 mi = m[i], vi = v[i], wi = var[i];
    float* mf = reinterpret_cast<float*>(&mi);
    float* vf = reinterpret_cast<float*>(&vi);
    float* wf = reinterpret_cast<float*>(&wi);
    const float* gf = reinterpret_cast<const float*>(&gi);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      mf[c] = mf[c] * p.beta1 + gf[c] * p.one_minus_beta1;
      vf[c] = vf[c] * p.beta2 + (gf[c] * gf[c]) * p.one_minus_beta2;
      wf[c] = wf[c] - (mf[c] * lr) / (sqrtf(vf[c]) + p.epsilon);
    }
    m[i] = mi;
    v[i] = vi;
    var[i] = wi;
  }
}
}  // namespace rs

extern "C" int32_t rs_keras_adam_flat(float* var, float* m, float* v, const float* grad, int64_t n,
                                      const float* lr_hist, const int64_t* step_idx,
                                      const rs_adam_params* params, void* stream) {
  using namespace rs;
  RS_CHECK_ARG(var && m && v && grad && lr_hist && step_idx && params, "null pointer");
  RS_CHECK_ARG(n > 0 && n % 4 == 0, "rs_keras_adam_flat: n must be a positive multiple of 4");
  RS_CHECK_ARG(((uintptr_t)var | (uintptr_t)m | (uintptr_t)v | (uintptr_t)grad) % 16 == 0,
               "rs_keras_adam_flat: buffers must be 16-byte aligned");
  const int64_t n4 = n / 4;
  const int64_t blocks = std::min<int64_t>(ceil_div(n4, 256), 2048);
  keras_adam_flat_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(
      reinterpret_cast<float4*>(var), reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v),
      reinterpret_cast<const float4*>(grad), n4, lr_hist, step_idx, *params);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
