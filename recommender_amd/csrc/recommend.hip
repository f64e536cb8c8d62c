// recommend.hip — PinSage evaluation on device (pinsage/train/evaluation.py).
//
//   rs_latest_item   recommend :33-34   dgl.sampling.select_topk(u2i slice, 1, timestamp): the
//                    item of each user's latest interaction (ties → smaller item id).
//   rs_masked_topk   recommend :39-46   similarity rows (latest item repr · all item reprs,
//                    computed by the caller's GEMM), the user's interacted items set to -inf,
//                    top-k. One 256-thread block per row: the exclusion set becomes an LDS
//                    bitmap; a threshold pass (k-th best of the threads' maxima) bounds the
//                    candidates, which a second pass collects in LDS (see masked_topk_kernel).
//                    Order (score desc, item asc); rows come out best first (the reference's
//                    argpartition leaves them unordered — same set).
//   rs_hit_flags     hit_rate_eval :54-65  relevance.any(axis=1) per user against a CSR of
//                    ground-truth items.
#include <climits>

#include "common.hpp"

namespace rs {

constexpr int kTopkThreads = 256;

__global__ __launch_bounds__(256) void latest_item_kernel(const int64_t* __restrict__ indptr,
                                                          const int32_t* __restrict__ items,
                                                          const int64_t* __restrict__ ts,
                                                          int64_t n_users,
                                                          int32_t* __restrict__ out,
                                                          int32_t* __restrict__ n_missing) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n_users) return;
  int32_t best = -1;
  int64_t bt = LLONG_MIN;
  for (int64_t e = indptr[u]; e < indptr[u + 1]; ++e) {
    const int64_t t = ts[e];
    const int32_t it = items[e];
    if (best < 0 || t > bt || (t == bt && it < best)) {
      best = it;
      bt = t;
    }
  }
  out[u] = best;
  if (best < 0 && n_missing) atomicAdd(n_missing, 1);
}

__device__ __forceinline__ bool better(float a, int32_t ia, float b, int32_t ib) {
  return a > b || (a == b && ia < ib);
}

// the new entry (better than the current last) replaces the last and bubbles up: one
// compare-exchange per position keeps the list sorted
template <int KM>
__device__ __forceinline__ void list_insert(float (&v)[KM], int32_t (&ix)[KM], float s, int32_t i) {
  v[KM - 1] = s;
  ix[KM - 1] = i;
#pragma unroll
  for (int p = KM - 1; p > 0; --p) {
    const bool sw = better(v[p], ix[p], v[p - 1], ix[p - 1]);
    const float tv = v[p];
    const int32_t ti = ix[p];
    v[p] = sw ? v[p - 1] : tv;
    ix[p] = sw ? ix[p - 1] : ti;
    v[p - 1] = sw ? tv : v[p - 1];
    ix[p - 1] = sw ? ti : ix[p - 1];
  }
}

template <int KM>
__device__ __forceinline__ void list_pop(float (&v)[KM], int32_t (&ix)[KM]) {
#pragma unroll
  for (int p = 0; p < KM - 1; ++p) {
    v[p] = v[p + 1];
    ix[p] = ix[p + 1];
  }
  v[KM - 1] = -INFINITY;
  ix[KM - 1] = INT_MAX;
}

constexpr int kTopkCand = 2048;  // LDS candidate slots
constexpr int kTopkWaves = kTopkThreads / kWave;

// K rounds of wave argmax over one (value, index) per lane; lane 0 stores the wave's sorted top
// K at out_v/out_i[0..K). The winner's lane advances via `next` (pops its list head).
template <typename Next>
__device__ __forceinline__ void wave_topk(float& hv, int32_t& hi, int32_t K, int lane,
                                          float* out_v, int32_t* out_i, Next next) {
  for (int32_t k = 0; k < K; ++k) {
    float bv = hv;
    int32_t bi = hi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, kWave);
      const int32_t oi = __shfl_xor(bi, o, kWave);
      if (better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (hi == bi) next();  // indices are unique across lanes
    if (lane == 0) {
      out_v[k] = bv;
      out_i[k] = bi;
    }
  }
}

// bitonic sort of one (value, index) per lane across the wave, best first (21 exchange steps)
__device__ __forceinline__ void wave_sort(float& v, int32_t& ix, int lane) {
#pragma unroll
  for (int k = 2; k <= kWave; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const float ov = __shfl_xor(v, j, kWave);
      const int32_t oi = __shfl_xor(ix, j, kWave);
      const bool keep_better = ((lane & k) == 0) == ((lane & j) == 0);
      const bool ob = better(ov, oi, v, ix);
      if (keep_better ? ob : (!ob && (ov != v || oi != ix))) {
        v = ov;
        ix = oi;
      }
    }
  }
}

// merge of the kTopkWaves sorted lists of K (list w at v/i + w*K): the k-th best, k < K
__device__ __forceinline__ void merge_waves(const float* v, const int32_t* ix, int32_t K,
                                            int32_t upto, float* out_v, int32_t* out_i,
                                            float& last_v, int32_t& last_i) {
  int32_t head[kTopkWaves] = {};
  for (int32_t k = 0; k < upto; ++k) {
    int w_best = -1;
    float bv = -INFINITY;
    int32_t bi = INT_MAX;
#pragma unroll
    for (int w = 0; w < kTopkWaves; ++w) {
      if (head[w] >= K) continue;
      const float cv = v[w * K + head[w]];
      const int32_t ci = ix[w * K + head[w]];
      if (w_best < 0 || better(cv, ci, bv, bi)) {
        bv = cv;
        bi = ci;
        w_best = w;
      }
    }
#pragma unroll
    for (int w = 0; w < kTopkWaves; ++w) head[w] += w == w_best;  // static indices: no scratch
    if (out_v) out_v[k] = bv;
    if (out_i) out_i[k] = bi;
    last_v = bv;
    last_i = bi;
  }
}

// Three passes over the row, all coalesced:
//  1. each thread's best item; θ = the K-th best of those 256 (by the total order (score desc,
//     item asc)). At least K items rank ≤ θ, so the top K all rank ≤ θ; at most K threads own
//     such items, so there are ≤ K·⌈I/256⌉ candidates.
//  2. the items ranking ≤ θ go to an LDS candidate list (re-read of the row: L2 / MALL hits).
//  3. the top K of the candidates: ≤ 64 (the usual case) → one wave bitonic sort; else
//     per-thread register lists, wave argmax, 4-way merge. If the candidates overflow
//     kTopkCand (only when K·⌈I/256⌉ > 2048) the lists are built from the whole row instead.
// θ itself comes from a bitonic sort of each wave's 64 thread maxima and one more sort of the
// waves' top K lists (K ≤ 16; else a serial 4-way merge).
template <int KM>
__global__ __launch_bounds__(kTopkThreads) void masked_topk_kernel(
    const float* __restrict__ scores, int64_t ld, int32_t I, int64_t user_base,
    const int64_t* __restrict__ excl_indptr, const int32_t* __restrict__ excl_idx, int32_t K,
    int32_t* __restrict__ out_idx, float* __restrict__ out_val) {
  extern __shared__ uint32_t lds[];
  __shared__ float wv[kTopkWaves * 64];
  __shared__ int32_t wi[kTopkWaves * 64];
  __shared__ int32_t n_cand;
  __shared__ float th_v;
  __shared__ int32_t th_i;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t r = blockIdx.x;
  const bool excl = excl_indptr != nullptr;
  const int32_t bitmap_words = excl ? (I + 31) >> 5 : 0;
  uint32_t* bitmap = lds;
  float* cv = reinterpret_cast<float*>(lds + bitmap_words);
  int32_t* ci = reinterpret_cast<int32_t*>(cv + kTopkCand);
  if (tid == 0) n_cand = 0;
  if (excl) {
    for (int32_t w = tid; w < bitmap_words; w += kTopkThreads) bitmap[w] = 0u;
    __syncthreads();
    const int64_t u = user_base + r;
    for (int64_t e = excl_indptr[u] + tid; e < excl_indptr[u + 1]; e += kTopkThreads) {
      const int32_t it = excl_idx[e];
      if (it >= 0 && it < I) atomicOr(&bitmap[it >> 5], 1u << (it & 31));
    }
  }
  __syncthreads();
  const float* row = scores + r * ld;
  auto score = [&](int32_t i, float x) {
    return (excl && ((bitmap[i >> 5] >> (i & 31)) & 1u)) ? -INFINITY : x;
  };
  constexpr int U = 8;  // loads in flight per thread

  // pass 1
  float mv = -INFINITY;
  int32_t mi = INT_MAX;
  for (int32_t base = 0; base < I; base += kTopkThreads * U) {
    float s[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int32_t i = base + tid + kTopkThreads * j;
      s[j] = i < I ? row[i] : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int32_t i = base + tid + kTopkThreads * j;
      if (i < I) {
        const float x = score(i, s[j]);
        if (better(x, i, mv, mi)) {
          mv = x;
          mi = i;
        }
      }
    }
  }
  // θ: every wave sorts its 64 maxima; the K-th best of the waves' top K lists
  wave_sort(mv, mi, lane);
  if (lane < K) {
    wv[wid * K + lane] = mv;
    wi[wid * K + lane] = mi;
  }
  __syncthreads();
  if (K * kTopkWaves <= kWave) {
    if (wid == 0) {
      float x = lane < K * kTopkWaves ? wv[lane] : -INFINITY;
      int32_t xi = lane < K * kTopkWaves ? wi[lane] : INT_MAX;
      wave_sort(x, xi, lane);
      if (lane == K - 1) {
        th_v = x;
        th_i = xi;
      }
    }
  } else if (tid == 0) {
    float lv;
    int32_t li;
    merge_waves(wv, wi, K, K, nullptr, nullptr, lv, li);
    th_v = lv;
    th_i = li;
  }
  __syncthreads();
  const float tv = th_v;
  const int32_t ti = th_i;

  // pass 2
  for (int32_t base = 0; base < I; base += kTopkThreads * U) {
    float s[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int32_t i = base + tid + kTopkThreads * j;
      s[j] = i < I ? row[i] : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int32_t i = base + tid + kTopkThreads * j;
      if (i < I) {
        const float x = score(i, s[j]);
        if (!better(tv, ti, x, i)) {
          const int32_t slot = atomicAdd(&n_cand, 1);
          if (slot < kTopkCand) {
            cv[slot] = x;
            ci[slot] = i;
          }
        }
      }
    }
  }
  __syncthreads();
  const int32_t nc = n_cand;
  if (nc <= kWave) {  // the usual case: one wave sorts the candidates
    if (wid == 0) {
      float x = lane < nc ? cv[lane] : -INFINITY;
      int32_t xi = lane < nc ? ci[lane] : INT_MAX;
      wave_sort(x, xi, lane);
      if (lane < K) {
        out_idx[r * K + lane] = xi;
        if (out_val) out_val[r * K + lane] = x;
      }
    }
    return;
  }

  // pass 3
  float v[KM];
  int32_t ix[KM];
#pragma unroll
  for (int p = 0; p < KM; ++p) {
    v[p] = -INFINITY;
    ix[p] = INT_MAX;
  }
  if (nc <= kTopkCand) {
    for (int32_t c = tid; c < nc; c += kTopkThreads)
      if (better(cv[c], ci[c], v[KM - 1], ix[KM - 1])) list_insert<KM>(v, ix, cv[c], ci[c]);
  } else {
    for (int32_t i = tid; i < I; i += kTopkThreads) {
      const float x = score(i, row[i]);
      if (better(x, i, v[KM - 1], ix[KM - 1])) list_insert<KM>(v, ix, x, i);
    }
  }
  __syncthreads();  // wv / wi reuse
  wave_topk(v[0], ix[0], K, lane, wv + wid * K, wi + wid * K, [&] { list_pop<KM>(v, ix); });
  __syncthreads();
  if (tid == 0) {
    float lv;
    int32_t li;
    merge_waves(wv, wi, K, K, out_val ? out_val + r * K : nullptr, out_idx + r * K, lv, li);
  }
}

__global__ __launch_bounds__(256) void hit_flags_kernel(const int32_t* __restrict__ recs,
                                                        int64_t U, int32_t K, int64_t user_base,
                                                        const int64_t* __restrict__ indptr,
                                                        const int32_t* __restrict__ truth,
                                                        int32_t* __restrict__ hit) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= U) return;
  const int64_t u = user_base + r;
  const int64_t lo = indptr[u], hi = indptr[u + 1];
  int32_t h = 0;
  for (int32_t k = 0; k < K && !h; ++k) {
    const int32_t it = recs[r * K + k];
    for (int64_t e = lo; e < hi; ++e) h |= truth[e] == it;
  }
  hit[r] = h;
}

template <int KM>
static int32_t launch_topk(const float* scores, int64_t ld, int32_t R, int32_t I, int64_t user_base,
                           const int64_t* excl_indptr, const int32_t* excl_idx, int32_t K,
                           int32_t* out_idx, float* out_val, hipStream_t st) {
  const size_t lds = (excl_indptr ? (size_t)((I + 31) / 32) * 4 : 0) + (size_t)kTopkCand * 8;
  if (lds > 48 * 1024)
    RS_CHECK_HIP(hipFuncSetAttribute((const void*)masked_topk_kernel<KM>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  masked_topk_kernel<KM><<<(unsigned)R, kTopkThreads, lds, st>>>(
      scores, ld, I, user_base, excl_indptr, excl_idx, K, out_idx, out_val);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_latest_item(const int64_t* u2i_indptr, const int32_t* u2i_items,
                                  const int64_t* timestamps, int64_t n_users, int32_t* latest,
                                  int32_t* n_missing, void* stream) {
  RS_CHECK_ARG(n_users >= 0, "rs_latest_item: bad sizes");
  if (n_users == 0) return RS_OK;
  latest_item_kernel<<<(unsigned)ceil_div(n_users, 256), 256, 0, as_stream(stream)>>>(
      u2i_indptr, u2i_items, timestamps, n_users, latest, n_missing);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_masked_topk(const float* scores, int64_t ld, int32_t n_rows, int32_t n_items,
                                  int64_t user_base, const int64_t* excl_indptr,
                                  const int32_t* excl_items, int32_t k, int32_t* out_items,
                                  float* out_scores, void* stream) {
  RS_CHECK_ARG(n_rows >= 0 && n_items >= 1 && ld >= n_items && k >= 1 && k <= n_items && k <= 64,
               "rs_masked_topk: need 1 <= k <= min(64, n_items), ld >= n_items");
  RS_CHECK_ARG(n_items <= (1 << 20), "rs_masked_topk: n_items > 2^20 (LDS exclusion bitmap)");
  if (n_rows == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  if (k <= 8)
    return launch_topk<8>(scores, ld, n_rows, n_items, user_base, excl_indptr, excl_items, k,
                          out_items, out_scores, st);
  if (k <= 16)
    return launch_topk<16>(scores, ld, n_rows, n_items, user_base, excl_indptr, excl_items, k,
                           out_items, out_scores, st);
  if (k <= 32)
    return launch_topk<32>(scores, ld, n_rows, n_items, user_base, excl_indptr, excl_items, k,
                           out_items, out_scores, st);
  return launch_topk<64>(scores, ld, n_rows, n_items, user_base, excl_indptr, excl_items, k,
                         out_items, out_scores, st);
}

extern "C" int32_t rs_hit_flags(const int32_t* recs, int64_t n_rows, int32_t k, int64_t user_base,
                                const int64_t* truth_indptr, const int32_t* truth_items,
                                int32_t* hit, void* stream) {
  RS_CHECK_ARG(n_rows >= 0 && k >= 1, "rs_hit_flags: bad sizes");
  if (n_rows == 0) return RS_OK;
  hit_flags_kernel<<<(unsigned)ceil_div(n_rows, 256), 256, 0, as_stream(stream)>>>(
      recs, n_rows, k, user_base, truth_indptr, truth_items, hit);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
