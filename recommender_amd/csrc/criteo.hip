// criteo.hip — Criteo TSV ingestion on the GPU (reference
// ctr/tfrecord_io.py:15-96). The raw text sits in HBM; everything up to device-resident id
// batches runs here:
//   line index      newline flags per 4 KiB block → block counts → scan → line starts
//   parse           one wave per line: field boundaries by ballots over 256-B chunks, lanes
//                   0..12 parse the integer features (''/negative → 0, log(x + 1) in fp32),
//                   lanes 13..38 hash the 26 categorical tokens (FNV-1a 64; empty → the
//                   column's imputation token, tfrecord_io.py:24-25), lane 0 the label
//   vocab count     open-addressing table keyed by token hash: count (atomicAdd) and first
//                   flattened position line*26 + col (atomicMin) — the reference's dict
//                   insertion order (tfrecord_io.py:15-30)
//   vocab finalise  keys with count > 10 (tfrecord_io.py:33) sorted by first position get
//                   ids 0, 1, ... (the caller sorts; rs_vocab_collect / rs_vocab_assign)
//   lookup          id of every token, 0 when absent (OOV → 0, tfrecord_io.py:64-67)
// Token identity is a 64-bit hash (collision odds ~N²/2^65, ~3e-5 for 33M distinct tokens).
#include "common.hpp"
#include "hashtab.hpp"

namespace rs {

int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* total, void* ws,
                           size_t ws_bytes, hipStream_t st);
size_t exclusive_scan_ws_size(int64_t n);

constexpr int kLineBlock = 4096;  // bytes per newline-count block

// the imputation token of an empty categorical field in column c (deterministic stand-in for
// the reference's random 10-character string per column)
__host__ __device__ __forceinline__ uint64_t imputation_hash(int c) {
  uint64_t h = kFnvBasis;
  h = (h ^ 0xFFu) * kFnvPrime;  // a byte no Criteo token contains
  h = (h ^ (uint64_t)(c & 0xFF)) * kFnvPrime;
  return h;
}

__global__ __launch_bounds__(256) void nl_count_kernel(const uint8_t* __restrict__ text,
                                                       int64_t n, int32_t* __restrict__ cnt) {
  __shared__ int32_t red[4];
  const int64_t base = (int64_t)blockIdx.x * kLineBlock;
  int32_t c = 0;
  for (int64_t i = base + threadIdx.x; i < base + kLineBlock && i < n; i += 256)
    c += text[i] == '\n';
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// line k starts after the k-th newline (line 0 at byte 0); a final line without '\n' counts
__global__ __launch_bounds__(256) void nl_write_kernel(const uint8_t* __restrict__ text, int64_t n,
                                                       const int32_t* __restrict__ offs,
                                                       int64_t* __restrict__ starts) {
  __shared__ int32_t wbase[4];
  const int64_t base = (int64_t)blockIdx.x * kLineBlock;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // each wave owns a contiguous quarter of the block, in order
  const int64_t wb = base + (int64_t)wave * (kLineBlock / 4);
  int32_t c = 0;
  for (int64_t i = wb + lane; i < wb + kLineBlock / 4 && i < n; i += 64) c += text[i] == '\n';
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if (lane == 0) wbase[wave] = c;
  __syncthreads();
  int32_t run = offs[blockIdx.x];
  for (int w = 0; w < wave; ++w) run += wbase[w];
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int64_t i0 = wb; i0 < wb + kLineBlock / 4 && i0 < n; i0 += 64) {
    const int64_t i = i0 + lane;
    const bool nl = i < n && i < wb + kLineBlock / 4 && text[i] == '\n';
    const uint64_t m = __ballot(nl);
    if (nl) starts[1 + run + __popcll(m & lt)] = i + 1;
    run += __popcll(m);
  }
}

// one wave per line; F = 1 + n_int + n_cat fields separated by '\t'
constexpr int kMaxFields = 64;

__global__ __launch_bounds__(256) void criteo_parse_kernel(
    const uint8_t* __restrict__ text, int64_t n_bytes, const int64_t* __restrict__ starts,
    int64_t n_lines, int n_int, int n_cat, float* __restrict__ label, float* __restrict__ dense,
    uint64_t* __restrict__ hashes, int32_t* __restrict__ err_flag) {
  __shared__ int32_t fpos[4][kMaxFields + 1];  // field k spans [fpos[k], fpos[k+1] - 1)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t line = (int64_t)blockIdx.x * 4 + wave;
  if (line >= n_lines) return;
  const int F = 1 + n_int + n_cat;
  const int64_t s = starts[line];
  int64_t e = line + 1 < n_lines ? starts[line + 1] : n_bytes;
  // Python text mode hands the reference each line WITH its '\n' ('\r\n' folded to '\n'),
  // and line.split('\t') leaves it on the last token: a non-empty last categorical is hashed
  // with a trailing '\n' (so "x" in C26 is a different vocab key than "x" in C1, as there)
  bool has_nl = false;
  if (e > s && text[e - 1] == '\n') {
    --e;
    has_nl = true;
    if (e > s && text[e - 1] == '\r') --e;
  }
  const int len = (int)(e - s);
  int32_t* fp = fpos[wave];
  if (lane == 0) fp[0] = 0;
  int nf = 1;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int c0 = 0; c0 < len; c0 += 64) {
    const int i = c0 + lane;
    const bool tab = i < len && text[s + i] == '\t';
    const uint64_t m = __ballot(tab);
    const int k = nf + __popcll(m & lt);
    if (tab && k <= kMaxFields) fp[k] = i + 1;
    nf += __popcll(m);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);
  if (nf != F) {  // malformed line: every output zero, flagged
    if (lane == 0) {
      flag_oob(err_flag);
      label[line] = 0.f;
    }
    for (int k = lane; k < n_int; k += 64) dense[line * n_int + k] = 0.f;
    for (int k = lane; k < n_cat; k += 64) hashes[line * n_cat + k] = imputation_hash(k);
    return;
  }
  if (lane == 0) fp[F] = len + 1;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);
  for (int k = lane; k < F; k += 64) {
    const int a = fp[k], b = fp[k + 1] - 1;  // [a, b)
    const uint8_t* p = text + s + a;
    const int n = b - a;
    if (k == 0) {
      int64_t v = 0;
      for (int q = 0; q < n; ++q) v = v * 10 + (p[q] - '0');
      label[line] = (float)v;
    } else if (k <= n_int) {
      // '' → 0; negative → 0 (tfrecord_io.py:47-50); log(x + 1) in float32 (:53)
      int64_t v = 0;
      bool neg = n > 0 && p[0] == '-';
      for (int q = neg ? 1 : 0; q < n; ++q) v = v * 10 + (p[q] - '0');
      if (neg) v = 0;
      dense[line * n_int + (k - 1)] = logf((float)v + 1.f);
    } else {
      const int c = k - 1 - n_int;
      uint64_t hv = n == 0 ? imputation_hash(c) : fnv1a(p, n);
      if (n > 0 && k == F - 1 && has_nl) hv = (hv ^ (uint64_t)'\n') * kFnvPrime;
      hashes[line * n_cat + c] = hv;
    }
  }
}


// one table insert + one atomicAdd / atomicMin per distinct key of the wave (wave_key_group);
// the group's lowest lane holds its first position (positions ascend with the lane)
__global__ __launch_bounds__(256) void vocab_count_kernel(const uint64_t* __restrict__ hashes,
                                                          const uint8_t* __restrict__ present,
                                                          int64_t n, int64_t pos_base,
                                                          uint64_t* keys, uint32_t* counts,
                                                          unsigned long long* first,
                                                          uint32_t mask, int32_t* err_flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n && (!present || present[i]);
  const uint64_t key = act ? table_key(hashes[i]) : 0;
  const uint64_t grp = wave_key_group(key, act);
  if (!act || __builtin_ctzll(grp) != (int)__lane_id()) return;
  const int64_t h = table_insert(keys, mask, key);
  if (h < 0) {
    flag_oob(err_flag);  // table full
    return;
  }
  atomicAdd(counts + h, (uint32_t)__popcll(grp));
  atomicMin(first + h, (unsigned long long)(pos_base + i));
}

// slots whose count > min_count: (first position, slot) pairs, compacted in slot order
__global__ __launch_bounds__(256) void vocab_flag_kernel(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ counts,
                                                         int64_t cap, uint32_t min_count,
                                                         int32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) flag[i] = keys[i] != kEmptySlot && counts[i] > min_count;
}

__global__ __launch_bounds__(256) void vocab_emit_kernel(const int32_t* __restrict__ flag,
                                                         const int32_t* __restrict__ offs,
                                                         const unsigned long long* __restrict__ first,
                                                         int64_t cap, uint64_t* __restrict__ first_out,
                                                         int32_t* __restrict__ slot_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap && flag[i]) {
    first_out[offs[i]] = first[i];
    slot_out[offs[i]] = (int32_t)i;
  }
}

// sorted_slots[r] (slots ordered by first appearance) gets id r
__global__ __launch_bounds__(256) void vocab_assign_kernel(const int32_t* __restrict__ sorted_slots,
                                                           int64_t n, int32_t* __restrict__ ids) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n) ids[sorted_slots[r]] = (int32_t)r;
}

__global__ __launch_bounds__(256) void vocab_lookup_kernel(const uint64_t* __restrict__ hashes,
                                                           int64_t n, const uint64_t* __restrict__ keys,
                                                           const int32_t* __restrict__ ids,
                                                           uint32_t mask, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t h = table_find(keys, mask, hashes[i]);
  out[i] = (h >= 0 && ids[h] >= 0) ? ids[h] : 0;  // OOV → 0
}

inline unsigned grid256(int64_t n) { return (unsigned)ceil_div(n < 1 ? 1 : n, 256); }

}  // namespace rs

using namespace rs;

extern "C" size_t rs_line_index_workspace_size(int64_t n_bytes) {
  const int64_t nb = ceil_div(n_bytes < 1 ? 1 : n_bytes, kLineBlock);
  Carver c(nullptr, 0);
  c.take<int32_t>(nb);
  c.take<int32_t>(nb);
  c.take<char>(exclusive_scan_ws_size(nb));
  return c.off + 256;
}

extern "C" int32_t rs_line_index(const uint8_t* text, int64_t n_bytes, int64_t* line_starts,
                                 int32_t* n_newlines, void* workspace, size_t ws_bytes,
                                 void* stream) {
  RS_CHECK_ARG(n_bytes >= 1 && n_bytes < ((int64_t)1 << 40), "rs_line_index: bad size");
  hipStream_t st = as_stream(stream);
  const int64_t nb = ceil_div(n_bytes, kLineBlock);
  Carver c(workspace, ws_bytes);
  int32_t* cnt = c.take<int32_t>(nb);
  int32_t* offs = c.take<int32_t>(nb);
  void* sws = c.take<char>(exclusive_scan_ws_size(nb));
  if (!c.ok()) {
    set_error("rs_line_index: workspace too small");
    return RS_E_WORKSPACE;
  }
  nl_count_kernel<<<(unsigned)nb, 256, 0, st>>>(text, n_bytes, cnt);
  RS_CHECK_LAUNCH();
  int32_t s = exclusive_scan_i32(cnt, offs, nb, n_newlines, sws, exclusive_scan_ws_size(nb), st);
  if (s) return s;
  if (!line_starts) return RS_OK;  // count only (the caller sizes line_starts from it)
  RS_CHECK_HIP(hipMemsetAsync(line_starts, 0, sizeof(int64_t), st));
  nl_write_kernel<<<(unsigned)nb, 256, 0, st>>>(text, n_bytes, offs, line_starts);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_criteo_parse(const uint8_t* text, int64_t n_bytes, const int64_t* line_starts,
                                   int64_t n_lines, int32_t n_int, int32_t n_cat, float* label,
                                   float* dense, uint64_t* hashes, int32_t* err_flag,
                                   void* stream) {
  RS_CHECK_ARG(n_lines >= 0 && n_int >= 0 && n_cat >= 0 && 1 + n_int + n_cat <= kMaxFields,
               "rs_criteo_parse: bad sizes");
  if (n_lines == 0) return RS_OK;
  criteo_parse_kernel<<<(unsigned)ceil_div(n_lines, 4), 256, 0, as_stream(stream)>>>(
      text, n_bytes, line_starts, n_lines, n_int, n_cat, label, dense, hashes, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_vocab_count(const uint64_t* hashes, int64_t n, int64_t pos_base,
                                  uint64_t* keys, uint32_t* counts, uint64_t* first_pos,
                                  int64_t capacity, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(capacity >= 2 && (capacity & (capacity - 1)) == 0 && capacity <= ((int64_t)1 << 32),
               "rs_vocab_count: capacity must be a power of two");
  if (n == 0) return RS_OK;
  vocab_count_kernel<<<grid256(n), 256, 0, as_stream(stream)>>>(
      hashes, nullptr, n, pos_base, keys, counts, reinterpret_cast<unsigned long long*>(first_pos),
      (uint32_t)(capacity - 1), err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_vocab_count_masked(const uint64_t* hashes, const uint8_t* present, int64_t n,
                                         int64_t pos_base, uint64_t* keys, uint32_t* counts,
                                         uint64_t* first_pos, int64_t capacity, int32_t* err_flag,
                                         void* stream) {
  RS_CHECK_ARG(capacity >= 2 && (capacity & (capacity - 1)) == 0 && capacity <= ((int64_t)1 << 32),
               "rs_vocab_count_masked: capacity must be a power of two");
  if (n == 0) return RS_OK;
  vocab_count_kernel<<<grid256(n), 256, 0, as_stream(stream)>>>(
      hashes, present, n, pos_base, keys, counts, reinterpret_cast<unsigned long long*>(first_pos),
      (uint32_t)(capacity - 1), err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_vocab_collect_workspace_size(int64_t capacity) {
  Carver c(nullptr, 0);
  c.take<int32_t>(capacity);
  c.take<int32_t>(capacity);
  c.take<char>(exclusive_scan_ws_size(capacity));
  return c.off + 256;
}

extern "C" int32_t rs_vocab_collect(const uint64_t* keys, const uint32_t* counts,
                                    const uint64_t* first_pos, int64_t capacity,
                                    uint32_t min_count, uint64_t* first_out, int32_t* slot_out,
                                    int32_t* n_kept, void* workspace, size_t ws_bytes,
                                    void* stream) {
  hipStream_t st = as_stream(stream);
  Carver c(workspace, ws_bytes);
  int32_t* flag = c.take<int32_t>(capacity);
  int32_t* offs = c.take<int32_t>(capacity);
  void* sws = c.take<char>(exclusive_scan_ws_size(capacity));
  if (!c.ok()) {
    set_error("rs_vocab_collect: workspace too small");
    return RS_E_WORKSPACE;
  }
  vocab_flag_kernel<<<grid256(capacity), 256, 0, st>>>(keys, counts, capacity, min_count, flag);
  RS_CHECK_LAUNCH();
  int32_t s = exclusive_scan_i32(flag, offs, capacity, n_kept, sws, exclusive_scan_ws_size(capacity), st);
  if (s) return s;
  vocab_emit_kernel<<<grid256(capacity), 256, 0, st>>>(
      flag, offs, reinterpret_cast<const unsigned long long*>(first_pos), capacity, first_out,
      slot_out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_vocab_assign(const int32_t* sorted_slots, int64_t n_kept, int32_t* ids,
                                   void* stream) {
  if (n_kept == 0) return RS_OK;
  vocab_assign_kernel<<<grid256(n_kept), 256, 0, as_stream(stream)>>>(sorted_slots, n_kept, ids);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_vocab_lookup(const uint64_t* hashes, int64_t n, const uint64_t* keys,
                                   const int32_t* ids, int64_t capacity, int64_t* out,
                                   void* stream) {
  RS_CHECK_ARG(capacity >= 2 && (capacity & (capacity - 1)) == 0, "rs_vocab_lookup: capacity");
  if (n == 0) return RS_OK;
  vocab_lookup_kernel<<<grid256(n), 256, 0, as_stream(stream)>>>(hashes, n, keys, ids,
                                                                 (uint32_t)(capacity - 1), out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
