// textpipe.hip — the Ali-CCP and Amazon (DIEN) text → id pipelines on the GPU (SURVEY §8f rank 4;
// reference esmm/process_public_dataset.py:40-153, dien/util.py:4-37, dien/data_loader.py:27-63).
// The raw text sits in HBM (line index from rs_line_index); every step up to device-resident id
// tensors runs here:
//   rs_kv_parse          one wave per CSV line: comma fields by ballots, re.split('\x01|\x02|\x03')
//                        token numbering by ballots over 64-B chunks, each key token hashed by the
//                        lane that owns its start and matched against the wanted columns; the last
//                        occurrence of a column wins (LDS atomicMax over the value's byte offset,
//                        dict(zip(keys, values)) semantics), then one lane per column hashes it
//   rs_map_insert        common-feature id → line (a later duplicate line wins, as dict assignment)
//   rs_aliccp_join       drop (click '0', purchase '1') lines, overlay the common features,
//                        key = (column, value) hash, '0' for an absent column; compacted by a scan
//   rs_vocab_regroup / rs_vocab_assign_grouped
//                        per-column ids 1.. in first-appearance order (the caller's radix sort)
//   rs_dien_parse        one wave per line: 6 tab fields, '\x02'-separated histories, count pass
//                        then a fill pass into line-major ragged token streams
//   rs_dien_item_cat     item_id2cat_id: the last (item, cat) pair of the stream wins, mapped to ids
//   rs_dien_encode       lookups (unknown item → unk, unknown cat → error), pad_sequences(post, pre)
//                        and the DIEN negative history (Philox keyed by (seed, line, position))
#include "common.hpp"
#include "hashtab.hpp"
#include "rng.hpp"

namespace rs {

int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* total, void* ws,
                           size_t ws_bytes, hipStream_t st);
size_t exclusive_scan_ws_size(int64_t n);

namespace {

constexpr int kMaxCols = 32;
constexpr int kMaxCommas = 8;
constexpr uint32_t kPurposeDienNeg = 0xD1E40001u;

inline unsigned grid256(int64_t n) { return (unsigned)ceil_div(n < 1 ? 1 : n, 256); }

// Python str.strip() whitespace among single bytes: ' ', \t..\r, \x1c..\x1f
__device__ __forceinline__ bool py_ws(uint8_t b) {
  return b == ' ' || (b >= 9 && b <= 13) || (b >= 0x1c && b <= 0x1f);
}

__device__ __forceinline__ uint64_t lanes_below(int lane) {
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);
}

// [s, e) of line `line` after strip() (lane-uniform result)
__device__ __forceinline__ void stripped_line(const uint8_t* text, int64_t n_bytes,
                                              const int64_t* starts, int64_t n_lines, int64_t line,
                                              int64_t& s, int64_t& e) {
  s = starts[line];
  e = line + 1 < n_lines ? starts[line + 1] : n_bytes;
  while (e > s && py_ws(text[e - 1])) --e;
  while (s < e && py_ws(text[s])) ++s;
}

struct KvSep {  // re.split('\x01|\x02|\x03')
  __device__ __forceinline__ bool operator()(uint8_t b) const { return b >= 1 && b <= 3; }
};

// FNV-1a of [p, end) up to the first byte for which stop() holds; *q = that byte's offset
template <typename Stop>
__device__ __forceinline__ uint64_t hash_token(const uint8_t* text, int64_t p, int64_t end,
                                               Stop stop, int64_t* q) {
  uint64_t h = kFnvBasis;
  while (p < end && !stop(text[p])) {
    h = (h ^ text[p]) * kFnvPrime;
    ++p;
  }
  *q = p;
  return h;
}

// (column, value) key of the Ali-CCP vocabulary: one more FNV step over a non-byte symbol
__device__ __forceinline__ uint64_t col_key(int c, uint64_t vh) {
  return (vh ^ (uint64_t)(0x100 + c)) * kFnvPrime;
}

__device__ __forceinline__ uint64_t zero_token_hash() {  // the string '0'
  return (kFnvBasis ^ (uint64_t)'0') * kFnvPrime;
}

// ---- Ali-CCP --------------------------------------------------------------------------------

// the line's bytes staged in LDS when they fit (coalesced byte loads), else read in place
constexpr int kStage = 4096;

__device__ __forceinline__ const uint8_t* stage_line(const uint8_t* text, int64_t s, int len,
                                                     uint8_t* buf, int lane) {
  if (len > kStage) return text + s;
  for (int i = lane; i < len; i += 64) buf[i] = text[s + i];
  wave_sync_lds();
  return buf;
}

__global__ __launch_bounds__(256) void kv_parse_kernel(
    const uint8_t* __restrict__ text, int64_t n_bytes, const int64_t* __restrict__ starts,
    int64_t n_lines, int key_field, int kv_field, int with_labels,
    const uint64_t* __restrict__ col_hashes, int n_cols, uint64_t* __restrict__ key_hash,
    int32_t* __restrict__ keep, int32_t* __restrict__ labels, uint64_t* __restrict__ vals,
    uint8_t* __restrict__ present, int32_t* __restrict__ err_flag) {
  __shared__ uint8_t stage[4][kStage];
  __shared__ int32_t commas[4][kMaxCommas];
  __shared__ int32_t best[4][kMaxCols];  // offset (in the line) of the column's value token
  __shared__ uint64_t wanted[kMaxCols];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x < n_cols) wanted[threadIdx.x] = col_hashes[threadIdx.x];
  __syncthreads();
  const int64_t line = (int64_t)blockIdx.x * 4 + wave;
  if (line >= n_lines) return;
  int64_t s, e;
  stripped_line(text, n_bytes, starts, n_lines, line, s, e);
  const int len = (int)(e - s);
  if (lane < n_cols) best[wave][lane] = -1;
  const uint8_t* lp = stage_line(text, s, len, stage[wave], lane);
  // comma positions (the first kMaxCommas)
  int nc = 0;
  const uint64_t lt = lanes_below(lane);
  for (int c0 = 0; c0 < len && nc < kMaxCommas; c0 += 64) {
    const int i = c0 + lane;
    const bool cm = i < len && lp[i] == ',';
    const uint64_t m = __ballot(cm);
    const int k = nc + __popcll(m & lt);
    if (cm && k < kMaxCommas) commas[wave][k] = i;
    nc += __popcll(m);
  }
  wave_sync_lds();
  const int need = kv_field > key_field ? kv_field : key_field;
  if (nc < need || (with_labels && nc < 2)) {  // ll[k] raises IndexError in the reference
    if (lane == 0) flag_oob(err_flag);
    if (lane < n_cols) present[line * n_cols + lane] = 0;
    if (lane == 0) {
      if (key_hash) key_hash[line] = kFnvBasis;
      if (keep) keep[line] = 0;
      if (labels) labels[2 * line] = labels[2 * line + 1] = 0;
    }
    return;
  }
  const int* cp = commas[wave];
  auto field_lo = [&](int k) { return k == 0 ? 0 : cp[k - 1] + 1; };
  auto field_hi = [&](int k) { return k < nc && k < kMaxCommas ? cp[k] : len; };
  if (lane == 0) {
    if (key_hash) {
      int64_t q;
      key_hash[line] = hash_token(lp, field_lo(key_field), field_hi(key_field),
                                  [](uint8_t) { return false; }, &q);
    }
    if (with_labels) {
      const int a1 = field_lo(1), b1 = field_hi(1), a2 = field_lo(2), b2 = field_hi(2);
      int v1 = 0, v2 = 0;
      for (int q = a1; q < b1; ++q) v1 = v1 * 10 + (lp[q] - '0');
      for (int q = a2; q < b2; ++q) v2 = v2 * 10 + (lp[q] - '0');
      if (labels) {
        labels[2 * line] = v1;
        labels[2 * line + 1] = v2;
      }
      // `ll[1] == '0' and ll[2] == '1'` on the strings (:56)
      const bool drop = b1 - a1 == 1 && lp[a1] == '0' && b2 - a2 == 1 && lp[a2] == '1';
      if (keep) keep[line] = drop ? 0 : 1;
    }
  }
  // kv tokens: token 0 starts at a, token t + 1 right after the t-th separator
  const int a = field_lo(kv_field), b = field_hi(kv_field);
  auto visit = [&](int start, int t) {  // a token start owned by this lane
    if (t % 3) return;                  // keys are tokens 0, 3, 6, ..
    int64_t q;
    const uint64_t kh = hash_token(lp, start, b, KvSep{}, &q);
    if (q >= b) return;  // no value token follows: zip drops the key
    for (int c = 0; c < n_cols; ++c)
      if (wanted[c] == kh) atomicMax(&best[wave][c], (int32_t)(q + 1));
  };
  int tcount = 0;  // separators before the current chunk
  if (lane == 0) visit(a, 0);
  for (int c0 = a; c0 < b; c0 += 64) {
    const int i = c0 + lane;
    const bool sep = i < b && KvSep{}(lp[i]);
    const uint64_t m = __ballot(sep);
    if (sep) visit(i + 1, tcount + __popcll(m & lt) + 1);
    tcount += __popcll(m);
  }
  wave_sync_lds();
  if (lane < n_cols) {
    const int o = best[wave][lane];
    uint64_t vh = 0;
    if (o >= 0) {
      int64_t q;
      vh = hash_token(lp, o, b, KvSep{}, &q);
    }
    vals[line * n_cols + lane] = vh;
    present[line * n_cols + lane] = o >= 0;
  }
}

__global__ __launch_bounds__(256) void map_insert_kernel(const uint64_t* __restrict__ key_hash,
                                                         int64_t n, uint64_t* keys, int32_t* vals,
                                                         uint32_t mask, int32_t* err_flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t h = table_insert(keys, mask, key_hash[i]);
  if (h < 0) {
    flag_oob(err_flag);
    return;
  }
  atomicMax(vals + h, (int32_t)i);
}

// one thread per (skeleton line, column); rows compacted by offs = exclusive scan of keep
__global__ __launch_bounds__(256) void aliccp_join_kernel(
    const int32_t* __restrict__ keep, const int32_t* __restrict__ offs, int64_t n_lines,
    int n_cols, const uint64_t* __restrict__ common_id, const uint64_t* __restrict__ svals,
    const uint8_t* __restrict__ spresent, const int32_t* __restrict__ slabels,
    const uint64_t* __restrict__ map_keys, const int32_t* __restrict__ map_vals, uint32_t map_mask,
    const uint64_t* __restrict__ cvals, const uint8_t* __restrict__ cpresent,
    uint64_t* __restrict__ out_keys, uint8_t* __restrict__ out_present,
    int32_t* __restrict__ out_labels, int32_t* __restrict__ err_flag) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_lines * n_cols) return;
  const int64_t line = t / n_cols;
  const int c = (int)(t % n_cols);
  if (!keep[line]) return;
  const int64_t r = offs[line];
  const int64_t h = table_find(map_keys, map_mask, common_id[line]);
  int64_t cr = -1;
  if (h >= 0) cr = map_vals[h];
  else if (c == 0) flag_oob(err_flag);  // common_feat_dict[...] KeyError (:61)
  uint64_t vh = zero_token_hash();
  bool pres = false;
  if (cr >= 0 && cpresent[cr * n_cols + c]) {
    vh = cvals[cr * n_cols + c];
    pres = true;
  } else if (spresent[line * n_cols + c]) {
    vh = svals[line * n_cols + c];
    pres = true;
  }
  out_keys[r * n_cols + c] = col_key(c, vh);
  out_present[r * n_cols + c] = pres;
  if (c < 2) out_labels[2 * r + c] = slabels[2 * line + c];
}

// sort key (group, first position) for per-group first-appearance numbering; group = pos % G
__global__ __launch_bounds__(256) void regroup_kernel(const uint64_t* __restrict__ first, int64_t n,
                                                      int32_t n_groups, int64_t per_group,
                                                      int64_t* __restrict__ sort_key,
                                                      int32_t* __restrict__ group) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t p = (int64_t)first[i];
  const int32_t g = (int32_t)(p % n_groups);
  sort_key[i] = (int64_t)g * per_group + p / n_groups;
  group[i] = g;
}

// ids[slots[order[r]]] = base + r - (first rank of r's group)
__global__ __launch_bounds__(256) void assign_grouped_kernel(const int32_t* __restrict__ order,
                                                             const int32_t* __restrict__ slots,
                                                             const int32_t* __restrict__ group,
                                                             int64_t n, int32_t base,
                                                             int32_t* __restrict__ ids) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int32_t k = order ? order[r] : (int32_t)r;
  int64_t start = 0;
  if (group) {
    const int32_t g = group[k];
    int64_t lo = 0, hi = r;  // first rank whose group is g (groups ascend along the order)
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      const int32_t gm = group[order ? order[mid] : mid];
      if (gm < g) lo = mid + 1;
      else hi = mid;
    }
    start = lo;
  }
  ids[slots[k]] = base + (int32_t)(r - start);
}

__global__ __launch_bounds__(256) void lookup_i32_kernel(const uint64_t* __restrict__ hashes,
                                                         int64_t n, const uint64_t* __restrict__ keys,
                                                         const int32_t* __restrict__ ids,
                                                         uint32_t mask, int32_t oov_id, int err_on_oov,
                                                         int32_t* __restrict__ out,
                                                         int32_t* __restrict__ err_flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t h = table_find(keys, mask, hashes[i]);
  int32_t id = h >= 0 ? ids[h] : -1;
  if (id < 0) {
    id = oov_id;
    if (err_on_oov) flag_oob(err_flag);
  }
  out[i] = id;
}

// ---- Amazon / DIEN ----------------------------------------------------------------------------

// fields of a DIEN line: label, user, item, cat, his_items, his_cats (5 tabs exactly)
__device__ __forceinline__ bool dien_fields(const uint8_t* lp, int len, int lane, int32_t* fp) {
  int nt = 0;
  const uint64_t lt = lanes_below(lane);
  if (lane == 0) fp[0] = 0;
  for (int c0 = 0; c0 < len; c0 += 64) {
    const int i = c0 + lane;
    const bool tab = i < len && lp[i] == '\t';
    const uint64_t m = __ballot(tab);
    const int k = nt + __popcll(m & lt) + 1;
    if (tab && k <= 6) fp[k] = i + 1;
    nt += __popcll(m);
  }
  if (lane == 0) fp[6] = len + 1;  // field k spans [fp[k], fp[k+1] - 1)
  wave_sync_lds();
  return nt == 5;
}

struct IsX02 {
  __device__ __forceinline__ bool operator()(uint8_t x) const { return x == 2; }
};

// number of '\x02'-separated tokens of [a, b) (an empty field is one empty token), and with
// `out` the token hashes written to out[0..n)
__device__ __forceinline__ int dien_tokens(const uint8_t* lp, int a, int b, int lane,
                                           uint64_t* out) {
  const uint64_t lt = lanes_below(lane);
  int n = 1;
  if (out && lane == 0) {
    int64_t q;
    out[0] = hash_token(lp, a, b, IsX02{}, &q);
  }
  for (int c0 = a; c0 < b; c0 += 64) {
    const int i = c0 + lane;
    const bool sep = i < b && lp[i] == 2;
    const uint64_t m = __ballot(sep);
    if (sep && out) {
      int64_t q;
      out[n + __popcll(m & lt)] = hash_token(lp, i + 1, b, IsX02{}, &q);
    }
    n += __popcll(m);
  }
  return n;
}

__device__ __forceinline__ float parse_label(const uint8_t* p, int n) {
  double v = 0.0, scale = 1.0;
  bool frac = false, neg = false;
  for (int q = 0; q < n; ++q) {
    const uint8_t ch = p[q];
    if (q == 0 && (ch == '-' || ch == '+')) {
      neg = ch == '-';
    } else if (ch == '.') {
      frac = true;
    } else if (frac) {
      scale *= 0.1;
      v += (ch - '0') * scale;
    } else {
      v = v * 10.0 + (ch - '0');
    }
  }
  return (float)(neg ? -v : v);
}

// count pass (item_off == nullptr): n_hi / n_hc / label per line; fill pass: token hashes at
// item_off[line] (target item, then history) and cat_off[line] (target cat, then history)
__global__ __launch_bounds__(256) void dien_parse_kernel(
    const uint8_t* __restrict__ text, int64_t n_bytes, const int64_t* __restrict__ starts,
    int64_t n_lines, const int64_t* __restrict__ item_off, const int64_t* __restrict__ cat_off,
    int32_t* __restrict__ n_hi, int32_t* __restrict__ n_hc, float* __restrict__ label,
    uint64_t* __restrict__ item_hash, uint64_t* __restrict__ cat_hash,
    int32_t* __restrict__ err_flag) {
  __shared__ uint8_t stage[4][kStage];
  __shared__ int32_t fpos[4][8];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t line = (int64_t)blockIdx.x * 4 + wave;
  if (line >= n_lines) return;
  int64_t s, e;
  stripped_line(text, n_bytes, starts, n_lines, line, s, e);
  const int len = (int)(e - s);
  const uint8_t* lp = stage_line(text, s, len, stage[wave], lane);
  int32_t* fp = fpos[wave];
  if (!dien_fields(lp, len, lane, fp)) {  // unpacking 6 fields raises in the reference
    if (!item_off && lane == 0) {
      flag_oob(err_flag);
      n_hi[line] = n_hc[line] = 1;
      label[line] = 0.f;
    }
    if (item_off && lane == 0) {
      item_hash[item_off[line]] = item_hash[item_off[line] + 1] = kFnvBasis;
      cat_hash[cat_off[line]] = cat_hash[cat_off[line] + 1] = kFnvBasis;
    }
    return;
  }
  auto lo = [&](int k) { return fp[k]; };
  auto hi = [&](int k) { return fp[k + 1] - 1; };
  if (!item_off) {
    const int a = dien_tokens(lp, lo(4), hi(4), lane, nullptr);
    const int c = dien_tokens(lp, lo(5), hi(5), lane, nullptr);
    if (lane == 0) {
      n_hi[line] = a;
      n_hc[line] = c;
      label[line] = parse_label(lp + lo(0), hi(0) - lo(0));
    }
    return;
  }
  if (lane == 0) {
    int64_t q;
    auto never = [](uint8_t) { return false; };
    item_hash[item_off[line]] = hash_token(lp, lo(2), hi(2), never, &q);
    cat_hash[cat_off[line]] = hash_token(lp, lo(3), hi(3), never, &q);
  }
  dien_tokens(lp, lo(4), hi(4), lane, item_hash + item_off[line] + 1);
  dien_tokens(lp, lo(5), hi(5), lane, cat_hash + cat_off[line] + 1);
}

// item_id2cat_id: pairs (item_off[l] + j, cat_off[l] + j) for j < 1 + min(n_hi, n_hc); the pair
// latest in the stream wins (pass 0: atomicMax of its position, pass 1: the winner writes)
__global__ __launch_bounds__(256) void dien_pairs_kernel(
    const uint64_t* __restrict__ item_hash, const uint64_t* __restrict__ cat_hash,
    const int64_t* __restrict__ item_off, const int64_t* __restrict__ cat_off,
    const int32_t* __restrict__ n_hi, const int32_t* __restrict__ n_hc, int64_t n_lines,
    const uint64_t* __restrict__ keys, uint32_t mask, int pass,
    unsigned long long* __restrict__ last_pos, uint64_t* __restrict__ slot_cat) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t line = (int64_t)blockIdx.x * 4 + wave;
  if (line >= n_lines) return;
  const int np = 1 + min(n_hi[line], n_hc[line]);
  for (int j0 = 0; j0 < np; j0 += 64) {  // wave-uniform trip count: wave_key_group needs all lanes
    const int j = j0 + lane;
    const int64_t p = item_off[line] + j;
    const int64_t h = j < np ? table_find(keys, mask, item_hash[p]) : -1;
    if (pass == 0) {
      // the latest position of each distinct item in this chunk is its highest lane
      const uint64_t grp = wave_key_group((uint64_t)h, h >= 0);
      if (h >= 0 && 63 - __builtin_clzll(grp) == lane)
        atomicMax(last_pos + h, (unsigned long long)(p + 1));
    } else if (h >= 0 && last_pos[h] == (unsigned long long)(p + 1)) {
      slot_cat[h] = cat_hash[cat_off[line] + j];
    }
  }
}

// cat_of_item[id] for every item slot; -1 for an item that never had a cat partner
__global__ __launch_bounds__(256) void dien_cat_map_kernel(
    const uint64_t* __restrict__ item_keys, const int32_t* __restrict__ item_ids, int64_t item_cap,
    const unsigned long long* __restrict__ last_pos, const uint64_t* __restrict__ slot_cat,
    const uint64_t* __restrict__ cat_keys, const int32_t* __restrict__ cat_ids, uint32_t cat_mask,
    int32_t* __restrict__ cat_of_item) {
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= item_cap || item_keys[h] == kEmptySlot || item_ids[h] < 0) return;
  int32_t c = -1;
  if (last_pos[h] != 0) {
    const int64_t ch = table_find(cat_keys, cat_mask, slot_cat[h]);
    if (ch >= 0) c = cat_ids[ch];
  }
  cat_of_item[item_ids[h]] = c;
}

struct DienTables {
  const uint64_t* item_keys;
  const int32_t* item_ids;
  uint32_t item_mask;
  int32_t unk_item;
  const uint64_t* cat_keys;
  const int32_t* cat_ids;
  uint32_t cat_mask;
};

__device__ __forceinline__ int32_t find_id(const uint64_t* keys, const int32_t* ids, uint32_t mask,
                                           uint64_t h) {
  const int64_t s = table_find(keys, mask, h);
  return s >= 0 ? ids[s] : -1;
}

// one wave per line: lanes over the maxlen history positions
__global__ __launch_bounds__(256) void dien_encode_kernel(
    const uint64_t* __restrict__ item_hash, const uint64_t* __restrict__ cat_hash,
    const int64_t* __restrict__ item_off, const int64_t* __restrict__ cat_off,
    const int32_t* __restrict__ n_hi, const int32_t* __restrict__ n_hc, int64_t n_lines,
    DienTables tb, int maxlen, const int32_t* __restrict__ cat_of_item, int32_t n_item_ids,
    uint64_t seed, int64_t line_base, int32_t* __restrict__ target_item,
    int32_t* __restrict__ target_cat, int32_t* __restrict__ his_item, int32_t* __restrict__ his_cat,
    int32_t* __restrict__ neg_item, int32_t* __restrict__ neg_cat, int32_t* __restrict__ err_flag) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t line = (int64_t)blockIdx.x * 4 + wave;
  if (line >= n_lines) return;
  const int64_t io = item_off[line], co = cat_off[line];
  bool bad = false;
  if (lane == 0) {
    int32_t it = find_id(tb.item_keys, tb.item_ids, tb.item_mask, item_hash[io]);
    int32_t ct = find_id(tb.cat_keys, tb.cat_ids, tb.cat_mask, cat_hash[co]);
    if (ct < 0) bad = true;  // cat_vocab[cat] KeyError (data_loader.py:32)
    target_item[line] = it < 0 ? tb.unk_item : it;
    target_cat[line] = ct < 0 ? 0 : ct;
  }
  const int ni = n_hi[line], nc = n_hc[line];
  const int ki = min(ni, maxlen), kc = min(nc, maxlen);  // keep the LAST maxlen tokens
  for (int j = lane; j < maxlen; j += 64) {
    int32_t v = 0;
    if (j < ki) {
      v = find_id(tb.item_keys, tb.item_ids, tb.item_mask, item_hash[io + 1 + (ni - ki) + j]);
      if (v < 0) v = tb.unk_item;
    }
    his_item[line * maxlen + j] = v;
    int32_t w = 0;
    if (j < kc) {
      w = find_id(tb.cat_keys, tb.cat_ids, tb.cat_mask, cat_hash[co + 1 + (nc - kc) + j]);
      if (w < 0) {
        bad = true;
        w = 0;
      }
    }
    his_cat[line * maxlen + j] = w;
    if (neg_item) {  // np.random.randint(1, len(item_vocab)) (data_loader.py:52)
      const uint32_t r = draw(seed, kPurposeDienNeg, (uint32_t)(line_base + line),
                              (uint32_t)((uint64_t)(line_base + line) >> 32), 0u, (uint32_t)j);
      const int32_t item = 1 + (int32_t)bounded(r, (uint32_t)(n_item_ids - 1));
      int32_t c = cat_of_item[item];
      if (c < 0) {  // item_id2cat_id KeyError
        bad = true;
        c = 0;
      }
      neg_item[line * maxlen + j] = item;
      neg_cat[line * maxlen + j] = c;
    }
  }
  if (bad) flag_oob(err_flag);
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int32_t rs_kv_parse(const uint8_t* text, int64_t n_bytes, const int64_t* line_starts,
                               int64_t n_lines, int32_t key_field, int32_t kv_field,
                               int32_t with_labels, const uint64_t* col_hashes, int32_t n_cols,
                               uint64_t* key_hash, int32_t* keep, int32_t* labels, uint64_t* vals,
                               uint8_t* present, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(n_lines >= 0 && n_cols >= 1 && n_cols <= kMaxCols && key_field >= 0 &&
                   key_field < kMaxCommas && kv_field >= 0 && kv_field < kMaxCommas &&
                   (!with_labels || keep),
               "rs_kv_parse: bad arguments");
  if (n_lines == 0) return RS_OK;
  kv_parse_kernel<<<(unsigned)ceil_div(n_lines, 4), 256, 0, as_stream(stream)>>>(
      text, n_bytes, line_starts, n_lines, key_field, kv_field, with_labels, col_hashes, n_cols,
      key_hash, keep, labels, vals, present, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_map_insert(const uint64_t* key_hash, int64_t n, uint64_t* keys, int32_t* vals,
                                 int64_t capacity, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(capacity >= 2 && (capacity & (capacity - 1)) == 0 && capacity <= ((int64_t)1 << 32) &&
                   n < ((int64_t)1 << 31),
               "rs_map_insert: capacity must be a power of two");
  if (n == 0) return RS_OK;
  map_insert_kernel<<<grid256(n), 256, 0, as_stream(stream)>>>(key_hash, n, keys, vals,
                                                               (uint32_t)(capacity - 1), err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_aliccp_join_workspace_size(int64_t n_lines) {
  Carver c(nullptr, 0);
  c.take<int32_t>(n_lines);
  c.take<char>(exclusive_scan_ws_size(n_lines));
  return c.off + 256;
}

extern "C" int32_t rs_aliccp_join(const int32_t* keep, int64_t n_lines, int32_t n_cols,
                                  const uint64_t* common_id, const uint64_t* skel_vals,
                                  const uint8_t* skel_present, const int32_t* skel_labels,
                                  const uint64_t* map_keys, const int32_t* map_vals,
                                  int64_t map_capacity, const uint64_t* common_vals,
                                  const uint8_t* common_present, uint64_t* out_keys,
                                  uint8_t* out_present, int32_t* out_labels, int32_t* n_kept,
                                  int32_t* err_flag, void* workspace, size_t ws_bytes,
                                  void* stream) {
  RS_CHECK_ARG(n_lines >= 0 && n_lines < ((int64_t)1 << 31) && n_cols >= 2 && n_cols <= kMaxCols &&
                   map_capacity >= 2 && (map_capacity & (map_capacity - 1)) == 0,
               "rs_aliccp_join: bad arguments");
  hipStream_t st = as_stream(stream);
  if (n_lines == 0) {
    RS_CHECK_HIP(hipMemsetAsync(n_kept, 0, sizeof(int32_t), st));
    return RS_OK;
  }
  Carver c(workspace, ws_bytes);
  int32_t* offs = c.take<int32_t>(n_lines);
  void* sws = c.take<char>(exclusive_scan_ws_size(n_lines));
  if (!c.ok()) {
    set_error("rs_aliccp_join: workspace too small");
    return RS_E_WORKSPACE;
  }
  int32_t s = exclusive_scan_i32(keep, offs, n_lines, n_kept, sws, exclusive_scan_ws_size(n_lines), st);
  if (s) return s;
  aliccp_join_kernel<<<grid256(n_lines * n_cols), 256, 0, st>>>(
      keep, offs, n_lines, n_cols, common_id, skel_vals, skel_present, skel_labels, map_keys,
      map_vals, (uint32_t)(map_capacity - 1), common_vals, common_present, out_keys, out_present,
      out_labels, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_vocab_regroup(const uint64_t* first_pos, int64_t n, int32_t n_groups,
                                    int64_t per_group, int64_t* sort_key, int32_t* group,
                                    void* stream) {
  RS_CHECK_ARG(n >= 0 && n_groups >= 1 && per_group >= 1, "rs_vocab_regroup: bad sizes");
  if (n == 0) return RS_OK;
  regroup_kernel<<<grid256(n), 256, 0, as_stream(stream)>>>(first_pos, n, n_groups, per_group,
                                                            sort_key, group);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_vocab_assign_grouped(const int32_t* order, const int32_t* slots,
                                           const int32_t* group, int64_t n_kept, int32_t id_base,
                                           int32_t* ids, void* stream) {
  RS_CHECK_ARG(n_kept >= 0 && n_kept < ((int64_t)1 << 31), "rs_vocab_assign_grouped: bad size");
  if (n_kept == 0) return RS_OK;
  assign_grouped_kernel<<<grid256(n_kept), 256, 0, as_stream(stream)>>>(order, slots, group, n_kept,
                                                                         id_base, ids);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_vocab_lookup_i32(const uint64_t* hashes, int64_t n, const uint64_t* keys,
                                       const int32_t* ids, int64_t capacity, int32_t oov_id,
                                       int32_t err_on_oov, int32_t* out, int32_t* err_flag,
                                       void* stream) {
  RS_CHECK_ARG(capacity >= 2 && (capacity & (capacity - 1)) == 0, "rs_vocab_lookup_i32: capacity");
  if (n == 0) return RS_OK;
  lookup_i32_kernel<<<grid256(n), 256, 0, as_stream(stream)>>>(
      hashes, n, keys, ids, (uint32_t)(capacity - 1), oov_id, err_on_oov, out, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_dien_parse(const uint8_t* text, int64_t n_bytes, const int64_t* line_starts,
                                 int64_t n_lines, const int64_t* item_off, const int64_t* cat_off,
                                 int32_t* n_hi, int32_t* n_hc, float* label, uint64_t* item_hash,
                                 uint64_t* cat_hash, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(n_lines >= 0 && (item_off == nullptr) == (cat_off == nullptr) &&
                   (!item_off || (item_hash && cat_hash)),
               "rs_dien_parse: bad arguments");
  if (n_lines == 0) return RS_OK;
  dien_parse_kernel<<<(unsigned)ceil_div(n_lines, 4), 256, 0, as_stream(stream)>>>(
      text, n_bytes, line_starts, n_lines, item_off, cat_off, n_hi, n_hc, label, item_hash,
      cat_hash, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" size_t rs_dien_item_cat_workspace_size(int64_t item_capacity) {
  Carver c(nullptr, 0);
  c.take<unsigned long long>(item_capacity);
  c.take<uint64_t>(item_capacity);
  return c.off + 256;
}

extern "C" int32_t rs_dien_item_cat(const uint64_t* item_hash, const uint64_t* cat_hash,
                                    const int64_t* item_off, const int64_t* cat_off,
                                    const int32_t* n_hi, const int32_t* n_hc, int64_t n_lines,
                                    const uint64_t* item_keys, const int32_t* item_ids,
                                    int64_t item_capacity, const uint64_t* cat_keys,
                                    const int32_t* cat_ids, int64_t cat_capacity,
                                    int32_t* cat_of_item, void* workspace, size_t ws_bytes,
                                    void* stream) {
  RS_CHECK_ARG(n_lines >= 0 && item_capacity >= 2 && (item_capacity & (item_capacity - 1)) == 0 &&
                   cat_capacity >= 2 && (cat_capacity & (cat_capacity - 1)) == 0,
               "rs_dien_item_cat: bad arguments");
  hipStream_t st = as_stream(stream);
  Carver c(workspace, ws_bytes);
  unsigned long long* last = c.take<unsigned long long>(item_capacity);
  uint64_t* slot_cat = c.take<uint64_t>(item_capacity);
  if (!c.ok()) {
    set_error("rs_dien_item_cat: workspace too small");
    return RS_E_WORKSPACE;
  }
  // last[h] = 1 + the stream position of the item's latest pair (0: none)
  RS_CHECK_HIP(hipMemsetAsync(last, 0, sizeof(unsigned long long) * item_capacity, st));
  if (n_lines > 0) {
    for (int pass = 0; pass < 2; ++pass) {
      dien_pairs_kernel<<<(unsigned)ceil_div(n_lines, 4), 256, 0, st>>>(
          item_hash, cat_hash, item_off, cat_off, n_hi, n_hc, n_lines, item_keys,
          (uint32_t)(item_capacity - 1), pass, last, slot_cat);
      RS_CHECK_LAUNCH();
    }
  }
  dien_cat_map_kernel<<<grid256(item_capacity), 256, 0, st>>>(
      item_keys, item_ids, item_capacity, last, slot_cat, cat_keys, cat_ids,
      (uint32_t)(cat_capacity - 1), cat_of_item);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_dien_encode(const uint64_t* item_hash, const uint64_t* cat_hash,
                                  const int64_t* item_off, const int64_t* cat_off,
                                  const int32_t* n_hi, const int32_t* n_hc, int64_t n_lines,
                                  const uint64_t* item_keys, const int32_t* item_ids,
                                  int64_t item_capacity, int32_t unk_item, const uint64_t* cat_keys,
                                  const int32_t* cat_ids, int64_t cat_capacity, int32_t maxlen,
                                  const int32_t* cat_of_item, int32_t n_item_ids, uint64_t seed,
                                  int64_t line_base, int32_t* target_item, int32_t* target_cat,
                                  int32_t* his_item, int32_t* his_cat, int32_t* neg_item,
                                  int32_t* neg_cat, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(n_lines >= 0 && maxlen >= 1 && item_capacity >= 2 &&
                   (item_capacity & (item_capacity - 1)) == 0 && cat_capacity >= 2 &&
                   (cat_capacity & (cat_capacity - 1)) == 0 &&
                   (!neg_item || (neg_cat && cat_of_item && n_item_ids >= 2)),
               "rs_dien_encode: bad arguments");
  if (n_lines == 0) return RS_OK;
  DienTables tb{item_keys, item_ids, (uint32_t)(item_capacity - 1), unk_item,
                cat_keys,  cat_ids,  (uint32_t)(cat_capacity - 1)};
  dien_encode_kernel<<<(unsigned)ceil_div(n_lines, 4), 256, 0, as_stream(stream)>>>(
      item_hash, cat_hash, item_off, cat_off, n_hi, n_hc, n_lines, tb, maxlen, cat_of_item,
      n_item_ids, seed, line_base, target_item, target_cat, his_item, his_cat, neg_item, neg_cat,
      err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
