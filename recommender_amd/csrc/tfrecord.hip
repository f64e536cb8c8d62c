// tfrecord.hip — the reference's Criteo TFRecord files read into device batches (SURVEY §8f
// rank 1, second half; reference ctr/tfrecord_io.py:39-96).
//
// Wire format (public specs; TensorFlow is not in this image):
//   TFRecord   per record: uint64 length, uint32 masked CRC32C(length), data, uint32 masked
//              CRC32C(data); masked(c) = ((c >> 15) | (c << 17)) + 0xa282ead8.
//   data       a tf.train.Example protobuf: Example.features (1) → Features.feature (1, a map:
//              entries {key (1): string, value (2): Feature}) → Feature.bytes_list (1) /
//              float_list (2) / int64_list (3), each {value (1): repeated}.
//   features   'int_features' / 'cat_features': one bytes value = tf.io.serialize_tensor of a
//              float32 [13] / int64 [26] array — a TensorProto {dtype (1), tensor_shape (2) {dim
//              (2) {size (1)}}, tensor_content (4) raw little-endian}; 'label': int64_list.
//
// Framing (host, rs_tfrecord_index): a sequential walk over the length prefixes (each record's
// offset depends on every earlier length) that checks the length CRCs; it yields the record
// offsets. Parsing (device, rs_tfrecord_parse_criteo): one wave per record stages the record in
// LDS (coalesced byte loads), lane 0 walks the protobuf (varints, nested lengths, any field
// order, unknown fields skipped, packed or unpacked int64 lists) and optionally checks the
// record's data CRC32C with an LDS table; then the lanes copy the tensors out. A malformed
// record gets zero features and sets bit RS_ERRBIT_FORMAT of err_flag.
#include <cstring>

#include "common.hpp"

namespace rs {

constexpr uint32_t kCrcMaskDelta = 0xa282ead8u;
constexpr int kRecMax = 4096;  // bytes of one Example staged per wave

// CRC32C (Castagnoli, reflected polynomial 0x82F63B78)
__host__ __device__ constexpr uint32_t crc32c_table_entry(uint32_t i) {
  uint32_t c = i;
  for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
  return c;
}

static uint32_t host_crc_table[256];
static bool host_crc_ready = false;

static void host_crc_init() {
  if (host_crc_ready) return;
  for (uint32_t i = 0; i < 256; ++i) host_crc_table[i] = crc32c_table_entry(i);
  host_crc_ready = true;
}

static uint32_t host_crc32c(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = host_crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

__host__ __device__ __forceinline__ uint32_t mask_crc(uint32_t c) {
  return ((c >> 15) | (c << 17)) + kCrcMaskDelta;
}

static uint64_t load_le64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
static uint32_t load_le32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

// ---- device protobuf walking (lane 0, over the LDS image of one record) ----------------------
struct Cursor {
  const uint8_t* b;
  int pos, end;
  bool ok;
};

__device__ __forceinline__ uint64_t rd_varint(Cursor& c) {
  uint64_t v = 0;
  for (int sh = 0; sh < 64; sh += 7) {
    if (c.pos >= c.end) {
      c.ok = false;
      return 0;
    }
    const uint8_t byte = c.b[c.pos++];
    v |= (uint64_t)(byte & 0x7F) << sh;
    if (!(byte & 0x80)) return v;
  }
  c.ok = false;
  return 0;
}

// skip one field's payload of wire type wt
__device__ __forceinline__ void skip_field(Cursor& c, uint32_t wt) {
  if (wt == 0) {
    rd_varint(c);
  } else if (wt == 1) {
    c.pos += 8;
  } else if (wt == 2) {
    const uint64_t n = rd_varint(c);
    if (n > (uint64_t)(c.end - c.pos)) {
      c.ok = false;
      return;
    }
    c.pos += (int)n;
  } else if (wt == 5) {
    c.pos += 4;
  } else {
    c.ok = false;
  }
  if (c.pos > c.end) c.ok = false;
}

// a length-delimited field's body as a sub-cursor
__device__ __forceinline__ Cursor sub(Cursor& c) {
  const uint64_t n = rd_varint(c);
  if (!c.ok || n > (uint64_t)(c.end - c.pos)) {
    c.ok = false;
    return Cursor{c.b, c.pos, c.pos, false};
  }
  Cursor s{c.b, c.pos, c.pos + (int)n, true};
  c.pos += (int)n;
  return s;
}

__device__ __forceinline__ bool key_is(const Cursor& k, const char* s, int n) {
  if (k.end - k.pos != n) return false;
  for (int i = 0; i < n; ++i)
    if (k.b[k.pos + i] != (uint8_t)s[i]) return false;
  return true;
}

// TensorProto: dtype must be `want_dtype`, shape [want_n] (or a scalar-free 1-D shape of that
// size); returns the byte offset of tensor_content (size want_n * elem) in the record, or -1.
// float_val (5) / int64_val (10) packed forms are accepted too (content offset then marks the
// packed run and `content_len` its byte length; `packed` is set).
__device__ int parse_tensor(Cursor t, int want_dtype, int want_n, int elem, bool& packed,
                            int& content_len) {
  int dtype = -1, content = -1, dims = 0;
  int64_t size = -1;
  packed = false;
  content_len = 0;
  while (t.ok && t.pos < t.end) {
    const uint64_t tag = rd_varint(t);
    const uint32_t f = (uint32_t)(tag >> 3), wt = (uint32_t)(tag & 7);
    if (f == 1 && wt == 0) {
      dtype = (int)rd_varint(t);
    } else if (f == 2 && wt == 2) {  // TensorShapeProto
      Cursor sh = sub(t);
      while (sh.ok && sh.pos < sh.end) {
        const uint64_t st = rd_varint(sh);
        if ((st >> 3) == 2 && (st & 7) == 2) {  // Dim
          Cursor d = sub(sh);
          ++dims;
          while (d.ok && d.pos < d.end) {
            const uint64_t dt = rd_varint(d);
            if ((dt >> 3) == 1 && (dt & 7) == 0) size = (int64_t)rd_varint(d);
            else skip_field(d, (uint32_t)(dt & 7));
          }
          if (!d.ok) sh.ok = false;
        } else {
          skip_field(sh, (uint32_t)(st & 7));
        }
      }
      if (!sh.ok) t.ok = false;
    } else if (f == 4 && wt == 2) {  // tensor_content
      const uint64_t n = rd_varint(t);
      if (n != (uint64_t)want_n * elem || n > (uint64_t)(t.end - t.pos)) return -1;
      content = t.pos;
      content_len = (int)n;
      t.pos += (int)n;
    } else if (((f == 5 && want_dtype == 1) || (f == 10 && want_dtype == 9)) && wt == 2) {
      // float_val (fixed 4-byte values, the tensor_content bytes) / int64_val (varints), packed
      const uint64_t n = rd_varint(t);
      if (n > (uint64_t)(t.end - t.pos) || (f == 5 && n != (uint64_t)want_n * 4)) return -1;
      content = t.pos;
      content_len = (int)n;
      packed = f == 10;
      t.pos += (int)n;
    } else {
      skip_field(t, wt);
    }
  }
  if (!t.ok || dtype != want_dtype || dims != 1 || size != want_n || content < 0) return -1;
  return content;
}

// Feature (bytes_list with one value) → the value's body as a cursor
__device__ __forceinline__ Cursor feature_bytes(Cursor f) {
  Cursor none{f.b, 0, 0, false};
  while (f.ok && f.pos < f.end) {
    const uint64_t tag = rd_varint(f);
    if ((tag >> 3) == 1 && (tag & 7) == 2) {  // bytes_list
      Cursor bl = sub(f);
      while (bl.ok && bl.pos < bl.end) {
        const uint64_t bt = rd_varint(bl);
        if ((bt >> 3) == 1 && (bt & 7) == 2) return sub(bl);
        skip_field(bl, (uint32_t)(bt & 7));
      }
      return none;
    }
    skip_field(f, (uint32_t)(tag & 7));
  }
  return none;
}

// Feature (int64_list with one value, packed or not)
__device__ __forceinline__ bool feature_int64(Cursor f, int64_t& out) {
  while (f.ok && f.pos < f.end) {
    const uint64_t tag = rd_varint(f);
    if ((tag >> 3) == 3 && (tag & 7) == 2) {  // int64_list
      Cursor il = sub(f);
      while (il.ok && il.pos < il.end) {
        const uint64_t it = rd_varint(il);
        if ((it >> 3) == 1 && (it & 7) == 2) {  // packed
          Cursor pk = sub(il);
          out = (int64_t)rd_varint(pk);
          return pk.ok;
        }
        if ((it >> 3) == 1 && (it & 7) == 0) {
          out = (int64_t)rd_varint(il);
          return il.ok;
        }
        skip_field(il, (uint32_t)(it & 7));
      }
      return false;
    }
    skip_field(f, (uint32_t)(tag & 7));
  }
  return false;
}

struct CriteoOut {
  float* dense;     // [n, n_int]
  int64_t* cat;     // [n, n_cat]
  int64_t* label;   // [n]
  int n_int, n_cat;
};

__global__ __launch_bounds__(256) void tfrecord_criteo_kernel(
    const uint8_t* __restrict__ data, const int64_t* __restrict__ offs,
    const int32_t* __restrict__ lens, int64_t n_rec, int32_t verify_crc, CriteoOut o,
    int32_t* err_flag) {
  __shared__ uint8_t rec[4][kRecMax];
  __shared__ uint32_t crc_tab[256];
  __shared__ int meta[4][6];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (verify_crc)
    for (int i = threadIdx.x; i < 256; i += 256) crc_tab[i] = crc32c_table_entry((uint32_t)i);
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= n_rec) return;
  const int len = lens[r];
  const uint8_t* src = data + offs[r] + 12;  // past the length and its CRC
  const bool fits = len >= 0 && len <= kRecMax;
  if (fits)
    for (int i = lane; i < len; i += 64) rec[wave][i] = src[i];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (lane == 0) {
    bool ok = fits;
    int dense_at = -1, cat_at = -1, dense_len = 0, cat_len = 0;
    bool dense_pk = false, cat_pk = false;
    int64_t label = 0;
    bool have_label = false;
    if (ok && verify_crc) {
      uint32_t c = 0xFFFFFFFFu;
      for (int i = 0; i < len; ++i) c = crc_tab[(c ^ rec[wave][i]) & 0xFF] ^ (c >> 8);
      uint32_t stored;
      const uint8_t* sc = src + len;
      stored = (uint32_t)sc[0] | ((uint32_t)sc[1] << 8) | ((uint32_t)sc[2] << 16) | ((uint32_t)sc[3] << 24);
      ok = mask_crc(c ^ 0xFFFFFFFFu) == stored;
    }
    Cursor ex{rec[wave], 0, fits ? len : 0, ok};
    while (ex.ok && ex.pos < ex.end) {
      const uint64_t tag = rd_varint(ex);
      if ((tag >> 3) == 1 && (tag & 7) == 2) {  // Features
        Cursor fs = sub(ex);
        while (fs.ok && fs.pos < fs.end) {
          const uint64_t ft = rd_varint(fs);
          if ((ft >> 3) == 1 && (ft & 7) == 2) {  // map entry
            Cursor e = sub(fs);
            Cursor key{e.b, 0, 0, false}, val{e.b, 0, 0, false};
            while (e.ok && e.pos < e.end) {
              const uint64_t et = rd_varint(e);
              if ((et >> 3) == 1 && (et & 7) == 2) key = sub(e);
              else if ((et >> 3) == 2 && (et & 7) == 2) val = sub(e);
              else skip_field(e, (uint32_t)(et & 7));
            }
            if (!e.ok || !key.ok || !val.ok) {
              fs.ok = false;
              break;
            }
            if (key_is(key, "int_features", 12)) {
              Cursor t = feature_bytes(val);
              if (t.ok) dense_at = parse_tensor(t, 1 /*DT_FLOAT*/, o.n_int, 4, dense_pk, dense_len);
            } else if (key_is(key, "cat_features", 12)) {
              Cursor t = feature_bytes(val);
              if (t.ok) cat_at = parse_tensor(t, 9 /*DT_INT64*/, o.n_cat, 8, cat_pk, cat_len);
            } else if (key_is(key, "label", 5)) {
              have_label = feature_int64(val, label);
            }
          } else {
            skip_field(fs, (uint32_t)(ft & 7));
          }
        }
        if (!fs.ok) ex.ok = false;
      } else {
        skip_field(ex, (uint32_t)(tag & 7));
      }
    }
    ok = ok && ex.ok && dense_at >= 0 && cat_at >= 0 && have_label;
    // packed float_val: fixed 4-byte values, same bytes as tensor_content; packed int64_val:
    // varints (decoded below by lane 0)
    meta[wave][0] = ok ? 1 : 0;
    meta[wave][1] = dense_at;
    meta[wave][2] = cat_at;
    meta[wave][3] = cat_pk ? 1 : 0;
    meta[wave][4] = (int)(label & 0xFFFFFFFF);
    meta[wave][5] = (int)(label >> 32);
    if (ok && cat_pk) {  // varint-packed int64_val: exactly n_cat varints filling the field
      Cursor pk{rec[wave], cat_at, cat_at + cat_len, true};
      for (int i = 0; i < o.n_cat; ++i) {
        const int64_t v = (int64_t)rd_varint(pk);
        o.cat[r * o.n_cat + i] = pk.ok ? v : 0;
      }
      if (!pk.ok || pk.pos != pk.end) {
        meta[wave][0] = 0;
        for (int i = 0; i < o.n_cat; ++i) o.cat[r * o.n_cat + i] = 0;
      }
    }
    if (!meta[wave][0] && err_flag) atomicOr(err_flag, RS_ERRBIT_FORMAT);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const bool ok = meta[wave][0] != 0;
  const int dense_at = meta[wave][1], cat_at = meta[wave][2];
  const bool cat_pk = meta[wave][3] != 0;
  if (lane < o.n_int) {
    float v = 0.f;
    if (ok) {
      const uint8_t* p = rec[wave] + dense_at + 4 * lane;
      const uint32_t u = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
      v = __uint_as_float(u);
    }
    o.dense[r * o.n_int + lane] = v;
  }
  if (lane < o.n_cat && !(ok && cat_pk)) {
    int64_t v = 0;
    if (ok) {
      const uint8_t* p = rec[wave] + cat_at + 8 * lane;
      uint64_t u = 0;
      for (int k = 7; k >= 0; --k) u = (u << 8) | p[k];
      v = (int64_t)u;
    }
    o.cat[r * o.n_cat + lane] = v;
  }
  if (lane == 0)
    o.label[r] = ok ? (int64_t)(((uint64_t)(uint32_t)meta[wave][5] << 32) | (uint32_t)meta[wave][4]) : 0;
}

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_crc32c_masked(const uint8_t* data, int64_t n_bytes, uint32_t* out) {
  RS_CHECK_ARG(out && n_bytes >= 0 && (n_bytes == 0 || data), "bad arguments");
  host_crc_init();
  *out = mask_crc(host_crc32c(data, (size_t)n_bytes));
  return RS_OK;
}

extern "C" int32_t rs_tfrecord_index(const uint8_t* data, int64_t n_bytes, int32_t verify_crc,
                                     int64_t* offsets, int32_t* lengths, int64_t capacity,
                                     int64_t* n_records) {
  RS_CHECK_ARG(n_bytes >= 0 && capacity >= 0 && n_records, "bad arguments");
  RS_CHECK_ARG(n_bytes == 0 || data, "data is null");
  host_crc_init();
  int64_t pos = 0, n = 0;
  while (pos < n_bytes) {
    if (n_bytes - pos < 16) {  // length (8) + its CRC (4) + the data CRC (4) at the least
      set_error("truncated TFRecord header at byte %lld", (long long)pos);
      return RS_E_INVALID;
    }
    const uint64_t len = load_le64(data + pos);
    if (verify_crc && mask_crc(host_crc32c(data + pos, 8)) != load_le32(data + pos + 8)) {
      set_error("TFRecord length CRC mismatch at byte %lld", (long long)pos);
      return RS_E_INVALID;
    }
    if (len > 0x7FFFFFFFull || (int64_t)len > n_bytes - pos - 16) {
      set_error("TFRecord length %llu at byte %lld runs past the data", (unsigned long long)len,
                (long long)pos);
      return RS_E_INVALID;
    }
    if (n < capacity) {
      if (offsets) offsets[n] = pos;
      if (lengths) lengths[n] = (int32_t)len;
    }
    ++n;
    pos += 16 + (int64_t)len;
  }
  *n_records = n;
  if (n > capacity && (offsets || lengths)) {
    set_error("%lld records, capacity %lld", (long long)n, (long long)capacity);
    return RS_E_WORKSPACE;
  }
  return RS_OK;
}

extern "C" int32_t rs_tfrecord_parse_criteo(const uint8_t* data, const int64_t* offsets,
                                            const int32_t* lengths, int64_t n_records,
                                            int32_t n_int, int32_t n_cat, int32_t verify_crc,
                                            float* int_features, int64_t* cat_features,
                                            int64_t* label, int32_t* err_flag, void* stream) {
  RS_CHECK_ARG(n_records >= 0 && n_int >= 0 && n_int <= 64 && n_cat >= 0 && n_cat <= 64,
               "bad sizes (at most 64 features of each kind)");
  if (n_records == 0) return RS_OK;
  RS_CHECK_ARG(data && offsets && lengths && int_features && cat_features && label, "null pointer");
  CriteoOut o{int_features, cat_features, label, n_int, n_cat};
  tfrecord_criteo_kernel<<<ceil_div(n_records, 4), 256, 0, as_stream(stream)>>>(
      data, offsets, lengths, n_records, verify_crc, o, err_flag);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
