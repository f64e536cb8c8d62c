// common.hpp — shared helpers for the gfx950 kernels behind include/recsys_hip.h.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/recsys_hip.h"

namespace rs {

// ---- host-side error reporting (thread-local, see rs_last_error) --------------------
void set_error(const char* fmt, ...);

#define RS_CHECK_ARG(cond, ...)        \
  do {                                 \
    if (!(cond)) {                     \
      ::rs::set_error(__VA_ARGS__);    \
      return RS_E_INVALID;             \
    }                                  \
  } while (0)

#define RS_CHECK_HIP(expr)                                                              \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      ::rs::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
      return RS_E_HIP;                                                                  \
    }                                                                                   \
  } while (0)

// after a kernel launch: catch launch-configuration errors without synchronising
#define RS_CHECK_LAUNCH() RS_CHECK_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t a, size_t b) { return (a + b - 1) / b * b; }

// workspace carving: 256-B aligned sub-buffers
struct Carver {
  char* base;
  size_t off = 0;
  size_t cap;
  Carver(void* p, size_t c) : base(static_cast<char*>(p)), cap(c) {}
  template <typename T>
  T* take(size_t n) {
    off = align_up(off, 256);
    T* r = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += n * sizeof(T);
    return r;
  }
  bool ok() const { return off <= cap; }
};

// ---- device helpers ------------------------------------------------------------------
constexpr int kWave = 64;

__device__ __forceinline__ int64_t load_id(const void* ids, int32_t dtype, int64_t i) {
  return dtype == RS_ID_I64 ? static_cast<const int64_t*>(ids)[i]
                            : static_cast<int64_t>(static_cast<const int32_t*>(ids)[i]);
}

// Global row of the id at flattened position p (slot = p % n_slots). Returns -1 if the id
// is outside its table (TF-GPU: zero row, SURVEY §8.1 "OOB ids").
__device__ __forceinline__ int64_t global_row(const void* ids, int32_t dtype, int64_t p,
                                              const int64_t* slot_offsets, int32_t n_slots,
                                              int64_t n_rows) {
  int64_t id = load_id(ids, dtype, p);
  if (slot_offsets) {
    int s = static_cast<int>(p % n_slots);
    int64_t lo = slot_offsets[s], hi = slot_offsets[s + 1];
    if (id < 0 || id >= hi - lo) return -1;
    return lo + id;
  }
  if (id < 0 || id >= n_rows) return -1;
  return id;
}

__device__ __forceinline__ void flag_oob(int32_t* err_flag) {
  if (err_flag) atomicOr(err_flag, RS_ERRBIT_OOB);
}

}  // namespace rs
