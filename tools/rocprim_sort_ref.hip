// A/B reference only (not product code): rocPRIM's device radix sort of (key, position) pairs,
// to price the engine's rs_sort_ids against the library's onesweep sort on the same keys.
// Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/rocprim_sort_ref.hip -o tools/librocprim_sort_ref.so
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

extern "C" size_t ref_sort_ws(int64_t n, int end_bit) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                            (const int32_t*)nullptr, (int32_t*)nullptr, (unsigned)n, 0, end_bit);
  return bytes;
}

extern "C" int ref_sort_pairs(const uint32_t* kin, uint32_t* kout, const int32_t* vin, int32_t* vout,
                              int64_t n, int end_bit, void* ws, size_t ws_bytes, void* stream) {
  size_t bytes = ws_bytes;
  return (int)rocprim::radix_sort_pairs(ws, bytes, kin, kout, vin, vout, (unsigned)n, 0, end_bit,
                                        (hipStream_t)stream);
}
