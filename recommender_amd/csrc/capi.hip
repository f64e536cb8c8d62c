// capi.hip — library-level entry points of librecsys_hip.so (error reporting, version).
#include <cstring>

#include "common.hpp"

namespace rs {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

}  // namespace rs

extern "C" const char* rs_last_error(void) { return rs::g_last_error; }

extern "C" int32_t rs_version(void) { return 1; }

extern "C" int32_t rs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

namespace rs {
// STREAM copy: the HBM-bandwidth reference the roofline reports beside the spec peak (SURVEY
// §8(d) "also report measured STREAM-copy bandwidth"): one 16-byte load and store per thread, a
// grid over the whole buffer. Measured against its variants (tools/microbench_copy.hip, one
// box): this shape 6.24 TB/s, the same with 4 / 8 / 16 float4 per thread 4.4 / 4.0 / 3.8, a
// 2048-block grid-stride loop 4.7, hipMemcpy D2D 4.5.
__global__ __launch_bounds__(256) void stream_copy_kernel(const float4* __restrict__ src,
                                                          float4* __restrict__ dst, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) dst[i] = src[i];
}
}  // namespace rs

extern "C" int32_t rs_stream_copy(const void* src, void* dst, size_t bytes, void* stream) {
  RS_CHECK_ARG(bytes % 16 == 0, "bytes must be a multiple of 16");
  if (bytes == 0) return RS_OK;
  RS_CHECK_ARG(src && dst, "null pointer");
  RS_CHECK_ARG(reinterpret_cast<uintptr_t>(src) % 16 == 0 && reinterpret_cast<uintptr_t>(dst) % 16 == 0,
               "16-byte aligned buffers only");
  const int64_t n4 = (int64_t)(bytes / 16);
  RS_CHECK_ARG(n4 <= (int64_t)256 * 0x7fffffff, "buffer too large for one launch");
  rs::stream_copy_kernel<<<(unsigned)rs::ceil_div(n4, 256), 256, 0, rs::as_stream(stream)>>>(
      static_cast<const float4*>(src), static_cast<float4*>(dst), n4);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

// Device-scope stream ordering (round 6). A default HIP event's record performs a system-scope
// release (cache write-back / invalidate for host visibility); ordering two streams of ONE device
// needs only a device-scope one. These events are created with hipEventDisableSystemFence and are
// used only to order the engine's own streams (never for host synchronisation or across devices
// or processes).
extern "C" void* rs_event_create(void) {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
    rs::set_error("hipEventCreateWithFlags failed");
    return nullptr;
  }
  return e;
}

extern "C" int32_t rs_event_destroy(void* ev) {
  if (ev && hipEventDestroy(static_cast<hipEvent_t>(ev)) != hipSuccess) {
    rs::set_error("hipEventDestroy failed");
    return RS_E_HIP;
  }
  return RS_OK;
}

extern "C" int32_t rs_event_record(void* ev, void* stream) {
  RS_CHECK_ARG(ev, "null event");
  if (hipEventRecord(static_cast<hipEvent_t>(ev), rs::as_stream(stream)) != hipSuccess) {
    rs::set_error("hipEventRecord failed");
    return RS_E_HIP;
  }
  return RS_OK;
}

extern "C" int32_t rs_stream_wait_event(void* stream, void* ev) {
  RS_CHECK_ARG(ev, "null event");
  if (hipStreamWaitEvent(rs::as_stream(stream), static_cast<hipEvent_t>(ev), 0) != hipSuccess) {
    rs::set_error("hipStreamWaitEvent failed");
    return RS_E_HIP;
  }
  return RS_OK;
}
