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
