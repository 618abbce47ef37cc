// Error reporting + device queries for the C ABI.
#include <stdarg.h>
#include "common.h"

namespace {
thread_local char g_err[1024] = "";
}

namespace mia {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code < 0 ? code : -1;
}
int cu_count() {
  static int ncu = 0;  // every device of the node is the same part
  if (!ncu) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      ncu = n;
    else
      ncu = 256;
  }
  return ncu;
}
}  // namespace mia

extern "C" const char* mia_last_error_string(void) { return g_err; }

extern "C" int mia_device_arch(char* buf, int32_t len) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return mia::fail(-(int)e, "hipGetDevice: %s", hipGetErrorString(e));
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return mia::fail(-(int)e, "hipGetDeviceProperties: %s", hipGetErrorString(e));
  snprintf(buf, (size_t)len, "%s", prop.gcnArchName);
  return 0;
}
