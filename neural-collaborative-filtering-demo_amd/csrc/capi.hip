// C-ABI plumbing: version, thread-local error string.
#include <stdarg.h>
#include "ncf_common.h"

static thread_local char g_err[512] = "";

void ncf_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* ncf_last_error(void) { return g_err; }

extern "C" int ncf_version(void) { return 10000; }  // 1.0.0

// Sanity probe used by the loader: returns the HIP device count seen by the runtime the
// library is bound to (torch's libamdhip64 when torch is imported first).
extern "C" int ncf_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
