// C-ABI support: error reporting and version query for libgsplat_hip.so.
// Every entry point returns 0 on success, 1 on an argument error and 2 on a
// HIP launch error; gsplat_hip_last_error() gives the message (thread-local).
#include <stdarg.h>
#include <stdio.h>

namespace gs {
static thread_local char g_err[512] = {0};

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace gs

extern "C" const char *gsplat_hip_last_error(void) { return gs::g_err; }

// Bumped whenever an entry point's signature changes.
extern "C" int gsplat_hip_abi_version(void) { return 35; }
