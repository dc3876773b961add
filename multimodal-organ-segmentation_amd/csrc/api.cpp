// C-ABI plumbing shared by every entry point: error reporting and version.
// No exception crosses the ABI; every entry point returns 0 or 1 and the
// message of the last failure on this thread is kept for mmseg_last_error().
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

namespace mmseg {
static thread_local char g_err[1024] = {0};
static thread_local const char* g_kernel = "";

void note_kernel(const char* name) { g_kernel = name; }

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return 1;
  }
  return 0;
}
}  // namespace mmseg

extern "C" {
const char* mmseg_last_error(void) { return mmseg::g_err; }
const char* mmseg_last_kernel(void) { return mmseg::g_kernel; }
int mmseg_abi_version(void) { return 1; }
}
