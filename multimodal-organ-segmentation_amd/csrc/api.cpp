// C-ABI plumbing shared by every entry point: error reporting and version.
// No exception crosses the ABI; every entry point returns 0 or 1 and the
// message of the last failure on this thread is kept for mmseg_last_error().
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/mmseg_hip.h"

#include <vector>

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

// launch timing: one process drives one GPU from one host thread (mmseg_hip.h conventions)
static bool g_timing = false;
static std::vector<hipEvent_t> g_tev;        // start / stop pairs, reused across windows
static std::vector<const char*> g_tname;     // the launch site's kernel expression (a string literal)
static long long g_tn = 0;

bool timing_on() { return g_timing; }

void timing_events(const char* name, hipEvent_t* start, hipEvent_t* stop) {
  if ((size_t)(2 * g_tn + 2) > g_tev.size()) {
    hipEvent_t a = nullptr, b = nullptr;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
      *start = *stop = nullptr;                // untimed launch (the kernel still runs)
      return;
    }
    g_tev.push_back(a);
    g_tev.push_back(b);
  }
  if ((size_t)g_tn >= g_tname.size()) g_tname.resize(g_tn + 1);
  g_tname[g_tn] = name;
  *start = g_tev[2 * g_tn];
  *stop = g_tev[2 * g_tn + 1];
  ++g_tn;
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

int mmseg_timing_begin(void) {
  mmseg::g_tn = 0;
  mmseg::g_timing = true;
  return 0;
}
int mmseg_timing_end(void) {
  mmseg::g_timing = false;
  return 0;
}
long long mmseg_timing_count(void) { return mmseg::g_tn; }
int mmseg_timing_get(long long i, float* ms, const char** name) {
  if (i < 0 || i >= mmseg::g_tn) {
    mmseg::set_error("mmseg_timing_get: launch %lld of %lld", i, mmseg::g_tn);
    return 1;
  }
  *name = mmseg::g_tname[i];
  hipError_t e = hipEventElapsedTime(ms, mmseg::g_tev[2 * i], mmseg::g_tev[2 * i + 1]);
  if (e != hipSuccess) {
    mmseg::set_error("mmseg_timing_get: %s", hipGetErrorString(e));
    return 1;
  }
  return 0;
}
}
