// runtime.cpp -- error reporting and version of libpcr_amd.so.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "common.hpp"

namespace pcr {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

pcr_status launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
    return PCR_ERR_LAUNCH;
  }
  return PCR_OK;
}

}  // namespace pcr

extern "C" const char* pcr_last_error(void) { return pcr::g_err; }

extern "C" const char* pcr_version(void) { return "pcr_amd 0.1.0 gfx950"; }
