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

// A stream whose kernels run only on the CUs set in `mask` (nwords 32-bit
// words, bit i = CU i in the runtime's CU numbering), e.g. to keep the
// HBM-bound grid stream and the VALU-bound KNN chain on disjoint CUs.
extern "C" pcr_status pcr_stream_create_cu_mask(const unsigned* mask, int nwords, void** out) {
  PCR_REQUIRE(mask != nullptr && nwords >= 1 && out != nullptr,
              "stream_create_cu_mask: invalid arguments");
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask);
  if (e != hipSuccess) {
    pcr::set_error("stream_create_cu_mask: %s", hipGetErrorString(e));
    return PCR_ERR_LAUNCH;
  }
  *out = s;
  return PCR_OK;
}

extern "C" pcr_status pcr_stream_destroy(void* stream) {
  PCR_REQUIRE(stream != nullptr, "stream_destroy: NULL stream");
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  if (e != hipSuccess) {
    pcr::set_error("stream_destroy: %s", hipGetErrorString(e));
    return PCR_ERR_LAUNCH;
  }
  return PCR_OK;
}
