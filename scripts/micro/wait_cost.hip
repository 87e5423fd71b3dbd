// Diagnostic micro-benchmark (not part of the product): queue time of a
// cross-stream dependency whose producer completed long ago.  Stream A runs
// N short kernels back to back; between consecutive kernels it waits on
//   none      -- nothing (baseline)
//   event     -- hipStreamWaitEvent on an event recorded (and completed) on
//                stream B before the loop (sync event flags as the runner's)
//   value     -- hipStreamWaitValue32 on a device word already >= 1
//   record    -- an event record on A itself (no wait)
// and reports the wall time per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void spin(float* p, int iters) {
  float v = p[threadIdx.x];
  for (int i = 0; i < iters; i++) v = v * 0.999f + 0.001f;
  if (v == 12345.0f) p[threadIdx.x] = v;
}

int main() {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  float* buf;
  CK(hipMalloc(&buf, 4096));
  CK(hipMemset(buf, 0, 4096));
  unsigned* flag;
  CK(hipMalloc((void**)&flag, 64));
  CK(hipMemset(flag, 0, 64));
  hipEvent_t done, rec, t0, t1;
  CK(hipEventCreateWithFlags(&done, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&rec, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, b, buf, 100);
  CK(hipEventRecord(done, b));
  CK(hipStreamWriteValue32(b, flag, 1, 0));
  CK(hipStreamSynchronize(b));
  const int N = 200;
  const char* names[4] = {"none", "event", "value", "record"};
  for (int rep = 0; rep < 2; rep++) {
    for (int mode = 0; mode < 4; mode++) {
      CK(hipStreamSynchronize(a));
      CK(hipEventRecord(t0, a));
      for (int i = 0; i < N; i++) {
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, buf, 2000);
        if (mode == 1) CK(hipStreamWaitEvent(a, done, 0));
        if (mode == 2) CK(hipStreamWaitValue32(a, flag, 1, hipStreamWaitValueGte, 0xFFFFFFFFu));
        if (mode == 3) CK(hipEventRecord(rec, a));
      }
      CK(hipEventRecord(t1, a));
      CK(hipEventSynchronize(t1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, t0, t1));
      if (rep == 1) printf("%-7s %7.2f us per kernel\n", names[mode], ms * 1000.0f / N);
    }
  }
  return 0;
}
