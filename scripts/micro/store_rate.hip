// Diagnostic micro-benchmark (not part of the product): the HBM write rate
// of a pure 16-byte-per-lane store stream with the grid stream's shape
// (vox_stream_kernel: every workgroup writes whole 256 KB items, one 1 KB
// wave-instruction at a time, buffer stores with cache policy AUX), as a
// function of workgroups, store waves per workgroup and policy.  Each launch
// writes TOTAL bytes into one of NBUF buffers in turn (the Infinity Cache
// (256 MiB) cannot hold a buffer, so every launch writes HBM), back to back
// on one stream; HIP events around REPS launches.
//   hipcc -O3 --offload-arch=gfx950 store_rate.hip -o store_rate && ./store_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr size_t TOTAL = 283ull << 20;  // ~ the c2 grid stream's bytes per launch
constexpr int NBUF = 4;
constexpr int REPS = 40;
constexpr int ITEM = 256 << 10;  // bytes per item (two channels of a 32^3 grid)

// workgroup g writes items g, g + G, ... ; its W waves sweep each item in
// 1 KB wave-instructions (lane l: bytes 16 l .. 16 l + 15 of the KB)
template <int AUX>
__global__ void k_store(char* buf, int nitems, int per_wave_unroll) {
  const int W = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(buf + (size_t)it * ITEM, (short)0, ITEM,
                                                      0x00020000);
    for (int kb = w; kb < ITEM / 1024; kb += W)
      __builtin_amdgcn_raw_buffer_store_b128(z, rs, kb * 1024 + lane * 16, 0, AUX);
  }
}

int main() {
  char* bufs[NBUF];
  for (int i = 0; i < NBUF; i++)
    if (hipMalloc(&bufs[i], TOTAL) != hipSuccess) return 1;
  const int nitems = (int)(TOTAL / ITEM);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct Cfg {
    int wgs, waves, aux;
  };
  const Cfg cfgs[] = {{256, 4, 16}, {256, 4, 0},  {256, 4, 2},  {256, 8, 16}, {256, 8, 0},
                      {512, 4, 16}, {512, 8, 16}, {1024, 4, 16}, {1024, 4, 0}, {2048, 4, 16},
                      {256, 16, 16}, {512, 4, 0}};
  for (const Cfg& c : cfgs) {
    auto launch = [&](int i) {
      char* b = bufs[i % NBUF];
      if (c.aux == 16)
        hipLaunchKernelGGL(k_store<16>, dim3(c.wgs), dim3(c.waves * 64), 0, 0, b, nitems, 0);
      else if (c.aux == 2)
        hipLaunchKernelGGL(k_store<2>, dim3(c.wgs), dim3(c.waves * 64), 0, 0, b, nitems, 0);
      else
        hipLaunchKernelGGL(k_store<0>, dim3(c.wgs), dim3(c.waves * 64), 0, 0, b, nitems, 0);
    };
    for (int i = 0; i < 8; i++) launch(i);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < REPS; i++) launch(i);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / REPS;
    printf("wgs %5d  waves/wg %2d  aux %2d  %7.1f us per launch  %.2f TB/s\n", c.wgs, c.waves,
           c.aux, us, (double)TOTAL / (us * 1e-6) / 1e12);
  }
  // the same buffer every launch (what an "alone" loop over one output set measures)
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < REPS; i++)
    hipLaunchKernelGGL(k_store<16>, dim3(256), dim3(256), 0, 0, bufs[0], nitems, 0);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("same buffer, wgs 256 waves 4 aux 16: %.1f us per launch  %.2f TB/s\n", ms * 1e3 / REPS,
         (double)TOTAL / (ms * 1e-3 / REPS) / 1e12);
  return 0;
}
