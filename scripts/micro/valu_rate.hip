// Diagnostic micro-benchmark (not part of the product): how many shader
// cycles one wave64 VALU instruction occupies a SIMD on gfx950, with
// independent instruction chains, as a function of the waves per SIMD.
//
// Each kernel runs ITER x 64 instructions per wave in 16 independent chains
// (no instruction waits on its predecessor's result for 15 issues).  The
// in-kernel clock is measured, not assumed: every wave stamps s_memtime
// (shader clock) and s_memrealtime (100 MHz) around its loop, so
//   clock  = d(memtime) / d(memrealtime) * 100 MHz            (median wave)
//   cyc/instr per SIMD = kernel wall time * clock / (instructions per SIMD)
// with the wall time from HIP events.  The launches put W waves on every
// SIMD (256 CUs x W workgroups of 4 waves; a workgroup's 4 waves land on the
// CU's 4 SIMDs).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int ITER = 2048;
constexpr int NCH = 16;
typedef float pf2 __attribute__((ext_vector_type(2)));

struct Stamp {
  unsigned long long t0, t1, r0, r1;
};

#define STAMP_BEGIN                                      \
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(); \
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#define STAMP_END(st)                                                            \
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();                    \
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();                \
  if ((threadIdx.x & 63) == 0) {                                                 \
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);                           \
    st[w] = Stamp{t0, t1, r0, r1};                                               \
  }

__global__ __launch_bounds__(256) void k_fma(float* out, Stamp* st, float s) {
  float a[NCH];
  for (int i = 0; i < NCH; i++) a[i] = s + i;
  STAMP_BEGIN
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int r = 0; r < 64 / NCH; r++)
#pragma unroll
      for (int i = 0; i < NCH; i++) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
  }
  STAMP_END(st)
  float t = 0;
  for (int i = 0; i < NCH; i++) t += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_pk_fma(float* out, Stamp* st, float s) {
  pf2 a[NCH];
  for (int i = 0; i < NCH; i++) a[i] = pf2{s + i, s - i};
  const pf2 m = pf2{s, s * 0.5f};
  STAMP_BEGIN
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int r = 0; r < 64 / NCH; r++)
#pragma unroll
      for (int i = 0; i < NCH; i++) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(m));
  }
  STAMP_END(st)
  float t = 0;
  for (int i = 0; i < NCH; i++) t += a[i][0] + a[i][1];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_add_u32(float* out, Stamp* st, float s) {
  unsigned a[NCH];
  const unsigned m = (unsigned)s;
  for (int i = 0; i < NCH; i++) a[i] = m + i;
  STAMP_BEGIN
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int r = 0; r < 64 / NCH; r++)
#pragma unroll
      for (int i = 0; i < NCH; i++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
  }
  STAMP_END(st)
  unsigned t = 0;
  for (int i = 0; i < NCH; i++) t += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = (float)t;
}

// v_cmp (writes an SGPR pair) followed by v_cndmask reading it: the pair a
// count or a select per element costs
__global__ __launch_bounds__(256) void k_cmp_cnd(float* out, Stamp* st, float s) {
  float a[NCH];
  for (int i = 0; i < NCH; i++) a[i] = s + i;
  STAMP_BEGIN
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int r = 0; r < 32 / NCH; r++)
#pragma unroll
      for (int i = 0; i < NCH; i++)
        asm volatile(
            "v_cmp_lt_f32 vcc, %0, %1\n\t"
            "v_cndmask_b32 %0, %0, %1, vcc"
            : "+v"(a[i])
            : "v"(s)
            : "vcc");
  }
  STAMP_END(st)
  float t = 0;
  for (int i = 0; i < NCH; i++) t += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

// one 32-bit-register instruction "OP %0, %0, %1" in 16 independent chains
#define K32(NAME, ASM)                                                              \
  __global__ __launch_bounds__(256) void NAME(float* out, Stamp* st, float s) {    \
    float a[NCH];                                                                   \
    for (int i = 0; i < NCH; i++) a[i] = s + i;                                     \
    STAMP_BEGIN                                                                     \
    for (int it = 0; it < ITER; it++) {                                             \
      _Pragma("unroll") for (int r = 0; r < 64 / NCH; r++)                          \
      _Pragma("unroll") for (int i = 0; i < NCH; i++)                               \
        asm volatile(ASM : "+v"(a[i]) : "v"(s));                                    \
    }                                                                               \
    STAMP_END(st)                                                                   \
    float t = 0;                                                                    \
    for (int i = 0; i < NCH; i++) t += a[i];                                        \
    out[blockIdx.x * 256 + threadIdx.x] = t;                                        \
  }
// the same on 64-bit register pairs
#define K64(NAME, ASM)                                                              \
  __global__ __launch_bounds__(256) void NAME(float* out, Stamp* st, float s) {    \
    double a[NCH];                                                                  \
    const double m = (double)s;                                                     \
    for (int i = 0; i < NCH; i++) a[i] = m + i;                                     \
    STAMP_BEGIN                                                                     \
    for (int it = 0; it < ITER; it++) {                                             \
      _Pragma("unroll") for (int r = 0; r < 64 / NCH; r++)                          \
      _Pragma("unroll") for (int i = 0; i < NCH; i++)                               \
        asm volatile(ASM : "+v"(a[i]) : "v"(m));                                    \
    }                                                                               \
    STAMP_END(st)                                                                   \
    double t = 0;                                                                   \
    for (int i = 0; i < NCH; i++) t += a[i];                                        \
    out[blockIdx.x * 256 + threadIdx.x] = (float)t;                                 \
  }
K32(k_add_f32, "v_add_f32 %0, %0, %1")
K32(k_mul_f32, "v_mul_f32 %0, %0, %1")
K32(k_min_f32, "v_min_f32 %0, %0, %1")
K32(k_lshr, "v_lshrrev_b32 %0, 3, %0")
K32(k_med3, "v_med3_i32 %0, %0, %1, 7")
K32(k_mbcnt, "v_mbcnt_lo_u32_b32 %0, -1, %0")
K32(k_dpp, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
K32(k_dpp_add, "v_add_u32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
K32(k_cmpu, "v_cmp_lt_u32 vcc, %0, %1")
K32(k_min_u32, "v_min_u32 %0, %0, %1")
K32(k_max_u32, "v_max_u32 %0, %0, %1")
K32(k_min_dpp, "v_min_u32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
K32(k_lshl_add, "v_lshl_add_u32 %0, %0, 2, %1")
K32(k_and, "v_and_b32 %0, %0, %1")
K32(k_bfe, "v_bfe_u32 %0, %0, 3, 5")
K32(k_sub_f32, "v_sub_f32 %0, %1, %0")
K32(k_cnd_s, "v_cndmask_b32_e64 %0, %0, %1, s[4:5]")
K32(k_cmp_s, "v_cmp_le_u32_e64 s[4:5], %0, %1")
K64(k_pk_add, "v_pk_add_f32 %0, %0, %1")
K64(k_pk_mul, "v_pk_mul_f32 %0, %0, %1")
K64(k_min_f64, "v_min_f64 %0, %0, %1")
K64(k_cmp_u64, "v_cmp_lt_u64 vcc, %0, %1")

template <typename K>
void run(const char* name, K kern, float* d, Stamp* st, int W) {
  const int wgs = 256 * W;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(kern, dim3(wgs), dim3(256), 0, 0, d, st, 1.0f);
  (void)hipEventRecord(e0, 0);
  const int reps = 5;
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, dim3(wgs), dim3(256), 0, 0, d, st, 1.0f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  std::vector<Stamp> h(wgs * 4);
  (void)hipMemcpy(h.data(), st, h.size() * sizeof(Stamp), hipMemcpyDeviceToHost);
  std::vector<double> clk, cyc;
  for (const Stamp& x : h) {
    clk.push_back((double)(x.t1 - x.t0) / (double)(x.r1 - x.r0) * 100e6);
    cyc.push_back((double)(x.t1 - x.t0));
  }
  std::sort(clk.begin(), clk.end());
  std::sort(cyc.begin(), cyc.end());
  const double ghz = clk[clk.size() / 2] / 1e9;
  const double per_simd = (double)W * ITER * 64;  // wave-instructions per SIMD
  const double cpi_wall = ms * 1e-3 * ghz * 1e9 / per_simd;
  // one wave's loop in its own cycles, divided by its instructions and
  // multiplied by the W waves sharing the SIMD: the SIMD's cycles per
  // instruction while all W are in their loops
  const double cpi_wave = cyc[cyc.size() / 2] / (ITER * 64.0) / W;
  printf("%-9s W=%d  %8.3f ms  clock %.2f GHz  cyc/instr per SIMD: %.2f (wall) %.2f (in-loop)\n",
         name, W, ms, ghz, cpi_wall, cpi_wave);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

int main() {
  float* d;
  Stamp* st;
  const int maxw = 8;
  (void)hipMalloc(&d, (size_t)256 * maxw * 256 * 4);
  (void)hipMalloc(&st, (size_t)256 * maxw * 4 * sizeof(Stamp));
  for (int W : {4}) {
    run("fma", k_fma, d, st, W);
    run("pk_fma", k_pk_fma, d, st, W);
    run("add_u32", k_add_u32, d, st, W);
    run("cmp+cnd", k_cmp_cnd, d, st, W);
    if (W < 2) continue;
    run("add_f32", k_add_f32, d, st, W);
    run("mul_f32", k_mul_f32, d, st, W);
    run("min_f32", k_min_f32, d, st, W);
    run("lshr", k_lshr, d, st, W);
    run("med3_i32", k_med3, d, st, W);
    run("mbcnt_lo", k_mbcnt, d, st, W);
    run("mov_dpp", k_dpp, d, st, W);
    run("add_dpp", k_dpp_add, d, st, W);
    run("cmp_u32", k_cmpu, d, st, W);
    run("min_u32", k_min_u32, d, st, W);
    run("max_u32", k_max_u32, d, st, W);
    run("min_dpp", k_min_dpp, d, st, W);
    run("lshl_add", k_lshl_add, d, st, W);
    run("and_b32", k_and, d, st, W);
    run("bfe_u32", k_bfe, d, st, W);
    run("sub_f32", k_sub_f32, d, st, W);
    run("cnd_sgpr", k_cnd_s, d, st, W);
    run("cmp_sgpr", k_cmp_s, d, st, W);
    run("pk_add", k_pk_add, d, st, W);
    run("pk_mul", k_pk_mul, d, st, W);
    run("min_f64", k_min_f64, d, st, W);
    run("cmp_u64", k_cmp_u64, d, st, W);
  }
  (void)hipFree(d);
  (void)hipFree(st);
  return 0;
}
