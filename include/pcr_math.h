/*
 * pcr_math.h -- bit-exact scalar math shared by the HIP kernels (device) and
 * the CPU oracle (host C).  Every function here is a fixed sequence of IEEE-754
 * operations that are correctly rounded on both x86-64 and gfx950 (add, mul,
 * div, sqrt, fma, floor, conversions), so host and device produce identical
 * bits for identical inputs.  Both sides MUST be compiled with
 * -ffp-contract=off: every fused multiply-add the reference's nvcc build is
 * assumed to contract is written out explicitly with fmaf()/fma().
 *
 * Why a private acos/atan: the reference calls CUDA's float acos/atan
 * (spherical_vox.cu:46,54; spherical_trilinear_devox.cu:58,62) and double acos
 * (ppf.cu:62-64).  glibc, OCML and CUDA libm disagree in the last ulp, and one
 * ulp on a spherical angle can move a point across a voxel-bin edge.  We use a
 * double-precision polynomial (max rel. error ~1e-17, fitted with mpmath; see
 * oracle/fit_math.py) rounded once to float, i.e. a correctly rounded acosf /
 * atanf except in ~1e-9 of double-rounding cases.  Against genuine sm_61
 * output the voxel index can differ only for points whose pre-floor bin value
 * sits within a few ulp of an integer (flagged by the oracle).
 *
 * The FMA-contraction convention ("nvcc-FMA") follows LLVM's DAG combine for
 * (a*b + c*d) + e*f:  fma(e, f, fma(a, b, c*d)).
 */
#ifndef PCR_MATH_H
#define PCR_MATH_H

#if defined(__HIP__)
#define PCR_HD static inline __host__ __device__
#else
#define PCR_HD static inline
#endif

/* acos(-1.0) in double: the reference's `#define PI acos(-1.0)`
 * (spherical_vox.cu:5, spherical_trilinear_devox.cu:5). */
#define PCR_PI 3.141592653589793115997963468544185161590576171875
#define PCR_PIO2 1.5707963267948965579989817342720925807952880859375
#define PCR_PIO4 0.78539816339744827899949086713604629039764404296875
#define PCR_TAN_PI8 0.41421356237309503

/* KNN "undefined" sentinel, knn.cuh:3 (UNDEFINE_VALUE 10000). */
#define PCR_KNN_UNDEF 10000.0f

/* ---- conversions with CUDA/AMD hardware semantics (cvt.rzi / v_cvt_i32):
 * truncate toward zero, saturate, NaN -> 0.  Plain C (int) of NaN is UB. ---- */
PCR_HD int pcr_f2i(float v) {
  if (v != v) return 0;
  if (v >= 2147483648.0f) return 2147483647;
  if (v <= -2147483648.0f) return (-2147483647 - 1);
  return (int)v;
}
PCR_HD int pcr_d2i(double v) {
  if (v != v) return 0;
  if (v >= 2147483648.0) return 2147483647;
  if (v <= -2147483649.0) return (-2147483647 - 1);
  return (int)v;
}

/* NaN-ignoring min/max with CUDA fmin/fmax semantics (used by ppf.cu:38,62). */
PCR_HD double pcr_fmax_d(double a, double b) {
  if (a != a) return b;
  if (b != b) return a;
  return a > b ? a : b;
}
PCR_HD double pcr_fmin_d(double a, double b) {
  if (a != a) return b;
  if (b != b) return a;
  return a < b ? a : b;
}

/* ---- contracted sums of products (nvcc-FMA convention) ---- */
/* x*x + y*y + z*z  -> fma(z, z, fma(x, x, y*y)) */
PCR_HD float pcr_sumsq3f(float x, float y, float z) {
  return __builtin_fmaf(z, z, __builtin_fmaf(x, x, y * y));
}
/* uncontracted variant, only used by the oracle to flag FMA-sensitive elements */
PCR_HD float pcr_sumsq3f_nofma(float x, float y, float z) {
  float a = x * x;
  float b = y * y;
  float c = z * z;
  float s = a + b;
  return s + c;
}
/* a0*b0 + a1*b1 + a2*b2 */
PCR_HD float pcr_dot3f(float a0, float a1, float a2, float b0, float b1, float b2) {
  return __builtin_fmaf(a2, b2, __builtin_fmaf(a0, b0, a1 * b1));
}
/* w0*f0 + w1*f1 + ... + w7*f7 (trilinear_devox.cu:73-77 as nvcc contracts it) */
PCR_HD float pcr_wsum8(const float w[8], const float f[8]) {
  float acc = w[1] * f[1];
  acc = __builtin_fmaf(w[0], f[0], acc);
  acc = __builtin_fmaf(w[2], f[2], acc);
  acc = __builtin_fmaf(w[3], f[3], acc);
  acc = __builtin_fmaf(w[4], f[4], acc);
  acc = __builtin_fmaf(w[5], f[5], acc);
  acc = __builtin_fmaf(w[6], f[6], acc);
  acc = __builtin_fmaf(w[7], f[7], acc);
  return acc;
}

/* ---- double-precision asin/acos/atan kernels (Horner, explicit fma) ---- */
/* asin(s) = s + s*z*P(z), z = s*s, |s| <= 0.5; P fitted on z in [0, 0.25] */
PCR_HD double pcr_asin_core(double s) {
  double z = s * s;
  double p = 0.03207412686712179;
  p = __builtin_fma(p, z, -0.029288652492291928);
  p = __builtin_fma(p, z, 0.026492027340877928);
  p = __builtin_fma(p, z, -0.0027168811083041495);
  p = __builtin_fma(p, z, 0.00874110307727393);
  p = __builtin_fma(p, z, 0.006869444870499221);
  p = __builtin_fma(p, z, 0.008452406065746546);
  p = __builtin_fma(p, z, 0.009755275316163535);
  p = __builtin_fma(p, z, 0.011552268573915126);
  p = __builtin_fma(p, z, 0.013964819214172544);
  p = __builtin_fma(p, z, 0.017352765309284954);
  p = __builtin_fma(p, z, 0.022372159069960183);
  p = __builtin_fma(p, z, 0.03038194444474315);
  p = __builtin_fma(p, z, 0.04464285714285491);
  p = __builtin_fma(p, z, 0.07500000000000001);
  p = __builtin_fma(p, z, 0.16666666666666666);
  return __builtin_fma(s * z, p, s);
}

/* atan(t) = t + t*z*Q(z), z = t*t, |t| <= tan(pi/8) */
PCR_HD double pcr_atan_core(double t) {
  double z = t * t;
  double q = -0.01391822929102443;
  q = __builtin_fma(q, z, 0.030635704112969498);
  q = __builtin_fma(q, z, -0.04104436265755082);
  q = __builtin_fma(q, z, 0.04719395030027433);
  q = __builtin_fma(q, z, -0.05258041554297779);
  q = __builtin_fma(q, z, 0.058819252531928636);
  q = __builtin_fma(q, z, -0.06666642020055166);
  q = __builtin_fma(q, z, 0.07692306736000173);
  q = __builtin_fma(q, z, -0.0909090906700999);
  q = __builtin_fma(q, z, 0.11111111110754729);
  q = __builtin_fma(q, z, -0.14285714285711518);
  q = __builtin_fma(q, z, 0.19999999999999993);
  q = __builtin_fma(q, z, -0.3333333333333333);
  return __builtin_fma(t * z, q, t);
}

PCR_HD double pcr_acos_d(double x) {
  /* three ranges, evaluated without branches (one polynomial, one sqrt):
   *   |x| <= 0.5:  pi/2 - asin(x)
   *   x > 0.5:     2 asin(sqrt((1 - x) / 2))
   *   x < -0.5:    pi - 2 asin(sqrt((1 + x) / 2))   (also the NaN path)
   * 1 - |x| is exactly the 1 - x resp. 1 + x of the branches. */
  double ax = __builtin_fabs(x);
  int mid = ax <= 0.5;
  double s = mid ? x : __builtin_sqrt((1.0 - ax) * 0.5);
  double p = pcr_asin_core(s);
  return mid ? PCR_PIO2 - p : (x > 0.0 ? 2.0 * p : PCR_PI - 2.0 * p);
}

PCR_HD double pcr_atan_d(double x) {
  double a = __builtin_fabs(x);
  int inv = 0;
  double base = 0.0, t, r;
  if (a > 1.0) {
    a = 1.0 / a;
    inv = 1;
  }
  if (a > PCR_TAN_PI8) {
    t = (a - 1.0) / (a + 1.0);
    base = PCR_PIO4;
  } else {
    t = a;
  }
  r = base + pcr_atan_core(t);
  if (inv) r = PCR_PIO2 - r;
  return (x < 0.0) ? -r : r;
}

/* float acos/atan of the reference (CUDA float overloads), rounded once */
PCR_HD float pcr_acosf(float x) { return (float)pcr_acos_d((double)x); }

/* Faithful fp32 acos (error <= ~2 ulp, checked against float64 acos in
 * tests/test_oracle_kat.py) for the local PPF: the reference evaluates it
 * with torch.acos on fp32 tensors (pvcnn_classify.py:264-266), itself not
 * correctly rounded, and the PPF angles carry a 1e-5 tolerance; the voxel
 * bins keep the correctly rounded pcr_acosf.  asin(s) = s + s z P(z), z = s^2,
 * |s| <= 0.5 (cephes asinf coefficients); the same three ranges as
 * pcr_acos_d, without branches; pi/2 and pi split into hi + lo. */
PCR_HD float pcr_asinf_core(float s) {
  float z = s * s;
  float p = __builtin_fmaf(4.2163199048e-2f, z, 2.4181311049e-2f);
  p = __builtin_fmaf(p, z, 4.5470025998e-2f);
  p = __builtin_fmaf(p, z, 7.4953002686e-2f);
  p = __builtin_fmaf(p, z, 1.6666752422e-1f);
  return __builtin_fmaf(s * z, p, s);
}

PCR_HD float pcr_acosf_fast(float x) {
  const float pio2_hi = 1.57079637e+00f, pio2_lo = -4.37113883e-08f;
  const float pi_hi = 3.14159274e+00f, pi_lo = -8.74227766e-08f;
  float ax = __builtin_fabsf(x);
  int mid = ax <= 0.5f;
  float s = mid ? x : __builtin_sqrtf((1.0f - ax) * 0.5f);
  float p = pcr_asinf_core(s);
  return mid ? pio2_hi - (p - pio2_lo) : (x > 0.0f ? 2.0f * p : pi_hi - (2.0f * p - pi_lo));
}
PCR_HD float pcr_atanf(float x) { return (float)pcr_atan_d((double)x); }

/* ---- spherical coordinates of a normalised point (spherical_vox.cu:34-56,
 * spherical_trilinear_devox.cu:48-65).  Returns 0 when the reference drops
 * the point (gama==0, gama>=1, |z/gama|>1, beta>=PI), else 1. ---- */
PCR_HD int pcr_sph_coords(float x, float y, float z, int r, int use_fma,
                          float *gama_o, float *alpha_o, float *beta_o) {
  float g2 = use_fma ? pcr_sumsq3f(x, y, z) : pcr_sumsq3f_nofma(x, y, z);
  float gama = __builtin_sqrtf(g2);
  float beta, alpha;
  if ((gama == 0.0f) || (gama >= 1.0f) || ((z / gama) > 1.0f) || ((z / gama) < -1.0f))
    return 0;
  beta = pcr_acosf(z / gama);
  if ((double)beta >= PCR_PI) return 0;
  if (x == 0.0f && y != 0.0f)
    alpha = (float)((double)(y / __builtin_fabsf(y)) * PCR_PI * 0.5);
  else if (x == 0.0f && y == 0.0f)
    alpha = 0.0f;
  else
    alpha = (float)((double)pcr_atanf(y / x) +
                    PCR_PI * (double)(1.0f - (x / __builtin_fabsf(x))) / 2.0);
  alpha = (float)((double)alpha + PCR_PI / (double)r);
  if (alpha < 0.0f) alpha = (float)((double)alpha + 2.0 * PCR_PI);
  *gama_o = gama;
  *alpha_o = alpha;
  *beta_o = beta;
  return 1;
}

/* voxel index of a normalised point, -1 when dropped (spherical_vox.cu:59-65) */
PCR_HD int pcr_sph_index_v(float x, float y, float z, int r, int use_fma) {
  float gama, alpha, beta;
  int gx, gy, gz;
  if (!pcr_sph_coords(x, y, z, r, use_fma, &gama, &alpha, &beta)) return -1;
  gx = pcr_f2i(__builtin_floorf(gama * (float)r));
  gy = pcr_d2i(__builtin_floor((double)((alpha * (float)r) / 2.0f) / PCR_PI));
  gz = pcr_d2i(__builtin_floor((double)(beta * (float)r) / PCR_PI));
  if (gx >= r) gx = r - 1;
  if (gy >= r) gy = r - 1;
  if (gz >= r) gz = r - 1;
  return gx * r * r + gy * r + gz;
}
PCR_HD int pcr_sph_index(float x, float y, float z, int r) {
  return pcr_sph_index_v(x, y, z, r, 1);
}

/* ---- spherical "trilinear" corners (spherical_trilinear_devox.cu:67-105),
 * quirks preserved: integer division gama_lo = (pos/r2)/r == 0, radian-valued
 * alpha/beta fractions, (int) of radian values.  Returns 0 when the point is
 * dropped by the recomputed coordinates (the reference then writes nothing). */
PCR_HD int pcr_sph_corners(float x, float y, float z, int pos, int r, int idx[8], float w[8]) {
  float gama, alpha, beta;
  int r2 = r * r;
  int gg, ga, gb, glo, alo, blo, ghi, ahi, bhi;
  float glo_f, alo_f, blo_f, gd1, ad1, bd1, gd0, ad0, bd0;
  if (!pcr_sph_coords(x, y, z, r, 1, &gama, &alpha, &beta)) return 0;
  gg = pos / r2;
  ga = (pos - gg * r2) / r;
  gb = pos - gg * r2 - ga * r;
  glo_f = (float)(gg / r);
  alo_f = (float)(PCR_PI * 2.0 * (double)ga / (double)r);
  blo_f = (float)(PCR_PI * (double)gb / (double)r);
  gd1 = gama - glo_f;
  ad1 = alpha - alo_f;
  bd1 = beta - blo_f;
  gd0 = 1.0f - gd1;
  ad0 = 1.0f - ad1;
  bd0 = 1.0f - bd1;
  w[0] = gd0 * ad0 * bd0;
  w[1] = gd0 * ad0 * bd1;
  w[2] = gd0 * ad1 * bd0;
  w[3] = gd0 * ad1 * bd1;
  w[4] = gd1 * ad0 * bd0;
  w[5] = gd1 * ad0 * bd1;
  w[6] = gd1 * ad1 * bd0;
  w[7] = gd1 * ad1 * bd1;
  glo = pcr_f2i(glo_f);
  alo = pcr_f2i(alo_f);
  blo = pcr_f2i(blo_f);
  ghi = (gd1 > 0.0f) ? -1 : 0;
  ahi = (ad1 > 0.0f) ? -1 : 0;
  bhi = (bd1 > 0.0f) ? 1 : 0;
  idx[0] = glo * r2 + alo * r + blo;
  idx[1] = idx[0] + bhi;
  idx[2] = idx[0] + (ahi & r);
  idx[3] = idx[2] + bhi;
  idx[4] = idx[0] + (ghi & r2);
  idx[5] = idx[4] + bhi;
  idx[6] = idx[4] + (ahi & r);
  idx[7] = idx[6] + bhi;
  return 1;
}

/* voxel index (pcr_sph_index) and spherical corners (pcr_sph_corners of that
 * index) of one point from ONE evaluation of its spherical coordinates: both
 * functions recompute pcr_sph_coords from the same (x, y, z), so this is
 * bit-identical to calling them in turn, at half the fp64 trig.  Returns the
 * index (-1 when dropped); *corners_ok = pcr_sph_corners' return value (0
 * for a dropped point). */
PCR_HD int pcr_sph_index_corners(float x, float y, float z, int r, int idx[8], float w[8],
                                 int *corners_ok) {
  float gama, alpha, beta;
  int gx, gy, gz, pos, r2 = r * r;
  int gg, ga, gb, glo, alo, blo, ghi, ahi, bhi;
  float glo_f, alo_f, blo_f, gd1, ad1, bd1, gd0, ad0, bd0;
  *corners_ok = 0;
  if (!pcr_sph_coords(x, y, z, r, 1, &gama, &alpha, &beta)) return -1;
  /* pcr_sph_index_v */
  gx = pcr_f2i(__builtin_floorf(gama * (float)r));
  gy = pcr_d2i(__builtin_floor((double)((alpha * (float)r) / 2.0f) / PCR_PI));
  gz = pcr_d2i(__builtin_floor((double)(beta * (float)r) / PCR_PI));
  if (gx >= r) gx = r - 1;
  if (gy >= r) gy = r - 1;
  if (gz >= r) gz = r - 1;
  pos = gx * r * r + gy * r + gz;
  /* pcr_sph_corners(x, y, z, pos, r) after its pcr_sph_coords */
  gg = pos / r2;
  ga = (pos - gg * r2) / r;
  gb = pos - gg * r2 - ga * r;
  glo_f = (float)(gg / r);
  alo_f = (float)(PCR_PI * 2.0 * (double)ga / (double)r);
  blo_f = (float)(PCR_PI * (double)gb / (double)r);
  gd1 = gama - glo_f;
  ad1 = alpha - alo_f;
  bd1 = beta - blo_f;
  gd0 = 1.0f - gd1;
  ad0 = 1.0f - ad1;
  bd0 = 1.0f - bd1;
  w[0] = gd0 * ad0 * bd0;
  w[1] = gd0 * ad0 * bd1;
  w[2] = gd0 * ad1 * bd0;
  w[3] = gd0 * ad1 * bd1;
  w[4] = gd1 * ad0 * bd0;
  w[5] = gd1 * ad0 * bd1;
  w[6] = gd1 * ad1 * bd0;
  w[7] = gd1 * ad1 * bd1;
  glo = pcr_f2i(glo_f);
  alo = pcr_f2i(alo_f);
  blo = pcr_f2i(blo_f);
  ghi = (gd1 > 0.0f) ? -1 : 0;
  ahi = (ad1 > 0.0f) ? -1 : 0;
  bhi = (bd1 > 0.0f) ? 1 : 0;
  idx[0] = glo * r2 + alo * r + blo;
  idx[1] = idx[0] + bhi;
  idx[2] = idx[0] + (ahi & r);
  idx[3] = idx[2] + bhi;
  idx[4] = idx[0] + (ghi & r2);
  idx[5] = idx[4] + bhi;
  idx[6] = idx[4] + (ahi & r);
  idx[7] = idx[6] + bhi;
  *corners_ok = 1;
  return pos;
}

/* ---- cube trilinear corners (trilinear_devox.cu:45-80) on continuous
 * voxel coordinates already clamped to [0, r-1] ---- */
PCR_HD void pcr_cube_corners(float x, float y, float z, int r, int idx[8], float w[8]) {
  int r2 = r * r;
  float xl = __builtin_floorf(x), yl = __builtin_floorf(y), zl = __builtin_floorf(z);
  float xd1 = x - xl, yd1 = y - yl, zd1 = z - zl;
  float xd0 = 1.0f - xd1, yd0 = 1.0f - yd1, zd0 = 1.0f - zd1;
  int xlo = pcr_f2i(xl), ylo = pcr_f2i(yl), zlo = pcr_f2i(zl);
  int xhi = (xd1 > 0.0f) ? -1 : 0;
  int yhi = (yd1 > 0.0f) ? -1 : 0;
  int zhi = (zd1 > 0.0f) ? 1 : 0;
  w[0] = xd0 * yd0 * zd0;
  w[1] = xd0 * yd0 * zd1;
  w[2] = xd0 * yd1 * zd0;
  w[3] = xd0 * yd1 * zd1;
  w[4] = xd1 * yd0 * zd0;
  w[5] = xd1 * yd0 * zd1;
  w[6] = xd1 * yd1 * zd0;
  w[7] = xd1 * yd1 * zd1;
  idx[0] = xlo * r2 + ylo * r + zlo;
  idx[1] = idx[0] + zhi;
  idx[2] = idx[0] + (yhi & r);
  idx[3] = idx[2] + zhi;
  idx[4] = idx[0] + (xhi & r2);
  idx[5] = idx[4] + zhi;
  idx[6] = idx[4] + (yhi & r);
  idx[7] = idx[6] + zhi;
}

/* 1.0 / (float)cnt narrowed to float (spherical_vox.cu:112, vox.cu:67) */
PCR_HD float pcr_inv_count(int cnt) { return (float)(1.0 / (double)(float)cnt); }

/* ---- point-pair feature of one (point, centre) pair (ppf.cu:37-90).
 * out = {a1, a2, a3, d_norm}; all zero when either normal is ~0. ---- */
PCR_HD void pcr_global_ppf(float x, float y, float z, float cx, float cy, float cz,
                           float nx, float ny, float nz, float cnx, float cny,
                           float cnz, float out[4]) {
  float dx = cx - x, dy = cy - y, dz = cz - z;
  float s = __builtin_sqrtf(pcr_sumsq3f(dx, dy, dz));
  float dn = (float)pcr_fmax_d((double)s, 1e-20);
  float n1, n2;
  dx /= dn;
  dy /= dn;
  dz /= dn;
  n1 = __builtin_sqrtf(pcr_sumsq3f(cnx, cny, cnz));
  n2 = __builtin_sqrtf(pcr_sumsq3f(nx, ny, nz));
  if ((double)n2 <= 1e-10 || (double)n1 <= 1e-10) {
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    return;
  }
  cnx /= n1;
  cny /= n1;
  cnz /= n1;
  nx /= n2;
  ny /= n2;
  nz /= n2;
  out[0] = (float)pcr_acos_d(pcr_fmax_d(pcr_fmin_d((double)pcr_dot3f(dx, dy, dz, cnx, cny, cnz), 1.0), -1.0));
  out[1] = (float)pcr_acos_d(pcr_fmax_d(pcr_fmin_d((double)pcr_dot3f(dx, dy, dz, nx, ny, nz), 1.0), -1.0));
  out[2] = (float)pcr_acos_d(pcr_fmax_d(pcr_fmin_d((double)pcr_dot3f(cnx, cny, cnz, nx, ny, nz), 1.0), -1.0));
  out[3] = dn;
}

/* torch.clamp(v, -1, 1) on float: NaN propagates */
PCR_HD float pcr_clamp1f(float v) {
  if (v != v) return v;
  return v < -1.0f ? -1.0f : (v > 1.0f ? 1.0f : v);
}

/* ---- local (k-neighbour) PPF of the model (pvcnn_classify.py:261-269).
 * g = grouped neighbour minus centre as BallQuery returns it
 * (modules/ball_query.py:24); d = c - g (the model's 2c - p quirk when
 * relative != 0), else d = c - p.  out = {nr_d, ni_d, nr_ni, |d|}. ---- */
PCR_HD void pcr_local_ppf(float cx, float cy, float cz, float cnx, float cny, float cnz,
                          float px, float py, float pz, float pnx, float pny, float pnz,
                          int relative, float out[4]) {
  float gx = relative ? px - cx : px;
  float gy = relative ? py - cy : py;
  float gz = relative ? pz - cz : pz;
  float dx = cx - gx, dy = cy - gy, dz = cz - gz;
  float dn = __builtin_sqrtf(pcr_sumsq3f(dx, dy, dz));
  float ux = dx / dn, uy = dy / dn, uz = dz / dn;
  out[0] = pcr_acosf_fast(pcr_clamp1f(pcr_dot3f(pnx, pny, pnz, ux, uy, uz)));
  out[1] = pcr_acosf_fast(pcr_clamp1f(pcr_dot3f(cnx, cny, cnz, ux, uy, uz)));
  out[2] = pcr_acosf_fast(pcr_clamp1f(pcr_dot3f(pnx, pny, pnz, cnx, cny, cnz)));
  out[3] = dn;
}

/* ---- feature-space mutual nearest neighbours (datasets/deepgmr_mn40.py:
 * 232-244, find_correspondence_one_pair).  numpy computes, in fp32,
 *   diff = norm(f1)^2 + norm(f2)^2.T - 2 f1 . f2.T
 * with BLAS-order sums; here every sum over channels is the k-ordered fmaf
 * chain an fp32 MFMA produces (acc = fma(a_k, b_k, acc), k ascending), so the
 * device and this restatement agree bit for bit. ---- */
/* norm(f)^2 as np.power(np.linalg.norm(f), 2): sqrt of the sum, squared */
PCR_HD float pcr_match_sqnorm(const float *f, int c) {
  float s = 0.0f, r;
  int k;
  for (k = 0; k < c; k++) s = __builtin_fmaf(f[k], f[k], s);
  r = __builtin_sqrtf(s);
  return r * r;
}
/* (sq1 + sq2) - 2 dot, the broadcast order of the numpy expression */
PCR_HD float pcr_match_diff(float sq1, float sq2, float dot) {
  return (sq1 + sq2) - 2.0f * dot;
}
/* ascending-unsigned key of (diff, index): np.argmin's order -- the least
 * value, the first index among equal ones, NaN before everything (argmin
 * returns the first NaN); -0 and +0 compare equal */
PCR_HD unsigned long long pcr_match_key(float v, int idx) {
  unsigned u;
  float w = v + 0.0f; /* -0 -> +0 */
  __builtin_memcpy(&u, &w, 4);
  if (v != v)
    u = 0u;
  else
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned)idx;
}

/* ---- furthest point sampling (sampling/sampling.cu:87-173).  Each sample
 * step keeps min(d, dist) per point and picks the farthest point.  The
 * reference's 512 threads each take points t, t+512, ... and keep the first
 * strict maximum; the LDS tree keeps the left entry on ties.  The winner is
 * therefore the largest d2, then the smallest k % 512, then the smallest k.
 * This key orders exactly that way under an unsigned max (d2 >= 0). ---- */
PCR_HD unsigned long long pcr_fps_key(float d2, int k) {
  unsigned u, rank = ((unsigned)(k & 511) << 22) | ((unsigned)k >> 9);
  __builtin_memcpy(&u, &d2, 4);
  return ((unsigned long long)u << 32) | (unsigned)(0xFFFFFFFFu - rank);
}
PCR_HD int pcr_fps_key_index(unsigned long long key) {
  unsigned rank = 0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull);
  return (int)(((rank & 0x3FFFFFu) << 9) | (rank >> 22));
}

/* ---- three nearest neighbours (interpolate/neighbor_interpolate.cu:21-76).
 * The reference keeps best0..2 in double, but they only ever hold fp32
 * distances or the 1e40 init.  Its clamp and the double products of two
 * floats rounded back to float equal fp32 min/max and multiplies. So the
 * weights are computed in fp32 here, with +inf for "no centre yet". ---- */
PCR_HD void pcr_three_nn_insert(float d, int k, float best[3], int besti[3]) {
  if (d < best[2]) {
    best[2] = d;
    besti[2] = k;
    if (d < best[1]) {
      best[2] = best[1];
      besti[2] = besti[1];
      best[1] = d;
      besti[1] = k;
      if (d < best[0]) {
        best[1] = best[0];
        besti[1] = besti[0];
        best[0] = d;
        besti[0] = k;
      }
    }
  }
}
PCR_HD void pcr_three_nn_weights(const float best[3], float w[3]) {
  float b0 = best[0] < 1e10f ? best[0] : 1e10f;
  float b1 = best[1] < 1e10f ? best[1] : 1e10f;
  float b2 = best[2] < 1e10f ? best[2] : 1e10f;
  float d0d1, d0d2, d1d2, inv;
  b0 = b0 > 1e-10f ? b0 : 1e-10f;
  b1 = b1 > 1e-10f ? b1 : 1e-10f;
  b2 = b2 > 1e-10f ? b2 : 1e-10f;
  d0d1 = b0 * b1;
  d0d2 = b0 * b2;
  d1d2 = b1 * b2;
  inv = 1.0f / ((d0d1 + d0d2) + d1d2);
  w[0] = d1d2 * inv;
  w[1] = d0d2 * inv;
  w[2] = d0d1 * inv;
}
/* f1*w1 + f2*w2 + f3*w3 (neighbor_interpolate.cu:112-114, nvcc-FMA) */
PCR_HD float pcr_wsum3(float f0, float w0, float f1, float w1, float f2, float w2) {
  return __builtin_fmaf(f2, w2, __builtin_fmaf(f0, w0, f1 * w1));
}

/* ---- LRF "change_coords" (models/pvcnn_classify.py:153-184).  PyTorch
 * elementwise ops do not contract, so the basis arithmetic below is unfused.
 * Rank order is descending norm, ties by ascending index (the reference's
 * unstable argsort leaves ties open). ---- */
PCR_HD float pcr_norm3f(float x, float y, float z) {
  return __builtin_sqrtf(pcr_sumsq3f_nofma(x, y, z));
}
PCR_HD float pcr_dot3f_nofma(float a0, float a1, float a2, float b0, float b1, float b2) {
  float p0 = a0 * b0, p1 = a1 * b1, p2 = a2 * b2;
  float s = p0 + p1;
  return s + p2;
}
/* larger key = earlier in the descending-norm rank; NaN norms never win */
PCR_HD unsigned long long pcr_rank_key(float nrm, int idx) {
  unsigned u;
  if (!(nrm >= 0.0f)) return 0ull;
  __builtin_memcpy(&u, &nrm, 4);
  return ((unsigned long long)(u + 1u) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)idx);
}
PCR_HD int pcr_rank_key_index(unsigned long long key) {
  return (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
}
/* Does rank entry p (norm nrm) qualify as base_y for base_x bx?
 * (pvcnn_classify.py:163-168).  Python floats compare against the fp32
 * tensors in fp32. */
PCR_HD int pcr_lrf_base_y_ok(float px, float py, float pz, float nrm, const float bx[3]) {
  float lam;
  if (nrm < 1e-5f) return 0;
  lam = pcr_dot3f_nofma(bx[0], bx[1], bx[2], px / nrm, py / nrm, pz / nrm);
  return lam < 0.9f && lam > -0.9f;
}
/* Gram-Schmidt + cross (pvcnn_classify.py:176-182): basis rows x, y, z.
 * Returns 0, or 3 when the reference's orthogonality assert would fire. */
PCR_HD int pcr_lrf_basis(const float p0[3], float n0, const float p1[3], float n1,
                         float basis[9]) {
  float bx[3], by[3], bz[3], t, nx, nz;
  int a;
  for (a = 0; a < 3; a++) {
    bx[a] = p0[a] / n0;
    by[a] = p1[a] / n1;
  }
  t = pcr_dot3f_nofma(bx[0], bx[1], bx[2], by[0], by[1], by[2]);
  for (a = 0; a < 3; a++) {
    float m = by[a] * t;
    bx[a] = bx[a] - m;
  }
  nx = __builtin_sqrtf(pcr_sumsq3f_nofma(bx[0], bx[1], bx[2]));
  if (nx < 1e-5f) return 3;
  for (a = 0; a < 3; a++) bx[a] = bx[a] / nx;
  {
    float c0a = bx[1] * by[2], c0b = bx[2] * by[1];
    float c1a = bx[2] * by[0], c1b = bx[0] * by[2];
    float c2a = bx[0] * by[1], c2b = bx[1] * by[0];
    bz[0] = c0a - c0b;
    bz[1] = c1a - c1b;
    bz[2] = c2a - c2b;
  }
  nz = __builtin_sqrtf(pcr_sumsq3f_nofma(bz[0], bz[1], bz[2]));
  for (a = 0; a < 3; a++) {
    basis[a] = bx[a];
    basis[3 + a] = by[a];
    basis[6 + a] = bz[a] / nz;
  }
  return 0;
}

/* ---- normal estimation (utils/open3d_func.py:77-83,
 * Open3D PointCloud.estimate_normals(KDTreeSearchParamRadius(0.1)) +
 * orient_normals_towards_camera_location() + normalize_normals()).  Open3D
 * is not installed and its version is unpinned, so this is a restatement of
 * its published algorithm in double precision: neighbour cumulants ->
 * covariance -> the smallest eigenvector from the robust closed-form 3x3
 * solver (Eberly, "A Robust Eigensolver for 3x3 Symmetric Matrices"), which
 * Open3D's FastEigen3x3 implements.  Parity against Open3D is UNPINNED.
 * Every operation is explicit, so host and device agree bit for bit. ---- */
/* cos(x) for x in [0, pi]: Taylor series through x^22 in Horner form on
 * [0, pi/2] (truncation < 1e-19), with cos(x) = -cos(pi - x) above pi/2 */
PCR_HD double pcr_cos_d(double x) {
  double s = 1.0, z, p;
  if (x > PCR_PIO2) {
    x = PCR_PI - x;
    s = -1.0;
  }
  z = x * x;
  p = -8.896791392450574e-22; /* -1/22! */
  p = __builtin_fma(p, z, 4.110317623312165e-19); /* 1/20! */
  p = __builtin_fma(p, z, -1.5619206968586225e-16); /* -1/18! */
  p = __builtin_fma(p, z, 4.779477332387385e-14); /* 1/16! */
  p = __builtin_fma(p, z, -1.1470745597729725e-11); /* -1/14! */
  p = __builtin_fma(p, z, 2.08767569878681e-09); /* 1/12! */
  p = __builtin_fma(p, z, -2.755731922398589e-07); /* -1/10! */
  p = __builtin_fma(p, z, 2.48015873015873e-05); /* 1/8! */
  p = __builtin_fma(p, z, -0.001388888888888889); /* -1/6! */
  p = __builtin_fma(p, z, 0.041666666666666664); /* 1/4! */
  p = __builtin_fma(p, z, -0.5); /* -1/2! */
  p = __builtin_fma(p, z, 1.0); /* 1/0! */
  return s * p;
}
PCR_HD void pcr_cross_d(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
PCR_HD double pcr_dot_d(const double a[3], const double b[3]) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
/* A = {a00, a01, a02, a11, a12, a22} */
PCR_HD void pcr_eigvec0_d(const double A[6], double ev, double out[3]) {
  double r0[3] = {A[0] - ev, A[1], A[2]}, r1[3] = {A[1], A[3] - ev, A[4]};
  double r2[3] = {A[2], A[4], A[5] - ev};
  double c01[3], c02[3], c12[3], d0, d1, d2, dmax, s;
  const double *c;
  int imax = 0, a;
  pcr_cross_d(r0, r1, c01);
  pcr_cross_d(r0, r2, c02);
  pcr_cross_d(r1, r2, c12);
  d0 = pcr_dot_d(c01, c01);
  d1 = pcr_dot_d(c02, c02);
  d2 = pcr_dot_d(c12, c12);
  dmax = d0;
  if (d1 > dmax) {
    dmax = d1;
    imax = 1;
  }
  if (d2 > dmax) imax = 2;
  c = imax == 0 ? c01 : (imax == 1 ? c02 : c12);
  s = __builtin_sqrt(imax == 0 ? d0 : (imax == 1 ? d1 : d2));
  for (a = 0; a < 3; a++) out[a] = c[a] / s;
}
PCR_HD void pcr_eigvec1_d(const double A[6], const double e0[3], double ev, double out[3]) {
  double U[3], V[3], AU[3], AV[3], m00, m01, m11, am00, am01, am11, inv;
  int a;
  if (__builtin_fabs(e0[0]) > __builtin_fabs(e0[1])) {
    inv = 1.0 / __builtin_sqrt(e0[0] * e0[0] + e0[2] * e0[2]);
    U[0] = -e0[2] * inv;
    U[1] = 0.0;
    U[2] = e0[0] * inv;
  } else {
    inv = 1.0 / __builtin_sqrt(e0[1] * e0[1] + e0[2] * e0[2]);
    U[0] = 0.0;
    U[1] = e0[2] * inv;
    U[2] = -e0[1] * inv;
  }
  pcr_cross_d(e0, U, V);
  AU[0] = (A[0] * U[0] + A[1] * U[1]) + A[2] * U[2];
  AU[1] = (A[1] * U[0] + A[3] * U[1]) + A[4] * U[2];
  AU[2] = (A[2] * U[0] + A[4] * U[1]) + A[5] * U[2];
  AV[0] = (A[0] * V[0] + A[1] * V[1]) + A[2] * V[2];
  AV[1] = (A[1] * V[0] + A[3] * V[1]) + A[4] * V[2];
  AV[2] = (A[2] * V[0] + A[4] * V[1]) + A[5] * V[2];
  m00 = pcr_dot_d(U, AU) - ev;
  m01 = pcr_dot_d(U, AV);
  m11 = pcr_dot_d(V, AV) - ev;
  am00 = __builtin_fabs(m00);
  am01 = __builtin_fabs(m01);
  am11 = __builtin_fabs(m11);
  if (am00 >= am11) {
    if ((am00 > am01 ? am00 : am01) > 0.0) {
      if (am00 >= am01) {
        m01 /= m00;
        m00 = 1.0 / __builtin_sqrt(1.0 + m01 * m01);
        m01 *= m00;
      } else {
        m00 /= m01;
        m01 = 1.0 / __builtin_sqrt(1.0 + m00 * m00);
        m00 *= m01;
      }
      for (a = 0; a < 3; a++) out[a] = m01 * U[a] - m00 * V[a];
      return;
    }
  } else {
    if ((am11 > am01 ? am11 : am01) > 0.0) {
      if (am11 >= am01) {
        m01 /= m11;
        m11 = 1.0 / __builtin_sqrt(1.0 + m01 * m01);
        m01 *= m11;
      } else {
        m11 /= m01;
        m01 = 1.0 / __builtin_sqrt(1.0 + m11 * m11);
        m11 *= m01;
      }
      for (a = 0; a < 3; a++) out[a] = m11 * U[a] - m01 * V[a];
      return;
    }
  }
  for (a = 0; a < 3; a++) out[a] = U[a];
}
/* eigenvector of the smallest eigenvalue of the symmetric C (6 entries as
 * above); (0,0,0) when the largest entry is 0 (FastEigen3x3) */
PCR_HD void pcr_fast_eigen3x3(const double C[6], double out[3]) {
  double A[6], mx = C[0], nrm;
  int a;
  for (a = 1; a < 6; a++) mx = C[a] > mx ? C[a] : mx;
  if (mx == 0.0) {
    out[0] = out[1] = out[2] = 0.0;
    return;
  }
  for (a = 0; a < 6; a++) A[a] = C[a] / mx;
  nrm = (A[1] * A[1] + A[2] * A[2]) + A[4] * A[4];
  if (nrm > 0.0) {
    double q = ((A[0] + A[3]) + A[5]) / 3.0;
    double b00 = A[0] - q, b11 = A[3] - q, b22 = A[5] - q;
    double p = __builtin_sqrt(((((b00 * b00 + b11 * b11) + b22 * b22) + nrm * 2.0)) / 6.0);
    double c00 = b11 * b22 - A[4] * A[4];
    double c01 = A[1] * b22 - A[4] * A[2];
    double c02 = A[1] * A[4] - b11 * A[2];
    double det = ((b00 * c00 - A[1] * c01) + A[2] * c02) / ((p * p) * p);
    double hd = det * 0.5, ang, beta0, beta1, beta2, ev0, ev1, ev2, e0[3], e1[3];
    hd = hd < -1.0 ? -1.0 : (hd > 1.0 ? 1.0 : hd);
    ang = pcr_acos_d(hd) / 3.0;
    beta2 = pcr_cos_d(ang) * 2.0;
    beta0 = pcr_cos_d(ang + 2.09439510239319549) * 2.0;
    beta1 = -(beta0 + beta2);
    ev0 = q + p * beta0;
    ev1 = q + p * beta1;
    ev2 = q + p * beta2;
    if (hd >= 0.0) {
      pcr_eigvec0_d(A, ev2, e0); /* evec2 */
      if (ev2 < ev0 && ev2 < ev1) {
        for (a = 0; a < 3; a++) out[a] = e0[a];
        return;
      }
      pcr_eigvec1_d(A, e0, ev1, e1);
      if (ev1 < ev0 && ev1 < ev2) {
        for (a = 0; a < 3; a++) out[a] = e1[a];
        return;
      }
      pcr_cross_d(e1, e0, out);
    } else {
      pcr_eigvec0_d(A, ev0, e0);
      if (ev0 < ev1 && ev0 < ev2) {
        for (a = 0; a < 3; a++) out[a] = e0[a];
        return;
      }
      pcr_eigvec1_d(A, e0, ev1, e1);
      if (ev1 < ev0 && ev1 < ev2) {
        for (a = 0; a < 3; a++) out[a] = e1[a];
        return;
      }
      pcr_cross_d(e0, e1, out);
    }
    return;
  }
  if (C[0] < C[3] && C[0] < C[5]) {
    out[0] = 1.0;
    out[1] = out[2] = 0.0;
  } else if (C[3] < C[0] && C[3] < C[5]) {
    out[1] = 1.0;
    out[0] = out[2] = 0.0;
  } else {
    out[2] = 1.0;
    out[0] = out[1] = 0.0;
  }
}
/* One point's normal from its neighbour cumulants
 * cum = {sx, sy, sz, sxx, sxy, sxz, syy, syz, szz} over cnt neighbours
 * (itself included): fewer than 3 -> (0,0,1); zero eigenvector -> (0,0,1);
 * flip towards the camera at the origin (dot(n, -p) < 0 -> -n; a zero
 * normal cannot reach here); normalise; round to float. */
PCR_HD void pcr_estimate_normal(const double cum[9], int cnt, float px, float py, float pz,
                                float out[3]) {
  double n[3], C[6], m[9], ref[3], len;
  int a;
  if (cnt < 3) {
    out[0] = out[1] = 0.0f;
    out[2] = 1.0f;
    return;
  }
  for (a = 0; a < 9; a++) m[a] = cum[a] / (double)cnt;
  C[0] = m[3] - m[0] * m[0];
  C[1] = m[4] - m[0] * m[1];
  C[2] = m[5] - m[0] * m[2];
  C[3] = m[6] - m[1] * m[1];
  C[4] = m[7] - m[1] * m[2];
  C[5] = m[8] - m[2] * m[2];
  pcr_fast_eigen3x3(C, n);
  if (n[0] == 0.0 && n[1] == 0.0 && n[2] == 0.0) {
    n[2] = 1.0;
  }
  ref[0] = -(double)px;
  ref[1] = -(double)py;
  ref[2] = -(double)pz;
  if (pcr_dot_d(n, ref) < 0.0)
    for (a = 0; a < 3; a++) n[a] = -n[a];
  len = __builtin_sqrt(pcr_dot_d(n, n));
  for (a = 0; a < 3; a++) out[a] = (float)(n[a] / len);
}

#endif /* PCR_MATH_H */
