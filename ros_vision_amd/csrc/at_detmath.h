// at_detmath.h -- deterministic transcendental math for the AprilTag path.
//
// The reference evaluates atan2f (apriltag_gpu.cu:402-404), hypotf
// (apriltag_gpu.cu:656, line_fit_filter.cu:33,820,857, apriltag_detect.cu:48,
// 180) and cosf/sinf/atan2f (apriltag_detect.cu:523-525) through the platform
// libm, whose last-ulp behaviour differs between CUDA, glibc and ROCm's ocml.
// Those ulps feed integer quantisation (theta = llrintf(...), W = (int)(...))
// and strict comparisons (peak finding, quad argmin), so we pin them: each
// function is a fixed sequence of IEEE double operations (correctly rounded
// +,-,*,/,sqrt and explicit fma on both x86 and gfx950) rounded once to float.
// Compile with -ffp-contract=off so no other a*b+c is fused.  All are within 1 float
// ulp of the correctly rounded result.
#pragma once

#if defined(__HIPCC__)
#define AT_HD __host__ __device__ __forceinline__
#else
#define AT_HD static inline
#endif

#include <math.h>
#include <stdint.h>

namespace at {

// atan2 with ONE division: the octant reduction t = (b - a) / (a + b) (b <= a the
// smaller and larger of |y|, |x|, when b > tan(pi/8) a) or t = b / a, so |t| <= tan(pi/8)
// < 7/16, then fdlibm's odd minimax polynomial for atan on |t| < 7/16 (s_atan.c, error
// < 2^-58) by explicit fma (correctly rounded on gfx950 and x86 alike), and the octant
// constants in two parts.  Max relative error 2.3e-16 over 2*10^7 inputs (the former
// three-division Cephes form: 2.6e-16); its float-rounded results equal the former's on
// every one of them.  (k_extents: 1 instead of 3 fp64 divisions per point.)
AT_HD double det_atan2(double y, double x) {
  const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
               aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
               aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
               aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
               aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
               aT10 = 1.62858201153657823623e-02;
  const double ax = fabs(x), ay = fabs(y);
  const bool sw = ay > ax;
  const double a = sw ? ay : ax, b = sw ? ax : ay;
  if (a == 0.0) return 0.0;
  const bool s = b > 0.41421356237309504880 * a;
  const double t = (s ? b - a : b) / (s ? a + b : a);
  const double z = t * t, w = z * z;
  double s1 = fma(w, aT10, aT8);
  s1 = fma(w, s1, aT6);
  s1 = fma(w, s1, aT4);
  s1 = fma(w, s1, aT2);
  s1 = fma(w, s1, aT0);
  s1 = z * s1;
  double s2 = fma(w, aT9, aT7);
  s2 = fma(w, s2, aT5);
  s2 = fma(w, s2, aT3);
  s2 = fma(w, s2, aT1);
  s2 = w * s2;
  const double hi = s ? 7.85398163397448278999e-01 : 0.0, lo = s ? 3.06161699786838301793e-17 : 0.0;
  double r = hi - ((t * (s1 + s2) - lo) - t);
  if (sw) r = (1.57079632679489655800e+00 - r) + 6.12323399573676603587e-17;
  if (x < 0.0) r = (3.14159265358979311600e+00 - r) + 1.22464679914735317723e-16;
  return y < 0.0 ? -r : r;
}

AT_HD float det_atan2f(float y, float x) { return (float)det_atan2((double)y, (double)x); }

AT_HD double det_sin_poly(double x) {
  const double z = x * x;
  double p = 1.58962301576546568060E-10;
  p = p * z + -2.50507477628578072866E-8;
  p = p * z + 2.75573136213857245213E-6;
  p = p * z + -1.98412698295895385996E-4;
  p = p * z + 8.33333333332211858878E-3;
  p = p * z + -1.66666666666666307295E-1;
  return x + x * z * p;
}

AT_HD double det_cos_poly(double x) {
  const double z = x * x;
  double p = -1.13585365213876817300E-11;
  p = p * z + 2.08757008419747316778E-9;
  p = p * z + -2.75573141792967388112E-7;
  p = p * z + 2.48015872888517045348E-5;
  p = p * z + -1.38888888888730564116E-3;
  p = p * z + 4.16666666666665929218E-2;
  return 1.0 - 0.5 * z + z * z * p;
}

AT_HD void det_sincos(double x, double* s, double* c) {
  const double kPio2 = 1.57079632679489661923;
  const double kPio2Hi = 1.57079632673412561417e+00;
  const double kPio2Lo = 6.07710050650619224932e-11;
  const double jf = rint(x / kPio2);
  const int j = (int)jf;
  const double r = (x - jf * kPio2Hi) - jf * kPio2Lo;
  const double sr = det_sin_poly(r), cr = det_cos_poly(r);
  switch (j & 3) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
  }
}

AT_HD float det_cosf(float x) { double s, c; det_sincos((double)x, &s, &c); return (float)c; }
AT_HD float det_sinf(float x) { double s, c; det_sincos((double)x, &s, &c); return (float)s; }

AT_HD float det_hypotf(float a, float b) {
  const double x = a, y = b;
  return (float)sqrt(x * x + y * y);
}

}  // namespace at
