// at_detmath.h -- deterministic transcendental math for the AprilTag path.
//
// The reference evaluates atan2f (apriltag_gpu.cu:402-404), hypotf
// (apriltag_gpu.cu:656, line_fit_filter.cu:33,820,857, apriltag_detect.cu:48,
// 180) and cosf/sinf/atan2f (apriltag_detect.cu:523-525) through the platform
// libm, whose last-ulp behaviour differs between CUDA, glibc and ROCm's ocml.
// Those ulps feed integer quantisation (theta = llrintf(...), W = (int)(...))
// and strict comparisons (peak finding, quad argmin), so we pin them: each
// function is a fixed sequence of IEEE double operations (correctly rounded
// +,-,*,/,sqrt on both x86 and gfx950) rounded once to float.  Compile with
// -ffp-contract=off so no a*b+c is fused.  All are within 1 float ulp of the
// correctly rounded result.
#pragma once

#if defined(__HIPCC__)
#define AT_HD __host__ __device__ __forceinline__
#else
#define AT_HD static inline
#endif

#include <math.h>
#include <stdint.h>

namespace at {

AT_HD double det_atan_pos(double t) {
  // Cephes atan(): three-interval reduction + rational minimax, |rel err| < 2.3e-16
  const double P0 = -8.750608600031904122785E-1, P1 = -1.615753718733365076637E1,
               P2 = -7.500855792314704667340E1, P3 = -1.228866684490136173410E2,
               P4 = -6.485021904942025371773E1;
  const double Q0 = 2.485846490142306297962E1, Q1 = 1.650270098316988542046E2,
               Q2 = 4.328810604912902668951E2, Q3 = 4.853903996359136964868E2,
               Q4 = 1.945506571482613964425E2;
  const double kMoreBits = 6.123233995736765886130E-17;
  double y0, x;
  int flag;
  if (t > 2.41421356237309504880) {
    y0 = 1.57079632679489661923; flag = 1; x = -1.0 / t;
  } else if (t <= 0.66) {
    y0 = 0.0; flag = 0; x = t;
  } else {
    y0 = 0.78539816339744830962; flag = 2; x = (t - 1.0) / (t + 1.0);
  }
  double z = x * x;
  double p = P0;
  p = p * z + P1; p = p * z + P2; p = p * z + P3; p = p * z + P4;
  double q = z + Q0;
  q = q * z + Q1; q = q * z + Q2; q = q * z + Q3; q = q * z + Q4;
  z = z * p / q;
  z = x * z + x;
  if (flag == 2) z = z + 0.5 * kMoreBits;
  else if (flag == 1) z = z + kMoreBits;
  return y0 + z;
}

AT_HD double det_atan2(double y, double x) {
  if (x == 0.0) {
    if (y > 0.0) return 1.57079632679489661923;
    if (y < 0.0) return -1.57079632679489661923;
    return 0.0;
  }
  double a = det_atan_pos(fabs(y) / fabs(x));
  if (x < 0.0) a = 3.14159265358979323846 - a;
  if (y < 0.0) a = -a;
  return a;
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
