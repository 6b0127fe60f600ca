// at_pose.h -- device tag pose (§8 row A23): estimate_tag_pose as the
// reference node calls it on every detection (apriltags_cuda_detector.cu:433,
// info_ filled at :185-189 with TAGSIZE 0.1651, apriltags_cuda_detector.hpp:39).
//
// The algorithm is the un-vendored AprilTag 3.x library's (apriltag_pose.c):
// homography_to_pose initialisation, 50 steps of orthogonal iteration, the
// second local minimum from fix_pose_ambiguities, smaller error wins.  The
// polar factors that library takes from a general SVD are computed here in
// closed form, which is exact for the shapes that occur:
//   * homography_to_pose: R = M (M'M)^-1/2 of a full-rank 3x3 (Newton polar
//     iteration X <- (X + X^-T)/2, quadratically convergent from a scaled
//     near-rotation);
//   * orthogonal_iteration: M3 = sum (q_j - q_mean) p_res_j' has a zero third
//     column (tag corners lie in z = 0), so U V' restricted to the first two
//     columns is the polar factor of the 3x2 block A (A'A)^-1/2 (2x2 closed
//     form), and the det(R) < 0 column-2 flip leaves column 2 = c0 x c1.
// Four lanes per detection (the quartic's root brackets in parallel); everything
// in double.  The k_pose chain is latency-bound, so FMA contraction is allowed here
// (float tolerance 1e-4, unlike the bit-exact integer stages) and the
// per-step sums are balanced trees.
#pragma once

#include "at_detmath.h"

#pragma clang fp contract(fast)

namespace at {
namespace pose {

struct M3 {
  double m[3][3];
};
struct V3 {
  double v[3];
};

__device__ __forceinline__ M3 m3_eye() {
  M3 r;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) r.m[i][j] = i == j ? 1.0 : 0.0;
  return r;
}
__device__ __forceinline__ M3 m3_mul(const M3& a, const M3& b) {
  M3 r;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      double acc = 0;
#pragma unroll
      for (int k = 0; k < 3; k++) acc += a.m[i][k] * b.m[k][j];
      r.m[i][j] = acc;
    }
  return r;
}
__device__ __forceinline__ M3 m3_t(const M3& a) {
  M3 r;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) r.m[i][j] = a.m[j][i];
  return r;
}
__device__ __forceinline__ V3 mv(const M3& a, const V3& x) {
  V3 r;
#pragma unroll
  for (int i = 0; i < 3; i++) r.v[i] = a.m[i][0] * x.v[0] + a.m[i][1] * x.v[1] + a.m[i][2] * x.v[2];
  return r;
}
__device__ __forceinline__ V3 v_add(V3 a, const V3& b) {
#pragma unroll
  for (int i = 0; i < 3; i++) a.v[i] += b.v[i];
  return a;
}
__device__ __forceinline__ V3 v_sub(V3 a, const V3& b) {
#pragma unroll
  for (int i = 0; i < 3; i++) a.v[i] -= b.v[i];
  return a;
}
__device__ __forceinline__ V3 v_scale(V3 a, double s) {
#pragma unroll
  for (int i = 0; i < 3; i++) a.v[i] *= s;
  return a;
}
__device__ __forceinline__ double v_dot(const V3& a, const V3& b) {
  return a.v[0] * b.v[0] + a.v[1] * b.v[1] + a.v[2] * b.v[2];
}
__device__ __forceinline__ V3 v_cross(const V3& a, const V3& b) {
  V3 r;
  r.v[0] = a.v[1] * b.v[2] - a.v[2] * b.v[1];
  r.v[1] = a.v[2] * b.v[0] - a.v[0] * b.v[2];
  r.v[2] = a.v[0] * b.v[1] - a.v[1] * b.v[0];
  return r;
}
__device__ __forceinline__ double m3_det(const M3& a) {
  return a.m[0][0] * (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]) -
         a.m[0][1] * (a.m[1][0] * a.m[2][2] - a.m[1][2] * a.m[2][0]) +
         a.m[0][2] * (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]);
}
// inverse via the adjugate
__device__ __forceinline__ M3 m3_inv(const M3& a) {
  const double id = 1.0 / m3_det(a);
  M3 r;
  r.m[0][0] = (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]) * id;
  r.m[0][1] = (a.m[0][2] * a.m[2][1] - a.m[0][1] * a.m[2][2]) * id;
  r.m[0][2] = (a.m[0][1] * a.m[1][2] - a.m[0][2] * a.m[1][1]) * id;
  r.m[1][0] = (a.m[1][2] * a.m[2][0] - a.m[1][0] * a.m[2][2]) * id;
  r.m[1][1] = (a.m[0][0] * a.m[2][2] - a.m[0][2] * a.m[2][0]) * id;
  r.m[1][2] = (a.m[0][2] * a.m[1][0] - a.m[0][0] * a.m[1][2]) * id;
  r.m[2][0] = (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]) * id;
  r.m[2][1] = (a.m[0][1] * a.m[2][0] - a.m[0][0] * a.m[2][1]) * id;
  r.m[2][2] = (a.m[0][0] * a.m[1][1] - a.m[0][1] * a.m[1][0]) * id;
  return r;
}

// polar factor of a full-rank 3x3 (== U V' of its SVD)
__device__ M3 polar3(M3 x) {
  for (int it = 0; it < 40; it++) {
    const M3 xit = m3_t(m3_inv(x));
    double delta = 0;
    M3 n;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) {
        n.m[i][j] = 0.5 * (x.m[i][j] + xit.m[i][j]);
        delta = fmax(delta, fabs(n.m[i][j] - x.m[i][j]));
      }
    x = n;
    if (delta < 1e-15) break;
  }
  return x;
}

// 1/sqrt(x), x > 0: the hardware estimate and one second-order correction
// (y (1 + e/2 + 3e^2/8), e = 1 - x y^2) -- ocml's refinement without its
// special-case select.  x = 0 does reach it: polar_rank2_cols passes
// D = max(ac - b^2, 0), which is 0 when the iterate's two columns are parallel
// (all four image rays in one plane through the camera centre, i.e. collinear
// corners).  Then rsq(0) = inf and the pose and its error come out NaN --
// a documented outcome, not reachable from the pipeline:
// UpdateFitQuads' area test (>= 0.95 * 4^2, apriltag_detect.cu:190-200) rejects
// such quads before k_pose sees them.
__device__ __forceinline__ double rsqrt_pos(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double e = fma(-x * y, y, 1.0);
  return fma(y * e, fma(0.375, e, 0.5), y);
}

// polar factor of the 3x2 block [m0 m1] (third column of M3 is zero): the
// columns (q0, q1) of Q = A (A'A)^-1/2.  With S = A'A = [a b; b c],
// sqrt(S) = (S + d I) / tau, d = sqrt(det S), tau = sqrt(tr S + 2d);
// det(S + d I) = d tau^2, so (S + d I)^-1 tau = adj(S + d I) / (d tau):
// two reciprocal square roots, no square root and no division on the chain.
// The third column of U V' after orthogonal_iteration's det < 0 fix is q0 x q1.
__device__ __forceinline__ void polar_rank2_cols(const V3& m0, const V3& m1, V3& q0, V3& q1) {
  const double a = m0.v[0] * m0.v[0] + m0.v[1] * m0.v[1] + m0.v[2] * m0.v[2];
  const double b = m0.v[0] * m1.v[0] + m0.v[1] * m1.v[1] + m0.v[2] * m1.v[2];
  const double c = m1.v[0] * m1.v[0] + m1.v[1] * m1.v[1] + m1.v[2] * m1.v[2];
  const double D = fmax(a * c - b * b, 0.0);
  const double rd = rsqrt_pos(D);
  const double d = D * rd;
  const double rt = rsqrt_pos(a + c + 2 * d);
  const double k = rd * rt;
  const double i00 = (c + d) * k, i01 = -b * k, i11 = (a + d) * k;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    q0.v[i] = m0.v[i] * i00 + m1.v[i] * i01;
    q1.v[i] = m0.v[i] * i01 + m1.v[i] * i11;
  }
}

// (one reciprocal instead of nine divisions: within the pose tolerance, like the
// contracted products above)
__device__ __forceinline__ M3 calculate_F(const V3& v) {
  M3 F;
  const double ri = 1.0 / v_dot(v, v);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) F.m[i][j] = v.v[i] * v.v[j] * ri;
  return F;
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}

// orthogonal_iteration over the 4 tag corners p_j = (sx_j, sy_j, 0).
// Every quantity of one step is linear in the first two columns (r0, r1) of
// R (p_j has no z), so with G_x = sum sx_j F_j, G_y = sum sy_j F_j,
// F_s = sum F_j, F_xy = sum sx_j sy_j F_j and T_x,y = M1^-1 G_x,y / 4:
//   t       = T_x r0 + T_y r1                      ((F - I) R p averaged, M1^-1)
//   M3[:,0] = (s^2 F_s + G_x T_x) r0 + (F_xy + G_x T_y) r1
//   M3[:,1] = (F_xy + G_y T_x) r0 + (s^2 F_s + G_y T_y) r1
// (sum_j sx_j = sum_j sy_j = 0 removes the I and q_mean terms).  The step is
// then R <- polar(M3).  As upstream, the returned t belongs to the R before the last step
// and the error to the final (R, t).
// WAVE (a whole wave per detection): lane c < 6 evaluates component c of (m0, m1) -- the
// same balanced 6-term dot product -- and every lane reads the six back, so a step issues
// one dot product and six lane reads instead of six dot products.
template <bool WAVE = false>
__device__ double orthogonal_iteration(const V3* v, const V3* p, V3* t, M3* R, int n_steps, int* steps = nullptr) {
  M3 Gx, Gy, Fs, Fxy;
  {
  // (F_j is recomputed for the error below instead of being held across the loop:
  // 72 registers fewer while the iteration runs)
  M3 F[4];
#pragma unroll
  for (int k = 0; k < 4; k++) F[k] = calculate_F(v[k]);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      double gx = 0, gy = 0, fs = 0, fxy = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        gx += p[k].v[0] * F[k].m[i][j];
        gy += p[k].v[1] * F[k].m[i][j];
        fs += F[k].m[i][j];
        fxy += p[k].v[0] * p[k].v[1] * F[k].m[i][j];
      }
      Gx.m[i][j] = gx;
      Gy.m[i][j] = gy;
      Fs.m[i][j] = fs;
      Fxy.m[i][j] = fxy;
    }
  }
  M3 ImA;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) ImA.m[i][j] = (i == j ? 1.0 : 0.0) - Fs.m[i][j] * 0.25;
  const M3 M1_inv = m3_inv(ImA);
  M3 Tx = m3_mul(M1_inv, Gx), Ty = m3_mul(M1_inv, Gy);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      Tx.m[i][j] *= 0.25;
      Ty.m[i][j] *= 0.25;
    }
  const double s2 = p[0].v[0] * p[0].v[0];
  const M3 GxTx = m3_mul(Gx, Tx), GxTy = m3_mul(Gx, Ty), GyTx = m3_mul(Gy, Tx), GyTy = m3_mul(Gy, Ty);
  M3 A00, A01, A10, A11;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      A00.m[i][j] = s2 * Fs.m[i][j] + GxTx.m[i][j];
      A01.m[i][j] = Fxy.m[i][j] + GxTy.m[i][j];
      A10.m[i][j] = Fxy.m[i][j] + GyTx.m[i][j];
      A11.m[i][j] = s2 * Fs.m[i][j] + GyTy.m[i][j];
    }
  // iterate on (r0, r1).  The step contracts slowly (rate ~0.9 for typical
  // tag geometry, so the iterate still moves ~1e-5..1e-4 at step 50): all
  // n_steps run, with no per-step exit test; (q0, q1) keeps iterate k - 1,
  // whose t upstream returns
  V3 r0 = {{R->m[0][0], R->m[1][0], R->m[2][0]}}, r1 = {{R->m[0][1], R->m[1][1], R->m[2][1]}};
  V3 q0 = r0, q1 = r1;
  // (WAVE) this lane's row of [A00 A01; A10 A11]: component c = lane % 6 of (m0, m1)
  double cr[6];
  if constexpr (WAVE) {
    const int c = (int)(__lane_id() % 6), i = c % 3;
    const M3& L = c < 3 ? A00 : A10;
    const M3& Rm = c < 3 ? A01 : A11;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      cr[j] = L.m[i][j];
      cr[3 + j] = Rm.m[i][j];
    }
  }
  auto step = [&](const V3& x0, const V3& x1, V3& y0, V3& y1) {
    V3 m0, m1;
    if constexpr (WAVE) {
      const double mine = ((cr[0] * x0.v[0] + cr[1] * x0.v[1]) + (cr[2] * x0.v[2] + cr[3] * x1.v[0])) +
                          (cr[4] * x1.v[1] + cr[5] * x1.v[2]);
#pragma unroll
      for (int i = 0; i < 3; i++) {
        m0.v[i] = readlane_f64(mine, i);
        m1.v[i] = readlane_f64(mine, 3 + i);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 3; i++) {  // balanced 6-term dot products
        m0.v[i] = ((A00.m[i][0] * x0.v[0] + A00.m[i][1] * x0.v[1]) + (A00.m[i][2] * x0.v[2] + A01.m[i][0] * x1.v[0])) +
                  (A01.m[i][1] * x1.v[1] + A01.m[i][2] * x1.v[2]);
        m1.v[i] = ((A10.m[i][0] * x0.v[0] + A10.m[i][1] * x0.v[1]) + (A10.m[i][2] * x0.v[2] + A11.m[i][0] * x1.v[0])) +
                  (A11.m[i][1] * x1.v[1] + A11.m[i][2] * x1.v[2]);
      }
    }
    polar_rank2_cols(m0, m1, y0, y1);
  };
  int k = 0;
  for (; k + 2 <= n_steps; k += 2) {  // two steps per trip: no register rotation
    step(r0, r1, q0, q1);
    step(q0, q1, r0, r1);
  }
  if (k < n_steps) {  // odd n_steps
    step(r0, r1, q0, q1);
    const V3 a0 = r0, a1 = r1;
    r0 = q0; r1 = q1;
    q0 = a0; q1 = a1;
  }
  if (steps) *steps = n_steps + 1;
  M3 Rn;
  const V3 r2 = v_cross(r0, r1);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    Rn.m[i][0] = r0.v[i];
    Rn.m[i][1] = r1.v[i];
    Rn.m[i][2] = r2.v[i];
  }
  *R = Rn;
  *t = v_add(mv(Tx, q0), mv(Ty, q1));
  double error = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const M3 Fj = calculate_F(v[j]);
    const V3 x = v_add(mv(*R, p[j]), *t);
    const V3 e = v_sub(x, mv(Fj, x));  // (I - F) x
    error += v_dot(e, e);
  }
  return error;
}

// sum_i p[i] * x^i in the upstream summation order; x^i by repeated products
// (upstream pow(x, i): the two differ in the last bit only)
__device__ __forceinline__ double polyval(const double* p, int degree, double x) {
  double ret = 0, xi = 1;
  for (int i = 0; i <= degree; i++) {
    ret += p[i] * xi;
    xi *= x;
  }
  return ret;
}

// Element i (0 .. 3) of a 4-entry local array, read or written by selects over the
// four static slots: a lane-varying or runtime index into a private array otherwise
// keeps the array in scratch memory (a global-memory round trip per access)
__device__ __forceinline__ double pick4(const double* a, int i) {
  return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}
__device__ __forceinline__ void put4(double* a, int i, double v) {
  a[0] = i == 0 ? v : a[0];
  a[1] = i == 1 ? v : a[1];
  a[2] = i == 2 ? v : a[2];
  a[3] = i == 3 ? v : a[3];
}

// Four lanes (a DPP quad) work on one detection: every quantity is computed
// redundantly on all four, except the root brackets of solve_poly_approx, which
// are independent and are solved one per lane; the roots are then gathered in
// bracket order by quad broadcasts, so each lane ends up with exactly the
// sequential result.
template <int J>
__device__ __forceinline__ double quad_bcast(double v) {
  constexpr int kCtrl = J | (J << 2) | (J << 4) | (J << 6);  // quad_perm:[J,J,J,J]
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, kCtrl, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), kCtrl, 0xf, 0xf, false);
  return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}
template <int J>
__device__ __forceinline__ int quad_bcast(int v) {
  return __builtin_amdgcn_update_dpp(0, v, J | (J << 2) | (J << 4) | (J << 6), 0xf, 0xf, false);
}

// solve_poly_approx for degree <= 4, unrolled over degrees 1..4 (no recursion).
// The outer brackets [-1000, r_1] and [r_n, 1000] are shrunk to the Cauchy
// bound 1 + max|p_i / p_deg| when it is smaller: no real root lies beyond it
// (nor, by Gauss-Lucas, a derivative root), so the sign test and the bracketed
// root are unchanged while the safeguarded Newton needs far fewer steps.
// Bracket `sub` (<= n_der <= 3) is this lane's; the caller's quad supplies the rest.
// (der_roots and roots: 4-entry arrays, indexed through pick4 / put4)
__device__ __forceinline__ int solve_poly_level(const double* p, int degree, const double* der_roots, int n_der, double* roots,
                                int sub) {
  double MAX_ROOT = 1000;
  if (p[degree] != 0) {
    double cb = 0;
    for (int i = 0; i < degree; i++) cb = fmax(cb, fabs(p[i] / p[degree]));
    MAX_ROOT = fmin(MAX_ROOT, 1 + cb);
  }
  double p_der[4];
  for (int i = 0; i < degree; i++) p_der[i] = (i + 1) * p[i + 1];
  double my_root = 0;
  int my_has = 0;
  if (sub <= n_der) {
    const int i = sub;
    const double mn = i == 0 ? -MAX_ROOT : pick4(der_roots, i - 1);
    const double mx = i == n_der ? MAX_ROOT : pick4(der_roots, i);
    const double fmn = polyval(p, degree, mn), fmx = polyval(p, degree, mx);
    if (fmn * fmx < 0) {
      double lower, upper;
      if (fmn < fmx) {
        lower = mn;
        upper = mx;
      } else {
        lower = mx;
        upper = mn;
      }
      double root = 0.5 * (lower + upper);
      double dx_old = upper - lower, dx = dx_old;
      double f = polyval(p, degree, root), df = polyval(p_der, degree - 1, root);
      for (int j = 0; j < 100; j++) {
        if (((f + df * (upper - root)) * (f + df * (lower - root)) > 0) || (fabs(2 * f) > fabs(dx_old * df))) {
          dx_old = dx;
          dx = 0.5 * (upper - lower);
          root = lower + dx;
        } else {
          dx_old = dx;
          dx = -f / df;
          root += dx;
        }
        if (root == upper || root == lower) break;
        f = polyval(p, degree, root);
        df = polyval(p_der, degree - 1, root);
        if (f > 0) upper = root;
        else lower = root;
      }
      my_root = root;
      my_has = 1;
    } else if (fmx == 0) {
      my_root = mx;
      my_has = 1;
    }
  }
  int n = 0;
  double r;
  r = quad_bcast<0>(my_root);
  if (quad_bcast<0>(my_has)) put4(roots, n++, r);
  r = quad_bcast<1>(my_root);
  if (quad_bcast<1>(my_has)) put4(roots, n++, r);
  r = quad_bcast<2>(my_root);
  if (quad_bcast<2>(my_has)) put4(roots, n++, r);
  r = quad_bcast<3>(my_root);
  if (quad_bcast<3>(my_has)) put4(roots, n++, r);
  return n;
}

// The same level with a whole wave per detection (latency mode, k_decode<true>):
// bracket s (<= n_der <= 3) belongs to lanes 16 s .. 16 s + 15, which search it in
// parallel -- each round every lane evaluates the polynomial at one of 16 interior
// points of (lower, upper) and the group keeps the sub-interval where the sign
// changes (a ballot), shrinking the bracket 17-fold per round, until no interior
// point is representable.  The end points and the sign test are upstream's; the root
// is the converged bracket end on the f <= 0 side (upstream's safeguarded Newton
// converges to the same double to within an ulp or two; orthogonal iteration then
// contracts any such difference).  No divisions, ~20 rounds instead of a
// data-dependent Newton/bisection loop.
__device__ __forceinline__ double horner(const double* p, int degree, double x) {
  double r = p[degree];
  for (int i = degree - 1; i >= 0; i--) r = fma(r, x, p[i]);
  return r;
}
// This lane's bracket root (my_has: one exists); the caller gathers.
__device__ __forceinline__ void solve_poly_level_wave_lane(const double* p, int degree, const double* der_roots, int n_der,
                                           double& my_root, int& my_has) {
  double MAX_ROOT = 1000;
  if (p[degree] != 0) {
    double cb = 0;
    const double rl = 1.0 / fabs(p[degree]);  // (the bound only has to exceed every root)
    for (int i = 0; i < degree; i++) cb = fmax(cb, fabs(p[i]) * rl);
    MAX_ROOT = fmin(MAX_ROOT, 1 + cb * (1 + 0x1p-40));
  }
  const int lane = (int)__lane_id();
  const int sub = lane >> 4, j = lane & 15;
  my_root = 0;
  my_has = 0;
  if (sub <= n_der) {
    const double mn = sub == 0 ? -MAX_ROOT : pick4(der_roots, sub - 1);
    const double mx = sub == n_der ? MAX_ROOT : pick4(der_roots, sub);
    const double fmn = polyval(p, degree, mn), fmx = polyval(p, degree, mx);
    if (fmn * fmx < 0) {
      double lower = fmn < fmx ? mn : mx, upper = fmn < fmx ? mx : mn;
      if (degree == 2 && p[2] != 0) {
        // a quadratic's bracketed root in closed form (the cancellation-free pair
        // q / a, c / q); the search below only if rounding put it outside the bracket
        const double disc = p[1] * p[1] - 4 * p[2] * p[0];
        if (disc >= 0) {
          const double q = -0.5 * (p[1] + copysign(sqrt(disc), p[1]));
          const double ra = q / p[2], rb = q != 0 ? p[0] / q : ra;
          const double lo = fmin(mn, mx), hi = fmax(mn, mx);
          const bool ina = ra >= lo && ra <= hi, inb = rb >= lo && rb <= hi;
          if (ina != inb) {
            lower = upper = ina ? ra : rb;
          }
        }
      }
      // down to 2^-30 of max(1, |root|), then two Newton steps kept inside the
      // final bracket (quadratic convergence: far below what orthogonal iteration
      // resolves; upstream's Newton stops at the same double within an ulp or two)
      for (int it = 0; it < 24 && fabs(upper - lower) > 0x1p-30 * fmax(1.0, fabs(lower)); it++) {
        const double h = (upper - lower) * (1.0 / 17.0);
        const double x = fma((double)(j + 1), h, lower);
        const uint64_t neg = __ballot(horner(p, degree, x) <= 0);
        const int k = __popcll((neg >> (lane & 48)) & 0xffffull);
        const double nl = k == 0 ? lower : fma((double)k, h, lower);
        const double nu = k == 16 ? upper : fma((double)(k + 1), h, lower);
        if (nl == lower && nu == upper) break;
        lower = nl;
        upper = nu;
      }
      if (lower != upper) {
        double pd[4];
        for (int i = 0; i < degree; i++) pd[i] = (i + 1) * p[i + 1];
        const double blo = fmin(lower, upper), bhi = fmax(lower, upper);
        double x = 0.5 * (lower + upper);
#pragma unroll
        for (int it = 0; it < 2; it++) {
          const double f = horner(p, degree, x), df = horner(pd, degree - 1, x);
          if (df != 0) x = fmin(bhi, fmax(blo, x - f / df));
        }
        lower = x;
      }
      my_root = lower;
      my_has = 1;
    } else if (fmx == 0) {
      my_root = mx;
      my_has = 1;
    }
  }
}
__device__ __forceinline__ int solve_poly_level_wave(const double* p, int degree, const double* der_roots, int n_der, double* roots) {
  double my_root;
  int my_has;
  solve_poly_level_wave_lane(p, degree, der_roots, n_der, my_root, my_has);
  int n = 0;
#pragma unroll
  for (int s2 = 0; s2 < 4; s2++) {
    const double r = readlane_f64(my_root, 16 * s2);
    if (__builtin_amdgcn_readlane(my_has, 16 * s2)) put4(roots, n++, r);
  }
  return n;
}

template <bool WAVE>
__device__ __forceinline__ int solve_quartic_approx(const double* p4, double* roots, int sub) {
  // derivative chain: p4 (deg 4) -> p3 -> p2 -> p1 (linear)
  double d3[4], d2[3], d1[2];
  for (int i = 0; i < 4; i++) d3[i] = (i + 1) * p4[i + 1];
  for (int i = 0; i < 3; i++) d2[i] = (i + 1) * d3[i + 1];
  for (int i = 0; i < 2; i++) d1[i] = (i + 1) * d2[i + 1];
  double r1[4] = {0, 0, 0, 0}, r2[4] = {0, 0, 0, 0}, r3[4] = {0, 0, 0, 0};
  int n1 = 0;
  if (!(fabs(d1[0]) > 1000 * fabs(d1[1]))) {
    r1[0] = -d1[0] / d1[1];
    n1 = 1;
  }
  if constexpr (WAVE) {
    const int n2 = solve_poly_level_wave(d2, 2, r1, n1, r2);
    const int n3 = solve_poly_level_wave(d3, 3, r2, n2, r3);
    return solve_poly_level_wave(p4, 4, r3, n3, roots);
  } else {
    const int n2 = solve_poly_level(d2, 2, r1, n1, r2, sub);
    const int n3 = solve_poly_level(d3, 3, r2, n2, r3, sub);
    return solve_poly_level(p4, 4, r3, n3, roots, sub);
  }
}

template <bool WAVE>
__device__ bool fix_pose_ambiguities(const V3* v, const V3* p, const V3& t, const M3& R, M3* out, int sub,
                                     uint64_t* stamps = nullptr) {
  const V3 R_t_3 = v_scale(t, 1.0 / sqrt(v_dot(t, t)));
  const V3 e_x = {{1, 0, 0}};
  V3 R_t_1 = v_sub(e_x, v_scale(R_t_3, v_dot(e_x, R_t_3)));
  R_t_1 = v_scale(R_t_1, 1.0 / sqrt(v_dot(R_t_1, R_t_1)));
  const V3 R_t_2 = v_cross(R_t_3, R_t_1);
  M3 R_t;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    R_t.m[0][i] = R_t_1.v[i];
    R_t.m[1][i] = R_t_2.v[i];
    R_t.m[2][i] = R_t_3.v[i];
  }
  const M3 R1p = m3_mul(R_t, R);
  double r31 = R1p.m[2][0], r32 = R1p.m[2][1];
  double hyp = sqrt(r31 * r31 + r32 * r32);
  if (hyp < 1e-100) {
    r31 = 1;
    r32 = 0;
    hyp = 1;
  }
  const M3 R_z = {{{r31 / hyp, -r32 / hyp, 0}, {r32 / hyp, r31 / hyp, 0}, {0, 0, 1}}};
  const M3 R_trans = m3_mul(R1p, R_z);
  const double sin_gamma = -R_trans.m[0][1], cos_gamma = R_trans.m[1][1];
  const M3 R_gamma = {{{cos_gamma, -sin_gamma, 0}, {sin_gamma, cos_gamma, 0}, {0, 0, 1}}};
  const double sin_beta = -R_trans.m[2][0], cos_beta = R_trans.m[2][2];
  const double t_initial = atan2(sin_beta, cos_beta);
  const M3 R_zt = m3_t(R_z);
  V3 p_tr[4];
  M3 F[4], avg;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) avg.m[i][j] = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    p_tr[k] = mv(R_zt, p[k]);
    F[k] = calculate_F(mv(R_t, v[k]));
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) avg.m[i][j] += F[k].m[i][j];
  }
  M3 ImA;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) ImA.m[i][j] = (i == j ? 1.0 : 0.0) - avg.m[i][j] * 0.25;
  M3 G = m3_inv(ImA);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) G.m[i][j] *= 0.25;
  const M3 M1 = {{{0, 0, 2}, {0, 0, 0}, {-2, 0, 0}}};
  const M3 M2 = {{{-1, 0, 0}, {0, 1, 0}, {0, 0, -1}}};
  V3 b0 = {{0, 0, 0}}, b1 = b0, b2 = b0;
  V3 g0[4], g1[4], g2[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    g0[k] = mv(R_gamma, p_tr[k]);
    g1[k] = mv(R_gamma, mv(M1, p_tr[k]));
    g2[k] = mv(R_gamma, mv(M2, p_tr[k]));
    b0 = v_add(b0, v_sub(mv(F[k], g0[k]), g0[k]));  // (F - I) x
    b1 = v_add(b1, v_sub(mv(F[k], g1[k]), g1[k]));
    b2 = v_add(b2, v_sub(mv(F[k], g2[k]), g2[k]));
  }
  const V3 b0_ = mv(G, b0), b1_ = mv(G, b1), b2_ = mv(G, b2);
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const V3 x0 = v_add(g0[k], b0_), x1 = v_add(g1[k], b1_), x2 = v_add(g2[k], b2_);
    const V3 c0 = v_sub(x0, mv(F[k], x0)), c1 = v_sub(x1, mv(F[k], x1)), c2 = v_sub(x2, mv(F[k], x2));
    a0 += v_dot(c0, c0);
    a1 += 2 * v_dot(c0, c1);
    a2 += v_dot(c1, c1) + 2 * v_dot(c0, c2);
    a3 += 2 * v_dot(c1, c2);
    a4 += v_dot(c2, c2);
  }
  const double poly[5] = {a1, 2 * a2 - 4 * a0, 3 * a3 - 3 * a1, 4 * a4 - 2 * a2, -a3};
  if (stamps) stamps[10] = wall_clock64();
  double minimum = 0;
  int n_minima = 0;
  if constexpr (WAVE) {
    // the quartic's brackets on their lane groups; each group tests its own root
    // (second-derivative sign, distance from t_initial: upstream's loop body) and
    // the results are gathered in bracket order (= upstream's root order)
    double d3[4], d2[3], d1[2];
    for (int i = 0; i < 4; i++) d3[i] = (i + 1) * poly[i + 1];
    for (int i = 0; i < 3; i++) d2[i] = (i + 1) * d3[i + 1];
    for (int i = 0; i < 2; i++) d1[i] = (i + 1) * d2[i + 1];
    double r1[4] = {0, 0, 0, 0}, r2[4] = {0, 0, 0, 0}, r3[4] = {0, 0, 0, 0};
    int n1 = 0;
    if (!(fabs(d1[0]) > 1000 * fabs(d1[1]))) {
      r1[0] = -d1[0] / d1[1];
      n1 = 1;
    }
    const int n2 = solve_poly_level_wave(d2, 2, r1, n1, r2);
    if (stamps) stamps[11] = wall_clock64();
    const int n3 = solve_poly_level_wave(d3, 3, r2, n2, r3);
    if (stamps) stamps[12] = wall_clock64();
    double rt;
    int has;
    solve_poly_level_wave_lane(poly, 4, r3, n3, rt, has);
    if (stamps) stamps[13] = wall_clock64();
    int is_min = 0;
    if (has) {
      const double t1 = rt, t2 = t1 * t1, t3 = t1 * t2, t4 = t1 * t3, t5 = t1 * t4;
      if (a2 - 2 * a0 + (3 * a3 - 6 * a1) * t1 + (6 * a4 - 8 * a2 + 10 * a0) * t2 + (-8 * a3 + 6 * a1) * t3 +
              (-6 * a4 + 3 * a2) * t4 + a3 * t5 >= 0)
        is_min = fabs(2 * atan(rt) - t_initial) > 0.1;
    }
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) {
      const double r = readlane_f64(rt, 16 * s2);
      if (__builtin_amdgcn_readlane(is_min, 16 * s2)) {
        minimum = r;
        n_minima++;
      }
    }
  } else {
  double roots[4] = {0, 0, 0, 0};
  const int n_roots = solve_quartic_approx<false>(poly, roots, sub);
#pragma unroll
  for (int i = 0; i < 4; i++) {  // (static slots: the roots stay in registers)
    if (i >= n_roots) break;
    const double t1 = roots[i], t2 = t1 * t1, t3 = t1 * t2, t4 = t1 * t3, t5 = t1 * t4;
    if (a2 - 2 * a0 + (3 * a3 - 6 * a1) * t1 + (6 * a4 - 8 * a2 + 10 * a0) * t2 + (-8 * a3 + 6 * a1) * t3 +
            (-6 * a4 + 3 * a2) * t4 + a3 * t5 >= 0) {
      const double tt = 2 * atan(roots[i]);
      if (fabs(tt - t_initial) > 0.1) {
        minimum = roots[i];
        n_minima++;
      }
    }
  }
  }
  if (stamps) stamps[14] = wall_clock64();
  if (n_minima != 1) return false;
  const double tm = minimum;
  M3 Rb;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) Rb.m[i][j] = ((M2.m[i][j] * tm + M1.m[i][j]) * tm + (i == j ? 1.0 : 0.0)) / (1 + tm * tm);
  *out = m3_mul(m3_mul(m3_mul(m3_t(R_t), R_gamma), Rb), R_zt);
  return true;
}

// estimate_tag_pose: writes R (row-major), t and the winning error.
// WAVE = false: sub is this lane's index in the detection's quad (see
// solve_poly_level); all four lanes return the same pose.  WAVE = true: the whole
// wave works on one detection (solve_poly_level_wave); every lane returns it.
template <bool WAVE = false>
__device__ void estimate_tag_pose(const double H[9], const double corners[4][2], double fx, double fy, double cx,
                                  double cy, double tagsize, double* R_out, double* t_out, double* err_out, int sub,
                                  uint64_t* stamps = nullptr) {
  if (stamps) stamps[0] = wall_clock64();
  const double s = tagsize / 2.0;
  const V3 p[4] = {{{-s, s, 0}}, {{s, s, 0}}, {{s, -s, 0}}, {{-s, -s, 0}}};
  V3 v[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    v[i].v[0] = (corners[i][0] - cx) / fx;
    v[i].v[1] = (corners[i][1] - cy) / fy;
    v[i].v[2] = 1;
  }
  // homography_to_pose(H, -fx, fy, cx, cy)
  const double nfx = -fx;
  double R20 = H[6], R21 = H[7], TZ = H[8];
  double R00 = (H[0] - cx * R20) / nfx, R01 = (H[1] - cx * R21) / nfx, TX = (H[2] - cx * TZ) / nfx;
  double R10 = (H[3] - cy * R20) / fy, R11 = (H[4] - cy * R21) / fy, TY = (H[5] - cy * TZ) / fy;
  // sqrtf on double arguments: correctly rounded single precision
  const double length1 = (float)sqrt((double)(float)(R00 * R00 + R10 * R10 + R20 * R20));
  const double length2 = (float)sqrt((double)(float)(R01 * R01 + R11 * R11 + R21 * R21));
  double sc = 1.0 / (double)(float)sqrt((double)(float)(length1 * length2));
  if (TZ > 0) sc *= -1;
  R20 *= sc; R21 *= sc; TZ *= sc;
  R00 *= sc; R01 *= sc; TX *= sc;
  R10 *= sc; R11 *= sc; TY *= sc;
  const M3 A = {{{R00, R01, R10 * R21 - R20 * R11}, {R10, R11, R20 * R01 - R00 * R21}, {R20, R21, R00 * R11 - R10 * R01}}};
  M3 R1 = polar3(A);
  if (stamps) stamps[1] = wall_clock64();
  // estimate_pose_for_tag_homography: scale t, then diag(1, -1, -1)
  V3 t1 = {{TX * s, -TY * s, -TZ * s}};
#pragma unroll
  for (int c = 0; c < 3; c++) {
    R1.m[1][c] = -R1.m[1][c];
    R1.m[2][c] = -R1.m[2][c];
  }
  int k1 = 0, k2 = 0;
  const double err1 = orthogonal_iteration<WAVE>(v, p, &t1, &R1, 50, &k1);
  if (stamps) stamps[2] = wall_clock64();
  M3 R2;
  V3 t2 = {{0, 0, 0}};
  double err2 = HUGE_VAL;
  const bool amb = fix_pose_ambiguities<WAVE>(v, p, t1, R1, &R2, sub, stamps);
  if (stamps) stamps[3] = wall_clock64();
  if (amb) err2 = orthogonal_iteration<WAVE>(v, p, &t2, &R2, 50, &k2);
  if (stamps) {
    stamps[4] = wall_clock64();
    stamps[8] = k1;
    stamps[9] = k2;
  }
  const bool second = !(err1 <= err2);
  const M3& R = second ? R2 : R1;
  const V3& t = second ? t2 : t1;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) R_out[i * 3 + j] = R.m[i][j];
#pragma unroll
  for (int i = 0; i < 3; i++) t_out[i] = t.v[i];
  err_out[0] = err1;
  err_out[1] = err2;
}

}  // namespace pose
}  // namespace at

// back to the translation unit's -ffp-contract=off for everything after this header
#pragma clang fp contract(off)
