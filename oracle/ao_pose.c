/*
 * ao_pose.c -- TEST INFRASTRUCTURE (CPU oracle).  Restatement of the tag pose
 * step the reference node runs on every detection (§8 row A23):
 *
 *   estimate_tag_pose(&info_, &pose)      apriltags_cuda_detector.cu:425-436
 *   transformCameraToRobot(t)             apriltags_cuda_detector.cu:595-599
 *   std::sort by |t|                      apriltags_cuda_detector.cu:441-462
 *
 * estimate_tag_pose lives in the un-vendored third-party AprilTag library
 * (AprilRobotics/apriltag 3.x, apriltag_pose.c + common/homography.c, not in
 * /root/reference).  Restated here from its published algorithm: homography
 * pose initialisation (homography_to_pose with camera looking down -Z, sqrtf
 * column norms, polar decomposition), Lu/Hager/Mjolsness orthogonal
 * iteration (50 steps), Schweighofer & Pinz second-minimum search
 * (fix_pose_ambiguities, quartic via solve_poly_approx), and the smaller of
 * the two object-space errors wins.  Parity against the upstream library is
 * UNPINNED (no fixture in the reference holds a pose); the product is
 * checked against this file, which deliberately uses a different SVD method
 * (one-sided Jacobi) from the device code (closed-form polar factors).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use it.
 */
#include <math.h>
#include <string.h>

#include "ao_oracle.h"

typedef struct { double m[3][3]; } M3;
typedef struct { double v[3]; } V3;

static M3 m3_zero(void) { M3 r; memset(&r, 0, sizeof r); return r; }
static M3 m3_eye(void) { M3 r = m3_zero(); r.m[0][0] = r.m[1][1] = r.m[2][2] = 1; return r; }
static M3 m3_mul(M3 a, M3 b) {
  M3 r = m3_zero();
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      for (int k = 0; k < 3; k++) r.m[i][j] += a.m[i][k] * b.m[k][j];
  return r;
}
static M3 m3_t(M3 a) {
  M3 r;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r.m[i][j] = a.m[j][i];
  return r;
}
static M3 m3_sub(M3 a, M3 b) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) a.m[i][j] -= b.m[i][j];
  return a;
}
static M3 m3_scale(M3 a, double s) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) a.m[i][j] *= s;
  return a;
}
static V3 mv(M3 a, V3 x) {
  V3 r;
  for (int i = 0; i < 3; i++) r.v[i] = a.m[i][0] * x.v[0] + a.m[i][1] * x.v[1] + a.m[i][2] * x.v[2];
  return r;
}
static V3 v_add(V3 a, V3 b) { for (int i = 0; i < 3; i++) a.v[i] += b.v[i]; return a; }
static V3 v_sub(V3 a, V3 b) { for (int i = 0; i < 3; i++) a.v[i] -= b.v[i]; return a; }
static V3 v_scale(V3 a, double s) { for (int i = 0; i < 3; i++) a.v[i] *= s; return a; }
static double v_dot(V3 a, V3 b) { return a.v[0] * b.v[0] + a.v[1] * b.v[1] + a.v[2] * b.v[2]; }
static V3 v_cross(V3 a, V3 b) {
  V3 r = {{a.v[1] * b.v[2] - a.v[2] * b.v[1], a.v[2] * b.v[0] - a.v[0] * b.v[2], a.v[0] * b.v[1] - a.v[1] * b.v[0]}};
  return r;
}
static double m3_det(M3 a) {
  return a.m[0][0] * (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]) -
         a.m[0][1] * (a.m[1][0] * a.m[2][2] - a.m[1][2] * a.m[2][0]) +
         a.m[0][2] * (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]);
}
static M3 m3_inv(M3 a) {
  const double d = m3_det(a);
  M3 r;
  r.m[0][0] = (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]) / d;
  r.m[0][1] = (a.m[0][2] * a.m[2][1] - a.m[0][1] * a.m[2][2]) / d;
  r.m[0][2] = (a.m[0][1] * a.m[1][2] - a.m[0][2] * a.m[1][1]) / d;
  r.m[1][0] = (a.m[1][2] * a.m[2][0] - a.m[1][0] * a.m[2][2]) / d;
  r.m[1][1] = (a.m[0][0] * a.m[2][2] - a.m[0][2] * a.m[2][0]) / d;
  r.m[1][2] = (a.m[0][2] * a.m[1][0] - a.m[0][0] * a.m[1][2]) / d;
  r.m[2][0] = (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]) / d;
  r.m[2][1] = (a.m[0][1] * a.m[2][0] - a.m[0][0] * a.m[2][1]) / d;
  r.m[2][2] = (a.m[0][0] * a.m[1][1] - a.m[0][1] * a.m[1][0]) / d;
  return r;
}

/* One-sided (Hestenes) Jacobi SVD of a 3x3 matrix: A = U diag(s) V'.  A zero
 * singular value leaves U's column undefined; it is completed to an
 * orthonormal basis (its sign is arbitrary, as in any SVD). */
static void svd3(M3 a, M3 *U, M3 *V) {
  M3 u = a, v = m3_eye();
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = 0;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        double alpha = 0, beta = 0, gamma = 0;
        for (int i = 0; i < 3; i++) {
          alpha += u.m[i][p] * u.m[i][p];
          beta += u.m[i][q] * u.m[i][q];
          gamma += u.m[i][p] * u.m[i][q];
        }
        if (gamma == 0) continue;
        const double conv = fabs(gamma) / sqrt(alpha * beta);
        if (!(conv > 1e-17)) continue;
        if (conv > off) off = conv;
        const double zeta = (beta - alpha) / (2 * gamma);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
        const double c = 1 / sqrt(1 + t * t), s = c * t;
        for (int i = 0; i < 3; i++) {
          const double up = u.m[i][p], uq = u.m[i][q];
          u.m[i][p] = c * up - s * uq;
          u.m[i][q] = s * up + c * uq;
          const double vp = v.m[i][p], vq = v.m[i][q];
          v.m[i][p] = c * vp - s * vq;
          v.m[i][q] = s * vp + c * vq;
        }
      }
    if (off < 1e-16) break;
  }
  double sv[3];
  for (int j = 0; j < 3; j++) sv[j] = sqrt(u.m[0][j] * u.m[0][j] + u.m[1][j] * u.m[1][j] + u.m[2][j] * u.m[2][j]);
  /* order singular values descending (matd_svd convention) */
  int ord[3] = {0, 1, 2};
  for (int i = 0; i < 3; i++)
    for (int j = i + 1; j < 3; j++)
      if (sv[ord[j]] > sv[ord[i]]) { int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
  const double smax = sv[ord[0]];
  M3 Uo = m3_zero(), Vo = m3_zero();
  for (int k = 0; k < 3; k++) {
    const int j = ord[k];
    for (int i = 0; i < 3; i++) {
      Vo.m[i][k] = v.m[i][j];
      Uo.m[i][k] = sv[j] > 1e-14 * smax ? u.m[i][j] / sv[j] : 0;
    }
  }
  /* complete rank-deficient U */
  for (int k = 0; k < 3; k++) {
    if (sv[ord[k]] > 1e-14 * smax) continue;
    V3 c0 = {{Uo.m[0][(k + 1) % 3], Uo.m[1][(k + 1) % 3], Uo.m[2][(k + 1) % 3]}};
    V3 c1 = {{Uo.m[0][(k + 2) % 3], Uo.m[1][(k + 2) % 3], Uo.m[2][(k + 2) % 3]}};
    V3 n = v_cross(c0, c1);
    const double nn = sqrt(v_dot(n, n));
    for (int i = 0; i < 3; i++) Uo.m[i][k] = nn > 0 ? n.v[i] / nn : (i == k);
  }
  *U = Uo;
  *V = Vo;
}

/* homography_to_pose(H, -fx, fy, cx, cy) (common/homography.c), 3x4 [R|t]. */
static void homography_to_pose(const double H[9], double fx, double fy, double cx, double cy, M3 *R, V3 *t) {
  double R20 = H[6], R21 = H[7], TZ = H[8];
  double R00 = (H[0] - cx * R20) / fx, R01 = (H[1] - cx * R21) / fx, TX = (H[2] - cx * TZ) / fx;
  double R10 = (H[3] - cy * R20) / fy, R11 = (H[4] - cy * R21) / fy, TY = (H[5] - cy * TZ) / fy;
  /* column norms in single precision, as upstream (sqrtf on a double argument) */
  const double length1 = sqrtf((float)(R00 * R00 + R10 * R10 + R20 * R20));
  const double length2 = sqrtf((float)(R01 * R01 + R11 * R11 + R21 * R21));
  double s = 1.0 / sqrtf((float)(length1 * length2));
  if (TZ > 0) s *= -1; /* tag in front of a camera that looks down -Z */
  R20 *= s; R21 *= s; TZ *= s;
  R00 *= s; R01 *= s; TX *= s;
  R10 *= s; R11 *= s; TY *= s;
  const double R02 = R10 * R21 - R20 * R11;
  const double R12 = R20 * R01 - R00 * R21;
  const double R22 = R00 * R11 - R10 * R01;
  M3 A = {{{R00, R01, R02}, {R10, R11, R12}, {R20, R21, R22}}};
  M3 U, V;
  svd3(A, &U, &V);
  *R = m3_mul(U, m3_t(V)); /* polar decomposition */
  t->v[0] = TX; t->v[1] = TY; t->v[2] = TZ;
}

static M3 calculate_F(V3 v) {
  M3 F;
  const double inner = v_dot(v, v);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) F.m[i][j] = v.v[i] * v.v[j] / inner;
  return F;
}

/* orthogonal_iteration (apriltag_pose.c): returns the object-space error. */
static double orthogonal_iteration(const V3 *v, const V3 *p, V3 *t, M3 *R, int n_points, int n_steps) {
  V3 p_mean = {{0, 0, 0}};
  for (int i = 0; i < n_points; i++) p_mean = v_add(p_mean, p[i]);
  p_mean = v_scale(p_mean, 1.0 / n_points);
  V3 p_res[4];
  for (int i = 0; i < n_points; i++) p_res[i] = v_sub(p[i], p_mean);
  M3 F[4], avg_F = m3_zero();
  for (int i = 0; i < n_points; i++) {
    F[i] = calculate_F(v[i]);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) avg_F.m[r][c] += F[i].m[r][c];
  }
  avg_F = m3_scale(avg_F, 1.0 / n_points);
  const M3 I3 = m3_eye();
  const M3 M1_inv = m3_inv(m3_sub(I3, avg_F));
  double prev_error = HUGE_VAL;
  for (int it = 0; it < n_steps; it++) {
    V3 M2 = {{0, 0, 0}};
    for (int j = 0; j < n_points; j++) M2 = v_add(M2, mv(m3_sub(F[j], I3), mv(*R, p[j])));
    M2 = v_scale(M2, 1.0 / n_points);
    *t = mv(M1_inv, M2);
    V3 q[4], q_mean = {{0, 0, 0}};
    for (int j = 0; j < n_points; j++) {
      q[j] = mv(F[j], v_add(mv(*R, p[j]), *t));
      q_mean = v_add(q_mean, q[j]);
    }
    q_mean = v_scale(q_mean, 1.0 / n_points);
    M3 M3m = m3_zero();
    for (int j = 0; j < n_points; j++) {
      const V3 d = v_sub(q[j], q_mean);
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) M3m.m[r][c] += d.v[r] * p_res[j].v[c];
    }
    M3 U, V;
    svd3(M3m, &U, &V);
    *R = m3_mul(U, m3_t(V));
    if (m3_det(*R) < 0)
      for (int r = 0; r < 3; r++) R->m[r][2] = -R->m[r][2];
    double error = 0;
    for (int j = 0; j < 4; j++) {
      const V3 e = mv(m3_sub(I3, F[j]), v_add(mv(*R, p[j]), *t));
      error += v_dot(e, e);
    }
    prev_error = error;
  }
  return prev_error;
}

static double polyval(const double *p, int degree, double x) {
  double ret = 0;
  for (int i = 0; i <= degree; i++) ret += p[i] * pow(x, i);
  return ret;
}

/* solve_poly_approx (apriltag_pose.c): real roots in [-1000, 1000] by
 * recursion on the derivative's roots + safeguarded Newton/bisection. */
static void solve_poly_approx(const double *p, int degree, double *roots, int *n_roots) {
  const double MAX_ROOT = 1000;
  if (degree == 1) {
    if (fabs(p[0]) > MAX_ROOT * fabs(p[1])) {
      *n_roots = 0;
    } else {
      roots[0] = -p[0] / p[1];
      *n_roots = 1;
    }
    return;
  }
  double p_der[8];
  for (int i = 0; i < degree; i++) p_der[i] = (i + 1) * p[i + 1];
  double der_roots[8];
  int n_der_roots;
  solve_poly_approx(p_der, degree - 1, der_roots, &n_der_roots);
  *n_roots = 0;
  for (int i = 0; i <= n_der_roots; i++) {
    const double min = i == 0 ? -MAX_ROOT : der_roots[i - 1];
    const double max = i == n_der_roots ? MAX_ROOT : der_roots[i];
    if (polyval(p, degree, min) * polyval(p, degree, max) < 0) {
      double lower, upper;
      if (polyval(p, degree, min) < polyval(p, degree, max)) {
        lower = min;
        upper = max;
      } else {
        lower = max;
        upper = min;
      }
      double root = 0.5 * (lower + upper);
      double dx_old = upper - lower;
      double dx = dx_old;
      double f = polyval(p, degree, root);
      double df = polyval(p_der, degree - 1, root);
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
      roots[(*n_roots)++] = root;
    } else if (polyval(p, degree, max) == 0) {
      roots[(*n_roots)++] = max;
    }
  }
}

/* fix_pose_ambiguities (apriltag_pose.c): the second local minimum of the
 * object-space error over the rotation about the line of sight, or 0. */
static int fix_pose_ambiguities(const V3 *v, const V3 *p, V3 t, M3 R, int n_points, M3 *out) {
  const M3 I3 = m3_eye();
  const V3 R_t_3 = v_scale(t, 1.0 / sqrt(v_dot(t, t)));
  const V3 e_x = {{1, 0, 0}};
  V3 R_t_1 = v_sub(e_x, v_scale(R_t_3, v_dot(e_x, R_t_3)));
  R_t_1 = v_scale(R_t_1, 1.0 / sqrt(v_dot(R_t_1, R_t_1)));
  const V3 R_t_2 = v_cross(R_t_3, R_t_1);
  const M3 R_t = {{{R_t_1.v[0], R_t_1.v[1], R_t_1.v[2]},
                   {R_t_2.v[0], R_t_2.v[1], R_t_2.v[2]},
                   {R_t_3.v[0], R_t_3.v[1], R_t_3.v[2]}}};
  const M3 R_1_prime = m3_mul(R_t, R);
  double r31 = R_1_prime.m[2][0], r32 = R_1_prime.m[2][1];
  double hyp = sqrt(r31 * r31 + r32 * r32);
  if (hyp < 1e-100) {
    r31 = 1;
    r32 = 0;
    hyp = 1;
  }
  const M3 R_z = {{{r31 / hyp, -r32 / hyp, 0}, {r32 / hyp, r31 / hyp, 0}, {0, 0, 1}}};
  const M3 R_trans = m3_mul(R_1_prime, R_z);
  const double sin_gamma = -R_trans.m[0][1], cos_gamma = R_trans.m[1][1];
  const M3 R_gamma = {{{cos_gamma, -sin_gamma, 0}, {sin_gamma, cos_gamma, 0}, {0, 0, 1}}};
  const double sin_beta = -R_trans.m[2][0], cos_beta = R_trans.m[2][2];
  const double t_initial = atan2(sin_beta, cos_beta);
  V3 v_trans[4], p_trans[4];
  M3 F_trans[4], avg_F = m3_zero();
  for (int i = 0; i < n_points; i++) {
    p_trans[i] = mv(m3_t(R_z), p[i]);
    v_trans[i] = mv(R_t, v[i]);
    F_trans[i] = calculate_F(v_trans[i]);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) avg_F.m[r][c] += F_trans[i].m[r][c];
  }
  avg_F = m3_scale(avg_F, 1.0 / n_points);
  const M3 G = m3_scale(m3_inv(m3_sub(I3, avg_F)), 1.0 / n_points);
  const M3 M1 = {{{0, 0, 2}, {0, 0, 0}, {-2, 0, 0}}};
  const M3 M2 = {{{-1, 0, 0}, {0, 1, 0}, {0, 0, -1}}};
  V3 b0 = {{0, 0, 0}}, b1 = b0, b2 = b0;
  for (int i = 0; i < n_points; i++) {
    const M3 FmI = m3_sub(F_trans[i], I3);
    b0 = v_add(b0, mv(FmI, mv(R_gamma, p_trans[i])));
    b1 = v_add(b1, mv(FmI, mv(R_gamma, mv(M1, p_trans[i]))));
    b2 = v_add(b2, mv(FmI, mv(R_gamma, mv(M2, p_trans[i]))));
  }
  const V3 b0_ = mv(G, b0), b1_ = mv(G, b1), b2_ = mv(G, b2);
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
  for (int i = 0; i < n_points; i++) {
    const M3 ImF = m3_sub(I3, F_trans[i]);
    const V3 c0 = mv(ImF, v_add(mv(R_gamma, p_trans[i]), b0_));
    const V3 c1 = mv(ImF, v_add(mv(R_gamma, mv(M1, p_trans[i])), b1_));
    const V3 c2 = mv(ImF, v_add(mv(R_gamma, mv(M2, p_trans[i])), b2_));
    a0 += v_dot(c0, c0);
    a1 += 2 * v_dot(c0, c1);
    a2 += v_dot(c1, c1) + 2 * v_dot(c0, c2);
    a3 += 2 * v_dot(c1, c2);
    a4 += v_dot(c2, c2);
  }
  const double poly[5] = {a1, 2 * a2 - 4 * a0, 3 * a3 - 3 * a1, 4 * a4 - 2 * a2, -a3};
  double roots[4];
  int n_roots = 0;
  solve_poly_approx(poly, 4, roots, &n_roots);
  double minima[4];
  int n_minima = 0;
  for (int i = 0; i < n_roots; i++) {
    const double t1 = roots[i], t2 = t1 * t1, t3 = t1 * t2, t4 = t1 * t3, t5 = t1 * t4;
    if (a2 - 2 * a0 + (3 * a3 - 6 * a1) * t1 + (6 * a4 - 8 * a2 + 10 * a0) * t2 + (-8 * a3 + 6 * a1) * t3 +
            (-6 * a4 + 3 * a2) * t4 + a3 * t5 >= 0) {
      const double tt = 2 * atan(roots[i]);
      if (fabs(tt - t_initial) > 0.1) minima[n_minima++] = roots[i];
    }
  }
  if (n_minima != 1) return 0; /* none, or ambiguous (upstream logs and gives up) */
  const double tm = minima[0];
  M3 R_beta = m3_scale(M2, tm);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R_beta.m[r][c] += M1.m[r][c];
  R_beta = m3_scale(R_beta, tm);
  R_beta.m[0][0] += 1;
  R_beta.m[1][1] += 1;
  R_beta.m[2][2] += 1;
  R_beta = m3_scale(R_beta, 1 / (1 + tm * tm));
  *out = m3_mul(m3_mul(m3_mul(m3_t(R_t), R_gamma), R_beta), m3_t(R_z));
  return 1;
}

int ao_estimate_tag_pose(const double H[9], const double corners[4][2], double fx, double fy, double cx, double cy,
                         double tagsize, double R_out[9], double t_out[3], double err_out[2]) {
  const double scale = tagsize / 2.0;
  const V3 p[4] = {{{-scale, scale, 0}}, {{scale, scale, 0}}, {{scale, -scale, 0}}, {{-scale, -scale, 0}}};
  V3 v[4];
  for (int i = 0; i < 4; i++) {
    v[i].v[0] = (corners[i][0] - cx) / fx;
    v[i].v[1] = (corners[i][1] - cy) / fy;
    v[i].v[2] = 1;
  }
  /* estimate_pose_for_tag_homography: fix = diag(1,-1,-1) applied to [R|t*scale] */
  M3 R1;
  V3 t1;
  homography_to_pose(H, -fx, fy, cx, cy, &R1, &t1);
  t1 = v_scale(t1, scale);
  for (int c = 0; c < 3; c++) {
    R1.m[1][c] = -R1.m[1][c];
    R1.m[2][c] = -R1.m[2][c];
  }
  t1.v[1] = -t1.v[1];
  t1.v[2] = -t1.v[2];
  const double err1 = orthogonal_iteration(v, p, &t1, &R1, 4, 50);
  M3 R2;
  V3 t2 = {{0, 0, 0}};
  double err2 = HUGE_VAL;
  if (fix_pose_ambiguities(v, p, t1, R1, 4, &R2)) err2 = orthogonal_iteration(v, p, &t2, &R2, 4, 50);
  const int second = !(err1 <= err2);
  const M3 *R = second ? &R2 : &R1;
  const V3 *t = second ? &t2 : &t1;
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R_out[r * 3 + c] = R->m[r][c];
  for (int i = 0; i < 3; i++) t_out[i] = t->v[i];
  err_out[0] = err1;
  err_out[1] = err2;
  return second;
}
