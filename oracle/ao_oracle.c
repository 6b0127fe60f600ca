/*
 * ao_oracle.c -- CPU ORACLE (test infrastructure only; see ao_oracle.h).
 *
 * Plain-C restatement of the reference AprilTag pipeline.  Reference paths are
 * relative to /root/reference/src/apriltags_cuda/.  Compiled with
 * -ffp-contract=off: every float/double expression is evaluated exactly as
 * written (no fused multiply-add), which is also how the HIP kernels are built,
 * so the two agree bit-for-bit.
 *
 * libm transcendental calls of the reference (atan2f, cosf, sinf, hypotf) are
 * replaced by the deterministic functions det_* below (double-precision
 * evaluations -- fdlibm / Cephes polynomials -- rounded to float).  They are within 1 float ulp of
 * libm; the HIP path evaluates the identical operation sequence.
 */
#include "ao_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* deterministic math                                                          */
/* ------------------------------------------------------------------------- */
static const double kPi = 3.14159265358979323846;
static const double kPio2 = 1.57079632679489661923;

/* atan2 with one division (ros_vision_amd/csrc/at_detmath.h det_atan2, the same
 * operation sequence): octant reduction t = (b - a) / (a + b) or b / a, |t| <= tan(pi/8),
 * fdlibm's odd minimax polynomial for atan on |t| < 7/16 (s_atan.c) by explicit fma
 * (correctly rounded), the octant constants in two parts. */
static const double kAtanT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                                  1.42857142725034663711e-01, -1.11111104054623557880e-01,
                                  9.09088713343650656196e-02, -7.69187620504482999495e-02,
                                  6.66107313738753120669e-02, -5.83357013379057348645e-02,
                                  4.97687799461593236017e-02, -3.65315727442169155270e-02,
                                  1.62858201153657823623e-02};
static double det_atan2(double y, double x) {
  const double ax = fabs(x), ay = fabs(y);
  const int sw = ay > ax;
  const double a = sw ? ay : ax, b = sw ? ax : ay;
  if (a == 0.0) return 0.0;
  const int s = b > 0.41421356237309504880 * a;
  const double t = (s ? b - a : b) / (s ? a + b : a);
  const double z = t * t, w = z * z;
  double s1 = fma(w, kAtanT[10], kAtanT[8]);
  s1 = fma(w, s1, kAtanT[6]);
  s1 = fma(w, s1, kAtanT[4]);
  s1 = fma(w, s1, kAtanT[2]);
  s1 = fma(w, s1, kAtanT[0]);
  s1 = z * s1;
  double s2 = fma(w, kAtanT[9], kAtanT[7]);
  s2 = fma(w, s2, kAtanT[5]);
  s2 = fma(w, s2, kAtanT[3]);
  s2 = fma(w, s2, kAtanT[1]);
  s2 = w * s2;
  const double hi = s ? 7.85398163397448278999e-01 : 0.0, lo = s ? 3.06161699786838301793e-17 : 0.0;
  double r = hi - ((t * (s1 + s2) - lo) - t);
  if (sw) r = (1.57079632679489655800e+00 - r) + 6.12323399573676603587e-17;
  if (x < 0.0) r = (3.14159265358979311600e+00 - r) + 1.22464679914735317723e-16;
  return y < 0.0 ? -r : r;
}

/* Sensitivity hook (tools/fp_sensitivity.py, tests only): bit k of ao_fp_perturb
 * (0 atan2f, 1 hypotf, 2 cosf, 3 sinf) moves the results of that function one
 * ulp, towards -inf when bit 8 is set, else towards +inf; with bit 9 set, results
 * that are exact (a faithful libm returns them unchanged: hypotf of a Pythagorean
 * pair, atan2f(0, x > 0), sinf(0), cosf(0)) are left alone.  0 = exact restatement. */
static int ao_fp_perturb = 0;
void ao_set_fp_perturb(int mask) { ao_fp_perturb = mask; }
static float fp_perturb(float v, int bit, int exact) {
  if (!(ao_fp_perturb & (1 << bit))) return v;
  if (exact && (ao_fp_perturb & 512)) return v;
  return nextafterf(v, (ao_fp_perturb & 256) ? -INFINITY : INFINITY);
}

float ao_det_atan2f(float y, float x) {
  return fp_perturb((float)det_atan2((double)y, (double)x), 0, y == 0.0f && x > 0.0f);
}


static const double kSinC[6] = {1.58962301576546568060E-10, -2.50507477628578072866E-8,
                                2.75573136213857245213E-6,  -1.98412698295895385996E-4,
                                8.33333333332211858878E-3,  -1.66666666666666307295E-1};
static const double kCosC[6] = {-1.13585365213876817300E-11, 2.08757008419747316778E-9,
                                -2.75573141792967388112E-7,  2.48015872888517045348E-5,
                                -1.38888888888730564116E-3,  4.16666666666665929218E-2};
static double det_sin_poly(double x) {
  double z = x * x, p = kSinC[0];
  for (int i = 1; i < 6; i++) p = p * z + kSinC[i];
  return x + x * z * p;
}
static double det_cos_poly(double x) {
  double z = x * x, p = kCosC[0];
  for (int i = 1; i < 6; i++) p = p * z + kCosC[i];
  return 1.0 - 0.5 * z + z * z * p;
}
/* quadrant reduction by pi/2 with a 2-part Cody-Waite constant */
static void det_sincos(double x, double *s, double *c) {
  const double kPio2Hi = 1.57079632673412561417e+00;
  const double kPio2Lo = 6.07710050650619224932e-11;
  double jf = rint(x / kPio2);
  int j = (int)jf;
  double r = (x - jf * kPio2Hi) - jf * kPio2Lo;
  double sr = det_sin_poly(r), cr = det_cos_poly(r);
  switch (j & 3) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
  }
}
float ao_det_cosf(float x) { double s, c; det_sincos((double)x, &s, &c); return fp_perturb((float)c, 2, x == 0.0f); }
float ao_det_sinf(float x) { double s, c; det_sincos((double)x, &s, &c); return fp_perturb((float)s, 3, x == 0.0f); }
float ao_det_hypotf(float a, float b) {
  double x = a, y = b;
  const double d = x * x + y * y, r = sqrt(d);
  return fp_perturb((float)r, 1, r == (double)(float)r && r * r == d);
}
#define det_atan2f ao_det_atan2f
#define det_cosf ao_det_cosf
#define det_sinf ao_det_sinf
#define det_hypotf ao_det_hypotf

/* ------------------------------------------------------------------------- */
/* tag families (third party: apriltag 3.x tag36h11.c, tag25h9.c, tag16h5.c;    */
/* selected by name in setup_tag_family, apriltag_utils.cu:10-32)              */
/* ------------------------------------------------------------------------- */
typedef struct { int id; uint64_t code; } CodeEntry;
static const CodeEntry kCodes36h11[] = {
#include "ao_tag36h11_codes.inc"
};
static const CodeEntry kCodes25h9[] = {
#include "ao_tag25h9_codes.inc"
};
static const CodeEntry kCodes16h5[] = {
#include "ao_tag16h5_codes.inc"
};
/* the classic square families: d x d data cells inside a one-cell black border
 * (width_at_border = d + 2), one white cell outside it (total_width = d + 4),
 * normal border; bits in the 3.x spiral order (bit_x/bit_y of tagXXhY.c) */
typedef struct {
  const char *name;
  int d, nbits, width_at_border, total_width, reversed_border;
  const CodeEntry *codes;
  int ncodes;
  int bitx[64], bity[64];
} Family;
#define AO_NCODES(a) ((int)(sizeof(a) / sizeof((a)[0])))
static Family kFamilies[] = {
    {"tag36h11", 6, 36, 8, 10, 0, kCodes36h11, AO_NCODES(kCodes36h11), {0}, {0}},
    {"tag25h9", 5, 25, 7, 9, 0, kCodes25h9, AO_NCODES(kCodes25h9), {0}, {0}},
    {"tag16h5", 4, 16, 6, 8, 0, kCodes16h5, AO_NCODES(kCodes16h5), {0}, {0}},
};
enum { kNumFamilies = 3, kMaxHamming = 2 }; /* apriltag_detector_add_family: 2 bits corrected */

/* 3.x layout of tagXXhY.c: the upper triangle of the top-left quadrant row by
 * row (y = 1 .. d/2, x = y .. d-y), that block rotated by 90 degrees three more
 * times ((x, y) -> (d+1-y, x)), the centre cell last when d is odd */
static void family_layout(Family *f) {
  int n = 0;
  for (int r = 0; r < 4; r++)
    for (int y = 1; y <= f->d / 2; y++)
      for (int x = y; x <= f->d - y; x++) {
        int xx = x, yy = y;
        for (int i = 0; i < r; i++) { const int t = xx; xx = f->d + 1 - yy; yy = t; }
        f->bitx[n] = xx; f->bity[n] = yy; n++;
      }
  if (f->d & 1) { f->bitx[n] = f->d / 2 + 1; f->bity[n] = f->d / 2 + 1; n++; }
}

static const Family *family_by_name(const char *name) {
  static int init = 0;
  if (!init) {
    for (int i = 0; i < kNumFamilies; i++) family_layout(&kFamilies[i]);
    init = 1;
  }
  if (!name) name = "tag36h11";
  for (int i = 0; i < kNumFamilies; i++)
    if (!strcmp(kFamilies[i].name, name)) return &kFamilies[i];
  return NULL;
}

int ao_family_ncodes(const char *fam) {
  const Family *f = family_by_name(fam);
  return f ? f->ncodes : -1;
}
uint64_t ao_family_code(const char *fam, int i) {
  const Family *f = family_by_name(fam);
  return (f && i >= 0 && i < f->ncodes) ? f->codes[i].code : 0;
}
int ao_family_id(const char *fam, int i) {
  const Family *f = family_by_name(fam);
  return (f && i >= 0 && i < f->ncodes) ? f->codes[i].id : -1;
}
void ao_family_bit(const char *fam, int i, int *x, int *y) {
  const Family *f = family_by_name(fam);
  *x = f ? f->bitx[i] : -1;
  *y = f ? f->bity[i] : -1;
}
int ao_family_nbits(const char *fam) {
  const Family *f = family_by_name(fam);
  return f ? f->nbits : -1;
}

/* apriltag.c rotate90 (3.x): the spiral layout turns a 90-degree rotation into
 * a rotation of the bit string by nbits/4, the centre bit (LSB) fixed for odd d */
uint64_t ao_rotate90_n(uint64_t w, int nbits) {
  int p = nbits;
  uint64_t l = 0;
  if (nbits % 4 == 1) { p = nbits - 1; l = 1; }
  w = ((w >> l) << (p / 4 + l)) | (w >> (3 * p / 4 + l) << l) | (w & l);
  return w & ((1ULL << nbits) - 1);
}
uint64_t ao_rotate90(uint64_t w) { return ao_rotate90_n(w, 36); }

/* ------------------------------------------------------------------------- */
/* state                                                                      */
/* ------------------------------------------------------------------------- */
typedef struct {
  uint16_t min_x, min_y, max_x, max_y;
  uint32_t starting_offset, count;
  int32_t gx_sum, gy_sum;
  int64_t pxgx_plus_pygy_sum;
} Extents; /* MinMaxExtents, line_fit_filter.h:14-59 */

typedef struct {
  int64_t Mxx, Myy, Mxy;
  int32_t Mx, My, W;
  uint32_t blob_index;
} LFP; /* LineFitPoint, line_fit_filter.h:61-83 */

typedef struct {
  float error;
  uint32_t filtered_point_index;
  uint16_t blob_index;
} Peak; /* line_fit_filter.h:99-106 */

struct ao_state {
  ao_params p;
  const Family *fam;
  int W, H, Wd, Hd;
  int min_tag_width;
  int status;
  int n_pts_pairs; /* >= 0: points of the first 4096 pairs (capacity-capped frame) */
  uint8_t *gray, *dec, *thr;
  uint8_t *mm_unf, *mm; /* uchar2 tiles */
  uint32_t *parent, *labels, *sizes;
  uint64_t *plane;      /* dense 4-plane boundary image */
  uint64_t *pts;        /* compacted, then sorted */
  uint64_t *tmp64;
  int n_pts;
  Extents *ext;
  int n_pairs;
  Extents *sel;         /* selected extents (count, starting_offset, bbox) */
  uint64_t *ipts;       /* IndexPoint keys, sorted */
  int n_sel;
  LFP *lfp;
  double *errs, *filt;
  Peak *peaks;
  int n_peaks;
  ao_fitquad *fq;
  int n_fq;
  ao_quad *quads;
  int n_quads;
  ao_detection *dets;
  int n_dets;
  int cap_pts;
  uint64_t *rcodes; /* per quad: sampled code word (debug tap) */
  float *margins;
};

void ao_default_params(ao_params *p, int width, int height) {
  memset(p, 0, sizeof(*p));
  p->width = width;
  p->height = height;
  p->fx = 905.495617; p->fy = 907.909470; p->cx = 609.916016; p->cy = 352.682645;
  p->k1 = 0.059238; p->k2 = -0.075154; p->p1 = -0.003801; p->p2 = 0.001113; p->k3 = 0.0;
  p->min_white_black_diff = 5;
  p->min_cluster_pixels = 5;
  p->max_nmaxima = 10;
  p->max_line_fit_mse = 10.0f;
  p->cos_critical_rad = cos(10.0 * M_PI / 180.0);
  p->decode_sharpening = 0.25;
  p->refine_edges = 1;
}

ao_state *ao_create(const ao_params *p) {
  if (p->width % 8 || p->height % 8) return NULL;
  if ((long)p->width * p->height >= (1L << 22)) return NULL; /* apriltag_gpu.cu:774 */
  const Family *fam = family_by_name(p->family);
  if (!fam) return NULL; /* setup_tag_family: unknown name (apriltag_utils.cu:26-29) */
  ao_state *s = (ao_state *)calloc(1, sizeof(ao_state));
  s->p = *p;
  s->fam = fam;
  s->W = p->width; s->H = p->height; s->Wd = s->W / 2; s->Hd = s->H / 2;
  /* GpuDetector ctor, apriltag_gpu.cu:169-181: width_at_border / quad_decimate 2 */
  s->min_tag_width = fam->width_at_border / 2;
  if (s->min_tag_width < 3) s->min_tag_width = 3;
  size_t npix = (size_t)s->W * s->H, nd = (size_t)s->Wd * s->Hd;
  size_t nt = (size_t)(s->Wd / 4) * (s->Hd / 4);
  s->gray = (uint8_t *)malloc(npix);
  s->dec = (uint8_t *)malloc(nd);
  s->thr = (uint8_t *)malloc(nd);
  s->mm_unf = (uint8_t *)malloc(nt * 2);
  s->mm = (uint8_t *)malloc(nt * 2);
  s->parent = (uint32_t *)malloc(nd * 4);
  s->labels = (uint32_t *)malloc(nd * 4);
  s->sizes = (uint32_t *)malloc(nd * 4);
  s->cap_pts = 4 * (s->Wd - 2) * (s->Hd - 2);
  s->plane = (uint64_t *)malloc((size_t)s->cap_pts * 8);
  s->pts = (uint64_t *)malloc((size_t)s->cap_pts * 8);
  s->tmp64 = (uint64_t *)malloc((size_t)s->cap_pts * 8);
  s->ext = (Extents *)malloc((size_t)s->cap_pts * sizeof(Extents));
  s->sel = (Extents *)malloc((size_t)s->cap_pts * sizeof(Extents));
  s->ipts = (uint64_t *)malloc((size_t)s->cap_pts * 8);
  s->lfp = (LFP *)malloc((size_t)s->cap_pts * sizeof(LFP));
  s->errs = (double *)malloc((size_t)s->cap_pts * 8);
  s->filt = (double *)malloc((size_t)s->cap_pts * 8);
  s->peaks = (Peak *)malloc((size_t)s->cap_pts * sizeof(Peak));
  s->fq = (ao_fitquad *)malloc(4096 * sizeof(ao_fitquad));
  s->quads = (ao_quad *)malloc(4096 * sizeof(ao_quad));
  s->dets = (ao_detection *)malloc(4096 * sizeof(ao_detection));
  s->rcodes = (uint64_t *)calloc(4096, 8);
  s->margins = (float *)calloc(4096, 4);
  return s;
}

void ao_destroy(ao_state *s) {
  if (!s) return;
  free(s->gray); free(s->dec); free(s->thr); free(s->mm_unf); free(s->mm);
  free(s->parent); free(s->labels); free(s->sizes); free(s->plane); free(s->pts);
  free(s->tmp64); free(s->ext); free(s->sel); free(s->ipts); free(s->lfp);
  free(s->errs); free(s->filt); free(s->peaks); free(s->fq); free(s->quads);
  free(s->dets); free(s->rcodes); free(s->margins); free(s);
}

/* ------------------------------------------------------------------------- */
/* Stage 1: gray / decimate / tile min-max / threshold                        */
/* threshold.cu:16-147                                                         */
/* ------------------------------------------------------------------------- */
static void stage_threshold(ao_state *s, const uint8_t *frame, int pixfmt) {
  const int W = s->W, H = s->H, Wd = s->Wd, Hd = s->Hd;
  /* InternalCudaToGreyscaleAndDecimateHalide (threshold.cu:16-40): gray = Y
   * byte; dec = gray at even (row, col) (subsample, no averaging). */
  for (int i = 0; i < W * H; i++) {
    uint8_t g;
    if (pixfmt == 0) {
      g = frame[2 * i];
    } else if (pixfmt == 1) {
      /* OpenCV cvtColor(BGR2YUV_YUYV) Y (apriltags_cuda_detector.cu:401),
       * BT.601 limited range fixed point, ITUR_BT_601_SHIFT = 20 */
      int b = frame[3 * i], gg = frame[3 * i + 1], r = frame[3 * i + 2];
      g = (uint8_t)((269484 * r + 528482 * gg + 102760 * b + (1 << 19) + (16 << 20)) >> 20);
    } else {
      g = frame[i];
    }
    s->gray[i] = g;
    int row = i / W, col = i - W * row;
    if ((row % 2) == 0 && (col % 2) == 0) s->dec[(row / 2) * (W / 2) + col / 2] = g;
  }
  const int TW = Wd / 4, TH = Hd / 4;
  /* InternalBlockMinMax (threshold.cu:60-80) */
  for (int ty = 0; ty < TH; ty++)
    for (int tx = 0; tx < TW; tx++) {
      uint8_t mn = 255, mx = 0;
      for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
          uint8_t v = s->dec[(ty * 4 + r) * Wd + tx * 4 + c];
          if (v < mn) mn = v;
          if (v > mx) mx = v;
        }
      s->mm_unf[2 * (ty * TW + tx)] = mn;
      s->mm_unf[2 * (ty * TW + tx) + 1] = mx;
    }
  /* InternalBlockFilter (threshold.cu:84-118): clipped 3x3 tile neighbourhood */
  for (int ty = 0; ty < TH; ty++)
    for (int tx = 0; tx < TW; tx++) {
      uint8_t mn = 255, mx = 0;
      for (int i = -1; i <= 1; i++)
        for (int j = -1; j <= 1; j++) {
          int rx = tx + i, ry = ty + j;
          if (rx < 0 || rx >= TW || ry < 0 || ry >= TH) continue;
          uint8_t a = s->mm_unf[2 * (ry * TW + rx)], b = s->mm_unf[2 * (ry * TW + rx) + 1];
          if (a < mn) mn = a;
          if (b > mx) mx = b;
        }
      s->mm[2 * (ty * TW + tx)] = mn;
      s->mm[2 * (ty * TW + tx) + 1] = mx;
    }
  /* InternalThreshold (threshold.cu:121-147) */
  for (int y = 0; y < Hd; y++)
    for (int x = 0; x < Wd; x++) {
      int t = (y / 4) * TW + x / 4;
      int mn = s->mm[2 * t], mx = s->mm[2 * t + 1];
      uint8_t res;
      if (mx - mn < s->p.min_white_black_diff) {
        res = 127;
      } else {
        uint8_t thresh = (uint8_t)(mn + (mx - mn) / 2);
        res = (s->dec[y * Wd + x] > thresh) ? 255 : 0;
      }
      s->thr[y * Wd + x] = res;
    }
}

/* ------------------------------------------------------------------------- */
/* Stage 2: connected components (labeling_allegretti_2019_BKE.cu:114-462)     */
/* Restated as a sequential union-find over the same node graph: per 2x2 block */
/* a foreground node (8-connectivity, id = top-left pixel index), a left and   */
/* a right background node (4-connectivity, ids = bottom-left / bottom-right   */
/* pixel index); 127 never joins.  The reference links every root to the       */
/* smaller root (Union, :90-110) and all initial fathers point to smaller ids  */
/* (:212-269), so a component's label is its MINIMUM node id.                  */
/* ------------------------------------------------------------------------- */
static uint32_t uf_find(uint32_t *par, uint32_t n) {
  uint32_t r = n;
  while (par[r] != r) r = par[r];
  while (par[n] != r) { uint32_t nx = par[n]; par[n] = r; n = nx; }
  return r;
}
static void uf_union(uint32_t *par, uint32_t a, uint32_t b) {
  a = uf_find(par, a); b = uf_find(par, b);
  if (a < b) par[b] = a;
  else if (b < a) par[a] = b;
}

static void stage_ccl(ao_state *s) {
  const int Wd = s->Wd, Hd = s->Hd;
  const uint8_t *img = s->thr;
  uint32_t *par = s->parent;
  for (int i = 0; i < Wd * Hd; i++) par[i] = (uint32_t)i;
  for (int row = 0; row < Hd; row += 2)
    for (int col = 0; col < Wd; col += 2) {
      const int idx = row * Wd + col;
      const uint32_t F = (uint32_t)idx, L = (uint32_t)(idx + Wd), R = (uint32_t)(idx + Wd + 1);
      const uint8_t a = img[idx], b = img[idx + 1], c = img[idx + Wd], d = img[idx + Wd + 1];
      const int up = row > 0, left = col > 0, right = col + 2 < Wd;
      /* foreground, InitLabeling P/Q/R/S (:212-250) */
      if (up && left && a == 255 && img[idx - Wd - 1] == 255) uf_union(par, F, F - 2 * Wd - 2);
      if (up && (a == 255 || b == 255) && (img[idx - Wd] == 255 || img[idx - Wd + 1] == 255))
        uf_union(par, F, F - 2 * Wd);
      if (up && right && b == 255 && img[idx - Wd + 2] == 255) uf_union(par, F, F - 2 * Wd + 2);
      /* S: P bits 4/8 are set by a or c (masks 0x777, 0x777<<4), so either
       * left-column pixel joins either of a, c (8-connectivity) */
      if (left && (a == 255 || c == 255) && (img[idx - 1] == 255 || img[idx + Wd - 1] == 255))
        uf_union(par, F, F - 2);
      /* background (:226-269) */
      if (up && a == 0 && img[idx - Wd] == 0) uf_union(par, L, L - 2 * Wd);
      if (up && b == 0 && img[idx - Wd + 1] == 0) uf_union(par, R, R - 2 * Wd);
      if (left && ((a == 0 && img[idx - 1] == 0) || (c == 0 && img[idx + Wd - 1] == 0)))
        uf_union(par, L, L - 1);
      if ((a == 0 && b == 0) || (c == 0 && d == 0)) uf_union(par, R, L);
      (void)Hd;
    }
  /* FinalLabeling (:340-462) */
  memset(s->sizes, 0, (size_t)Wd * Hd * 4);
  for (int row = 0; row < Hd; row += 2)
    for (int col = 0; col < Wd; col += 2) {
      const int idx = row * Wd + col;
      const uint8_t px[4] = {img[idx], img[idx + 1], img[idx + Wd], img[idx + Wd + 1]};
      const int pos[4] = {idx, idx + 1, idx + Wd, idx + Wd + 1};
      int any = 0;
      for (int k = 0; k < 4; k++) any |= (px[k] != 127);
      if (!any) {
        for (int k = 0; k < 4; k++) s->labels[pos[k]] = (uint32_t)pos[k];
        continue;
      }
      const uint32_t fl = uf_find(par, (uint32_t)idx);
      const uint32_t ll = uf_find(par, (uint32_t)(idx + Wd));
      const uint32_t rl = uf_find(par, (uint32_t)(idx + Wd + 1));
      for (int k = 0; k < 4; k++) {
        uint32_t lab = 0;
        if (px[k] == 255) lab = fl;
        else if (px[k] == 0) lab = (k == 0 || k == 2) ? ll : rl;
        s->labels[pos[k]] = lab;
        if (px[k] != 127) s->sizes[lab] += 1;
      }
    }
}

/* ------------------------------------------------------------------------- */
/* Stage 3: boundary points (BlobDiff, apriltag_gpu.cu:226-360; points.h)       */
/* ------------------------------------------------------------------------- */
static inline int qbp_dx(uint64_t k) { static const int t[4] = {1, 1, 0, -1}; return t[k & 3]; }
static inline int qbp_dy(uint64_t k) { static const int t[4] = {0, 1, 1, 1}; return t[k & 3]; }
static inline uint32_t qbp_bx(uint64_t k) { return (uint32_t)((k >> 14) & 0x3ff); }
static inline uint32_t qbp_by(uint64_t k) { return (uint32_t)((k >> 4) & 0x3ff); }
static inline uint32_t qbp_x(uint64_t k) { return (uint32_t)((int32_t)(qbp_bx(k) * 2) + qbp_dx(k)); }
static inline uint32_t qbp_y(uint64_t k) { return (uint32_t)((int32_t)(qbp_by(k) * 2) + qbp_dy(k)); }
static inline int qbp_b2w(uint64_t k) { return (k & 8) != 0; }
static inline int qbp_gx(uint64_t k) { return qbp_b2w(k) ? qbp_dx(k) : -qbp_dx(k); }
static inline int qbp_gy(uint64_t k) { return qbp_b2w(k) ? qbp_dy(k) : -qbp_dy(k); }

static uint64_t make_qbp(uint32_t rep0, uint32_t rep1, uint32_t x, uint32_t y, int dxy, int b2w) {
  uint32_t lo = rep0 < rep1 ? rep0 : rep1, hi = rep0 < rep1 ? rep1 : rep0;
  return ((uint64_t)(hi & 0xfffff) << 44) | ((uint64_t)(lo & 0xfffff) << 24) |
         ((uint64_t)(x & 0x3ff) << 14) | ((uint64_t)(y & 0x3ff) << 4) | ((uint64_t)(b2w ? 1 : 0) << 3) |
         (uint64_t)(dxy & 3);
}

static int cmp_u64(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}

static void stage_boundary(ao_state *s) {
  const int Wd = s->Wd, Hd = s->Hd;
  const int pw = Wd - 2, ph = Hd - 2;
  const size_t plane = (size_t)pw * ph;
  memset(s->plane, 0, plane * 4 * 8);
  const uint8_t *thr = s->thr;
  const uint32_t *lab = s->labels, *sz = s->sizes;
  static const int ddx[4] = {1, 1, 0, -1}, ddy[4] = {0, 1, 1, 1};
  for (int y = 1; y <= Hd - 2; y++)
    for (int x = 1; x <= Wd - 2; x++) {
      const size_t out = (size_t)(x - 1) + (size_t)(y - 1) * pw;
      const uint8_t v0 = thr[y * Wd + x];
      const uint32_t rep0 = lab[y * Wd + x];
      if (v0 == 127 || sz[rep0] < 25) continue; /* all 4 empty (:284-292) */
      for (int dxy = 0; dxy < 4; dxy++) {
        if (dxy == 3) {
          /* dedup of direction 3 (:342-357) */
          const uint8_t vl = thr[y * Wd + x - 1], v2 = thr[(y + 1) * Wd + x];
          const uint32_t rl = lab[y * Wd + x - 1], r2 = lab[(y + 1) * Wd + x];
          if (vl != 127 && v2 != 127 && v2 != vl && x != 1 && sz[rl] >= 25 && sz[r2] >= 25) continue;
        }
        const int x1 = x + ddx[dxy], y1 = y + ddy[dxy];
        const uint8_t v1 = thr[y1 * Wd + x1];
        const uint32_t rep1 = lab[y1 * Wd + x1];
        if ((int)v0 + (int)v1 == 255 && sz[rep1] >= 25)
          s->plane[plane * dxy + out] = make_qbp(rep0, rep1, (uint32_t)x, (uint32_t)y, dxy, v1 > v0);
      }
    }
  /* P1 DeviceSelect::If(NonZero) -- stable compaction (:788-802) */
  int n = 0;
  for (size_t i = 0; i < plane * 4; i++)
    if (s->plane[i]) s->pts[n++] = s->plane[i];
  s->n_pts = n;
  /* P2 stable radix sort on bits [24,64) (:813-825): sort (rep01, index) */
  for (int i = 0; i < n; i++) s->tmp64[i] = ((s->pts[i] >> 24) << 22) | (uint64_t)i;
  qsort(s->tmp64, (size_t)n, 8, cmp_u64);
  for (int i = 0; i < n; i++) s->tmp64[i] = s->pts[s->tmp64[i] & ((1u << 22) - 1)];
  memcpy(s->pts, s->tmp64, (size_t)n * 8);
  /* P3 ReduceByKey -> MinMaxExtents (:829-862, functors :418-454) */
  int q = -1;
  uint64_t prev = ~0ULL;
  for (int i = 0; i < n; i++) {
    uint64_t k = s->pts[i], r01 = (k >> 24) & 0xffffffffffULL;
    uint16_t x = (uint16_t)qbp_x(k), y = (uint16_t)qbp_y(k);
    int gx = qbp_gx(k), gy = qbp_gy(k);
    int64_t pg = (int64_t)qbp_x(k) * gx + (int64_t)qbp_y(k) * gy;
    if (r01 != prev) {
      q++;
      Extents *e = &s->ext[q];
      e->min_x = e->max_x = x; e->min_y = e->max_y = y;
      e->starting_offset = (uint32_t)i; e->count = 1;
      e->gx_sum = gx; e->gy_sum = gy; e->pxgx_plus_pygy_sum = pg;
      prev = r01;
    } else {
      Extents *e = &s->ext[q];
      if (x < e->min_x) e->min_x = x;
      if (x > e->max_x) e->max_x = x;
      if (y < e->min_y) e->min_y = y;
      if (y > e->max_y) e->max_y = y;
      e->count += 1; e->gx_sum += gx; e->gy_sum += gy; e->pxgx_plus_pygy_sum += pg;
    }
  }
  s->n_pairs = q + 1;
}

/* MinMaxExtents::cx/cy/dot (line_fit_filter.h:44-58) */
static double ext_cx(const Extents *e) { return (double)((float)(e->min_x + e->max_x) * 0.5f) + 0.05118; }
static double ext_cy(const Extents *e) { return (double)((float)(e->min_y + e->max_y) * 0.5f) + -0.028581; }
static float ext_dot(const Extents *e) {
  int64_t t = e->pxgx_plus_pygy_sum * 2 - (int64_t)((e->min_x + e->max_x) * e->gx_sum) -
              (int64_t)((e->min_y + e->max_y) * e->gy_sum);
  double a = (double)t * 0.5;
  double b = 0.05118 * (double)e->gx_sum;
  double c = 0.028581 * (double)e->gy_sum;
  return (float)(a - b + c);
}

/* SelectBlobs (apriltag_gpu.cu:522-575) for one family (normal_border_/reversed_border_ from it) */
static int select_blob(const ao_state *s, const Extents *e) {
  const uint32_t minc = s->p.min_cluster_pixels > 24 ? (uint32_t)s->p.min_cluster_pixels : 24u;
  const uint32_t maxc = (uint32_t)(2 * (s->W + s->H)); /* :871 */
  if (e->count < minc) return 0;
  if (e->count > maxc) return 0;
  if ((e->max_x - e->min_x) * (e->max_y - e->min_y) < s->min_tag_width) return 0;
  const int quad_reversed = (double)ext_dot(e) < 0.0;
  const int reversed_border = s->fam->reversed_border, normal_border = !s->fam->reversed_border;
  if (!reversed_border && quad_reversed) return 0;
  if (!normal_border && !quad_reversed) return 0;
  return 1;
}

/* ------------------------------------------------------------------------- */
/* Stage 4: selected extents scan, index points with theta, sort              */
/* apriltag_gpu.cu:873-956, functors :380-412, :577-629                        */
/* ------------------------------------------------------------------------- */
static void stage_select(ao_state *s) {
  const int nq = s->n_pairs;
  uint32_t acc = 0;
  for (int i = 0; i < nq; i++) {
    s->sel[i] = s->ext[i];
    s->sel[i].count = select_blob(s, &s->ext[i]) ? s->ext[i].count : 0;
    s->sel[i].starting_offset = acc; /* SumPoints: exclusive prefix of kept counts */
    acc += s->sel[i].count;
  }
  /* P5: keep points of kept blobs, blob index = run rank masked to 12 bits,
   * theta = llrintf((atan2f(y - cy, x - cx) + pi) * 8e6) */
  int n = 0, q = -1;
  uint64_t prev = ~0ULL;
  const int npts = s->n_pts_pairs >= 0 ? s->n_pts_pairs : s->n_pts;  /* points of the kept pairs */
  for (int i = 0; i < npts; i++) {
    const uint64_t k = s->pts[i], r01 = (k >> 24) & 0xffffffffffULL;
    if (r01 != prev) { q++; prev = r01; }
    const uint32_t bi = (uint32_t)q & 0xfff;
    if (s->sel[bi].count == 0) continue;
    const Extents *e = &s->ext[bi];
    const float dyf = (float)((double)qbp_y(k) - ext_cy(e));
    const float dxf = (float)((double)qbp_x(k) - ext_cx(e));
    const float theta = (float)(((double)det_atan2f(dyf, dxf) + kPi) * 8e6);
    long long ti = (long long)rintf(theta);
    if (ti < 0) ti = 0;
    const uint64_t ip = ((uint64_t)bi << 52) | ((uint64_t)(ti & 0xfffffff) << 24) | (k & 0xffffff);
    s->ipts[n++] = ip;
  }
  s->n_sel = n;
  /* P6 stable sort on bits [24,64) */
  for (int i = 0; i < n; i++) s->tmp64[i] = ((s->ipts[i] >> 24) << 22) | (uint64_t)i;
  qsort(s->tmp64, (size_t)n, 8, cmp_u64);
  for (int i = 0; i < n; i++) s->tmp64[i] = s->ipts[s->tmp64[i] & ((1u << 22) - 1)];
  memcpy(s->ipts, s->tmp64, (size_t)n * 8);
}

/* ------------------------------------------------------------------------- */
/* Stage 5: line-fit points, per-blob prefix sums, errors, filter, peaks      */
/* apriltag_gpu.cu:631-687 (P7), line_fit_filter.cu:22-36, 66-592 (K10)        */
/* ------------------------------------------------------------------------- */
static double fit_line_error(int64_t N, int64_t Mx, int64_t My, int64_t Mxx, int64_t Myy, int64_t Mxy,
                             int64_t W) {
  /* line_fit_filter.cu:22-36 (int64 products wrap like the device code) */
  const int64_t Cxx = (int64_t)((uint64_t)Mxx * (uint64_t)W - (uint64_t)Mx * (uint64_t)Mx);
  const int64_t Cxy = (int64_t)((uint64_t)Mxy * (uint64_t)W - (uint64_t)Mx * (uint64_t)My);
  const int64_t Cyy = (int64_t)((uint64_t)Myy * (uint64_t)W - (uint64_t)My * (uint64_t)My);
  const float h = det_hypotf((float)(Cxx - Cyy), (float)(2 * Cxy));
  const float eig_small = ((float)(Cxx + Cyy) - h) / (float)((double)(W * W) * 8.0);
  return (double)((float)N * eig_small);
}

static void blob_window_moments(const LFP *P, uint32_t n, uint32_t i0, uint32_t i1, int32_t *Mx, int32_t *My,
                                int32_t *W, int64_t *Mxx, int64_t *Myy, int64_t *Mxy, int32_t *N) {
  /* ReadMoments (line_fit_filter.cu:745-796) == CalculateError's (:217-278) */
  if (i0 < i1) {
    *N = (int32_t)(i1 - i0 + 1);
    *Mx = P[i1].Mx; *My = P[i1].My; *W = P[i1].W;
    *Mxx = P[i1].Mxx; *Myy = P[i1].Myy; *Mxy = P[i1].Mxy;
    if (i0 > 0) {
      *Mx = (int32_t)((uint32_t)*Mx - (uint32_t)P[i0 - 1].Mx);
      *My = (int32_t)((uint32_t)*My - (uint32_t)P[i0 - 1].My);
      *W = (int32_t)((uint32_t)*W - (uint32_t)P[i0 - 1].W);
      *Mxx -= P[i0 - 1].Mxx; *Myy -= P[i0 - 1].Myy; *Mxy -= P[i0 - 1].Mxy;
    }
  } else {
    const LFP *l0 = &P[i0 - 1], *lz = &P[n - 1], *l1 = &P[i1];
    *Mx = (int32_t)((uint32_t)lz->Mx - (uint32_t)l0->Mx + (uint32_t)l1->Mx);
    *My = (int32_t)((uint32_t)lz->My - (uint32_t)l0->My + (uint32_t)l1->My);
    *W = (int32_t)((uint32_t)lz->W - (uint32_t)l0->W + (uint32_t)l1->W);
    *Mxx = lz->Mxx - l0->Mxx + l1->Mxx;
    *Myy = lz->Myy - l0->Myy + l1->Myy;
    *Mxy = lz->Mxy - l0->Mxy + l1->Mxy;
    *N = (int32_t)(n - i0 + i1 + 1);
  }
}

static const float kFilter[7] = {0.01110899634659290314f, 0.13533528149127960205f, 0.60653066635131835938f,
                                 1.00000000000000000000f, 0.60653066635131835938f, 0.13533528149127960205f,
                                 0.01110899634659290314f}; /* line_fit_filter.h:122-128 */

static int cmp_peak(const void *a, const void *b) {
  const Peak *x = (const Peak *)a, *y = (const Peak *)b;
  if (x->blob_index != y->blob_index) return x->blob_index < y->blob_index ? -1 : 1;
  /* cub radix float ordering (sign-twiddled bits) */
  uint32_t ux, uy;
  memcpy(&ux, &x->error, 4); memcpy(&uy, &y->error, 4);
  ux = (ux & 0x80000000u) ? ~ux : (ux | 0x80000000u);
  uy = (uy & 0x80000000u) ? ~uy : (uy | 0x80000000u);
  if (ux != uy) return ux < uy ? -1 : 1;
  /* stable: original (point) order */
  return x->filtered_point_index < y->filtered_point_index ? -1 : (x->filtered_point_index > y->filtered_point_index);
}

static void stage_linefit(ao_state *s) {
  const int Wd = s->Wd, Hd = s->Hd, n = s->n_sel;
  for (int i = 0; i < n; i++) {
    const uint64_t k = s->ipts[i];
    const int32_t ix2 = (int32_t)qbp_x(k) + 1, iy2 = (int32_t)qbp_y(k) + 1;
    const int32_t ix = ix2 / 2, iy = iy2 / 2;
    int32_t Wt = 1;
    if (ix > 0 && ix + 1 < Wd && iy > 0 && iy + 1 < Hd) {
      const int32_t gx = (int32_t)s->dec[iy * Wd + ix + 1] - (int32_t)s->dec[iy * Wd + ix - 1];
      const int32_t gy = (int32_t)s->dec[(iy + 1) * Wd + ix] - (int32_t)s->dec[(iy - 1) * Wd + ix];
      Wt = (int32_t)(det_hypotf((float)gx, (float)gy) + 1.0f);
    }
    LFP l;
    l.Mx = Wt * ix2; l.My = Wt * iy2;
    l.Mxx = (int64_t)(Wt * ix2 * ix2); l.Mxy = (int64_t)(Wt * ix2 * iy2); l.Myy = (int64_t)(Wt * iy2 * iy2);
    l.W = Wt;
    l.blob_index = (uint32_t)(k >> 52) & 0xfff;
    /* InclusiveScanByKey(SumLineFitPoints) */
    if (i > 0 && s->lfp[i - 1].blob_index == l.blob_index) {
      const LFP *p = &s->lfp[i - 1];
      l.Mx = (int32_t)((uint32_t)l.Mx + (uint32_t)p->Mx);
      l.My = (int32_t)((uint32_t)l.My + (uint32_t)p->My);
      l.W = (int32_t)((uint32_t)l.W + (uint32_t)p->W);
      l.Mxx += p->Mxx; l.Myy += p->Myy; l.Mxy += p->Mxy;
    }
    s->lfp[i] = l;
  }
  /* errors / filtered / peaks with clean per-blob cyclic windows */
  int np = 0;
  int i = 0;
  while (i < n) {
    const uint32_t bi = s->lfp[i].blob_index;
    const uint32_t so = s->sel[bi].starting_offset, cnt = s->sel[bi].count;
    const LFP *P = &s->lfp[so];
    const uint32_t ksz = cnt / 12 < 20 ? cnt / 12 : 20;
    for (uint32_t b = 0; b < cnt; b++) {
      const uint32_t i0 = (b + 2 * cnt - ksz) % cnt, i1 = (b + cnt + ksz) % cnt;
      int32_t Mx, My, Wt, N; int64_t Mxx, Myy, Mxy;
      blob_window_moments(P, cnt, i0, i1, &Mx, &My, &Wt, &Mxx, &Myy, &Mxy, &N);
      s->errs[so + b] = fit_line_error(N, Mx, My, Mxx, Myy, Mxy, Wt);
    }
    for (uint32_t b = 0; b < cnt; b++) {
      double acc = 0.0;
      for (int j = 0; j < 7; j++) {
        const uint32_t idx = (uint32_t)((int64_t)b + j - 3 + cnt) % cnt;
        acc += s->errs[so + idx] * (double)kFilter[j];
      }
      s->filt[so + b] = acc;
    }
    for (uint32_t b = 0; b < cnt; b++) {
      const double me = s->filt[so + b];
      const double bef = s->filt[so + (b + cnt - 1) % cnt], aft = s->filt[so + (b + 1) % cnt];
      if (me > bef && me > aft) {
        Peak pk;
        pk.error = (float)(-me);
        pk.filtered_point_index = so + b;
        pk.blob_index = (uint16_t)bi;
        s->peaks[np++] = pk;
      }
    }
    i += (int)cnt;
  }
  s->n_peaks = np;
  /* P9: sort peaks by (blob_index, error) stable */
  qsort(s->peaks, (size_t)np, sizeof(Peak), cmp_peak);
}

/* ------------------------------------------------------------------------- */
/* Stage 6: FitQuads (line_fit_filter.cu:709-1212)                            */
/* ------------------------------------------------------------------------- */
static void fit_line(const LFP *P, uint32_t n, uint32_t i0, uint32_t i1, double *lp23, double *err, double *mse) {
  int32_t Mx, My, Wt, N; int64_t Mxx, Myy, Mxy;
  blob_window_moments(P, n, i0, i1, &Mx, &My, &Wt, &Mxx, &Myy, &Mxy, &N);
  const int64_t Cxx = (int64_t)((uint64_t)Mxx * (uint64_t)(int64_t)Wt - (uint64_t)((int64_t)Mx * (int64_t)Mx));
  const int64_t Cxy = (int64_t)((uint64_t)Mxy * (uint64_t)(int64_t)Wt - (uint64_t)((int64_t)Mx * (int64_t)My));
  const int64_t Cyy = (int64_t)((uint64_t)Myy * (uint64_t)(int64_t)Wt - (uint64_t)((int64_t)My * (int64_t)My));
  const float h = det_hypotf((float)(Cxx - Cyy), (float)(2 * Cxy));
  const float e8 = (float)((double)((int64_t)Wt * (int64_t)Wt) * 8.0);
  const float eig = ((float)(Cxx + Cyy) - h) / e8;
  if (lp23) {
    const float nx1 = (float)(Cxx - Cyy) - h, ny1 = (float)(2 * Cxy);
    const float M1 = nx1 * nx1 + ny1 * ny1;
    const float nx2 = (float)(2 * Cxy), ny2 = (float)(Cyy - Cxx) - h;
    const float M2 = nx2 * nx2 + ny2 * ny2;
    float nx, ny;
    if (M1 > M2) { nx = nx1; ny = ny1; } else { nx = nx2; ny = ny2; }
    const float len = det_hypotf(nx, ny);
    lp23[0] = nx / len; lp23[1] = ny / len;
  }
  *err = (double)((float)N * eig);
  *mse = (double)eig;
}

/* Unrank (line_fit_filter.cu:709-728) restated: i-th 4-combination of 0..9 in
 * lexicographic order.  ao_unrank is checked against a literal transcription
 * of the reference FindM0/FindM1/FindM2 in tests. */
int ao_unrank(int i, int *m0, int *m1, int *m2, int *m3) {
  int c = 0;
  for (int a = 0; a < 10; a++)
    for (int b = a + 1; b < 10; b++)
      for (int d = b + 1; d < 10; d++)
        for (int e = d + 1; e < 10; e++) {
          if (c == i) { *m0 = a; *m1 = b; *m2 = d; *m3 = e; return 1; }
          c++;
        }
  return 0;
}

static void stage_fitquads(ao_state *s) {
  const int kNMax = 10;
  int nfq = 0;
  int i = 0;
  while (i < s->n_peaks) {
    const uint16_t bi = s->peaks[i].blob_index;
    int cnt = 0;
    while (i + cnt < s->n_peaks && s->peaks[i + cnt].blob_index == bi) cnt++;
    const Extents *se = &s->sel[bi];
    const LFP *P = &s->lfp[se->starting_offset];
    const uint32_t sz = se->count;
    uint16_t pi[16];
    for (int t = 0; t < 16; t++)
      pi[t] = (t < cnt && t < kNMax) ? (uint16_t)(s->peaks[i + t].filtered_point_index - se->starting_offset)
                                     : (uint16_t)0xffff;
    /* WarpMergeSort ascending */
    for (int a = 1; a < 16; a++) {
      uint16_t v = pi[a]; int b = a - 1;
      while (b >= 0 && pi[b] > v) { pi[b + 1] = pi[b]; b--; }
      pi[b + 1] = v;
    }
    double e01[7][7], lp01[7][7][2];
    for (int m0 = 0; m0 < 7; m0++)
      for (int m1 = m0 + 1; m1 < 8; m1++) {
        if (cnt < 4) continue;
        if (m1 < kNMax && m1 < cnt) {
          double err, mse;
          fit_line(P, sz, pi[m0], pi[m1], lp01[m0][m1 - 1], &err, &mse);
          if (mse > (double)s->p.max_line_fit_mse) err = DBL_MAX;
          e01[m0][m1 - 1] = err;
        } else {
          e01[m0][m1 - 1] = DBL_MAX;
        }
      }
    double best = DBL_MAX;
    int bm[4] = {0, 1, 2, 3};
    int first = 1;
    for (int t = 0; t < 210; t++) {
      int m0, m1, m2, m3;
      ao_unrank(t, &m0, &m1, &m2, &m3);
      double err = DBL_MAX;
      if (cnt >= 4 && m3 < kNMax && m3 < cnt && e01[m0][m1 - 1] != DBL_MAX) {
        double e12, mse12, p12[2];
        fit_line(P, sz, pi[m1], pi[m2], p12, &e12, &mse12);
        if (!(mse12 > (double)s->p.max_line_fit_mse)) {
          const double *p01 = lp01[m0][m1 - 1];
          const double dot = p01[0] * p12[0] + p01[1] * p12[1];
          if (!(fabs(dot) > s->p.cos_critical_rad)) {
            double e23, mse23, e30, mse30;
            fit_line(P, sz, pi[m2], pi[m3], NULL, &e23, &mse23);
            if (!(mse23 > (double)s->p.max_line_fit_mse)) {
              fit_line(P, sz, pi[m3], pi[m0], NULL, &e30, &mse30);
              if (!(mse30 > (double)s->p.max_line_fit_mse)) err = e01[m0][m1 - 1] + e12 + e23 + e30;
            }
          }
        }
      }
      /* BlockReduce(MinQuadError): a.error <= b.error keeps the lower index */
      if (first || err < best) {
        best = err; bm[0] = m0; bm[1] = m1; bm[2] = m2; bm[3] = m3; first = 0;
      }
    }
    ao_fitquad *f = &s->fq[nfq++];
    memset(f, 0, sizeof(*f));
    f->blob_index = bi;
    f->valid = best < (double)(s->p.max_line_fit_mse * (float)sz);
    for (int k = 0; k < 4; k++) f->indices[k] = pi[bm[k]];
    if (f->valid) {
      for (int k = 0; k < 4; k++) {
        blob_window_moments(P, sz, f->indices[k], f->indices[(k + 1) & 3], &f->Mx[k], &f->My[k], &f->W[k],
                            &f->Mxx[k], &f->Myy[k], &f->Mxy[k], &f->N[k]);
      }
    }
    i += cnt;
  }
  s->n_fq = nfq;
}

/* ------------------------------------------------------------------------- */
/* Stage 7: UpdateFitQuads + AdjustPixelCenters (apriltag_detect.cu:38-282)   */
/* ------------------------------------------------------------------------- */
static void host_fit_line(const ao_fitquad *f, int k, double *l01, double *l23) {
  const int64_t W = f->W[k];
  const int64_t Cxx = (int64_t)((uint64_t)f->Mxx[k] * (uint64_t)W - (uint64_t)((int64_t)f->Mx[k] * f->Mx[k]));
  const int64_t Cxy = (int64_t)((uint64_t)f->Mxy[k] * (uint64_t)W - (uint64_t)((int64_t)f->Mx[k] * f->My[k]));
  const int64_t Cyy = (int64_t)((uint64_t)f->Myy[k] * (uint64_t)W - (uint64_t)((int64_t)f->My[k] * f->My[k]));
  const float h = det_hypotf((float)(Cxx - Cyy), (float)(2 * Cxy));
  l01[0] = (double)((float)f->Mx[k] / (float)(f->W[k] * 2));
  l01[1] = (double)((float)f->My[k] / (float)(f->W[k] * 2));
  const float nx1 = (float)(Cxx - Cyy) - h, ny1 = (float)(Cxy * 2);
  const float M1 = nx1 * nx1 + ny1 * ny1;
  const float nx2 = (float)(Cxy * 2), ny2 = (float)(Cyy - Cxx) - h;
  const float M2 = nx2 * nx2 + ny2 * ny2;
  float nx, ny;
  if (M1 > M2) { nx = nx1; ny = ny1; } else { nx = nx2; ny = ny2; }
  const float len = det_hypotf(nx, ny);
  l23[0] = (double)(nx / len); l23[1] = (double)(ny / len);
}

static void stage_quads(ao_state *s) {
  int nq = 0;
  for (int qi = 0; qi < s->n_fq; qi++) {
    const ao_fitquad *f = &s->fq[qi];
    if (!f->valid) continue;
    ao_quad qc;
    qc.blob_index = f->blob_index;
    qc.reversed_border = s->fam->reversed_border;
    double lines[4][4];
    for (int k = 0; k < 4; k++) host_fit_line(f, k, lines[k], lines[k] + 2);
    int bad = 0;
    for (int k = 0; k < 4; k++) {
      const int k1 = (k + 1) & 3;
      const double A00 = lines[k][3], A01 = -lines[k1][3];
      const double A10 = -lines[k][2], A11 = lines[k1][2];
      const double B0 = -lines[k][0] + lines[k1][0];
      const double B1 = -lines[k][1] + lines[k1][1];
      const double det = A00 * A11 - A10 * A01;
      const double W00 = A11 / det, W01 = -A01 / det;
      if (fabs(det) < 0.001) { bad = 1; break; }
      const double L0 = W00 * B0 + W01 * B1;
      qc.corners[k][0] = (float)(lines[k][0] + L0 * A00);
      qc.corners[k][1] = (float)(lines[k][1] + L0 * A10);
    }
    if (bad) continue;
    {
      float area = 0, len[3], pp;
      for (int k = 0; k < 3; k++) {
        const int a = k, b = (k + 1) % 3;
        len[k] = det_hypotf(qc.corners[b][0] - qc.corners[a][0], qc.corners[b][1] - qc.corners[a][1]);
      }
      pp = (len[0] + len[1] + len[2]) / 2;
      area += sqrtf(pp * (pp - len[0]) * (pp - len[1]) * (pp - len[2]));
      static const int idxs[4] = {2, 3, 0, 2};
      for (int k = 0; k < 3; k++) {
        const int a = idxs[k], b = idxs[k + 1];
        len[k] = det_hypotf(qc.corners[b][0] - qc.corners[a][0], qc.corners[b][1] - qc.corners[a][1]);
      }
      pp = (len[0] + len[1] + len[2]) / 2;
      area += sqrtf(pp * (pp - len[0]) * (pp - len[1]) * (pp - len[2]));
      if ((double)area < 0.95 * s->min_tag_width * s->min_tag_width) continue;
    }
    {
      int reject = 0;
      for (int k = 0; k < 4; k++) {
        const int i0 = k, i1 = (k + 1) & 3, i2 = (k + 2) & 3;
        const float dx1 = qc.corners[i1][0] - qc.corners[i0][0];
        const float dy1 = qc.corners[i1][1] - qc.corners[i0][1];
        const float dx2 = qc.corners[i2][0] - qc.corners[i1][0];
        const float dy2 = qc.corners[i2][1] - qc.corners[i1][1];
        const float cos_dtheta = (dx1 * dx2 + dy1 * dy2) / sqrtf((dx1 * dx1 + dy1 * dy1) * (dx2 * dx2 + dy2 * dy2));
        if ((double)fabsf(cos_dtheta) > s->p.cos_critical_rad || dx1 * dy2 < dy1 * dx2) { reject = 1; break; }
      }
      if (reject) continue;
    }
    /* AdjustPixelCenters, quad_decimate = 2 */
    for (int k = 0; k < 4; k++) {
      qc.corners[k][0] = (qc.corners[k][0] - 0.5f) * 2.0f + 0.5f;
      qc.corners[k][1] = (qc.corners[k][1] - 0.5f) * 2.0f + 0.5f;
    }
    s->quads[nq++] = qc;
  }
  s->n_quads = nq;
}

/* ------------------------------------------------------------------------- */
/* Stage 8: RefineEdges with UnDistort/ReDistort (apriltag_detect.cu:307-564) */
/* ------------------------------------------------------------------------- */
static void redistort(const ao_params *p, double *x, double *y) {
  const double xP = (*x - p->cx) / p->fx, yP = (*y - p->cy) / p->fy;
  const double rSq = xP * xP + yP * yP;
  const double lin = 1 + p->k1 * rSq + p->k2 * rSq * rSq + p->k3 * rSq * rSq * rSq;
  const double xPP = xP * lin + 2 * p->p1 * xP * yP + p->p2 * (rSq + 2 * xP * xP);
  const double yPP = yP * lin + p->p1 * (rSq + 2 * yP * yP) + 2 * p->p2 * xP * yP;
  *x = xPP * p->fx + p->cx;
  *y = yPP * p->fy + p->cy;
}

static void undistort(const ao_params *p, double *u, double *v) {
  const double xPP = (*u - p->cx) / p->fx, yPP = (*v - p->cy) / p->fy;
  double xP = xPP, yP = yPP;
  const double x0 = xP, y0 = yP;
  double prev_x, prev_y;
  int it = 0;
  do {
    prev_x = xP; prev_y = yP;
    const double rSq = xP * xP + yP * yP;
    const double rad = 1 + (p->k1 * rSq) + (p->k2 * rSq * rSq) + (p->k3 * rSq * rSq * rSq);
    const double rinv = 1 / rad;
    /* NB: reference tangential term p2*(rSq + k3*rSq^3) kept as-is (:372) */
    const double tdx = 2 * p->p1 * xP * yP + p->p2 * (rSq + p->k3 * rSq * rSq * rSq);
    const double tdy = p->p1 * (rSq + 2 * yP * yP) + 2 * p->p2 * xP * yP;
    xP = (x0 - tdx) * rinv;
    yP = (y0 - tdy) * rinv;
    if (it > 100) break;
    it++;
  } while (fabs(xP - prev_x) > 1e-6 || fabs(yP - prev_y) > 1e-6);
  *u = xP * p->fx + p->cx;
  *v = yP * p->fy + p->cy;
}

static void refine_edges(const ao_state *s, float qp[4][2], int reversed) {
  const ao_params *pr = &s->p;
  const int W = s->W, H = s->H;
  const uint8_t *im = s->gray;
  double lines[4][4];
  for (int edge = 0; edge < 4; edge++) {
    const int a = edge, b = (edge + 1) & 3;
    float nx = qp[b][1] - qp[a][1];
    float ny = -qp[b][0] + qp[a][0];
    const float mag = sqrtf(nx * nx + ny * ny);
    nx /= mag; ny /= mag;
    if (reversed) { nx = -nx; ny = -ny; }
    const int ns_f = (int)(mag / 8);
    const int nsamples = 16 > ns_f ? 16 : ns_f;
    double Mx = 0, My = 0, Mxx = 0, Mxy = 0, Myy = 0, N = 0;
    for (int sidx = 0; sidx < nsamples; sidx++) {
      const double alpha = (1.0 + sidx) / (nsamples + 1);
      const double x0 = alpha * qp[a][0] + (1 - alpha) * qp[b][0];
      const double y0 = alpha * qp[a][1] + (1 - alpha) * qp[b][1];
      double Mn = 0, Mcount = 0;
      const double range = (double)(2.0f + 1);
      for (double n = -range; n <= range; n += 0.25) {
        const double grange = 1;
        const int x1 = (int)(x0 + (n + grange) * nx);
        const int y1 = (int)(y0 + (n + grange) * ny);
        if (x1 < 0 || x1 >= W || y1 < 0 || y1 >= H) continue;
        const int x2 = (int)(x0 + (n - grange) * nx);
        const int y2 = (int)(y0 + (n - grange) * ny);
        if (x2 < 0 || x2 >= W || y2 < 0 || y2 >= H) continue;
        const int g1 = im[y1 * W + x1], g2 = im[y2 * W + x2];
        if (g1 < g2) continue;
        const double weight = (double)((g2 - g1) * (g2 - g1));
        Mn += weight * n;
        Mcount += weight;
      }
      if (Mcount == 0) continue;
      const double n0 = Mn / Mcount;
      double bestx = x0 + n0 * nx, besty = y0 + n0 * ny;
      undistort(pr, &bestx, &besty);
      Mx += bestx; My += besty; Mxx += bestx * bestx; Mxy += bestx * besty; Myy += besty * besty; N++;
    }
    const double Ex = Mx / N, Ey = My / N;
    const double Cxx = Mxx / N - Ex * Ex, Cxy = Mxy / N - Ex * Ey, Cyy = Myy / N - Ey * Ey;
    const double normal_theta = .5 * (double)det_atan2f((float)(-2 * Cxy), (float)(Cyy - Cxx));
    const float nxf = det_cosf((float)normal_theta), nyf = det_sinf((float)normal_theta);
    lines[edge][0] = Ex; lines[edge][1] = Ey; lines[edge][2] = nxf; lines[edge][3] = nyf;
  }
  for (int i = 0; i < 4; i++) {
    const int i1 = (i + 1) & 3;
    const double A00 = lines[i][3], A01 = -lines[i1][3];
    const double A10 = -lines[i][2], A11 = lines[i1][2];
    const double B0 = -lines[i][0] + lines[i1][0];
    const double B1 = -lines[i][1] + lines[i1][1];
    const double det = A00 * A11 - A10 * A01;
    if (fabs(det) > 0.001) {
      const double W00 = A11 / det, W01 = -A01 / det;
      const double L0 = W00 * B0 + W01 * B1;
      double px = lines[i][0] + L0 * A00, py = lines[i][1] + L0 * A10;
      redistort(pr, &px, &py);
      qp[i1][0] = (float)px;
      qp[i1][1] = (float)py;
    }
  }
}

/* ------------------------------------------------------------------------- */
/* Stage 9: quad_decode_index (third party: apriltag 3.x apriltag.c)           */
/* ------------------------------------------------------------------------- */
static int homography_compute2(const double c[4][4], double H[9]) {
  double A[72];
  for (int i = 0; i < 4; i++) {
    double *r0 = &A[(2 * i) * 9], *r1 = &A[(2 * i + 1) * 9];
    r0[0] = c[i][0]; r0[1] = c[i][1]; r0[2] = 1; r0[3] = 0; r0[4] = 0; r0[5] = 0;
    r0[6] = -c[i][0] * c[i][2]; r0[7] = -c[i][1] * c[i][2]; r0[8] = c[i][2];
    r1[0] = 0; r1[1] = 0; r1[2] = 0; r1[3] = c[i][0]; r1[4] = c[i][1]; r1[5] = 1;
    r1[6] = -c[i][0] * c[i][3]; r1[7] = -c[i][1] * c[i][3]; r1[8] = c[i][3];
  }
  for (int col = 0; col < 8; col++) {
    double max_val = 0; int max_idx = -1;
    for (int row = col; row < 8; row++) {
      const double v = fabs(A[row * 9 + col]);
      if (v > max_val) { max_val = v; max_idx = row; }
    }
    if (max_val < 1e-10) return -1;
    if (max_idx != col)
      for (int i = col; i < 9; i++) { double t = A[col * 9 + i]; A[col * 9 + i] = A[max_idx * 9 + i]; A[max_idx * 9 + i] = t; }
    for (int i = col + 1; i < 8; i++) {
      const double f = A[i * 9 + col] / A[col * 9 + col];
      A[i * 9 + col] = 0;
      for (int j = col + 1; j < 9; j++) A[i * 9 + j] -= f * A[col * 9 + j];
    }
  }
  for (int col = 7; col >= 0; col--) {
    double sum = 0;
    for (int i = col + 1; i < 8; i++) sum += A[col * 9 + i] * A[i * 9 + 8];
    A[col * 9 + 8] = (A[col * 9 + 8] - sum) / A[col * 9 + col];
  }
  H[0] = A[8]; H[1] = A[17]; H[2] = A[26]; H[3] = A[35]; H[4] = A[44]; H[5] = A[53];
  H[6] = A[62]; H[7] = A[71]; H[8] = 1;
  return 0;
}

static void hproject(const double H[9], double x, double y, double *ox, double *oy) {
  const double xx = H[0] * x + H[1] * y + H[2];
  const double yy = H[3] * x + H[4] * y + H[5];
  const double zz = H[6] * x + H[7] * y + H[8];
  *ox = xx / zz; *oy = yy / zz;
}

typedef struct { double A[3][3], B[3], C[3]; } graymodel;
static void gm_add(graymodel *g, double x, double y, double gray) {
  g->A[0][0] += x * x; g->A[0][1] += x * y; g->A[0][2] += x;
  g->A[1][1] += y * y; g->A[1][2] += y; g->A[2][2] += 1;
  g->B[0] += x * gray; g->B[1] += y * gray; g->B[2] += gray;
}
static void gm_solve(graymodel *g) {
  const double *A = &g->A[0][0];
  double L[9], M[9];
  L[0] = sqrt(A[0]); L[3] = A[1] / L[0]; L[6] = A[2] / L[0];
  L[4] = sqrt(A[4] - L[3] * L[3]); L[7] = (A[5] - L[3] * L[6]) / L[4];
  L[8] = sqrt(A[8] - L[6] * L[6] - L[7] * L[7]);
  L[1] = 0; L[2] = 0; L[5] = 0;
  M[0] = 1 / L[0]; M[3] = -L[3] * M[0] / L[4]; M[4] = 1 / L[4];
  M[6] = (-L[6] * M[0] - L[7] * M[3]) / L[8]; M[7] = -L[7] * M[4] / L[8]; M[8] = 1 / L[8];
  double t0 = M[0] * g->B[0];
  double t1 = M[3] * g->B[0] + M[4] * g->B[1];
  double t2 = M[6] * g->B[0] + M[7] * g->B[1] + M[8] * g->B[2];
  g->C[0] = M[0] * t0 + M[3] * t1 + M[6] * t2;
  g->C[1] = M[4] * t1 + M[7] * t2;
  g->C[2] = M[8] * t2;
}
static double gm_interp(const graymodel *g, double x, double y) { return g->C[0] * x + g->C[1] * y + g->C[2]; }

static double value_for_pixel(const ao_state *s, double px, double py) {
  const int x1 = (int)floor(px - 0.5), x2 = (int)ceil(px - 0.5);
  const double x = px - 0.5 - x1;
  const int y1 = (int)floor(py - 0.5), y2 = (int)ceil(py - 0.5);
  const double y = py - 0.5 - y1;
  if (x1 < 0 || x2 >= s->W || y1 < 0 || y2 >= s->H) return -1;
  const uint8_t *b = s->gray;
  const int st = s->W;
  return b[y1 * st + x1] * (1 - x) * (1 - y) + b[y1 * st + x2] * x * (1 - y) + b[y2 * st + x1] * (1 - x) * y +
         b[y2 * st + x2] * x * y;
}

static float quad_decode(const ao_state *s, const double H[9], int *out_id, int *out_ham, int *out_rot,
                         uint64_t *out_rcode) {
  const Family *fam = s->fam;
  const int wabi = fam->width_at_border, tw = fam->total_width;
  const float wab = (float)wabi;
  const float patterns[40] = {
      -0.5f, 0.5f, 0, 1, 1,   0.5f, 0.5f, 0, 1, 0,   wab + 0.5f, .5f, 0, 1, 1,  wab - 0.5f, .5f, 0, 1, 0,
      0.5f, -0.5f, 1, 0, 1,   0.5f, 0.5f, 1, 0, 0,   0.5f, wab + 0.5f, 1, 0, 1, 0.5f, wab - 0.5f, 1, 0, 0};
  graymodel wm, bm;
  memset(&wm, 0, sizeof(wm)); memset(&bm, 0, sizeof(bm));
  for (int pi = 0; pi < 8; pi++) {
    const float *pat = &patterns[pi * 5];
    const int is_white = (int)pat[4];
    for (int i = 0; i < wabi; i++) {
      const double tagx01 = (double)((pat[0] + (float)i * pat[2]) / (float)wabi);
      const double tagy01 = (double)((pat[1] + (float)i * pat[3]) / (float)wabi);
      const double tagx = 2 * (tagx01 - 0.5), tagy = 2 * (tagy01 - 0.5);
      double px, py;
      hproject(H, tagx, tagy, &px, &py);
      const int ix = (int)px, iy = (int)py;
      if (ix < 0 || iy < 0 || ix >= s->W || iy >= s->H) continue;
      const int v = s->gray[iy * s->W + ix];
      if (is_white) gm_add(&wm, tagx, tagy, v);
      else gm_add(&bm, tagx, tagy, v);
    }
  }
  gm_solve(&wm);
  gm_solve(&bm);
  if ((gm_interp(&wm, 0, 0) - gm_interp(&bm, 0, 0) < 0) != fam->reversed_border) return -1;
  float black_score = 0, white_score = 0, black_cnt = 1, white_cnt = 1;
  double values[16 * 16];
  memset(values, 0, sizeof(values));
  const int min_coord = (wabi - tw) / 2;
  for (int i = 0; i < fam->nbits; i++) {
    const int bity = fam->bity[i], bitx = fam->bitx[i];
    const double tagx01 = (bitx + 0.5) / wabi, tagy01 = (bity + 0.5) / wabi;
    const double tagx = 2 * (tagx01 - 0.5), tagy = 2 * (tagy01 - 0.5);
    double px, py;
    hproject(H, tagx, tagy, &px, &py);
    const double v = value_for_pixel(s, px, py);
    if (v == -1) continue;
    const double thresh = (gm_interp(&bm, tagx, tagy) + gm_interp(&wm, tagx, tagy)) / 2.0;
    values[tw * (bity - min_coord) + bitx - min_coord] = v - thresh;
  }
  /* sharpen (apriltag.c) over the total_width x total_width grid */
  {
    double sh[16 * 16];
    static const double kern[9] = {0, -1, 0, -1, 4, -1, 0, -1, 0};
    const int size = tw;
    for (int y = 0; y < size; y++)
      for (int x = 0; x < size; x++) {
        sh[y * size + x] = 0;
        for (int i = 0; i < 3; i++)
          for (int j = 0; j < 3; j++) {
            if ((y + i - 1) < 0 || (y + i - 1) > size - 1 || (x + j - 1) < 0 || (x + j - 1) > size - 1) continue;
            sh[y * size + x] += values[(y + i - 1) * size + (x + j - 1)] * kern[i * 3 + j];
          }
      }
    for (int y = 0; y < size; y++)
      for (int x = 0; x < size; x++)
        values[y * size + x] = values[y * size + x] + s->p.decode_sharpening * sh[y * size + x];
  }
  uint64_t rcode = 0;
  for (int i = 0; i < fam->nbits; i++) {
    const int bity = fam->bity[i], bitx = fam->bitx[i];
    rcode = rcode << 1;
    const double v = values[tw * (bity - min_coord) + bitx - min_coord];
    if (v > 0) { white_score = (float)(white_score + v); white_cnt++; rcode |= 1; }
    else { black_score = (float)(black_score - v); black_cnt++; }
  }
  *out_rcode = rcode;
  /* quick_decode_codeword: first rotation with a codeword within kMaxHamming
   * (the family's codes are >= 5 apart, so at most one entry matches a rotation) */
  *out_id = 65535; *out_ham = 255; *out_rot = 0;
  for (int r = 0; r < 4; r++) {
    int found = 0;
    for (int c = 0; c < fam->ncodes; c++) {
      const int hd = __builtin_popcountll(rcode ^ fam->codes[c].code);
      if (hd <= kMaxHamming) { *out_id = fam->codes[c].id; *out_ham = hd; *out_rot = r; found = 1; break; }
    }
    if (found) break;
    rcode = ao_rotate90_n(rcode, fam->nbits);
  }
  return (float)fmin((double)(white_score / white_cnt), (double)(black_score / black_cnt));
}

/* cos/sin(rotation * pi/2) as glibc returns them (apriltag.c det rotation) */
static const double kRotC[4] = {1.0, 6.123233995736766e-17, -1.0, -1.8369701987210297e-16};
static const double kRotS[4] = {0.0, 1.0, 1.2246467991473532e-16, -1.0};

static void decode_quad(ao_state *s, const ao_quad *q, int qi) {
  float qp[4][2];
  memcpy(qp, q->corners, sizeof(qp));
  if (s->p.refine_edges) refine_edges(s, qp, q->reversed_border);
  double corr[4][4];
  for (int i = 0; i < 4; i++) {
    corr[i][0] = (i == 0 || i == 3) ? -1 : 1;
    corr[i][1] = (i == 0 || i == 1) ? -1 : 1;
    corr[i][2] = qp[i][0];
    corr[i][3] = qp[i][1];
  }
  double H[9];
  if (homography_compute2(corr, H)) return;
  const double hdet = H[0] * (H[4] * H[8] - H[5] * H[7]) - H[1] * (H[3] * H[8] - H[5] * H[6]) +
                      H[2] * (H[3] * H[7] - H[4] * H[6]);
  if (hdet == 0) return; /* matd_inverse == NULL */
  int id, ham, rot;
  uint64_t rcode = 0;
  const float margin = quad_decode(s, H, &id, &ham, &rot, &rcode);
  s->rcodes[qi] = rcode;
  s->margins[qi] = margin;
  if (!(margin >= 0 && ham < 255)) return;
  ao_detection *d = &s->dets[s->n_dets++];
  memset(d, 0, sizeof(*d));
  d->id = id; d->hamming = ham; d->decision_margin = margin; d->blob_index = (int32_t)q->blob_index;
  const double c = kRotC[rot], sn = kRotS[rot];
  const double R[9] = {c, -sn, 0, sn, c, 0, 0, 0, 1};
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double acc = 0;
      for (int k = 0; k < 3; k++) acc += H[i * 3 + k] * R[k * 3 + j];
      d->H[i * 3 + j] = acc;
    }
  hproject(d->H, 0, 0, &d->c[0], &d->c[1]);
  for (int i = 0; i < 4; i++) {
    const int tcx = (i == 1 || i == 2) ? 1 : -1;
    const int tcy = (i < 2) ? 1 : -1;
    hproject(d->H, tcx, tcy, &d->p[i][0], &d->p[i][1]);
  }
}

/* ------------------------------------------------------------------------- */
/* Stage 10: reconcile_detections + zarray_sort by id                         */
/* ------------------------------------------------------------------------- */
static int seg_intersect(const double *a0, const double *a1, const double *b0, const double *b1) {
  /* g2d_line_segment_intersect_segment: intersection of the two lines, then
   * both segments must contain the point. */
  const double p0[2] = {a0[0], a0[1]}, u[2] = {a1[0] - a0[0], a1[1] - a0[1]};
  const double q0[2] = {b0[0], b0[1]}, v[2] = {b1[0] - b0[0], b1[1] - b0[1]};
  const double den = u[0] * v[1] - u[1] * v[0];
  if (fabs(den) < 1e-12) return 0;
  const double t = ((q0[0] - p0[0]) * v[1] - (q0[1] - p0[1]) * v[0]) / den;
  const double w = ((q0[0] - p0[0]) * u[1] - (q0[1] - p0[1]) * u[0]) / den;
  return t >= 0 && t <= 1 && w >= 0 && w <= 1;
}
static int poly_contains(const double poly[4][2], const double *pt) {
  int inside = 0;
  for (int i = 0, j = 3; i < 4; j = i++) {
    if (((poly[i][1] > pt[1]) != (poly[j][1] > pt[1])) &&
        (pt[0] < (poly[j][0] - poly[i][0]) * (pt[1] - poly[i][1]) / (poly[j][1] - poly[i][1]) + poly[i][0]))
      inside = !inside;
  }
  return inside;
}
static int poly_overlap(const double a[4][2], const double b[4][2]) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++)
      if (seg_intersect(a[i], a[(i + 1) & 3], b[j], b[(j + 1) & 3])) return 1;
  if (poly_contains(a, b[0])) return 1;
  if (poly_contains(b, a[0])) return 1;
  return 0;
}
static int prefer_smaller(int pref, double q0, double q1) {
  if (pref) return pref;
  if (q0 < q1) return -1;
  if (q1 < q0) return 1;
  return 0;
}
static void reconcile(ao_state *s) {
  ao_detection *d = s->dets;
  int n = s->n_dets;
  for (int i0 = 0; i0 < n; i0++) {
    for (int i1 = i0 + 1; i1 < n; i1++) {
      if (d[i0].id != d[i1].id) continue;
      if (!poly_overlap(d[i0].p, d[i1].p)) continue;
      int pref = 0;
      pref = prefer_smaller(pref, d[i0].hamming, d[i1].hamming);
      pref = prefer_smaller(pref, -d[i0].decision_margin, -d[i1].decision_margin);
      for (int k = 0; k < 3; k++) pref = prefer_smaller(pref, d[i0].H[k], d[i1].H[k]);
      if (pref < 0) {
        if (i1 < n - 1) d[i1] = d[n - 1];
        n--; i1--;
      } else {
        if (i0 < n - 1) d[i0] = d[n - 1];
        n--; i0--;
        break;
      }
    }
  }
  /* zarray_sort by id (glibc qsort == stable merge sort here) */
  for (int a = 1; a < n; a++) {
    ao_detection v = d[a]; int b = a - 1;
    while (b >= 0 && d[b].id > v.id) { d[b + 1] = d[b]; b--; }
    d[b + 1] = v;
  }
  s->n_dets = n;
}

/* ------------------------------------------------------------------------- */
int ao_detect(ao_state *s, const uint8_t *frame, int pixfmt) {
  s->status = 0;
  s->n_pts = s->n_pairs = s->n_sel = s->n_peaks = s->n_fq = s->n_quads = s->n_dets = 0;
  s->n_pts_pairs = -1;
  stage_threshold(s, frame, pixfmt);
  stage_ccl(s);
  stage_boundary(s);
  if (s->n_pairs > 4096) {
    /* More pairs than the 12-bit blob index holds (points.h:183-193; the reference
     * overflows its 2048-entry extents buffer here, apriltag_gpu.cu:129,899-902:
     * undefined).  This build keeps the first 4096 pairs in rank order (rep01
     * ascending, P2's order), drops the points of the others and reports the
     * capacity status with the kept pairs' detections. */
    s->status = -3;
    s->n_pairs = 4096;
    s->n_pts_pairs = (int)(s->ext[4095].starting_offset + s->ext[4095].count);
  }
  stage_select(s);
  stage_linefit(s);
  stage_fitquads(s);
  stage_quads(s);
  for (int i = 0; i < s->n_quads; i++) { s->rcodes[i] = 0; s->margins[i] = -1; decode_quad(s, &s->quads[i], i); }
  reconcile(s);
  return s->n_dets;
}

const uint8_t *ao_gray(const ao_state *s) { return s->gray; }
const uint8_t *ao_decimated(const ao_state *s) { return s->dec; }
const uint8_t *ao_thresholded(const ao_state *s) { return s->thr; }
const uint32_t *ao_labels(const ao_state *s) { return s->labels; }
const uint32_t *ao_sizes(const ao_state *s) { return s->sizes; }
int ao_num_points(const ao_state *s) { return s->n_pts; }
const uint64_t *ao_sorted_points(const ao_state *s) { return s->pts; }
int ao_num_pairs(const ao_state *s) { return s->n_pairs; }
int ao_num_selected_points(const ao_state *s) { return s->n_sel; }
const uint64_t *ao_sorted_index_points(const ao_state *s) { return s->ipts; }
const double *ao_errs(const ao_state *s) { return s->errs; }
const double *ao_filtered_errs(const ao_state *s) { return s->filt; }
int ao_num_peaks(const ao_state *s) { return s->n_peaks; }
int ao_num_fitquads(const ao_state *s) { return s->n_fq; }
const ao_fitquad *ao_fitquads(const ao_state *s) { return s->fq; }
int ao_num_quads(const ao_state *s) { return s->n_quads; }
const ao_quad *ao_quads(const ao_state *s) { return s->quads; }
int ao_num_detections(const ao_state *s) { return s->n_dets; }
const ao_detection *ao_detections(const ao_state *s) { return s->dets; }
int ao_status(const ao_state *s) { return s->status; }
uint64_t ao_quad_rcode(const ao_state *s, int i) { return s->rcodes[i]; }
float ao_quad_margin(const ao_state *s, int i) { return s->margins[i]; }
