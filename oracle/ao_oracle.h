/*
 * ao_oracle.h -- CPU ORACLE for the AprilTag detection hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (ros_vision_amd/, include/)
 * may include, link or call this code; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker.
 *
 * This is a plain-C restatement of the reference per-frame pipeline
 * (Team766/ros_vision src/apriltags_cuda, GpuDetector::Detect,
 * apriltag_gpu.cu:725-1166 plus the host tail apriltag_detect.cu:98-663) and
 * of the third-party pieces it calls (cgpadwick/apriltag@3.3.0:
 * quad_decode_index, reconcile_detections, tag36h11).  Every stage cites the
 * reference lines it follows.  Parity pin: see DESIGN.md "Oracle" (the
 * reference cannot be built or run offline; the oracle is pinned by the
 * reference's own fixture test/data/colorimage.jpg (1 tag, id 554) and
 * colorimage_notags.jpg (0 tags), and by the tag36h11 generator arithmetic).
 */
#ifndef AO_ORACLE_H_
#define AO_ORACLE_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* apriltag_detector_t defaults the reference relies on (upstream
 * apriltag_detector_create, set/overridden at apriltags_cuda_detector.cu:139-147). */
typedef struct {
  int width, height;               /* full-resolution frame, W%8==0, H%8==0 */
  double fx, fy, cx, cy;           /* CameraMatrix (apriltag_gpu.h:61-66) */
  double k1, k2, p1, p2, k3;       /* DistCoeffs (apriltag_gpu.h:68-74) */
  int min_white_black_diff;        /* qtp.min_white_black_diff = 5 */
  int min_cluster_pixels;          /* qtp.min_cluster_pixels = 5 */
  int max_nmaxima;                 /* qtp.max_nmaxima = 10 (fixed, line_fit_filter.cu:1205) */
  float max_line_fit_mse;          /* qtp.max_line_fit_mse = 10.0 */
  double cos_critical_rad;         /* qtp.cos_critical_rad = cos(10 deg) */
  double decode_sharpening;        /* td->decode_sharpening = 0.25 */
  int refine_edges;                /* td->refine_edges = 1 */
  const char *family;              /* "tag36h11" (default when NULL), "tag25h9", "tag16h5" */
} ao_params;

typedef struct {
  int32_t id, hamming;
  float decision_margin;
  double H[9];
  double c[2];
  double p[4][2];
  int32_t blob_index;
} ao_detection;

typedef struct {
  uint16_t blob_index;
  uint8_t valid;
  uint16_t indices[4];
  /* LineFitMoments: Mx, My, W, Mxx, Myy, Mxy, N (line_fit_filter.h:85-94) */
  int32_t Mx[4], My[4], W[4];
  int64_t Mxx[4], Myy[4], Mxy[4];
  int32_t N[4];
} ao_fitquad;

typedef struct {
  float corners[4][2];
  int reversed_border;
  uint32_t blob_index;
} ao_quad;

typedef struct ao_state ao_state;

void ao_default_params(ao_params *p, int width, int height);
ao_state *ao_create(const ao_params *p);
void ao_destroy(ao_state *s);

/* pixfmt: 0 = YUYV (2 bytes/pixel), 1 = BGR8, 2 = GRAY8 */
int ao_detect(ao_state *s, const uint8_t *frame, int pixfmt);

/* stage taps */
const uint8_t *ao_gray(const ao_state *s);
const uint8_t *ao_decimated(const ao_state *s);
const uint8_t *ao_thresholded(const ao_state *s);
const uint32_t *ao_labels(const ao_state *s);
const uint32_t *ao_sizes(const ao_state *s);
int ao_num_points(const ao_state *s);              /* N_c */
const uint64_t *ao_sorted_points(const ao_state *s); /* QuadBoundaryPoint keys after P2 */
int ao_num_pairs(const ao_state *s);               /* N_q */
int ao_num_selected_points(const ao_state *s);     /* N_s */
const uint64_t *ao_sorted_index_points(const ao_state *s); /* IndexPoint keys after P6 */
const double *ao_errs(const ao_state *s);
const double *ao_filtered_errs(const ao_state *s);
int ao_num_peaks(const ao_state *s);
int ao_num_fitquads(const ao_state *s);
const ao_fitquad *ao_fitquads(const ao_state *s);
int ao_num_quads(const ao_state *s);
const ao_quad *ao_quads(const ao_state *s);        /* after UpdateFitQuads+AdjustPixelCenters */
int ao_num_detections(const ao_state *s);
const ao_detection *ao_detections(const ao_state *s);
int ao_status(const ao_state *s);                  /* 0 ok, <0 capacity error */
uint64_t ao_quad_rcode(const ao_state *s, int i);   /* sampled code word of quad i */
float ao_quad_margin(const ao_state *s, int i);

/* tag families by name (NULL = tag36h11); -1 / 0 for an unknown name */
int ao_family_ncodes(const char *fam);
uint64_t ao_family_code(const char *fam, int i);   /* i-th entry */
int ao_family_id(const char *fam, int i);          /* its tag id */
void ao_family_bit(const char *fam, int i, int *x, int *y);
int ao_family_nbits(const char *fam);

/* deterministic math (exported for the accuracy tests) */
float ao_det_atan2f(float y, float x);
float ao_det_cosf(float x);
float ao_det_sinf(float x);
float ao_det_hypotf(float a, float b);

/* tag pose (ao_pose.c; estimate_tag_pose of the un-vendored AprilTag 3.x library,
 * called at apriltags_cuda_detector.cu:433).  R row-major, t in metres,
 * err = {err1, err2} object-space errors of the two minima (err2 = HUGE_VAL when
 * there is no second minimum).  Returns 1 when the second solution won. */
int ao_estimate_tag_pose(const double H[9], const double corners[4][2], double fx, double fy, double cx, double cy,
                         double tagsize, double R[9], double t[3], double err[2]);

/* shared game-piece preprocessing (ao_gp.c; preprocess_image of
 * game_piece_detection_node.cu:347-379): bgr h x w x 3 -> out channels x oh x ow */
int ao_gp_preprocess(const uint8_t *bgr, int w, int h, float *out, int ow, int oh, int channels);

/* helpers exposed for tests */
uint64_t ao_rotate90(uint64_t w);                 /* 36 bits */
uint64_t ao_rotate90_n(uint64_t w, int nbits);
int ao_unrank(int i, int *m0, int *m1, int *m2, int *m3);
/* ulp-sensitivity hook (tests only): see ao_oracle.c */
void ao_set_fp_perturb(int mask);

#ifdef __cplusplus
}
#endif
#endif
