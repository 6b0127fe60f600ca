/*
 * at_api.h -- C ABI of the MI355X-native AprilTag detection stage.
 *
 * Drop-in boundary for the reference's per-frame detector
 * frc971::apriltag::GpuDetector (Team766/ros_vision,
 * src/apriltags_cuda/include/apriltags_cuda/apriltag_gpu.h:77-359), whose
 * caller is ApriltagsDetector::imageCallback
 * (src/apriltags_cuda/src/apriltags_cuda_detector.cu:382-557).  Plain C types
 * only; every entry point returns 0 or a negative AT_E* code (the reference
 * aborts through glog CHECK instead, cuda_frc971.h:14-17).
 *
 * Threading: one at_detector per camera stream (the reference owns one
 * GpuDetector + one CUDA stream per node, apriltag_gpu.h:240); calls on one
 * instance must not overlap.
 */
#ifndef AT_API_H_
#define AT_API_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AT_ABI_VERSION 5

enum {
  AT_OK = 0,
  AT_E_INVALID = -1,    /* bad argument / unsupported geometry */
  AT_E_HIP = -2,        /* HIP runtime error (no device, launch failure) */
  AT_E_CAPACITY = -3,   /* frame exceeded a fixed capacity (see at_frame_status) */
  AT_E_FAMILY = -4,     /* unknown tag family */
  AT_E_NOMEM = -5
};

typedef struct at_detector at_detector; /* opaque: device buffers + hipStream_t */

typedef enum { AT_FMT_YUYV = 0, AT_FMT_BGR8 = 1, AT_FMT_GRAY8 = 2 } at_pixfmt;

/* CameraMatrix + DistCoeffs (apriltag_gpu.h:61-74), read from
 * calibrationmatrix_<serial>.json by apriltags_cuda_detector.cu:315-371. */
typedef struct {
  double fx, fy, cx, cy;
  double k1, k2, p1, p2, k3;
} at_camera;

/* apriltag_detector_t fields the reference consults
 * (apriltags_cuda_detector.cu:139-147; apriltag_gpu.cu:166-181, 737, 884, 1084-1086). */
typedef struct {
  int width, height;          /* frame size; width%8==0, height%8==0, width*height < 2^22 */
  const char *family;         /* "tag36h11" (apriltags_cuda_detector.hpp:213), "tag25h9", "tag16h5";
                                 the apriltag 3 layouts give AT_E_FAMILY (apriltag_utils.cu:10-32) */
  float quad_decimate;        /* must be 2.0 (apriltag_gpu.cu:166) */
  int refine_edges;           /* 1 */
  double decode_sharpening;   /* 0.25 */
  int min_white_black_diff;   /* 5 */
  int min_cluster_pixels;     /* 5 */
  int max_nmaxima;            /* must be 10 (line_fit_filter.cu:1205) */
  float max_line_fit_mse;     /* 10.0 */
  double cos_critical_rad;    /* cos(10 deg) */
  int device;                 /* HIP device ordinal */
  int max_batch;              /* frames per at_detect_batch / at_detect_device call (1..256) */
  double tag_size;            /* metres; > 0 also estimates every tag's pose on the GPU
                                 (info_.tagsize = TAGSIZE 0.1651, apriltags_cuda_detector.cu:185,
                                 apriltags_cuda_detector.hpp:39); 0 = detection only */
} at_config;

/* apriltag_detection_t fields published downstream (apriltag.h; consumed at
 * apriltags_cuda_detector.cu:425-496). */
typedef struct {
  int32_t id;
  int32_t hamming;
  float decision_margin;
  double H[9];      /* row-major 3x3 homography, tag [-1,1]^2 -> pixels */
  double c[2];      /* centre */
  double p[4][2];   /* corners */
} at_detection;

/* Fills the reference defaults for a width x height camera. */
int at_config_default(at_config *cfg, int width, int height);

/* GpuDetector::GpuDetector (apriltag_gpu.cu:111-188): allocates every buffer
 * at worst-case size for max_batch frames; nothing is allocated per frame. */
int at_create(const at_config *cfg, const at_camera *cam, at_detector **out);

/* GpuDetector::Detect + Detections (apriltag_gpu.cu:725-1166,
 * apriltag_detect.cu:618-663): one host frame in, detections sorted by id out.
 * *n receives the total found; at most cap are written. Synchronous. */
int at_detect(at_detector *d, const uint8_t *frame, at_pixfmt fmt, at_detection *out, int cap, int *n);

/* Batched host frames (one launch sequence for all frames; multi-camera). */
int at_detect_batch(at_detector *d, const uint8_t *const *frames, int nframes, at_pixfmt fmt,
                    at_detection *out, int cap_per_frame, int *n_per_frame);

/* Frames already resident in device memory: d_frames is a device pointer to
 * nframes frames laid out back to back (frame_stride bytes apart).  The kernels
 * read the frames until the last stage (the decode samples luma from YUYV / GRAY8
 * frames in place), so the buffer must stay unmodified until the call returns --
 * for at_enqueue_device, until at_collect returns. */
int at_detect_device(at_detector *d, const void *d_frames, size_t frame_stride, int nframes, at_pixfmt fmt,
                     at_detection *out, int cap_per_frame, int *n_per_frame);

/* Split-phase form of at_detect_device for pipelining: enqueue the batch on
 * the detector's stream and return immediately; at_collect waits for it and
 * runs the host tail (reconcile + sort by id).  d_frames must stay unmodified
 * until at_collect returns (see at_detect_device): a producer that reuses the
 * buffer must order its writes after at_collect, not after earlier work. */
int at_enqueue_device(at_detector *d, const void *d_frames, size_t frame_stride, int nframes, at_pixfmt fmt);
int at_collect(at_detector *d, at_detection *out, int cap_per_frame, int *n_per_frame);
/* Split-phase form of at_detect_batch (camera-fed pipelines): the host-to-device
 * copies of the frames (one per run of back-to-back frames; page-locked sources,
 * e.g. hipHostMalloc'd or registered, copy asynchronously) and the batch are
 * enqueued on the detector's stream, so with several detectors in turn the copies
 * of one batch overlap the kernels of another.  The frames must stay untouched
 * until at_collect. */
int at_enqueue_host(at_detector *d, const uint8_t *const *frames, int nframes, at_pixfmt fmt);

/* Stream ordering without a host wait: the detector's next enqueued batch starts
 * only after everything queued so far on `stream` (a hipStream_t of the same
 * device, e.g. the stream a frame scatter or copy was issued on; NULL = the null
 * stream) has completed.  Replaces a host synchronize between a producer of
 * device-resident frames and at_enqueue_device. */
int at_stream_wait(at_detector *d, void *stream);

/* Per-frame status of the last batch: 0 or AT_E_CAPACITY (a frame whose blob
 * pair count exceeded the reference's 12-bit blob index, points.h:183-193). */
int at_frame_status(at_detector *d, int frame);

/* Per-stage parity taps (the reference's Copy*To debug accessors,
 * apriltag_gpu.h:98-183).  Copies the named stage of frame `frame` of the
 * last batch into dst (host memory). Returns bytes copied or < 0. */
enum {
  AT_STAGE_GRAY = 0,        /* u8  [H][W] */
  AT_STAGE_DECIMATED = 1,   /* u8  [H/2][W/2] */
  AT_STAGE_THRESHOLD = 2,   /* u8  [H/2][W/2] in {0,127,255} */
  AT_STAGE_LABELS = 3,      /* u32 [H/2][W/2] */
  AT_STAGE_SIZES = 4,       /* u32 [H/2 * W/2] */
  AT_STAGE_NUM_POINTS = 5,  /* u32 count of boundary points N_c */
  AT_STAGE_NUM_PAIRS = 6,   /* u32 count of blob pairs N_q */
  AT_STAGE_QUADS = 7,       /* at_quad_record[] of fitted quads (see below) */
  AT_STAGE_POINTS = 8,      /* u64 QuadBoundaryPoint keys, in emission order (unordered) */
  AT_STAGE_BLOB_POINTS = 9, /* u64 IndexPoint keys of selected blobs, sorted (blob, theta) */
  AT_STAGE_NUM_PAIR_ENTRIES = 10, /* u32 per-tile pair-histogram entries (diagnostic) */
  AT_STAGE_PROBE = 11       /* u64[256] kernel phase clock stamps when AT_PHASE_PROBE is set (diagnostic) */
};
long long at_debug_copy(at_detector *d, int stage, int frame, void *dst, size_t bytes);
/* AT_STAGE_GRAY: the full-resolution gray plane is written for BGR8 batches (k_decode
 * samples it) and, for YUYV / GRAY8 batches, only while the debug taps are on (k_decode
 * then reads the frame's own luma); AT_E_INVALID otherwise.
 * AT_STAGE_BLOB_POINTS needs the blob kernels to write the sorted IndexPoint keys
 * back (8 B per point of every selected blob): off by default (production), on
 * with at_set_debug_taps(d, 1) for parity checks; AT_E_INVALID while off.
 * AT_STAGE_SIZES of a throughput-mode batch (max_batch >= 8) likewise needs the taps
 * (that mode carries the size test in the root words, not in the size plane), and so
 * does AT_STAGE_QUADS (the fitted-quad records are debug output only). */
int at_set_debug_taps(at_detector *d, int enable);

/* Fitted quad record (FitQuad + QuadCorners, line_fit_filter.h:130-135 and
 * apriltag_gpu.h:55-59). */
typedef struct {
  uint32_t blob_index;
  uint32_t valid;          /* FitQuads valid flag */
  uint32_t accepted;       /* passed UpdateFitQuads checks */
  uint16_t indices[4];
  float corners[4][2];     /* after AdjustPixelCenters (full resolution) */
} at_quad_record;

/* Per-stage GPU timing with HIP events between the kernels of the launch
 * sequence (the reference times every stage with CudaEvents and logs them at
 * VLOG(1), apriltag_gpu.cu:1118-1163).  at_stage_times writes the mean
 * milliseconds per batch of each stage to ms[0..n-1] and the number of timed
 * batches to ms[n]; returns n (the stage count) or < 0. */
int at_set_profiling(at_detector *d, int enable);
int at_stage_times(at_detector *d, double *ms, int cap);
const char *at_stage_name(int stage);

/* Live per-launch time of ONE kernel (stage index as at_stage_name) inside
 * the normal launch sequence (concurrent streams; direct launches instead of
 * the graph replay while a timer is set): HIP events bracket that kernel on
 * its own stream.  stage -1 switches it off.
 * at_kernel_time: mean ms per launch and number of launches since set. */
int at_set_kernel_timer(at_detector *d, int stage);
int at_kernel_time(at_detector *d, double *avg_ms, long long *launches);
/* The same launches timed on the device: first workgroup's start to last
 * workgroup's end on the GPU wall clock (the kernel's execution span, as a
 * rocprofv3 kernel trace measures it; the HIP events of at_kernel_time also
 * hold the time the launch waits on the stream for free compute units).
 * Stamped by k_thr_ccl, k_ccl_border, k_boundary, k_extents, k_blob_small,
 * k_blob and k_decode; 0 launches for the other stages. */
int at_kernel_span(at_detector *d, double *avg_ms, long long *launches);

/* Work counts of the last collected batch: [0] frames, [1] boundary points,
 * [2] blob pairs, [3] points processed by the small-blob kernel, [4] by the
 * large-blob kernel, [5] fitted quads, [6] decoded candidates (pre-reconcile);
 * host time of this detector since creation, microseconds: [7] waiting in
 * at_collect for the GPU, [8] in the host tail (reconcile, sort, poses);
 * CCL: [9] local roots listed for the cross-tile merge (all frames), [10] their
 * maximum over the frames, [11] frames merged by the multi-workgroup fallback.
 * Returns the number of entries written. */
int at_batch_stats(at_detector *d, uint64_t *out, int cap);

/* Tag pose of each detection of the last collected batch (row A23): the
 * reference node's estimate_tag_pose(&info_, &pose) per detection
 * (apriltags_cuda_detector.cu:425-436; AprilTag 3.x orthogonal iteration with
 * the second-minimum check), computed on the GPU by the k_pose kernel when
 * at_config.tag_size > 0.  Entry i belongs to detection i of the frame (the
 * id-sorted order at_collect returned).  Returns the count or < 0. */
typedef struct {
  int32_t id;
  double R[9];     /* row-major rotation, tag -> camera */
  double t[3];     /* tag centre in the camera frame, metres (pose.t) */
  double err;      /* object-space error returned by estimate_tag_pose */
} at_pose;
int at_poses(at_detector *d, int frame, at_pose *out, int cap);

/* Detections of frame `frame` of the last collected batch again (the same records
 * at_collect wrote, id order), e.g. when its cap_per_frame was smaller than the
 * count it reported.  Returns the count or < 0. */
int at_detections(at_detector *d, int frame, at_detection *out, int cap);
/* Most detections one frame can yield (candidates before reconcile; the reference
 * keeps every detection, apriltag_detect.cu:618-663): a cap_per_frame this large
 * never truncates. */
int at_max_detections(void);

/* The node's per-frame tail over those poses (apriltags_cuda_detector.cu:425-462,
 * 595-599): robot = R_ext * t + t_ext (transformCameraToRobot), distance = |t|
 * in the camera frame, records sorted by ascending distance (stable).  Host
 * only; extr_R row-major 3x3 (NULL = identity), extr_t 3 (NULL = zero). */
typedef struct {
  int32_t id;
  double camera[3];   /* aprilTagInCameraFrame */
  double robot[3];    /* aprilTagInRobotFrame */
  double distance;
  double err;         /* pose_error */
} at_tag_detection;
int at_tag_detections(const at_pose *poses, int n, const double *extr_R, const double *extr_t,
                      at_tag_detection *out);

/* Shared game-piece preprocessing: the network input of
 * preprocess_image (src/game_piece_detection/src/game_piece_detection_node.cu:347-379:
 * cv::resize INTER_LINEAR to out_width x out_height, BGR->RGB for 3 channels or
 * BGR->GRAY for 1, x 1/255, NCHW float) computed on the GPU from the same BGR8
 * frames the detector reads.  at_gp_enable adds it to the launch sequence (every
 * later batch of AT_FMT_BGR8 frames); at_gp_tensor gives frame `frame`'s tensor of
 * the last batch in device memory (channels x out_height x out_width floats, valid
 * until the next batch); at_gp_copy copies it to the host.  AT_E_INVALID when the
 * last batch was not BGR8.  at_gp_preprocess_device runs it standalone on one
 * device-resident BGR8 image on `stream` (a hipStream_t, NULL = default stream). */
int at_gp_enable(at_detector *d, int out_width, int out_height, int channels);
int at_gp_tensor(at_detector *d, int frame, const float **dev_ptr);
int at_gp_copy(at_detector *d, int frame, float *dst, size_t count);
int at_gp_preprocess_device(const uint8_t *bgr, int width, int height, float *out, int out_width, int out_height,
                            int channels, void *stream);

/* The annotated image on the GPU: the node's outlined frame
 * (apriltag_utils.cu:54-79, drawn on the host with cv::line / cv::putText by
 * apriltags_cuda_detector.cu:514-518) drawn onto a device-resident BGR8 image of
 * the detector's geometry (width x height x 3, row-major): per detection the four
 * sides (0-1 green, 0-3 red, 1-2 / 2-3 blue; corners truncated to int as
 * cv::Point does) and the id centred on c, 2-px segments.  Pixel-identical to
 * node/at_node.cpp's draw_detection_outlines (its digit glyphs, not OpenCV's
 * Hershey font).  `dets` as at_collect returned them (host memory).  Runs on the
 * detector's stream and returns when the image is drawn. */
int at_draw_outlines_device(at_detector *d, const at_detection *dets, int n, uint8_t *bgr);

/* The node's published image for a host-fed BGR8 frame without a host copy and
 * redraw: draws those outlines onto frame `frame` of the last batch where
 * at_detect / at_detect_batch staged it in HBM, and copies the annotated image
 * (width x height x 3) to `bgr_out` in host memory.  AT_E_INVALID unless the last
 * batch was host BGR8 frames.  The staged copy is consumed (overwritten). */
int at_annotate_staged(at_detector *d, int frame, const at_detection *dets, int n, uint8_t *bgr_out);

/* Page-locked host memory (hipHostMalloc) for buffers the detector copies into on
 * its stream by DMA, e.g. at_annotate_staged's bgr_out: a pageable destination
 * goes through the runtime's staging buffers instead.  (No counterpart in the
 * reference: its node copies the image with cv_bridge, apriltags_cuda_detector.cu:514-518.)
 * Returns AT_OK / AT_E_NOMEM; at_host_free(NULL) is a no-op. */
int at_host_alloc(size_t bytes, void **out);
void at_host_free(void *p);

void at_destroy(at_detector *d);
const char *at_strerror(int code);

/* Family data (host only, no device needed). */
int at_family_num_known(const char *family);
int at_family_entry(const char *family, int i, int *id, uint64_t *code);

/* Library self-description. */
int at_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* AT_API_H_ */
