// at_common.h -- shared host/device definitions of the MI355X AprilTag stage.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "at_detmath.h"

namespace at {

// ---- capacities -----------------------------------------------------------
// CCL tile: TW x 32 decimated pixels = TW/2 x 16 2x2-blocks per workgroup (one thread
// per block).  Throughput mode (max_batch >= kWideBlobMaxBatch) uses 64-wide tiles:
// twice the pixels per workgroup of a 32-wide tile for the same dependent round
// trips and a third fewer tile-border unions per pixel.  Latency mode (small
// batches, few workgroups per frame) uses 32-wide tiles: twice the workgroups,
// each with half the serial chain.
template <int TW>
struct CclTile {
  static constexpr int W = TW, H = 32;
  static constexpr int BW = TW / 2, BH = H / 2;  // blocks per tile row / column
  static constexpr int NT = BW * BH;            // threads per workgroup
  static constexpr int NODES = 3 * NT;          // union-find nodes of one tile
  static constexpr int ROW_NODES = 3 * BW;      // node slots per block row
};
constexpr int kCclTileH = 32;
constexpr int kCclTileNodesMax = CclTile<64>::NODES;  // stride of the per-tile local-root lists
// per-frame open-addressing table of blob pairs: 4096 slots hold every frame the
// 12-bit blob index admits (<= kMaxPairs keys; typical frames fill ~10 %), and keep
// k_pairs' LDS copy at 84 KB so it co-resides with other kernels' workgroups
constexpr int kHashSlots = 4096;
constexpr int kHashBits = 12;
constexpr int kPairEntCap = 65536;     // per-frame overflow (tile, pair, count) entries (tiles with > kLdsPairSlots pairs)
// k_boundary tiles: 64 x (4 * kBndRows) interior pixels per 256-thread workgroup;
// each tile owns a fixed region of kBndPts points and kLdsPairSlots pair entries
constexpr int kBndRows = 4;
constexpr int kBndPts = 64 * 4 * kBndRows * 4;  // worst case: 4 points per pixel (global region per tile)
constexpr int kBndStage = 1024;                 // of which staged in LDS (1 per pixel; typical tiles hold ~0.7)
constexpr int kLdsPairSlots = 512;
// tcnt flag: the tile's points are 4-B (entry index, point bits) words (k_boundary)
constexpr uint32_t kTileNarrow = 0x80000000u;
constexpr int kMaxTilesPerFrame = 1024;  // k_boundary tiles of one frame (k_pairs' LDS prefix); 1080p: 510
constexpr int kMaxCclTiles = 1024;       // CCL tiles of one frame (k_ccl_merge: one per thread)
// Border descriptor of a throughput-mode CCL tile (64 x 32 decimated pixels, 32 x 16
// blocks), written by k_thr_ccl, read by k_ccl_merge; u32 word offsets.  *thr:
// threshold bytes of row 0 (T), row 31 (B), column 0 (L), column 63 (R); *s?: the
// list slot (u16, 0xffff: no pixels) of the root of node F / L / R of each block of
// the top row, bottom row, left and right block column.
struct CclDesc {
  static constexpr int Tthr = 0, Bthr = 16, Lthr = 32, Rthr = 40;
  static constexpr int TsF = 48, TsL = 64, TsR = 80, BsF = 96, BsL = 112, BsR = 128;
  static constexpr int LsF = 144, LsL = 152, RsF = 160, RsR = 168;
  static constexpr int kWords = 176;
};
// k_ccl_merge's LDS: 12 B per listed local root (parent key, pixel count), or 10 B
// (parent key, tile) for frames with more roots (counts summed at L2)
// next to the per-tile prefix, within the 160 KiB one workgroup may hold
constexpr int kMergeCapMax = 15360;
constexpr int kMergeLdsMax = kMergeCapMax * 10;  // (+ the per-tile prefix: within 160 KiB)
constexpr int kMaxPairs = 4096;        // 12-bit blob index of IndexPoint (points.h:183-193)
constexpr int kSortCap = 8192;         // points of one blob sorted in LDS (>= 2*(W+H) for 1080p)
constexpr int kBlobThreads = 256;
// Blobs of more than kSmallBlob points: one workgroup each, 512 threads for
// small batches (latency: the biggest blob is the critical path), 256 for
// large batches (throughput: more blobs in flight per CU).
constexpr int kWideBlobMaxBatch = 8;
constexpr int kSmallBlob = 512;        // blobs up to this many points go one-wave-per-blob
constexpr int kNMaxima = 10;
// RefineEdges samples of one quad (<= perimeter / 8 + 64, k_decode): the first
// kLdsRefine in LDS, the rest in the decode workgroup's global scratch
constexpr int kMaxRefineSamples = 1536;
#ifndef AT_LDS_REFINE
#define AT_LDS_REFINE 256
#endif
constexpr int kLdsRefine = AT_LDS_REFINE;
constexpr int kDecodeGridPerBlobWg = 8;  // k_decode workgroups <= nblobwg * this
// k_decode's persistent grid for a batch of B frames: enough one-wave groups for
// every quad of a full batch to start at once (16 per CU at 8.5 KB LDS)
inline int decode_grid(int nblobwg, int B) {
  const int hi = nblobwg * kDecodeGridPerBlobWg, want = 64 * B;
  return nblobwg * 2 > (want < hi ? want : hi) ? nblobwg * 2 : (want < hi ? want : hi);
}

// ---- stages of one launch sequence (per-stage event timing) ----------------
constexpr int kNumStages = 12;
constexpr const char* kStageNames[kNumStages] = {"k_pre",   "k_thr_ccl", "k_ccl_merge", "k_ccl_roots",
                                                 "k_boundary", "k_pairs", "k_group",     "k_extents",
                                                 "k_blob_small", "k_blob", "k_decode",   "k_pose"};

// ---- blob size classes of the work lists, processed largest first ----------
// 0-2: large blobs (> kSmallBlob points, workgroup per blob), 3-6: small blobs
// (wave per blob).  Longest-first order shortens the persistent kernels' tail.
constexpr int kNumCls = 7;
constexpr int kNumLargeCls = 3;

// ---- per-frame status bits -------------------------------------------------
constexpr uint32_t kStatusPairsOverflow = 1u;   // N_q > kMaxPairs
constexpr uint32_t kStatusHashFull = 2u;
constexpr uint32_t kStatusDetsOverflow = 4u;
constexpr uint32_t kStatusPointsOverflow = 8u;
constexpr uint32_t kStatusQuadsOverflow = 16u;
constexpr uint32_t kStatusPairsCapped = 32u;  // > kMaxPairs pairs: the first kMaxPairs (rank order) processed
constexpr int kMaxBatch = 256;          // frames per launch sequence (at_config.max_batch)
// Every kept blob pair can yield one accepted quad and every accepted quad at most
// one detection, so sizing both queues by kMaxPairs makes neither of them a cap:
// the reference decodes every quad (apriltag_detect.cu:618-663).
constexpr int kQcStride = 32;  // words between two frames' accepted-quad counters (DevBufs::nqcand)
constexpr int kQuadCandPerFrame = kMaxPairs;  // accepted quads queued for decode, per frame
constexpr int kMaxDets = kQuadCandPerFrame;   // candidate detections one frame can have (before reconcile)
// Candidate detections: every frame owns kMaxDets records in HBM (frame f's k-th
// candidate, k from the frame's own counter, at f * kMaxDets + k: no frame can take
// another's slots, so what a frame returns depends on that frame alone).  The first
// kDetPoolPerFrame of them are mirrored into the pinned, mapped host buffer as they
// are written (zero-copy results); a frame with more candidates (pathological
// inputs) has the rest copied from HBM at at_collect.
constexpr int kDetPoolPerFrame = 128;
constexpr int kMaxCodes = 1024;               // codebook entries (tag36h11: 587)
constexpr int kMaxFamilyBits = 64;

// Tag family as quad_decode_index uses it (apriltag_family_t: nbits, bit_x/bit_y,
// width_at_border, total_width, reversed_border); the codebook itself lives in
// HBM (DevBufs::book_code / book_id), one per detector.
struct FamilyDesc {
  int nbits;            // data bits (16, 25, 36)
  int width_at_border;  // cells across the black border (d + 2)
  int total_width;      // cells across incl. the white quiet zone (d + 4)
  int reversed_border;
  int ncodes;
  int8_t bitx[kMaxFamilyBits], bity[kMaxFamilyBits];  // 3.x layout, border coordinates
};

// Frame geometry (all derived from W, H).
struct Geom {
  int W, H, Wd, Hd;     // full / decimated
  int TW, TH;           // 4x4 threshold tiles
  int BW, BH;           // 2x2 CCL blocks
  int CTX, CTY;         // CCL tiles
  int ctw;              // CCL tile width (32: latency mode, 64: throughput mode)
  int merge_cap;        // k_ccl_merge: listed local roots one frame's LDS holds (0: no k_ccl_merge)
  int merge_lds;        // k_ccl_merge's dynamic LDS bytes (12 B per root + link lists, up to kMergeLdsMax)
  int nlarge;           // size classes 0 .. nlarge-1 go to the workgroup-team blob kernel
  int bnd_region;       // points per k_boundary tile region (kBndPts)
  int cap_pts;          // 4 * (Wd-2) * (Hd-2)
  int BTX, BTY, ntb;    // k_boundary tiles (64 x 4*kBndRows interior pixels each)
  uint32_t min_cluster; // max(24, min_cluster_pixels)
  uint32_t max_cluster; // 2 * (W + H)
  int min_tag_width;    // width_at_border / quad_decimate, >= 3
};

struct Params {
  int min_white_black_diff;
  float max_line_fit_mse;
  double cos_critical_rad;
  double decode_sharpening;
  int refine_edges;
  double fx, fy, cx, cy, k1, k2, p1, p2, k3;
  int diag_stop;  // diagnostics only (AT_DIAG_BLOB_STOP): k_blob returns after phase N; 0 = full
  double tag_size;  // metres; > 0 runs k_pose (apriltags_cuda_detector.hpp:39 TAGSIZE)
  int probe;      // diagnostics only (AT_PHASE_PROBE): kernels stamp phase clocks into DevBufs::probe
  int taps;       // write the sorted IndexPoint parity tap (AT_STAGE_BLOB_POINTS) over the grouped points
  int wide_blob;  // AT_WIDE_BLOB=1: 512-thread large-blob teams at every batch size (experiment)
  int pipe_stop;  // diagnostics only (AT_DIAG_PIPE_STOP): launch the stages < N only; 0 = all
  int lblob_wg;   // throughput-mode large-blob kernel's persistent grid (AT_LBLOB_WG; 0: nblobwg)
  int sblob_wg;   // small-blob kernel's persistent grid (AT_SBLOB_WG; 0: 2 nblobwg)
  int dec_wg;     // k_decode's persistent grid (AT_DEC_WG, experiment; 0: decode_grid)
  FamilyDesc fam;
  int gp_w, gp_h, gp_c;  // game-piece preprocessing output (at_gp_enable); gp_c == 0: off
};
constexpr int kProbeWords = 256;

// The diagnostics above (stage cut-offs, phase probes) exist only in a build with
// -DAT_EXPERIMENTS (`make exp`); in the product build they are compile-time off,
// whatever Params holds.
#ifdef AT_EXPERIMENTS
#define AT_DIAG_STOP(prm, n) ((prm).diag_stop == (n))
#define AT_PIPE_STOP(prm) ((prm).pipe_stop)
#define AT_PROBE_ON(prm) ((prm).probe != 0)
#define AT_DIAG_ANY(prm) ((prm).diag_stop != 0)
#else
#define AT_DIAG_STOP(prm, n) false
#define AT_PIPE_STOP(prm) 0
#define AT_PROBE_ON(prm) false
#define AT_DIAG_ANY(prm) false
#endif

// HIP events bracketing one kernel of the launch sequence (bench roofline).
// With `split` set (graph replay), the launch sequence calls split(ctx, 0) before
// and split(ctx, 1) after the timed kernel instead of recording the events, so
// the caller can cut its stream capture there and record the events between
// graph segments.
struct KernelTimer {
  int stage;
  hipEvent_t t0, t1;
  hipError_t (*split)(void* ctx, int which);
  void* ctx;
};

// One detection candidate as produced on the device (before reconcile).
struct DevDetection {
  int32_t id;
  int16_t hamming;
  uint16_t frame;  // frame of the batch (the pool is batch-wide)
  float decision_margin;
  int32_t blob_rank;
  double H[9];
  double c[2];
  double p[4][2];
  // estimate_tag_pose (k_pose, when Params::tag_size > 0)
  double pose_R[9];
  double pose_t[3];
  double pose_err[2];  // errors of the first / second minimum (HUGE_VAL: none)
};

// Accepted quad (corners after AdjustPixelCenters) queued for RefineEdges + decode
// (the blob kernels append accepted quads only, through the per-frame counter).
struct QuadCand {
  uint32_t frame, rank;
  float p[4][2];
};

struct QuadRecord {
  uint32_t blob_index, valid, accepted;
  uint16_t indices[4];
  float corners[4][2];
};

// Moments of a run of line-fit points in the reference's widths (LineFitPoint sums,
// line_fit_filter.h:61-83), with the run's point count.
struct Moments {
  int32_t Mx, My, W;
  int64_t Mxx, Myy, Mxy;
  int32_t N;
};

// A kept blob's side fits left to k_quad_fin (throughput mode): per side segment of its
// best combination, FitLine's (float)(Cxx - Cyy), (float)(2 Cxy) and centroid quotients
// (all the corners need of the fit), and the record's fields.  The blob's team writes
// them (threads 0-3 a segment each); k_quad_fin finishes the four lines, the corners
// and the Heron / angle tests.
struct QuadPend {
  float fit[4][4];
  uint32_t blob_index, valid;
  uint16_t indices[4];
};
static_assert(sizeof(QuadPend) == 80, "QuadPend: 80 B per kept blob");

// One 2-px-thick segment of the annotated image (at_draw_outlines_device).
struct DrawPrim {
  double x0, y0, x1, y1;
  uint8_t bgr[3];
};

// Device buffers; every per-frame array is [max_batch][per-frame size].
struct DevBufs {
  const uint8_t* const* frames;   // device table of frame pointers
  uint8_t* gray;      // [B][W*H]
  uint8_t* dec;       // [B][Wd*Hd]
  uint8_t* mm;        // [B][TW*TH*2]   unfiltered 4x4 min/max
  uint8_t* thr;       // [B][Wd*Hd]
  uint32_t* par;      // [B][Wd*Hd]     union-find parents indexed by node id
  uint32_t* lroot;    // [B][CTX*CTY][kCclTileNodesMax] local roots of each CCL tile (global node ids)
  uint32_t* nlroot;   // [B][CTX*CTY]
  uint32_t* lcnt;     // [B][CTX*CTY][kCclTileNodesMax] pixel count of each listed local root
  uint32_t* cdesc;    // [B][CTX*CTY][CclDesc::kWords] border descriptors (throughput mode)
  uint32_t* ccl_ovf;  // [B] (control block) frames whose listed local roots exceeded k_ccl_merge's LDS
                      //     (k_ccl_merge resolves them in global memory: slow, rare)
  uint32_t* nlr_tot;  // [B] (control block) listed local roots of the frame (k_ccl_merge; statistics)
  uint32_t* size;     // [B][Wd*Hd]
  uint64_t* pts;      // [B][ntb][kBndPts] boundary points of each k_boundary tile, emission order
  uint32_t* tcnt;     // [B][ntb]        points of each tile
  uint32_t* tent;     // [B][ntb]        pair entries of each tile
  uint32_t* grp;      // [B][cap_pts]   boundary points grouped by pair rank: the low 24 bits of the
                      //                point key, (x << 14) | (y << 4) | (b2w << 3) | dxy
  uint64_t* keys;     // [B][cap_pts]   k_extents' (theta, plane, y, x | W) sort keys, same slots as grp
                      //                (and the blob kernels' IndexPoint parity tap)
  uint64_t* pent_key; // [B][ntb][kLdsPairSlots] per-tile pair histogram entries (rep01)
  uint32_t* pent_cnt; // [B][ntb][kLdsPairSlots]
  uint64_t* povf_key; // [B][kPairEntCap] entries of tiles whose LDS pair table overflowed
  uint32_t* povf_cnt; // [B][kPairEntCap]
  uint32_t* npent;    // [B] (control block) overflow entries; k_pairs then stores the frame's total entries
  uint64_t* ht_key;   // [B][kHashSlots]  written whole by k_pairs
  uint32_t* ht_cnt;   // [B][kHashSlots]
  uint32_t* ht_rank;  // [B][kHashSlots]
  uint32_t* ht_off;   // [B][kHashSlots]
  uint32_t* ht_cur;   // [B][kHashSlots]
  uint32_t* pair_cnt; // [B][kMaxPairs]
  uint32_t* pair_off; // [B][kMaxPairs]
  uint32_t* pair_sel; // [B][kMaxPairs]  1 if SelectBlobs kept the pair
  uint32_t* work;     // [kNumCls][wcap] (frame << 16) | rank of candidate pairs, by size class
  uint32_t wcap;      // B * kMaxPairs
  DevDetection* dets; // [B][kMaxDets] candidates of each frame (slot f * kMaxDets + k)
  uint32_t* det_work; // [B * kMaxDets] slots of the batch's candidates in claim order (k_pose's work list)
  uint32_t* det_head; // [1] k_pose work-list cursor (control block)
  uint32_t* dec_done; // [1] finished k_decode workgroups (control block; latency mode's fused pose)
  // zero-copy results: the detections (k_decode, poses added by k_pose) and the
  // control block (copied by k_pose) are also written straight into the
  // caller-visible pinned host buffers (device pointers of mapped host memory),
  // which replaces two device-to-host copies per batch
  DevDetection* hdets;  // [B][kDetPoolPerFrame] host mirror of each frame's first candidates
  uint32_t* hctrl;      // [ctrl_words] host
  uint32_t* ctrl;       // device control block base
  uint32_t ctrl_words;
  QuadRecord* quads;  // [B][kMaxPairs]  fitted-quad debug record of each kept blob, slot = pair rank
  QuadPend* qpend;    // [B][kMaxPairs]  side-fit inputs of each kept blob (throughput mode), slot = pair rank
  // control block (zeroed every batch)
  uint32_t* npts;     // [B]
  uint32_t* npairs;   // [B]
  uint32_t* ndets;    // [B] candidates per frame (the frame's slot cursor)
  uint32_t* nquads;   // [B]
  uint32_t* status;   // [B]
  uint32_t* ncls;     // [kNumCls] candidate pairs per size class
  uint32_t* workhead; // [1]
  uint64_t* probe;    // [kProbeWords] phase clock stamps (diagnostics)
  uint32_t* blob_pts;       // [2] points processed by the small / large blob kernels (batch statistics)
  uint32_t* workhead_small; // [1] dequeue head of the stage's second large-blob launch
  uint32_t* workhead_mid;   // [1] ... and of its third
  uint32_t* nqcand;   // [B][kQcStride] accepted quads queued for decode, per frame (qcand[f][kQuadCandPerFrame]):
                      //     a 128-B line per frame, so one frame's appends never wait behind another's
                      //     (zeroed with the control block, by the first kernel's block 0)
  uint32_t qc_words;  // B * kQcStride
  uint32_t* qhead;    // [1]
  QuadCand* qcand;    // [qcand_cap]
  uint32_t qcand_cap;
  double* rsamp;      // [decode workgroups][2][kMaxRefineSamples - kLdsRefine] refine samples past LDS
  const uint64_t* book_code;  // [fam.ncodes] codebook (3.x bit order)
  const int32_t* book_id;     // [fam.ncodes] tag id of each code
  float* gp_out;              // [B][gp_c][gp_h][gp_w] game-piece network input (at_gp_enable)
  // device-clock span of the timed kernel (bench roofline): the stage it is
  // (-1: none, set in the split graph's copy of DevBufs only), the control-block
  // words of its first workgroup's start / last workgroup's end (wall clock) and
  // the count of finished workgroups that finds the last one
  int32_t kt_stage;
  uint64_t* kstamp;   // [2] in the control block: span start / end (k_kt_span)
  uint32_t* kgrid;    // [1] in the control block: workgroups of the timed launch
  uint64_t* kwg;      // [2][kwg_cap] each workgroup's start / end stamp (plain stores)
  uint32_t kwg_cap;
  // per-workgroup scratch of the blob kernel
  uint64_t* s_pk;     // [nblobwg][kSortCap/2] peak keys beyond a large-blob team's LDS peak area
                      // (pathological blobs only; every other per-blob array lives in LDS)
};

}  // namespace at
