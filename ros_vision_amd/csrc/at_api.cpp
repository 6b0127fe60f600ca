// at_api.cpp -- host side of the C ABI (include/at_api.h).
//
// Owns the device buffers (sized once, for max_batch frames at worst case,
// like GpuDetector's constructor, apriltag_gpu.cu:111-188), launches the
// kernel pipeline on one HIP stream and runs the small host tail: order the
// per-frame candidates by blob rank (the reference decodes quads in blob-index
// order, apriltag_detect.cu:642-658), reconcile_detections and zarray_sort by
// id (apriltag_detect.cu:660-662).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/at_api.h"
#include "at_common.h"

namespace at {
hipError_t launch_tap_sizes(const uint8_t* thr, const uint32_t* par, const uint32_t* size, uint32_t* out, int Wd,
                            int Hd, hipStream_t st);
hipError_t launch_tap_labels(const uint8_t* thr, const uint32_t* par, uint32_t* out, int Wd, int Hd, hipStream_t st);
hipError_t launch_gp_preprocess(const uint8_t* src, int w, int h, float* out, int ow, int oh, int c, hipStream_t st);
hipError_t launch_draw(const DrawPrim* prims, int n, uint32_t* last, uint8_t* bgr, int W, int H, hipStream_t st);
hipError_t prepare_kernels(const Geom& g);
hipError_t launch_pipeline(const DevBufs& b, const Geom& g, const Params& prm, int B, int fmt, int nblobwg,
                           hipStream_t st, hipEvent_t* ev, hipStream_t st2, hipEvent_t fork, hipEvent_t join,
                           const KernelTimer* kt);

struct CodeEntry {
  int id;
  uint64_t code;
};
static const CodeEntry kTag36h11[] = {
#include "at_tag36h11_codes.inc"
};
static const CodeEntry kTag25h9[] = {
#include "at_tag25h9_codes.inc"
};
static const CodeEntry kTag16h5[] = {
#include "at_tag16h5_codes.inc"
};

// The families setup_tag_family selects by name (apriltag_utils.cu:10-32).  The
// classic square ones are built: d x d data cells, a one-cell black border
// (width_at_border d + 2), a white quiet zone (total_width d + 4), normal border,
// 2 bits corrected (apriltag_detector_add_family).  The apriltag 3 layouts
// (tagCircle21h7, tagCircle49h12, tagStandard41h12, tagStandard52h13,
// tagCustom48h12) are named but have no codebook here: their tables live in the
// un-vendored upstream sources and could not be regenerated offline, so
// at_create reports AT_E_FAMILY for them.
struct FamilyInfo {
  const char* name;
  int d;
  const CodeEntry* codes;
  int ncodes;
};
#define AT_NCODES(a) ((int)(sizeof(a) / sizeof((a)[0])))
static const FamilyInfo kFamilies[] = {
    {"tag36h11", 6, kTag36h11, AT_NCODES(kTag36h11)},
    {"tag25h9", 5, kTag25h9, AT_NCODES(kTag25h9)},
    {"tag16h5", 4, kTag16h5, AT_NCODES(kTag16h5)},
};

static const FamilyInfo* find_family(const char* name) {
  if (!name) return nullptr;
  for (const FamilyInfo& f : kFamilies)
    if (!strcmp(f.name, name)) return &f;
  return nullptr;
}

// apriltag_family_t fields quad_decode_index reads; bit_x / bit_y in the 3.x
// layout of tagXXhY.c: the upper triangle of the top-left quadrant row by row,
// rotated by 90 degrees three more times ((x, y) -> (d+1-y, x)), the centre
// cell last when d is odd
static FamilyDesc family_desc(const FamilyInfo& f) {
  FamilyDesc fd{};
  const int d = f.d;
  fd.nbits = d * d;
  fd.width_at_border = d + 2;
  fd.total_width = d + 4;
  fd.reversed_border = 0;
  fd.ncodes = f.ncodes;
  int n = 0;
  for (int r = 0; r < 4; r++)
    for (int y = 1; y <= d / 2; y++)
      for (int x = y; x <= d - y; x++) {
        int xx = x, yy = y;
        for (int i = 0; i < r; i++) {
          const int t = xx;
          xx = d + 1 - yy;
          yy = t;
        }
        fd.bitx[n] = (int8_t)xx;
        fd.bity[n] = (int8_t)yy;
        n++;
      }
  if (d & 1) {
    fd.bitx[n] = (int8_t)(d / 2 + 1);
    fd.bity[n] = (int8_t)(d / 2 + 1);
  }
  return fd;
}
}  // namespace at

using namespace at;

// control block layout (u32 words, zeroed every batch): per-frame arrays of B
// words, then scalars
enum { kCtlNpts, kCtlNpairs, kCtlNdets, kCtlNquads, kCtlStatus, kCtlNpent, kCtlNqcand, kCtlCclOvf, kCtlNlr,
       kCtlPerFrame };
enum { kCtlWorkhead = 0, kCtlQhead = 1, kCtlWorkheadSmall = 2, kCtlBlobPts = 3, kCtlNcls = 5,
       kCtlDetHead = kCtlNcls + kNumCls, kCtlDecDone = kCtlDetHead + 1, kCtlWorkheadMid = kCtlDecDone + 1,
       kCtlScalars = kCtlWorkheadMid + 1 };

static constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;

struct at_detector {
  at_config cfg;
  at_camera cam;
  Geom g;
  Params prm;
  int B;
  int device;
  int nblobwg;
  hipStream_t st;
  hipStream_t st2;          // fork/join branch for the large-blob kernel (latency mode)
  hipEvent_t ev_fork, ev_join;
  DevBufs d;
  std::vector<void*> allocs;
  uint8_t* d_in;            // staging for host frames [B][max frame bytes]
  size_t in_stride;
  const uint8_t** h_ftab;   // frame pointer table (mapped, fine-grained host memory; k_pre reads it)
  uint32_t* d_ctrl;         // control block (zeroed each batch)
  size_t ctrl_words;
  size_t kstamp_word;       // first of the timed kernel's stamp words in the control block
  double wclk_khz;          // device wall clock (s_memrealtime) rate
  double kd_ms;             // device-clock spans of the timed kernel (sum) and their count
  long long kd_n;
  uint32_t* h_ctrl;         // pinned copy of the control block
  DevDetection* h_dets;     // pinned [B][kDetPoolPerFrame]: mirror of each frame's first candidates (mapped)
  // results of the last collected batch: frame f's detections are the records
  // res_base[f][res_idx[f * kMaxDets + i]], i < res_n[f], in id order (after reconcile);
  // res_base[f] is the frame's host mirror, or res_ovf[f] (its candidates copied from
  // HBM) when it had more than kDetPoolPerFrame
  std::vector<int> res_idx, res_n;
  std::vector<const DevDetection*> res_base;
  std::vector<std::vector<DevDetection>> res_ovf;
  int last_nframes;
  int last_fmt;
  int last_gray;            // the last batch wrote the gray plane (AT_STAGE_GRAY)
  int last_sizes;           // ... and the size plane (AT_STAGE_SIZES)
  int last_staged;          // the last batch's frames were host frames staged in d_in (at_detect*)
  int last_gp;              // the last batch ran the game-piece preprocessing (k_gp_pre)
  int pending;
  hipEvent_t ev_done;
  hipEvent_t ev_ext;                      // at_stream_wait: recorded on the producer's stream
  int use_graphs;                         // replay the launch sequence as a hipGraph (AT_NO_GRAPH=1 disables)
  std::map<int, hipGraphExec_t> graphs;   // key: nframes * 4 + fmt
  // kernel timer under graph replay: the sequence cut around the timed kernel into
  // three graphs, timing events recorded between them (key: graph key * 32 + stage)
  struct SplitGraphs { hipGraphExec_t seg[3]; };
  std::map<int, SplitGraphs> split_graphs;
  std::vector<hipGraph_t> cap_segs;      // segments collected during one capture
  KernelTimer kt;                         // kt.stage < 0: off
  double kt_ms;
  long long kt_n;
  int profiling;
  hipEvent_t ev_stage[kNumStages + 1];
  double stage_ms[kNumStages];
  long stage_batches;
  double host_wait_us, host_tail_us;  // cumulative time of at_collect in the event wait / the host tail
  // annotated image (at_draw_outlines_device): segments, last-writer plane (lazily allocated)
  DrawPrim* d_prims;
  size_t prims_cap;
  uint32_t* d_last;
};

// Experiment and diagnostic knobs (stage cut-offs, grid / tile overrides, phase
// probes, graph / fork switches) are read from the environment only by a build
// with -DAT_EXPERIMENTS (`make exp`, the A/B tools' library): a product build
// ignores the environment, so no variable can truncate the pipeline of a deployed
// detector (the reference either detects or aborts, cuda_frc971.h:14-17).
static const char* knob(const char* name) {
#ifdef AT_EXPERIMENTS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
static int knob_int(const char* name, int dflt) {
  const char* v = knob(name);
  return v ? atoi(v) : dflt;
}

static int hip_fail(hipError_t e) {
  if (e != hipSuccess) {
    fprintf(stderr, "at_api: HIP error %s\n", hipGetErrorString(e));
    return AT_E_HIP;
  }
  return AT_OK;
}
#define HIPCHK(x)                          \
  do {                                     \
    hipError_t e_ = (x);                   \
    if (e_ != hipSuccess) return hip_fail(e_); \
  } while (0)

extern "C" {

int at_abi_version(void) { return AT_ABI_VERSION; }

const char* at_strerror(int code) {
  switch (code) {
    case AT_OK: return "ok";
    case AT_E_INVALID: return "invalid argument or unsupported frame geometry";
    case AT_E_HIP: return "HIP runtime error";
    case AT_E_CAPACITY: return "frame exceeded a fixed capacity";
    case AT_E_FAMILY: return "unknown tag family";
    case AT_E_NOMEM: return "out of memory";
    default: return "unknown error";
  }
}

int at_family_num_known(const char* family) {
  const FamilyInfo* f = find_family(family);
  return f ? f->ncodes : AT_E_FAMILY;
}

int at_family_entry(const char* family, int i, int* id, uint64_t* code) {
  const FamilyInfo* f = find_family(family);
  if (!f) return AT_E_FAMILY;
  if (i < 0 || i >= f->ncodes) return AT_E_INVALID;
  if (id) *id = f->codes[i].id;
  if (code) *code = f->codes[i].code;
  return AT_OK;
}

int at_config_default(at_config* cfg, int width, int height) {
  if (!cfg) return AT_E_INVALID;
  memset(cfg, 0, sizeof(*cfg));
  cfg->width = width;
  cfg->height = height;
  cfg->family = "tag36h11";
  cfg->quad_decimate = 2.0f;
  cfg->refine_edges = 1;
  cfg->decode_sharpening = 0.25;
  cfg->min_white_black_diff = 5;
  cfg->min_cluster_pixels = 5;
  cfg->max_nmaxima = 10;
  cfg->max_line_fit_mse = 10.0f;
  cfg->cos_critical_rad = cos(10.0 * M_PI / 180.0);
  cfg->device = 0;
  cfg->max_batch = 1;
  cfg->tag_size = 0.1651;  // TAGSIZE, apriltags_cuda_detector.hpp:39
  return AT_OK;
}

void at_destroy(at_detector* d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->st) (void)hipStreamSynchronize(d->st);
  if (d->st2) (void)hipStreamSynchronize(d->st2);
  for (auto& kv : d->graphs) (void)hipGraphExecDestroy(kv.second);
  d->graphs.clear();
  for (auto& kv : d->split_graphs)
    for (auto* g : kv.second.seg) (void)hipGraphExecDestroy(g);
  d->split_graphs.clear();
  for (void* p : d->allocs) (void)hipFree(p);
  if (d->h_ftab) (void)hipHostFree(d->h_ftab);
  if (d->h_ctrl) (void)hipHostFree(d->h_ctrl);
  if (d->h_dets) (void)hipHostFree(d->h_dets);
  if (d->d_prims) (void)hipFree(d->d_prims);
  if (d->d_last) (void)hipFree(d->d_last);
  if (d->ev_done) (void)hipEventDestroy(d->ev_done);
  if (d->ev_ext) (void)hipEventDestroy(d->ev_ext);
  for (int i = 0; i <= kNumStages; i++)
    if (d->ev_stage[i]) (void)hipEventDestroy(d->ev_stage[i]);
  if (d->kt.t0) (void)hipEventDestroy(d->kt.t0);
  if (d->kt.t1) (void)hipEventDestroy(d->kt.t1);
  if (d->ev_fork) (void)hipEventDestroy(d->ev_fork);
  if (d->ev_join) (void)hipEventDestroy(d->ev_join);
  if (d->st2) (void)hipStreamDestroy(d->st2);
  if (d->st) (void)hipStreamDestroy(d->st);
  delete d;
}

int at_create(const at_config* cfg, const at_camera* cam, at_detector** out) {
  if (!cfg || !cam || !out) return AT_E_INVALID;
  *out = nullptr;
  const FamilyInfo* fam = find_family(cfg->family);
  if (!fam || fam->ncodes > kMaxCodes) return AT_E_FAMILY;
  const int W = cfg->width, H = cfg->height;
  // GpuDetector preconditions (apriltag_gpu.cu:166-167, 754-755, 774; line_fit_filter.cu:1205)
  if (W <= 16 || H <= 16 || W % 8 || H % 8 || (long)W * H >= (1L << 22)) return AT_E_INVALID;
  if (cfg->quad_decimate != 2.0f || cfg->max_nmaxima != 10 || cfg->max_batch < 1 || cfg->max_batch > kMaxBatch)
    return AT_E_INVALID;
  if (2 * (W + H) > kSortCap) return AT_E_INVALID;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg->device) return AT_E_HIP;
  at_detector* d = new at_detector();  // value-initialised: every pointer null
  d->cfg = *cfg;
  d->cfg.family = fam->name;
  d->cam = *cam;
  d->device = cfg->device;
  d->B = cfg->max_batch;
  Geom& g = d->g;
  g.W = W; g.H = H; g.Wd = W / 2; g.Hd = H / 2;
  g.TW = g.Wd / 4; g.TH = g.Hd / 4;
  g.BW = g.Wd / 2; g.BH = g.Hd / 2;
  g.ctw = d->B < kWideBlobMaxBatch ? 32 : 64;
  if (knob("AT_CCL_TILE")) g.ctw = knob_int("AT_CCL_TILE", 64) == 32 ? 32 : 64;
  // size classes of the workgroup-team blob kernel (the rest: one wave per blob);
  // latency mode gives the team blobs of more than 256 points too (its chain is
  // the slowest single blob)
  g.nlarge = g.ctw == 32 ? std::max(kNumLargeCls, std::min(kNumCls, knob_int("AT_NLARGE", kNumLargeCls)))
                        : kNumLargeCls;  // (experiment knob: 3..kNumCls)
  g.CTX = (g.Wd + g.ctw - 1) / g.ctw;
  g.CTY = (g.Hd + kCclTileH - 1) / kCclTileH;
  // throughput mode: the cross-tile merge of the CCL in one workgroup's LDS per
  // frame (k_ccl_merge), room for 80 listed local roots per tile (typical 720p
  // frames list ~40), at most what 160 KiB hold; latency mode keeps the
  // multi-workgroup border / roots kernels (one frame: their parallelism is the chain)
  g.merge_cap = g.ctw == 64 ? std::min(kMergeCapMax, 80 * g.CTX * g.CTY) : 0;
  // 12 B per root (parent key + pixel count) and the wave link lists (8 KB)
  g.merge_lds = std::min(g.merge_cap * 12 + 8192, kMergeLdsMax);
  if (g.CTX * g.CTY > kMaxCclTiles) {
    at_destroy(d);
    return AT_E_INVALID;
  }
  g.cap_pts = 4 * (g.Wd - 2) * (g.Hd - 2);
  g.BTX = (g.Wd - 2 + 63) / 64;
  g.BTY = (g.Hd - 2 + 4 * kBndRows - 1) / (4 * kBndRows);
  g.ntb = g.BTX * g.BTY;
  g.bnd_region = kBndPts;
  g.bnd_region = std::max(kBndStage, std::min(kBndPts, knob_int("AT_BND_REGION", kBndPts)));  // (experiment knob)
  if (g.ntb > kMaxTilesPerFrame) {
    at_destroy(d);
    return AT_E_INVALID;
  }
  g.min_cluster = (uint32_t)std::max(24, cfg->min_cluster_pixels);
  g.max_cluster = (uint32_t)(2 * (W + H));
  // GpuDetector ctor (apriltag_gpu.cu:169-181): width_at_border / quad_decimate, >= 3
  g.min_tag_width = std::max(3, (fam->d + 2) / 2);
  Params& p = d->prm;
  p.min_white_black_diff = cfg->min_white_black_diff;
  p.max_line_fit_mse = cfg->max_line_fit_mse;
  p.cos_critical_rad = cfg->cos_critical_rad;
  p.decode_sharpening = cfg->decode_sharpening;
  p.refine_edges = cfg->refine_edges;
  p.fx = cam->fx; p.fy = cam->fy; p.cx = cam->cx; p.cy = cam->cy;
  p.k1 = cam->k1; p.k2 = cam->k2; p.p1 = cam->p1; p.p2 = cam->p2; p.k3 = cam->k3;
  p.diag_stop = knob_int("AT_DIAG_BLOB_STOP", 0);
  p.probe = knob_int("AT_PHASE_PROBE", 0);
  p.taps = 0;  // debug taps off: at_set_debug_taps
  p.wide_blob = knob_int("AT_WIDE_BLOB", 0);
  p.pipe_stop = knob_int("AT_DIAG_PIPE_STOP", 0);
  p.lblob_wg = knob("AT_LBLOB_WG") ? std::max(16, knob_int("AT_LBLOB_WG", 0)) : 0;  // experiment
  p.sblob_wg = knob("AT_SBLOB_WG") ? std::max(16, knob_int("AT_SBLOB_WG", 0)) : 0;  // experiment
  p.dec_wg = knob("AT_DEC_WG") ? std::max(16, knob_int("AT_DEC_WG", 0)) : 0;  // experiment
  p.fam = family_desc(*fam);
  d->use_graphs = !knob_int("AT_NO_GRAPH", 0);
  if (!(cfg->tag_size >= 0) || !std::isfinite(cfg->tag_size)) {
    at_destroy(d);
    return AT_E_INVALID;
  }
  p.tag_size = cfg->tag_size;

  auto fail = [&](int code) {
    at_destroy(d);
    return code;
  };
  if (hipSetDevice(d->device) != hipSuccess) return fail(AT_E_HIP);
  if (hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking) != hipSuccess) return fail(AT_E_HIP);
  if (hipEventCreateWithFlags(&d->ev_done, hipEventDisableTiming) != hipSuccess) return fail(AT_E_HIP);
  if (hipEventCreateWithFlags(&d->ev_ext, hipEventDisableTiming) != hipSuccess) return fail(AT_E_HIP);
  // Latency mode (max_batch < kWideBlobMaxBatch): the small-blob kernel runs on a
  // second stream beside the large-blob one.  Throughput mode: both on the one
  // stream -- concurrency comes from several detector instances (batches in
  // flight), which then each need one hardware queue only.  AT_NO_FORK=1 forces
  // the single-stream form.
  const bool fork = d->B < kWideBlobMaxBatch && !knob_int("AT_NO_FORK", 0);
  if (fork && hipStreamCreateWithFlags(&d->st2, hipStreamNonBlocking) != hipSuccess) return fail(AT_E_HIP);
  if (hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming) != hipSuccess) return fail(AT_E_HIP);
  if (hipEventCreateWithFlags(&d->ev_join, hipEventDisableTiming) != hipSuccess) return fail(AT_E_HIP);
  d->kt.stage = -1;
  d->kt.split = nullptr;
  d->kt.ctx = nullptr;
  // timing-only events: no system-scope fence (cache writeback) when they complete,
  // so bracketing a kernel does not slow it or its neighbours on other streams
  if (hipEventCreateWithFlags(&d->kt.t0, kTimingEventFlags) != hipSuccess ||
      hipEventCreateWithFlags(&d->kt.t1, kTimingEventFlags) != hipSuccess)
    return fail(AT_E_HIP);
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d->device);
  int wclk = 0;
  (void)hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, d->device);
  d->wclk_khz = wclk > 0 ? (double)wclk : 100000.0;  // s_memrealtime: 100 MHz
  d->nblobwg = std::max(64, ncu * 2);
  if (knob("AT_BLOB_WG")) d->nblobwg = std::max(16, knob_int("AT_BLOB_WG", 0));  // experiment: persistent grid size

  const size_t B = (size_t)d->B;
  const size_t npix = (size_t)W * H, nd = (size_t)g.Wd * g.Hd, nt = (size_t)g.TW * g.TH * 2;
  bool oom = false;
  auto dalloc = [&](size_t bytes) -> void* {
    void* ptr = nullptr;
    if (hipMalloc(&ptr, std::max<size_t>(bytes, 256)) != hipSuccess) {
      oom = true;
      return nullptr;
    }
    d->allocs.push_back(ptr);
    return ptr;
  };
  d->in_stride = (npix * 3 + 255) & ~(size_t)255;
  d->d_in = (uint8_t*)dalloc(B * d->in_stride);
  DevBufs& b = d->d;
  b.gray = (uint8_t*)dalloc(B * npix);
  b.dec = (uint8_t*)dalloc(B * nd);
  b.mm = (uint8_t*)dalloc(B * nt);
  b.thr = (uint8_t*)dalloc(B * nd);
  b.par = (uint32_t*)dalloc(B * nd * 4);
  b.lroot = (uint32_t*)dalloc(B * (size_t)g.CTX * g.CTY * kCclTileNodesMax * 4);
  b.nlroot = (uint32_t*)dalloc(B * (size_t)g.CTX * g.CTY * 4);
  b.lcnt = (uint32_t*)dalloc(B * (size_t)g.CTX * g.CTY * kCclTileNodesMax * 4);
  b.cdesc = (uint32_t*)dalloc(B * (size_t)g.CTX * g.CTY * CclDesc::kWords * 4);
  b.size = (uint32_t*)dalloc(B * nd * 4);
  const size_t ntb = (size_t)g.ntb;
  b.pts = (uint64_t*)dalloc(B * ntb * (size_t)g.bnd_region * 8);
  b.tcnt = (uint32_t*)dalloc(B * ntb * 4);
  b.tent = (uint32_t*)dalloc(B * ntb * 4);
  b.grp = (uint32_t*)dalloc(B * g.cap_pts * 4);
  b.keys = (uint64_t*)dalloc(B * g.cap_pts * 8);
  b.pent_key = (uint64_t*)dalloc(B * ntb * kLdsPairSlots * 8);
  b.pent_cnt = (uint32_t*)dalloc(B * ntb * kLdsPairSlots * 4);
  b.povf_key = (uint64_t*)dalloc(B * kPairEntCap * 8);
  b.povf_cnt = (uint32_t*)dalloc(B * kPairEntCap * 4);
  b.ht_key = (uint64_t*)dalloc(B * kHashSlots * 8);
  b.ht_cnt = (uint32_t*)dalloc(B * kHashSlots * 4);
  b.ht_rank = (uint32_t*)dalloc(B * kHashSlots * 4);
  b.ht_off = (uint32_t*)dalloc(B * kHashSlots * 4);
  b.ht_cur = (uint32_t*)dalloc(B * kHashSlots * 4);
  b.pair_cnt = (uint32_t*)dalloc(B * kMaxPairs * 4);
  b.pair_off = (uint32_t*)dalloc(B * kMaxPairs * 4);
  b.pair_sel = (uint32_t*)dalloc(B * kMaxPairs * 4);
  b.wcap = (uint32_t)(B * kMaxPairs);
  b.work = (uint32_t*)dalloc((size_t)kNumCls * B * kMaxPairs * 4);
  b.probe = (uint64_t*)dalloc(kProbeWords * 8);
  b.dets = (DevDetection*)dalloc(B * kMaxDets * sizeof(DevDetection));
  b.det_work = (uint32_t*)dalloc(B * kMaxDets * 4);
  b.quads = (QuadRecord*)dalloc(B * kMaxPairs * sizeof(QuadRecord));
  b.qpend = (QuadPend*)dalloc(B * kMaxPairs * sizeof(QuadPend));
  // control block: per-frame words, scalars, then (8-byte aligned) the timed
  // kernel's two wall-clock stamps and its finished-workgroup count
  d->kstamp_word = (kCtlPerFrame * B + kCtlScalars + 1) & ~(size_t)1;
  d->ctrl_words = d->kstamp_word + 5;
  d->d_ctrl = (uint32_t*)dalloc(((d->ctrl_words * 4 + 15) / 16) * 16);
  b.npts = d->d_ctrl + kCtlNpts * B;
  b.npairs = d->d_ctrl + kCtlNpairs * B;
  b.ndets = d->d_ctrl + kCtlNdets * B;
  b.nquads = d->d_ctrl + kCtlNquads * B;
  b.status = d->d_ctrl + kCtlStatus * B;
  b.npent = d->d_ctrl + kCtlNpent * B;
  b.qc_words = (uint32_t)(B * kQcStride);
  b.nqcand = (uint32_t*)dalloc((size_t)b.qc_words * 4);
  b.ccl_ovf = d->d_ctrl + kCtlCclOvf * B;
  b.nlr_tot = d->d_ctrl + kCtlNlr * B;
  uint32_t* sc = d->d_ctrl + kCtlPerFrame * B;
  b.workhead = sc + kCtlWorkhead;
  b.qhead = sc + kCtlQhead;
  b.workhead_small = sc + kCtlWorkheadSmall;
  b.workhead_mid = sc + kCtlWorkheadMid;
  b.blob_pts = sc + kCtlBlobPts;
  b.ncls = sc + kCtlNcls;
  b.det_head = sc + kCtlDetHead;
  b.dec_done = sc + kCtlDecDone;
  b.kt_stage = -1;
  b.kstamp = reinterpret_cast<uint64_t*>(d->d_ctrl + d->kstamp_word);
  b.kgrid = d->d_ctrl + d->kstamp_word + 4;
  b.kwg_cap = (uint32_t)(B * 1024 + 4096);  // >= the workgroups of any stamped launch (1080p: 510 tiles per frame)
  b.kwg = (uint64_t*)dalloc((size_t)b.kwg_cap * 2 * 8);
  b.qcand_cap = (uint32_t)(B * kQuadCandPerFrame);
  b.qcand = (QuadCand*)dalloc((size_t)b.qcand_cap * sizeof(QuadCand));
  // overflow area for the peak keys of pathological large blobs (one per large-blob team)
  b.s_pk = (uint64_t*)dalloc((size_t)2 * d->nblobwg * (kSortCap / 2) * 8);  // a slot per team (<= 2 nblobwg teams)
  // refine samples past LDS, one region per k_decode workgroup of the grid
  // launch_pipeline uses for a full batch (decode_grid)
  b.rsamp = (double*)dalloc((size_t)decode_grid(d->nblobwg, d->B) * 2 * (kMaxRefineSamples - kLdsRefine) * 8);
  if (oom) return fail(AT_E_NOMEM);
  if (prepare_kernels(g) != hipSuccess) return fail(AT_E_HIP);
  // frame pointer table: fine-grained mapped host memory read by k_pre directly
  // (no host-to-device copy per batch; the GPU does not cache it)
  if (hipHostMalloc((void**)&d->h_ftab, B * sizeof(void*), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return fail(AT_E_NOMEM);
  if (hipHostGetDevicePointer((void**)&b.frames, (void*)d->h_ftab, 0) != hipSuccess) return fail(AT_E_HIP);
  d->res_idx.assign(B * kMaxDets, 0);
  d->res_n.assign(B, 0);
  d->res_base.assign(B, nullptr);
  d->res_ovf.resize(B);
  if (hipHostMalloc((void**)&d->h_ctrl, d->ctrl_words * 4, hipHostMallocMapped) != hipSuccess) return fail(AT_E_NOMEM);
  if (hipHostMalloc((void**)&d->h_dets, B * kDetPoolPerFrame * sizeof(DevDetection), hipHostMallocMapped) != hipSuccess)
    return fail(AT_E_NOMEM);
  // device views of the mapped host result buffers (k_decode / k_pose write them)
  if (hipHostGetDevicePointer((void**)&b.hdets, d->h_dets, 0) != hipSuccess ||
      hipHostGetDevicePointer((void**)&b.hctrl, d->h_ctrl, 0) != hipSuccess)
    return fail(AT_E_HIP);
  b.ctrl = d->d_ctrl;
  b.ctrl_words = (uint32_t)d->ctrl_words;
  {
    // this detector's codebook in HBM (k_decode matches every entry in parallel)
    std::vector<uint64_t> codes(fam->ncodes);
    std::vector<int32_t> ids(fam->ncodes);
    for (int i = 0; i < fam->ncodes; i++) {
      codes[i] = fam->codes[i].code;
      ids[i] = fam->codes[i].id;
    }
    uint64_t* dc = (uint64_t*)dalloc(codes.size() * 8);
    int32_t* di = (int32_t*)dalloc(ids.size() * 4);
    if (oom) return fail(AT_E_NOMEM);
    if (hipMemcpy(dc, codes.data(), codes.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(di, ids.data(), ids.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      return fail(AT_E_HIP);
    b.book_code = dc;
    b.book_id = di;
  }
  // size arrays are read for every label by k_boundary: start defined
  if (hipMemsetAsync(b.size, 0, B * nd * 4, d->st) != hipSuccess) return fail(AT_E_HIP);
  if (hipStreamSynchronize(d->st) != hipSuccess) return fail(AT_E_HIP);
  *out = d;
  return AT_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// host tail: reconcile_detections + zarray_sort (apriltag 3.x apriltag.c,
// called at apriltag_detect.cu:660-662)
// ---------------------------------------------------------------------------
static bool seg_intersect(const double* a0, const double* a1, const double* b0, const double* b1) {
  const double ux = a1[0] - a0[0], uy = a1[1] - a0[1];
  const double vx = b1[0] - b0[0], vy = b1[1] - b0[1];
  const double den = ux * vy - uy * vx;
  if (fabs(den) < 1e-12) return false;
  const double t = ((b0[0] - a0[0]) * vy - (b0[1] - a0[1]) * vx) / den;
  const double w = ((b0[0] - a0[0]) * uy - (b0[1] - a0[1]) * ux) / den;
  return t >= 0 && t <= 1 && w >= 0 && w <= 1;
}
static bool poly_contains(const double poly[4][2], const double* pt) {
  bool inside = false;
  for (int i = 0, j = 3; i < 4; j = i++) {
    if (((poly[i][1] > pt[1]) != (poly[j][1] > pt[1])) &&
        (pt[0] < (poly[j][0] - poly[i][0]) * (pt[1] - poly[i][1]) / (poly[j][1] - poly[i][1]) + poly[i][0]))
      inside = !inside;
  }
  return inside;
}
static bool poly_overlap(const double a[4][2], const double b[4][2]) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++)
      if (seg_intersect(a[i], a[(i + 1) & 3], b[j], b[(j + 1) & 3])) return true;
  return poly_contains(a, b[0]) || poly_contains(b, a[0]);
}
static int prefer_smaller(int pref, double q0, double q1) {
  if (pref) return pref;
  if (q0 < q1) return -1;
  if (q1 < q0) return 1;
  return 0;
}

static void write_detection(const DevDetection& v, at_detection* o) {
  o->id = v.id;
  o->hamming = v.hamming;
  o->decision_margin = v.decision_margin;
  memcpy(o->H, v.H, sizeof(o->H));
  memcpy(o->c, v.c, sizeof(o->c));
  memcpy(o->p, v.p, sizeof(o->p));
}

// One frame's candidates: idx[0..ncand) are pool indices; on return idx[0..n) are
// the detections in id order (n is returned).
static int host_tail(const DevDetection* cand, int* idx, int ncand, at_detection* out, int cap) {
  // the reference's zarray operations on an index array (the 280-byte records stay
  // where k_decode / k_pose wrote them): order by blob rank, reconcile with the
  // same swap-with-last removals, stable sort by id
  std::stable_sort(idx, idx + ncand, [&](int a, int b) { return cand[a].blob_rank < cand[b].blob_rank; });
  int n = ncand;
  for (int i0 = 0; i0 < n; i0++) {
    for (int i1 = i0 + 1; i1 < n; i1++) {
      const DevDetection& a = cand[idx[i0]];
      const DevDetection& b = cand[idx[i1]];
      if (a.id != b.id) continue;
      if (!poly_overlap(a.p, b.p)) continue;
      int pref = 0;
      pref = prefer_smaller(pref, a.hamming, b.hamming);
      pref = prefer_smaller(pref, -a.decision_margin, -b.decision_margin);
      for (int k = 0; k < 3; k++) pref = prefer_smaller(pref, a.H[k], b.H[k]);
      if (pref < 0) {  // keep i0; zarray_remove_index(shuffle=1)
        if (i1 < n - 1) idx[i1] = idx[n - 1];
        n--;
        i1--;
      } else {
        if (i0 < n - 1) idx[i0] = idx[n - 1];
        n--;
        i0--;
        break;
      }
    }
  }
  std::stable_sort(idx, idx + n, [&](int a, int b) { return cand[a].id < cand[b].id; });
  for (int i = 0; i < n && i < cap; i++) write_detection(cand[idx[i]], out + i);
  return n;
}

// The per-batch sequence: frame table H2D, control block reset, the kernels,
// control block + detections D2H (all to/from pinned buffers whose addresses
// never change, so it can be captured once per (nframes, fmt) and replayed).
static hipError_t record_sequence(at_detector* d, int nframes, int fmt, hipStream_t st, hipEvent_t* ev,
                                  const KernelTimer* kt) {
  hipError_t e;
  DevBufs b = d->d;
  b.kt_stage = kt ? kt->stage : -1;  // the timed kernel stamps its device-clock span
  if ((e = launch_pipeline(b, d->g, d->prm, nframes, fmt, d->nblobwg, st, ev, d->st2, d->ev_fork, d->ev_join, kt)))
    return e;
  // results reach the host zero-copy: k_decode writes the detections into the
  // mapped host buffer and k_pose adds the poses and the control block; without
  // k_pose (tag_size == 0) the control block is copied here
  if (d->prm.tag_size > 0) return hipSuccess;
  return hipMemcpyAsync(d->h_ctrl, d->d_ctrl, d->ctrl_words * 4, hipMemcpyDeviceToHost, st);
}

// KernelTimer::split hook while capturing: close the current segment, open the next
static hipError_t split_capture(void* ctx, int /*which*/) {
  at_detector* d = (at_detector*)ctx;
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(d->st, &g);
  if (e != hipSuccess) return e;
  d->cap_segs.push_back(g);
  return hipStreamBeginCapture(d->st, hipStreamCaptureModeThreadLocal);
}

static hipError_t instantiate(hipGraph_t g, hipGraphExec_t* exec) {
  const hipError_t e = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  return e;
}

// Timed kernel under graph replay (bench roofline): segment before it, the kernel,
// segment after it, as three graphs with the timing events recorded between them.
// Not used when the timed kernel sits on the fork branch (its capture spans two
// streams and cannot be cut there): those launch directly.
static int enqueue_split(at_detector* d, int nframes, int fmt) {
  hipStream_t st = d->st;
  const int key = (nframes * 4 + fmt) * 32 + d->kt.stage;
  auto it = d->split_graphs.find(key);
  if (it == d->split_graphs.end()) {
    d->cap_segs.clear();
    KernelTimer kt = d->kt;
    kt.split = split_capture;
    kt.ctx = d;
    HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    hipError_t rec = record_sequence(d, nframes, fmt, st, nullptr, &kt);
    hipGraph_t last = nullptr;
    const hipError_t end = hipStreamEndCapture(st, &last);
    if (last) d->cap_segs.push_back(last);
    if (rec == hipSuccess && end == hipSuccess && d->cap_segs.size() != 3) rec = hipErrorInvalidValue;
    if (rec != hipSuccess || end != hipSuccess) {
      for (auto* g : d->cap_segs) (void)hipGraphDestroy(g);
      d->cap_segs.clear();
      HIPCHK(rec);
      HIPCHK(end);
    }
    at_detector::SplitGraphs sg{};
    hipError_t inst = hipSuccess;
    for (int i = 0; i < 3; i++) {
      const hipError_t r = instantiate(d->cap_segs[i], &sg.seg[i]);
      if (r != hipSuccess && inst == hipSuccess) inst = r;
    }
    d->cap_segs.clear();
    if (inst != hipSuccess) {
      for (auto* g : sg.seg)
        if (g) (void)hipGraphExecDestroy(g);
      HIPCHK(inst);
    }
    it = d->split_graphs.emplace(key, sg).first;
  }
  HIPCHK(hipGraphLaunch(it->second.seg[0], st));
  HIPCHK(hipEventRecord(d->kt.t0, st));
  HIPCHK(hipGraphLaunch(it->second.seg[1], st));
  HIPCHK(hipEventRecord(d->kt.t1, st));
  HIPCHK(hipGraphLaunch(it->second.seg[2], st));
  return AT_OK;
}

static int enqueue(at_detector* d, int nframes, int fmt) {
  hipStream_t st = d->st;
  const bool timed = d->kt.stage >= 0;
  const bool timed_on_fork = timed && d->st2 && (d->kt.stage == 8 || d->kt.stage == 9);
  if (d->profiling || !d->use_graphs || timed_on_fork) {
    HIPCHK(record_sequence(d, nframes, fmt, st, d->profiling ? d->ev_stage : nullptr, timed ? &d->kt : nullptr));
  } else if (timed) {
    const int rc = enqueue_split(d, nframes, fmt);
    if (rc != AT_OK) return rc;
  } else {
    const int key = nframes * 4 + fmt;
    auto it = d->graphs.find(key);
    if (it == d->graphs.end()) {
      hipGraph_t graph = nullptr;
      HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      const hipError_t rec = record_sequence(d, nframes, fmt, st, nullptr, nullptr);
      const hipError_t end = hipStreamEndCapture(st, &graph);
      HIPCHK(rec);
      HIPCHK(end);
      hipGraphExec_t exec = nullptr;
      HIPCHK(instantiate(graph, &exec));
      it = d->graphs.emplace(key, exec).first;
    }
    HIPCHK(hipGraphLaunch(it->second, st));
  }
  HIPCHK(hipEventRecord(d->ev_done, st));
  d->last_nframes = nframes;
  d->last_fmt = fmt;
  d->last_gray = fmt == AT_FMT_BGR8 || d->prm.taps;  // (YUYV / GRAY8: k_decode samples the frame)
  d->last_sizes = d->g.ctw == 32 || d->prm.taps;     // (throughput mode: the size plane for the taps only)
  d->last_gp = d->prm.gp_c && fmt == AT_FMT_BGR8;
  d->pending = 1;
  return AT_OK;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int collect(at_detector* d, at_detection* out, int cap_per_frame, int* n_per_frame) {
  if (!d->pending) return AT_E_INVALID;
  const double t0 = now_us();
  HIPCHK(hipEventSynchronize(d->ev_done));
  const double t1 = now_us();
  d->host_wait_us += t1 - t0;
  d->pending = 0;
  if (d->profiling) {
    for (int i = 0; i < kNumStages; i++) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, d->ev_stage[i], d->ev_stage[i + 1]));
      d->stage_ms[i] += ms;
    }
    d->stage_batches++;
  }
  if (d->kt.stage >= 0) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, d->kt.t0, d->kt.t1));
    d->kt_ms += ms;
    d->kt_n++;
    uint64_t st[2];
    memcpy(st, d->h_ctrl + d->kstamp_word, sizeof(st));
    st[0] = ~st[0];  // (k_kt_span keeps the complement of the first start: atomicMax on a zeroed word)
    if (st[1] > st[0] && st[0] && d->wclk_khz > 0) {  // (kernels without stamps leave zeros)
      d->kd_ms += (double)(st[1] - st[0]) / d->wclk_khz;
      d->kd_n++;
    }
  }
  const int B = d->B;
  int rc = AT_OK;
  // each frame's candidates: its slots 0 .. ndets[f] (the first kDetPoolPerFrame
  // already in the host mirror; a frame with more is copied from HBM)
  const int nf = d->last_nframes;
  int* cnt = d->res_n.data();
  // a failed copy leaves no stale counts: every frame reads empty until it is done
  for (int f = 0; f < nf; f++) {
    cnt[f] = 0;
    if (n_per_frame) n_per_frame[f] = 0;
  }
  for (int f = 0; f < nf; f++) {
    const uint32_t status = d->h_ctrl[kCtlStatus * B + f];
    const int ncand = (int)std::min<uint32_t>(d->h_ctrl[kCtlNdets * B + f], kMaxDets);
    int* idx = d->res_idx.data() + (size_t)f * kMaxDets;
    int n = 0;
    if (status & kStatusPairsCapped) rc = AT_E_CAPACITY;  // the first kMaxPairs pairs' detections are kept
    if (status & (kStatusPairsOverflow | kStatusHashFull | kStatusPointsOverflow | kStatusQuadsOverflow | kStatusDetsOverflow)) {
      rc = AT_E_CAPACITY;
    } else {
      const DevDetection* cand = d->h_dets + (size_t)f * kDetPoolPerFrame;
      if (ncand > kDetPoolPerFrame) {
        std::vector<DevDetection>& v = d->res_ovf[f];
        v.resize(ncand);
        // on the detector's own (non-blocking) stream: a copy on the null stream would
        // serialize with every blocking stream of the process (torch's default stream)
        HIPCHK(hipMemcpyAsync(v.data(), d->d.dets + (size_t)f * kMaxDets, ncand * sizeof(DevDetection),
                              hipMemcpyDeviceToHost, d->st));
        HIPCHK(hipStreamSynchronize(d->st));
        cand = v.data();
      }
      d->res_base[f] = cand;
      for (int i = 0; i < ncand; i++) idx[i] = i;
      n = host_tail(cand, idx, ncand, out ? out + (size_t)f * cap_per_frame : nullptr, out ? cap_per_frame : 0);
    }
    cnt[f] = n;
    if (n_per_frame) n_per_frame[f] = n;
  }
  d->host_tail_us += now_us() - t1;
  return rc;
}

static int check_fmt(int fmt) { return fmt == AT_FMT_YUYV || fmt == AT_FMT_BGR8 || fmt == AT_FMT_GRAY8; }
static size_t frame_bytes(const at_detector* d, int fmt) {
  const size_t npix = (size_t)d->g.W * d->g.H;
  return fmt == AT_FMT_YUYV ? 2 * npix : (fmt == AT_FMT_BGR8 ? 3 * npix : npix);
}

extern "C" {

int at_enqueue_host(at_detector* d, const uint8_t* const* frames, int nframes, at_pixfmt fmt) {
  if (!d || !frames || nframes < 1 || nframes > d->B || !check_fmt(fmt)) return AT_E_INVALID;
  for (int f = 0; f < nframes; f++)
    if (!frames[f]) return AT_E_INVALID;
  HIPCHK(hipSetDevice(d->device));
  if (d->pending) HIPCHK(hipEventSynchronize(d->ev_done));  // the frame table is read by the pending batch
  const size_t fb = frame_bytes(d, fmt);
  // frames back to back in host memory go over in one copy (their staging slots
  // are in_stride apart: one 2-D copy)
  for (int f = 0; f < nframes;) {
    int r = 1;
    while (f + r < nframes && frames[f + r] == frames[f] + (size_t)r * fb) r++;
    uint8_t* dst = d->d_in + (size_t)f * d->in_stride;
    if (r == 1)
      HIPCHK(hipMemcpyAsync(dst, frames[f], fb, hipMemcpyHostToDevice, d->st));
    else
      HIPCHK(hipMemcpy2DAsync(dst, d->in_stride, frames[f], fb, fb, (size_t)r, hipMemcpyHostToDevice, d->st));
    for (int k = 0; k < r; k++) d->h_ftab[f + k] = d->d_in + (size_t)(f + k) * d->in_stride;
    f += r;
  }
  const int rc = enqueue(d, nframes, fmt);
  if (rc) return rc;
  d->last_staged = 1;
  return AT_OK;
}

int at_detect_batch(at_detector* d, const uint8_t* const* frames, int nframes, at_pixfmt fmt, at_detection* out,
                    int cap_per_frame, int* n_per_frame) {
  const int rc = at_enqueue_host(d, frames, nframes, fmt);
  if (rc) return rc;
  return collect(d, out, cap_per_frame, n_per_frame);
}

int at_detect(at_detector* d, const uint8_t* frame, at_pixfmt fmt, at_detection* out, int cap, int* n) {
  const uint8_t* frames[1] = {frame};
  int nn = 0;
  const int rc = at_detect_batch(d, frames, 1, fmt, out, cap, &nn);
  if (n) *n = nn;
  return rc;
}

int at_enqueue_device(at_detector* d, const void* d_frames, size_t frame_stride, int nframes, at_pixfmt fmt) {
  if (!d || !d_frames || nframes < 1 || nframes > d->B || !check_fmt(fmt)) return AT_E_INVALID;
  if (fmt == AT_FMT_YUYV && frame_stride % 16) return AT_E_INVALID;
  if (frame_stride % 8) return AT_E_INVALID;
  HIPCHK(hipSetDevice(d->device));
  if (d->pending) HIPCHK(hipEventSynchronize(d->ev_done));  // pinned buffers are reused
  for (int f = 0; f < nframes; f++) d->h_ftab[f] = (const uint8_t*)d_frames + (size_t)f * frame_stride;
  const int rc = enqueue(d, nframes, fmt);
  d->last_staged = 0;
  return rc;
}

int at_stream_wait(at_detector* d, void* stream) {
  if (!d) return AT_E_INVALID;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipEventRecord(d->ev_ext, (hipStream_t)stream));
  HIPCHK(hipStreamWaitEvent(d->st, d->ev_ext, 0));
  return AT_OK;
}

int at_collect(at_detector* d, at_detection* out, int cap_per_frame, int* n_per_frame) {
  if (!d) return AT_E_INVALID;
  HIPCHK(hipSetDevice(d->device));
  return collect(d, out, cap_per_frame, n_per_frame);
}

int at_detect_device(at_detector* d, const void* d_frames, size_t frame_stride, int nframes, at_pixfmt fmt,
                     at_detection* out, int cap_per_frame, int* n_per_frame) {
  int rc = at_enqueue_device(d, d_frames, frame_stride, nframes, fmt);
  if (rc) return rc;
  return at_collect(d, out, cap_per_frame, n_per_frame);
}

int at_set_profiling(at_detector* d, int enable) {
  if (!d) return AT_E_INVALID;
  HIPCHK(hipSetDevice(d->device));
  if (d->pending) HIPCHK(hipEventSynchronize(d->ev_done));
  if (enable && !d->ev_stage[0])
    for (int i = 0; i <= kNumStages; i++) HIPCHK(hipEventCreateWithFlags(&d->ev_stage[i], kTimingEventFlags));
  d->profiling = enable ? 1 : 0;
  for (int i = 0; i < kNumStages; i++) d->stage_ms[i] = 0;
  d->stage_batches = 0;
  return AT_OK;
}

int at_stage_times(at_detector* d, double* ms, int cap) {
  if (!d || !ms || cap < kNumStages + 1) return AT_E_INVALID;
  for (int i = 0; i < kNumStages; i++) ms[i] = d->stage_batches ? d->stage_ms[i] / d->stage_batches : 0.0;
  ms[kNumStages] = (double)d->stage_batches;
  return kNumStages;
}

const char* at_stage_name(int stage) {
  return (stage >= 0 && stage < kNumStages) ? kStageNames[stage] : "";
}

int at_set_kernel_timer(at_detector* d, int stage) {
  if (!d || stage < -1 || stage >= kNumStages) return AT_E_INVALID;
  HIPCHK(hipSetDevice(d->device));
  if (d->pending) HIPCHK(hipEventSynchronize(d->ev_done));
  d->kt.stage = stage;
  d->kt_ms = 0;
  d->kt_n = 0;
  d->kd_ms = 0;
  d->kd_n = 0;
  return AT_OK;
}

int at_kernel_time(at_detector* d, double* avg_ms, long long* launches) {
  if (!d || !avg_ms) return AT_E_INVALID;
  *avg_ms = d->kt_n ? d->kt_ms / (double)d->kt_n : 0.0;
  if (launches) *launches = d->kt_n;
  return AT_OK;
}

int at_kernel_span(at_detector* d, double* avg_ms, long long* launches) {
  if (!d || !avg_ms) return AT_E_INVALID;
  *avg_ms = d->kd_n ? d->kd_ms / (double)d->kd_n : 0.0;
  if (launches) *launches = d->kd_n;
  return AT_OK;
}

int at_batch_stats(at_detector* d, uint64_t* out, int cap) {
  if (!d || !out || cap < 1) return AT_E_INVALID;
  if (d->pending) return AT_E_INVALID;
  const int B = d->B;
  uint64_t v[12] = {0};
  v[0] = (uint64_t)d->last_nframes;
  for (int f = 0; f < d->last_nframes; f++) {
    v[1] += d->h_ctrl[kCtlNpts * B + f];
    v[2] += d->h_ctrl[kCtlNpairs * B + f];
    v[6] += d->h_ctrl[kCtlNdets * B + f];
    v[9] += d->h_ctrl[kCtlNlr * B + f];
    v[10] = std::max<uint64_t>(v[10], d->h_ctrl[kCtlNlr * B + f]);
    v[11] += d->h_ctrl[kCtlCclOvf * B + f] != 0;
  }
  v[5] = d->h_ctrl[kCtlNquads * B];  // FitQuads records of the batch (counted per blob team)
  v[3] = d->h_ctrl[kCtlPerFrame * B + kCtlBlobPts];
  v[4] = d->h_ctrl[kCtlPerFrame * B + kCtlBlobPts + 1];
  v[7] = (uint64_t)d->host_wait_us;
  v[8] = (uint64_t)d->host_tail_us;
  const int n = std::min(cap, 12);
  for (int i = 0; i < n; i++) out[i] = v[i];
  return n;
}

int at_poses(at_detector* d, int frame, at_pose* out, int cap) {
  if (!d || frame < 0 || frame >= d->last_nframes || (cap > 0 && !out)) return AT_E_INVALID;
  if (d->pending) return AT_E_INVALID;  // collect first
  if (!(d->prm.tag_size > 0)) return 0;
  const int n = d->res_n[frame];
  for (int i = 0; i < n && i < cap; i++) {
    const DevDetection& v = d->res_base[frame][d->res_idx[(size_t)frame * kMaxDets + i]];
    at_pose& p = out[i];
    p.id = v.id;
    memcpy(p.R, v.pose_R, sizeof(p.R));
    memcpy(p.t, v.pose_t, sizeof(p.t));
    p.err = v.pose_err[0] <= v.pose_err[1] ? v.pose_err[0] : v.pose_err[1];  // estimate_tag_pose
  }
  return n;
}

int at_detections(at_detector* d, int frame, at_detection* out, int cap) {
  if (!d || frame < 0 || frame >= d->last_nframes || (cap > 0 && !out)) return AT_E_INVALID;
  if (d->pending) return AT_E_INVALID;
  const int n = d->res_n[frame];
  for (int i = 0; i < n && i < cap; i++)
    write_detection(d->res_base[frame][d->res_idx[(size_t)frame * kMaxDets + i]], out + i);
  return n;
}

int at_max_detections(void) { return kMaxDets; }

int at_tag_detections(const at_pose* poses, int n, const double* extr_R, const double* extr_t,
                      at_tag_detection* out) {
  if (n < 0 || (n > 0 && (!poses || !out))) return AT_E_INVALID;
  static const double kEye[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, kZero[3] = {0, 0, 0};
  const double* Re = extr_R ? extr_R : kEye;
  const double* te = extr_t ? extr_t : kZero;
  std::vector<at_tag_detection> v((size_t)n);
  for (int i = 0; i < n; i++) {
    at_tag_detection& o = v[i];
    o.id = poses[i].id;
    for (int k = 0; k < 3; k++) o.camera[k] = poses[i].t[k];
    for (int r = 0; r < 3; r++)  // extrinsic_rotation_ * camera_point_mat + extrinsic_offset_
      o.robot[r] = Re[r * 3 + 0] * o.camera[0] + Re[r * 3 + 1] * o.camera[1] + Re[r * 3 + 2] * o.camera[2] + te[r];
    o.distance = std::sqrt(o.camera[0] * o.camera[0] + o.camera[1] * o.camera[1] + o.camera[2] * o.camera[2]);
    o.err = poses[i].err;
  }
  std::stable_sort(v.begin(), v.end(),
                   [](const at_tag_detection& a, const at_tag_detection& b) { return a.distance < b.distance; });
  for (int i = 0; i < n; i++) out[i] = v[i];
  return n;
}

// ---- annotated image ------------------------------------
// The segments of node/at_node.cpp's draw_detection_outlines, in its drawing order:
// per detection the four sides (apriltag_utils.cu:58-65: corners truncated to int
// as cv::Point does; 0-1 green, 0-3 red, 1-2 and 2-3 blue), then the id's digit
// strokes centred on c (:67-77).  The digit strokes are the node's.
static void outline_prims(const at_detection* dets, int n, std::vector<DrawPrim>* out) {
  static const uint8_t kGreen[3] = {0, 0xff, 0}, kRed[3] = {0, 0, 0xff}, kBlue[3] = {0xff, 0, 0},
                       kText[3] = {0xff, 0x99, 0};
  static const std::vector<std::vector<std::pair<int, int>>> kDigits[10] = {
      {{{0, 1}, {1, 0}, {3, 0}, {4, 1}, {4, 7}, {3, 8}, {1, 8}, {0, 7}, {0, 1}}},
      {{{1, 2}, {2, 0}, {2, 8}}, {{1, 8}, {3, 8}}},
      {{{0, 1}, {1, 0}, {3, 0}, {4, 1}, {4, 3}, {0, 8}, {4, 8}}},
      {{{0, 0}, {4, 0}, {2, 3}, {3, 3}, {4, 4}, {4, 7}, {3, 8}, {1, 8}, {0, 7}}},
      {{{3, 8}, {3, 0}, {0, 5}, {4, 5}}},
      {{{4, 0}, {0, 0}, {0, 3}, {3, 3}, {4, 4}, {4, 7}, {3, 8}, {0, 8}}},
      {{{4, 0}, {2, 0}, {0, 3}, {0, 7}, {1, 8}, {3, 8}, {4, 7}, {4, 5}, {3, 4}, {0, 4}}},
      {{{0, 0}, {4, 0}, {1, 8}}},
      {{{1, 4}, {0, 3}, {0, 1}, {1, 0}, {3, 0}, {4, 1}, {4, 3}, {3, 4}, {1, 4}, {0, 5}, {0, 7}, {1, 8},
        {3, 8}, {4, 7}, {4, 5}, {3, 4}}},
      {{{4, 4}, {1, 4}, {0, 3}, {0, 1}, {1, 0}, {3, 0}, {4, 1}, {4, 5}, {2, 8}, {0, 8}}},
  };
  auto seg = [&](double x0, double y0, double x1, double y1, const uint8_t c[3]) {
    DrawPrim q;
    q.x0 = x0; q.y0 = y0; q.x1 = x1; q.y1 = y1;
    q.bgr[0] = c[0]; q.bgr[1] = c[1]; q.bgr[2] = c[2];
    out->push_back(q);
  };
  for (int i = 0; i < n; i++) {
    const at_detection& d = dets[i];
    auto P = [&](int k, int c) { return (double)(int)d.p[k][c]; };
    seg(P(0, 0), P(0, 1), P(1, 0), P(1, 1), kGreen);
    seg(P(0, 0), P(0, 1), P(3, 0), P(3, 1), kRed);
    seg(P(1, 0), P(1, 1), P(2, 0), P(2, 1), kBlue);
    seg(P(2, 0), P(2, 1), P(3, 0), P(3, 1), kBlue);
    const std::string text = std::to_string(d.id);
    const double sc = 2.5, adv = 7 * sc;
    const double tw = adv * text.size() - 2 * sc, th = 8 * sc;
    const double ox = (int)(d.c[0] - tw / 2), oy = (int)(d.c[1] - th / 2);
    for (size_t k = 0; k < text.size(); ++k) {
      if (text[k] < '0' || text[k] > '9') continue;
      for (const auto& stroke : kDigits[text[k] - '0'])
        for (size_t t = 1; t < stroke.size(); ++t)
          seg(ox + k * adv + stroke[t - 1].first * sc, oy + stroke[t - 1].second * sc, ox + k * adv + stroke[t].first * sc,
              oy + stroke[t].second * sc, kText);
    }
  }
}

// the outline segments drawn onto `bgr` on the detector's stream (not waited for)
static int draw_outlines(at_detector* d, const at_detection* dets, int n, uint8_t* bgr) {
  if (!d || n < 0 || (n > 0 && !dets) || !bgr) return AT_E_INVALID;
  HIPCHK(hipSetDevice(d->device));
  std::vector<DrawPrim> prims;
  outline_prims(dets, n, &prims);
  if (prims.empty()) return AT_OK;
  const size_t W = (size_t)d->g.W, H = (size_t)d->g.H;
  if (!d->d_last) {
    HIPCHK(hipMalloc((void**)&d->d_last, W * H * 4));
    HIPCHK(hipMemset(d->d_last, 0, W * H * 4));  // kept zero by the paint pass
  }
  if (prims.size() > d->prims_cap) {
    if (d->d_prims) HIPCHK(hipFree(d->d_prims));
    d->d_prims = nullptr;
    d->prims_cap = 0;
    const size_t cap = std::max<size_t>(1024, prims.size() * 2);
    HIPCHK(hipMalloc((void**)&d->d_prims, cap * sizeof(DrawPrim)));
    d->prims_cap = cap;
  }
  HIPCHK(hipMemcpyAsync(d->d_prims, prims.data(), prims.size() * sizeof(DrawPrim), hipMemcpyHostToDevice, d->st));
  HIPCHK(launch_draw(d->d_prims, (int)prims.size(), d->d_last, bgr, (int)W, (int)H, d->st));
  return AT_OK;
}

int at_draw_outlines_device(at_detector* d, const at_detection* dets, int n, uint8_t* bgr) {
  const int rc = draw_outlines(d, dets, n, bgr);
  if (rc != AT_OK) return rc;
  HIPCHK(hipStreamSynchronize(d->st));
  return AT_OK;
}

int at_annotate_staged(at_detector* d, int frame, const at_detection* dets, int n, uint8_t* bgr_out) {
  if (!d || !bgr_out || n < 0 || (n > 0 && !dets)) return AT_E_INVALID;
  if (!d->last_staged || d->last_fmt != AT_FMT_BGR8 || frame < 0 || frame >= d->last_nframes) return AT_E_INVALID;
  HIPCHK(hipSetDevice(d->device));
  if (d->pending) HIPCHK(hipEventSynchronize(d->ev_done));
  uint8_t* img = d->d_in + (size_t)frame * d->in_stride;
  const int rc = draw_outlines(d, dets, n, img);
  if (rc != AT_OK) return rc;
  // in stream order after the drawing, on the detector's stream (no null-stream copy);
  // DMA straight into a page-locked bgr_out (at_host_alloc)
  HIPCHK(hipMemcpyAsync(bgr_out, img, (size_t)d->g.W * d->g.H * 3, hipMemcpyDeviceToHost, d->st));
  HIPCHK(hipStreamSynchronize(d->st));
  return AT_OK;
}

int at_host_alloc(size_t bytes, void** out) {
  if (!out) return AT_E_INVALID;
  *out = nullptr;
  if (hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) {
    *out = nullptr;
    return AT_E_NOMEM;
  }
  return AT_OK;
}

void at_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

// ---- shared game-piece preprocessing ---------------------
static void drop_graphs(at_detector* d) {
  for (auto& kv : d->graphs) (void)hipGraphExecDestroy(kv.second);
  d->graphs.clear();
  for (auto& kv : d->split_graphs)
    for (auto* g : kv.second.seg) (void)hipGraphExecDestroy(g);
  d->split_graphs.clear();
}

int at_gp_enable(at_detector* d, int out_width, int out_height, int channels) {
  if (!d || out_width < 1 || out_height < 1 || out_width > 8192 || out_height > 8192 ||
      (channels != 1 && channels != 3))
    return AT_E_INVALID;
  if (hipSetDevice(d->device) != hipSuccess) return AT_E_HIP;
  if (d->pending && hipEventSynchronize(d->ev_done) != hipSuccess) return AT_E_HIP;
  const size_t bytes = (size_t)d->B * channels * out_width * out_height * sizeof(float);
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return AT_E_NOMEM;
  if (d->d.gp_out) {
    for (auto& a : d->allocs)
      if (a == d->d.gp_out) a = nullptr;
    (void)hipFree(d->d.gp_out);
  }
  d->allocs.push_back(p);
  d->d.gp_out = (float*)p;
  d->prm.gp_w = out_width;
  d->prm.gp_h = out_height;
  d->prm.gp_c = channels;
  d->last_gp = 0;  // no tensor until a BGR8 batch has produced one
  drop_graphs(d);  // the captured sequences carry the old parameters
  return AT_OK;
}

int at_gp_tensor(at_detector* d, int frame, const float** dev_ptr) {
  if (!d || !dev_ptr || !d->prm.gp_c || !d->last_gp || frame < 0 || frame >= d->last_nframes) return AT_E_INVALID;
  *dev_ptr = d->d.gp_out + (size_t)frame * d->prm.gp_c * d->prm.gp_w * d->prm.gp_h;
  return AT_OK;
}

int at_gp_copy(at_detector* d, int frame, float* dst, size_t count) {
  const float* src = nullptr;
  const int rc = at_gp_tensor(d, frame, &src);
  if (rc != AT_OK) return rc;
  const size_t n = (size_t)d->prm.gp_c * d->prm.gp_w * d->prm.gp_h;
  if (!dst || count < n) return AT_E_INVALID;
  if (hipSetDevice(d->device) != hipSuccess) return AT_E_HIP;
  if (d->pending && hipEventSynchronize(d->ev_done) != hipSuccess) return AT_E_HIP;
  return hipMemcpy(dst, src, n * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess ? AT_OK : AT_E_HIP;
}

int at_gp_preprocess_device(const uint8_t* bgr, int width, int height, float* out, int out_width, int out_height,
                            int channels, void* stream) {
  if (!bgr || !out || width < 2 || height < 2 || out_width < 1 || out_height < 1 || out_width > 8192 ||
      out_height > 8192 || (channels != 1 && channels != 3))
    return AT_E_INVALID;
  return launch_gp_preprocess(bgr, width, height, out, out_width, out_height, channels, (hipStream_t)stream) ==
                 hipSuccess
             ? AT_OK
             : AT_E_HIP;
}

int at_set_debug_taps(at_detector* d, int enable) {
  if (!d) return AT_E_INVALID;
  if (hipSetDevice(d->device) != hipSuccess) return AT_E_HIP;
  if (d->pending && hipEventSynchronize(d->ev_done) != hipSuccess) return AT_E_HIP;
  if (d->prm.taps != (enable ? 1 : 0)) {
    d->prm.taps = enable ? 1 : 0;
    drop_graphs(d);  // the captured sequences carry the old parameters
  }
  return AT_OK;
}

int at_frame_status(at_detector* d, int frame) {
  if (!d || frame < 0 || frame >= d->last_nframes) return AT_E_INVALID;
  const uint32_t s = d->h_ctrl[kCtlStatus * d->B + frame];
  return (s & (kStatusPairsOverflow | kStatusHashFull | kStatusPointsOverflow | kStatusQuadsOverflow | kStatusDetsOverflow |
               kStatusPairsCapped))
             ? AT_E_CAPACITY
             : AT_OK;
}

long long at_debug_copy(at_detector* d, int stage, int frame, void* dst, size_t bytes) {
  if (!d || !dst || frame < 0 || frame >= d->last_nframes) return AT_E_INVALID;
  if (hipSetDevice(d->device) != hipSuccess) return AT_E_HIP;
  if (d->pending && hipEventSynchronize(d->ev_done) != hipSuccess) return AT_E_HIP;
  const Geom& g = d->g;
  const size_t npix = (size_t)g.W * g.H, nd = (size_t)g.Wd * g.Hd;
  const void* src = nullptr;
  size_t n = 0;
  const int B = d->B;
  std::vector<uint8_t> tmp;
  switch (stage) {
    case AT_STAGE_GRAY:
      if (!d->last_gray) return AT_E_INVALID;  // YUYV / GRAY8 batches without the debug taps
      src = d->d.gray + frame * npix; n = npix; break;
    case AT_STAGE_DECIMATED: src = d->d.dec + frame * nd; n = nd; break;
    case AT_STAGE_THRESHOLD: src = d->d.thr + frame * nd; n = nd; break;
    case AT_STAGE_LABELS: {
      // LabelImage's output (labeling_allegretti_2019_BKE.cu:340-462), resolved from
      // the union-find forest on the device (k_tap_labels)
      if (bytes < nd * 4) return AT_E_INVALID;
      uint32_t* tmp_d = nullptr;
      if (hipMalloc(&tmp_d, nd * 4) != hipSuccess) return AT_E_NOMEM;
      hipError_t e = launch_tap_labels(d->d.thr + frame * nd, d->d.par + frame * nd, tmp_d, g.Wd, g.Hd, d->st);
      if (e == hipSuccess) e = hipStreamSynchronize(d->st);
      if (e == hipSuccess) e = hipMemcpy(dst, tmp_d, nd * 4, hipMemcpyDeviceToHost);
      (void)hipFree(tmp_d);
      return e == hipSuccess ? (long long)(nd * 4) : AT_E_HIP;
    }
    case AT_STAGE_SIZES: {
      // the dense plane of the reference, masked from the forest on the device
      if (bytes < nd * 4 || !d->last_sizes) return AT_E_INVALID;
      uint32_t* tmp_d = nullptr;
      if (hipMalloc(&tmp_d, nd * 4) != hipSuccess) return AT_E_NOMEM;
      hipError_t e = launch_tap_sizes(d->d.thr + frame * nd, d->d.par + frame * nd, d->d.size + frame * nd, tmp_d,
                                      g.Wd, g.Hd, d->st);
      if (e == hipSuccess) e = hipStreamSynchronize(d->st);
      if (e == hipSuccess) e = hipMemcpy(dst, tmp_d, nd * 4, hipMemcpyDeviceToHost);
      (void)hipFree(tmp_d);
      return e == hipSuccess ? (long long)(nd * 4) : AT_E_HIP;
    }
    case AT_STAGE_NUM_POINTS:
      if (bytes < 4) return AT_E_INVALID;
      memcpy(dst, &d->h_ctrl[kCtlNpts * B + frame], 4);
      return 4;
    case AT_STAGE_NUM_PAIRS:
      if (bytes < 4) return AT_E_INVALID;
      memcpy(dst, &d->h_ctrl[kCtlNpairs * B + frame], 4);
      return 4;
    case AT_STAGE_NUM_PAIR_ENTRIES:
      if (bytes < 4) return AT_E_INVALID;
      memcpy(dst, &d->h_ctrl[kCtlNpent * B + frame], 4);
      return 4;
    case AT_STAGE_PROBE: src = d->d.probe; n = kProbeWords * 8; break;
    case AT_STAGE_QUADS: {
      // one record per kept blob, in the slot of its pair rank (pair_sel marks them),
      // written while the debug taps are on
      if (!d->prm.taps) return AT_E_INVALID;
      const uint32_t npairs = std::min<uint32_t>(d->h_ctrl[kCtlNpairs * B + frame], (uint32_t)kMaxPairs);
      std::vector<QuadRecord> all(npairs);
      std::vector<uint32_t> sel(npairs);
      if (npairs && (hipMemcpy(all.data(), d->d.quads + (size_t)frame * kMaxPairs, npairs * sizeof(QuadRecord),
                               hipMemcpyDeviceToHost) != hipSuccess ||
                     hipMemcpy(sel.data(), d->d.pair_sel + (size_t)frame * kMaxPairs, npairs * 4,
                               hipMemcpyDeviceToHost) != hipSuccess))
        return AT_E_HIP;
      std::vector<QuadRecord> q;
      for (uint32_t i = 0; i < npairs; i++)
        if (sel[i]) q.push_back(all[i]);
      const uint32_t nq = (uint32_t)q.size();
      const size_t need = nq * sizeof(at_quad_record);
      if (bytes < need) return AT_E_INVALID;
      for (uint32_t i = 0; i < nq; i++) {
        at_quad_record r;
        r.blob_index = q[i].blob_index;
        r.valid = q[i].valid;
        r.accepted = q[i].accepted;
        memcpy(r.indices, q[i].indices, sizeof(r.indices));
        memcpy(r.corners, q[i].corners, sizeof(r.corners));
        memcpy((uint8_t*)dst + i * sizeof(at_quad_record), &r, sizeof(r));
      }
      return (long long)need;
    }
    case AT_STAGE_POINTS: {
      // the tiles' regions concatenated in tile order
      const size_t ntb = (size_t)g.ntb;
      std::vector<uint32_t> tc(ntb);
      std::vector<uint64_t> all(ntb * (size_t)g.bnd_region);
      if (hipMemcpy(tc.data(), d->d.tcnt + frame * ntb, ntb * 4, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(all.data(), d->d.pts + frame * ntb * g.bnd_region, all.size() * 8, hipMemcpyDeviceToHost) !=
              hipSuccess)
        return AT_E_HIP;
      size_t np = 0;
      for (size_t t = 0; t < ntb; t++) np += tc[t] & ~kTileNarrow;
      if (bytes < np * 8) return AT_E_INVALID;
      // narrow tiles hold (entry index, point bits) words: the key is the entry's pair
      // key over the point bits
      std::vector<uint64_t> ekey(ntb * (size_t)kLdsPairSlots);
      if (hipMemcpy(ekey.data(), d->d.pent_key + frame * ntb * kLdsPairSlots, ekey.size() * 8,
                    hipMemcpyDeviceToHost) != hipSuccess)
        return AT_E_HIP;
      // the device keys pairs by node index (node_F / node_L: three words per 2x2 block,
      // monotone in the node id); the reference's QuadBoundaryPoint carries the node ids
      auto node_id = [&](uint64_t n) -> uint64_t {
        const uint64_t P = 3 * (uint64_t)g.BW, by = n / P, r = n - by * P;
        return r < (uint64_t)g.BW ? 2 * by * g.Wd + 2 * r : (2 * by + 1) * g.Wd + (r - g.BW);
      };
      auto to_ref = [&](uint64_t k) -> uint64_t {
        return (node_id(k >> 44) << 44) | (node_id((k >> 24) & 0xfffff) << 24) | (k & 0xffffffu);
      };
      size_t o = 0;
      for (size_t t = 0; t < ntb; t++) {
        const uint32_t n = tc[t] & ~kTileNarrow;
        if (tc[t] & kTileNarrow) {
          const uint32_t* w = reinterpret_cast<const uint32_t*>(all.data() + t * g.bnd_region);
          for (uint32_t i = 0; i < n; i++) {
            const uint64_t key =
                to_ref((ekey[t * kLdsPairSlots + (w[i] >> 23)] << 24) | ((w[i] & 0x7ffffcu) << 1) | (w[i] & 3u));
            memcpy((uint8_t*)dst + (o + i) * 8, &key, 8);
          }
        } else {
          for (uint32_t i = 0; i < n; i++) {
            const uint64_t key = to_ref(all[t * g.bnd_region + i]);
            memcpy((uint8_t*)dst + (o + i) * 8, &key, 8);
          }
        }
        o += n;
      }
      return (long long)(np * 8);
    }
    case AT_STAGE_BLOB_POINTS: {
      // IndexPoint keys of the selected pairs, in rank order (written by the blob
      // kernels only while the debug taps are on)
      if (!d->prm.taps) return AT_E_INVALID;
      const uint32_t npairs = std::min<uint32_t>(d->h_ctrl[kCtlNpairs * B + frame], (uint32_t)kMaxPairs);
      std::vector<uint32_t> cnt(npairs), off(npairs), sel(npairs);
      if (npairs) {
        if (hipMemcpy(cnt.data(), d->d.pair_cnt + (size_t)frame * kMaxPairs, npairs * 4, hipMemcpyDeviceToHost) ||
            hipMemcpy(off.data(), d->d.pair_off + (size_t)frame * kMaxPairs, npairs * 4, hipMemcpyDeviceToHost) ||
            hipMemcpy(sel.data(), d->d.pair_sel + (size_t)frame * kMaxPairs, npairs * 4, hipMemcpyDeviceToHost))
          return AT_E_HIP;
      }
      size_t total = 0;
      for (uint32_t i = 0; i < npairs; i++)
        if (sel[i]) total += cnt[i];
      if (bytes < total * 8) return (long long)(total * 8);
      size_t o = 0;
      for (uint32_t i = 0; i < npairs; i++) {
        if (!sel[i]) continue;
        if (hipMemcpy((uint8_t*)dst + o * 8, d->d.keys + (size_t)frame * g.cap_pts + off[i], cnt[i] * 8,
                      hipMemcpyDeviceToHost) != hipSuccess)
          return AT_E_HIP;
        o += cnt[i];
      }
      return (long long)(total * 8);
    }
    default: return AT_E_INVALID;
  }
  if (bytes < n) return AT_E_INVALID;
  if (n && hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) != hipSuccess) return AT_E_HIP;
  return (long long)n;
}

}  // extern "C"
