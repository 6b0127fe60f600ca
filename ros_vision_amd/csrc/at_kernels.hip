// at_kernels.hip -- gfx950 kernels of the AprilTag detection stage.
//
// Pipeline for a batch of B frames, all on one HIP stream, no host round trip
// until the detections are copied back:
//   k_pre          YUYV/BGR/GRAY -> gray, decimated, 4x4 tile min/max   (threshold.cu:16-80)
//   k_thr_ccl      tile filter + threshold + LDS union-find per 32x32 tile (threshold.cu:84-147,
//                  labeling_allegretti_2019_BKE.cu:114-338)
//   k_ccl_border   unions across tile borders (global atomicMin)
//   k_ccl_final    root labels + blob sizes                              (:340-462)
//   k_boundary     boundary points + pair histogram, wave-compacted      (apriltag_gpu.cu:226-360,
//                                                                         P1, P3 counts)
//   k_pairs        rank pairs (rep1-major order), offsets, work list     (P2, P3, P4)
//   k_group        scatter points into per-pair segments
//   k_blob         per blob: extents, filter, theta sort, line fit, peaks, quad fit,
//                  corners, refine edges, homography, decode             (P4-P10, K10, K11,
//                                                                         apriltag_detect.cu)
// All float arithmetic is compiled with -ffp-contract=off and uses at_detmath.h
// for transcendental functions so that results are bit-identical to the CPU
// oracle (oracle/ao_oracle.c).
#include <limits>
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <stdint.h>

#include "at_common.h"
#include "at_pose.h"


namespace at {

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
// det_atan2f as a call: k_decode's refine evaluates it four times per quad, and its
// polynomial constants inlined there cost spills (VGPR spills 16 -> 27)
__device__ __attribute__((noinline)) float det_atan2f_call(float y, float x) { return det_atan2f(y, x); }

__device__ __forceinline__ uint64_t mix_hash(uint64_t k) {
  return (k * 0x9E3779B97F4A7C15ull) >> (64 - kHashBits);
}

// QuadBoundaryPoint direction decode (points.h:83-108): dxy 0:(1,0) 1:(1,1) 2:(0,1) 3:(-1,1)
__device__ __forceinline__ int dx_of(int dxy) { return dxy == 3 ? -1 : (dxy == 2 ? 0 : 1); }
__device__ __forceinline__ int dy_of(int dxy) { return dxy == 0 ? 0 : 1; }

// ---- wave64 primitives on DPP (GFX9 row_shr / row_bcast): one VALU move per
// dword and step instead of an LDS ds_bpermute / ds_swizzle round trip --------
template <int CTRL, int ROW_MASK, typename T>
__device__ __forceinline__ T dpp_move(T v, T old) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "dpp_move: 32- or 64-bit values");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                             CTRL, ROW_MASK, 0xf, false));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v), o = __builtin_bit_cast(uint64_t, old);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)o, (int)(uint32_t)u, CTRL, ROW_MASK, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(o >> 32), (int)(uint32_t)(u >> 32), CTRL,
                                                              ROW_MASK, 0xf, false);
    return __builtin_bit_cast(T, (uint64_t)lo | ((uint64_t)hi << 32));
  }
}

// inclusive wave scan: lanes whose DPP source is out of range combine `id`
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T x, Op op, T id) {
  x = op(x, dpp_move<0x111, 0xf>(x, id));  // row_shr:1
  x = op(x, dpp_move<0x112, 0xf>(x, id));  // row_shr:2
  x = op(x, dpp_move<0x114, 0xf>(x, id));  // row_shr:4
  x = op(x, dpp_move<0x118, 0xf>(x, id));  // row_shr:8
  x = op(x, dpp_move<0x142, 0xa>(x, id));  // row_bcast:15 -> rows 1, 3
  x = op(x, dpp_move<0x143, 0xc>(x, id));  // row_bcast:31 -> rows 2, 3
  return x;
}

// Value of lane l-1 in lane l (lane 0: `fill`): one DPP wave_shr:1 move per
// dword instead of a ds_bpermute round trip through LDS.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t fill) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xf, 0xf, false);
}

// Number of set bits of `mask` below this lane.
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// a wave's LDS stores visible to its other lanes (a wave-level barrier, no s_barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// value of lane + 1 (lane 63: 0): DPP wave_shl:1
__device__ __forceinline__ uint32_t wave_read_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}

// value of lane `l` in every lane (scalar read)
template <typename T>
__device__ __forceinline__ T wave_read(T v, int l) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(T, (uint64_t)lo | ((uint64_t)hi << 32));
  }
}

struct MinOp {
  template <typename T> __device__ T operator()(T a, T c) const { return a < c ? a : c; }
  template <typename T> __device__ static T identity() { return std::numeric_limits<T>::max(); }
};
struct MaxOp {
  template <typename T> __device__ T operator()(T a, T c) const { return a > c ? a : c; }
  template <typename T> __device__ static T identity() { return std::numeric_limits<T>::lowest(); }
};
struct AddOp {
  template <typename T> __device__ T operator()(T a, T c) const { return a + c; }
  template <typename T> __device__ static T identity() { return T(0); }
};

// Length of the run of equal keys starting at this lane (only meaningful for
// run heads); same_mask bit l means "lane l continues the run of lane l-1".
__device__ __forceinline__ uint32_t run_len(uint64_t same_mask, uint32_t lane) {
  if (lane == 63) return 1;
  const uint64_t rest = ~(same_mask >> (lane + 1));
  return 1 + (uint32_t)__builtin_ctzll(rest);
}

// ---- block reductions (256 threads = 4 waves) ------------------------------
template <typename T, typename Op>
__device__ T wave_reduce(T v, Op op) {
  return wave_read(wave_incl_scan(v, op, Op::template identity<T>()), 63);
}

template <typename T, typename Op>
__device__ T block_reduce(T v, Op op, T* s_tmp /* >= NW */, int NW) {
  v = wave_reduce(v, op);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (lane_id() == 0) s_tmp[w] = v;
  __syncthreads();
  T r = s_tmp[0];
  for (int i = 1; i < NW; i++) r = op(r, s_tmp[i]);
  return r;
}

// inclusive block scan of one value per thread (NW waves); returns the
// inclusive prefix, *total = block sum
template <typename T>
__device__ T block_incl_scan(T v, T* s_tmp, T* total, int NW) {
  const uint32_t lane = lane_id();
  v = wave_incl_scan(v, AddOp(), T(0));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 63) s_tmp[w] = v;
  __syncthreads();
  T base = 0, tot = 0;
  for (int i = 0; i < NW; i++) {
    if (i < w) base = base + s_tmp[i];
    tot = tot + s_tmp[i];
  }
  *total = tot;
  return base + v;
}


// Device-clock span of one launch of the timed kernel (DevBufs::kt_stage): every
// workgroup stores its start and, once its work is over, its end on the GPU wall
// clock (plain stores into its own slots: no shared counter to contend on);
// k_kt_span, launched after the timed kernel, reduces them to the first start
// and the last end -- the kernel's execution span, as rocprofv3's kernel trace
// times it, measured live without a profiler.  Nothing is stored unless this
// launch is the timed one.
// XCD-aware tile order.  Workgroups are dealt round-robin over the chip's 8 XCDs
// (MI355X_MICROARCH.md, Workgroup dispatch: blocks b and b + 8 share one), each with
// its own L2.  In blockIdx order, horizontally adjacent tiles -- which share the
// 64-B sectors of their halo columns and, for 64-pixel-wide decimated tiles, the
// 128-B lines of every row -- land on different XCDs and each fetches the shared
// sectors from the fabric.  xcd_block() renumbers the grid so that XCD k (the blocks
// b = k mod 8, in dispatch order) takes the k-th contiguous range of the (z, y, x)
// tile order: neighbours share an XCD and its L2.  A bijection for any grid size
// (XCDs 0 .. n%8-1 take one block more); placement-independent for correctness.
// Modes: 0 = blockIdx order; 1 = XCD k takes the k-th contiguous eighth of the
// (z, y, x) order; 2 = row chunks: XCD k takes grid rows (y, z) = k, k + 8, k + 16 ...
// whole (horizontal neighbours share the XCD, the 8 XCDs stay on nearby rows).
#ifndef AT_XCD_PRE
#define AT_XCD_PRE 1
#endif
#ifndef AT_XCD_THR
#define AT_XCD_THR 1
#endif
#ifndef AT_XCD_BND
#define AT_XCD_BND 0
#endif
#ifndef AT_XCD_GRP
#define AT_XCD_GRP 0
#endif
struct TileIdx {
  int x, y, z;
};
// a / d for a, d < 2^24 (grid sizes): a float reciprocal and two correction steps
// instead of the ~40-instruction integer division (k_boundary: +2.7 % with it)
__device__ __forceinline__ uint32_t udiv24(uint32_t a, uint32_t d) {
  // (v_rcp_f32 within 1 ulp, the product rounded: q is off by at most 2)
  uint32_t q = (uint32_t)((float)a * __builtin_amdgcn_rcpf((float)d));
  int32_t r = (int32_t)(a - q * d);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (r < 0) { q--; r += (int32_t)d; }
    if (r >= (int32_t)d) { q++; r -= (int32_t)d; }
  }
  return q;
}
template <int MODE>
__device__ __forceinline__ TileIdx xcd_block() {
  if constexpr (MODE == 0) return TileIdx{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  const uint32_t gx = gridDim.x, gxy = gridDim.x * gridDim.y, n = gxy * gridDim.z;
  const uint32_t lid = blockIdx.x + gx * blockIdx.y + gxy * blockIdx.z;
  uint32_t t;
  if constexpr (MODE == 1) {
    const uint32_t q = n >> 3, r = n & 7, xcd = lid & 7;
    t = xcd * q + min(xcd, r) + (lid >> 3);
  } else {
    // rows in complete groups of 8 (the first n8 blocks: the same count on every
    // XCD), the last partial group in blockIdx order
    const uint32_t rows = gridDim.y * gridDim.z, n8 = (rows & ~7u) * gx;
    if (lid < n8) {
      const uint32_t k = lid >> 3, j = udiv24(k, gx);
      t = ((j << 3) + (lid & 7)) * gx + (k - j * gx);
    } else {
      t = lid;
    }
  }
  const uint32_t z = udiv24(t, gxy), rem = t - z * gxy, y = udiv24(rem, gx);
  return TileIdx{(int)(rem - y * gx), (int)y, (int)z};
}

__device__ __forceinline__ uint32_t kt_wg_id() {
  return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
}
__device__ __forceinline__ void kt_begin(const DevBufs& b, int stage) {
  if (b.kt_stage != stage || threadIdx.x != 0 || threadIdx.y != 0) return;
  const uint32_t id = kt_wg_id();
  if (id == 0) *b.kgrid = gridDim.x * gridDim.y * gridDim.z;
  if (id < b.kwg_cap) b.kwg[id] = wall_clock64();
}
__device__ __forceinline__ void kt_end(const DevBufs& b, int stage) {  // one thread per workgroup, work done
  if (b.kt_stage != stage) return;
  const uint32_t id = kt_wg_id();
  if (id < b.kwg_cap) b.kwg[b.kwg_cap + id] = wall_clock64();
}
// kKtSpanWgs workgroups, each a strided share of the stamps, combined by 64-bit
// atomicMax into the control block (zeroed at the batch start): [0] holds the
// complement of the first start, [1] the last end.  One workgroup walking all
// 23,040 stamps of a 192-frame k_thr_ccl launch took 43 us on the batch's chain.
constexpr int kKtSpanWgs = 32;
__global__ __launch_bounds__(256) void k_kt_span(DevBufs b) {
  const uint32_t n = min(*b.kgrid, b.kwg_cap);
  uint64_t mn = ~0ull, mx = 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += kKtSpanWgs * 256) {
    mn = min(mn, b.kwg[i]);
    mx = max(mx, b.kwg[b.kwg_cap + i]);
  }
  mn = wave_reduce(mn, MinOp());
  mx = wave_reduce(mx, MaxOp());
  if (lane_id() == 0 && mx) {
    atomicMax((unsigned long long*)&b.kstamp[0], (unsigned long long)~mn);
    atomicMax((unsigned long long*)&b.kstamp[1], (unsigned long long)mx);
  }
}

__constant__ float c_filter[7] = {0.01110899634659290314f, 0.13533528149127960205f, 0.60653066635131835938f,
                                  1.00000000000000000000f, 0.60653066635131835938f, 0.13533528149127960205f,
                                  0.01110899634659290314f};

// ---------------------------------------------------------------------------
// K1: gray / decimate / 4x4 tile min-max.  One thread per 4x4 decimated tile
// (8x8 full-resolution pixels).  YUYV rows are read as 16-byte loads, so a
// wave reads 1 KiB contiguous per row.
// ---------------------------------------------------------------------------
// Y of the 8 full-resolution pixels (row, x .. x + 7) of a frame in format FMT
// (0 YUYV: one 16-B load; 1 BGR8: three 8-B loads, OpenCV BGR2YUV_YUYV luma with
// ITUR_BT_601_SHIFT 20; 2 GRAY8: one 8-B load).  x is a multiple of 8.
template <int FMT>
__device__ __forceinline__ void load_y8(const uint8_t* in, int W, int row, int x, uint32_t (&y)[8]) {
  if (FMT == 0) {  // YUYV: Y at even bytes
    const uint4 v = *reinterpret_cast<const uint4*>(in + ((size_t)row * W + x) * 2);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      y[2 * k] = w[k] & 0xff;
      y[2 * k + 1] = (w[k] >> 16) & 0xff;
    }
  } else if (FMT == 1) {
    const uint8_t* p = in + ((size_t)row * W + x) * 3;
    const uint2 v0 = *reinterpret_cast<const uint2*>(p);
    const uint2 v1 = *reinterpret_cast<const uint2*>(p + 8);
    const uint2 v2 = *reinterpret_cast<const uint2*>(p + 16);
    uint8_t bytes[24];
    *reinterpret_cast<uint2*>(bytes) = v0;
    *reinterpret_cast<uint2*>(bytes + 8) = v1;
    *reinterpret_cast<uint2*>(bytes + 16) = v2;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int bb = bytes[3 * k], gg = bytes[3 * k + 1], rr = bytes[3 * k + 2];
      y[k] = (uint32_t)((269484 * rr + 528482 * gg + 102760 * bb + (1 << 19) + (16 << 20)) >> 20);
    }
  } else {
    const uint2 v = *reinterpret_cast<const uint2*>(in + (size_t)row * W + x);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      y[k] = (v.x >> (8 * k)) & 0xff;
      y[4 + k] = (v.y >> (8 * k)) & 0xff;
    }
  }
}

// wgray: write the full-resolution gray plane (BGR8 input, whose luma k_decode
// samples from it, or the parity taps); YUYV / GRAY8 frames carry their luma
// already, so k_decode samples the frame and the plane is not written
template <int FMT>
__global__ __launch_bounds__(256) void k_pre(DevBufs b, Geom g, int wgray) {
  const TileIdx bi = xcd_block<AT_XCD_PRE>();
  const int f = bi.z;
  const int tx = bi.x * 64 + threadIdx.x;
  const int ty = bi.y * 4 + threadIdx.y;
  // the batch's control block starts at zero (no memset node): nothing in k_pre
  // reads it, every later kernel follows in stream order
  if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
    for (uint32_t w = threadIdx.y * 64 + threadIdx.x; w < b.ctrl_words; w += 256) b.ctrl[w] = 0;
    for (uint32_t w = threadIdx.y * 64 + threadIdx.x; w < b.qc_words; w += 256) b.nqcand[w] = 0;
  }
  if (tx >= g.TW || ty >= g.TH) return;
  const uint8_t* in = b.frames[f];
  uint8_t* gray = b.gray + (size_t)f * g.W * g.H;
  uint8_t* dec = b.dec + (size_t)f * g.Wd * g.Hd;
  uint32_t mn = 255, mx = 0;
  const int x0 = tx * 8;
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int row = ty * 8 + r;
    uint32_t y[8];
    load_y8<FMT>(in, g.W, row, x0, y);
    if (FMT == 1 || wgray) {
      uint2 gw;
      gw.x = y[0] | (y[1] << 8) | (y[2] << 16) | (y[3] << 24);
      gw.y = y[4] | (y[5] << 8) | (y[6] << 16) | (y[7] << 24);
      *reinterpret_cast<uint2*>(gray + (size_t)row * g.W + x0) = gw;
    }
    if ((r & 1) == 0) {
      const uint32_t d = y[0] | (y[2] << 8) | (y[4] << 16) | (y[6] << 24);
      *reinterpret_cast<uint32_t*>(dec + (size_t)(row >> 1) * g.Wd + (x0 >> 1)) = d;
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        mn = min(mn, y[k]);
        mx = max(mx, y[k]);
      }
    }
  }
  uint8_t* mm = b.mm + (size_t)f * g.TW * g.TH * 2;
  *reinterpret_cast<uint16_t*>(mm + 2 * ((size_t)ty * g.TW + tx)) = (uint16_t)(mn | (mx << 8));
}

// ---------------------------------------------------------------------------
// K3: threshold + tile-local union-find.
// One 512-thread workgroup per 64x32 decimated tile; thread (ty,tx) owns
// 2x2 block (ty,tx).  Node slots in LDS are ordered like the global node ids
// (per block row: 32 foreground nodes, then 64 background L/R nodes), so
// "link to the smaller slot" == "link to the smaller id" and every local root
// is the minimum node id of its local component.
// ---------------------------------------------------------------------------
// (relaxed atomic loads, not volatile: a volatile access through the generic
// pointer would be compiled to flat instructions instead of ds_read)
// Union-find node index (the parent plane, the size plane, the labels the later stages
// key pairs by): the nodes of 2x2-block row BY are stored contiguously, its BW fg nodes
// (F, the block's top-left pixel) then its 2 BW bg nodes (L, R: bottom-left, bottom-right)
// -- 3 words per block instead of one per pixel (the top-right pixel is no node).  The
// index is monotone in the reference's node id (the pixel index), so a component's
// minimum index is its minimum node id, the reference's label (node_pixel maps back).
__device__ __forceinline__ uint32_t node_F(const Geom& g, int BY, int BX) { return (uint32_t)(BY * 3 * g.BW + BX); }
__device__ __forceinline__ uint32_t node_L(const Geom& g, int BY, int BX) {
  return (uint32_t)(BY * 3 * g.BW + g.BW + 2 * BX);
}
__device__ __forceinline__ uint32_t node_pixel(int BW, int Wd, uint32_t n) {
  const uint32_t by = n / (uint32_t)(3 * BW), r = n - by * (uint32_t)(3 * BW);
  return r < (uint32_t)BW ? 2 * by * (uint32_t)Wd + 2 * r : (2 * by + 1) * (uint32_t)Wd + (r - (uint32_t)BW);
}

__device__ __forceinline__ uint32_t lds_load(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// find with path halving: every visited node is pointed at its grandparent (an
// ancestor with a smaller id, so the atomicMin never loses a link)
__device__ __forceinline__ uint32_t lds_find(uint32_t* par, uint32_t n) {
  uint32_t p = lds_load(par + n);
  while (p != n) {
    const uint32_t gp = lds_load(par + p);
    if (gp != p) atomicMin(&par[n], gp);
    n = p;
    p = gp;
  }
  return n;
}

__device__ __forceinline__ void lds_union(uint32_t* par, uint32_t a, uint32_t b) {
  while (true) {
    a = lds_find(par, a);
    b = lds_find(par, b);
    if (a == b) return;
    if (a < b) {
      const uint32_t old = atomicMin(&par[b], a);
      if (old == b) return;
      b = old;
    } else {
      const uint32_t old = atomicMin(&par[a], b);
      if (old == a) return;
      a = old;
    }
  }
}

template <int TW>
__device__ __forceinline__ uint32_t slot_of(int ty, int tx, int type) {
  using T = CclTile<TW>;
  return (uint32_t)(ty * T::ROW_NODES + (type == 0 ? tx : T::BW + 2 * tx + (type - 1)));
}

// One candidate union per thread (the reference's Merge, labeling_allegretti_2019_BKE.cu:302-338,
// over the tile's border blocks): threads 0..5*BW-1 the top block row (BW blocks x
// P, Q, R and the two background links), then the left block column (BH x P, S,
// background S), then the right column (BH-1 x R).  Every union is one short
// chain of global round trips instead of up to five in a row per lane.
template <int TW>
struct BorderRoles {
  static constexpr int Top = 5 * CclTile<TW>::BW, Left = 3 * CclTile<TW>::BH, Right = CclTile<TW>::BH - 1;
  static constexpr int NT = (Top + Left + Right + 63) / 64 * 64;
};

// kept bit of a root's parent word: the component has >= 25 pixels (BlobDiff's
// size test, apriltag_gpu.cu:331-337), throughput mode
constexpr uint32_t kKeptBit = 0x80000000u;
// par word of a listed local root between k_thr_ccl and k_ccl_merge (throughput
// mode): kListBit | its slot in the tile's list (node ids are < 2^22)
constexpr uint32_t kListBit = 0x40000000u;
// s_cnt flag of a local root whose component reaches a border block of the tile
// (only those can take part in k_ccl_border's unions)
constexpr uint32_t kTouchBit = 0x80000000u;

// SGPR budget of k_thr_ccl: .sgpr_count <= 80 keeps 8 waves per SIMD (4 of its 8-wave
// workgroups per CU); at 82 (the border descriptor's addressing) the CU holds 7 waves
// per SIMD, i.e. 3 workgroups: k_thr_ccl 0.24 -> 0.30 ms per 128 frames
// (MI355X_MICROARCH.md: admitted blocks = 800 / (ceil(sgpr / 16) * 16 + 16))
#ifndef AT_THR_SGPRS
#define AT_THR_SGPRS 80
#endif
// PRE < 0: the tile's decimated pixels and 4x4 min/max come from k_pre's planes.
// PRE = 0 / 1 / 2 (frame format YUYV / BGR8 / GRAY8): k_pre's work is done here --
// the workgroup reads its tile's full-resolution rows once (gray and decimated
// planes written for the later stages), plus the decimated samples of the
// 8-pixel halo its filtered tile min/max needs, so there is no min/max plane,
// no re-read of the decimated plane and one launch less.
// One CCL tile (k_thr_ccl: one workgroup per tile, bi from the XCD-aware order).
template <int TWD, int PRE>
__device__ __forceinline__ void thr_ccl_tile(const DevBufs& b, const Geom& g, const Params& prm, const TileIdx bi) {
  using CT = CclTile<TWD>;
  constexpr int NT = CT::NT;
  constexpr int kCclTileW = CT::W, kCclBW = CT::BW, kCclTileNodes = CT::NODES;
  constexpr int kTW = kCclTileW / 4, kTH = kCclTileH / 4;  // 4x4 threshold tiles per CCL tile
  constexpr int kHR = kCclTileH + 1, kHC = kCclTileW + 2;  // threshold halo: rows y0-1.., cols x0-1..x0+W
  const int f = bi.z;
  const int tid = threadIdx.x;
  const int y0 = bi.y * kCclTileH, x0 = bi.x * kCclTileW;
  const uint8_t* dec = b.dec + (size_t)f * g.Wd * g.Hd;
  const uint8_t* mm = b.mm + (size_t)f * g.TW * g.TH * 2;
  uint8_t* thr = b.thr + (size_t)f * g.Wd * g.Hd;

  __shared__ uint8_t s_umn[kTH + 3][kTW + 4], s_umx[kTH + 3][kTW + 4];
  __shared__ uint8_t s_fmn[kTH + 1][kTW + 2], s_fmx[kTH + 1][kTW + 2];
  __shared__ __attribute__((aligned(4))) uint8_t s_t[kHR][kHC + 2];  // thr of rows y0-1..y0+H-1, cols x0-1..x0+W (+pad)
  __shared__ uint32_t s_par[kCclTileNodes];
  __shared__ uint32_t s_cnt[kCclTileNodes];
  __shared__ uint32_t s_nlr;
  __shared__ uint16_t s_li[TWD == 64 ? kCclTileNodes : 1];  // list slot of each listed root (border descriptor)
  __shared__ uint32_t s_gid[kCclTileNodes];  // global node id of every slot (the publish reads its roots')
  if (tid == 0) s_nlr = 0;
  // unfiltered tile min/max for tile rows ty0-2..ty0+kTH, cols tx0-2..tx0+kTW+1
  const int ty0 = y0 / 4, tx0 = x0 / 4;
  constexpr int kDecPer = (kHR * kHC + NT - 1) / NT;
  uint8_t dv[kDecPer];
  // PRE < 0: the halo rows as 4-byte windows, window j of row r = cols x0-1+4j .. x0+2+4j
  // (s_t's dword j of row r), one task per window: 561 tasks instead of 2178 bytes
  constexpr int kWin = (kHC + 2) / 4, kWinN = kHR * kWin, kWinPer = (kWinN + NT - 1) / NT;
  uint32_t dw4[kWinPer];
  // PRE: decimated samples of rows y0-8 .. y0+35, cols x0-8 .. x0+TW+7 (the tiles
  // of s_umn), staged over s_par (unused until the labeling)
  constexpr int kDR = kCclTileH + 12, kDC = kCclTileW + 16;
  static_assert(PRE < 0 || kDR * kDC <= (int)sizeof(s_par), "decimated halo must fit over s_par");
  uint8_t(*s_dec)[kDC] = reinterpret_cast<uint8_t(*)[kDC]>(s_par);
  if constexpr (PRE >= 0) {
    // the batch's control block starts at zero (no memset node): nothing here
    // reads it, every later kernel follows in stream order
    if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
      for (uint32_t w = tid; w < b.ctrl_words; w += NT) b.ctrl[w] = 0;
      for (uint32_t w = tid; w < b.qc_words; w += NT) b.nqcand[w] = 0;
      __syncthreads();
    }
  }
  kt_begin(b, 1);
  // AT_PHASE_PROBE (throughput mode): per-phase wall-clock of workgroup thread 0
  // summed over the launch in probe[48 + k], workgroups in probe[63]
  uint64_t t_ph = 0;
  auto ph = [&](int k) {
    if (!AT_PROBE_ON(prm) || PRE >= 0 || tid != 0) return;
    const uint64_t t = wall_clock64();
    if (k > 0) atomicAdd((unsigned long long*)&b.probe[47 + k], (unsigned long long)(t - t_ph));
    else atomicAdd((unsigned long long*)&b.probe[63], 1ull);
    t_ph = t;
  };
  ph(0);
  if constexpr (PRE >= 0) {
    const uint8_t* in = b.frames[f];
    uint8_t* gray = b.gray + (size_t)f * g.W * g.H;
    uint8_t* decw = b.dec + (size_t)f * g.Wd * g.Hd;
    // (1) the tile's full-resolution rows 2y0 .. 2y0+63, cols 2x0 .. 2x0+2TW-1 in
    // 8-pixel chunks: gray out; even rows give 4 decimated samples each
    constexpr int kCR = 2 * kCclTileW / 8;               // chunks per full row
    constexpr int kIn = (2 * kCclTileH * kCR + NT - 1) / NT;
    // (2) the halo's decimated samples in 4-sample chunks (8 full pixels of an
    // even row) over the kDR x kDC region minus the interior
    constexpr int kHCc = kDC / 4;
    constexpr int kHal = (kDR * kHCc + NT - 1) / NT;
    uint32_t yin[kIn][8], yh[kHal][8];
    // every load of both parts is issued before any is used
#pragma unroll
    for (int k = 0; k < kIn; k++) {
      const int i = tid + NT * k;
      const int row = 2 * y0 + i / kCR, x = 2 * x0 + 8 * (i % kCR);
      if (i < 2 * kCclTileH * kCR && row < g.H && x < g.W) load_y8<PRE>(in, g.W, row, x, yin[k]);
    }
#pragma unroll
    for (int k = 0; k < kHal; k++) {
      const int i = tid + NT * k;
      const int r = i / kHCc, cc = i % kHCc;
      const int yd = y0 - 8 + r, xd = x0 - 8 + 4 * cc;
      const bool interior = r >= 8 && r < 8 + kCclTileH && cc >= 2 && cc < 2 + kCclTileW / 4;
      if (i < kDR * kHCc && !interior && yd >= 0 && yd < g.Hd && xd >= 0 && xd < g.Wd)
        load_y8<PRE>(in, g.W, 2 * yd, 2 * xd, yh[k]);
    }
#pragma unroll
    for (int k = 0; k < kIn; k++) {
      const int i = tid + NT * k;
      const int lr = i / kCR, row = 2 * y0 + lr, x = 2 * x0 + 8 * (i % kCR);
      if (i < 2 * kCclTileH * kCR && row < g.H && x < g.W) {
        const uint32_t(&y)[8] = yin[k];
        if (PRE == 1 || prm.taps)  // (k_decode samples YUYV / GRAY8 frames directly)
          *reinterpret_cast<uint2*>(gray + (size_t)row * g.W + x) =
              make_uint2(y[0] | (y[1] << 8) | (y[2] << 16) | (y[3] << 24), y[4] | (y[5] << 8) | (y[6] << 16) | (y[7] << 24));
        if ((lr & 1) == 0) {
          const uint32_t d = y[0] | (y[2] << 8) | (y[4] << 16) | (y[6] << 24);
          *reinterpret_cast<uint32_t*>(decw + (size_t)(row >> 1) * g.Wd + (x >> 1)) = d;
          *reinterpret_cast<uint32_t*>(&s_dec[8 + (lr >> 1)][8 + (x >> 1) - x0]) = d;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kHal; k++) {
      const int i = tid + NT * k;
      const int r = i / kHCc, cc = i % kHCc;
      const int yd = y0 - 8 + r, xd = x0 - 8 + 4 * cc;
      const bool interior = r >= 8 && r < 8 + kCclTileH && cc >= 2 && cc < 2 + kCclTileW / 4;
      if (i < kDR * kHCc && !interior && yd >= 0 && yd < g.Hd && xd >= 0 && xd < g.Wd) {
        const uint32_t(&y)[8] = yh[k];
        *reinterpret_cast<uint32_t*>(&s_dec[r][4 * cc]) = y[0] | (y[2] << 8) | (y[4] << 16) | (y[6] << 24);
      }
    }
    __syncthreads();
    // tile min/max of every staged tile inside the image (whole tiles: W, H % 8 == 0)
    for (int i = tid; i < (kTH + 3) * (kTW + 4); i += NT) {
      const int r = i / (kTW + 4), c = i % (kTW + 4);
      const int tr = ty0 - 2 + r, tc = tx0 - 2 + c;
      uint32_t mn = 255, mx = 0;  // out of range: neutral for min/max
      if (tr >= 0 && tr < g.TH && tc >= 0 && tc < g.TW) {
#pragma unroll
        for (int dr = 0; dr < 4; dr++) {
          const uint32_t w = *reinterpret_cast<const uint32_t*>(&s_dec[4 * r + dr][4 * c]);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            mn = min(mn, (w >> (8 * k)) & 0xff);
            mx = max(mx, (w >> (8 * k)) & 0xff);
          }
        }
      }
      s_umn[r][c] = (uint8_t)mn;
      s_umx[r][c] = (uint8_t)mx;
    }
#pragma unroll
    for (int k = 0; k < kDecPer; k++) {
      const int i = tid + NT * k;
      const int y = y0 - 1 + i / kHC, x = x0 - 1 + i % kHC;
      dv[k] = (i < kHR * kHC && y >= 0 && y < g.Hd && x >= 0 && x < g.Wd) ? s_dec[i / kHC + 7][i % kHC + 7] : 0;
    }
    __syncthreads();  // s_dec (over s_par) read before the labeling writes s_par
  } else {
  // the tile's decimated pixels (+1 halo) are loaded together with the tile
  // min/max: one global round trip instead of two.  A window straddles two aligned
  // dwords of its row (W/2 is a multiple of 4); loads from clamped addresses (no
  // branch per load), the bytes outside the image are masked by the threshold
  (void)dv;
#pragma unroll
  for (int k = 0; k < kWinPer; k++) {
    const int t = tid + NT * k, r = t / kWin, j = t % kWin;
    const int yc = min(max(y0 - 1 + r, 0), g.Hd - 1), wd4 = g.Wd >> 2, xa = (x0 >> 2) + j - 1;
    const uint32_t* row = reinterpret_cast<const uint32_t*>(dec + (size_t)yc * g.Wd);
    const uint32_t A = row[min(max(xa, 0), wd4 - 1)], B = row[min(xa + 1, wd4 - 1)];
    dw4[k] = __builtin_amdgcn_alignbyte(B, A, 3);  // A's last byte, B's first three
  }
  for (int i = tid; i < (kTH + 3) * (kTW + 4); i += NT) {
    const int r = i / (kTW + 4), c = i % (kTW + 4);
    const int tr = ty0 - 2 + r, tc = tx0 - 2 + c;
    const int trc = min(max(tr, 0), g.TH - 1), tcc = min(max(tc, 0), g.TW - 1);
    const uint16_t v = *reinterpret_cast<const uint16_t*>(mm + 2 * ((size_t)trc * g.TW + tcc));
    const bool in = tr == trc && tc == tcc;  // out of range: neutral for min/max
    s_umn[r][c] = in ? (uint8_t)(v & 0xff) : (uint8_t)255;
    s_umx[r][c] = in ? (uint8_t)(v >> 8) : (uint8_t)0;
  }
  __syncthreads();
  ph(1);
  }
  // InternalBlockFilter: clipped 3x3 min of mins / max of maxes for tile rows ty0-1..ty0+kTH-1
  for (int i = tid; i < (kTH + 1) * (kTW + 2); i += NT) {
    const int r = i / (kTW + 2), c = i % (kTW + 2);
    uint8_t mn = 255, mx = 0;
#pragma unroll
    for (int dr = 0; dr < 3; dr++)
#pragma unroll
      for (int dc = 0; dc < 3; dc++) {
        mn = min(mn, s_umn[r + dr][c + dc]);
        mx = max(mx, s_umx[r + dr][c + dc]);
      }
    s_fmn[r][c] = mn;
    s_fmx[r][c] = mx;
  }
  __syncthreads();
  ph(2);
  // InternalThreshold for the halo region; outside the image -> 127
  if constexpr (PRE < 0) {
    // one 4-byte window per task: byte 0 in 4x4 tile column j of the filtered
    // min/max, bytes 1-3 in column j + 1
#pragma unroll
    for (int k = 0; k < kWinPer; k++) {
      const int t = tid + NT * k, r = t / kWin, j = t % kWin, y = y0 - 1 + r;
      if (t < kWinN) {
        uint32_t out = 0x7f7f7f7fu;
        if (y >= 0 && y < g.Hd) {
          const int fr = (y >> 2) - (ty0 - 1);
          const int mn0 = s_fmn[fr][j], mx0 = s_fmx[fr][j], mn1 = s_fmn[fr][j + 1], mx1 = s_fmx[fr][j + 1];
          const int d0 = mx0 - mn0, d1 = mx1 - mn1;
          // (d < 0 only where every tile of the 3x3 is outside the image: its bytes are
          // outside too, 127 below whatever th is)
          const uint32_t th0 = (uint32_t)(mn0 + (d0 >> 1)), th1 = (uint32_t)(mn1 + (d1 >> 1));
          // v > th for the four bytes at once, in 16-bit lanes (bytes 0 and 2, bytes 1 and
          // 3): bit 8 of th + 0x100 - v (in 1 .. 0x1ff, no borrow between lanes) is clear
          // exactly when v > th
          const uint32_t wv = dw4[k];
          const uint32_t glo = ~((th0 | (th1 << 16)) + 0x01000100u - (wv & 0x00ff00ffu)) & 0x01000100u;
          const uint32_t ghi = ~((th1 | (th1 << 16)) + 0x01000100u - ((wv >> 8) & 0x00ff00ffu)) & 0x01000100u;
          out = ((glo >> 8) * 0xffu) | (((ghi >> 8) * 0xffu) << 8);
          // 127 where the tile's contrast is too low (byte 0: column j, bytes 1-3: j + 1)
          // or the byte lies outside the image (the windows at the left / right border)
          uint32_t bad = (d0 >= prm.min_white_black_diff ? 0u : 0xffu) | (d1 >= prm.min_white_black_diff ? 0u : 0xffffff00u);
          const int xs = x0 - 1 + 4 * j;
          if (xs < 0 || xs + 3 >= g.Wd) {
#pragma unroll
            for (int bb = 0; bb < 4; bb++)
              if (xs + bb < 0 || xs + bb >= g.Wd) bad |= 0xffu << (8 * bb);
          }
          out = (out & ~bad) | (0x7f7f7f7fu & bad);
        }
        *reinterpret_cast<uint32_t*>(&s_t[r][4 * j]) = out;
      }
    }
  } else {
#pragma unroll
  for (int k = 0; k < kDecPer; k++) {
    const int i = tid + NT * k;
    if (i < kHR * kHC) {
      const int r = i / kHC, c = i % kHC;
      const int y = y0 - 1 + r, x = x0 - 1 + c;
      uint8_t res = 127;
      if (y >= 0 && y < g.Hd && x >= 0 && x < g.Wd) {
        const int fr = (y >> 2) - (ty0 - 1), fc = (x >> 2) - (tx0 - 1);
        const int mn = s_fmn[fr][fc], mx = s_fmx[fr][fc];
        if (mx - mn < prm.min_white_black_diff) {
          res = 127;
        } else {
          const uint8_t th = (uint8_t)(mn + (mx - mn) / 2);
          res = dv[k] > th ? 255 : 0;
        }
      }
      s_t[r][c] = res;
    }
  }
  }
  for (int i = tid; i < kCclTileNodes; i += NT) s_cnt[i] = 0;
  __syncthreads();
  ph(3);

  // write this tile's threshold plane (4 bytes per thread)
  {
    const int r = tid / (kCclTileW / 4), c4 = (tid % (kCclTileW / 4)) * 4;
    const int y = y0 + r, x = x0 + c4;
    if (y < g.Hd && x < g.Wd) {
      const uint32_t w = s_t[r + 1][c4 + 1] | (s_t[r + 1][c4 + 2] << 8) | (s_t[r + 1][c4 + 3] << 16) |
                         ((uint32_t)s_t[r + 1][c4 + 4] << 24);
      *reinterpret_cast<uint32_t*>(thr + (size_t)y * g.Wd + x) = w;
    }
  }
  // Local labeling (InitLabeling P/Q/R/S + Merge, labeling_allegretti_2019_BKE.cu:114-338)
  // in two steps.  (1) Horizontal runs without atomics: within a block row the
  // fg nodes form a chain (F(x-1) - F(x)) and the bg nodes another
  // (... R(x-1) - L(x) - R(x) - L(x+1) ...); a wave holds whole block rows, so
  // every node finds its run head -- the leftmost node, i.e. the smallest id --
  // from two ballots.  (2) Vertical links (up-left, up, up-right for fg; up for
  // bg) as union-find unions on the run heads, a run linking to each run above
  // it once (a block skips a target its left neighbour in the same run links to).
  const int bty = tid / kCclBW, btx = tid % kCclBW;
#define T(rr, cc) s_t[(rr) + 1][(cc) + 1]
  const int pr = 2 * bty, pc = 2 * btx;
  const uint8_t a = T(pr, pc), bb = T(pr, pc + 1), c = T(pr + 1, pc), d = T(pr + 1, pc + 1);
  const uint32_t F = slot_of<TWD>(bty, btx, 0), L = slot_of<TWD>(bty, btx, 1), R = slot_of<TWD>(bty, btx, 2);
  const uint32_t lane = lane_id();
  bool headF, headL, headR;  // this block's F / L / R starts its run (the run's head)
  {
    const bool fg_left = btx > 0 && (a == 255 || c == 255) && (T(pr, pc - 1) == 255 || T(pr + 1, pc - 1) == 255);
    const bool bg_left = btx > 0 && ((a == 0 && T(pr, pc - 1) == 0) || (c == 0 && T(pr + 1, pc - 1) == 0));
    const bool bg_in = (a == 0 && bb == 0) || (c == 0 && d == 0);  // R(x) - L(x)
    headF = !fg_left;
    headL = !bg_left;
    headR = !bg_in;
    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1);  // lanes <= this one
    const uint64_t lt = (1ull << lane) - 1;                          // lanes < this one
    const uint64_t fs = __ballot(!fg_left);  // run starts (btx == 0 always starts: rows never merge)
    const int hf = 63 - __builtin_clzll(fs & le);
    const uint32_t hF = F - (uint32_t)(lane - hf);
    const uint64_t sl = __ballot(!bg_left), sr = __ballot(!bg_in);
    // L's run head: L itself, or the last run start before L(x) -- in the nearest lane
    // below with a start, its R if R starts there (selects, no branch)
    const int hl = 63 - __builtin_clzll(((sl | sr) & lt) | 1ull);
    const uint32_t hLl = ((sr >> hl) & 1) ? slot_of<TWD>(bty, btx - (lane - hl), 2) : slot_of<TWD>(bty, btx - (lane - hl), 1);
    const uint32_t hL = bg_left ? hLl : L, hR = bg_in ? hL : R;
    s_par[F] = hF;
    s_par[L] = hL;
    s_par[R] = hR;
    __syncthreads();
  ph(4);
    // heads of the run(s) above this block's vertical links (read before any union)
    constexpr uint32_t kNone = 0xffffffffu;
    // (branch-free: the five words read whatever the block -- block row 0 reads its own
    // row and the halo row of s_t, both in bounds -- and kept where the link holds)
    const int uy = bty > 0 ? bty - 1 : 0, ulx = btx > 0 ? btx - 1 : 0, urx = btx < kCclBW - 1 ? btx + 1 : btx;
    const uint32_t vUL = s_par[slot_of<TWD>(uy, ulx, 0)], vU = s_par[slot_of<TWD>(uy, btx, 0)],
                   vUR = s_par[slot_of<TWD>(uy, urx, 0)], vL = s_par[slot_of<TWD>(uy, btx, 1)],
                   vR = s_par[slot_of<TWD>(uy, btx, 2)];
    const uint8_t u0 = T(pr - 1, pc - 1), u1 = T(pr - 1, pc), u2 = T(pr - 1, pc + 1), u3 = T(pr - 1, pc + 2);
    const bool up = bty > 0;
    const uint32_t tUL = up && btx > 0 && a == 255 && u0 == 255 ? vUL : kNone;
    const uint32_t tU = up && (a == 255 || bb == 255) && (u1 == 255 || u2 == 255) ? vU : kNone;
    const uint32_t tUR = up && btx < kCclBW - 1 && bb == 255 && u3 == 255 ? vUR : kNone;
    const uint32_t tL = up && a == 0 && u1 == 0 ? vL : kNone;
    const uint32_t tR = up && bb == 0 && u2 == 0 ? vR : kNone;
    // the left neighbour's targets (same wave: rows never straddle waves)
    const uint32_t pUL = __shfl_up(tUL, 1), pU = __shfl_up(tU, 1), pUR = __shfl_up(tUR, 1), pR = __shfl_up(tR, 1);
    // (no barrier before the unions: a target read while another block's union or path
    // compression runs is a node of the same component -- unions and compressions only
    // lower a parent within its component -- so the union it takes part in is still the
    // right one; a changed value only defeats the left-neighbour dedup, an extra union)
  ph(5);
    auto seen_fg = [&](uint32_t t) { return fg_left && (t == pUL || t == pU || t == pUR); };
    // the wave's unions (at most five per block, mostly none) compacted into a
    // wave-private list in s_gid's storage (unused until the publish) and run with
    // every lane busy: ceil(n / 64) union rounds instead of five divergent sites in a
    // row, each as long as its slowest lane
    constexpr int kUnionPairs = kCclTileNodes / (NT / 64) / 2;
    uint32_t* wl = s_gid + (tid >> 6) * (2 * kUnionPairs);
    uint32_t nq = 0;  // (uniform)
    auto flush = [&]() {
      wave_sync();  // the list's stores before the other lanes' reads
      for (uint32_t i = lane; i < nq; i += 64) lds_union(s_par, wl[2 * i], wl[2 * i + 1]);
      wave_sync();  // (the list may be refilled)
      nq = 0;
    };
    auto push = [&](bool act, uint32_t a, uint32_t b) {
      const uint64_t m = __ballot(act);
      const uint32_t cnt = (uint32_t)__popcll(m);
      if (nq + cnt > (uint32_t)kUnionPairs) flush();
      if (act) {
        const uint32_t pos = nq + lanes_below(m);
        wl[2 * pos] = a;
        wl[2 * pos + 1] = b;
      }
      nq += cnt;
    };
    push(tUL != kNone && !seen_fg(tUL), hF, tUL);
    push(tU != kNone && tU != tUL && !seen_fg(tU), hF, tU);
    push(tUR != kNone && tUR != tUL && tUR != tU && !seen_fg(tUR), hF, tUR);
    push(tL != kNone && !(bg_left && tL == pR), hL, tL);
    push(tR != kNone && !(bg_in && tR == tL), hR, tR);
    if (nq) flush();
  }
#undef T
  __syncthreads();
  ph(6);

  // Every find path runs through run heads only (a run's other nodes point at its head,
  // and unions and path halving only ever link heads), so only the heads are found --
  // compacted per wave like the unions, with no barrier before the root writes (a root
  // written over a head's word is its component's smallest slot, which a concurrent
  // compression's atomicMin leaves, and a find that reads it lands on that root) --
  // and every node's root is then its parent's word: two loads, no loop.
  {
    constexpr int kFindList = kCclTileNodes / (NT / 64);  // 3 per lane
    uint32_t* wl = s_gid + (tid >> 6) * kFindList;       // (this wave's own slots of s_gid)
    uint32_t nh = 0;                                      // (uniform)
    auto push = [&](bool act, uint32_t v) {
      const uint64_t m = __ballot(act);
      if (act) wl[nh + lanes_below(m)] = v;
      nh += (uint32_t)__popcll(m);
    };
    push(headF, F);
    push(headL, L);
    push(headR, R);
    wave_sync();
    for (uint32_t i = lane; i < nh; i += 64) {
      const uint32_t h = wl[i];
      s_par[h] = lds_find(s_par, h);
    }
    wave_sync();  // (a run's heads are in the lanes of its own wave: rows never straddle waves)
  }
  const uint32_t rF = s_par[s_par[F]], rL = s_par[s_par[L]], rR = s_par[s_par[R]];
  ph(7);
  // every slot's global node id, by its owner (the publish looks its roots' ids up
  // instead of decoding slot numbers: ~15 VALU per decode)
  const uint32_t idF = node_F(g, y0 / 2 + bty, x0 / 2 + btx), idL = node_L(g, y0 / 2 + bty, x0 / 2 + btx);
  s_gid[F] = idF;
  s_gid[L] = idL;
  s_gid[R] = idL + 1;
  const uint32_t nfg = (a == 255) + (bb == 255) + (c == 255) + (d == 255);
  const uint32_t nbl = (a == 0) + (c == 0), nbr = (bb == 0) + (d == 0);
  // components reaching a border block may be merged across tiles (k_ccl_border);
  // every other component is complete here: root and pixel count are final
  const bool edge = bty == 0 || bty == CT::BH - 1 || btx == 0 || btx == kCclBW - 1;
  // runs of equal roots in consecutive lanes add their pixels with one atomic by the
  // run's head (same-address LDS atomics from a run's lanes serialize)
  auto count = [&](uint32_t r, uint32_t n) {
    const uint32_t key = n ? r : 0xffffffffu;
    const bool same = n && wave_shr1(key, 0xfffffffeu) == key;
    const uint64_t sm = __ballot(same), em = __ballot(edge && n);
    const uint32_t incl = wave_incl_scan(n, AddOp(), 0u);
    const bool head = n && !same;
    const uint32_t len = head ? run_len(sm, lane) : 1u;
    const uint32_t last = (uint32_t)__shfl((int)incl, (int)(lane + len - 1));
    if (head) {
      atomicAdd(&s_cnt[r], last - incl + n);
      const uint64_t run = len == 64 ? ~0ull : ((1ull << len) - 1);
      if ((em >> lane) & run) atomicOr(&s_cnt[r], kTouchBit);
    }
  };
  count(rF, nfg);
  count(rL, nbl);
  count(rR, nbr);
  __syncthreads();
  ph(8);

  // publish: gpar[node] = global id of its local root; size[root] = local pixel count
  const int BY = y0 / 2 + bty, BX = x0 / 2 + btx;
  const bool inimg = BY < g.BH && BX < g.BW;
  // sizes only at local roots with pixels: every other entry is never read
  // (k_boundary reads component roots, k_ccl_roots the listed local roots; the
  // AT_STAGE_SIZES tap masks the plane with the forest, k_tap_sizes)
  const uint32_t wF = inimg && rF == F ? s_cnt[F] : 0u, wL = inimg && rL == L ? s_cnt[L] : 0u,
                 wR = inimg && rR == R ? s_cnt[R] : 0u;
  const uint32_t cF = wF & ~kTouchBit, cL = wL & ~kTouchBit, cR = wR & ~kTouchBit;
  // the tile's local roots of components reaching its border (with pixels), listed for
  // the cross-tile merge (k_ccl_merge in throughput mode, k_ccl_border + k_ccl_roots in latency mode)
  const bool lF = cF && (wF & kTouchBit), lL = cL && (wL & kTouchBit), lR = cR && (wR & kTouchBit);
  // (their list slots: one LDS atomic per wave -- the same-address atomics of a wave's
  // listed roots serialized, three times over)
  const uint64_t mlF = __ballot(lF), mlL = __ballot(lL), mlR = __ballot(lR);
  const uint32_t nlF = (uint32_t)__popcll(mlF), nlL = (uint32_t)__popcll(mlL), nlR = (uint32_t)__popcll(mlR);
  uint32_t lb0 = 0;
  if (lane == 0 && nlF + nlL + nlR) lb0 = atomicAdd(&s_nlr, nlF + nlL + nlR);
  lb0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)lb0);
  const uint32_t iF = lb0 + lanes_below(mlF), iL = lb0 + nlF + lanes_below(mlL), iR = lb0 + nlF + nlL + lanes_below(mlR);
  constexpr bool kKeep = TWD != 32;
  if constexpr (kKeep) {  // list slots of the roots, for the border descriptor
    if (lF) s_li[F] = (uint16_t)iF;
    if (lL) s_li[L] = (uint16_t)iL;
    if (lR) s_li[R] = (uint16_t)iR;
    __syncthreads();  // (the descriptor below reads other threads' roots' slots)
  }
  const size_t tl = (size_t)f * g.CTX * g.CTY + bi.y * g.CTX + bi.x;
  if (inimg) {
    auto gid = [&](uint32_t s) -> uint32_t { return s_gid[s]; };
    uint32_t* par = b.par + (size_t)f * g.Wd * g.Hd;
    uint32_t* size = b.size + (size_t)f * g.Wd * g.Hd;
    // a root of a tile-interior component is final: in throughput mode (k_ccl_merge
    // sets the others' kept bits) its parent word gets the kept bit here and it is not listed
    auto fin = [&](uint32_t w, uint32_t c) -> uint32_t {
      return (kKeep && c && !(w & kTouchBit) && c >= 25) ? kKeptBit : 0u;
    };
    uint32_t* lr = b.lroot + tl * kCclTileNodesMax;
    uint32_t* lc = b.lcnt + tl * kCclTileNodesMax;
    if (lF) { lr[iF] = idF; lc[iF] = cF; }
    if (lL) { lr[iL] = idL; lc[iL] = cL; }
    if (lR) { lr[iR] = idL + 1; lc[iR] = cR; }
    // throughput mode: a listed root's own word names its list slot (kListBit | slot)
    // until k_ccl_merge overwrites it with the component's root
    auto word = [&](uint32_t r, uint32_t w, uint32_t c, bool listed, uint32_t li) -> uint32_t {
      return (kKeep && listed) ? kListBit | li : gid(r) | fin(w, c);
    };
    par[idF] = word(rF, wF, cF, lF, iF);
    *reinterpret_cast<uint2*>(par + idL) = make_uint2(word(rL, wL, cL, lL, iL), word(rR, wR, cR, lR, iR));
    // local counts at local roots: latency mode sums them at the component roots
    // (k_ccl_roots) and k_boundary tests them; throughput mode carries the kept bit
    // in the root words instead (and k_ccl_merge the counts in its lists), so the
    // plane is written only for the AT_STAGE_SIZES tap -- ~12 k scattered 4-B stores
    // per 720p frame (0.3 MB of write traffic) otherwise
    if (!kKeep || prm.taps) {
      if (cF) size[idF] = cF;
      if (cL | cR) {
        if (cL && cR) *reinterpret_cast<uint2*>(size + idL) = make_uint2(cL, cR);
        else if (cL) size[idL] = cL;
        else size[idL + 1] = cR;
      }
    }
  }
  if constexpr (TWD == 64) {
    // throughput mode: the tile's border descriptor for k_ccl_merge (CclDesc) --
    // the threshold bytes of its outer rows / columns and the list slots of the
    // roots of its border blocks' nodes (a node with pixels in a border block
    // belongs to a listed root), so the merge reads whole descriptors instead of
    // scattered threshold bytes and parent words.  Issued before the last barrier,
    // beside the other stores (after it, their latency lengthened every workgroup)
    uint32_t* dw = b.cdesc + tl * CclDesc::kWords;
    // whole-word stores: a wave holds two block rows, so the slots of blocks (x, x+1)
    // of a row are in lanes l, l+1 and those of block rows (2i, 2i+1) of a column in
    // lanes l, l+32 of wave i
    {
    const uint32_t sF = nfg ? s_li[rF] : 0xffffu, sL = nbl ? s_li[rL] : 0xffffu, sR = nbr ? s_li[rR] : 0xffffu;
    const uint32_t nF = wave_read_next(sF), nL = wave_read_next(sL), nR = wave_read_next(sR);
    const int w = tid >> 6;
    if ((bty == 0 || bty == CT::BH - 1) && !(btx & 1)) {
      const int o = bty == 0 ? 0 : CclDesc::BsF - CclDesc::TsF;
      dw[CclDesc::TsF + o + (btx >> 1)] = sF | (nF << 16);
      dw[CclDesc::TsL + o + (btx >> 1)] = sL | (nL << 16);
      dw[CclDesc::TsR + o + (btx >> 1)] = sR | (nR << 16);
    }
    const uint32_t dF = __shfl(sF, (int)(lane & 31) + 32), dL = __shfl(sL, (int)(lane & 31) + 32),
                   dR = __shfl(sR, (int)(lane & 31) + 32);
    if (lane == 0) {
      dw[CclDesc::LsF + w] = sF | (dF << 16);
      dw[CclDesc::LsL + w] = sL | (dL << 16);
    }
    if (lane == kCclBW - 1) {
      dw[CclDesc::RsF + w] = sF | (dF << 16);
      dw[CclDesc::RsR + w] = sR | (dR << 16);
    }
    }
    // threshold bytes (127 outside the image): rows 0 and 31, columns 0 and 63
    auto row4 = [&](int r, int c) -> uint32_t {  // (byte reads: the rows start at odd offsets)
      return s_t[r][c] | (s_t[r][c + 1] << 8) | (s_t[r][c + 2] << 16) | ((uint32_t)s_t[r][c + 3] << 24);
    };
    if (tid < 16) {
      dw[CclDesc::Tthr + tid] = row4(1, 1 + 4 * tid);
    } else if (tid < 32) {
      dw[CclDesc::Bthr + tid - 16] = row4(kCclTileH, 1 + 4 * (tid - 16));
    } else if (tid < 48) {
      const int k = tid - 32, c = k < 8 ? 1 : kCclTileW, r = 1 + 4 * (k & 7);
      dw[(k < 8 ? CclDesc::Lthr : CclDesc::Rthr) + (k & 7)] =
          s_t[r][c] | (s_t[r + 1][c] << 8) | (s_t[r + 2][c] << 16) | ((uint32_t)s_t[r + 3][c] << 24);
    }
  }
  __syncthreads();
  ph(9);
  if (tid == 0) {
    b.nlroot[(size_t)f * g.CTX * g.CTY + bi.y * g.CTX + bi.x] = s_nlr;
    kt_end(b, 1);
  }
}

template <int TWD, int PRE>
__global__ __launch_bounds__(CclTile<TWD>::NT) __attribute__((amdgpu_num_sgpr(AT_THR_SGPRS))) void k_thr_ccl(DevBufs b, Geom g, Params prm) {
  thr_ccl_tile<TWD, PRE>(b, g, prm, xcd_block<AT_XCD_THR>());
}

// ---------------------------------------------------------------------------
// K4: unions across CCL tile borders.  One wave per tile: lanes 0-15 own the
// tile's top block row (P, Q, R, bg Q), lanes 16-31 its left block column
// (S, bg S, P for rows >= 1), lanes 32-46 its right column (R for rows >= 1).
// Global union-find with atomicMin links to the smaller id; stale reads are
// tolerated because every link is decided by the atomic's return value.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t g_load(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ uint32_t g_find(uint32_t* par, uint32_t n) {
  uint32_t p = g_load(par + n);
  while (p != n) {
    n = p;
    p = g_load(par + n);
  }
  return n;
}
__device__ void g_union(uint32_t* par, uint32_t a, uint32_t b) {
  while (true) {
    a = g_find(par, a);
    b = g_find(par, b);
    if (a == b) return;
    if (a < b) {
      const uint32_t old = atomicMin(par + b, a);
      if (old == b) return;
      b = old;
    } else {
      const uint32_t old = atomicMin(par + a, b);
      if (old == a) return;
      a = old;
    }
  }
}

// Union of the components of a and b with both finds advanced in lockstep (their
// loads issued together), links by atomicMin to the smaller id as in g_union.
__device__ void g_union2(uint32_t* par, uint32_t a, uint32_t b) {
  while (true) {
    uint32_t pa = g_load(par + a), pb = g_load(par + b);
    while (pa != a || pb != b) {
      a = pa;
      b = pb;
      pa = g_load(par + a);
      pb = g_load(par + b);
    }
    if (a == b) return;
    if (a < b) {
      const uint32_t old = atomicMin(par + b, a);
      if (old == b) return;
      b = old;
    } else {
      const uint32_t old = atomicMin(par + a, b);
      if (old == a) return;
      a = old;
    }
  }
}

// Candidate cross-tile union t (0 .. BorderRoles::NT) of CCL tile (tx, ty) of frame
// f: the reference's Merge test on the threshold plane, then a global union.
template <int TWD>
__device__ __forceinline__ void border_candidate(const DevBufs& b, const Geom& g, int f, int tx, int ty, int t) {
  constexpr int kBorderTop = BorderRoles<TWD>::Top, kBorderLeft = BorderRoles<TWD>::Left,
                kBorderRight = BorderRoles<TWD>::Right;
  constexpr int kCclBW = CclTile<TWD>::BW, kCclBH = CclTile<TWD>::BH;
  int bty = 0, btx = 0, role = 3, kind = 0;  // role 3: no candidate (padding threads)
  if (t < kBorderTop) { role = 0; bty = 0; btx = t / 5; kind = t % 5; }
  else if (t < kBorderTop + kBorderLeft) { role = 1; bty = (t - kBorderTop) / 3; btx = 0; kind = (t - kBorderTop) % 3; }
  else if (t < kBorderTop + kBorderLeft + kBorderRight) {
    role = 2; bty = t - (kBorderTop + kBorderLeft) + 1; btx = kCclBW - 1; kind = 0;
  }
  const int BY = ty * kCclBH + bty, BX = tx * kCclBW + btx;
  if (BY >= g.BH || BX >= g.BW) role = 3;
  const uint8_t* thr = b.thr + (size_t)f * g.Wd * g.Hd;
  uint32_t* par = b.par + (size_t)f * g.Wd * g.Hd;
  const int Wd = g.Wd;
  const int row = 2 * BY, col = 2 * BX;
  const size_t idx = (size_t)row * Wd + col;
  auto px = [&](int r, int c) -> uint8_t {
    if (r < 0 || c < 0 || r >= g.Hd || c >= g.Wd) return 127;
    return thr[(size_t)r * Wd + c];
  };
  const bool act = role != 3;  // (no loads outside the image for the padding threads)
  const uint8_t a = act ? thr[idx] : 127, bb = act ? thr[idx + 1] : 127, c = act ? thr[idx + Wd] : 127;
  // nodes of this block and of its neighbours: F -/+ 1 (left / right), -/+ P (block row
  // above / below), L - 1 = the left block's R
  const uint32_t P = 3 * (uint32_t)g.BW;
  const uint32_t F = node_F(g, BY, BX), L = node_L(g, BY, BX), R = L + 1;
  uint32_t u = 0, v = 0;
  bool link = false;
  if (role == 0 && BY > 0) {
    if (kind == 0) { link = a == 255 && px(row - 1, col - 1) == 255; u = F; v = F - P - 1; }
    else if (kind == 1) {
      link = (a == 255 || bb == 255) && (px(row - 1, col) == 255 || px(row - 1, col + 1) == 255);
      u = F; v = F - P;
    }
    else if (kind == 2) { link = bb == 255 && px(row - 1, col + 2) == 255; u = F; v = F - P + 1; }
    else if (kind == 3) { link = a == 0 && px(row - 1, col) == 0; u = L; v = L - P; }
    else { link = bb == 0 && px(row - 1, col + 1) == 0; u = R; v = R - P; }
  } else if (role == 1 && BX > 0) {
    if (kind == 0) { link = BY > 0 && bty > 0 && a == 255 && px(row - 1, col - 1) == 255; u = F; v = F - P - 1; }
    else if (kind == 1) {
      link = (a == 255 || c == 255) && (px(row, col - 1) == 255 || px(row + 1, col - 1) == 255);
      u = F; v = F - 1;
    } else {
      link = (a == 0 && px(row, col - 1) == 0) || (c == 0 && px(row + 1, col - 1) == 0);
      u = L; v = L - 1;
    }
  } else if (role == 2 && BY > 0) {
    link = bb == 255 && px(row - 1, col + 2) == 255; u = F; v = F - P + 1;
  }
  if (link) g_union2(par, u, v);
}

// latency mode: one workgroup per CCL tile, one thread per candidate
template <int TWD>
__global__ __launch_bounds__(BorderRoles<TWD>::NT) void k_ccl_border(DevBufs b, Geom g) {
  kt_begin(b, 2);
  border_candidate<TWD>(b, g, blockIdx.z, blockIdx.x, blockIdx.y, threadIdx.x);
  if (b.kt_stage == 2) {  // (uniform: the timed launch only)
    __syncthreads();
    if (threadIdx.x == 0) kt_end(b, 2);
  }
}

// ---------------------------------------------------------------------------
// K5: component roots and sizes (FinalLabeling, :340-462, for the roots only).
// One wave per CCL tile, over the tile's local roots: find the global root
// (the minimum node id of the component), point the local root straight at it
// and move the local pixel count there.  Every node then reaches its label in
// two hops -- node -> local root (k_thr_ccl) -> root -- which k_boundary
// follows itself: there is no label plane.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_ccl_roots(DevBufs b, Geom g) {
  const int f = blockIdx.y;
  const size_t tl = (size_t)f * g.CTX * g.CTY + blockIdx.x;
  const size_t fo = (size_t)f * g.Wd * g.Hd;
  uint32_t* par = b.par + fo;
  uint32_t* size = b.size + fo;
  const uint32_t n = b.nlroot[tl];
  const uint32_t* lr = b.lroot + tl * kCclTileNodesMax;
  for (uint32_t k = threadIdx.x; k < n; k += 64) {
    const uint32_t l = lr[k];
    const uint32_t r = g_find(par, l);
    if (r != l) {
      par[l] = r;  // unions are over: a concurrent find sees the old parent or r, both lead to r
      const uint32_t cnt = size[l];
      atomicAdd(size + r, cnt);  // result unused: no round trip (size[l] is dead from here on)
    }
  }
}

// ---------------------------------------------------------------------------
// K4+K5 in one workgroup per frame (throughput mode): the cross-tile merge of
// the CCL (the reference's Merge across tiles and FinalLabeling's roots,
// labeling_allegretti_2019_BKE.cu:302-462) on the frame's listed local roots --
// the tile-local roots of components that reach a tile border, ~40 per tile --
// held in LDS.  Each listed root is a union-find node keyed (gid << 32 | slot):
// linking to the smaller key links to the smaller node id, so a component's root
// is its minimum node id, the reference's label.  The unions are k_ccl_border's
// candidate links (the same tests on the threshold plane); a node's slot is two
// hops away (node -> local root, whose word k_thr_ccl set to kListBit | list
// slot).  Then every listed root's word becomes root | kept (>= 25 pixels) and
// the root's count its component's size (k_boundary then reads label and size
// test in the same two hops and never touches the size plane).
// A frame with more listed roots than the LDS holds is merged by the same
// workgroup in global memory (k_ccl_border's unions, k_ccl_roots' pass, the kept
// bits; ccl_ovf set).
// ---------------------------------------------------------------------------
constexpr int kMergeList = 64;  // link pairs per wave list (k_ccl_merge)
constexpr int kMergePer = (kMergeCapMax + 1023) / 1024;  // listed roots per thread
constexpr int kMergeItems = 2;                          // border blocks per thread per pass

__device__ __forceinline__ uint32_t lcnt_of(const DevBufs& b, int f, int ntl, int t, uint32_t k) {
  return b.lcnt[((size_t)f * ntl + t) * kCclTileNodesMax + k];
}
// (keys change under other threads' atomics: every read is a relaxed atomic load,
// which the compiler may not reuse across iterations)
__device__ __forceinline__ uint64_t key_load(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t merge_find(uint64_t* key, uint32_t i) {
  uint64_t p = key_load(key + i);
  while ((uint32_t)p != i) {
    const uint64_t gp = key_load(key + (uint32_t)p);
    if ((uint32_t)gp != (uint32_t)p) atomicMin((unsigned long long*)&key[i], (unsigned long long)gp);  // halving
    i = (uint32_t)p;
    p = gp;
  }
  return i;
}

__device__ __forceinline__ void merge_union(uint64_t* key, uint32_t a, uint32_t c) {
  while (true) {
    a = merge_find(key, a);
    c = merge_find(key, c);
    if (a == c) return;
    const uint64_t ka = key_load(key + a), kc = key_load(key + c);  // roots: their own (gid << 32 | slot)
    // linked meanwhile (a key names its slot only while it is a root): find again;
    // a link succeeds only over the root's own key
    if ((uint32_t)ka != a || (uint32_t)kc != c) continue;
    if (ka < kc) {
      const uint64_t old = atomicMin((unsigned long long*)&key[c], (unsigned long long)ka);
      if (old == kc) return;
      c = (uint32_t)old;  // c was linked meanwhile: join a with its new parent
    } else {
      const uint64_t old = atomicMin((unsigned long long*)&key[a], (unsigned long long)kc);
      if (old == ka) return;
      a = (uint32_t)old;
    }
  }
}

template <int TWD>
__global__ __launch_bounds__(1024) void k_ccl_merge(DevBufs b, Geom g, Params prm) {
  using CT = CclTile<TWD>;
  constexpr int kBW = CT::BW, kBH = CT::BH;
  // LDS laid out by the frame's number of listed roots (total): parent keys (gid << 32 |
  // slot) and, when 12 B per root fit (up to 12,799 roots: 1080p stream frames list
  // ~11 k), the pixel counts -- the roots are then visited a wave per tile, so no slot
  // needs its tile; a frame whose counts do not fit (1080p noise) keeps the tile of each
  // slot and sums the counts in the size plane at L2 instead (10 B per root: up to
  // 15,360 roots).  (Counts at L2 for the ~11 k roots of a 1080p stream frame: the
  // root-word pass read them back at 53 us per frame, profiles/r06c.)
  extern __shared__ uint64_t s_key[];          // [total] parent key
  uint16_t* s_tile = nullptr;                  // [total] tile of each slot (!cnt_lds)
  uint32_t* s_cnt = nullptr;                   // [total] pixel counts (cnt_lds)
  __shared__ uint32_t s_base[kMaxCclTiles + 1];
  __shared__ uint32_t s_wsum[16];
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  kt_begin(b, 2);
  // AT_PHASE_PROBE: frame 0's phase clocks in probe[40 + k]
  auto stamp = [&](int k) {
    if (AT_PROBE_ON(prm) && f == 0 && tid == 0) b.probe[40 + k] = wall_clock64();
  };
  stamp(0);
  const int ntl = g.CTX * g.CTY;
  const size_t fo = (size_t)f * g.Wd * g.Hd;
  uint32_t* par = b.par + fo;
  uint32_t* size = b.size + fo;
  const uint32_t* lroot = b.lroot + (size_t)f * ntl * kCclTileNodesMax;
  // (0) list sizes -> slot bases, and the tile of every slot
  const uint32_t nt = tid < ntl ? b.nlroot[(size_t)f * ntl + tid] : 0u;
  uint32_t total = 0;
  const uint32_t incl = block_incl_scan(nt, s_wsum, &total, 16);
  if (tid < ntl) s_base[tid] = incl - nt;
  if (tid == 0) {
    s_base[ntl] = total;
    b.nlr_tot[f] = total;
  }
  const bool fits = total <= (uint32_t)g.merge_cap;
  const bool cnt_lds = (size_t)total * 12 + 4 <= (size_t)g.merge_lds;
  s_tile = reinterpret_cast<uint16_t*>(s_key + total);
  s_cnt = reinterpret_cast<uint32_t*>(s_key + total);
  __syncthreads();  // s_base complete
  if (fits && !cnt_lds)
    for (int t = tid >> 6; t < ntl; t += 16) {  // a wave per tile
      const uint32_t b0 = s_base[t], n = s_base[t + 1] - b0;
      for (uint32_t k = lane_id(); k < n; k += 64) s_tile[b0 + k] = (uint16_t)t;
    }
  __syncthreads();
  if (!fits) {
    // more listed roots than the LDS holds (fine checkers, noise): the same merge in
    // global memory by this workgroup -- k_ccl_border's unions (atomicMin links on the
    // parent words), then k_ccl_roots' pass and the kept bits over the lists.  Slow
    // (one workgroup for the frame) but rare; the frame's result is the same.
    for (int t = tid >> 6; t < ntl; t += 16) {  // plain root words and local counts back first
      const uint32_t n = s_base[t + 1] - s_base[t];
      for (uint32_t k = lane_id(); k < n; k += 64) {
        const uint32_t l = lroot[(size_t)t * kCclTileNodesMax + k];
        par[l] = l;
        size[l] = lcnt_of(b, f, ntl, t, k);  // (k_thr_ccl writes the plane for the taps only)
      }
    }
    if (tid == 0) b.ccl_ovf[f] = 1u;
    __threadfence();
    __syncthreads();
    constexpr int kNR = BorderRoles<TWD>::NT;
    for (int j = tid; j < ntl * kNR; j += 1024) {
      const int t = j / kNR;
      border_candidate<TWD>(b, g, f, t % g.CTX, t / g.CTX, j % kNR);
    }
    __threadfence();
    __syncthreads();
    for (int t = tid >> 6; t < ntl; t += 16) {  // roots: local root -> component root, counts to it
      const uint32_t n = s_base[t + 1] - s_base[t];
      for (uint32_t k = lane_id(); k < n; k += 64) {
        const uint32_t l = lroot[(size_t)t * kCclTileNodesMax + k];
        const uint32_t r = g_find(par, l);
        if (r != l) {
          par[l] = r;
          atomicAdd(size + r, lcnt_of(b, f, ntl, t, k));
        }
      }
    }
    __threadfence();
    __syncthreads();
    for (int t = tid >> 6; t < ntl; t += 16) {  // kept bit
      const uint32_t n = s_base[t + 1] - s_base[t];
      for (uint32_t k = lane_id(); k < n; k += 64) {
        const uint32_t l = lroot[(size_t)t * kCclTileNodesMax + k];
        const uint32_t r = g_load(par + l);
        par[l] = r | (g_load(size + r) >= 25 ? kKeptBit : 0u);
      }
    }
    if (b.kt_stage == 2) {
      __syncthreads();
      if (tid == 0) kt_end(b, 2);
    }
    return;
  }
  stamp(1);
  // (1) the listed roots: node id and local pixel count (k_thr_ccl's lists)
  const uint32_t* lcnt = b.lcnt + (size_t)f * ntl * kCclTileNodesMax;
  uint32_t mg[kMergePer];
  if (cnt_lds) {  // a wave per tile (slot = tile base + list index)
    for (int t = tid >> 6; t < ntl; t += 16) {
      const uint32_t b0 = s_base[t], n = s_base[t + 1] - b0;
      for (uint32_t k = lane_id(); k < n; k += 64) {
        const size_t e = (size_t)t * kCclTileNodesMax + k;
        s_cnt[b0 + k] = lcnt[e];
        s_key[b0 + k] = ((uint64_t)lroot[e] << 32) | (b0 + k);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kMergePer; j++) {
      const uint32_t i = tid + 1024u * j;
      mg[j] = 0;
      if (i < total) {
        const int t = s_tile[i];
        const size_t e = (size_t)t * kCclTileNodesMax + (i - s_base[t]);
        mg[j] = lroot[e];
        s_key[i] = ((uint64_t)mg[j] << 32) | i;
        size[mg[j]] = lcnt[e];  // the root's own count, summed into below (counts at L2)
      }
    }
    __threadfence();  // (those stores at L2 before any lane's atomicAdd to them)
  }
  __syncthreads();
  stamp(2);
  // (2) the cross-tile links: k_ccl_border's tests on the tiles' border descriptors
  // (CclDesc), items ordered by role so a wave's lanes read neighbouring entries:
  // the top-row blocks of every tile (role 0, vs the tile above), the left-column
  // blocks (role 1, vs the tile to the left), the right-column blocks of rows >= 1
  // (role 2, the up-right diagonal into the tile to the right).  A lane skips a
  // union equal to its left neighbour's (runs along a border link the same pair).
  const uint32_t* desc = b.cdesc + (size_t)f * ntl * CclDesc::kWords;
  auto dbyte = [&](int t, int w, int i) -> uint32_t {  // byte i of the u32 array at word w of tile t
    return (uint32_t)reinterpret_cast<const uint8_t*>(desc + (size_t)t * CclDesc::kWords + w)[i];
  };
  auto dslot = [&](int t, int w, int i) -> uint32_t {
    return (uint32_t)reinterpret_cast<const uint16_t*>(desc + (size_t)t * CclDesc::kWords + w)[i];
  };
  const int n0 = ntl * kBW, n1 = n0 + ntl * kBH, nitems = n1 + ntl * (kBH - 1);
  // a wave's links (ten candidate sites per lane per pass) compacted by ballot into a
  // wave-private list and run with every lane busy, as in k_thr_ccl -- in the dynamic
  // LDS past the roots when it has room (the usual frame), else the sites directly
  const size_t lused = (cnt_lds ? (size_t)total * 12 : (size_t)total * 10) + 7 & ~(size_t)7;
  const bool ulist = fits && lused + (size_t)16 * kMergeList * 8 <= (size_t)g.merge_lds;  // (uniform)
  uint32_t* wl = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(s_key) + lused) + (tid >> 6) * (2 * kMergeList);
  const uint32_t wlane = lane_id();
  uint32_t nl = 0;  // (uniform per wave)
  auto lflush = [&]() {
    wave_sync();
    for (uint32_t i = wlane; i < nl; i += 64) merge_union(s_key, wl[2 * i], wl[2 * i + 1]);
    wave_sync();
    nl = 0;
  };
  for (int j0 = 0; j0 < nitems; j0 += 1024 * kMergeItems) {
    uint32_t su[kMergeItems][5], sv[kMergeItems][5];  // slot pair per link (0xffffffff: none)
#pragma unroll
    for (int q = 0; q < kMergeItems; q++) {
#pragma unroll
      for (int k = 0; k < 5; k++) su[q][k] = sv[q][k] = 0xffffffffu;
      const int j = j0 + tid + 1024 * q;
      if (j >= nitems) continue;
      if (j < n0) {  // top-row block x of tile t vs the bottom row of the tile above
        const int t = j / kBW, x = j % kBW, ty = t / g.CTX, tx = t % g.CTX;
        if (ty == 0 || tx * kBW + x >= g.BW) continue;
        const int ta = t - g.CTX;
        const bool hl = tx > 0, hr = tx + 1 < g.CTX;
        const uint32_t a = dbyte(t, CclDesc::Tthr, 2 * x), bb = dbyte(t, CclDesc::Tthr, 2 * x + 1);
        const uint32_t ul = x > 0 ? dbyte(ta, CclDesc::Bthr, 2 * x - 1) : (hl ? dbyte(ta - 1, CclDesc::Bthr, 2 * kBW - 1) : 127u);
        const uint32_t u0 = dbyte(ta, CclDesc::Bthr, 2 * x), u1 = dbyte(ta, CclDesc::Bthr, 2 * x + 1);
        const uint32_t ur = x + 1 < kBW ? dbyte(ta, CclDesc::Bthr, 2 * x + 2) : (hr ? dbyte(ta + 1, CclDesc::Bthr, 0) : 127u);
        const uint32_t bF = s_base[t], bA = s_base[ta];
        const uint32_t oF = dslot(t, CclDesc::TsF, x), oL = dslot(t, CclDesc::TsL, x), oR = dslot(t, CclDesc::TsR, x);
        if (a == 255 && ul == 255) {  // P: up-left
          const int tv = x > 0 ? ta : ta - 1;
          su[q][0] = bF + oF;
          sv[q][0] = s_base[tv] + dslot(tv, CclDesc::BsF, x > 0 ? x - 1 : kBW - 1);
        }
        if ((a == 255 || bb == 255) && (u0 == 255 || u1 == 255)) {  // Q: up
          su[q][1] = bF + oF;
          sv[q][1] = bA + dslot(ta, CclDesc::BsF, x);
        }
        if (bb == 255 && ur == 255) {  // R: up-right
          const int tv = x + 1 < kBW ? ta : ta + 1;
          su[q][2] = bF + oF;
          sv[q][2] = s_base[tv] + dslot(tv, CclDesc::BsF, x + 1 < kBW ? x + 1 : 0);
        }
        if (a == 0 && u0 == 0) { su[q][3] = bF + oL; sv[q][3] = bA + dslot(ta, CclDesc::BsL, x); }  // bg up (left column)
        if (bb == 0 && u1 == 0) { su[q][4] = bF + oR; sv[q][4] = bA + dslot(ta, CclDesc::BsR, x); }  // bg up (right)
      } else if (j < n1) {  // left-column block y of tile t vs the right column of the tile to the left
        const int t = (j - n0) / kBH, y = (j - n0) % kBH, ty = t / g.CTX, tx = t % g.CTX;
        if (tx == 0 || ty * kBH + y >= g.BH) continue;
        const int tl = t - 1;
        const uint32_t a = dbyte(t, CclDesc::Lthr, 2 * y), c = dbyte(t, CclDesc::Lthr, 2 * y + 1);
        const uint32_t ul = y > 0 ? dbyte(tl, CclDesc::Rthr, 2 * y - 1) : 127u;
        const uint32_t l0 = dbyte(tl, CclDesc::Rthr, 2 * y), l1 = dbyte(tl, CclDesc::Rthr, 2 * y + 1);
        const uint32_t bF = s_base[t], bL = s_base[tl];
        const uint32_t oF = dslot(t, CclDesc::LsF, y), oL = dslot(t, CclDesc::LsL, y);
        if (y > 0 && a == 255 && ul == 255) { su[q][0] = bF + oF; sv[q][0] = bL + dslot(tl, CclDesc::RsF, y - 1); }
        if ((a == 255 || c == 255) && (l0 == 255 || l1 == 255)) { su[q][1] = bF + oF; sv[q][1] = bL + dslot(tl, CclDesc::RsF, y); }
        if ((a == 0 && l0 == 0) || (c == 0 && l1 == 0)) { su[q][2] = bF + oL; sv[q][2] = bL + dslot(tl, CclDesc::RsR, y); }
      } else {  // right-column block y >= 1 of tile t: up-right into the tile to the right
        const int t = (j - n1) / (kBH - 1), y = 1 + (j - n1) % (kBH - 1), ty = t / g.CTX, tx = t % g.CTX;
        if ((tx + 1) * kBW > g.BW || ty * kBH + y >= g.BH || tx + 1 >= g.CTX) continue;
        const uint32_t bb = dbyte(t, CclDesc::Rthr, 2 * y), ur = dbyte(t + 1, CclDesc::Lthr, 2 * y - 1);
        if (bb == 255 && ur == 255) {
          su[q][0] = s_base[t] + dslot(t, CclDesc::RsF, y);
          sv[q][0] = s_base[t + 1] + dslot(t + 1, CclDesc::LsF, y - 1);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < kMergeItems; q++)
#pragma unroll
      for (int k = 0; k < 5; k++) {
        const bool on = su[q][k] != 0xffffffffu && sv[q][k] < (uint32_t)total && su[q][k] < (uint32_t)total;
        const uint32_t pair = on ? (su[q][k] << 16 | sv[q][k]) : 0xffffffffu;
        const uint32_t prev = wave_shr1(pair, 0xfffffffeu);
        if (ulist) {
          const bool act = on && pair != prev;
          const uint64_t m = __ballot(act);
          const uint32_t c = (uint32_t)__popcll(m);
          if (nl + c > (uint32_t)kMergeList) lflush();
          if (act) {
            const uint32_t pos = nl + lanes_below(m);
            wl[2 * pos] = su[q][k];
            wl[2 * pos + 1] = sv[q][k];
          }
          nl += c;
          continue;
        }
        if (on && pair != prev) merge_union(s_key, su[q][k], sv[q][k]);
      }
  }
  if (ulist && nl) lflush();
  __syncthreads();
  stamp(3);
  // (3) component sizes at the roots: in LDS, or (counts not in LDS) every listed non-root
  // adds its local count to the size word of its component's root, which holds the
  // root's own local count (k_thr_ccl)
#pragma unroll
  for (int j = 0; j < kMergePer; j++) {
    const uint32_t i = tid + 1024u * j;
    if (i < total) {
      const uint32_t r = merge_find(s_key, i);
      if (r != i) {
        if (cnt_lds) {
          atomicAdd(&s_cnt[r], s_cnt[i]);
        } else {
          const int t = s_tile[i];
          atomicAdd(size + (uint32_t)(key_load(s_key + r) >> 32), lcnt[(size_t)t * kCclTileNodesMax + (i - s_base[t])]);
        }
      }
    }
  }
  if (!cnt_lds) __threadfence();  // (the adds done at L2 before any lane reads a size back)
  __syncthreads();
  stamp(4);
  // (4) every listed root's word: root | kept; the root's count: its component's size
  if (cnt_lds) {  // a wave per tile, the node ids read again from the tile's list (L2)
    for (int t = tid >> 6; t < ntl; t += 16) {
      const uint32_t b0 = s_base[t], n = s_base[t + 1] - b0;
      for (uint32_t k = lane_id(); k < n; k += 64) {
        const uint32_t node = lroot[(size_t)t * kCclTileNodesMax + k];
        const uint32_t i = b0 + k;
        const uint32_t r = merge_find(s_key, i);  // (one hop after (3)'s halving, mostly)
        const uint32_t root = (uint32_t)(key_load(s_key + r) >> 32);
        const uint32_t cnt = s_cnt[r];
        par[node] = root | (cnt >= 25 ? kKeptBit : 0u);
        if (prm.taps && r == i) size[node] = cnt;  // (the AT_STAGE_SIZES tap)
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kMergePer; j++) {
      const uint32_t i = tid + 1024u * j;
      if (i < total) {
        const uint32_t r = merge_find(s_key, i);
        const uint32_t root = (uint32_t)(key_load(s_key + r) >> 32);
        par[mg[j]] = root | (g_load(size + root) >= 25 ? kKeptBit : 0u);
      }
    }
  }
  stamp(5);
  if (b.kt_stage == 2) {  // (uniform: the timed launch only)
    __syncthreads();
    if (tid == 0) kt_end(b, 2);
  }
}

// ---------------------------------------------------------------------------
// K6: boundary points (BlobDiff) fused with stream compaction and the pair
// histogram.  Points are appended with one atomic per wave per direction; the
// pair histogram is pre-aggregated over runs of equal pairs in consecutive
// lanes (neighbouring pixels mostly border the same two blobs).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t make_qbp(uint32_t rep0, uint32_t rep1, uint32_t x, uint32_t y, int dxy,
                                             bool b2w) {
  const uint32_t lo = rep0 < rep1 ? rep0 : rep1, hi = rep0 < rep1 ? rep1 : rep0;
  return ((uint64_t)(hi & 0xfffff) << 44) | ((uint64_t)(lo & 0xfffff) << 24) | ((uint64_t)(x & 0x3ff) << 14) |
         ((uint64_t)(y & 0x3ff) << 4) | ((uint64_t)(b2w ? 1 : 0) << 3) | (uint64_t)(dxy & 3);
}

__device__ uint32_t ht_slot_find(const uint64_t* keys, uint64_t key) {
  uint32_t s = (uint32_t)mix_hash(key);
  for (int probe = 0; probe < kHashSlots; probe++) {
    const uint64_t k = keys[s];
    if (k == key) return s;
    if (k == 0) return 0xffffffffu;
    s = (s + 1) & (kHashSlots - 1);
  }
  return 0xffffffffu;
}

__device__ __forceinline__ uint64_t wave_shr1_u64(uint64_t v) {
  return (uint64_t)wave_shr1((uint32_t)v, 0) | ((uint64_t)wave_shr1((uint32_t)(v >> 32), 0) << 32);
}


// slot hash of a pair key in the tile's LDS table: the low word (the smaller label and
// 12 bits of the larger) times a 32-bit golden-ratio constant, top 9 bits -- one
// v_mul_lo_u32 instead of the 64-bit product (AT_BND_HASH32=0: the frame table's hash)
#ifndef AT_BND_HASH32
#define AT_BND_HASH32 1
#endif
__device__ __forceinline__ uint32_t pair_hash(uint64_t key) {
  static_assert(kLdsPairSlots == 512, "9-bit slot hash");
  if (AT_BND_HASH32) return ((uint32_t)key * 0x9E3779B1u) >> 23;
  return (uint32_t)(mix_hash(key) & (kLdsPairSlots - 1));
}
__device__ __forceinline__ bool lds_pair_add(uint64_t* keys, uint32_t* cnts, uint64_t key, uint32_t len) {
  uint32_t h = pair_hash(key);
  for (int probe = 0; probe < kLdsPairSlots; probe++) {
    const uint64_t k = keys[h];
    if (k == key) {
      atomicAdd(cnts + h, len);
      return true;
    }
    if (k == 0) {
      const uint64_t prev = atomicCAS((unsigned long long*)(keys + h), 0ull, (unsigned long long)key);
      if (prev == 0 || prev == key) {
        atomicAdd(cnts + h, len);
        return true;
      }
    }
    h = (h + 1) & (kLdsPairSlots - 1);
  }
  return false;
}

// slot of a key already in the tile's LDS pair table
__device__ __forceinline__ uint32_t lds_pair_slot(const uint64_t* keys, uint64_t key) {
  uint32_t h = pair_hash(key);
  while (keys[h] != key) h = (h + 1) & (kLdsPairSlots - 1);
  return h;
}

// Narrow tile points (tcnt flag kTileNarrow): 4-B words, the tile's pair-entry
// index (9 bits) over the point bits of the key -- x (10), y (10), b2w, dxy (2):
// the labels are the entry's key (pent_key), so they need not travel per point.
__device__ __forceinline__ uint32_t narrow_point(uint32_t entry, uint64_t key) {
  return (entry << 23) | ((uint32_t)(key >> 1) & 0x7ffffcu) | ((uint32_t)key & 3u);
}
// ... and back to the low 24 key bits (x << 14 | y << 4 | b2w << 3 | dxy)
__device__ __forceinline__ uint32_t narrow_bits(uint32_t w) { return ((w & 0x7ffffcu) << 1) | (w & 3u); }

// One 256-thread workgroup covers a 64 x (4*kBndRows) tile of interior pixels.
// Points are staged in LDS (wave-aggregated LDS atomics) and written out with
// ONE global atomic per workgroup; the pair histogram is aggregated in an LDS
// hash table (runs of equal pairs in consecutive lanes first) and appended to
// the frame's pair-entry list with one more global atomic per workgroup.

__device__ __forceinline__ void bnd_spill(const DevBufs& b, int f, uint64_t key, uint32_t cnt) {
  const uint32_t o = atomicAdd(b.npent + f, 1u);
  if (o < (uint32_t)kPairEntCap) {
    b.povf_key[(size_t)f * kPairEntCap + o] = key;
    b.povf_cnt[(size_t)f * kPairEntCap + o] = cnt;
  } else {
    atomicOr(b.status + f, kStatusHashFull);
  }
}

// SGPR budget (experiment builds: -DAT_BND_SGPRS=N): at .sgpr_count 106 a CU admits
// 6 of these 4-wave workgroups (800 / (112 + 16)); capped at 80 it admits 8 (the
// 19.5 KB of LDS allows 8 too): k_boundary 0.250 -> 0.236 ms per 128 frames
// serialized, but 2 % less concurrent throughput -- eight workgroups take a CU's
// whole LDS from the other batches' kernels (profiles/r04d/ab_sgpr_caps_stages.txt)
#ifdef AT_BND_SGPRS
#define AT_BND_ATTR __attribute__((amdgpu_num_sgpr(AT_BND_SGPRS)))
#else
#define AT_BND_ATTR
#endif
// KEPT (throughput mode): the size test comes with the root word (k_ccl_merge);
// latency mode skips that kernel and reads the size plane (one more round trip
// here, one launch less on the chain)
template <bool KEPT>
__global__ __launch_bounds__(256) AT_BND_ATTR void k_boundary(DevBufs b, Geom g) {
  __shared__ uint64_t s_pkey[kLdsPairSlots];
  __shared__ uint32_t s_pcnt[kLdsPairSlots];
  // points staged in LDS up to kBndStage (typical tiles hold ~0.7 points per
  // pixel); the rare denser tile writes the excess straight to its global
  // region.  Keeping the stage small keeps 6 workgroups (24 waves) per CU.
  __shared__ uint64_t s_pts[kBndStage];
  __shared__ uint32_t s_npts, s_nent, s_spill;
  // threshold values with pixels of blobs under 25 pixels folded to 127: every
  // BlobDiff condition then reads one byte per neighbour (v0 + v1 == 255 holds
  // only when both blobs are kept; the dedup rule's "!= 127 and kept" likewise)
  __shared__ __attribute__((aligned(4))) uint8_t s_tthr[(4 * kBndRows + 1) * 66];
  __shared__ uint32_t s_tlab[(4 * kBndRows + 1) * 66];
  const TileIdx bi = xcd_block<AT_XCD_BND>();
  const int f = bi.z;
  const int tid = threadIdx.y * 64 + threadIdx.x;
  kt_begin(b, 4);
  for (int i = tid; i < kLdsPairSlots; i += 256) {
    s_pkey[i] = 0;
    s_pcnt[i] = 0;
  }
  if (tid == 0) { s_npts = 0; s_nent = 0; s_spill = 0; }
  // stage the tile's threshold values and labels (+1 halo: rows y0..y0+16, cols
  // x0-1..x0+64) and, per pixel, whether its blob has >= 25 pixels: two
  // dependent global round trips per workgroup, then the point logic runs on LDS
  const size_t fo = (size_t)f * g.Wd * g.Hd;
  const uint8_t* thr = b.thr + fo;
  const uint32_t* par = b.par + fo;
  const int Wd = g.Wd;
  const int ty0 = 1 + bi.y * (4 * kBndRows), tx0 = bi.x * 64;  // halo origin: x0 - 1
  constexpr int kTR = 4 * kBndRows + 1, kTC = 66, kTN = kTR * kTC;
  constexpr int kPer = (kTN + 255) / 256;
  // label of a pixel = par[par[node]]: its block node (fg -> F, bg -> L / R by
  // column) -> local root -> component root | kept bit (k_ccl_merge / k_ccl_roots;
  // a local root's own word already holds root | kept, so the second hop masks)
  // (the threshold byte and both candidate nodes' parents are loaded together,
  // the byte then picks fg or bg: one round trip fewer than thr -> node -> parent)
  uint32_t lv[kPer], lb[kPer];
  uint8_t tv[kPer];
  // loads from clamped addresses, selected afterwards (no branch per load)
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const int e = tid + 256 * k, ec = min(e, kTN - 1);  // (lanes past the tile read its last element)
    const int yy = ty0 + ec / kTC, xx = tx0 + ec % kTC;
    const bool in = e < kTN && yy < g.Hd && xx < Wd;
    const int yc = min(yy, g.Hd - 1), xc = min(xx, Wd - 1);
    const uint32_t F = node_F(g, yc >> 1, xc >> 1), LR = node_L(g, yc >> 1, 0) + (uint32_t)xc;
    const uint8_t t = thr[(size_t)yc * Wd + xc];
    const uint32_t a = par[F], c = par[LR];
    tv[k] = in ? t : (uint8_t)127;
    lv[k] = in ? a : 0xffffffffu;
    lb[k] = in ? c : 0xffffffffu;
  }
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    lv[k] = tv[k] == 127 ? 0xffffffffu : (tv[k] == 255 ? lv[k] : lb[k]);
    const uint32_t r = par[lv[k] != 0xffffffffu ? (lv[k] & ~kKeptBit) : 0u];
    lv[k] = lv[k] != 0xffffffffu ? r : 0xffffffffu;
  }
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const int e = tid + 256 * k;
    if (e < kTN) {
      const bool kept = lv[k] != 0xffffffffu && (KEPT ? (lv[k] & kKeptBit) != 0 : b.size[fo + lv[k]] >= 25);
      s_tlab[e] = lv[k] & ~kKeptBit;
      s_tthr[e] = kept ? tv[k] : (uint8_t)127;
    }
  }
  __syncthreads();  // LDS tables initialised
  const uint32_t lane = lane_id();
  const size_t tb = (size_t)f * g.ntb + bi.y * gridDim.x + bi.x;
  uint64_t* pts_out = b.pts + tb * g.bnd_region;
  // two horizontally adjacent pixels per lane, a wave over two tile rows per step
  // (lanes 0-31 the upper row, 32-63 the lower): the wave-wide work of a step -- the
  // point-offset scan, the pair runs, the staging atomic -- serves 128 pixels.  (Pair
  // runs may continue from the upper row into the lower: only their counts are used.)
  const int cx = 2 * (int)(lane & 31);  // tile column of the lane's first pixel
  const int xa = 1 + bi.x * 64 + cx;    // its image column
  for (int r = 0; r < kBndRows / 2; r++) {
    const int ly = (r * 4 + threadIdx.y) * 2 + (int)(lane >> 5);  // tile row of the pixels
    const int y = ty0 + ly;
    // threshold bytes of halo columns cx .. cx+3 (left neighbour, the two pixels, right
    // neighbour) in rows ly and ly + 1: four aligned 16-bit LDS reads
    const int eb = ly * kTC + cx;
    const uint32_t ra = (uint32_t)*reinterpret_cast<const uint16_t*>(s_tthr + eb) |
                        ((uint32_t)*reinterpret_cast<const uint16_t*>(s_tthr + eb + 2) << 16);
    const uint32_t rb = (uint32_t)*reinterpret_cast<const uint16_t*>(s_tthr + eb + kTC) |
                        ((uint32_t)*reinterpret_cast<const uint16_t*>(s_tthr + eb + kTC + 2) << 16);
    // the pixels' points: direction mask (bit 4j + dir for pixel j), neighbour labels
    uint32_t hm = 0, nb[8], rep[2];
    bool b2w[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      rep[j] = 0;
      b2w[j] = false;
#pragma unroll
      for (int d = 0; d < 4; d++) nb[4 * j + d] = 0;
      const uint32_t v0 = (ra >> (8 * j + 8)) & 0xff;
      // branch-free: the five labels read whatever the pixel (the halo holds every
      // address; a label is used only where its direction's bit is set), so no exec-mask
      // region per direction
      const uint32_t vl = (ra >> (8 * j)) & 0xff, vr = (ra >> (8 * j + 16)) & 0xff;
      const uint32_t vdl = (rb >> (8 * j)) & 0xff, vd = (rb >> (8 * j + 8)) & 0xff, vdr = (rb >> (8 * j + 16)) & 0xff;
      const int e0 = eb + j + 1, ed = e0 + kTC;
      const bool pv = xa + j <= g.Wd - 2 && y <= g.Hd - 2 && v0 != 127;
      rep[j] = s_tlab[e0];
      b2w[j] = v0 == 0;
      nb[4 * j] = s_tlab[e0 + 1];
      nb[4 * j + 1] = s_tlab[ed + 1];
      nb[4 * j + 2] = s_tlab[ed];
      nb[4 * j + 3] = s_tlab[ed - 1];
      const bool dedup = vl != 127 && vd != 127 && vd != vl && xa + j != 1;
      const uint32_t pm = (v0 + vr == 255 ? 1u : 0u) | (v0 + vdr == 255 ? 2u : 0u) | (v0 + vd == 255 ? 4u : 0u) |
                          (!dedup && v0 + vdl == 255 ? 8u : 0u);
      hm |= pv ? pm << (4 * j) : 0u;
    }
    // pair histogram: the lane's first pair with the count of its points in it (labels
    // are < 2^20 -- decimated planes of at most 1024 x 1024 -- so label equality is
    // key equality), runs of equal first pairs in consecutive lanes summed (wave scan),
    // the rare other pairs of a lane one by one
    const bool got = hm != 0;
    const uint32_t rf = (hm & 0xfu) ? rep[0] : rep[1];
    uint32_t nf = nb[7];
#pragma unroll
    for (int d = 6; d >= 0; d--) nf = ((hm >> d) & 1) ? nb[d] : nf;
    uint32_t cnt = 0, xm = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
      const uint32_t rj = rep[d >> 2];
      const bool in = (hm >> d) & 1, eq = (rj == rf && nb[d] == nf) || (rj == nf && nb[d] == rf);
      cnt += in && eq;
      xm |= (in && !eq) ? 1u << d : 0u;
    }
    // one scan for both: the first-pair counts (low half) and the lane's points (high)
    const uint32_t npts = (uint32_t)__builtin_popcount(hm);
    const uint32_t sc = wave_incl_scan(cnt | (npts << 16), AddOp(), 0u);
    const uint32_t incl = sc & 0xffffu;
    const uint32_t below = (sc >> 16) - npts, wtot = wave_read(sc, 63) >> 16;
    const uint64_t kp = got ? make_qbp(rf, nf, 0, 0, 0, false) >> 24 : 0ull;
    {
      const uint64_t prev = wave_shr1_u64(kp);
      const bool same = got && lane > 0 && prev == kp;
      const uint64_t same_mask = __ballot(same);
      const bool head = got && !same;
      const uint32_t len = head ? run_len(same_mask, lane) : 1u;
      const uint32_t incl_end = (uint32_t)__shfl((int)incl, (int)(lane + len - 1));
      if (head) {
        const uint32_t tot = incl_end - incl + cnt;
        if (!lds_pair_add(s_pkey, s_pcnt, kp, tot)) {  // LDS table full
          bnd_spill(b, f, kp, tot);
          s_spill = 1;
        }
      }
      if (__ballot(xm != 0)) {
#pragma unroll
        for (int d = 0; d < 8; d++) {
          if ((xm >> d) & 1) {
            const uint64_t k = make_qbp(rep[d >> 2], nb[d], 0, 0, 0, false) >> 24;
            if (!lds_pair_add(s_pkey, s_pcnt, k, 1u)) {
              bnd_spill(b, f, k, 1u);
              s_spill = 1;
            }
          }
        }
      }
    }
    // wave-aggregated append of the points into the LDS staging buffer
    uint32_t wbase = 0;
    if (lane == 0 && wtot) wbase = atomicAdd(&s_npts, wtot);
    wbase = __shfl(wbase, 0);
    uint32_t pos = wbase + below;
    if (wbase + wtot <= (uint32_t)kBndStage) {  // (uniform) the usual step: every point staged
#pragma unroll
      for (int d = 0; d < 8; d++)
        if ((hm >> d) & 1) s_pts[pos++] = make_qbp(rep[d >> 2], nb[d], xa + (d >> 2), y, d & 3, b2w[d >> 2]);
    } else {
#pragma unroll
      for (int d = 0; d < 8; d++)
        if ((hm >> d) & 1) {
          const uint64_t k = make_qbp(rep[d >> 2], nb[d], xa + (d >> 2), y, d & 3, b2w[d >> 2]);
          if (pos < (uint32_t)kBndStage) s_pts[pos] = k;
          else if (pos < (uint32_t)g.bnd_region) pts_out[pos] = k;
          else atomicOr(b.status + f, kStatusPointsOverflow);
          pos++;
        }
    }
  }
  __syncthreads();
  // the tile's own regions: points and compacted pair entries, plain stores
  // (no per-frame counter: a device-scope atomic per tile on a per-frame
  // address serialized the tiles of a frame)
  const uint32_t total = s_npts;
  // narrow tile: every point staged and every pair in the LDS table -> 4-B points
  // carrying their entry index (half the bytes for k_group, which then needs no
  // key lookup); otherwise the 8-B keys
  const bool narrow = total <= (uint32_t)kBndStage && !s_spill;
  uint64_t* ekey = b.pent_key + tb * kLdsPairSlots;
  uint32_t* ecnt = b.pent_cnt + tb * kLdsPairSlots;
  uint32_t* s_ent = s_tlab;  // slot -> entry index (the label table is dead)
  for (int i = tid; i < kLdsPairSlots; i += 256) {
    const uint64_t k = s_pkey[i];
    if (k) {
      const uint32_t o = atomicAdd(&s_nent, 1u);
      ekey[o] = k;
      ecnt[o] = s_pcnt[i];
      s_ent[i] = o;
    }
  }
  if (narrow) {
    __syncthreads();
    uint32_t* out = reinterpret_cast<uint32_t*>(pts_out);
    for (uint32_t i = tid; i < total; i += 256) {
      const uint64_t k = s_pts[i];
      out[i] = narrow_point(s_ent[lds_pair_slot(s_pkey, k >> 24)], k);
    }
  } else {
    const uint32_t staged = total < (uint32_t)kBndStage ? total : (uint32_t)kBndStage;
    for (uint32_t i = tid; i < staged; i += 256) pts_out[i] = s_pts[i];
  }
  __syncthreads();
  if (tid == 0) {
    b.tcnt[tb] = min(total, (uint32_t)g.bnd_region) | (narrow ? kTileNarrow : 0u);
    b.tent[tb] = s_nent;
    kt_end(b, 4);
  }
}

// ---------------------------------------------------------------------------
// K7: rank the pairs of a frame (P2 radix order: rep1 major, rep0 minor ==
// numeric order of rep01), assign each its segment offset, and append the
// pairs whose point count passes the size filter to the global work list.
// One 1024-thread workgroup per frame; bitonic sort in LDS.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int size_class(uint32_t n) {
  if (n > 2048) return 0;
  if (n > 1024) return 1;
  if (n > (uint32_t)kSmallBlob) return 2;
  if (n > 256) return 3;
  if (n > 128) return 4;
  if (n > 64) return 5;
  return 6;
}

template <typename T, int NT>
__device__ void block_bitonic_sort(T* s, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const T a = s[i], c = s[ixj];
          const bool up = (i & k) == 0;
          if ((a > c) == up) {
            s[i] = c;
            s[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

// k_pairs turns the first kGrpEnt entries of every tile into the base slot of
// the tile's points in their pair segment (written over the entry's count), so
// k_group scatters a tile with one load round trip; kGrpDrop marks pairs outside
// the size bounds, kGrpFallback entries whose points reserve one slot each.
constexpr int kGrpEnt = 128;  // tile entries with an LDS cursor in k_group (typical tiles: ~10)
constexpr uint32_t kGrpDrop = 0xfffffffeu, kGrpFallback = 0xffffffffu;
constexpr int kPairsEntCache = 4;  // entries per thread whose hash slot k_pairs keeps in registers

__global__ __launch_bounds__(1024) void k_pairs(DevBufs b, Geom g, int probe) {
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  auto stamp = [&](int i) {
    if (probe && f == 0 && tid == 0) b.probe[i] = wall_clock64();
  };
  stamp(0);
  __shared__ uint64_t t_key[kHashSlots];
  __shared__ uint32_t t_cnt[kHashSlots];
  // the frame's pair list, sorted, lives in t_key's storage once the lookup table
  // is out (54 KB of LDS instead of 86 KB: the batches in flight co-reside better)
  uint64_t* s_list = t_key;
  static_assert(kMaxPairs <= kHashSlots, "the pair list fits in the hash table's storage");
  __shared__ uint32_t s_n, s_full, s_np;
  __shared__ uint32_t s_wsum[16];
  for (int i = tid; i < kHashSlots; i += 1024) {
    t_key[i] = 0;
    t_cnt[i] = 0;
  }
  if (tid == 0) { s_n = 0; s_full = 0; s_np = 0; }
  __syncthreads();
  // merge the per-tile pair histograms of k_boundary in LDS: wave w takes
  // tiles w, w + 16, ...; then the overflow entries of crowded tiles
  auto merge = [&](uint64_t key, uint32_t cnt) -> uint32_t {
    uint32_t h = (uint32_t)mix_hash(key) & (kHashSlots - 1);
    for (int probe = 0; probe < kHashSlots; probe++) {
      const uint64_t k = t_key[h];
      if (k == key) {
        atomicAdd(&t_cnt[h], cnt);
        return h;
      } else if (k == 0) {
        const uint64_t prev = atomicCAS((unsigned long long*)&t_key[h], 0ull, (unsigned long long)key);
        if (prev == 0 || prev == key) {
          atomicAdd(&t_cnt[h], cnt);
          return h;
        }
      }
      h = (h + 1) & (kHashSlots - 1);
    }
    s_full = 1;
    return 0xffffffffu;
  };
  // the first kPairsEntCache * 1024 tile entries of the flat pass: hash slot,
  // count and global index (for the segment bases written at the end)
  uint32_t c_slot[kPairsEntCache], c_cnt[kPairsEntCache], c_idx[kPairsEntCache];
  bool c_lds[kPairsEntCache];
  __shared__ uint32_t s_tpre[kMaxTilesPerFrame + 1];
  uint32_t tot_e = 0;
  const int ntb = g.ntb;
  uint32_t novf = 0;
  {
    // tile entry counts -> exclusive prefix in LDS (one load round trip), then
    // every entry of the frame in one flat pass
    // thread t owns tile t (ntb <= kMaxTilesPerFrame = 1024)
    const uint32_t ne = tid < ntb ? b.tent[(size_t)f * ntb + tid] : 0u;
    const uint32_t np = tid < ntb ? b.tcnt[(size_t)f * ntb + tid] & ~kTileNarrow : 0u;
    const uint32_t incl_e = block_incl_scan(ne, s_wsum, &tot_e, 16);
    if (tid < ntb) s_tpre[tid] = incl_e - ne;
    if (tid == 0) s_tpre[ntb] = tot_e;
    if (np) atomicAdd(&s_np, np);
    novf = min(b.npent[f], (uint32_t)kPairEntCap);
    __syncthreads();
  }
  // entry i of the frame's flat list: (global index, index within its tile)
  auto entry = [&](uint32_t i, uint32_t* et) -> size_t {
    int lo = 0, hi = ntb - 1;  // last tile whose prefix <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_tpre[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    *et = i - s_tpre[lo];
    return ((size_t)f * ntb + lo) * kLdsPairSlots + *et;
  };
  // one pass over every entry of the frame, merging the keys below `limit`
  auto merge_pass = [&](uint64_t limit) {
#pragma unroll
    for (int k = 0; k < kPairsEntCache; k++) { c_slot[k] = 0xffffffffu; c_cnt[k] = 0; c_idx[k] = 0; c_lds[k] = false; }
    {
      // the thread's first kPairsEntCache entries: every index first, then every
      // load, then the merges (one global round trip for all of them)
      uint32_t et[kPairsEntCache], cnt[kPairsEntCache];
      uint64_t key[kPairsEntCache];
      size_t e[kPairsEntCache];
#pragma unroll
      for (int k = 0; k < kPairsEntCache; k++) {
        const uint32_t i = tid + 1024u * k;
        e[k] = i < tot_e ? entry(i, &et[k]) : 0;
      }
#pragma unroll
      for (int k = 0; k < kPairsEntCache; k++) {
        const bool in = tid + 1024u * k < tot_e;
        cnt[k] = in ? b.pent_cnt[e[k]] : 0u;
        key[k] = in ? b.pent_key[e[k]] : 0ull;
      }
#pragma unroll
      for (int k = 0; k < kPairsEntCache; k++) {
        if (tid + 1024u * k >= tot_e) continue;
        c_slot[k] = key[k] < limit ? merge(key[k], cnt[k]) : 0xffffffffu;
        c_cnt[k] = cnt[k];
        c_idx[k] = (uint32_t)e[k];
        c_lds[k] = et[k] < (uint32_t)kGrpEnt;
      }
    }
    for (uint32_t i = tid + 1024u * kPairsEntCache; i < tot_e; i += 1024) {  // (crowded frames)
      uint32_t et;
      const size_t e = entry(i, &et);
      const uint64_t key = b.pent_key[e];
      if (key < limit) merge(key, b.pent_cnt[e]);
    }
    for (uint32_t i = tid; i < novf; i += 1024) {
      const uint64_t key = b.povf_key[(size_t)f * kPairEntCap + i];
      if (key < limit) merge(key, b.povf_cnt[(size_t)f * kPairEntCap + i]);
    }
    __syncthreads();
  };
  merge_pass(~0ull);
  bool capped = false;
  if (s_full) {
    // More than kMaxPairs pairs (the 12-bit blob index, points.h:183-193; the
    // reference overflows its 2048-entry extents buffer here, apriltag_gpu.cu:129,
    // 899-902): keep exactly the first kMaxPairs pairs in rank order (rep01
    // ascending) -- the largest limit T below which the frame has at most kMaxPairs
    // distinct keys, by bisection with the LDS table as the distinct counter --
    // and flag the frame (kStatusPairsCapped: AT_E_CAPACITY with its detections).
    capped = true;
    uint64_t lo = 0, hi = 1ull << 40;  // ok(lo), !ok(hi)
    while (hi - lo > 1) {
      const uint64_t mid = lo + ((hi - lo) >> 1);
      for (int i = tid; i < kHashSlots; i += 1024) { t_key[i] = 0; t_cnt[i] = 0; }
      if (tid == 0) s_full = 0;
      __syncthreads();
      for (uint32_t i = tid; i < tot_e; i += 1024) {
        uint32_t et;
        const uint64_t key = b.pent_key[entry(i, &et)];
        if (key < mid && !s_full) merge(key, 1u);
      }
      for (uint32_t i = tid; i < novf; i += 1024) {
        const uint64_t key = b.povf_key[(size_t)f * kPairEntCap + i];
        if (key < mid && !s_full) merge(key, 1u);
      }
      __syncthreads();
      const bool ok = !s_full;
      __syncthreads();
      if (ok) lo = mid;
      else hi = mid;
    }
    for (int i = tid; i < kHashSlots; i += 1024) { t_key[i] = 0; t_cnt[i] = 0; }
    if (tid == 0) s_full = 0;
    __syncthreads();
    merge_pass(lo);
  }
  // tile entries beyond the register cache that k_group would look up in LDS:
  // their points reserve per point (kGrpFallback) -- written after the merge
  // passes, which read the counts
  for (uint32_t i = tid + 1024 * kPairsEntCache; i < tot_e; i += 1024) {
    uint32_t et;
    const size_t e = entry(i, &et);
    if (et < (uint32_t)kGrpEnt) b.pent_cnt[e] = kGrpFallback;
  }
  __syncthreads();
  if (tid == 0) {
    b.npts[f] = s_np;           // boundary points of the frame (N_c)
    b.npent[f] = tot_e + novf;  // entries merged (diagnostic)
    if (capped) atomicOr(b.status + f, kStatusPairsCapped);
  }
  __syncthreads();
  stamp(1);
  // the lookup table used by k_group (keys of every slot, 0 = empty), then the
  // occupied slots listed over t_key's storage
  static_assert(kHashSlots == 4 * 1024, "four hash slots per thread");
  uint64_t kreg[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int s = tid + 1024 * k;
    kreg[k] = t_key[s];
    b.ht_key[(size_t)f * kHashSlots + s] = kreg[k];
    b.ht_cnt[(size_t)f * kHashSlots + s] = t_cnt[s];
  }
  __syncthreads();  // every t_key read before the list overwrites it
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (kreg[k]) {
      const uint32_t i = atomicAdd(&s_n, 1u);
      if (i < kMaxPairs) s_list[i] = (kreg[k] << kHashBits) | (uint64_t)(tid + 1024 * k);
    }
  }
  __syncthreads();
  const uint32_t n = s_n;
  if (tid == 0) b.npairs[f] = n;
  if (n > (uint32_t)kMaxPairs || s_full) {
    if (tid == 0) atomicOr(b.status + f, s_full ? kStatusHashFull : kStatusPairsOverflow);
    return;
  }
  int np2 = 64;
  while (np2 < (int)n) np2 <<= 1;
  for (int i = (int)n + tid; i < np2; i += 1024) s_list[i] = ~0ull;
  __syncthreads();
  stamp(2);
  if (n <= 1024) {
    // rank sort (keys are unique: the slot rides in the low bits), the list in
    // t_key[0, n), the ranked copy in t_key[1024, 1024 + n), the ranks after it.
    // P = 1024 / n threads per key, each counting the smaller keys of a 1/P slice
    // of the list (a frame's ~400 pairs: 2 threads per key, half the serial LDS reads)
    const int P = (int)(1024 / (n ? n : 1u));
    uint32_t* s_rank = reinterpret_cast<uint32_t*>(t_key + 2048);
    if (tid < (int)n) s_rank[tid] = 0;
    __syncthreads();
    if (tid < P * (int)n) {
      const int i = tid % (int)n, h = tid / (int)n;
      const uint64_t key = s_list[i];
      const int j1 = (int)(((uint32_t)h + 1) * n / (uint32_t)P);
      int j = (int)((uint32_t)h * n / (uint32_t)P);
      uint32_t r = 0;
      for (; j + 4 <= j1; j += 4)
        r += (s_list[j] < key) + (s_list[j + 1] < key) + (s_list[j + 2] < key) + (s_list[j + 3] < key);
      for (; j < j1; j++) r += s_list[j] < key;
      if (r) atomicAdd(&s_rank[i], r);
    }
    __syncthreads();
    if (tid < (int)n) t_key[1024 + s_rank[tid]] = s_list[tid];
    __syncthreads();
    if (tid < (int)n) s_list[tid] = t_key[1024 + tid];
    __syncthreads();
  } else {
    block_bitonic_sort<uint64_t, 1024>(s_list, np2);
  }
  stamp(3);
  // counts in rank order (straight from the hash slots), exclusive scan -> offsets;
  // each thread owns 4 consecutive ranks, whose hash slots it keeps in registers
  // (t_key's storage is reused for the segment cursors below)
  const int i0 = tid * 4;
  uint32_t lslt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) lslt[k] = i0 + k < (int)n ? (uint32_t)(s_list[i0 + k] & (kHashSlots - 1)) : 0u;
  auto cnt_at = [&](int k) -> uint32_t { return i0 + k < (int)n ? t_cnt[lslt[k]] : 0u; };
  const uint32_t c0 = cnt_at(0), c1 = cnt_at(1), c2 = cnt_at(2), c3 = cnt_at(3);
  const uint32_t tsum = c0 + c1 + c2 + c3;
  const uint32_t incl = wave_incl_scan(tsum, AddOp(), 0u);
  const uint32_t lane = lane_id();
  if (lane == 63) s_wsum[tid >> 6] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (int w = 0; w < (tid >> 6); w++) wbase += s_wsum[w];
  const uint32_t excl = wbase + incl - tsum;
  const uint32_t offs[4] = {excl, excl + c0, excl + c0 + c1, excl + c0 + c1 + c2};
  const uint32_t cs[4] = {c0, c1, c2, c3};
  stamp(4);
  // work-list appends by size class: LDS slots, then one global atomic per
  // class per workgroup
  __shared__ uint32_t s_ccnt[kNumCls], s_cbase[kNumCls];
  __syncthreads();  // s_n / s_full / s_wsum reads done
  if (tid < kNumCls) s_ccnt[tid] = 0;
  __syncthreads();
  int cls[4];
  uint32_t lslot[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    cls[k] = -1;
    lslot[k] = 0;
    if (i0 + k < (int)n && cs[k] >= g.min_cluster && cs[k] <= g.max_cluster) {
      cls[k] = size_class(cs[k]);
      lslot[k] = atomicAdd(&s_ccnt[cls[k]], 1u);
    }
  }
  __syncthreads();
  if (tid < kNumCls) s_cbase[tid] = s_ccnt[tid] ? atomicAdd(b.ncls + tid, s_ccnt[tid]) : 0u;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = i0 + k;
    if (i < (int)n) {
      const uint32_t slot = lslt[k];
      b.ht_rank[(size_t)f * kHashSlots + slot] = (uint32_t)i;
      b.ht_off[(size_t)f * kHashSlots + slot] = offs[k];
      b.pair_cnt[(size_t)f * kMaxPairs + i] = cs[k];
      b.pair_off[(size_t)f * kMaxPairs + i] = offs[k];
      b.pair_sel[(size_t)f * kMaxPairs + i] = 0;
      if (cls[k] >= 0)
        b.work[(size_t)cls[k] * b.wcap + s_cbase[cls[k]] + lslot[k]] = ((uint32_t)f << 16) | (uint32_t)i;
    }
  }
  // segment bases of the tiles' first kGrpEnt entries (LDS cursors per pair slot;
  // t_key's storage is free since the sort), then the cursors' final values seed
  // k_group's per-point reservations
  uint32_t* t_off = reinterpret_cast<uint32_t*>(t_key);
  uint32_t* t_cur = t_off + kHashSlots;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = i0 + k;
    if (i < (int)n) {
      const uint32_t slot = lslt[k];
      t_off[slot] = offs[k];
      t_cur[slot] = 0;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPairsEntCache; k++) {
    if (c_lds[k] && c_slot[k] != 0xffffffffu) {
      const uint32_t tc = t_cnt[c_slot[k]];
      const bool keep = tc >= g.min_cluster && tc <= g.max_cluster;
      b.pent_cnt[c_idx[k]] = keep ? t_off[c_slot[k]] + atomicAdd(&t_cur[c_slot[k]], c_cnt[k]) : kGrpDrop;
    } else if (c_lds[k]) {
      b.pent_cnt[c_idx[k]] = kGrpDrop;  // a pair past the first kMaxPairs (capped frame)
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = i0 + k;
    if (i < (int)n) {
      const uint32_t slot = lslt[k];
      b.ht_cur[(size_t)f * kHashSlots + slot] = t_cur[slot];
    }
  }
  stamp(5);
}

// ---------------------------------------------------------------------------
// K8: scatter the points into their pair segments (grouped by pair rank).
// ---------------------------------------------------------------------------
// One workgroup per k_boundary tile.  k_pairs has reserved each of the tile's
// first kGrpEnt (tile, pair) entries its range of the pair segment (the entry's
// count word now holds the base, kGrpDrop for pairs outside SelectBlobs' count
// bounds -- P4's size filter: nothing reads their segments); the tile's points
// take consecutive slots of their entry's range (LDS cursor).  The tile's
// counters, its entries and its first 512 points are loaded in ONE round trip
// (speculatively: reads past the counts stay inside the tile's regions).  Points
// of later entries (crowded tiles) and of pairs missing from the tile's entries
// (LDS table overflow in k_boundary) reserve one slot each.
// loaded up front, before the tile's counts are known: the first 256 8-B keys or 512
// narrow words and 32 entries (typical tiles: ~700 narrow points, ~10 entries), so the
// speculation reads nothing past the counts of most tiles; the rest follows once they
// are known.  (1024 narrow words up front read ~1.2 KB past a typical tile's points:
// 11.08 -> 10.83 MB per frame with half of that, concurrent throughput unchanged,
// profiles/r06/pmc_grp_pre_ab.txt)
#ifndef AT_GRP_PRE
#define AT_GRP_PRE 1
#endif
constexpr int kGrpPre = AT_GRP_PRE;
constexpr int kGrpEntPre = 32;
__global__ __launch_bounds__(256) void k_group(DevBufs b, Geom g) {
  const TileIdx bi = xcd_block<AT_XCD_GRP>();
  const int f = bi.y;
  __shared__ uint64_t s_hk[2 * kGrpEnt];
  __shared__ uint32_t s_he[2 * kGrpEnt];
  __shared__ uint32_t s_base[kGrpEnt], s_cur[kGrpEnt];
  const int tid = threadIdx.x;
  const size_t tb = (size_t)f * g.ntb + bi.x;
  const uint64_t* pts = b.pts + tb * g.bnd_region;
  // one round trip: status, counters, entry, points (the first 512 8-B keys or
  // 1024 narrow words: the same bytes)
  const uint32_t st = b.status[f];
  const uint32_t tc = b.tcnt[tb], ne = b.tent[tb];
  const uint32_t n = tc & ~kTileNarrow;
  const bool narrow = (tc & kTileNarrow) != 0;
  uint64_t ekey = 0;
  uint32_t ebase = kGrpFallback;
  if (tid < kGrpEntPre) {
    ekey = b.pent_key[tb * kLdsPairSlots + tid];
    ebase = b.pent_cnt[tb * kLdsPairSlots + tid];
  }
  uint64_t pv[kGrpPre];
#pragma unroll
  for (int k = 0; k < kGrpPre; k++) pv[k] = pts[tid + 256 * k];
  if (st & (kStatusPairsOverflow | kStatusHashFull)) return;
  if (tid >= kGrpEntPre && tid < kGrpEnt && (uint32_t)tid < ne) {
    ekey = b.pent_key[tb * kLdsPairSlots + tid];
    ebase = b.pent_cnt[tb * kLdsPairSlots + tid];
  }
  const uint64_t* ht_key = b.ht_key + (size_t)f * kHashSlots;
  const uint32_t* ht_off = b.ht_off + (size_t)f * kHashSlots;
  const uint32_t* ht_cnt = b.ht_cnt + (size_t)f * kHashSlots;
  uint32_t* ht_cur = b.ht_cur + (size_t)f * kHashSlots;
  auto in_bounds = [&](uint32_t c) { return c >= g.min_cluster && c <= g.max_cluster; };
  uint32_t* grp = b.grp + (size_t)f * g.cap_pts;  // the point's low 24 key bits (labels dropped)
  // a point whose entry has no LDS cursor (the tile's entries past kGrpEnt, or an
  // LDS table overflow in k_boundary) reserves its slot in the frame's pair table
  auto place_global = [&](uint64_t r01, uint32_t bits) {
    const uint32_t slot = ht_slot_find(ht_key, r01);
    if (slot == 0xffffffffu || !in_bounds(ht_cnt[slot])) return;
    grp[ht_off[slot] + atomicAdd(ht_cur + slot, 1u)] = bits;
  };
  if (narrow) {
    // the words carry their entry index: entry -> base and cursor in LDS, no lookup
    if (tid < kGrpEnt && (uint32_t)tid < ne) {
      s_base[tid] = ebase;
      s_cur[tid] = 0;
    }
    __syncthreads();
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(pts);
    // called by every lane of the wave (valid: the lane holds a point): lanes in a
    // run of equal entries (points come in emission order, mostly one pair after
    // another) reserve their slots with ONE LDS atomic by the run's head
    const uint32_t lane = lane_id();
    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    auto place = [&](uint32_t w, bool valid) {
      const uint32_t e = w >> 23;
      const uint32_t base = (valid && e < (uint32_t)kGrpEnt) ? s_base[e] : kGrpFallback;
      const bool lds = valid && base != kGrpFallback && base != kGrpDrop;
      const uint32_t key = lds ? e : 0x80000000u + lane;  // (never equal to a neighbour's)
      const bool same = lds && wave_shr1(key, 0xffffffffu) == key;
      const uint64_t same_mask = __ballot(same);
      const bool head = lds && !same;
      uint32_t start = 0;
      if (head) start = atomicAdd(&s_cur[e], run_len(same_mask, lane));
      const uint64_t heads = __ballot(head);
      const int hl = (heads & le) ? 63 - __builtin_clzll(heads & le) : (int)lane;
      const uint32_t s0 = (uint32_t)__shfl((int)start, hl);
      if (lds) grp[base + s0 + (lane - (uint32_t)hl)] = narrow_bits(w);
      else if (valid && base == kGrpFallback) place_global(b.pent_key[tb * kLdsPairSlots + e], narrow_bits(w));
    };
#pragma unroll
    for (int k = 0; k < kGrpPre; k++) {
      const uint32_t i = 2 * (tid + 256 * k);
      place((uint32_t)pv[k], i < n);
      place((uint32_t)(pv[k] >> 32), i + 1 < n);
    }
    for (uint32_t i0 = 512 * kGrpPre; i0 < n; i0 += 256) {
      const uint32_t i = i0 + tid;
      place(i < n ? pw[i] : 0u, i < n);
    }
    return;
  }
  for (int i = tid; i < 2 * kGrpEnt; i += 256) s_hk[i] = 0;
  __syncthreads();
  if (tid < kGrpEnt && (uint32_t)tid < ne && ebase != kGrpFallback) {
    s_base[tid] = ebase;
    s_cur[tid] = 0;
    uint32_t h = (uint32_t)(mix_hash(ekey) & (2 * kGrpEnt - 1));
    while (true) {  // keys are distinct and the table is at most half full
      const uint64_t prev = atomicCAS((unsigned long long*)&s_hk[h], 0ull, (unsigned long long)ekey);
      if (prev == 0) {
        s_he[h] = (uint32_t)tid;
        break;
      }
      h = (h + 1) & (2 * kGrpEnt - 1);
    }
  }
  __syncthreads();
  // called by every lane of the wave (valid: the lane holds a point); runs of equal
  // entries in consecutive lanes reserve their slots with one LDS atomic by the head
  const uint32_t lane = lane_id();
  const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  auto place = [&](uint64_t key, bool valid) {
    const uint64_t r01 = key >> 24;
    uint32_t e = 0xffffffffu;
    if (valid) {
      uint32_t h = (uint32_t)(mix_hash(r01) & (2 * kGrpEnt - 1));
      for (int probe = 0; probe < 2 * kGrpEnt; probe++) {
        const uint64_t k = s_hk[h];
        if (k == r01) { e = s_he[h]; break; }
        if (k == 0) break;
        h = (h + 1) & (2 * kGrpEnt - 1);
      }
    }
    const uint32_t base = e != 0xffffffffu ? s_base[e] : kGrpDrop;
    const bool lds = base != kGrpDrop;
    const uint32_t ek = lds ? e : 0x80000000u + lane;  // (never equal to a neighbour's)
    const bool same = lds && wave_shr1(ek, 0xffffffffu) == ek;
    const uint64_t same_mask = __ballot(same);
    const bool head = lds && !same;
    uint32_t start = 0;
    if (head) start = atomicAdd(&s_cur[e], run_len(same_mask, lane));
    const uint64_t heads = __ballot(head);
    const int hl = (heads & le) ? 63 - __builtin_clzll(heads & le) : (int)lane;
    const uint32_t s0 = (uint32_t)__shfl((int)start, hl);
    if (lds) grp[base + s0 + (lane - (uint32_t)hl)] = (uint32_t)key & 0xffffffu;
    else if (valid && e == 0xffffffffu) place_global(r01, (uint32_t)key & 0xffffffu);
  };
#pragma unroll
  for (int k = 0; k < kGrpPre; k++) place(pv[k], (uint32_t)(tid + 256 * k) < n);
  for (uint32_t i0 = 256 * kGrpPre; i0 < n; i0 += 256) {
    const uint32_t i = i0 + tid;
    place(i < n ? pts[i] : 0ull, i < n);
  }
}

// ---------------------------------------------------------------------------
// K9: one blob pair per workgroup iteration (persistent, work-list driven).
// ---------------------------------------------------------------------------
struct Ext {
  uint32_t min_x, min_y, max_x, max_y, count;
  int32_t gx_sum, gy_sum;
  int64_t pg_sum;
};

__device__ __forceinline__ double ext_cx(const Ext& e) { return (double)((float)(e.min_x + e.max_x) * 0.5f) + 0.05118; }
__device__ __forceinline__ double ext_cy(const Ext& e) {
  return (double)((float)(e.min_y + e.max_y) * 0.5f) + -0.028581;
}
__device__ __forceinline__ float ext_dot(const Ext& e) {
  const int64_t t = e.pg_sum * 2 - (int64_t)((int)(e.min_x + e.max_x) * e.gx_sum) -
                    (int64_t)((int)(e.min_y + e.max_y) * e.gy_sum);
  const double a = (double)t * 0.5;
  const double bq = 0.05118 * (double)e.gx_sum;
  const double c = 0.028581 * (double)e.gy_sum;
  return (float)(a - bq + c);
}

// Line-fit weight of TransformLineFitPoint (apriltag_gpu.cu:631-687): (int)(hypotf(gx, gy)
// + 1), hypotf being (float)sqrt((double)gx^2 + (double)gy^2) (det_hypotf).  For byte
// differences (|gx|, |gy| <= 255) that is exactly floor(sqrt(gx^2 + gy^2)) + 1: a
// non-square s = gx^2 + gy^2 lies >= 1 / 724 below the next integer root, far above the
// float rounding near 362 (2^-15) -- so an integer square root instead of an fp64 one
__device__ __forceinline__ int32_t lf_weight(int32_t gx, int32_t gy) {
  const uint32_t sq = (uint32_t)(gx * gx + gy * gy);
  uint32_t r = (uint32_t)__builtin_amdgcn_sqrtf((float)sq);  // (v_sqrt_f32: within one of the root)
  r -= r * r > sq ? 1u : 0u;
  r += (r + 1) * (r + 1) <= sq ? 1u : 0u;
  return (int32_t)r + 1;
}

// FitLine's line normal (line_fit_filter.cu:798-872) from d = (float)(Cxx - Cyy),
// c = (float)(2 Cxy) and h = hypot(d, c); (float)(Cyy - Cxx) is -d exactly (the int64 ->
// float conversion rounds symmetrically)
__device__ __forceinline__ void line_normal(float d, float c, float h, double* lp23) {
  const float nx1 = d - h, ny1 = c;
  const float M1 = nx1 * nx1 + ny1 * ny1;
  const float nx2 = c, ny2 = -d - h;
  const float M2 = nx2 * nx2 + ny2 * ny2;
  float nx, ny;
  if (M1 > M2) { nx = nx1; ny = ny1; } else { nx = nx2; ny = ny2; }
  const float len = det_hypotf(nx, ny);
  lp23[0] = (double)(nx / len);
  lp23[1] = (double)(ny / len);
}

// FitLine (line_fit_filter.cu:798-872) / HostFitLine (apriltag_detect.cu:38-90).
// pre (optional): d, c and the centroid quotients, which are all UpdateFitQuads'
// corners need of the fit (k_quad_fin finishes from them)
__device__ void fit_line(const Moments& m, double* lp01, double* lp23, double* err, double* mse, float* pre = nullptr) {
  const int64_t W = m.W;
  const int64_t Cxx = (int64_t)((uint64_t)m.Mxx * (uint64_t)W - (uint64_t)((int64_t)m.Mx * (int64_t)m.Mx));
  const int64_t Cxy = (int64_t)((uint64_t)m.Mxy * (uint64_t)W - (uint64_t)((int64_t)m.Mx * (int64_t)m.My));
  const int64_t Cyy = (int64_t)((uint64_t)m.Myy * (uint64_t)W - (uint64_t)((int64_t)m.My * (int64_t)m.My));
  const float d = (float)(Cxx - Cyy), c = (float)(2 * Cxy);
  const float px = (float)m.Mx / (float)(m.W * 2), py = (float)m.My / (float)(m.W * 2);
  if (pre) {
    pre[0] = d; pre[1] = c; pre[2] = px; pre[3] = py;
    return;
  }
  const float h = det_hypotf(d, c);
  const float e8 = (float)((double)(W * W) * 8.0);
  const float eig = ((float)(Cxx + Cyy) - h) / e8;
  if (lp01) {
    lp01[0] = (double)px;
    lp01[1] = (double)py;
  }
  if (lp23) line_normal(d, c, h, lp23);
  *err = (double)((float)m.N * eig);
  *mse = (double)eig;
}

// ---- team-generic primitives: a team is the whole 256-thread workgroup
// (large blobs) or one 64-lane wave (small blobs, 4 independent teams per WG)
template <int NT>
__device__ __forceinline__ void team_sync() {
  if constexpr (NT == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

template <int NT>
__device__ __forceinline__ int team_rank() {
  return NT == 64 ? (int)lane_id() : (int)threadIdx.x;
}

template <int NT, typename T, typename Op>
__device__ T team_reduce(T v, Op op, T* s_tmp) {
  if constexpr (NT == 64) {
    return wave_reduce(v, op);
  } else {
    return block_reduce(v, op, s_tmp, NT / 64);
  }
}

template <int NT, typename T>
__device__ T team_incl_scan(T v, T* s_tmp, T* total) {
  if constexpr (NT == 64) {
    v = wave_incl_scan(v, AddOp(), T(0));
    *total = wave_read(v, 63);
    return v;
  } else {
    return block_incl_scan(v, s_tmp, total, NT / 64);
  }
}

template <typename T, int NT>
__device__ void team_bitonic_sort(T* s, int n) {
  const int r = team_rank<NT>();
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = r; i < n; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const T a = s[i], c = s[ixj];
          const bool up = (i & k) == 0;
          if ((a > c) == up) {
            s[i] = c;
            s[ixj] = a;
          }
        }
      }
      team_sync<NT>();
    }
  }
}


__device__ void redistort(const Params& p, double* x, double* y) {
  const double xP = (*x - p.cx) / p.fx, yP = (*y - p.cy) / p.fy;
  const double rSq = xP * xP + yP * yP;
  const double lin = 1 + p.k1 * rSq + p.k2 * rSq * rSq + p.k3 * rSq * rSq * rSq;
  const double xPP = xP * lin + 2 * p.p1 * xP * yP + p.p2 * (rSq + 2 * xP * xP);
  const double yPP = yP * lin + p.p1 * (rSq + 2 * yP * yP) + 2 * p.p2 * xP * yP;
  *x = xPP * p.fx + p.cx;
  *y = yPP * p.fy + p.cy;
}

__device__ void undistort(const Params& p, double* u, double* v) {
  const double xPP = (*u - p.cx) / p.fx, yPP = (*v - p.cy) / p.fy;
  double xP = xPP, yP = yPP;
  const double x0 = xP, y0 = yP;
  double prev_x, prev_y;
  int it = 0;
  do {
    prev_x = xP;
    prev_y = yP;
    const double rSq = xP * xP + yP * yP;
    const double rad = 1 + (p.k1 * rSq) + (p.k2 * rSq * rSq) + (p.k3 * rSq * rSq * rSq);
    const double rinv = 1 / rad;
    const double tdx = 2 * p.p1 * xP * yP + p.p2 * (rSq + p.k3 * rSq * rSq * rSq);  // apriltag_detect.cu:372
    const double tdy = p.p1 * (rSq + 2 * yP * yP) + 2 * p.p2 * xP * yP;
    xP = (x0 - tdx) * rinv;
    yP = (y0 - tdy) * rinv;
    if (it > 100) break;
    it++;
  } while (fabs(xP - prev_x) > 1e-6 || fabs(yP - prev_y) > 1e-6);
  *u = xP * p.fx + p.cx;
  *v = yP * p.fy + p.cy;
}

__device__ void hproject(const double* H, double x, double y, double* ox, double* oy) {
  const double xx = H[0] * x + H[1] * y + H[2];
  const double yy = H[3] * x + H[4] * y + H[5];
  const double zz = H[6] * x + H[7] * y + H[8];
  *ox = xx / zz;
  *oy = yy / zz;
}

// homography_compute2 (apriltag 3.x common/homography.c) for the 8x9 DLT system
// held in LDS (A[8][9]), spread over one wave: pivot search (first maximum,
// strict >, rows col..7), row swap and elimination in parallel.  Every element
// goes through exactly the serial sequence of operations (fct = A[i][col] /
// A[col][col]; A[i][j] -= fct * A[col][j]), so the result is bit-identical to
// the one-lane restatement (oracle/ao_oracle.c homography_compute2).  The
// eliminated sub-diagonal entries are never read again and are not zeroed.
// Returns 0 / -1 (singular), uniform across the wave; H valid on every lane.
__device__ int homography_wave(const float (*qc)[2], double* A, double* H) {
  const int lane = (int)lane_id();
  for (int e = lane; e < 72; e += 64) {
    const int row = e / 9, col = e % 9, i = row >> 1;
    const double c0 = (i == 0 || i == 3) ? -1 : 1, c1 = (i == 0 || i == 1) ? -1 : 1;
    const double c2 = qc[i][0], c3 = qc[i][1];
    // row 2i: (c0, c1, 1, 0, 0, 0, -c0 c2, -c1 c2, c2); row 2i+1: (0, 0, 0, c0, c1, 1, -c0 c3, -c1 c3, c3)
    const int k = (row & 1) ? col - 3 : col;  // position inside the (c0, c1, 1) triple
    const double cz = (row & 1) ? c3 : c2;
    double v = 0;
    if (k == 0) v = c0;
    else if (k == 1) v = c1;
    else if (k == 2) v = 1;
    if (col == 6) v = -c0 * cz;
    else if (col == 7) v = -c1 * cz;
    else if (col == 8) v = cz;
    A[e] = v;
  }
  team_sync<64>();  // (wave-level: k_decode<true> runs a second, independent wave)
  for (int col = 0; col < 8; col++) {
    // pivot: first row (col..7) holding the strict maximum of |A[row][col]| > 0
    double v = -1.0;
    int row = 64;
    if (lane < 8 - col) {
      row = col + lane;
      v = fabs(A[row * 9 + col]);
      if (!(v > 0.0)) { v = -1.0; row = 64; }  // NaN and 0 never win the serial strict '>'
    }
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) {
      const double ov = __shfl_xor(v, d);
      const int orow = __shfl_xor(row, d);
      if (ov > v || (ov == v && orow < row)) { v = ov; row = orow; }
    }
    v = __shfl(v, 0);
    row = __shfl(row, 0);
    if (!(v >= 1e-10)) return -1;  // max_val < 1e-10 (max_val starts at 0)
    if (row != col && lane <= 8 - col) {
      const int i = col + lane;
      const double t = A[col * 9 + i];
      A[col * 9 + i] = A[row * 9 + i];
      A[row * 9 + i] = t;
    }
    team_sync<64>();  // (wave-level: k_decode<true> runs a second, independent wave)
    const int nc = 8 - col;  // columns col+1..8
    if (lane < (7 - col) * nc) {
      const int i = col + 1 + lane / nc, j = col + 1 + lane % nc;
      const double fct = A[i * 9 + col] / A[col * 9 + col];
      A[i * 9 + j] -= fct * A[col * 9 + j];
    }
    team_sync<64>();  // (wave-level: k_decode<true> runs a second, independent wave)
  }
  // back substitution, every lane in the serial order with the solution in
  // registers (the row's A reads are independent LDS broadcasts, issued together)
  double x[8];
#pragma unroll
  for (int col = 7; col >= 0; col--) {
    double sum = 0;
#pragma unroll
    for (int i = col + 1; i < 8; i++) sum += A[col * 9 + i] * x[i];
    x[col] = (A[col * 9 + 8] - sum) / A[col * 9 + col];
  }
#pragma unroll
  for (int k = 0; k < 8; k++)
    if (lane == k) H[k] = x[k];
  if (lane == 8) H[8] = 1;
  team_sync<64>();  // (wave-level: k_decode<true> runs a second, independent wave)
  return 0;
}

struct GrayModel {
  double A[3][3], B[3], C[3];
};
__device__ void gm_add(GrayModel& g, double x, double y, double gray) {
  g.A[0][0] += x * x; g.A[0][1] += x * y; g.A[0][2] += x;
  g.A[1][1] += y * y; g.A[1][2] += y; g.A[2][2] += 1;
  g.B[0] += x * gray; g.B[1] += y * gray; g.B[2] += gray;
}
__device__ void gm_solve(GrayModel& g) {
  const double* A = &g.A[0][0];
  double L[9], M[9];
  L[0] = sqrt(A[0]); L[3] = A[1] / L[0]; L[6] = A[2] / L[0];
  L[4] = sqrt(A[4] - L[3] * L[3]); L[7] = (A[5] - L[3] * L[6]) / L[4];
  L[8] = sqrt(A[8] - L[6] * L[6] - L[7] * L[7]);
  M[0] = 1 / L[0]; M[3] = -L[3] * M[0] / L[4]; M[4] = 1 / L[4];
  M[6] = (-L[6] * M[0] - L[7] * M[3]) / L[8]; M[7] = -L[7] * M[4] / L[8]; M[8] = 1 / L[8];
  const double t0 = M[0] * g.B[0];
  const double t1 = M[3] * g.B[0] + M[4] * g.B[1];
  const double t2 = M[6] * g.B[0] + M[7] * g.B[1] + M[8] * g.B[2];
  g.C[0] = M[0] * t0 + M[3] * t1 + M[6] * t2;
  g.C[1] = M[4] * t1 + M[7] * t2;
  g.C[2] = M[8] * t2;
}
__device__ __forceinline__ double gm_interp(const GrayModel& g, double x, double y) {
  return g.C[0] * x + g.C[1] * y + g.C[2];
}

// lexicographic 4-combinations of 10 maxima == Unrank (line_fit_filter.cu:709-728)
__constant__ uint8_t c_combo[210][4] = {{0,1,2,3},{0,1,2,4},{0,1,2,5},{0,1,2,6},{0,1,2,7},{0,1,2,8},{0,1,2,9},{0,1,3,4},{0,1,3,5},{0,1,3,6},{0,1,3,7},{0,1,3,8},{0,1,3,9},{0,1,4,5},{0,1,4,6},{0,1,4,7},{0,1,4,8},{0,1,4,9},{0,1,5,6},{0,1,5,7},{0,1,5,8},{0,1,5,9},{0,1,6,7},{0,1,6,8},{0,1,6,9},{0,1,7,8},{0,1,7,9},{0,1,8,9},{0,2,3,4},{0,2,3,5},{0,2,3,6},{0,2,3,7},{0,2,3,8},{0,2,3,9},{0,2,4,5},{0,2,4,6},{0,2,4,7},{0,2,4,8},{0,2,4,9},{0,2,5,6},{0,2,5,7},{0,2,5,8},{0,2,5,9},{0,2,6,7},{0,2,6,8},{0,2,6,9},{0,2,7,8},{0,2,7,9},{0,2,8,9},{0,3,4,5},{0,3,4,6},{0,3,4,7},{0,3,4,8},{0,3,4,9},{0,3,5,6},{0,3,5,7},{0,3,5,8},{0,3,5,9},{0,3,6,7},{0,3,6,8},{0,3,6,9},{0,3,7,8},{0,3,7,9},{0,3,8,9},{0,4,5,6},{0,4,5,7},{0,4,5,8},{0,4,5,9},{0,4,6,7},{0,4,6,8},{0,4,6,9},{0,4,7,8},{0,4,7,9},{0,4,8,9},{0,5,6,7},{0,5,6,8},{0,5,6,9},{0,5,7,8},{0,5,7,9},{0,5,8,9},{0,6,7,8},{0,6,7,9},{0,6,8,9},{0,7,8,9},{1,2,3,4},{1,2,3,5},{1,2,3,6},{1,2,3,7},{1,2,3,8},{1,2,3,9},{1,2,4,5},{1,2,4,6},{1,2,4,7},{1,2,4,8},{1,2,4,9},{1,2,5,6},{1,2,5,7},{1,2,5,8},{1,2,5,9},{1,2,6,7},{1,2,6,8},{1,2,6,9},{1,2,7,8},{1,2,7,9},{1,2,8,9},{1,3,4,5},{1,3,4,6},{1,3,4,7},{1,3,4,8},{1,3,4,9},{1,3,5,6},{1,3,5,7},{1,3,5,8},{1,3,5,9},{1,3,6,7},{1,3,6,8},{1,3,6,9},{1,3,7,8},{1,3,7,9},{1,3,8,9},{1,4,5,6},{1,4,5,7},{1,4,5,8},{1,4,5,9},{1,4,6,7},{1,4,6,8},{1,4,6,9},{1,4,7,8},{1,4,7,9},{1,4,8,9},{1,5,6,7},{1,5,6,8},{1,5,6,9},{1,5,7,8},{1,5,7,9},{1,5,8,9},{1,6,7,8},{1,6,7,9},{1,6,8,9},{1,7,8,9},{2,3,4,5},{2,3,4,6},{2,3,4,7},{2,3,4,8},{2,3,4,9},{2,3,5,6},{2,3,5,7},{2,3,5,8},{2,3,5,9},{2,3,6,7},{2,3,6,8},{2,3,6,9},{2,3,7,8},{2,3,7,9},{2,3,8,9},{2,4,5,6},{2,4,5,7},{2,4,5,8},{2,4,5,9},{2,4,6,7},{2,4,6,8},{2,4,6,9},{2,4,7,8},{2,4,7,9},{2,4,8,9},{2,5,6,7},{2,5,6,8},{2,5,6,9},{2,5,7,8},{2,5,7,9},{2,5,8,9},{2,6,7,8},{2,6,7,9},{2,6,8,9},{2,7,8,9},{3,4,5,6},{3,4,5,7},{3,4,5,8},{3,4,5,9},{3,4,6,7},{3,4,6,8},{3,4,6,9},{3,4,7,8},{3,4,7,9},{3,4,8,9},{3,5,6,7},{3,5,6,8},{3,5,6,9},{3,5,7,8},{3,5,7,9},{3,5,8,9},{3,6,7,8},{3,6,7,9},{3,6,8,9},{3,7,8,9},{4,5,6,7},{4,5,6,8},{4,5,6,9},{4,5,7,8},{4,5,7,9},{4,5,8,9},{4,6,7,8},{4,6,7,9},{4,6,8,9},{4,7,8,9},{5,6,7,8},{5,6,7,9},{5,6,8,9},{5,7,8,9},{6,7,8,9}};

// the combinations in colexicographic order (by m3, then m2, m1, m0), as indices into
// c_combo: those with m3 < cnt are exactly the first C(cnt, 4), so a blob's FitQuads
// loop visits only its valid combinations
__constant__ uint8_t c_colex[210] = {0,1,7,28,84,2,8,29,85,13,34,90,49,105,140,3,9,30,86,14,35,91,50,106,141,18,39,95,54,110,145,64,120,155,175,4,10,31,87,15,36,92,51,107,142,19,40,96,55,111,146,65,121,156,176,22,43,99,58,114,149,68,124,159,179,74,130,165,185,195,5,11,32,88,16,37,93,52,108,143,20,41,97,56,112,147,66,122,157,177,23,44,100,59,115,150,69,125,160,180,75,131,166,186,196,25,46,102,61,117,152,71,127,162,182,77,133,168,188,198,80,136,171,191,201,205,6,12,33,89,17,38,94,53,109,144,21,42,98,57,113,148,67,123,158,178,24,45,101,60,116,151,70,126,161,181,76,132,167,187,197,26,47,103,62,118,153,72,128,163,183,78,134,169,189,199,81,137,172,192,202,206,27,48,104,63,119,154,73,129,164,184,79,135,170,190,200,82,138,173,193,203,207,83,139,174,194,204,208,209};

struct LineFitOut {
  double err, mse;
  double p01[2], p23[2];
};

// FitLine by value (no pointers -> no scratch traffic)
template <bool kP01, bool kP23>
__device__ __forceinline__ LineFitOut fit_line_v(const Moments& m) {
  LineFitOut o;
  fit_line(m, kP01 ? o.p01 : nullptr, kP23 ? o.p23 : nullptr, &o.err, &o.mse);
  return o;
}

// Moments of a run of line-fit points (LineFitPoint, line_fit_filter.h:61-83) in
// the reference's integer widths: Mx, My, W wrap as int32 and Mxx, Myy, Mxy as
// int64 (kept here as u32 / u64 so wrapping is defined).  Sums, differences and
// prefix differences are then exact modulo 2^32 / 2^64, which is what the
// reference's int32 / int64 prefix sums compute.
struct Mom6 {
  uint32_t Mx, My, W;
  uint64_t Mxx, Myy, Mxy;
};
__device__ __forceinline__ Mom6 mom_zero() { return Mom6{0, 0, 0, 0, 0, 0}; }
__device__ __forceinline__ void mom_add(Mom6& a, const Mom6& c) {
  a.Mx += c.Mx; a.My += c.My; a.W += c.W; a.Mxx += c.Mxx; a.Myy += c.Myy; a.Mxy += c.Mxy;
}
__device__ __forceinline__ void mom_sub(Mom6& a, const Mom6& c) {
  a.Mx -= c.Mx; a.My -= c.My; a.W -= c.W; a.Mxx -= c.Mxx; a.Myy -= c.Myy; a.Mxy -= c.Mxy;
}
__device__ __forceinline__ Mom6 mom_shfl(const Mom6& m, int src) {
  Mom6 r;
  r.Mx = __shfl(m.Mx, src); r.My = __shfl(m.My, src); r.W = __shfl(m.W, src);
  r.Mxx = __shfl(m.Mxx, src); r.Myy = __shfl(m.Myy, src); r.Mxy = __shfl(m.Mxy, src);
  return r;
}
__device__ __forceinline__ Mom6 mom_shfl_up(const Mom6& m, int d) {
  Mom6 r;
  r.Mx = __shfl_up(m.Mx, d); r.My = __shfl_up(m.My, d); r.W = __shfl_up(m.W, d);
  r.Mxx = __shfl_up(m.Mxx, d); r.Myy = __shfl_up(m.Myy, d); r.Mxy = __shfl_up(m.Mxy, d);
  return r;
}

// Blob point sort key (written by k_extents): theta [59:32], dxy [31:30],
// by [29:20], bx [19:10], b2w [9], W [8:0] (W = (int)(hypotf(gx, gy) + 1) <= 361).
constexpr int kKeyTheta = 32;

// Compact point word of a sorted blob point: bx [9:0], by [19:10], dxy [21:20],
// W [30:22].
__device__ __forceinline__ uint32_t compact_word(uint64_t sk) {
  return (uint32_t)((sk >> 10) & 0x3ff) | ((uint32_t)((sk >> 20) & 0x3ff) << 10) | ((uint32_t)((sk >> 30) & 3) << 20) |
         ((uint32_t)(sk & 0x1ff) << 22);
}

// TransformLineFitPoint (apriltag_gpu.cu:631-687) of one compact point word
__device__ __forceinline__ Mom6 point_mom(uint32_t cw) {
  const int dxy = (int)((cw >> 20) & 3);
  const uint32_t ix2 = (cw & 0x3ff) * 2 + dx_of(dxy) + 1;
  const uint32_t iy2 = ((cw >> 10) & 0x3ff) * 2 + dy_of(dxy) + 1;
  const uint32_t Wt = cw >> 22;
  Mom6 m;
  m.Mx = Wt * ix2;
  m.My = Wt * iy2;
  m.W = Wt;
  // (int64_t)(int32 W * ix2 * ix2): the product wraps as int32, then sign-extends
  m.Mxx = (uint64_t)(int64_t)(int32_t)(Wt * ix2 * ix2);
  m.Mxy = (uint64_t)(int64_t)(int32_t)(Wt * ix2 * iy2);
  m.Myy = (uint64_t)(int64_t)(int32_t)(Wt * iy2 * iy2);
  return m;
}

__device__ __forceinline__ Moments to_moments(const Mom6& s, int32_t N) {
  Moments m;
  m.Mx = (int32_t)s.Mx; m.My = (int32_t)s.My; m.W = (int32_t)s.W;
  m.Mxx = (int64_t)s.Mxx; m.Myy = (int64_t)s.Myy; m.Mxy = (int64_t)s.Mxy;
  m.N = N;
  return m;
}

// FitLineError (line_fit_filter.cu:22-36) of one window, as ErrorCalculator
// evaluates it (float result)
__device__ __forceinline__ float window_err(const Mom6& s, int32_t N) {
  const Moments m = to_moments(s, N);
  // a window's weight sum is below 2^14 (at most 41 points of weight <= 362): 64 x 32-bit
  // products, and 8 W^2 < 2^32 converts exactly as an unsigned int (the double product the
  // reference rounds to float is the same integer)
  const uint64_t Wl = (uint32_t)m.W;
  const int64_t Cxx = (int64_t)((uint64_t)m.Mxx * Wl - (uint64_t)((int64_t)m.Mx * (int64_t)m.Mx));
  const int64_t Cxy = (int64_t)((uint64_t)m.Mxy * Wl - (uint64_t)((int64_t)m.Mx * (int64_t)m.My));
  const int64_t Cyy = (int64_t)((uint64_t)m.Myy * Wl - (uint64_t)((int64_t)m.My * (int64_t)m.My));
  // the three int64 -> float conversions through double: |values| < 2^51 here (a window's
  // second moments), so the double is exact and the one rounding is the direct cast's
  auto tof = [](int64_t v) { return (float)(double)v; };
  const float h = det_hypotf(tof(Cxx - Cyy), tof(2 * Cxy));
  const float eig = (tof(Cxx + Cyy) - h) / (float)(8u * (uint32_t)Wl * (uint32_t)Wl);
  return (float)m.N * eig;
}

// Per-team shared state of one blob.  After the theta sort `keys` is reused:
// u32 compact point words in bytes [0, 4n) and f32 window errors in bytes
// [4 CAP, 4 CAP + 4n).  The union holds, in turn, the bucket-sort counts, the
// peak keys and the 90 segment fits of FitQuads.

template <int NT, int CAP>
constexpr int kKeySlots = (NT >= 512 && CAP <= 4096) ? 2 * CAP  // latency-mode teams: bucket scatter room for CAP keys
                          : CAP < 400 ? 400                      // (SegFits lives over the keys: 3.2 KB)
                                      : CAP;

// the 90 distinct segment fits of FitQuads: [a][b], a < b forward pi[a]->pi[b],
// a > b wrap-around pi[a]->pi[b] (the closing side m3->m0).  They live over the
// team's key area, which is dead by then (3.2 KB <= 8 CAP bytes).
struct SegFits {
  double err[kNMaxima][kNMaxima];
  double mse[kNMaxima][kNMaxima];
  double p[kNMaxima][kNMaxima][2];
};

template <int NT, int CAP>
struct BlobShared {
  uint64_t keys[kKeySlots<NT, CAP>];
  uint32_t bcnt[kKeySlots<NT, CAP> / 4];  // theta bucket counts, two u16 per word (team_bucket_sort)
  uint64_t pks[16];                        // the top-10 peak keys (peaks themselves stay in registers)
  uint64_t wtop[NT > 64 ? NT / 64 * 10 : 1];  // each wave's top-10 peak keys (teams of more than one wave)
  // inclusive prefix moments at the indices FitQuads reads: [k] = P[pi[k]],
  // [10 + k] = P[pi[k] - 1], [20] = P[n - 1]
  uint32_t tMx[21], tMy[21], tW[21];
  uint64_t tMxx[21], tMyy[21], tMxy[21];
  // exclusive prefix of each thread's chunk (teams of more than one wave)
  uint32_t bMx[NT > 64 ? NT : 1], bMy[NT > 64 ? NT : 1], bW[NT > 64 ? NT : 1];
  uint64_t bMxx[NT > 64 ? NT : 1], bMyy[NT > 64 ? NT : 1], bMxy[NT > 64 ? NT : 1];
  Mom6 wsum[NT / 64];
  int64_t red7[NT / 64][8];
  double red_f64[16];
  uint32_t red_u32[16];
  uint32_t red_idx[16];
  uint32_t item, nwork, npeaks;
  int32_t pi[16];
  double lines[4][4];
  uint32_t pacc[22];  // probe accumulators + processed-point and FitQuads counts of this team
  uint32_t ph[10];    // probe: phase durations of the current item
  uint32_t slow_dt, slow_n, slow_ph[10];  // probe: this team's slowest item
  uint64_t t_last, t_item;
};

// Sort of a blob's (theta, plane, y, x) keys: theta is near-uniform around the
// blob centre, so the keys are bucketed by theta (counting sort: LDS histogram,
// scan, scatter into the upper half of S.keys) and each key's final slot is its
// bucket start + its rank inside the (small) bucket.  Exactly the order of a
// full sort.  Returns false -- caller falls back to the bitonic sort -- when
// the keys do not fit twice in S.keys or a bucket holds more than 32 keys.
constexpr uint64_t kThetaSpan = 50265600;  // > max theta = rint((2 pi) * 8e6)

template <int NT, int CAP>
__device__ bool team_bucket_sort(BlobShared<NT, CAP>& S, int n) {
  constexpr int KEYS = kKeySlots<NT, CAP>;
  if (n < 64 || 2 * n > KEYS) return false;
  const int tid = team_rank<NT>();
  int nb = 32;
  while (2 * nb < n) nb <<= 1;  // n/2 <= nb < n buckets, power of two, <= KEYS/2
  auto bucket = [&](uint64_t k) { return (uint32_t)(((k >> kKeyTheta) * (uint64_t)nb) / kThetaSpan); };
  uint32_t* bcnt = S.bcnt;
  for (int i = tid; i < nb / 2; i += NT) bcnt[i] = 0;
  team_sync<NT>();
  for (int t = tid; t < n; t += NT) {
    const uint32_t bk = bucket(S.keys[t]);
    atomicAdd(&bcnt[bk >> 1], 1u << ((bk & 1) * 16));
  }
  team_sync<NT>();
  // exclusive scan of the nb counts: each thread owns nb/NT (or 1) consecutive buckets
  const int per = nb >= NT ? nb / NT : 1;
  const int b0 = tid * per;
  uint32_t loc = 0, mx = 0;
  uint32_t cval[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    cval[j] = 0;
    if (j < per && b0 + j < nb) {
      const uint32_t bb = (uint32_t)(b0 + j);
      cval[j] = (bcnt[bb >> 1] >> ((bb & 1) * 16)) & 0xffffu;
      loc += cval[j];
      mx = cval[j] > mx ? cval[j] : mx;
    }
  }
  uint32_t tot;
  const uint32_t incl = team_incl_scan<NT>(loc, S.red_u32, &tot);
  mx = team_reduce<NT>(mx, MaxOp(), S.red_u32);
  if (mx > 32) return false;  // uniform across the team
  team_sync<NT>();
  // starts, written back in place (u16, < n)
  uint32_t run = incl - loc;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    if (j < per && b0 + j < nb && (j & 1) == 0) {
      const uint32_t bb = (uint32_t)(b0 + j);  // even: owns the whole word when per >= 2
      if (per >= 2) {
        const uint32_t s0 = run, s1 = run + cval[j];
        bcnt[bb >> 1] = s0 | (s1 << 16);
      }
    }
    if (j < per && b0 + j < nb) run += cval[j];
  }
  if (per == 1 && b0 < nb) {
    // one bucket per thread: neighbours share a word; even lane writes both halves
    const uint32_t mine = incl - loc;
    const uint32_t other = __shfl_down(mine, 1);
    if ((b0 & 1) == 0) bcnt[b0 >> 1] = mine | (other << 16);
  }
  team_sync<NT>();
  uint64_t* T = S.keys + KEYS / 2;
  for (int t = tid; t < n; t += NT) {
    const uint64_t k = S.keys[t];
    const uint32_t bk = bucket(k);
    const uint32_t old = atomicAdd(&bcnt[bk >> 1], 1u << ((bk & 1) * 16));
    T[(old >> ((bk & 1) * 16)) & 0xffffu] = k;
  }
  team_sync<NT>();
  for (int s = tid; s < n; s += NT) {
    const uint64_t k = T[s];
    const uint32_t bk = bucket(k);
    int lo = s, hi = s + 1;
    while (lo > 0 && bucket(T[lo - 1]) == bk) lo--;
    while (hi < n && bucket(T[hi]) == bk) hi++;
    int r = lo;
    for (int j = lo; j < hi; j++) r += T[j] < k;
    S.keys[r] = k;
  }
  team_sync<NT>();
  return true;
}

// bitonic sort of n (power of two) peak keys: slots below cap in LDS, the rest
// in the team's global overflow area (kGlob: large blobs with pathological peak
// counts only; the small-blob LDS area always holds n/2 peaks)
template <bool kGlob>
__device__ __forceinline__ uint64_t pk_get(const uint64_t* lds, const uint64_t* gpk, int cap, int i) {
  if constexpr (kGlob) return i < cap ? lds[i] : gpk[i - cap];
  else return lds[i];
}
template <bool kGlob>
__device__ __forceinline__ void pk_put(uint64_t* lds, uint64_t* gpk, int cap, int i, uint64_t v) {
  if constexpr (kGlob) {
    if (i < cap) lds[i] = v;
    else gpk[i - cap] = v;
  } else {
    lds[i] = v;
  }
}
template <int NT, bool kGlob>
__device__ void team_bitonic_sort_pk(uint64_t* lds, uint64_t* gpk, int cap, int n) {
  const int r = team_rank<NT>();
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = r; i < n; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t a = pk_get<kGlob>(lds, gpk, cap, i), c = pk_get<kGlob>(lds, gpk, cap, ixj);
          const bool up = (i & k) == 0;
          if ((a > c) == up) {
            pk_put<kGlob>(lds, gpk, cap, i, c);
            pk_put<kGlob>(lds, gpk, cap, ixj, a);
          }
        }
      }
      team_sync<NT>();
    }
  }
}

// one extents reduction of seven values across the team (P3 MinMaxExtents)
template <int NT, int CAP>
__device__ __forceinline__ void team_extents(BlobShared<NT, CAP>& S, uint32_t& mnx, uint32_t& mxx, uint32_t& mny,
                                             uint32_t& mxy, int32_t& sgx, int32_t& sgy, int64_t& spg) {
  mnx = wave_reduce(mnx, MinOp()); mxx = wave_reduce(mxx, MaxOp());
  mny = wave_reduce(mny, MinOp()); mxy = wave_reduce(mxy, MaxOp());
  sgx = wave_reduce(sgx, AddOp()); sgy = wave_reduce(sgy, AddOp());
  spg = wave_reduce(spg, AddOp());
  if constexpr (NT > 64) {
    const int w = threadIdx.x >> 6;
    team_sync<NT>();
    if (lane_id() == 0) {
      S.red7[w][0] = mnx; S.red7[w][1] = mxx; S.red7[w][2] = mny; S.red7[w][3] = mxy;
      S.red7[w][4] = sgx; S.red7[w][5] = sgy; S.red7[w][6] = spg;
    }
    team_sync<NT>();
    for (int i = 0; i < NT / 64; i++) {
      mnx = min(mnx, (uint32_t)S.red7[i][0]); mxx = max(mxx, (uint32_t)S.red7[i][1]);
      mny = min(mny, (uint32_t)S.red7[i][2]); mxy = max(mxy, (uint32_t)S.red7[i][3]);
    }
    int32_t gx = 0, gy = 0;
    int64_t pg = 0;
    for (int i = 0; i < NT / 64; i++) {
      gx += (int32_t)S.red7[i][4]; gy += (int32_t)S.red7[i][5]; pg += S.red7[i][6];
    }
    sgx = gx; sgy = gy; spg = pg;
  }
}

// Exclusive team scan of each thread's chunk moments (one pass for all six);
// *total = the sum over the team
template <int NT, int CAP>
__device__ __forceinline__ Mom6 team_excl_scan_mom(BlobShared<NT, CAP>& S, const Mom6& v, Mom6* total) {
  const uint32_t lane = lane_id();
  Mom6 incl;
  incl.Mx = wave_incl_scan(v.Mx, AddOp(), 0u);
  incl.My = wave_incl_scan(v.My, AddOp(), 0u);
  incl.W = wave_incl_scan(v.W, AddOp(), 0u);
  incl.Mxx = wave_incl_scan(v.Mxx, AddOp(), (uint64_t)0);
  incl.Myy = wave_incl_scan(v.Myy, AddOp(), (uint64_t)0);
  incl.Mxy = wave_incl_scan(v.Mxy, AddOp(), (uint64_t)0);
  Mom6 ex = incl;
  mom_sub(ex, v);
  if constexpr (NT > 64) {
    const int w = threadIdx.x >> 6;
    team_sync<NT>();
    if (lane == 63) S.wsum[w] = incl;
    team_sync<NT>();
    Mom6 tot = mom_zero();
    for (int i = 0; i < NT / 64; i++) {
      if (i < w) mom_add(ex, S.wsum[i]);
      mom_add(tot, S.wsum[i]);
    }
    *total = tot;
  } else {
    *total = Mom6{wave_read(incl.Mx, 63), wave_read(incl.My, 63), wave_read(incl.W, 63),
                  wave_read(incl.Mxx, 63), wave_read(incl.Myy, 63), wave_read(incl.Mxy, 63)};
  }
  return ex;
}

// largest theta bucket ranked in place: a rank costs one LDS read per bucket
// key, still well below a bitonic sort (log2(n)^2 / 2 passes) for crowded
// buckets (long straight borders seen from the blob centre)
constexpr uint32_t kRegSortMaxBucket = 512;

// Wave-team sort (NT == 64, 64 <= n <= CAP <= 512 keys): the keys stay in
// registers (CAP / 64 per lane) through a counting sort by theta bucket (LDS
// histogram, scan, scatter with LDS atomics) and an in-bucket rank, so no second
// LDS key array is needed and blobs up to CAP points take this path.  Buckets
// are theta >> s (nb = 2^m buckets of width 2^(26-m); theta < 2^26).  Returns
// false with the keys in S.keys in load order when a bucket exceeds 32 keys.
template <int CAP>
__device__ bool wave_bucket_sort_kv(BlobShared<64, CAP>& S, uint64_t (&kv)[CAP / 64], int n) {
  static_assert(CAP % 64 == 0 && CAP <= 1024, "wave sort: at most 16 keys per lane");
  constexpr int PB = CAP > 512 ? 8 : 4;  // buckets per lane at most (nb < n <= CAP: nb <= CAP / 2)
  static_assert(kThetaSpan <= (1ull << 26), "theta fits 26 bits");
  constexpr int KPL = CAP / 64;
  const uint32_t lane = lane_id();
  int nb = 32;
  while (2 * nb < n) nb <<= 1;  // n/2 <= nb < n, power of two, <= 256
  const int sh = 26 - __builtin_ctz((unsigned)nb);
  auto bucket = [&](uint64_t k) { return (uint32_t)((k >> kKeyTheta) >> sh); };
  uint32_t* bcnt = S.bcnt;  // two u16 counters per word
  for (int i = (int)lane; i < nb / 2; i += 64) bcnt[i] = 0;
  team_sync<64>();
#pragma unroll
  for (int j = 0; j < KPL; j++) {
    if (j * 64 + (int)lane < n) {
      const uint32_t bk = bucket(kv[j]);
      atomicAdd(&bcnt[bk >> 1], 1u << ((bk & 1) * 16));
    }
  }
  team_sync<64>();
  // exclusive scan of the nb counts, each lane owning nb/64 (or one) consecutive buckets
  const int per = nb >= 64 ? nb / 64 : 1;
  const int b0 = (int)lane * per;
  uint32_t cval[PB], loc = 0, mx = 0;
#pragma unroll
  for (int j = 0; j < PB; j++) {
    cval[j] = 0;
    if (j < per && b0 + j < nb) {
      const uint32_t bb = (uint32_t)(b0 + j);
      cval[j] = (bcnt[bb >> 1] >> ((bb & 1) * 16)) & 0xffffu;
      loc += cval[j];
      mx = cval[j] > mx ? cval[j] : mx;
    }
  }
  const uint32_t incl = wave_incl_scan(loc, AddOp(), 0u);
  mx = wave_reduce(mx, MaxOp());
  if (mx > kRegSortMaxBucket) {  // uniform: fall back to the bitonic sort on S.keys
#pragma unroll
    for (int j = 0; j < KPL; j++) {
      const int t = j * 64 + (int)lane;
      if (t < n) S.keys[t] = kv[j];
    }
    team_sync<64>();
    return false;
  }
  team_sync<64>();
  // bucket starts in place (u16 each)
  uint32_t run = incl - loc;
  uint32_t st[PB];
#pragma unroll
  for (int j = 0; j < PB; j++) {
    st[j] = run;
    if (j < per && b0 + j < nb) run += cval[j];
  }
  if (per >= 2) {
#pragma unroll
    for (int j = 0; j < PB; j += 2)
      if (j < per) bcnt[(b0 + j) >> 1] = st[j] | (st[j + 1] << 16);
  } else if (b0 < nb) {  // one bucket per lane: the even lane writes both halves of the word
    const uint32_t other = wave_read_next(st[0]);
    if ((b0 & 1) == 0) bcnt[b0 >> 1] = st[0] | (other << 16);
  }
  team_sync<64>();
  // scatter: after it each bucket's counter holds its end
#pragma unroll
  for (int j = 0; j < KPL; j++) {
    if (j * 64 + (int)lane < n) {
      const uint32_t bk = bucket(kv[j]);
      const uint32_t old = atomicAdd(&bcnt[bk >> 1], 1u << ((bk & 1) * 16));
      S.keys[(old >> ((bk & 1) * 16)) & 0xffffu] = kv[j];
    }
  }
  team_sync<64>();
  uint32_t rk[KPL];
#pragma unroll
  for (int j = 0; j < KPL; j++) {
    rk[j] = 0;
    if (j * 64 + (int)lane < n) {
      const uint32_t bk = bucket(kv[j]);
      const uint32_t hi = (bcnt[bk >> 1] >> ((bk & 1) * 16)) & 0xffffu;
      const uint32_t lo = bk ? (bcnt[(bk - 1) >> 1] >> (((bk - 1) & 1) * 16)) & 0xffffu : 0u;
      uint32_t r = lo;
      for (uint32_t i = lo; i < hi; i++) r += S.keys[i] < kv[j];
      rk[j] = r;
    }
  }
  team_sync<64>();
#pragma unroll
  for (int j = 0; j < KPL; j++)
    if (j * 64 + (int)lane < n) S.keys[rk[j]] = kv[j];
  team_sync<64>();
  return true;
}

// keys (theta, plane, y, x) from global memory: slot t = j * 64 + lane
template <int CAP>
__device__ bool wave_bucket_sort(BlobShared<64, CAP>& S, const uint64_t* keys, int n) {
  constexpr int KPL = CAP / 64;
  const uint32_t lane = lane_id();
  uint64_t kv[KPL];
#pragma unroll
  for (int j = 0; j < KPL; j++) {
    const int t = j * 64 + (int)lane;
    kv[j] = t < n ? keys[t] : ~0ull;
  }
  return wave_bucket_sort_kv<CAP>(S, kv, n);
}

// Workgroup-team variant of wave_bucket_sort for the blobs whose keys do not
// fit twice in S.keys (n > KEYS / 2): the keys stay in registers (CAP / NT per
// thread) through the counting sort and the in-bucket rank, instead of falling
// back to a bitonic sort of the next power of two.
// keys in registers (slot t = j * NT + tid); on failure they are left in S.keys
// (load order) for the bitonic fallback
template <int NT, int CAP>
__device__ bool team_reg_bucket_sort_kv(BlobShared<NT, CAP>& S, uint64_t (&kv)[CAP / NT], int n) {
  static_assert(NT > 64 && CAP % NT == 0, "workgroup teams");
  constexpr int KPL = CAP / NT;
  constexpr int KEYS = kKeySlots<NT, CAP>;
  static_assert(KPL <= 16, "at most 16 keys per thread");
  const int tid = team_rank<NT>();
  int nb = 32;
  while (2 * nb < n) nb <<= 1;  // n/2 <= nb < n, power of two
  if (nb / 2 > KEYS / 4) {  // (uniform)
#pragma unroll
    for (int j = 0; j < KPL; j++) {
      const int t = j * NT + tid;
      if (t < n) S.keys[t] = kv[j];
    }
    team_sync<NT>();
    return false;
  }
  const int sh = 26 - __builtin_ctz((unsigned)nb);
  auto bucket = [&](uint64_t k) { return (uint32_t)((k >> kKeyTheta) >> sh); };
  uint32_t* bcnt = S.bcnt;
  for (int i = tid; i < nb / 2; i += NT) bcnt[i] = 0;
  team_sync<NT>();
#pragma unroll
  for (int j = 0; j < KPL; j++) {
    if (j * NT + tid < n) {
      const uint32_t bk = bucket(kv[j]);
      atomicAdd(&bcnt[bk >> 1], 1u << ((bk & 1) * 16));
    }
  }
  team_sync<NT>();
  const int per = nb >= NT ? nb / NT : 1;  // <= 8 (nb <= 2048 for 256 threads)
  const int b0 = tid * per;
  uint32_t cval[8], loc = 0, mx = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    cval[j] = 0;
    if (j < per && b0 + j < nb) {
      const uint32_t bb = (uint32_t)(b0 + j);
      cval[j] = (bcnt[bb >> 1] >> ((bb & 1) * 16)) & 0xffffu;
      loc += cval[j];
      mx = cval[j] > mx ? cval[j] : mx;
    }
  }
  uint32_t tot;
  const uint32_t incl = team_incl_scan<NT>(loc, S.red_u32, &tot);
  mx = team_reduce<NT>(mx, MaxOp(), S.red_u32);
  if (mx > kRegSortMaxBucket) {  // uniform: keys back to S.keys for the bitonic fallback
#pragma unroll
    for (int j = 0; j < KPL; j++) {
      const int t = j * NT + tid;
      if (t < n) S.keys[t] = kv[j];
    }
    team_sync<NT>();
    return false;
  }
  team_sync<NT>();
  uint32_t run = incl - loc;
  uint32_t st[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    st[j] = run;
    if (j < per && b0 + j < nb) run += cval[j];
  }
  if (per >= 2) {
#pragma unroll
    for (int j = 0; j < 8; j += 2)
      if (j < per) bcnt[(b0 + j) >> 1] = st[j] | (st[j + 1] << 16);
  } else if (b0 < nb) {
    const uint32_t other = wave_read_next(st[0]);  // neighbours share a word (same wave: NT >= nb's lane pairs)
    if ((b0 & 1) == 0) bcnt[b0 >> 1] = st[0] | (other << 16);
  }
  team_sync<NT>();
#pragma unroll
  for (int j = 0; j < KPL; j++) {
    if (j * NT + tid < n) {
      const uint32_t bk = bucket(kv[j]);
      const uint32_t old = atomicAdd(&bcnt[bk >> 1], 1u << ((bk & 1) * 16));
      S.keys[(old >> ((bk & 1) * 16)) & 0xffffu] = kv[j];
    }
  }
  team_sync<NT>();
  uint32_t rk[KPL];
#pragma unroll
  for (int j = 0; j < KPL; j++) {
    rk[j] = 0;
    if (j * NT + tid < n) {
      const uint32_t bk = bucket(kv[j]);
      const uint32_t hi = (bcnt[bk >> 1] >> ((bk & 1) * 16)) & 0xffffu;
      const uint32_t lo = bk ? (bcnt[(bk - 1) >> 1] >> (((bk - 1) & 1) * 16)) & 0xffffu : 0u;
      uint32_t r = lo;
      for (uint32_t i = lo; i < hi; i++) r += S.keys[i] < kv[j];
      rk[j] = r;
    }
  }
  team_sync<NT>();
#pragma unroll
  for (int j = 0; j < KPL; j++)
    if (j * NT + tid < n) S.keys[rk[j]] = kv[j];
  team_sync<NT>();
  return true;
}

template <int NT, int CAP>
__device__ bool team_reg_bucket_sort(BlobShared<NT, CAP>& S, const uint64_t* keys, int n) {
  constexpr int KPL = CAP / NT;
  const int tid = team_rank<NT>();
  uint64_t kv[KPL];
#pragma unroll
  for (int j = 0; j < KPL; j++) {
    const int t = j * NT + tid;
    kv[j] = t < n ? keys[t] : ~0ull;
  }
  return team_reg_bucket_sort_kv<NT, CAP>(S, kv, n);
}

// Inclusive prefix moments P(i) of the blob's points: the owning chunk's base
// plus the chunk's words up to i.  Called by every lane of the team (the base
// of a wave-sized team comes by lane shuffle); inactive lanes get zero.
template <int NT, int CAP>
__device__ __forceinline__ Mom6 prefix_at(const BlobShared<NT, CAP>& S, const uint32_t* cw, const Mom6& cbase,
                                          uint32_t c, uint32_t i, bool active) {
  const uint32_t o = active ? i / c : 0;
  Mom6 p;
  if constexpr (NT == 64) {
    p = mom_shfl(cbase, (int)o);
  } else {
    p = Mom6{S.bMx[o], S.bMy[o], S.bW[o], S.bMxx[o], S.bMyy[o], S.bMxy[o]};
  }
  if (!active) return mom_zero();
  for (uint32_t j = o * c; j <= i; j++) mom_add(p, point_mom(cw[j]));
  return p;
}

// Latency mode: k_extents' work for one small candidate (<= kSmallBlob points)
// inside the small-blob wave itself: MinMaxExtents (P3), SelectBlobs (P4) and the
// (theta, plane, y, x) keys with the line-fit weight (P5, TransformLineFitPoint),
// the same expressions as extents_item, but the keys stay in registers (slot
// t = j * 64 + lane) for the sort: no key store and reload through HBM, no
// separate launch: 6 us less on the B = 1 chain.  (Throughput mode keeps
// k_extents: the fused item's extra dependent round trip, with four waves per
// SIMD, costs more there than the key store and reload.)  Returns SelectBlobs'
// decision (uniform across the wave).
__device__ bool small_extents_keys(const DevBufs& b, const Geom& g, int f, uint32_t rank, uint32_t n,
                                   const uint32_t* grp, uint64_t (&kv)[kSmallBlob / 64]) {
  constexpr int U = kSmallBlob / 64;
  const int lane = (int)lane_id();
  const uint8_t* dec = b.dec + (size_t)f * g.Wd * g.Hd;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t t = (uint32_t)(u * 64 + lane);
    kv[u] = t < n ? grp[t] : 0;
  }
  uint32_t mnx = 0xffff, mny = 0xffff, mxx = 0, mxy = 0;
  int32_t sgx = 0, sgy = 0;
  int64_t spg = 0;
#pragma unroll
  for (int u = 0; u < U; u++) {
    if ((uint32_t)(u * 64 + lane) >= n) continue;
    const uint64_t k = kv[u];
    const int dxy = (int)(k & 3);
    const uint32_t px = ((k >> 14) & 0x3ff) * 2 + dx_of(dxy);
    const uint32_t py = ((k >> 4) & 0x3ff) * 2 + dy_of(dxy);
    const bool b2w = (k & 8) != 0;
    const int gx = b2w ? dx_of(dxy) : -dx_of(dxy), gy = b2w ? dy_of(dxy) : -dy_of(dxy);
    mnx = min(mnx, px); mxx = max(mxx, px); mny = min(mny, py); mxy = max(mxy, py);
    sgx += gx; sgy += gy;
    spg += (int64_t)px * gx + (int64_t)py * gy;
  }
  Ext e;
  e.min_x = wave_reduce(mnx, MinOp()); e.max_x = wave_reduce(mxx, MaxOp());
  e.min_y = wave_reduce(mny, MinOp()); e.max_y = wave_reduce(mxy, MaxOp());
  e.gx_sum = wave_reduce(sgx, AddOp()); e.gy_sum = wave_reduce(sgy, AddOp());
  e.pg_sum = wave_reduce(spg, AddOp());
  e.count = n;
  bool keep = (int)((e.max_x - e.min_x) * (e.max_y - e.min_y)) >= g.min_tag_width;
  keep = keep && !((double)ext_dot(e) < 0.0);
  if (!keep) return false;
  if (lane == 0) b.pair_sel[(size_t)f * kMaxPairs + rank] = 1;  // (parity taps, host statistics)
  const double cx = ext_cx(e), cy = ext_cy(e);
  uint32_t gp[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t k = kv[u];
    const int dxy = (int)(k & 3);
    const int32_t ix = (int32_t)(((k >> 14) & 0x3ff) * 2 + dx_of(dxy) + 1) / 2;
    const int32_t iy = (int32_t)(((k >> 4) & 0x3ff) * 2 + dy_of(dxy) + 1) / 2;
    const bool in = (uint32_t)(u * 64 + lane) < n && ix > 0 && ix + 1 < g.Wd && iy > 0 && iy + 1 < g.Hd;
    const int32_t at = in ? iy * g.Wd + ix : g.Wd + 1;
    gp[u] = (uint32_t)dec[at - 1] | ((uint32_t)dec[at + 1] << 8) | ((uint32_t)dec[at - g.Wd] << 16) |
            ((uint32_t)dec[at + g.Wd] << 24);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    if ((uint32_t)(u * 64 + lane) >= n) {
      kv[u] = ~0ull;
      continue;
    }
    const uint64_t k = kv[u];
    const int dxy = (int)(k & 3);
    const uint32_t bx = (k >> 14) & 0x3ff, by = (k >> 4) & 0x3ff;
    const uint32_t px = bx * 2 + dx_of(dxy), py = by * 2 + dy_of(dxy);
    const float dyf = (float)((double)py - cy);
    const float dxf = (float)((double)px - cx);
    const float theta = (float)(((double)det_atan2f(dyf, dxf) + 3.14159265358979323846) * 8e6);
    long long ti = (long long)rintf(theta);
    if (ti < 0) ti = 0;
    const int32_t ix = (int32_t)(px + 1) / 2, iy = (int32_t)(py + 1) / 2;
    int32_t Wt = 1;
    if (ix > 0 && ix + 1 < g.Wd && iy > 0 && iy + 1 < g.Hd) {
      const int32_t gxv = (int32_t)((gp[u] >> 8) & 0xff) - (int32_t)(gp[u] & 0xff);
      const int32_t gyv = (int32_t)(gp[u] >> 24) - (int32_t)((gp[u] >> 16) & 0xff);
      Wt = lf_weight(gxv, gyv);
    }
    kv[u] = ((uint64_t)(ti & 0xfffffff) << kKeyTheta) | ((uint64_t)dxy << 30) | ((uint64_t)by << 20) |
            ((uint64_t)bx << 10) | (((k >> 3) & 1) << 9) | (uint64_t)Wt;
  }
  return true;
}

// Latency mode, large candidates (> kSmallBlob points, a workgroup team): the
// same as small_extents_keys -- MinMaxExtents, SelectBlobs, the (theta, plane, y,
// x) keys with the line-fit weight in registers (slot t = j * NT + tid) -- so
// k_extents drops out of the B = 1 chain.  Returns SelectBlobs' decision
// (uniform across the team).
template <int NT, int CAP>
__device__ bool large_extents_keys(const DevBufs& b, const Geom& g, BlobShared<NT, CAP>& S, int f, uint32_t rank,
                                   uint32_t n, const uint32_t* grp, uint64_t (&kv)[CAP / NT]) {
  constexpr int U = CAP / NT;
  const int tid = team_rank<NT>();
  const uint8_t* dec = b.dec + (size_t)f * g.Wd * g.Hd;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t t = (uint32_t)(u * NT + tid);
    kv[u] = t < n ? grp[t] : 0;
  }
  uint32_t mnx = 0xffff, mny = 0xffff, mxx = 0, mxy = 0;
  int32_t sgx = 0, sgy = 0;
  int64_t spg = 0;
#pragma unroll
  for (int u = 0; u < U; u++) {
    if ((uint32_t)(u * NT + tid) >= n) continue;
    const uint64_t k = kv[u];
    const int dxy = (int)(k & 3);
    const uint32_t px = ((k >> 14) & 0x3ff) * 2 + dx_of(dxy);
    const uint32_t py = ((k >> 4) & 0x3ff) * 2 + dy_of(dxy);
    const bool b2w = (k & 8) != 0;
    const int gx = b2w ? dx_of(dxy) : -dx_of(dxy), gy = b2w ? dy_of(dxy) : -dy_of(dxy);
    mnx = min(mnx, px); mxx = max(mxx, px); mny = min(mny, py); mxy = max(mxy, py);
    sgx += gx; sgy += gy;
    spg += (int64_t)px * gx + (int64_t)py * gy;
  }
  team_extents<NT, CAP>(S, mnx, mxx, mny, mxy, sgx, sgy, spg);
  Ext e;
  e.min_x = mnx; e.max_x = mxx; e.min_y = mny; e.max_y = mxy;
  e.gx_sum = sgx; e.gy_sum = sgy; e.pg_sum = spg;
  e.count = n;
  bool keep = (int)((e.max_x - e.min_x) * (e.max_y - e.min_y)) >= g.min_tag_width;
  keep = keep && !((double)ext_dot(e) < 0.0);
  if (!keep) return false;
  if (tid == 0) b.pair_sel[(size_t)f * kMaxPairs + rank] = 1;  // (parity taps, host statistics)
  const double cx = ext_cx(e), cy = ext_cy(e);
  uint32_t gp[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t k = kv[u];
    const int dxy = (int)(k & 3);
    const int32_t ix = (int32_t)(((k >> 14) & 0x3ff) * 2 + dx_of(dxy) + 1) / 2;
    const int32_t iy = (int32_t)(((k >> 4) & 0x3ff) * 2 + dy_of(dxy) + 1) / 2;
    const bool in = (uint32_t)(u * NT + tid) < n && ix > 0 && ix + 1 < g.Wd && iy > 0 && iy + 1 < g.Hd;
    const int32_t at = in ? iy * g.Wd + ix : g.Wd + 1;
    gp[u] = (uint32_t)dec[at - 1] | ((uint32_t)dec[at + 1] << 8) | ((uint32_t)dec[at - g.Wd] << 16) |
            ((uint32_t)dec[at + g.Wd] << 24);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    if ((uint32_t)(u * NT + tid) >= n) {
      kv[u] = ~0ull;
      continue;
    }
    const uint64_t k = kv[u];
    const int dxy = (int)(k & 3);
    const uint32_t bx = (k >> 14) & 0x3ff, by = (k >> 4) & 0x3ff;
    const uint32_t px = bx * 2 + dx_of(dxy), py = by * 2 + dy_of(dxy);
    const float dyf = (float)((double)py - cy);
    const float dxf = (float)((double)px - cx);
    const float theta = (float)(((double)det_atan2f(dyf, dxf) + 3.14159265358979323846) * 8e6);
    long long ti = (long long)rintf(theta);
    if (ti < 0) ti = 0;
    const int32_t ix = (int32_t)(px + 1) / 2, iy = (int32_t)(py + 1) / 2;
    int32_t Wt = 1;
    if (ix > 0 && ix + 1 < g.Wd && iy > 0 && iy + 1 < g.Hd) {
      const int32_t gxv = (int32_t)((gp[u] >> 8) & 0xff) - (int32_t)(gp[u] & 0xff);
      const int32_t gyv = (int32_t)(gp[u] >> 24) - (int32_t)((gp[u] >> 16) & 0xff);
      Wt = lf_weight(gxv, gyv);
    }
    kv[u] = ((uint64_t)(ti & 0xfffffff) << kKeyTheta) | ((uint64_t)dxy << 30) | ((uint64_t)by << 20) |
            ((uint64_t)bx << 10) | (((k >> 3) & 1) << 9) | (uint64_t)Wt;
  }
  return true;
}

// Processes one work item (frame, pair rank) with a team of NT threads.
// gpk: this team's global overflow area for peak keys beyond kPeakCap (large
// blobs only; nullptr when the LDS area always suffices).
// A work item's pair-table entries (count, segment offset, SelectBlobs flag),
// loaded one item ahead by the persistent loops so their round trip overlaps
// the previous blob's work.
struct PairInfo {
  uint32_t n, off, sel;
};
__device__ __forceinline__ PairInfo load_pair_info(const DevBufs& b, uint32_t w) {
  const size_t i = (size_t)(w >> 16) * kMaxPairs + (w & 0xffff);
  return PairInfo{b.pair_cnt[i], b.pair_off[i], b.pair_sel[i]};
}


template <int NT, int CAP, bool FUSE = false>
__device__ void blob_item(const DevBufs& b, const Geom& g, const Params& prm, BlobShared<NT, CAP>& S, uint64_t* gpk,
                          const uint32_t* combo, uint32_t w, PairInfo pi_, uint32_t* pacc) {
  constexpr int kC = (CAP + NT - 1) / NT;  // max points per thread chunk
  static_assert(kC <= 32, "chunk too long");
  const int tid = team_rank<NT>();
  const uint32_t lane = lane_id();
  // AT_PHASE_PROBE: accumulated wall-clock per phase (probe[64 + 16*(NT>64) + k]);
  // the accumulators live in the team's LDS, not in registers
  if (AT_PROBE_ON(prm) && tid == 0) S.t_last = S.t_item = wall_clock64();
  bool big = false;
  auto phase = [&](int k) {  // accumulated per team, flushed once per kernel
    if (AT_PROBE_ON(prm) && tid == 0) {
      if (k == 9) __builtin_amdgcn_s_waitcnt(0);  // the item's stores are acknowledged inside its own time
      const uint64_t now = wall_clock64();
      pacc[k] += (uint32_t)(now - S.t_last);
      S.ph[k] = (uint32_t)(now - S.t_last);
      pacc[10 + k] += 1;
      if (NT > 64 && big) {  // the few very large blobs (> 2048 points) separately: probe[208 + k], count [220]
        atomicAdd((unsigned long long*)&b.probe[208 + k], (unsigned long long)(now - S.t_last));
        if (k == 0) atomicAdd((unsigned long long*)&b.probe[220], 1ull);
      }
      S.t_last = now;
    }
  };
  const int f = (int)(w >> 16);
  const uint32_t rank = w & 0xffff;
  const uint32_t n = pi_.n;
  big = n > 2048;
  const uint32_t* grp = b.grp + (size_t)f * g.cap_pts + pi_.off;  // points (fused extents)
  uint64_t* keys = b.keys + (size_t)f * g.cap_pts + pi_.off;      // k_extents' sort keys

  // extents, SelectBlobs and the theta keys: from k_extents, or here (FUSE)
  bool sorted = false, in_lds = false;
  const uint32_t bi = rank & 0xfff;
  if constexpr (NT > 64 && FUSE) {
    uint64_t kv[CAP / NT];
    if (!large_extents_keys<NT, CAP>(b, g, S, f, rank, n, grp, kv)) return;  // uniform across the team
    if (tid == 0) pacc[20] += n;
    phase(0);
    phase(1);
    sorted = team_reg_bucket_sort_kv<NT, CAP>(S, kv, (int)n);  // n > kSmallBlob >= 64
    in_lds = true;
  } else if constexpr (NT == 64 && FUSE) {
    uint64_t kv[kSmallBlob / 64];
    if (!small_extents_keys(b, g, f, rank, n, grp, kv)) return;  // uniform across the wave
    if (tid == 0) pacc[20] += n;
    phase(0);
    phase(1);
    if (n >= 64) {
      sorted = wave_bucket_sort_kv<CAP>(S, kv, (int)n);
    } else {
#pragma unroll
      for (int j = 0; j < kSmallBlob / 64; j++)
        if (j * 64 + (int)lane < (int)n) S.keys[j * 64 + lane] = kv[j];
      team_sync<NT>();
      sorted = team_bucket_sort<NT, CAP>(S, (int)n);
    }
    in_lds = true;
  } else {
  if (pi_.sel == 0) return;  // uniform across the team
  if (tid == 0) pacc[20] += n;  // points of kept blobs this team processed (batch statistics)
  phase(0);
  if constexpr (NT == 64) {
    if (n >= 64) {  // keys go straight from global memory into registers
      phase(1);
      sorted = wave_bucket_sort<CAP>(S, keys, (int)n);
      in_lds = true;
    }
  } else if constexpr (CAP / NT <= 16) {
    if (n >= 64) {
      phase(1);
      sorted = team_reg_bucket_sort<NT, CAP>(S, keys, (int)n);
      in_lds = true;
    }
  }
  if (!sorted && !in_lds) {
    for (uint32_t t = tid; t < n; t += NT) S.keys[t] = keys[t];
    phase(1);
    team_sync<NT>();
    sorted = team_bucket_sort<NT, CAP>(S, (int)n);
  }
  }
  if (!sorted) {
    int np2 = 64;
    while (np2 < (int)n) np2 <<= 1;
    for (int t = (int)n + tid; t < np2; t += NT) S.keys[t] = ~0ull;
    team_sync<NT>();
    team_bitonic_sort<uint64_t, NT>(S.keys, np2);
  }
  phase(2);
  if (AT_DIAG_STOP(prm, 2)) return;

  // ---- line-fit points (P7): blocked chunks, W from the decimated gradient,
  // sorted keys -> compact words in place; chunk sums -> exclusive team scan
  const uint32_t c = (n + NT - 1) / NT;
  const uint32_t t0 = min(n, (uint32_t)tid * c), t1 = min(n, t0 + c);
  uint32_t* cw = reinterpret_cast<uint32_t*>(S.keys);
  float* errv = reinterpret_cast<float*>(S.keys) + CAP;
  uint32_t word[kC];
  Mom6 csum = mom_zero();
#pragma unroll
  for (int k = 0; k < kC; k++) {
    word[k] = 0;
    if (k >= (int)c) break;  // c is uniform across the team
    const uint32_t t = t0 + k;
    if (t < t1) {
      const uint64_t sk = S.keys[t];
      word[k] = compact_word(sk);
      // parity tap: IndexPoint key (blob, theta, point bits) in place of the grouped point
      const uint64_t pbits = (((sk >> 10) & 0x3ff) << 14) | (((sk >> 20) & 0x3ff) << 4) | (((sk >> 9) & 1) << 3) |
                             ((sk >> 30) & 3);
      if (prm.taps) keys[t] = ((uint64_t)bi << 52) | (((sk >> kKeyTheta) & 0xfffffff) << 24) | pbits;
      mom_add(csum, point_mom(word[k]));
    }
  }
  team_sync<NT>();  // every key read before the compact words overwrite them
#pragma unroll
  for (int k = 0; k < kC; k++) {
    if (k >= (int)c) break;
    if (t0 + k < t1) cw[t0 + k] = word[k];
  }
  Mom6 total;
  const Mom6 cbase = team_excl_scan_mom<NT, CAP>(S, csum, &total);
  if constexpr (NT > 64) {
    S.bMx[tid] = cbase.Mx; S.bMy[tid] = cbase.My; S.bW[tid] = cbase.W;
    S.bMxx[tid] = cbase.Mxx; S.bMyy[tid] = cbase.Myy; S.bMxy[tid] = cbase.Mxy;
  }
  team_sync<NT>();
  phase(3);
  if (AT_DIAG_STOP(prm, 3)) return;

  // ---- errors (K10 ErrorCalculator, restated per blob, cyclic): the window
  // [t0 - ksz, t0 + ksz] of the chunk's first point from two prefix lookups
  // (P(hi) - P(lo - 1), plus the total when it wraps), then slid across the chunk
  const uint32_t ksz = n / 12 < 20 ? n / 12 : 20;
  const int32_t Nw = (int32_t)(2 * ksz + 1);
  const bool act = t0 < t1;
  {
    const int lo = (int)t0 - (int)ksz, hi = (int)t0 + (int)ksz;
    const int ia = hi >= (int)n ? hi - (int)n : hi;
    const int ib = (lo >= 0 ? lo : lo + (int)n) - 1;
    const Mom6 pa = prefix_at<NT, CAP>(S, cw, cbase, c, (uint32_t)ia, act);
    const Mom6 pb = prefix_at<NT, CAP>(S, cw, cbase, c, (uint32_t)(ib >= 0 ? ib : 0), act && ib >= 0);
    Mom6 s = pa;
    mom_sub(s, pb);
    if (lo < 0 || hi >= (int)n) mom_add(s, total);
    if (act) errv[t0] = window_err(s, Nw);
    for (uint32_t t = t0 + 1; t < t1; t++) {
      uint32_t ja = t + ksz, jr = t + n - ksz - 1;
      ja -= ja >= n ? n : 0;
      jr -= jr >= n ? n : 0;
      mom_add(s, point_mom(cw[ja]));
      mom_sub(s, point_mom(cw[jr]));
      errv[t] = window_err(s, Nw);
    }
  }
  team_sync<NT>();
  phase(4);

  // ---- 7-tap filter and strict local maxima; peak keys (P8-P10: -filtered
  // error in cub's float radix order, then point index).  Each thread keeps its
  // chunk's peaks in registers: strict maxima are never adjacent, so chunk
  // position k has slot k / 2 to itself
  // the chunk's error window errv[t0 - 4 .. t0 + kC + 3] (cyclic) staged in
  // registers, every LDS read issued at once; filt(k) = filtered error of point
  // t0 + k, k = -1 .. c, summed in the reference's tap order
  constexpr int kEW = kC + 8;
  float ew[kEW];
  if (t0 < t1) {
#pragma unroll
    for (int j = 0; j < kEW; j++) {
      uint32_t idx = t0 + 2 * n + j - 4;
      idx -= idx >= n ? n : 0;
      idx -= idx >= n ? n : 0;
      idx -= idx >= n ? n : 0;
      ew[j] = errv[idx];
    }
  }
  auto filt_k = [&](int k) -> double {  // k + 1 + j indexes ew: constant after unrolling
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 7; j++) acc += (double)ew[k + 1 + j] * (double)c_filter[j];
    return acc;
  };
  constexpr int kPR = (kC + 1) / 2;
  uint64_t mine[kPR];
#pragma unroll
  for (int j = 0; j < kPR; j++) mine[j] = ~0ull;
  uint32_t nmine = 0;
  if (t0 < t1) {
    double fprev = filt_k(-1), fcur = filt_k(0);
#pragma unroll
    for (int k = 0; k < kC; k++) {
      const uint32_t t = t0 + k;
      if (k >= (int)c || t >= t1) break;
      const double fnext = filt_k(k + 1);
      if (fcur > fprev && fcur > fnext) {
        const float ef = (float)(-fcur);
        uint32_t u = __float_as_uint(ef);
        u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // cub radix float order
        mine[k >> 1] = ((uint64_t)u << 32) | t;
        nmine++;
      }
      fprev = fcur;
      fcur = fnext;
    }
  }
  const uint32_t npk = team_reduce<NT>(nmine, AddOp(), S.red_u32);
  uint64_t* pks = S.pks;
  {
    // FitQuads reads only the first min(10, npk) entries of the peak order (P9
    // sorts all of a blob's peaks): select them -- 10 rounds of a team minimum
    // over the keys (unique: the point index is in the low word) above the
    // previous pick -- instead of sorting every peak
    const int ntop = npk < (uint32_t)kNMaxima ? (int)npk : kNMaxima;
    uint64_t last = 0;
    if constexpr (NT == 64) {
      if (npk <= 64) {  // (uniform) the usual blob: the peaks compacted in LDS, each lane ranks one
        uint64_t* pall = reinterpret_cast<uint64_t*>(errv);  // (errv is dead: staged in ew)
        team_sync<64>();
        uint32_t pos = wave_incl_scan(nmine, AddOp(), 0u) - nmine;
#pragma unroll
        for (int j = 0; j < kPR; j++)
          if (mine[j] != ~0ull) pall[pos++] = mine[j];
        team_sync<64>();
        if (lane < npk) {
          const uint64_t pv = pall[lane];
          uint32_t r = 0;
          for (uint32_t j = 0; j < npk; j++) r += pall[j] < pv;  // (broadcast reads)
          if (r < (uint32_t)kNMaxima) pks[r] = pv;
        }
      } else {
      for (int r = 0; r < ntop; r++) {
        uint64_t m = ~0ull;
#pragma unroll
        for (int j = 0; j < kPR; j++) {
          const uint64_t k = mine[j];
          if ((r == 0 || k > last) && k < m) m = k;
        }
        m = wave_reduce(m, MinOp());
        if (tid == 0) pks[r] = m;
        last = m;
      }
      }
    } else {
      // every wave selects its own top ntop (wave minima, no barriers), then wave 0
      // the top ntop of those candidates: the team's top ntop is among them
      const int w = tid >> 6, ln = tid & 63;
      for (int r = 0; r < ntop; r++) {
        uint64_t m = ~0ull;
#pragma unroll
        for (int j = 0; j < kPR; j++) {
          const uint64_t k = mine[j];
          if ((r == 0 || k > last) && k < m) m = k;
        }
        m = wave_reduce(m, MinOp());
        if (ln == 0) S.wtop[w * kNMaxima + r] = m;
        last = m;
      }
      team_sync<NT>();
      if (w == 0) {
        constexpr int NC = NT / 64 * kNMaxima;  // <= 80 candidates, two per lane
        uint64_t c0 = ~0ull, c1 = ~0ull;
        if (ln < NC && (ln % kNMaxima) < ntop) c0 = S.wtop[ln];
        if (ln + 64 < NC && ((ln + 64) % kNMaxima) < ntop) c1 = S.wtop[ln + 64];
        last = 0;
        for (int r = 0; r < ntop; r++) {
          uint64_t m = ~0ull;
          if ((r == 0 || c0 > last) && c0 < m) m = c0;
          if ((r == 0 || c1 > last) && c1 < m) m = c1;
          m = wave_reduce(m, MinOp());
          if (ln == 0) pks[r] = m;
          last = m;
        }
      }
    }
    team_sync<NT>();
  }
  phase(5);
  if (AT_DIAG_STOP(prm, 4)) return;
  // ---- FitQuads (K11) --------------------------------------------------------
  const int cnt = (int)npk;
  if (tid < 16) {
    // top min(10, cnt) peaks, re-sorted by point index (WarpMergeSort), pad 0xffff
    const int v = (tid < cnt && tid < kNMaxima) ? (int)(pks[tid] & 0xffffffffu) : 0xffff;
    int r = 0;
    for (int j = 0; j < 16; j++) {
      const int u = (j < cnt && j < kNMaxima) ? (int)(pks[j] & 0xffffffffu) : 0xffff;
      r += (u < v) || (u == v && j < tid);
    }
    S.pi[r] = v;
  }
  team_sync<NT>();
  // inclusive prefix moments at pi[k], pi[k] - 1 and n - 1: the owning chunk's
  // base plus the chunk's words up to the index
  {
    const int k = tid;
    uint32_t idx = 0;
    bool need = false;
    if (k < 10) { need = k < cnt && k < kNMaxima; idx = need ? (uint32_t)S.pi[k] : 0; }
    else if (k < 20) { need = k - 10 < cnt && k - 10 < kNMaxima && S.pi[k - 10] > 0; idx = need ? (uint32_t)S.pi[k - 10] - 1 : 0; }
    else if (k == 20) { need = true; idx = n - 1; }
    const Mom6 p = prefix_at<NT, CAP>(S, cw, cbase, c, idx, need);
    if (need) {
      S.tMx[k] = p.Mx; S.tMy[k] = p.My; S.tW[k] = p.W;
      S.tMxx[k] = p.Mxx; S.tMyy[k] = p.Myy; S.tMxy[k] = p.Mxy;
    }
  }
  team_sync<NT>();
  phase(6);
  // read_moments (line_fit_filter.cu:745-796) of the segment pi[a] -> pi[b]
  auto seg_moments = [&](int a, int bb) -> Moments {
    const uint32_t i0 = (uint32_t)S.pi[a], i1 = (uint32_t)S.pi[bb];
    Mom6 m = Mom6{S.tMx[bb], S.tMy[bb], S.tW[bb], S.tMxx[bb], S.tMyy[bb], S.tMxy[bb]};
    const Mom6 pm = Mom6{S.tMx[10 + a], S.tMy[10 + a], S.tW[10 + a], S.tMxx[10 + a], S.tMyy[10 + a], S.tMxy[10 + a]};
    int32_t N;
    if (i0 < i1) {
      if (i0 > 0) mom_sub(m, pm);
      N = (int32_t)(i1 - i0 + 1);
    } else {
      Mom6 z = Mom6{S.tMx[20], S.tMy[20], S.tW[20], S.tMxx[20], S.tMyy[20], S.tMxy[20]};
      mom_sub(z, pm);
      mom_add(z, m);
      m = z;
      N = (int32_t)(n - i0 + i1 + 1);
    }
    return to_moments(m, N);
  };
  // every segment a combination can use, fitted once (FitLine on the same
  // moments as QuadFitCalculator's per-combination fits: identical results),
  // over the key area (its compact words were last read by the prefix lookups)
  SegFits& seg = *reinterpret_cast<SegFits*>(S.keys);
  static_assert(sizeof(SegFits) <= sizeof(S.keys), "segment fits must fit over the keys");
  // the cn x cn (segment start, end) pairs of the top cn = min(cnt, 10) peaks, one per
  // lane (cn <= 8: one round)
  const int cn = min(cnt, kNMaxima);
  const float rcn = 1.0f / (float)max(cn, 1);
  for (int ci = tid; cnt >= 4 && ci < cn * cn; ci += NT) {
    const int a = (int)(((float)ci + 0.5f) * rcn), bb = ci - a * cn;  // (exact: ci + 0.5 is >= 0.05 from a multiple of cn)
    if (a != bb) {
      const LineFitOut o = fit_line_v<false, true>(seg_moments(a, bb));
      seg.err[a][bb] = o.err;
      seg.mse[a][bb] = o.mse;
      seg.p[a][bb][0] = o.p23[0];
      seg.p[a][bb][1] = o.p23[1];
    }
  }
  team_sync<NT>();
  phase(7);
  if (AT_DIAG_STOP(prm, 7)) return;
  // the C(cnt, 4) valid combinations (the first in colexicographic order); each lane
  // keeps its minimum, the lowest lexicographic index on ties (the reference's first)
  double err = DBL_MAX;
  uint32_t bt = 0xffffffffu;
  const double mse_max = (double)prm.max_line_fit_mse;
  const int ncomb = cnt < 4 ? 0 : cnt >= kNMaxima ? 210 : (cnt * (cnt - 1) * (cnt - 2) * (cnt - 3)) / 24;
  for (int cj = tid; cj < ncomb; cj += NT) {
    double e4 = DBL_MAX;
    const int ci = (int)combo[210 + cj];
    {
      const uint32_t cb = combo[ci];  // LDS copy of c_combo: no vector-memory wait in this loop
      const int m0 = cb & 0xff, m1 = (cb >> 8) & 0xff, m2 = (cb >> 16) & 0xff, m3 = cb >> 24;
      if (!(seg.mse[m0][m1] > mse_max)) {
        if (!(seg.mse[m1][m2] > mse_max)) {
          const double dot =
              seg.p[m0][m1][0] * seg.p[m1][m2][0] + seg.p[m0][m1][1] * seg.p[m1][m2][1];
          if (!(fabs(dot) > prm.cos_critical_rad)) {
            if (!(seg.mse[m2][m3] > mse_max) && !(seg.mse[m3][m0] > mse_max))
              e4 = seg.err[m0][m1] + seg.err[m1][m2] + seg.err[m2][m3] + seg.err[m3][m0];
          }
        }
      }
    }
    if (bt == 0xffffffffu || e4 < err || (e4 == err && (uint32_t)ci < bt)) { err = e4; bt = (uint32_t)ci; }
  }
  // BlockReduce(MinQuadError): minimum error, first (lowest) combination on ties
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const double oe = __shfl_xor(err, d);
    const uint32_t ot = __shfl_xor(bt, d);
    if (oe < err || (oe == err && ot < bt)) { err = oe; bt = ot; }
  }
  if constexpr (NT > 64) {
    if (lane == 0) { S.red_f64[tid >> 6] = err; S.red_idx[tid >> 6] = bt; }
    team_sync<NT>();
    err = S.red_f64[0];
    bt = S.red_idx[0];
    for (int i = 1; i < NT / 64; i++)
      if (S.red_f64[i] < err || (S.red_f64[i] == err && S.red_idx[i] < bt)) { err = S.red_f64[i]; bt = S.red_idx[i]; }
  }
  phase(8);
  if (AT_DIAG_STOP(prm, 8)) return;
  const double best = err;
  if (bt >= 210) bt = 0;
  const bool valid = best < (double)(prm.max_line_fit_mse * (float)n);
  uint16_t qidx[4];
  const uint32_t cbt = combo[bt];
  for (int k = 0; k < 4; k++) qidx[k] = (uint16_t)S.pi[(cbt >> (8 * k)) & 0xff];
  if constexpr (!FUSE) {
    // throughput mode: the side segments' moments for k_quad_fin (a thread per blob
    // there, instead of a few lanes of this team on a serial fp64 chain here)
    QuadPend& qp = b.qpend[(size_t)f * kMaxPairs + rank];
    if (valid && tid < 4) {
      float pre[4];
      double e_, m_;
      fit_line(seg_moments((cbt >> (8 * tid)) & 0xff, (cbt >> (8 * ((tid + 1) & 3))) & 0xff), nullptr, nullptr, &e_, &m_,
               pre);
      *reinterpret_cast<float4*>(qp.fit[tid]) = make_float4(pre[0], pre[1], pre[2], pre[3]);
    }
    if (tid == 0) {
      qp.blob_index = bi;
      qp.valid = valid;
      for (int k = 0; k < 4; k++) qp.indices[k] = qidx[k];
      pacc[21] += 1;  // FitQuads records of this team (batch statistics)
    }
    phase(9);
    team_sync<NT>();
    return;
  }
  // UpdateFitQuads (apriltag_detect.cu:98-241): side lines in parallel, rest on one lane
  if (valid && tid < 4) {
    const LineFitOut o =
        fit_line_v<true, true>(seg_moments((cbt >> (8 * tid)) & 0xff, (cbt >> (8 * ((tid + 1) & 3))) & 0xff));
    S.lines[tid][0] = o.p01[0];
    S.lines[tid][1] = o.p01[1];
    S.lines[tid][2] = o.p23[0];
    S.lines[tid][3] = o.p23[1];
  }
  team_sync<NT>();
  // the four corners (lanes 0-3), the six Heron sides (lanes 0-5) and the four
  // corner angles (lanes 0-3) of wave 0 in parallel, each with the reference's
  // float / double expression; the record is then written by lane 0
  if (tid < 64) {
    const uint32_t ln = lane_id();
    float cxk = 0.f, cyk = 0.f;
    bool cok = true;
    if (valid && ln < 4) {
      const int k = (int)ln, k1 = (k + 1) & 3;
      const double A00 = S.lines[k][3], A01 = -S.lines[k1][3];
      const double A10 = -S.lines[k][2], A11 = S.lines[k1][2];
      const double B0 = -S.lines[k][0] + S.lines[k1][0];
      const double B1 = -S.lines[k][1] + S.lines[k1][1];
      const double det = A00 * A11 - A10 * A01;
      const double W00 = A11 / det, W01 = -A01 / det;
      cok = !(fabs(det) < 0.001);
      if (cok) {
        const double L0 = W00 * B0 + W01 * B1;
        cxk = (float)(S.lines[k][0] + L0 * A00);
        cyk = (float)(S.lines[k][1] + L0 * A10);
      }
    }
    int ok = valid && __ballot(ln < 4 && !cok) == 0;
    float qc[4][2];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      qc[k][0] = wave_read(cxk, k);
      qc[k][1] = wave_read(cyk, k);
    }
    if (ok) {
      // sides of triangles (0,1,2) and (2,3,0): 0->1, 1->2, 2->0, 2->3, 3->0, 0->2
      float lj = 0.f;
      if (ln < 6) {
        const int a2 = ln == 0 ? 0 : ln == 1 ? 1 : ln == 2 ? 2 : ln == 3 ? 2 : ln == 4 ? 3 : 0;
        const int b2 = ln == 0 ? 1 : ln == 1 ? 2 : ln == 2 ? 0 : ln == 3 ? 3 : ln == 4 ? 0 : 2;
        const float xa = a2 == 0 ? qc[0][0] : a2 == 1 ? qc[1][0] : a2 == 2 ? qc[2][0] : qc[3][0];
        const float ya = a2 == 0 ? qc[0][1] : a2 == 1 ? qc[1][1] : a2 == 2 ? qc[2][1] : qc[3][1];
        const float xb = b2 == 0 ? qc[0][0] : b2 == 1 ? qc[1][0] : b2 == 2 ? qc[2][0] : qc[3][0];
        const float yb = b2 == 0 ? qc[0][1] : b2 == 1 ? qc[1][1] : b2 == 2 ? qc[2][1] : qc[3][1];
        lj = det_hypotf(xb - xa, yb - ya);
      }
      float len[6];
#pragma unroll
      for (int j = 0; j < 6; j++) len[j] = wave_read(lj, j);
      float area = 0, pp;
      pp = (len[0] + len[1] + len[2]) / 2;
      area += sqrtf(pp * (pp - len[0]) * (pp - len[1]) * (pp - len[2]));
      pp = (len[3] + len[4] + len[5]) / 2;
      area += sqrtf(pp * (pp - len[3]) * (pp - len[4]) * (pp - len[5]));
      if ((double)area < 0.95 * g.min_tag_width * g.min_tag_width) ok = 0;
    }
    if (ok) {
      bool abad = false;
      if (ln < 4) {
        const int i0 = (int)ln, i1 = (i0 + 1) & 3, i2 = (i0 + 2) & 3;
        auto cx = [&](int i) { return i == 0 ? qc[0][0] : i == 1 ? qc[1][0] : i == 2 ? qc[2][0] : qc[3][0]; };
        auto cy = [&](int i) { return i == 0 ? qc[0][1] : i == 1 ? qc[1][1] : i == 2 ? qc[2][1] : qc[3][1]; };
        const float dx1 = cx(i1) - cx(i0), dy1 = cy(i1) - cy(i0);
        const float dx2 = cx(i2) - cx(i1), dy2 = cy(i2) - cy(i1);
        const float cosd = (dx1 * dx2 + dy1 * dy2) / sqrtf((dx1 * dx1 + dy1 * dy1) * (dx2 * dx2 + dy2 * dy2));
        abad = (double)fabsf(cosd) > prm.cos_critical_rad || dx1 * dy2 < dy1 * dx2;
      }
      if (__ballot(abad)) ok = 0;
    }
  if (ln == 0) {
    QuadRecord rec;
    rec.blob_index = bi;
    rec.valid = valid;
    for (int k = 0; k < 4; k++) rec.indices[k] = qidx[k];
    QuadCand qcand;
    for (int k = 0; k < 4; k++) {  // AdjustPixelCenters, quad_decimate 2
      const float x = ok ? (qc[k][0] - 0.5f) * 2.0f + 0.5f : 0.f;
      const float y = ok ? (qc[k][1] - 0.5f) * 2.0f + 0.5f : 0.f;
      rec.corners[k][0] = qcand.p[k][0] = x;
      rec.corners[k][1] = qcand.p[k][1] = y;
    }
    rec.accepted = ok;
    if (prm.taps) b.quads[(size_t)f * kMaxPairs + rank] = rec;  // slot = pair rank (debug record: taps only)
    pacc[21] += 1;  // FitQuads records of this team (batch statistics, one atomic per team at the end)
    if (ok && !AT_DIAG_STOP(prm, 5)) {
      qcand.frame = (uint32_t)f;
      qcand.rank = rank;
      const uint32_t ci = atomicAdd(b.nqcand + (size_t)f * kQcStride, 1u);  // per-frame counters spread the contention
      if (ci < (uint32_t)kQuadCandPerFrame) b.qcand[(size_t)f * kQuadCandPerFrame + ci] = qcand;
      else atomicOr(b.status + f, kStatusQuadsOverflow);
    }
  }
  }
  phase(9);
  if (AT_PROBE_ON(prm) && tid == 0) {  // slowest item of this team (flushed at kernel end): ticks, points, phases
    const uint32_t dt = (uint32_t)(S.t_last - S.t_item);
    if (dt > S.slow_dt) {
      S.slow_dt = dt;
      S.slow_n = n;
      for (int k = 0; k < 10; k++) S.slow_ph[k] = S.ph[k];
    }
  }
  team_sync<NT>();
}

// s_combo[0, 210): the combinations packed (m0 | m1 << 8 | m2 << 16 | m3 << 24) in
// c_combo's lexicographic order (the reference's tie-break order); s_combo[210, 420):
// c_colex, the lexicographic indices in colexicographic order
__device__ __forceinline__ void load_combos(uint32_t* s_combo, int tid, int nt) {
  for (int i = tid; i < 210; i += nt) {
    s_combo[i] = (uint32_t)c_combo[i][0] | ((uint32_t)c_combo[i][1] << 8) | ((uint32_t)c_combo[i][2] << 16) |
                 ((uint32_t)c_combo[i][3] << 24);
    s_combo[210 + i] = c_colex[i];
  }
}

// ---------------------------------------------------------------------------
// K8b: per candidate pair (one wave each, every size class): MinMaxExtents
// (P3, line_fit_filter.h:14-59), SelectBlobs (apriltag_gpu.cu:534-559; tag36h11:
// normal border only) and, for kept blobs, the (theta, plane, y, x) sort keys of
// P5/P6 (apriltag_gpu.cu:380-412) written over the grouped points in place.
// The blob kernels then see kept blobs only.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool work_item(const DevBufs& b, const uint32_t* cnt, int c0, int c1, uint32_t it,
                                          uint32_t* w) {
  for (int c = c0; c < c1; c++) {
    if (it < cnt[c]) {
      *w = b.work[(size_t)c * b.wcap + it];
      return true;
    }
    it -= cnt[c];
  }
  return false;
}

// One candidate with a team of NT threads (a wave, or the whole workgroup for
// large candidates); red: NT/64 x 8 LDS words for the cross-wave reduction.
template <int NT>
__device__ __forceinline__ void extents_item(const DevBufs& b, const Geom& g, uint32_t w, int64_t (*red)[8]) {
  const int tid = team_rank<NT>();
  const int f = (int)(w >> 16);
  const uint32_t rank = w & 0xffff;
  const uint32_t n = b.pair_cnt[(size_t)f * kMaxPairs + rank];
  const size_t so = (size_t)f * g.cap_pts + b.pair_off[(size_t)f * kMaxPairs + rank];
  const uint32_t* grp = b.grp + so;
  uint64_t* keys = b.keys + so;
  const uint8_t* dec = b.dec + (size_t)f * g.Wd * g.Hd;
  uint32_t mnx = 0xffff, mny = 0xffff, mxx = 0, mxy = 0;
  int32_t sgx = 0, sgy = 0;
  int64_t spg = 0;
  // U points per lane per round, every load of a round issued before any is
  // used; the first round's keys stay in registers for the key pass below
#ifndef AT_EXT_U
#define AT_EXT_U 4
#endif
  constexpr int U = AT_EXT_U;
#ifndef AT_EXT_KEY_UNROLL
#define AT_EXT_KEY_UNROLL 4
#endif
#ifndef AT_EXT_KR
#define AT_EXT_KR 1  // the first round's grouped points kept in registers for the key pass
#endif
  uint32_t kr[U];
  for (uint32_t base = 0; base < n; base += NT * U) {
    uint32_t kk[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t t = base + u * NT + tid;
      kk[u] = t < n ? grp[t] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (AT_EXT_KR && base == 0) kr[u] = kk[u];
      if (base + u * NT + tid >= n) continue;
      const uint64_t k = kk[u];
      const int dxy = (int)(k & 3);
      const uint32_t px = ((k >> 14) & 0x3ff) * 2 + dx_of(dxy);
      const uint32_t py = ((k >> 4) & 0x3ff) * 2 + dy_of(dxy);
      const bool b2w = (k & 8) != 0;
      const int gx = b2w ? dx_of(dxy) : -dx_of(dxy), gy = b2w ? dy_of(dxy) : -dy_of(dxy);
      mnx = min(mnx, px); mxx = max(mxx, px); mny = min(mny, py); mxy = max(mxy, py);
      sgx += gx; sgy += gy;
      spg += (int64_t)px * gx + (int64_t)py * gy;
    }
  }
  mnx = wave_reduce(mnx, MinOp()); mxx = wave_reduce(mxx, MaxOp());
  mny = wave_reduce(mny, MinOp()); mxy = wave_reduce(mxy, MaxOp());
  sgx = wave_reduce(sgx, AddOp()); sgy = wave_reduce(sgy, AddOp());
  spg = wave_reduce(spg, AddOp());
  if constexpr (NT > 64) {
    const int wv = threadIdx.x >> 6;
    if (lane_id() == 0) {
      red[wv][0] = mnx; red[wv][1] = mxx; red[wv][2] = mny; red[wv][3] = mxy;
      red[wv][4] = sgx; red[wv][5] = sgy; red[wv][6] = spg;
    }
    __syncthreads();
    int32_t gx = 0, gy = 0;
    int64_t pg = 0;
    for (int i = 0; i < NT / 64; i++) {
      mnx = min(mnx, (uint32_t)red[i][0]); mxx = max(mxx, (uint32_t)red[i][1]);
      mny = min(mny, (uint32_t)red[i][2]); mxy = max(mxy, (uint32_t)red[i][3]);
      gx += (int32_t)red[i][4]; gy += (int32_t)red[i][5]; pg += red[i][6];
    }
    sgx = gx; sgy = gy; spg = pg;
    __syncthreads();  // red is reused by the next item
  }
  Ext e;
  e.min_x = mnx; e.max_x = mxx; e.min_y = mny; e.max_y = mxy;
  e.gx_sum = sgx; e.gy_sum = sgy; e.pg_sum = spg;
  e.count = n;
  bool keep = (int)((e.max_x - e.min_x) * (e.max_y - e.min_y)) >= g.min_tag_width;
  keep = keep && !((double)ext_dot(e) < 0.0);
  if (!keep) return;  // uniform across the team
  if (tid == 0) b.pair_sel[(size_t)f * kMaxPairs + rank] = 1;
  const double cx = ext_cx(e), cy = ext_cy(e);
  for (uint32_t base = 0; base < n; base += NT * U) {
    uint32_t kk[U];
    uint32_t gp[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t t = base + u * NT + tid;
      kk[u] = (AT_EXT_KR && base == 0) ? kr[u] : (t < n ? grp[t] : 0);
    }
    // line-fit weight of TransformLineFitPoint (apriltag_gpu.cu:631-687): gradient
    // of the decimated image at ((px + 1) / 2, (py + 1) / 2); the four bytes of
    // every point of the round are loaded first (out-of-range: a fixed pixel)
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t k = kk[u];
      const int dxy = (int)(k & 3);
      const int32_t ix = (int32_t)(((k >> 14) & 0x3ff) * 2 + dx_of(dxy) + 1) / 2;
      const int32_t iy = (int32_t)(((k >> 4) & 0x3ff) * 2 + dy_of(dxy) + 1) / 2;
      const bool in = base + u * NT + tid < n && ix > 0 && ix + 1 < g.Wd && iy > 0 && iy + 1 < g.Hd;
      const int32_t at = in ? iy * g.Wd + ix : g.Wd + 1;
      gp[u] = (uint32_t)dec[at - 1] | ((uint32_t)dec[at + 1] << 8) | ((uint32_t)dec[at - g.Wd] << 16) |
              ((uint32_t)dec[at + g.Wd] << 24);
    }
#pragma unroll AT_EXT_KEY_UNROLL
    for (int u = 0; u < U; u++) {
      const uint32_t t = base + u * NT + tid;
      if (t >= n) continue;
      const uint64_t k = kk[u];
      const int dxy = (int)(k & 3);
      const uint32_t bx = (k >> 14) & 0x3ff, by = (k >> 4) & 0x3ff;
      const uint32_t px = bx * 2 + dx_of(dxy), py = by * 2 + dy_of(dxy);
      const float dyf = (float)((double)py - cy);
      const float dxf = (float)((double)px - cx);
      const float theta = (float)(((double)det_atan2f(dyf, dxf) + 3.14159265358979323846) * 8e6);
      long long ti = (long long)rintf(theta);
      if (ti < 0) ti = 0;
      const int32_t ix = (int32_t)(px + 1) / 2, iy = (int32_t)(py + 1) / 2;
      int32_t Wt = 1;
      if (ix > 0 && ix + 1 < g.Wd && iy > 0 && iy + 1 < g.Hd) {
        const int32_t gxv = (int32_t)((gp[u] >> 8) & 0xff) - (int32_t)(gp[u] & 0xff);
        const int32_t gyv = (int32_t)(gp[u] >> 24) - (int32_t)((gp[u] >> 16) & 0xff);
        Wt = lf_weight(gxv, gyv);
      }
      // sort key: order (theta, plane, y, x) == P6 stable order; b2w and W ride in
      // the low bits (never decide: (plane, y, x) is unique)
      keys[t] = ((uint64_t)(ti & 0xfffffff) << kKeyTheta) | ((uint64_t)dxy << 30) | ((uint64_t)by << 20) |
               ((uint64_t)bx << 10) | (((k >> 3) & 1) << 9) | (uint64_t)Wt;
    }
  }
}

// Large candidates (size classes 0-2) one per workgroup, then small ones one
// per wave.
// 4 points per lane in flight and a grid of 1536 persistent workgroups: at 6 waves per
// SIMD (80 VGPRs) k_extents took 0.131 ms per 128 frames against 0.152 at 4 waves / 8
// points per lane (profiles/r04n, r04o); at 5 (below) it runs without spills.
#ifndef AT_EXT_WAVES
#define AT_EXT_WAVES 5  // 6 (80 VGPRs) spilled 10 VGPRs since det_atan2's one-division form: +0.35 MB of
                        // scratch traffic per frame (profiles/r06/pmc_ext_ab.txt); 93 VGPRs fit 5
#endif
#ifndef AT_EXT_GRID
#define AT_EXT_GRID 2560  // workgroups (persistent over the candidates): two full rounds of the 1280 the chip holds at 5 waves per SIMD
                          // (1536 left a partial second round: 0.177 -> 0.160 ms serialized, concurrent
                          // throughput unchanged, profiles/r06/ab720_extents_grid.txt)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(AT_EXT_WAVES))) void k_extents(DevBufs b, Geom g) {
  __shared__ int64_t s_red[4][8];
  kt_begin(b, 7);
  uint32_t cnt[kNumCls], total = 0, nlarge = 0;
#pragma unroll
  for (int c = 0; c < kNumCls; c++) {
    cnt[c] = min(b.ncls[c], b.wcap);
    total += cnt[c];
    if (c < g.nlarge) nlarge += cnt[c];
  }
  for (uint32_t it = blockIdx.x; it < nlarge; it += gridDim.x) {
    uint32_t w = 0;
    work_item(b, cnt, 0, kNumCls, it, &w);
    extents_item<256>(b, g, w, s_red);
  }
  if (g.ctw != 32) {  // latency mode: k_blob_small<true> does the small candidates itself
    const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    for (uint32_t it = nlarge + gw; it < total; it += nw) {
      uint32_t w = 0;
      work_item(b, cnt, 0, kNumCls, it, &w);
      extents_item<64>(b, g, w, nullptr);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) kt_end(b, 7);
}

// slowest item over the teams: probe[200 | 201] = (ticks << 20) | points; the
// phases of the slowest small item of each team summed in probe[224 + k], [234] teams
template <int NT, int CAP>
__device__ __forceinline__ void probe_flush_slow(const DevBufs& b, const Params& prm, const BlobShared<NT, CAP>& S,
                                                 bool leader) {
  if (!AT_PROBE_ON(prm) || !leader || !S.slow_dt) return;
  atomicMax((unsigned long long*)&b.probe[NT == 64 ? 200 : 201], ((unsigned long long)S.slow_dt << 20) | S.slow_n);
  if (NT == 64) {
    for (int k = 0; k < 10; k++) atomicAdd((unsigned long long*)&b.probe[224 + k], (unsigned long long)S.slow_ph[k]);
    atomicAdd((unsigned long long*)&b.probe[234], 1ull);
  }
}

__device__ __forceinline__ void probe_flush(const DevBufs& b, const Params& prm, const uint32_t* pacc, int base,
                                            bool leader) {
  if (!AT_PROBE_ON(prm) || !leader) return;
  for (int k = 0; k < 10; k++) {
    if (pacc[k]) atomicAdd((unsigned long long*)&b.probe[base + k], (unsigned long long)pacc[k]);
    if (pacc[10 + k]) atomicAdd((unsigned long long*)&b.probe[base + 32 + k], (unsigned long long)pacc[10 + k]);
  }
}

// One team of NT threads over the large work list (dynamic dequeue, longest first:
// large blobs vary 8x in cost, and there are few of them, so one atomic per item
// is cheap); `slot` indexes the team's global sort scratch.
template <int NT, int CAP, bool FUSE>
__device__ __forceinline__ void large_blob_loop(const DevBufs& b, const Geom& g, const Params& prm, BlobShared<NT, CAP>& S,
                                const uint32_t* s_combo, const uint32_t* s_cnt, uint32_t nlo, uint32_t slot,
                                int c0, int c1, int launch) {
  const int tid = threadIdx.x;
  uint32_t* pacc = S.pacc;
  if (tid < 22) pacc[tid] = 0;
  if (tid == 0) S.slow_dt = 0;
  uint64_t* gpk = b.s_pk + (size_t)slot * (kSortCap / 2);
  __syncthreads();
  // size classes c0 .. c1-1 (blobs over 4096 points are all in class 0); every launch
  // of the stage dequeues from its own head
  uint32_t nwork = 0;
  for (int c = c0; c < c1; c++) nwork += s_cnt[c];
  uint32_t* head = launch == 0 ? b.workhead : launch == 1 ? b.workhead_small : b.workhead_mid;
  while (true) {
    if (tid == 0) S.item = atomicAdd(head, 1u);
    __syncthreads();
    const uint32_t item = S.item;
    __syncthreads();
    if (item >= nwork) break;
    uint32_t w = 0;
    work_item(b, s_cnt, c0, c1, item, &w);
    const PairInfo pi = FUSE ? PairInfo{b.pair_cnt[(size_t)(w >> 16) * kMaxPairs + (w & 0xffff)], b.pair_off[(size_t)(w >> 16) * kMaxPairs + (w & 0xffff)], 0u} : load_pair_info(b, w);
    if (pi.n > (uint32_t)CAP || pi.n <= nlo) continue;  // the other launch's item (uniform)
    blob_item<NT, CAP, FUSE>(b, g, prm, S, gpk, s_combo, w, pi, pacc);
  }
  __syncthreads();
  probe_flush(b, prm, pacc, 80, tid == 0);
  probe_flush_slow(b, prm, S, tid == 0);
  if (tid == 0 && pacc[20]) atomicAdd(b.blob_pts + 1, pacc[20]);
  if (tid == 0 && pacc[21]) atomicAdd(b.nquads, pacc[21]);  // batch total in nquads[0]
}

// One wave over the small work list: wave `wv` of `nwaves` takes items wv, wv +
// nwaves, ... (static round-robin over the size-ordered list: no dequeue atomic --
// a device-scope atomic on one hot address is serviced at the memory side; one per
// small blob serialized every wave of the chip behind that address).  Software
// pipeline: the work entry two items ahead and the pair-table entries one item
// ahead are in flight while a blob is processed.
template <bool FUSE, int CAP = kSmallBlob>
__device__ __forceinline__ void small_blob_loop(const DevBufs& b, const Geom& g, const Params& prm, BlobShared<64, CAP>& S,
                                const uint32_t* s_combo, const uint32_t* s_cnt, uint32_t wv, uint32_t nwaves,
                                int c0, int c1) {
  const uint32_t lane = lane_id();
  uint32_t* pacc = S.pacc;
  if (lane < 22) pacc[lane] = 0;
  if (lane == 0) S.slow_dt = 0;
  uint32_t nwork = 0;
  for (int c = c0; c < c1; c++) nwork += s_cnt[c];
  uint32_t item = wv;
  uint32_t w = 0, w1 = 0;
  PairInfo pi = {0, 0, 0};
  if (item < nwork) {
    work_item(b, s_cnt, c0, c1, item, &w);
    pi = load_pair_info(b, w);
  }
  if (item + nwaves < nwork) work_item(b, s_cnt, c0, c1, item + nwaves, &w1);
  for (; item < nwork; item += nwaves) {
    const bool has1 = item + nwaves < nwork;
    const PairInfo pi1 = has1 ? load_pair_info(b, w1) : PairInfo{0, 0, 0};
    uint32_t w2 = 0;
    if (item + 2 * nwaves < nwork) work_item(b, s_cnt, c0, c1, item + 2 * nwaves, &w2);
    [[clang::always_inline]] blob_item<64, CAP, FUSE>(b, g, prm, S, nullptr, s_combo, w, pi, pacc);
    w = w1;
    pi = pi1;
    w1 = w2;
  }
  probe_flush(b, prm, pacc, 64, lane == 0);
  probe_flush_slow(b, prm, S, lane == 0);
  if (lane == 0 && pacc[20]) atomicAdd(b.blob_pts + 0, pacc[20]);
  if (lane == 0 && pacc[21]) atomicAdd(b.nquads, pacc[21]);  // batch total in nquads[0]
}

// K9a (large blobs, > kSmallBlob points): one blob per NT-thread workgroup
// iteration, persistent over the large work list.  Throughput mode: CAP 4096 (49 KB
// LDS) over the items of 1025-4096 points, CAP 1024 (128 threads) over the 513-1024
// class, and -- geometries whose blobs can exceed 4096 points (max_cluster = 2 (W + H)
// > 4096, e.g. 1080p) -- CAP 8192 in 512-thread teams (97 KB, one workgroup per CU)
// over the few larger ones (nlo = 4096, size class 0 only); each launch dequeues from
// its own head.  (The 1080p CAP-8192 launch in 256-thread teams, 32 keys per thread,
// sorted by a bitonic fallback: k_blob 1.68 -> 0.68 ms per 192 frames, 1080p 45.8 k
// -> 53.0 k frames/s, profiles/r06/ab1080_big_blob_teams.txt.)
template <int NT, int CAP, bool FUSE = false>
// (the throughput-mode 256-thread CAP-4096 teams at 3 waves per SIMD: 166 VGPRs, no
// spills; +0.7 % over 2 waves in four interleaved rounds, profiles/r06/ab720_large_waves3.txt)
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 256 && CAP == 4096 && !FUSE ? 3 : 1))) void k_blob(DevBufs b, Geom g, Params prm, uint32_t nlo, int c0, int c1, int launch) {
  __shared__ BlobShared<NT, CAP> S;
  const int tid = threadIdx.x;
  // device-clock span: the first launch's workgroups stamp their slots as usual; the
  // second (nlo != 0) appends its stamps after them (a slot per workgroup claimed on
  // the grid counter the first launch set), so the span covers both launches, as
  // the HIP events around the stage do
  uint32_t kt_slot = ~0u;
  if (!launch) {
    kt_begin(b, 9);
  } else if (b.kt_stage == 9 && tid == 0) {
    kt_slot = atomicAdd(b.kgrid, 1u);
    if (kt_slot < b.kwg_cap) b.kwg[kt_slot] = wall_clock64();
  }
  __shared__ uint32_t s_combo[420], s_cnt[kNumCls];
  load_combos(s_combo, tid, NT);
  if (tid < kNumCls) s_cnt[tid] = min(b.ncls[tid], b.wcap);
  large_blob_loop<NT, CAP, FUSE>(b, g, prm, S, s_combo, s_cnt, nlo, blockIdx.x, c0, c1, launch);
  if (tid == 0 && !launch) kt_end(b, 9);
  if (tid == 0 && launch && kt_slot < b.kwg_cap) b.kwg[b.kwg_cap + kt_slot] = wall_clock64();
}

// K9a (small blobs, <= kSmallBlob points): one blob per wave, four independent
// waves per workgroup, persistent over the small work list.  Everything a blob
// needs lives in its wave's LDS slice (no global scratch).
#ifndef AT_BS_WAVES
#define AT_BS_WAVES 4
#endif

// Classes c0 .. c1-1 of blobs of up to CAP points, timed as stage STAGE; `launch` > 0:
// not the stage's first launch (appends its device-clock stamps).  (A CAP-128 launch for
// the blobs of up to 128 points kept 123 VGPRs -- the per-blob fits, not the per-point
// arrays, set the register count -- so the small blobs stay in one CAP-512 launch.)
// Throughput mode also runs the 513-1024-point class this way (CAP 1024, 16 keys per
// lane, 168 VGPRs: 3 waves per SIMD, +0.7 % over 2 at 188 VGPRs in three interleaved
// rounds, profiles/r06/ab720_mid_wave3_stages.txt) as the large-blob stage's second launch: one wave
// per blob and no workgroup barriers, where 128-thread teams spent 63 % of their
// wave-cycles waiting (+1.7 % frames/s, profiles/r06/ab720_mid_wave_stages.txt).
template <bool FUSE, int CAP = kSmallBlob, int WAVES = AT_BS_WAVES, int STAGE = 8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FUSE ? 2 : WAVES))) void k_blob_small(DevBufs b, Geom g, Params prm,
                                                                                                         int c0, int c1, int launch) {
  __shared__ BlobShared<64, CAP> Ss[4];
  const int wave = threadIdx.x >> 6;
  uint32_t kt_slot = ~0u;
  if (!launch) {
    kt_begin(b, STAGE);
  } else if (b.kt_stage == STAGE && threadIdx.x == 0) {
    kt_slot = atomicAdd(b.kgrid, 1u);
    if (kt_slot < b.kwg_cap) b.kwg[kt_slot] = wall_clock64();
  }
  __shared__ uint32_t s_combo[420], s_cnt[kNumCls];
  load_combos(s_combo, threadIdx.x, 256);
  if (threadIdx.x < kNumCls) s_cnt[threadIdx.x] = min(b.ncls[threadIdx.x], b.wcap);
  __syncthreads();
  small_blob_loop<FUSE, CAP>(b, g, prm, Ss[wave], s_combo, s_cnt, blockIdx.x * 4 + wave, gridDim.x * 4, c0, c1);
  if (b.kt_stage == STAGE) {  // (uniform: the timed launch only)
    __syncthreads();
    if (threadIdx.x == 0 && !launch) kt_end(b, STAGE);
    if (threadIdx.x == 0 && launch && kt_slot < b.kwg_cap) b.kwg[b.kwg_cap + kt_slot] = wall_clock64();
  }
}

// Latency mode (blobs of up to 4096 points): the large-blob teams and the small-blob
// waves in ONE launch, so the B = 1 chain has no fork / join between two kernels on
// two streams (their event edges cost ~15 us).  Even workgroups are 512-thread
// large-blob teams, odd ones eight small-blob waves each (in the large team's LDS);
// extents, SelectBlobs and keys inside both (FUSE).
__global__ __launch_bounds__(512) void k_blob_lat(DevBufs b, Geom g, Params prm) {
  using SL = BlobShared<512, 4096>;
  using SS = BlobShared<64, kSmallBlob>;
  static_assert(8 * sizeof(SS) <= sizeof(SL), "eight small-blob waves fit in a large team's LDS");
  __shared__ __attribute__((aligned(16))) unsigned char s_raw[sizeof(SL)];
  __shared__ uint32_t s_combo[420], s_cnt[kNumCls];
  const int tid = threadIdx.x;
  kt_begin(b, 9);
  load_combos(s_combo, tid, 512);
  if (tid < kNumCls) s_cnt[tid] = min(b.ncls[tid], b.wcap);
  const uint32_t team = blockIdx.x >> 1, nteam = gridDim.x >> 1;
  if ((blockIdx.x & 1) == 0) {
    large_blob_loop<512, 4096, true>(b, g, prm, *reinterpret_cast<SL*>(s_raw), s_combo, s_cnt, 0u, team, 0, g.nlarge, 0);
  } else {
    __syncthreads();
    const int wave = tid >> 6;
    small_blob_loop<true>(b, g, prm, reinterpret_cast<SS*>(s_raw)[wave], s_combo, s_cnt, team * 8 + wave, nteam * 8,
                          g.nlarge, kNumCls);
  }
  if (b.kt_stage == 9) {  // (uniform: the timed launch only)
    __syncthreads();
    if (tid == 0) kt_end(b, 9);
  }
}

// Throughput mode's end of FitQuads (UpdateFitQuads, apriltag_detect.cu:98-241) for the
// kept blobs of size classes c0 .. c1-1, four lanes (a DPP quad) per blob: lane k fits
// side line k from the moments the blob kernels left in QuadPend, intersects it with
// line k+1 (corner k), measures Heron side k (lanes 0, 1 also sides 4, 5) and tests
// corner angle k; lane 0 writes the debug record and the accepted quad's decode-queue
// entry.  The expressions are the team version's in blob_item (which latency mode keeps).
__global__ __launch_bounds__(256) void k_quad_fin(DevBufs b, Geom g, Params prm, int c0, int c1) {
  __shared__ uint32_t s_cnt[kNumCls];
  if (threadIdx.x < kNumCls) s_cnt[threadIdx.x] = min(b.ncls[threadIdx.x], b.wcap);
  __syncthreads();
  uint32_t nwork = 0;
  for (int c = c0; c < c1; c++) nwork += s_cnt[c];
  const uint32_t lane = lane_id(), base = lane & ~3u;
  const int k = (int)(lane & 3);
  auto from = [&](double v, int j) { return __shfl(v, (int)base + j); };
  auto fromf = [&](float v, int j) { return __shfl(v, (int)base + j); };
  auto quad_or = [&](int v) {
    v |= __shfl_xor(v, 1);
    return v | __shfl_xor(v, 2);
  };
  // (the four lanes of a quad share the item: every shuffle reads an active lane)
  for (uint32_t it = (blockIdx.x * 256 + threadIdx.x) >> 2; it < nwork; it += gridDim.x * 64) {
    uint32_t w = 0;
    work_item(b, s_cnt, c0, c1, it, &w);
    const uint32_t f = w >> 16, rank = w & 0xffff;
    const size_t slot = (size_t)f * kMaxPairs + rank;
    if (b.pair_sel[slot] == 0) continue;  // (the blob kernels skipped it too)
    const QuadPend& qp = b.qpend[slot];
    const bool valid = qp.valid != 0;
    float cx = 0.f, cy = 0.f;
    int bad = 0;
    {
      double l[4] = {0, 0, 0, 0};
      if (valid) {  // fit_line's p01 and p23 from the blob team's d, c and centroid
        const float4 pre = *reinterpret_cast<const float4*>(qp.fit[k]);
        l[0] = (double)pre.z;
        l[1] = (double)pre.w;
        line_normal(pre.x, pre.y, det_hypotf(pre.x, pre.y), l + 2);
      }
      double m[4];
#pragma unroll
      for (int j = 0; j < 4; j++) m[j] = from(l[j], (k + 1) & 3);  // line k+1
      if (valid) {
        const double A00 = l[3], A01 = -m[3];
        const double A10 = -l[2], A11 = m[2];
        const double B0 = -l[0] + m[0];
        const double B1 = -l[1] + m[1];
        const double det = A00 * A11 - A10 * A01;
        const double W00 = A11 / det, W01 = -A01 / det;
        if (fabs(det) < 0.001) {
          bad = 1;
        } else {
          const double L0 = W00 * B0 + W01 * B1;
          cx = (float)(l[0] + L0 * A00);
          cy = (float)(l[1] + L0 * A10);
        }
      }
    }
    bool ok = valid && !quad_or(bad);
    float qc[4][2];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      qc[j][0] = fromf(cx, j);
      qc[j][1] = fromf(cy, j);
    }
    if (ok) {
      // sides of triangles (0,1,2) and (2,3,0): 0->1, 1->2, 2->0, 2->3, 3->0, 0->2;
      // lane k side k, lanes 0 and 1 also side 4 + k
      auto side = [&](int j) {
        const int a2 = j == 0 ? 0 : j == 1 ? 1 : j == 2 ? 2 : j == 3 ? 2 : j == 4 ? 3 : 0;
        const int b2 = j == 0 ? 1 : j == 1 ? 2 : j == 2 ? 0 : j == 3 ? 3 : j == 4 ? 0 : 2;
        return det_hypotf(qc[b2][0] - qc[a2][0], qc[b2][1] - qc[a2][1]);
      };
      const float s0 = side(k), s1 = side(4 + (k & 1));
      float len[6];
#pragma unroll
      for (int j = 0; j < 4; j++) len[j] = fromf(s0, j);
      len[4] = fromf(s1, 0);
      len[5] = fromf(s1, 1);
      float area = 0, pp;
      pp = (len[0] + len[1] + len[2]) / 2;
      area += sqrtf(pp * (pp - len[0]) * (pp - len[1]) * (pp - len[2]));
      pp = (len[3] + len[4] + len[5]) / 2;
      area += sqrtf(pp * (pp - len[3]) * (pp - len[4]) * (pp - len[5]));
      if ((double)area < 0.95 * g.min_tag_width * g.min_tag_width) ok = false;
    }
    if (ok) {
      const int i0 = k, i1 = (i0 + 1) & 3, i2 = (i0 + 2) & 3;
      const float dx1 = qc[i1][0] - qc[i0][0], dy1 = qc[i1][1] - qc[i0][1];
      const float dx2 = qc[i2][0] - qc[i1][0], dy2 = qc[i2][1] - qc[i1][1];
      const float cosd = (dx1 * dx2 + dy1 * dy2) / sqrtf((dx1 * dx1 + dy1 * dy1) * (dx2 * dx2 + dy2 * dy2));
      const int abad = (double)fabsf(cosd) > prm.cos_critical_rad || dx1 * dy2 < dy1 * dx2;
      if (quad_or(abad)) ok = false;
    }
    if (k == 0) {
      QuadRecord rec;
      rec.blob_index = qp.blob_index;
      rec.valid = valid;
      for (int j = 0; j < 4; j++) rec.indices[j] = qp.indices[j];
      QuadCand qcand;
      for (int j = 0; j < 4; j++) {  // AdjustPixelCenters, quad_decimate 2
        const float x = ok ? (qc[j][0] - 0.5f) * 2.0f + 0.5f : 0.f;
        const float y = ok ? (qc[j][1] - 0.5f) * 2.0f + 0.5f : 0.f;
        rec.corners[j][0] = qcand.p[j][0] = x;
        rec.corners[j][1] = qcand.p[j][1] = y;
      }
      rec.accepted = ok;
      if (prm.taps) b.quads[slot] = rec;  // (debug record: AT_STAGE_QUADS with the taps on)
      if (ok && !AT_DIAG_STOP(prm, 5)) {
        qcand.frame = f;
        qcand.rank = rank;
        const uint32_t ci = atomicAdd(b.nqcand + (size_t)f * kQcStride, 1u);
        if (ci < (uint32_t)kQuadCandPerFrame) b.qcand[(size_t)f * kQuadCandPerFrame + ci] = qcand;
        else atomicOr(b.status + f, kStatusQuadsOverflow);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K9b: one accepted quad per 64-lane workgroup iteration (persistent):
// RefineEdges with UnDistort/ReDistort (apriltag_detect.cu:405-564),
// homography (quad_update_homographies) and quad_decode (apriltag 3.x).
// Order-dependent sums (line fit of the refined edge samples, gray models,
// decision scores) run on one lane in the reference's order.
// ---------------------------------------------------------------------------
constexpr int kDecodeThreads = 64;
// quad_decode border patterns (x0, y0, dx, dy; white for even p): left white /
// black column, right white / black column, top white / black row, bottom white /
// black row, in float as upstream's `float patterns[]` (wab = width_at_border)
__device__ __forceinline__ void border_pattern(int p, float wab, float& x0, float& y0, float& dx, float& dy) {
  const float far_ = (p & 1) ? wab - 0.5f : wab + 0.5f;
  const float near_ = (p & 1) ? 0.5f : -0.5f;
  const int side = p >> 1;  // 0 left, 1 right, 2 top, 3 bottom
  const float a = (side == 0 || side == 2) ? near_ : far_;
  if (side < 2) { x0 = a; y0 = 0.5f; dx = 0; dy = 1; }
  else { x0 = 0.5f; y0 = a; dx = 1; dy = 0; }
}

// apriltag.c rotate90 (3.x spiral layout): a rotation of the bit string by
// nbits/4, the centre bit (LSB) fixed when nbits % 4 == 1
__device__ __forceinline__ uint64_t rotate90_n(uint64_t w, int nbits) {
  int p = nbits;
  uint64_t l = 0;
  if (nbits % 4 == 1) { p = nbits - 1; l = 1; }
  w = ((w >> l) << (p / 4 + l)) | (w >> (3 * p / 4 + l) << l) | (w & l);
  return w & ((1ull << nbits) - 1);
}
constexpr int kMaxTotalWidth = 12;  // total_width of the largest family layout (d <= 8)

// value of lane `l` (uniform) on every lane
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}
// cos / sin of rot * pi/2 as libm returns them (quad_decode's rotation of H)
__constant__ double c_rot_c[4] = {1.0, 6.123233995736766e-17, -1.0, -1.8369701987210297e-16};
__constant__ double c_rot_s[4] = {0.0, 1.0, 1.2246467991473532e-16, -1.0};
// Refine samples of one quad: 4 edges of max(16, len / 8) samples, so at most
// perimeter / 8 + 64 for a quad inside the frame (perimeter <= 2 (W + H)).  The
// first kLdsRefine samples (every quad of side <= ~380 px) live in LDS, the rest
// of a huge quad in the workgroup's global scratch (DevBufs::rsamp): an 8.5 KB
// workgroup instead of 17 KB doubles the quads in flight per CU.

struct DecodeShared {
  double sx[kLdsRefine], sy[kLdsRefine];
  float qc[4][2];
  int nsamp[4], samp_off[4];
  float enx[4], eny[4];
  double lines[4][4];
  double H[9];
  double A[72];  // homography DLT system
  double gmx[64], gmy[64], gmv[64];
  int gmvalid[64];
  double wC[3], bC[3];
  double values[kMaxTotalWidth * kMaxTotalWidth];
  int ok;
  uint32_t item;
  uint32_t qpre[kMaxBatch + 1];
};

// POSE: the decode wave's hand-over to the pose wave (LDS): the homography and
// unrotated corners of quad `seq`, and the pose the pose wave acknowledges with `ack`
struct PoseHandoff {
  double H[9], p[4][2];
  double R[9], t[3], err[2];
  uint32_t seq, ack, exit;
};
__device__ void pose_worker(PoseHandoff& P, const Params& prm) {
  const uint32_t lane = lane_id();
  uint32_t seen = 0;
  while (true) {
    uint32_t sq;
    bool done = false;
    while ((sq = __hip_atomic_load(&P.seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == seen) {
      // (the decode wave raises exit only after the last pose was acknowledged)
      if (__hip_atomic_load(&P.exit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) { done = true; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (done) return;
    seen = sq;
    double H[9], pc[4][2];
#pragma unroll
    for (int k = 0; k < 9; k++) H[k] = P.H[k];
#pragma unroll
    for (int k = 0; k < 4; k++) { pc[k][0] = P.p[k][0]; pc[k][1] = P.p[k][1]; }
    double R[9], t[3], err[2];
    pose::estimate_tag_pose<true>(H, pc, prm.fx, prm.fy, prm.cx, prm.cy, prm.tag_size, R, t, err, (int)(lane & 3));
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 9; k++) P.R[k] = R[k];
#pragma unroll
      for (int k = 0; k < 3; k++) P.t[k] = t[k];
      P.err[0] = err[0];
      P.err[1] = err[1];
      __hip_atomic_store(&P.ack, seen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}
// POSE: the last decode workgroup to finish copies the (final) control block to
// the caller-visible host buffer (k_pose's job in the unfused sequence).  Only the
// min(grid, nq) workgroups that had a quad arrive (the others wrote nothing; one
// arrival per workgroup on one counter costs ~12 ns each); no quad: workgroup 0.
__device__ void decode_finish(const DevBufs& b, int lane, uint32_t nq) {
  const uint32_t nwg = min(gridDim.x, nq);
  if (blockIdx.x >= max(nwg, 1u)) return;
  uint32_t last = nwg == 0;
  if (lane == 0 && nwg) {
    __threadfence();
    last = atomicAdd(b.dec_done, 1u) == nwg - 1;
  }
  last = __shfl(last, 0);
  if (!last) return;
  __threadfence();
  for (uint32_t w = (uint32_t)lane; w < b.ctrl_words; w += 64)
    b.hctrl[w] = __hip_atomic_load(b.ctrl + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#ifndef AT_BIG_BLOB_WG
#define AT_BIG_BLOB_WG 256  // workgroups of the CAP-8192 large-blob launch (blobs over 4096 points):
// one per CU -- 64 left the 1080p stage at 4.03 ms per 192 frames serialized, 1.69 ms at 256
// (concurrent 1080p throughput +1.5 %, profiles/r04y)
#endif
#ifndef AT_BIG_NT
#define AT_BIG_NT 512  // threads per team of the CAP-8192 launch (16 keys per thread: register theta sort)
#endif
#ifndef AT_FORK_SMALL
#define AT_FORK_SMALL 1  // latency mode: fork the small-blob kernel (0: the large-blob one)
#endif
#ifndef AT_POSE_IN_DECODE
#define AT_POSE_IN_DECODE 1  // latency mode: the pose by a second wave of k_decode (0: k_pose)
#endif
// throughput-mode k_decode at 4 waves per SIMD (128 VGPRs, 80 B of spills) instead of
// the 3 its 155 VGPRs allowed: 0.180 -> 0.151 ms per 128 frames, concurrent throughput
// unchanged or better (profiles/r04p)
#ifndef AT_DEC_WAVES
#define AT_DEC_WAVES 4
#endif
// POSE (latency mode, tag_size > 0): a second wave per workgroup estimates the
// tag pose (k_pose's work) of every quad as soon as its homography is known,
// while the first wave decodes the bits; the pose is computed on the unrotated
// homography and corners and rotated with the decoded orientation afterwards
// (R = R0 Rz(rot), t = t0: the corner correspondence of a 90-degree turn of
// the tag frame), so the B = 1 chain is homography + pose instead of decode +
// pose.  The last workgroup to finish hands the control block to the host.
template <bool POSE>
__global__ __launch_bounds__(POSE ? 128 : kDecodeThreads) __attribute__((amdgpu_waves_per_eu(POSE ? 1 : AT_DEC_WAVES))) void k_decode(DevBufs b, Geom g, Params prm, int B, int fmt) {
  constexpr int RCAP = kMaxRefineSamples;
  __shared__ DecodeShared S;
  __shared__ PoseHandoff P;
  const int tid = threadIdx.x;
  kt_begin(b, 10);
  if (POSE) {
    if (tid == 0) { P.seq = 0; P.ack = 0; P.exit = 0; }
    __syncthreads();
    if (tid >= 64) {
      pose_worker(P, prm);
      return;
    }
  }
  double* gsx = b.rsamp + (size_t)blockIdx.x * (2 * (kMaxRefineSamples - kLdsRefine));
  double* gsy = gsx + (kMaxRefineSamples - kLdsRefine);
  // exclusive prefix of the per-frame candidate counts: item -> (frame, index)
  // (all lanes load the counts at once, B <= 256 = 4 per lane; wave scan)
  uint32_t* qpre = S.qpre;
  {
    uint32_t c[kMaxBatch / 64], sum = 0;
#pragma unroll
    for (int k = 0; k < kMaxBatch / 64; k++) {
      const int f = tid * (kMaxBatch / 64) + k;
      c[k] = f < B ? min(b.nqcand[(size_t)f * kQcStride], (uint32_t)kQuadCandPerFrame) : 0u;
      sum += c[k];
    }
    const uint32_t incl = wave_incl_scan(sum, AddOp(), 0u);
    uint32_t acc = incl - sum;
#pragma unroll
    for (int k = 0; k < kMaxBatch / 64; k++) {
      const int f = tid * (kMaxBatch / 64) + k;
      if (f < B) qpre[f] = acc;
      acc += c[k];
    }
    if (tid == 63) qpre[B] = incl;
  }
  team_sync<64>();
  const uint32_t nq = qpre[B];

  // AT_PHASE_PROBE: accumulated wall-clock per phase (probe[128 + k], counts [160 + k])
  uint32_t pacc[21] = {0};
  uint64_t t_last = 0;
  auto phase = [&](int k) {
    if (AT_PROBE_ON(prm) && tid == 0) {
      const uint64_t now = wall_clock64();
      if (k > 0) {
        pacc[k] += (uint32_t)(now - t_last);
        pacc[10 + k] += 1;
      }
      t_last = now;
    }
  };
  // static round-robin over the queue (every entry is an accepted quad: the blob
  // kernels append only those)
  const uint32_t G = gridDim.x;
  uint32_t pose_seq = 0;  // (POSE) quads handed to the pose wave
  // the next item's queue entry (its corners on lanes 0-3) and frame address are
  // loaded while this one is processed: an item's chain starts at its gray loads
  struct ItemPre {
    int f;
    uint32_t rank;
    float px, py;
    const uint8_t* gsrc;
  };
  auto prefetch = [&](uint32_t it) -> ItemPre {
    int lo = 0, hi = B - 1;  // last frame whose prefix <= it (the entry's frame)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (qpre[mid] <= it) lo = mid;
      else hi = mid - 1;
    }
    const QuadCand* q = &b.qcand[(size_t)lo * kQuadCandPerFrame + (it - qpre[lo])];
    ItemPre p;
    p.f = lo;
    p.rank = q->rank;
    p.px = tid < 4 ? q->p[tid & 3][0] : 0.f;
    p.py = tid < 4 ? q->p[tid & 3][1] : 0.f;
    // luma of pixel i = y W + x: the frame's own Y bytes for YUYV (every second byte)
    // and GRAY8 input, the gray plane k_pre wrote for BGR8
    p.gsrc = fmt == 1 ? b.gray + (size_t)lo * g.W * g.H : b.frames[lo];
    return p;
  };
  ItemPre nxt = {};
  if (blockIdx.x < nq) nxt = prefetch(blockIdx.x);
  for (uint32_t item = blockIdx.x; item < nq; item += G) {
    const ItemPre cur = nxt;
    if (item + G < nq) nxt = prefetch(item + G);
    const int f = cur.f;
    const uint32_t qrank = cur.rank;
    const uint8_t* gsrc = cur.gsrc;
    const int gsh = fmt == 0 ? 1 : 0;
    auto pix = [&](size_t i) -> uint32_t { return gsrc[i << gsh]; };
    if (tid < 4) { S.qc[tid][0] = cur.px; S.qc[tid][1] = cur.py; }
    team_sync<64>();
    phase(0);
    if (prm.refine_edges) {
      if (tid < 4) {
        const int a2 = tid, b2 = (tid + 1) & 3;
        float nx = S.qc[b2][1] - S.qc[a2][1];
        float ny = -S.qc[b2][0] + S.qc[a2][0];
        const float mag = sqrtf(nx * nx + ny * ny);
        nx /= mag;
        ny /= mag;
        const int nsf = (int)(mag / 8);
        S.nsamp[tid] = nsf > 16 ? nsf : 16;
        S.enx[tid] = nx;
        S.eny[tid] = ny;
      }
      team_sync<64>();
      if (tid == 0) {
        int acc = 0;
        for (int k = 0; k < 4; k++) { S.samp_off[k] = acc; acc += S.nsamp[k]; }
      }
      team_sync<64>();
      const int total = min(S.samp_off[3] + S.nsamp[3], RCAP);
      if (tid == 0 && S.samp_off[3] + S.nsamp[3] > RCAP) atomicOr(b.status + f, kStatusQuadsOverflow);
      for (int t = tid; t < total; t += kDecodeThreads) {
        int edge = 0;
        while (edge < 3 && t >= S.samp_off[edge + 1]) edge++;
        const int s = t - S.samp_off[edge];
        const int a2 = edge, b2 = (edge + 1) & 3;
        const int nsamples = S.nsamp[edge];
        const float nx = S.enx[edge], ny = S.eny[edge];
        const double alpha = (1.0 + s) / (nsamples + 1);
        const double x0 = alpha * S.qc[a2][0] + (1 - alpha) * S.qc[b2][0];
        const double y0 = alpha * S.qc[a2][1] + (1 - alpha) * S.qc[b2][1];
        // the 25 steps n = -3, -2.75, ..., 3 (exact in double): every gray load is
        // issued before the first is consumed, then the sums run in step order
        constexpr int kSteps = 25;
        int g1v[kSteps], g2v[kSteps];
#pragma unroll
        for (int k = 0; k < kSteps; k++) {
          const double nn = -3.0 + 0.25 * k;
          const int x1 = (int)(x0 + (nn + 1) * nx);
          const int y1 = (int)(y0 + (nn + 1) * ny);
          const int x2 = (int)(x0 + (nn - 1) * nx);
          const int y2 = (int)(y0 + (nn - 1) * ny);
          const bool in = !(x1 < 0 || x1 >= g.W || y1 < 0 || y1 >= g.H) && !(x2 < 0 || x2 >= g.W || y2 < 0 || y2 >= g.H);
          g1v[k] = -1;
          g2v[k] = 0;
          if (in) {
            g1v[k] = (int)pix((size_t)y1 * g.W + x1);
            g2v[k] = (int)pix((size_t)y2 * g.W + x2);
          }
        }
        double Mn = 0, Mcount = 0;
#pragma unroll
        for (int k = 0; k < kSteps; k++) {
          const double nn = -3.0 + 0.25 * k;
          const int g1 = g1v[k], g2 = g2v[k];
          if (g1 < g2) continue;  // also skips out-of-image steps (g1 = -1)
          const double weight = (double)((g2 - g1) * (g2 - g1));
          Mn += weight * nn;
          Mcount += weight;
        }
        double bx = __longlong_as_double(0x7ff8deadbeef0000ll), by = 0;
        if (Mcount != 0) {
          const double n0 = Mn / Mcount;
          bx = x0 + n0 * nx;
          by = y0 + n0 * ny;
          undistort(prm, &bx, &by);
        }
        if (t < kLdsRefine) {
          S.sx[t] = bx;
          S.sy[t] = by;
        } else {
          gsx[t - kLdsRefine] = bx;
          gsy[t - kLdsRefine] = by;
        }
      }
      team_sync<64>();
      phase(1);
      // per edge (lane e), the moments in the reference's sample order; samples are
      // staged 8 at a time in registers so their LDS reads overlap
      if (tid < 4) {
        double Mx = 0, My = 0, Mxx = 0, Mxy = 0, Myy = 0, N = 0;
        const int o = S.samp_off[tid];
        const int ns = min(S.nsamp[tid], RCAP - o);
        for (int c = 0; c < ns; c += 8) {
          double xs[8], ys[8];
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const int i = o + c + k;
            xs[k] = __longlong_as_double(0x7ff8deadbeef0000ll);
            ys[k] = 0;
            if (c + k < ns) {
              xs[k] = i < kLdsRefine ? S.sx[i] : gsx[i - kLdsRefine];
              ys[k] = i < kLdsRefine ? S.sy[i] : gsy[i - kLdsRefine];
            }
          }
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const double bx = xs[k], by = ys[k];
            if (isnan(bx)) continue;  // (also the padding past the edge's samples)
            Mx += bx; My += by; Mxx += bx * bx; Mxy += bx * by; Myy += by * by; N++;
          }
        }
        const double Ex = Mx / N, Ey = My / N;
        const double Cxx = Mxx / N - Ex * Ex, Cxy = Mxy / N - Ex * Ey, Cyy = Myy / N - Ey * Ey;
        const double nt = .5 * (double)det_atan2f_call((float)(-2 * Cxy), (float)(Cyy - Cxx));
        S.lines[tid][0] = Ex;
        S.lines[tid][1] = Ey;
        S.lines[tid][2] = (double)det_cosf((float)nt);
        S.lines[tid][3] = (double)det_sinf((float)nt);
      }
      team_sync<64>();
      phase(2);
      if (tid == 0) {
        float qp[4][2];
        for (int k = 0; k < 4; k++) { qp[k][0] = S.qc[k][0]; qp[k][1] = S.qc[k][1]; }
        for (int i = 0; i < 4; i++) {
          const int i1 = (i + 1) & 3;
          const double A00 = S.lines[i][3], A01 = -S.lines[i1][3];
          const double A10 = -S.lines[i][2], A11 = S.lines[i1][2];
          const double B0 = -S.lines[i][0] + S.lines[i1][0];
          const double B1 = -S.lines[i][1] + S.lines[i1][1];
          const double det = A00 * A11 - A10 * A01;
          if (fabs(det) > 0.001) {
            const double W00 = A11 / det, W01 = -A01 / det;
            const double L0 = W00 * B0 + W01 * B1;
            double px = S.lines[i][0] + L0 * A00, py = S.lines[i][1] + L0 * A10;
            redistort(prm, &px, &py);
            qp[i1][0] = (float)px;
            qp[i1][1] = (float)py;
          }
        }
        for (int k = 0; k < 4; k++) { S.qc[k][0] = qp[k][0]; S.qc[k][1] = qp[k][1]; }
      }
      team_sync<64>();
      phase(3);
    }
    if (AT_DIAG_STOP(prm, 6)) continue;
    // ---- homography (quad_update_homographies / homography_compute2) -----------
    if (homography_wave(S.qc, S.A, S.H) != 0) continue;
    if (tid == 0) {
      const double* H = S.H;
      const double hdet = H[0] * (H[4] * H[8] - H[5] * H[7]) - H[1] * (H[3] * H[8] - H[5] * H[6]) +
                          H[2] * (H[3] * H[7] - H[4] * H[6]);
      S.ok = hdet != 0;
    }
    team_sync<64>();
    phase(4);
    if (!S.ok) continue;
    uint32_t seq = 0;
    if (POSE) {  // hand the homography and the unrotated corners to the pose wave
      if (tid < 9) P.H[tid] = S.H[tid];
      if (tid < 4) {
        const int tcx = (tid == 1 || tid == 2) ? 1 : -1, tcy = tid < 2 ? 1 : -1;
        hproject(S.H, tcx, tcy, &P.p[tid][0], &P.p[tid][1]);
      }
      seq = ++pose_seq;
      team_sync<64>();
      if (tid == 0) __hip_atomic_store(&P.seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    uint32_t bc = 0xffffffffu;
    double margin_d = -1;
    do {
    // ---- quad_decode: border gray models (8 patterns x width_at_border <= 8
    // samples: lane = 8 * pattern + sample) ----
    const int wab = prm.fam.width_at_border, tw = prm.fam.total_width, nbits = prm.fam.nbits;
    const int minc = (wab - tw) / 2;
    {
      const int pidx = tid >> 3, i = tid & 7;
      float p0, p1, p2, p3;
      border_pattern(pidx, (float)wab, p0, p1, p2, p3);
      const double tagx01 = (double)((p0 + (float)i * p2) / (float)wab);
      const double tagy01 = (double)((p1 + (float)i * p3) / (float)wab);
      const double tagx = 2 * (tagx01 - 0.5), tagy = 2 * (tagy01 - 0.5);
      double px, py;
      hproject(S.H, tagx, tagy, &px, &py);
      const int ix = (int)px, iy = (int)py;
      S.gmx[tid] = tagx;
      S.gmy[tid] = tagy;
      S.gmvalid[tid] = i < wab && !(ix < 0 || iy < 0 || ix >= g.W || iy >= g.H);
      S.gmv[tid] = S.gmvalid[tid] ? (double)pix((size_t)iy * g.W + ix) : 0.0;
    }
    for (int t = tid; t < tw * tw; t += kDecodeThreads) S.values[t] = 0;
    team_sync<64>();
    phase(5);
    // lane 0 builds and solves the white model, lane 1 the black one, each over
    // its 32 samples in the serial order, eight samples staged in registers at a time
    double interp00 = 0;
    if (tid < 2) {
      GrayModel m;
      for (int k = 0; k < 3; k++) {
        m.B[k] = 0;
        for (int j = 0; j < 3; j++) m.A[k][j] = 0;
      }
      for (int grp = 0; grp < 4; grp++) {
        const int t0 = 16 * grp + 8 * tid;
        double xs[8], ys[8], vs[8];
        int ok[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
          xs[i] = S.gmx[t0 + i];
          ys[i] = S.gmy[t0 + i];
          vs[i] = S.gmv[t0 + i];
          ok[i] = S.gmvalid[t0 + i];
        }
#pragma unroll
        for (int i = 0; i < 8; i++)
          if (ok[i]) gm_add(m, xs[i], ys[i], vs[i]);
      }
      gm_solve(m);
      double* C = tid == 0 ? S.wC : S.bC;
      for (int k = 0; k < 3; k++) C[k] = m.C[k];
      interp00 = gm_interp(m, 0, 0);
    }
    const double w00 = __shfl(interp00, 0), b00 = __shfl(interp00, 1);
    team_sync<64>();
    if (w00 - b00 < 0) break;  // uniform
    phase(6);
    if (tid < nbits) {
      const int bity = prm.fam.bity[tid], bitx = prm.fam.bitx[tid];
      const double tagx01 = (bitx + 0.5) / wab, tagy01 = (bity + 0.5) / wab;
      const double tagx = 2 * (tagx01 - 0.5), tagy = 2 * (tagy01 - 0.5);
      double px, py;
      hproject(S.H, tagx, tagy, &px, &py);
      const int x1 = (int)floor(px - 0.5), x2 = (int)ceil(px - 0.5);
      const double xx = px - 0.5 - x1;
      const int y1 = (int)floor(py - 0.5), y2 = (int)ceil(py - 0.5);
      const double yy = py - 0.5 - y1;
      if (!(x1 < 0 || x2 >= g.W || y1 < 0 || y2 >= g.H)) {  // value_for_pixel
        const double v = (int)pix((size_t)y1 * g.W + x1) * (1 - xx) * (1 - yy) + (int)pix((size_t)y1 * g.W + x2) * xx * (1 - yy) +
                         (int)pix((size_t)y2 * g.W + x1) * (1 - xx) * yy + (int)pix((size_t)y2 * g.W + x2) * xx * yy;
        const double bth = S.bC[0] * tagx + S.bC[1] * tagy + S.bC[2];
        const double wth = S.wC[0] * tagx + S.wC[1] * tagy + S.wC[2];
        S.values[tw * (bity - minc) + bitx - minc] = v - (bth + wth) / 2.0;
      }
    }
    team_sync<64>();
    phase(7);
    // sharpen (apriltag.c) over the total_width^2 grid: each lane owns cells t, t+64, t+128
    constexpr int kShR = (kMaxTotalWidth * kMaxTotalWidth + kDecodeThreads - 1) / kDecodeThreads;
    double shv[kShR];
    // (the lane's cell indices recomputed per quad: hoisted out of the item loop they
    // were spilled to scratch and reloaded here, one round trip each)
    int tl = tid;
    __asm__ volatile("" : "+v"(tl));
#pragma unroll
    for (int r = 0; r < kShR; r++) {
      const int t = tl + 64 * r;
      shv[r] = 0;
      if (t < tw * tw) {
        // the kernel {0,-1,0; -1,4,-1; 0,-1,0} in the reference's tap order, its zero taps
        // left out: they add +-0, which changes no nonzero partial sum, and the sign of a
        // zero sum reaches no decision (a value is never -0: v - m is +0 when v == m).
        // The five reads are issued together (the 3x3 loop's reads went one at a time,
        // their addresses spilled to scratch)
        const int y = t / tw, x = t % tw;
        const double up = S.values[y > 0 ? t - tw : t], left = S.values[x > 0 ? t - 1 : t], c = S.values[t];
        const double right = S.values[x < tw - 1 ? t + 1 : t], down = S.values[y < tw - 1 ? t + tw : t];
        double acc = 0;
        if (y > 0) acc = acc - up;
        if (x > 0) acc = acc - left;
        acc = acc + c * 4;
        if (x < tw - 1) acc = acc - right;
        if (y < tw - 1) acc = acc - down;
        shv[r] = acc;
      }
    }
    team_sync<64>();
#pragma unroll
    for (int r = 0; r < kShR; r++) {
      const int t = tid + 64 * r;
      if (t < tw * tw) S.values[t] = S.values[t] + prm.decode_sharpening * shv[r];
    }
    team_sync<64>();
    // code word and scores: lane i reads bit i's value, the scores run in bit
    // order on every lane (uniform v_readlane loop), the word comes from a ballot
    double bitv = 0;
    if (tid < nbits) bitv = S.values[tw * (prm.fam.bity[tid] - minc) + prm.fam.bitx[tid] - minc];
    const uint64_t white_bits = __ballot(tid < nbits && bitv > 0);  // bit i: data bit i (MSB first in the word)
    const uint64_t rcode0 = __builtin_bitreverse64(white_bits) >> (64 - nbits);
    {
      float black_score = 0, white_score = 0, black_cnt = 1, white_cnt = 1;
      for (int i = 0; i < nbits; i++) {
        const double v = readlane_f64(bitv, i);
        if (v > 0) { white_score = (float)(white_score + v); white_cnt++; }
        else { black_score = (float)(black_score - v); black_cnt++; }
      }
      margin_d = fmin((double)(white_score / white_cnt), (double)(black_score / black_cnt));
    }
    phase(8);
    // quick_decode_codeword: first rotation, then entry, within hamming <= 2
    // (codes are >= 5 apart, so at most one entry matches a rotation)
    {
      uint64_t r[4];
      r[0] = rcode0;
#pragma unroll
      for (int k = 1; k < 4; k++) r[k] = rotate90_n(r[k - 1], nbits);
      // the codebook straight from HBM (L2-resident: every workgroup reads the same
      // table; an LDS copy cost 8 KB per one-wave workgroup, and the LDS freed lets
      // the concurrent batches' kernels co-reside: +2.8 % throughput, profiles/r03l),
      // ten of a lane's entries loaded together (tag36h11: one round trip instead of 10)
      constexpr int kBookChunk = 10;  // (every family in one round trip: ncodes <= 640)
      for (int e0 = 0; e0 < prm.fam.ncodes; e0 += kBookChunk * kDecodeThreads) {
        uint64_t cw[kBookChunk];
#pragma unroll
        for (int k = 0; k < kBookChunk; k++) {
          const int ent = e0 + tid + kDecodeThreads * k;
          cw[k] = ent < prm.fam.ncodes ? b.book_code[ent] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < kBookChunk; k++) {
          const int ent = e0 + tid + kDecodeThreads * k;
#pragma unroll
          for (int rot = 0; rot < 4; rot++) {
            const int hd = __popcll(r[rot] ^ cw[k]);
            if (ent < prm.fam.ncodes && hd <= 2) bc = min(bc, (uint32_t)((rot << 24) | (hd << 16) | ent));
          }
        }
      }
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) bc = min(bc, (uint32_t)__shfl_xor(bc, d));
    }
    } while (false);
    if (POSE) {  // the pose of this quad is done before the next one is handed over
      while (__hip_atomic_load(&P.ack, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != seq)
        __builtin_amdgcn_s_sleep(1);
    }
    if (tid == 0) {
      const float margin = (float)margin_d;
      if (margin >= 0 && bc != 0xffffffffu) {
        const int rot = bc >> 24, hd = (bc >> 16) & 0xff, ent = bc & 0xffff;
        DevDetection d;
        d.id = b.book_id[ent];
        d.hamming = hd;
        d.decision_margin = margin;
        d.blob_rank = (int32_t)qrank;
        const double R[9] = {c_rot_c[rot], -c_rot_s[rot], 0, c_rot_s[rot], c_rot_c[rot], 0, 0, 0, 1};
        for (int i = 0; i < 3; i++)
          for (int j = 0; j < 3; j++) {
            double acc = 0;
            for (int k = 0; k < 3; k++) acc += S.H[i * 3 + k] * R[k * 3 + j];
            d.H[i * 3 + j] = acc;
          }
        hproject(d.H, 0, 0, &d.c[0], &d.c[1]);
        for (int i = 0; i < 4; i++) {
          const int tcx = (i == 1 || i == 2) ? 1 : -1;
          const int tcy = (i < 2) ? 1 : -1;
          hproject(d.H, tcx, tcy, &d.p[i][0], &d.p[i][1]);
        }
        d.frame = (uint16_t)f;
        if (POSE) {
          // R = R0 Rz(rot) with the exact quarter turn, t = t0
          const int c = rot == 0 ? 1 : rot == 2 ? -1 : 0, sn = rot == 1 ? 1 : rot == 3 ? -1 : 0;
          for (int i = 0; i < 3; i++) {
            d.pose_R[i * 3 + 0] = P.R[i * 3 + 0] * c + P.R[i * 3 + 1] * sn;
            d.pose_R[i * 3 + 1] = -P.R[i * 3 + 0] * sn + P.R[i * 3 + 1] * c;
            d.pose_R[i * 3 + 2] = P.R[i * 3 + 2];
          }
          for (int k = 0; k < 3; k++) d.pose_t[k] = P.t[k];
          d.pose_err[0] = P.err[0];
          d.pose_err[1] = P.err[1];
        }
        // the frame's own slot; the first kDetPoolPerFrame also to the host mirror
        // (POSE: complete; else the pose fields follow from k_pose)
        const uint32_t k = atomicAdd(b.ndets + f, 1u);
        if (k < (uint32_t)kMaxDets) {
          const uint32_t slot = (uint32_t)f * kMaxDets + k;
          b.dets[slot] = d;
          if (k < (uint32_t)kDetPoolPerFrame) b.hdets[(uint32_t)f * kDetPoolPerFrame + k] = d;
          if (!POSE) b.det_work[atomicAdd(b.det_head, 1u)] = slot;
        } else {
          atomicOr(b.status + f, kStatusDetsOverflow);  // (more candidates than quads: unreachable)
        }
      }
    }
    team_sync<64>();
    phase(9);
  }
  probe_flush(b, prm, pacc, 128, tid == 0);
  if (tid == 0) kt_end(b, 10);
  if (POSE) {
    if (tid == 0) __hip_atomic_store(&P.exit, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    decode_finish(b, tid, nq);
  }
}

// ---------------------------------------------------------------------------
// AT_STAGE_SIZES parity tap (debug copy only): the dense size plane the oracle
// keeps (size[label] = pixels of the component, 0 elsewhere) from the forest:
// entry i is the component size when i is a node id (fg (2r, 2c), bg (2r+1, 2c)
// and (2r+1, 2c+1)) that is its own root and has pixels of its type in its block;
// every other entry is 0 (k_thr_ccl writes sizes at such roots only).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tap_sizes(const uint8_t* thr, const uint32_t* par, const uint32_t* size,
                                                   uint32_t* out, int Wd, int Hd) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Wd * Hd) return;
  const int y = i / Wd, x = i % Wd;
  const int F = (y & ~1) * Wd + (x & ~1);
  const int BW = Wd / 2;
  uint32_t v = 0;
  bool node = true, has = false;
  uint32_t n = 0;  // the node's index (node_F / node_L)
  if ((y & 1) == 0) {
    if (x & 1) node = false;  // (2r, 2c+1) is not a node
    else has = thr[F] == 255 || thr[F + 1] == 255 || (y + 1 < Hd && (thr[F + Wd] == 255 || thr[F + Wd + 1] == 255));
    n = (uint32_t)((y >> 1) * 3 * BW + (x >> 1));
  } else {
    has = thr[i] == 0 || thr[i - Wd] == 0;  // the block's column of this bg node
    n = (uint32_t)((y >> 1) * 3 * BW + BW + x);
  }
  if (node && has && (par[n] & ~kKeptBit) == n) v = size[n];
  out[i] = v;
}

// AT_STAGE_LABELS parity tap (debug copy only): LabelImage's output
// (labeling_allegretti_2019_BKE.cu:340-462) from the forest: label =
// par[par[node]] (node -> local root -> component root), 127 -> 0, a block of
// four 127 pixels -> the pixel index.
__global__ __launch_bounds__(256) void k_tap_labels(const uint8_t* thr, const uint32_t* par, uint32_t* out, int Wd,
                                                    int Hd) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Wd * Hd) return;
  const int y = i / Wd, x = i % Wd;
  const int F = (y & ~1) * Wd + (x & ~1);
  const bool all127 = thr[F] == 127 && thr[F + 1] == 127 && thr[F + Wd] == 127 && thr[F + Wd + 1] == 127;
  uint32_t lab;
  if (all127) lab = (uint32_t)i;
  else if (thr[i] == 127) lab = 0;
  else {
    const int BW = Wd / 2;
    const uint32_t n = thr[i] == 255 ? (uint32_t)((y >> 1) * 3 * BW + (x >> 1)) : (uint32_t)((y >> 1) * 3 * BW + BW + x);
    lab = node_pixel(BW, Wd, par[par[n] & ~kKeptBit] & ~kKeptBit);
  }
  out[i] = lab;
}

hipError_t launch_tap_labels(const uint8_t* thr, const uint32_t* par, uint32_t* out, int Wd, int Hd,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_tap_labels, dim3((Wd * Hd + 255) / 256), dim3(256), 0, st, thr, par, out, Wd, Hd);
  return hipGetLastError();
}

hipError_t launch_tap_sizes(const uint8_t* thr, const uint32_t* par, const uint32_t* size, uint32_t* out, int Wd,
                            int Hd, hipStream_t st) {
  hipLaunchKernelGGL(k_tap_sizes, dim3((Wd * Hd + 255) / 256), dim3(256), 0, st, thr, par, size, out, Wd, Hd);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launch helpers (called from at_api.cpp)
// ---------------------------------------------------------------------------

// Kernel order of one launch sequence; ev (optional, kNumStages+1 events)
// brackets every kernel for per-stage timing.
// ---------------------------------------------------------------------------
// K11: tag pose of every decoded candidate (row A23: estimate_tag_pose at
// apriltags_cuda_detector.cu:433), one thread per detection.
// ---------------------------------------------------------------------------
// One detection per quad of lanes (16 per wave): the four lanes compute the
// same pose, splitting only the quartic's root brackets; lane 0 of the quad stores.
constexpr int kPoseLanes = 4;
constexpr int kPoseGroupsPerFrame = 8;  // 128 detections per pass, looped beyond
#ifndef AT_POSE_WAVES
#define AT_POSE_WAVES 1
#endif
// WAVE (latency mode): a whole wave per detection (the quartic's root brackets
// searched by lane groups, solve_poly_level_wave); else four lanes (a DPP quad)
// per detection, one bracket each.
template <bool WAVE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(AT_POSE_WAVES))) void k_pose(DevBufs b, Params prm) {
  const int sub = (int)(threadIdx.x % kPoseLanes);
  // the control block is final once k_decode has finished: block 0 hands it to
  // the host (replaces a device-to-host copy)
  if (blockIdx.x == 0)
    for (uint32_t w = threadIdx.x; w < b.ctrl_words; w += 64) b.hctrl[w] = b.ctrl[w];
  // the batch's candidates, whatever their frame (k_decode's work list of slots)
  const uint32_t n = *b.det_head;
  constexpr uint32_t kPer = WAVE ? 1 : 64 / kPoseLanes;  // detections per wave
  for (uint32_t i = blockIdx.x * kPer + (WAVE ? 0 : threadIdx.x / kPoseLanes); i < n;  // uniform across the quad
       i += gridDim.x * kPer) {
    const uint32_t slot = b.det_work[i];
    DevDetection& d = b.dets[slot];
    double R[9], t[3], err[2];
    pose::estimate_tag_pose<WAVE>(d.H, d.p, prm.fx, prm.fy, prm.cx, prm.cy, prm.tag_size, R, t, err, sub,
                                  (AT_PROBE_ON(prm) && i == 0 && threadIdx.x == 0) ? b.probe + 16 : nullptr);
    if (WAVE ? threadIdx.x == 0 : sub == 0) {
#pragma unroll
      for (int k = 0; k < 9; k++) d.pose_R[k] = R[k];
#pragma unroll
      for (int k = 0; k < 3; k++) d.pose_t[k] = t[k];
      d.pose_err[0] = err[0];
      d.pose_err[1] = err[1];
      const uint32_t f = slot / kMaxDets, k = slot % kMaxDets;
      if (k < (uint32_t)kDetPoolPerFrame) {  // the host mirror
        DevDetection& h = b.hdets[f * kDetPoolPerFrame + k];
#pragma unroll
        for (int j = 0; j < 9; j++) h.pose_R[j] = R[j];
#pragma unroll
        for (int j = 0; j < 3; j++) h.pose_t[j] = t[j];
        h.pose_err[0] = err[0];
        h.pose_err[1] = err[1];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Shared game-piece preprocessing: preprocess_image of
// src/game_piece_detection/src/game_piece_detection_node.cu:347-379 --
// cv::resize (INTER_LINEAR, 8UC3), BGR->RGB (3 channels) or BGR->GRAY (1),
// convertTo(CV_32F, 1/255), HWC->CHW -- from the BGR frame in HBM, one thread per
// output pixel.  The 8-bit arithmetic is OpenCV 4.9's (imgproc resize.cpp):
//   both scales exactly 2: INTER_AREA's fast path, (s00 + s01 + s10 + s11 + 2) >> 2;
//   else fx = (float)((dx + 0.5) * scale_x - 0.5), sx = floor(fx), fx -= sx, with
//   sx < 0 -> (0, 0) and, from the first column with sx + 1 >= w on, S[sx] * 2048
//   alone (sx >= w - 1 -> (w - 1, 0)); coefficients saturate_cast<short>(c * 2048)
//   (round half even); rows sy, sy + 1 clamped to [0, h - 1];
//   H = S[sx] a0 + S[sx + 3] a1;  v = (((b0 (H0 >> 4)) >> 16) + ((b1 (H1 >> 4)) >> 16) + 2) >> 2;
//   gray Y = (1868 B + 9617 G + 4899 R + 8192) >> 14;  out = (float)v * (float)(1 / 255).
// Restated in oracle/ao_gp.c (parity unpinned against OpenCV itself: no fixture).
// ---------------------------------------------------------------------------
struct GpGeom {
  int w, h, ow, oh, c;
  double sx, sy;  // scale_x, scale_y
  int area2;      // both scales exactly 2
};
__device__ __forceinline__ int gp_coef(float c) { return (int)__builtin_rintf(c * 2048.f); }

__device__ __forceinline__ void gp_pixel(const uint8_t* src, const GpGeom& q, int dx, int dy, float* out) {
  int v[3];
  if (q.area2) {
    const uint8_t* s0 = src + ((size_t)(2 * dy) * q.w + 2 * dx) * 3;
    const uint8_t* s1 = s0 + (size_t)q.w * 3;
#pragma unroll
    for (int c = 0; c < 3; c++) v[c] = (s0[c] + s0[c + 3] + s1[c] + s1[c + 3] + 2) >> 2;
  } else {
    float fx = (float)((dx + 0.5) * q.sx - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { fx = 0.f; sx = 0; }
    const bool one = sx + 1 >= q.w;
    if (one && sx >= q.w - 1) { fx = 0.f; sx = q.w - 1; }
    const int a0 = gp_coef(1.f - fx), a1 = gp_coef(fx);
    float fy = (float)((dy + 0.5) * q.sy - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const int b0 = gp_coef(1.f - fy), b1 = gp_coef(fy);
    const int r0 = min(max(sy, 0), q.h - 1), r1 = min(max(sy + 1, 0), q.h - 1);
    const uint8_t* S0 = src + ((size_t)r0 * q.w + sx) * 3;
    const uint8_t* S1 = src + ((size_t)r1 * q.w + sx) * 3;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const int h0 = one ? S0[c] * 2048 : S0[c] * a0 + S0[c + 3] * a1;
      const int h1 = one ? S1[c] * 2048 : S1[c] * a0 + S1[c + 3] * a1;
      v[c] = (((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2;
    }
  }
  const float a = (float)(1.0 / 255.0);
  const size_t plane = (size_t)q.ow * q.oh, i = (size_t)dy * q.ow + dx;
  if (q.c == 3) {  // BGR -> RGB planes
    out[i] = (float)v[2] * a;
    out[plane + i] = (float)v[1] * a;
    out[2 * plane + i] = (float)v[0] * a;
  } else {
    out[i] = (float)((v[0] * 1868 + v[1] * 9617 + v[2] * 4899 + (1 << 13)) >> 14) * a;
  }
}

__device__ __forceinline__ GpGeom gp_geom(int w, int h, int ow, int oh, int c) {
  GpGeom q;
  q.w = w; q.h = h; q.ow = ow; q.oh = oh; q.c = c;
  q.sx = 1. / ((double)ow / w);
  q.sy = 1. / ((double)oh / h);
  q.area2 = q.sx == 2.0 && q.sy == 2.0;  // |scale - 2| < DBL_EPSILON <=> == 2 near 2
  return q;
}

// in the launch sequence (frames of the batch through the frame table)
__global__ __launch_bounds__(256) void k_gp_pre(DevBufs b, Geom g, Params prm) {
  const int f = blockIdx.z;
  const int dx = blockIdx.x * 64 + threadIdx.x, dy = blockIdx.y * 4 + threadIdx.y;
  if (dx >= prm.gp_w || dy >= prm.gp_h) return;
  const GpGeom q = gp_geom(g.W, g.H, prm.gp_w, prm.gp_h, prm.gp_c);
  gp_pixel(b.frames[f], q, dx, dy, b.gp_out + (size_t)f * prm.gp_c * prm.gp_w * prm.gp_h);
}

// standalone (at_gp_preprocess_device)
__global__ __launch_bounds__(256) void k_gp_pre_one(const uint8_t* src, int w, int h, float* out, int ow, int oh, int c) {
  const int dx = blockIdx.x * 64 + threadIdx.x, dy = blockIdx.y * 4 + threadIdx.y;
  if (dx >= ow || dy >= oh) return;
  gp_pixel(src, gp_geom(w, h, ow, oh, c), dx, dy, out);
}

hipError_t launch_gp_preprocess(const uint8_t* src, int w, int h, float* out, int ow, int oh, int c, hipStream_t st) {
  hipLaunchKernelGGL(k_gp_pre_one, dim3((ow + 63) / 64, (oh + 3) / 4), dim3(64, 4), 0, st, src, w, h, out, ow, oh, c);
  return hipGetLastError();
}

// st2/fork/join: a second stream on which the small-blob kernel runs beside
// the large-blob one (both read k_group's output, neither reads the other's);
// with stage profiling (ev != nullptr) everything stays on st, in order.
// kt (optional): HIP events bracketing one kernel (kt->stage, kStageNames
// order) on the stream it runs on -- the live per-launch duration bench.py
// reports for the roofline; recorded inside the captured graph as well.
// ---------------------------------------------------------------------------
// Annotated image on the GPU: the node's outlined frame
// (apriltag_utils.cu:54-79 -- cv::line of the four sides in green / red / blue /
// blue and the id text at the centre) drawn straight onto the BGR8 frame in HBM.
// Primitives are 2-px-thick segments in drawing order (at_api.cpp builds them as
// node/at_node.cpp's draw_detection_outlines does); a pixel whose centre lies
// within 1 px of a segment takes that segment's colour, the LAST covering segment
// winning as in the sequential CPU drawing: pass 1 records the highest covering
// primitive per pixel (atomicMax), pass 2 lets that primitive paint and clears the
// record (the scratch plane stays zero between calls).  Same double arithmetic as
// the CPU code (no contraction): the images are bit-identical.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool seg_box(const DrawPrim& q, int W, int H, int* x0, int* y0, int* bw, int* bh) {
  const double r = 1.0;  // thickness 2 / 2
  const int xa = (int)floor(fmin(q.x0, q.x1) - r), xb = (int)ceil(fmax(q.x0, q.x1) + r);
  const int ya = (int)floor(fmin(q.y0, q.y1) - r), yb = (int)ceil(fmax(q.y0, q.y1) + r);
  *x0 = max(xa, 0);
  *y0 = max(ya, 0);
  *bw = min(xb, W - 1) - *x0 + 1;
  *bh = min(yb, H - 1) - *y0 + 1;
  return *bw > 0 && *bh > 0;
}
__device__ __forceinline__ bool seg_covers(const DrawPrim& q, int x, int y) {
  const double r = 1.0;
  const double dx = q.x1 - q.x0, dy = q.y1 - q.y0, l2 = dx * dx + dy * dy;
  double u = l2 > 0 ? ((x - q.x0) * dx + (y - q.y0) * dy) / l2 : 0.0;
  u = fmin(1.0, fmax(0.0, u));
  const double ex = q.x0 + u * dx - x, ey = q.y0 + u * dy - y;
  return ex * ex + ey * ey <= r * r;
}
template <bool PAINT>
__global__ __launch_bounds__(256) void k_draw(const DrawPrim* prims, uint32_t* last, uint8_t* bgr, int W, int H) {
  const int p = blockIdx.x;
  const DrawPrim q = prims[p];
  int x0, y0, bw, bh;
  if (!seg_box(q, W, H, &x0, &y0, &bw, &bh)) return;
  for (int i = threadIdx.x; i < bw * bh; i += 256) {
    const int x = x0 + i % bw, y = y0 + i / bw;
    if (!seg_covers(q, x, y)) continue;
    const size_t o = (size_t)y * W + x;
    if (!PAINT) {
      atomicMax(last + o, (uint32_t)(p + 1));
    } else if (last[o] == (uint32_t)(p + 1)) {
      bgr[3 * o + 0] = q.bgr[0];
      bgr[3 * o + 1] = q.bgr[1];
      bgr[3 * o + 2] = q.bgr[2];
      last[o] = 0;
    }
  }
}

hipError_t launch_draw(const DrawPrim* prims, int n, uint32_t* last, uint8_t* bgr, int W, int H, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_draw<false>, dim3(n), dim3(256), 0, st, prims, last, bgr, W, H);
  hipLaunchKernelGGL(k_draw<true>, dim3(n), dim3(256), 0, st, prims, last, bgr, W, H);
  return hipGetLastError();
}

static size_t merge_lds_bytes(const Geom& g) { return (size_t)g.merge_lds; }

// one-time kernel attributes: k_ccl_merge's dynamic LDS beyond the default limit.  The
// attribute belongs to the function for the whole process, so it is set to the largest
// size any geometry launches with (never to this detector's: a later, smaller detector
// would lower the limit below an earlier, larger one's launches)
hipError_t prepare_kernels(const Geom& g) {
  if (!g.merge_cap) return hipSuccess;
  return hipFuncSetAttribute((const void*)k_ccl_merge<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             kMergeLdsMax);
}

hipError_t launch_pipeline(const DevBufs& b, const Geom& g, const Params& prm, int B, int fmt, int nblobwg,
                           hipStream_t st, hipEvent_t* ev, hipStream_t st2, hipEvent_t fork, hipEvent_t join,
                           const KernelTimer* kt) {
  int e = 0;
  auto on = [&](int stage) { return AT_PIPE_STOP(prm) <= 0 || stage < AT_PIPE_STOP(prm); };
  auto mark = [&]() {
    if (ev) (void)hipEventRecord(ev[e++], st);
  };
  hipError_t split_err = hipSuccess;
  auto tk = [&](int stage, hipStream_t s, int which) {
    if (!kt || kt->stage != stage) return;
    if (kt->split) {
      const hipError_t r = kt->split(kt->ctx, which);
      if (r != hipSuccess && split_err == hipSuccess) split_err = r;
    } else {
      (void)hipEventRecord(which ? kt->t1 : kt->t0, s);
    }
  };
  mark();
  {
    dim3 blk(64, 4), grd((g.TW + 63) / 64, (g.TH + 3) / 4, B);
    tk(0, st, 0);
    // latency mode: k_thr_ccl does k_pre's work (one launch less on the B = 1 chain;
    // in throughput mode the longer k_thr_ccl costs ~6 % of concurrent throughput)
    if (!on(0) || g.ctw == 32) {}
    else if (fmt == 0) hipLaunchKernelGGL(k_pre<0>, grd, blk, 0, st, b, g, prm.taps);
    else if (fmt == 1) hipLaunchKernelGGL(k_pre<1>, grd, blk, 0, st, b, g, 1);
    else hipLaunchKernelGGL(k_pre<2>, grd, blk, 0, st, b, g, prm.taps);
    tk(0, st, 1);
    // game-piece network input from the same BGR frames (counted in stage 0's time)
    if (on(0) && prm.gp_c && fmt == 1)
      hipLaunchKernelGGL(k_gp_pre, dim3((prm.gp_w + 63) / 64, (prm.gp_h + 3) / 4, B), dim3(64, 4), 0, st, b, g, prm);
  }
  mark();
  {
    dim3 grd(g.CTX, g.CTY, B);
    tk(1, st, 0);
    if (!on(1)) {}
    else if (g.ctw != 32) hipLaunchKernelGGL((k_thr_ccl<64, -1>), grd, dim3(CclTile<64>::NT), 0, st, b, g, prm);
    else if (fmt == 0) hipLaunchKernelGGL((k_thr_ccl<32, 0>), grd, dim3(CclTile<32>::NT), 0, st, b, g, prm);
    else if (fmt == 1) hipLaunchKernelGGL((k_thr_ccl<32, 1>), grd, dim3(CclTile<32>::NT), 0, st, b, g, prm);
    else hipLaunchKernelGGL((k_thr_ccl<32, 2>), grd, dim3(CclTile<32>::NT), 0, st, b, g, prm);
    tk(1, st, 1);
    mark();
    tk(2, st, 0);
    if (!on(2)) {}
    else if (g.ctw == 32) hipLaunchKernelGGL(k_ccl_border<32>, grd, dim3(BorderRoles<32>::NT), 0, st, b, g);
    else hipLaunchKernelGGL(k_ccl_merge<64>, dim3(B), dim3(1024), merge_lds_bytes(g), st, b, g, prm);
    tk(2, st, 1);
    mark();
  }
  tk(3, st, 0);
  if (on(3) && g.ctw == 32)  // (throughput mode: k_ccl_merge did it)
    hipLaunchKernelGGL(k_ccl_roots, dim3(g.CTX * g.CTY, B), dim3(64), 0, st, b, g);
  tk(3, st, 1);
  mark();
  {
    dim3 blk(64, 4), grd(g.BTX, g.BTY, B);
    tk(4, st, 0);
    if (!on(4)) {}
    else if (g.ctw != 32) hipLaunchKernelGGL(k_boundary<true>, grd, blk, 0, st, b, g);
    else hipLaunchKernelGGL(k_boundary<false>, grd, blk, 0, st, b, g);
    tk(4, st, 1);
    mark();
  }
  tk(5, st, 0);
  if (on(5)) hipLaunchKernelGGL(k_pairs, dim3(B), dim3(1024), 0, st, b, g, AT_PROBE_ON(prm));
  tk(5, st, 1);
  mark();
  tk(6, st, 0);
  if (on(6)) hipLaunchKernelGGL(k_group, dim3(g.ntb, B), dim3(256), 0, st, b, g);
  tk(6, st, 1);
  mark();
  tk(7, st, 0);
  // (latency mode: the blob kernels do k_extents' work themselves, up to 4096-point blobs)
  // latency mode: extents, SelectBlobs and keys inside the small-blob wave and (up to
  // 4096-point blobs) the 512-thread large-blob team.  (Throughput mode keeps
  // k_extents: the fused small-blob kernel needs 2 waves/SIMD, or spills at 4: k_blob_small
  // 0.37 -> 0.61 ms serialized and 5-7 % less concurrent throughput, 13 % with the large
  // blobs fused too and no k_extents launch, profiles/r05_more/fuse_extents_ab_stages.txt)
  const bool fuse_small = g.ctw == 32;
  // latency mode with blobs of up to 4096 points: k_blob_lat holds both kinds (stage
  // profiling and the kernel timer keep the two kernels, to time them apart)
  const bool lat_fused = g.ctw == 32 && g.max_cluster <= 4096 && !ev && !kt;
  if (on(7) && !(g.ctw == 32 && g.max_cluster <= 4096)) hipLaunchKernelGGL(k_extents, dim3(std::max(16, std::min(AT_EXT_GRID, 96 * B))), dim3(256), 0, st, b, g);
  tk(7, st, 1);
  mark();
  auto blob_large = [&](hipStream_t s) {
    tk(9, s, 0);
    // LDS sized for the largest blob the geometry admits (max_cluster = 2 (W + H))
    const bool cap4k = g.max_cluster <= 4096;
    if (!on(9)) return;
    if (lat_fused) {  // latency mode: both blob kinds in one launch (no k_extents, no fork / join)
      hipLaunchKernelGGL(k_blob_lat, dim3(nblobwg), dim3(512), 0, s, b, g, prm);
    } else if (g.ctw == 32 && cap4k) {  // latency mode, timed apart: extents, SelectBlobs and keys in the team
      hipLaunchKernelGGL((k_blob<512, 4096, true>), dim3(nblobwg), dim3(512), 0, s, b, g, prm, 0u, 0, g.nlarge, 0);
    } else if (B < kWideBlobMaxBatch || prm.wide_blob) {  // (latency: one launch, longest blob first)
      if (cap4k) hipLaunchKernelGGL((k_blob<512, 4096>), dim3(nblobwg), dim3(512), 0, s, b, g, prm, 0u, 0, g.nlarge, 0);
      else hipLaunchKernelGGL((k_blob<512, kSortCap>), dim3(nblobwg), dim3(512), 0, s, b, g, prm, 0u, 0, g.nlarge, 0);
    } else {
      // throughput: blobs of 1025-4096 points (size classes 0 .. nlarge-2) in 256-thread
      // teams, the 513-1024-point class (nlarge-1: two thirds of the large blobs) one
      // wave per blob (k_blob_small at CAP 1024: 16 points per lane, no workgroup
      // barriers; round 6's 128-thread teams waited at them 63 % of their wave-cycles);
      // geometries whose blobs exceed 4096 points (1080p) add a
      // launch of CAP-8192 teams over those (class 0 above 4096), AT_BIG_NT threads each:
      // 16 keys per thread keep its theta sort in registers (256-thread teams held 32 and
      // fell back to a bitonic sort of 8192 keys)
      const int lo = prm.lblob_wg ? std::min(prm.lblob_wg, nblobwg) : nblobwg;
      hipLaunchKernelGGL((k_blob<256, 4096>), dim3(lo), dim3(256), 0, s, b, g, prm, 0u, 0, g.nlarge - 1, 0);
      hipLaunchKernelGGL((k_blob_small<false, 1024, 3, 9>), dim3(nblobwg), dim3(256), 0, s, b, g, prm, g.nlarge - 1, g.nlarge, 1);
      if (!cap4k)
        hipLaunchKernelGGL((k_blob<AT_BIG_NT, kSortCap>), dim3(std::min(nblobwg, AT_BIG_BLOB_WG)), dim3(AT_BIG_NT), 0, s, b, g,
                           prm, 4096u, 0, 1, 2);
    }
    tk(9, s, 1);
  };
  auto blob_small = [&](hipStream_t s) {
    tk(8, s, 0);
    if (!on(8) || lat_fused) {}
    else if (fuse_small) hipLaunchKernelGGL(k_blob_small<true>, dim3(nblobwg * 2), dim3(256), 0, s, b, g, prm, g.nlarge, kNumCls, 0);
    else hipLaunchKernelGGL(k_blob_small<false>, dim3(prm.sblob_wg ? prm.sblob_wg : nblobwg * 2), dim3(256), 0, s, b, g, prm, g.nlarge, kNumCls, 0);
    tk(8, s, 1);
  };
  // the side fits of the blobs the throughput-mode (non-FUSE) blob kernels fitted:
  // every class, or (latency mode above 4096-point blobs) the large classes only.  In
  // the stage profile it counts with k_blob; the kernel timer's k_blob span leaves it out
  const int fin_c1 = g.ctw != 32 ? kNumCls : g.max_cluster > 4096 ? g.nlarge : 0;
  auto quad_fin = [&](hipStream_t s) {
    if (fin_c1 > 0 && on(9) && (!AT_DIAG_ANY(prm) || AT_DIAG_STOP(prm, 5)))  // (a blob-phase cut leaves no side moments)
      hipLaunchKernelGGL(k_quad_fin, dim3(std::max(1, std::min(2048, 8 * B))), dim3(256), 0, s, b, g, prm, 0, fin_c1);
  };
  if (ev || !st2 || lat_fused) {
    blob_small(st);
    mark();
    blob_large(st);
    quad_fin(st);
    mark();
  } else {
    hipError_t e;
    if ((e = hipEventRecord(fork, st))) return e;
    if ((e = hipStreamWaitEvent(st2, fork, 0))) return e;
    // the kernel that finishes last stays on the main stream, so neither the fork's
    // start delay nor the join's wait lies on the chain: the large-blob kernel
    // (extents, keys and up to 4096 points per team: ~43 us at B = 1) on the main
    // stream, the small-blob kernel (~35 us) forked
    if (AT_FORK_SMALL) {
      blob_large(st);
      blob_small(st2);
    } else {
      blob_small(st);
      blob_large(st2);
    }
    if ((e = hipEventRecord(join, st2))) return e;
    if ((e = hipStreamWaitEvent(st, join, 0))) return e;
    quad_fin(st);
  }
  // latency mode: the pose inside k_decode (a second wave per workgroup) unless
  // stages or one kernel are timed (the control block then leaves with k_pose,
  // after the timed kernel's device-clock span)
  const bool pose_fused = AT_POSE_IN_DECODE && prm.tag_size > 0 && on(11) && B < kWideBlobMaxBatch && !ev && b.kt_stage < 0 && !kt;
  tk(10, st, 0);
  {
    // one wave per workgroup, persistent over the accepted quads: enough groups
    // for every quad of a full batch to start at once (16 per CU at 8.5 KB LDS)
    // (the experiment knob never exceeds the grid the refine scratch was sized for)
    const dim3 grd(prm.dec_wg ? std::min(prm.dec_wg, decode_grid(nblobwg, B)) : decode_grid(nblobwg, B));
    if (on(10) && pose_fused) hipLaunchKernelGGL(k_decode<true>, grd, dim3(128), 0, st, b, g, prm, B, fmt);
    else if (on(10)) hipLaunchKernelGGL(k_decode<false>, grd, dim3(kDecodeThreads), 0, st, b, g, prm, B, fmt);
  }
  tk(10, st, 1);
  mark();
  // the timed kernel's device-clock span (after it, outside its timing events;
  // before k_pose hands the control block to the host)
  if (b.kt_stage >= 1 && b.kt_stage <= 10 && b.kt_stage != 3 && b.kt_stage != 5 && b.kt_stage != 6)
    hipLaunchKernelGGL(k_kt_span, dim3(kKtSpanWgs), dim3(256), 0, st, b);
  tk(11, st, 0);
  // latency mode: a wave per detection; throughput mode: four lanes per detection
  if (prm.tag_size > 0 && on(11) && !pose_fused) {
    if (B < kWideBlobMaxBatch) hipLaunchKernelGGL(k_pose<true>, dim3(32 * B), dim3(64), 0, st, b, prm);
    else hipLaunchKernelGGL(k_pose<false>, dim3(kPoseGroupsPerFrame * B), dim3(64), 0, st, b, prm);
  }
  tk(11, st, 1);
  mark();
  if (split_err != hipSuccess) return split_err;
  return hipGetLastError();
}

}  // namespace at
