"""Python mirror of the reference detector interface over the C ABI.

``GpuDetector`` follows frc971::apriltag::GpuDetector
(src/apriltags_cuda/include/apriltags_cuda/apriltag_gpu.h:77-359): construct
once per camera with width, height and calibration, call ``detect(frame)``
per frame, read ``detections()``; the debug copy-outs
(apriltag_gpu.h:98-183) are the ``copy_*`` methods.  Everything runs in
``libat_hip.so`` (HIP kernels for gfx950); there is no CPU fallback: if the
library or a GPU is missing the constructor raises.
"""
import ctypes as C
import math
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# AT_HIP_LIB overrides the library (A/B timing of build variants, tools/ab.sh)
LIB_PATH = os.environ.get("AT_HIP_LIB") or os.path.join(_HERE, "libat_hip.so")

AT_FMT_YUYV, AT_FMT_BGR8, AT_FMT_GRAY8 = 0, 1, 2
(AT_STAGE_GRAY, AT_STAGE_DECIMATED, AT_STAGE_THRESHOLD, AT_STAGE_LABELS, AT_STAGE_SIZES,
 AT_STAGE_NUM_POINTS, AT_STAGE_NUM_PAIRS, AT_STAGE_QUADS, AT_STAGE_POINTS, AT_STAGE_BLOB_POINTS,
 AT_STAGE_NUM_PAIR_ENTRIES, AT_STAGE_PROBE) = range(12)
AT_E_CAPACITY = -3

# Symbols declared in include/at_api.h (checked by tests/test_abi.py).
EXPORTS = [
    "at_config_default", "at_create", "at_detect", "at_detect_batch", "at_detect_device",
    "at_enqueue_device", "at_collect", "at_frame_status", "at_debug_copy", "at_destroy",
    "at_strerror", "at_family_num_known", "at_family_entry", "at_abi_version",
    "at_set_profiling", "at_stage_times", "at_stage_name", "at_poses", "at_tag_detections",
    "at_set_kernel_timer", "at_kernel_time", "at_batch_stats", "at_stream_wait",
    "at_gp_enable", "at_gp_tensor", "at_gp_copy", "at_gp_preprocess_device", "at_set_debug_taps",
    "at_draw_outlines_device", "at_detections", "at_max_detections", "at_annotate_staged", "at_enqueue_host",
    "at_kernel_span", "at_host_alloc", "at_host_free",
]

TAG_SIZE = 0.1651  # metres, apriltags_cuda_detector.hpp:39


class AtConfig(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("family", C.c_char_p),
        ("quad_decimate", C.c_float), ("refine_edges", C.c_int), ("decode_sharpening", C.c_double),
        ("min_white_black_diff", C.c_int), ("min_cluster_pixels", C.c_int), ("max_nmaxima", C.c_int),
        ("max_line_fit_mse", C.c_float), ("cos_critical_rad", C.c_double),
        ("device", C.c_int), ("max_batch", C.c_int), ("tag_size", C.c_double),
    ]


class AtCamera(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3")]


class AtDetection(C.Structure):
    _fields_ = [
        ("id", C.c_int32), ("hamming", C.c_int32), ("decision_margin", C.c_float),
        ("H", C.c_double * 9), ("c", C.c_double * 2), ("p", (C.c_double * 2) * 4),
    ]


class AtPose(C.Structure):
    _fields_ = [("id", C.c_int32), ("R", C.c_double * 9), ("t", C.c_double * 3), ("err", C.c_double)]


class AtTagDetection(C.Structure):
    _fields_ = [("id", C.c_int32), ("camera", C.c_double * 3), ("robot", C.c_double * 3),
                ("distance", C.c_double), ("err", C.c_double)]


class AtQuadRecord(C.Structure):
    _fields_ = [
        ("blob_index", C.c_uint32), ("valid", C.c_uint32), ("accepted", C.c_uint32),
        ("indices", C.c_uint16 * 4), ("corners", (C.c_float * 2) * 4),
    ]


@dataclass
class Detection:
    """apriltag_detection_t fields the node consumes (apriltags_cuda_detector.cu:425-496)."""
    id: int
    hamming: int
    decision_margin: float
    H: np.ndarray
    c: np.ndarray
    p: np.ndarray


@dataclass
class Pose:
    """apriltag_pose_t + the error estimate_tag_pose returns (apriltags_cuda_detector.cu:432-433)."""
    id: int
    R: np.ndarray
    t: np.ndarray
    err: float


@dataclass
class TagDetection:
    """DetectionData of the node loop (apriltags_cuda_detector.cu:425-462): camera- and
    robot-frame position, distance from the camera, pose error."""
    id: int
    camera: np.ndarray
    robot: np.ndarray
    distance: float
    err: float


@dataclass
class CameraMatrix:
    """apriltag_gpu.h:61-66"""
    fx: float
    cx: float
    fy: float
    cy: float


@dataclass
class DistCoeffs:
    """apriltag_gpu.h:68-74"""
    k1: float
    k2: float
    p1: float
    p2: float
    k3: float


# Intrinsics the reference's own test uses (test/gpu_detector_test.cu:62-73).
TEST_CAMERA = CameraMatrix(fx=905.495617, cx=609.916016, fy=907.909470, cy=352.682645)
TEST_DIST = DistCoeffs(k1=0.059238, k2=-0.075154, p1=-0.003801, p2=0.001113, k3=0.0)

_LIB = None


def load_library(path: str = LIB_PATH):
    """Load libat_hip.so; raises if it is missing (no CPU fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise RuntimeError("libat_hip.so not built: run `make -C ros_vision_amd/csrc` "
                           "(or __graft_entry__.build())")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7
    # (same soname as /opt/rocm's).  Whichever loads first is the one both use,
    # and torch only initialises on its own copy, so let torch load first when
    # it is installed (it provides device memory / torch.distributed to callers).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    L.at_config_default.argtypes = [C.POINTER(AtConfig), C.c_int, C.c_int]
    L.at_create.argtypes = [C.POINTER(AtConfig), C.POINTER(AtCamera), C.POINTER(C.c_void_p)]
    L.at_detect.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(AtDetection), C.c_int, C.POINTER(C.c_int)]
    L.at_detect_batch.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.c_int, C.c_int, C.POINTER(AtDetection),
                                  C.c_int, C.POINTER(C.c_int)]
    L.at_detect_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(AtDetection),
                                   C.c_int, C.POINTER(C.c_int)]
    L.at_enqueue_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int]
    if hasattr(L, "at_enqueue_host"):
        L.at_enqueue_host.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.c_int, C.c_int]
    L.at_collect.argtypes = [C.c_void_p, C.POINTER(AtDetection), C.c_int, C.POINTER(C.c_int)]
    L.at_stream_wait.argtypes = [C.c_void_p, C.c_void_p]
    L.at_frame_status.argtypes = [C.c_void_p, C.c_int]
    L.at_debug_copy.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t]
    L.at_debug_copy.restype = C.c_longlong
    L.at_destroy.argtypes = [C.c_void_p]
    L.at_strerror.restype = C.c_char_p
    L.at_strerror.argtypes = [C.c_int]
    L.at_family_num_known.argtypes = [C.c_char_p]
    L.at_family_entry.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_uint64)]
    L.at_set_profiling.argtypes = [C.c_void_p, C.c_int]
    L.at_stage_times.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int]
    L.at_stage_name.restype = C.c_char_p
    L.at_stage_name.argtypes = [C.c_int]
    L.at_poses.argtypes = [C.c_void_p, C.c_int, C.POINTER(AtPose), C.c_int]
    L.at_set_kernel_timer.argtypes = [C.c_void_p, C.c_int]
    L.at_kernel_time.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_longlong)]
    if hasattr(L, "at_kernel_span"):
        L.at_kernel_span.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_longlong)]
    L.at_batch_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    L.at_tag_detections.argtypes = [C.POINTER(AtPose), C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                    C.POINTER(AtTagDetection)]
    if hasattr(L, "at_set_debug_taps"):
        L.at_set_debug_taps.argtypes = [C.c_void_p, C.c_int]
    if hasattr(L, "at_gp_enable"):  # (A/B builds of older sources lack it)
        L.at_gp_enable.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
        L.at_gp_tensor.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
        L.at_gp_copy.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
        L.at_gp_preprocess_device.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                              C.c_void_p]
    if hasattr(L, "at_draw_outlines_device"):
        L.at_draw_outlines_device.argtypes = [C.c_void_p, C.POINTER(AtDetection), C.c_int, C.c_void_p]
    if hasattr(L, "at_detections"):  # (A/B builds of older sources lack them)
        L.at_detections.argtypes = [C.c_void_p, C.c_int, C.POINTER(AtDetection), C.c_int]
        L.at_annotate_staged.argtypes = [C.c_void_p, C.c_int, C.POINTER(AtDetection), C.c_int, C.c_void_p]
    _LIB = L
    return L


def game_piece_preprocess_device(bgr_ptr: int, width: int, height: int, out_ptr: int, out_width: int = 640,
                                 out_height: int = 640, channels: int = 3, stream: int = 0):
    """at_gp_preprocess_device: preprocess_image of one device-resident BGR8 image
    into a device NCHW float buffer, enqueued on `stream` (hipStream_t handle)."""
    _check(load_library().at_gp_preprocess_device(bgr_ptr, width, height, out_ptr, out_width, out_height, channels,
                                                  stream or None), "at_gp_preprocess_device")


def family_entries(family: str = "tag36h11"):
    """(id, code) pairs of the codewords known to the library."""
    L = load_library()
    n = L.at_family_num_known(family.encode())
    out = []
    for i in range(n):
        tid, code = C.c_int(), C.c_uint64()
        L.at_family_entry(family.encode(), i, C.byref(tid), C.byref(code))
        out.append((tid.value, code.value))
    return out


def tag_detections(poses, extrinsic_rotation=None, extrinsic_offset=None):
    """The node's per-frame tail (apriltags_cuda_detector.cu:425-462, 595-599):
    transformCameraToRobot + distance, sorted closest first.  Runs in libat_hip.so
    (host code, no device needed)."""
    L = load_library()
    n = len(poses)
    arr = (AtPose * max(1, n))()
    for i, p in enumerate(poses):
        arr[i].id = int(p.id)
        arr[i].R[:] = [float(x) for x in np.asarray(p.R, np.float64).ravel()]
        arr[i].t[:] = [float(x) for x in np.asarray(p.t, np.float64).ravel()]
        arr[i].err = float(p.err)
    Rp = tp = None
    if extrinsic_rotation is not None:
        Rv = np.ascontiguousarray(extrinsic_rotation, np.float64).reshape(9)
        Rp = Rv.ctypes.data_as(C.POINTER(C.c_double))
    if extrinsic_offset is not None:
        tv = np.ascontiguousarray(extrinsic_offset, np.float64).reshape(3)
        tp = tv.ctypes.data_as(C.POINTER(C.c_double))
    out = (AtTagDetection * max(1, n))()
    _check(L.at_tag_detections(arr, n, Rp, tp, out), "at_tag_detections")
    return [TagDetection(id=o.id, camera=np.array(list(o.camera)), robot=np.array(list(o.robot)),
                         distance=o.distance, err=o.err) for o in out[:n]]


def _check(rc, what):
    if rc < 0:
        raise RuntimeError("%s failed: %s (%d)" % (what, load_library().at_strerror(rc).decode(), rc))
    return rc


class GpuDetector:
    """Drop-in for frc971::apriltag::GpuDetector on MI355X (one instance per camera)."""

    MAX_DETECTIONS = 64  # per frame in the collect buffer; frames with more are fetched whole (at_detections)
    DEBUG_TAPS = False     # default of debug_taps (the parity tests turn it on for their module)

    def __init__(self, width, height, camera_matrix: CameraMatrix = TEST_CAMERA,
                 distortion_coefficients: DistCoeffs = TEST_DIST, family="tag36h11",
                 max_batch=1, device=0, pinned_out=False, debug_taps=None, **overrides):
        L = load_library()
        self.width, self.height, self.max_batch = int(width), int(height), int(max_batch)
        cfg = AtConfig()
        L.at_config_default(C.byref(cfg), self.width, self.height)
        self._family = family.encode()
        cfg.family = self._family
        cfg.max_batch = self.max_batch
        cfg.device = int(device)
        for k, v in overrides.items():
            setattr(cfg, k, v)
        cam = AtCamera(fx=camera_matrix.fx, fy=camera_matrix.fy, cx=camera_matrix.cx, cy=camera_matrix.cy,
                       k1=distortion_coefficients.k1, k2=distortion_coefficients.k2,
                       p1=distortion_coefficients.p1, p2=distortion_coefficients.p2,
                       k3=distortion_coefficients.k3)
        h = C.c_void_p()
        _check(L.at_create(C.byref(cfg), C.byref(cam), C.byref(h)), "at_create")
        self._h = h
        if self.DEBUG_TAPS if debug_taps is None else debug_taps:
            _check(L.at_set_debug_taps(h, 1), "at_set_debug_taps")  # copy_blob_points needs them
        self._cap = self.MAX_DETECTIONS
        self._out_t = None
        if pinned_out:
            # at_collect writes the detections straight into page-locked memory (torch owns
            # it), so a caller can copy them to the device asynchronously without staging
            import torch
            nb = C.sizeof(AtDetection) * self._cap * self.max_batch
            self._out_t = torch.empty(nb, dtype=torch.uint8).pin_memory()
            self._out = (AtDetection * (self._cap * self.max_batch)).from_address(self._out_t.data_ptr())
        else:
            self._out = (AtDetection * (self._cap * self.max_batch))()
        self._n = (C.c_int * self.max_batch)()
        self._last = [[] for _ in range(self.max_batch)]
        self._last_status = 0

    def close(self):
        if getattr(self, "_h", None):
            load_library().at_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    # ---- detection ---------------------------------------------------------
    def _frame_records(self, f):
        """at_detection records of frame f of the last batch (all of them: a frame with
        more than the collect buffer holds is fetched again with at_detections)."""
        n = self._n[f]
        if n <= self._cap:
            return [self._out[f * self._cap + i] for i in range(n)]
        buf = (AtDetection * n)()
        got = _check(load_library().at_detections(self._h, f, buf, n), "at_detections")
        return list(buf[:got])

    def frame_record_bytes(self, f):
        """Every at_detection record of frame f of the last batch, as bytes (what a peer
        sends rank 0, multigpu.RecordGather)."""
        return b"".join(bytes(r) for r in self._frame_records(f))

    def _unpack(self, nframes):
        res = []
        for f in range(nframes):
            dets = []
            for d in self._frame_records(f):
                dets.append(Detection(id=d.id, hamming=d.hamming, decision_margin=d.decision_margin,
                                      H=np.array(list(d.H)).reshape(3, 3), c=np.array(list(d.c)),
                                      p=np.array([[d.p[k][0], d.p[k][1]] for k in range(4)])))
            res.append(dets)
        self._last = res
        return res

    def detect(self, frame: np.ndarray, fmt: int = AT_FMT_YUYV):
        """GpuDetector::Detect (apriltag_gpu.cu:725): one host frame, synchronous."""
        frame = np.ascontiguousarray(frame, dtype=np.uint8)
        rc = load_library().at_detect(self._h, frame.ctypes.data, fmt, self._out, self._cap, self._n)
        self._last_status = rc
        if rc < 0 and rc != AT_E_CAPACITY:
            _check(rc, "at_detect")
        return self._unpack(1)[0]

    def detect_count(self, frame: np.ndarray, fmt: int = AT_FMT_YUYV):
        """at_detect without building Python objects: returns the detection count
        (the detections are in this detector's at_detection buffer)."""
        rc = load_library().at_detect(self._h, frame.ctypes.data, fmt, self._out, self._cap, self._n)
        if rc < 0 and rc != AT_E_CAPACITY:
            _check(rc, "at_detect")
        return self._n[0]

    def detect_batch(self, frames, fmt: int = AT_FMT_YUYV):
        frames = [np.ascontiguousarray(f, dtype=np.uint8) for f in frames]
        ptrs = (C.c_void_p * len(frames))(*[f.ctypes.data for f in frames])
        rc = load_library().at_detect_batch(self._h, ptrs, len(frames), fmt, self._out, self._cap, self._n)
        self._last_status = rc
        if rc < 0 and rc != AT_E_CAPACITY:
            _check(rc, "at_detect_batch")
        return self._unpack(len(frames))

    def detect_device(self, dev_ptr: int, frame_stride: int, nframes: int, fmt: int = AT_FMT_YUYV,
                      counts_only=False):
        """Frames already resident in device memory (e.g. a torch.cuda tensor's data_ptr())."""
        rc = load_library().at_detect_device(self._h, C.c_void_p(dev_ptr), frame_stride, nframes, fmt,
                                             self._out, self._cap, self._n)
        self._last_status = rc
        if rc < 0 and rc != AT_E_CAPACITY:
            _check(rc, "at_detect_device")
        if counts_only:
            return [self._n[f] for f in range(nframes)]
        return self._unpack(nframes)

    def enqueue_device(self, dev_ptr: int, frame_stride: int, nframes: int, fmt: int = AT_FMT_YUYV):
        _check(load_library().at_enqueue_device(self._h, C.c_void_p(dev_ptr), frame_stride, nframes, fmt),
               "at_enqueue_device")
        self._pending = nframes

    def enqueue_host(self, host_ptrs, fmt: int = AT_FMT_YUYV):
        """at_enqueue_host: host frames (addresses; page-locked for an asynchronous
        copy) copied and detected on this detector's stream; collect() later."""
        ptrs = (C.c_void_p * len(host_ptrs))(*host_ptrs)
        _check(load_library().at_enqueue_host(self._h, ptrs, len(host_ptrs), fmt), "at_enqueue_host")
        self._pending = len(host_ptrs)

    def wait_stream(self, stream_handle: int):
        """at_stream_wait: the next enqueued batch waits (on the GPU) for the work queued
        so far on a HIP stream, e.g. torch.cuda.current_stream().cuda_stream."""
        _check(load_library().at_stream_wait(self._h, C.c_void_p(stream_handle)), "at_stream_wait")

    def poses(self, frame=0):
        """Pose of each detection of `frame` of the last batch (same order as its
        detections), computed on the GPU (k_pose) when tag_size > 0."""
        cap = max(self._n[frame], 1)
        buf = (AtPose * cap)()
        n = _check(load_library().at_poses(self._h, frame, buf, cap), "at_poses")
        return [Pose(id=b.id, R=np.array(list(b.R)).reshape(3, 3), t=np.array(list(b.t)), err=b.err)
                for b in buf[:min(n, cap)]]

    def collect(self, counts_only=False):
        """at_collect: wait for the batch, run the host tail.  The detections land in
        this detector's at_detection buffer; counts_only=True skips building Python
        objects from it and returns the per-frame counts (what a C++ caller sees)."""
        rc = load_library().at_collect(self._h, self._out, self._cap, self._n)
        if rc < 0 and rc != AT_E_CAPACITY:
            _check(rc, "at_collect")
        if counts_only:
            return [self._n[f] for f in range(self._pending)]
        return self._unpack(self._pending)

    def results(self):
        """Detections of every frame of the last collected batch (after
        collect(counts_only=True), builds the Python objects from the buffer)."""
        return self._unpack(self._pending)

    # ---- per-stage timing (the reference's CudaEvent stage timers,
    #      apriltag_gpu.cu:1118-1163) ----------------------------------------
    def set_profiling(self, enable=True):
        _check(load_library().at_set_profiling(self._h, int(enable)), "at_set_profiling")

    def stage_times(self):
        """{stage name: (mean ms per batch, batches)} accumulated since profiling was enabled."""
        L = load_library()
        buf = (C.c_double * 32)()
        n = _check(L.at_stage_times(self._h, buf, 32), "at_stage_times")
        batches = int(buf[n]) if n < 32 else 0
        return {L.at_stage_name(i).decode(): buf[i] for i in range(n)}, batches

    def set_kernel_timer(self, stage_name=None):
        """Time one kernel live inside the normal launch sequence (None: off)."""
        L = load_library()
        stage = -1
        if stage_name is not None:
            names = [L.at_stage_name(i).decode() for i in range(32)]
            stage = names.index(stage_name)
        _check(L.at_set_kernel_timer(self._h, stage), "at_set_kernel_timer")

    def kernel_time(self):
        """(mean ms per launch, launches) of the timed kernel (HIP events on its stream)."""
        ms, n = C.c_double(), C.c_longlong()
        _check(load_library().at_kernel_time(self._h, C.byref(ms), C.byref(n)), "at_kernel_time")
        return ms.value, n.value

    def kernel_span(self):
        """(mean ms per launch, launches) of the timed kernel on the device clock (first
        workgroup start -> last workgroup end; the span a rocprofv3 kernel trace times)."""
        ms, n = C.c_double(), C.c_longlong()
        _check(load_library().at_kernel_span(self._h, C.byref(ms), C.byref(n)), "at_kernel_span")
        return ms.value, n.value

    BATCH_STATS = ("frames", "boundary_points", "pairs", "small_blob_points", "large_blob_points",
                   "quads", "candidates", "host_wait_us_total", "host_tail_us_total", "ccl_listed_roots",
                   "ccl_listed_roots_max", "ccl_fallback_frames")

    def batch_stats(self):
        """Work counts of the last collected batch (see at_batch_stats)."""
        buf = (C.c_uint64 * len(self.BATCH_STATS))()
        n = _check(load_library().at_batch_stats(self._h, buf, len(buf)), "at_batch_stats")
        return dict(zip(self.BATCH_STATS, [int(x) for x in buf[:n]]))

    def detections(self, frame=0):
        """GpuDetector::Detections (apriltag_gpu.h:93), sorted by id."""
        return self._last[frame]

    def _records_array(self, frame):
        recs = self._frame_records(frame)
        arr = (AtDetection * max(1, len(recs)))(*recs)
        return arr, len(recs)

    def draw_outlines_device(self, bgr_ptr: int, frame=0):
        """at_draw_outlines_device: the annotated image of `frame` of the last batch
        (outlines and ids, apriltag_utils.cu:54-79) drawn onto the device-resident
        BGR8 image at `bgr_ptr` (width x height x 3)."""
        arr, n = self._records_array(frame)
        _check(load_library().at_draw_outlines_device(self._h, arr, n, bgr_ptr), "at_draw_outlines_device")

    def annotate_staged(self, frame=0):
        """at_annotate_staged: the annotated image of host BGR8 frame `frame` of the last
        batch, drawn on its staged copy in HBM; returns it (H, W, 3) uint8."""
        arr, n = self._records_array(frame)
        out = np.empty((self.height, self.width, 3), np.uint8)
        _check(load_library().at_annotate_staged(self._h, frame, arr, n, out.ctypes.data), "at_annotate_staged")
        return out

    def frame_status(self, frame=0):
        return load_library().at_frame_status(self._h, frame)

    # ---- shared game-piece preprocessing (game_piece_detection_node.cu:347-379) ----
    def enable_game_piece_input(self, width=640, height=640, channels=3):
        """Also produce preprocess_image's NCHW float tensor of every BGR8 frame
        (resize INTER_LINEAR, BGR->RGB / GRAY, x 1/255) in each later batch."""
        _check(load_library().at_gp_enable(self._h, width, height, channels), "at_gp_enable")
        self._gp = (channels, height, width)

    def game_piece_tensor_ptr(self, frame=0):
        """Device pointer of frame `frame`'s tensor of the last (BGR8) batch."""
        ptr = C.c_void_p()
        _check(load_library().at_gp_tensor(self._h, frame, C.byref(ptr)), "at_gp_tensor")
        return ptr.value

    def game_piece_tensor(self, frame=0):
        """Host copy (channels, height, width) float32 of frame `frame`'s tensor."""
        out = np.empty(self._gp, np.float32)
        _check(load_library().at_gp_copy(self._h, frame, out.ctypes.data, out.size), "at_gp_copy")
        return out

    # ---- parity taps (apriltag_gpu.h:98-183) -------------------------------
    def _copy(self, stage, frame, nbytes, dtype):
        buf = np.empty(nbytes // np.dtype(dtype).itemsize, dtype=dtype)
        n = load_library().at_debug_copy(self._h, stage, frame, buf.ctypes.data, buf.nbytes)
        _check(int(n), "at_debug_copy")
        return buf[: n // np.dtype(dtype).itemsize]

    def copy_gray(self, frame=0):
        return self._copy(AT_STAGE_GRAY, frame, self.width * self.height, np.uint8).reshape(self.height, self.width)

    def copy_decimated(self, frame=0):
        return self._copy(AT_STAGE_DECIMATED, frame, self.width * self.height // 4,
                          np.uint8).reshape(self.height // 2, self.width // 2)

    def copy_thresholded(self, frame=0):
        return self._copy(AT_STAGE_THRESHOLD, frame, self.width * self.height // 4,
                          np.uint8).reshape(self.height // 2, self.width // 2)

    def copy_union_markers(self, frame=0):
        return self._copy(AT_STAGE_LABELS, frame, self.width * self.height,
                          np.uint32).reshape(self.height // 2, self.width // 2)

    def copy_union_markers_size(self, frame=0):
        return self._copy(AT_STAGE_SIZES, frame, self.width * self.height, np.uint32)

    def num_points(self, frame=0):
        return int(self._copy(AT_STAGE_NUM_POINTS, frame, 4, np.uint32)[0])

    def num_pairs(self, frame=0):
        return int(self._copy(AT_STAGE_NUM_PAIRS, frame, 4, np.uint32)[0])

    def num_pair_entries(self, frame=0):
        """Per-tile pair-histogram entries k_boundary handed to k_pairs (diagnostic)."""
        return int(self._copy(AT_STAGE_NUM_PAIR_ENTRIES, frame, 4, np.uint32)[0])

    def copy_probe(self):
        """Kernel phase clock stamps (100 MHz wall clock) written when AT_PHASE_PROBE is set."""
        return self._copy(AT_STAGE_PROBE, 0, 8 * 256, np.uint64)

    def copy_points(self, frame=0):
        """Boundary points (QuadBoundaryPoint keys), device emission order."""
        return self._copy(AT_STAGE_POINTS, frame, 8 * max(1, self.num_points(frame)), np.uint64)

    def copy_blob_points(self, frame=0):
        """IndexPoint keys of the selected blobs in (blob, theta, plane, y, x) order."""
        L = load_library()
        need = L.at_debug_copy(self._h, AT_STAGE_BLOB_POINTS, frame, C.c_void_p(1), 0)
        need = max(int(need), 8)
        return self._copy(AT_STAGE_BLOB_POINTS, frame, need, np.uint64)

    def copy_quads(self, frame=0):
        recs = (AtQuadRecord * 4096)()
        n = load_library().at_debug_copy(self._h, AT_STAGE_QUADS, frame, C.cast(recs, C.c_void_p), C.sizeof(recs))
        _check(int(n), "at_debug_copy")
        out = []
        for i in range(int(n) // C.sizeof(AtQuadRecord)):
            r = recs[i]
            out.append(dict(blob_index=r.blob_index, valid=bool(r.valid), accepted=bool(r.accepted),
                            indices=list(r.indices),
                            corners=np.array([[r.corners[k][0], r.corners[k][1]] for k in range(4)], np.float32)))
        return out


def default_cos_critical_rad():
    return math.cos(10.0 * math.pi / 180.0)
