"""ctypes binding of the CPU oracle (oracle/libao_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class Params(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int),
        ("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
        ("k1", C.c_double), ("k2", C.c_double), ("p1", C.c_double), ("p2", C.c_double), ("k3", C.c_double),
        ("min_white_black_diff", C.c_int), ("min_cluster_pixels", C.c_int), ("max_nmaxima", C.c_int),
        ("max_line_fit_mse", C.c_float), ("cos_critical_rad", C.c_double),
        ("decode_sharpening", C.c_double), ("refine_edges", C.c_int), ("family", C.c_char_p),
    ]


class Detection(C.Structure):
    _fields_ = [
        ("id", C.c_int32), ("hamming", C.c_int32), ("decision_margin", C.c_float),
        ("H", C.c_double * 9), ("c", C.c_double * 2), ("p", (C.c_double * 2) * 4),
        ("blob_index", C.c_int32),
    ]


class FitQuad(C.Structure):
    _fields_ = [
        ("blob_index", C.c_uint16), ("valid", C.c_uint8), ("indices", C.c_uint16 * 4),
        ("Mx", C.c_int32 * 4), ("My", C.c_int32 * 4), ("W", C.c_int32 * 4),
        ("Mxx", C.c_int64 * 4), ("Myy", C.c_int64 * 4), ("Mxy", C.c_int64 * 4), ("N", C.c_int32 * 4),
    ]


class Quad(C.Structure):
    _fields_ = [("corners", (C.c_float * 2) * 4), ("reversed_border", C.c_int), ("blob_index", C.c_uint32)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libao_oracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.ao_create.restype = C.c_void_p
        L.ao_create.argtypes = [C.POINTER(Params)]
        L.ao_destroy.argtypes = [C.c_void_p]
        L.ao_detect.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.ao_default_params.argtypes = [C.POINTER(Params), C.c_int, C.c_int]
        for name, rt in [("ao_gray", C.POINTER(C.c_uint8)), ("ao_decimated", C.POINTER(C.c_uint8)),
                         ("ao_thresholded", C.POINTER(C.c_uint8)), ("ao_labels", C.POINTER(C.c_uint32)),
                         ("ao_sizes", C.POINTER(C.c_uint32)), ("ao_sorted_points", C.POINTER(C.c_uint64)),
                         ("ao_sorted_index_points", C.POINTER(C.c_uint64)), ("ao_errs", C.POINTER(C.c_double)),
                         ("ao_filtered_errs", C.POINTER(C.c_double)), ("ao_fitquads", C.POINTER(FitQuad)),
                         ("ao_quads", C.POINTER(Quad)), ("ao_detections", C.POINTER(Detection))]:
            getattr(L, name).restype = rt
            getattr(L, name).argtypes = [C.c_void_p]
        for name in ["ao_num_points", "ao_num_pairs", "ao_num_selected_points", "ao_num_peaks",
                     "ao_num_fitquads", "ao_num_quads", "ao_num_detections", "ao_status"]:
            getattr(L, name).restype = C.c_int
            getattr(L, name).argtypes = [C.c_void_p]
        L.ao_family_code.restype = C.c_uint64
        L.ao_family_code.argtypes = [C.c_char_p, C.c_int]
        L.ao_family_ncodes.restype = C.c_int
        L.ao_family_ncodes.argtypes = [C.c_char_p]
        L.ao_family_nbits.restype = C.c_int
        L.ao_family_nbits.argtypes = [C.c_char_p]
        L.ao_family_id.restype = C.c_int
        L.ao_family_id.argtypes = [C.c_char_p, C.c_int]
        L.ao_family_bit.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.ao_rotate90_n.restype = C.c_uint64
        L.ao_rotate90_n.argtypes = [C.c_uint64, C.c_int]
        for n in ["ao_det_atan2f", "ao_det_hypotf"]:
            getattr(L, n).restype = C.c_float
            getattr(L, n).argtypes = [C.c_float, C.c_float]
        for n in ["ao_det_cosf", "ao_det_sinf"]:
            getattr(L, n).restype = C.c_float
            getattr(L, n).argtypes = [C.c_float]
        L.ao_rotate90.restype = C.c_uint64
        D = C.POINTER(C.c_double)
        L.ao_estimate_tag_pose.argtypes = [D, D, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                                           D, D, D]
        L.ao_rotate90.argtypes = [C.c_uint64]
        L.ao_unrank.argtypes = [C.c_int] + [C.POINTER(C.c_int)] * 4
        L.ao_set_fp_perturb.argtypes = [C.c_int]
        L.ao_gp_preprocess.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]
        _LIB = L
    return _LIB


def build():
    import subprocess
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)


FAMILIES = ("tag36h11", "tag25h9", "tag16h5")


def default_params(width, height, family="tag36h11"):
    p = Params()
    lib().ao_default_params(C.byref(p), width, height)
    p.family = family.encode()
    return p


class Oracle:
    """One oracle detector instance (mirrors GpuDetector's lifetime)."""

    def __init__(self, width, height, params=None, family="tag36h11"):
        self.W, self.H = width, height
        self.params = params if params is not None else default_params(width, height, family)
        self.h = lib().ao_create(C.byref(self.params))
        if not self.h:
            raise ValueError("oracle: unsupported frame size %dx%d or family" % (width, height))

    def __del__(self):
        if getattr(self, "h", None):
            lib().ao_destroy(self.h)
            self.h = None

    def detect(self, frame: np.ndarray, pixfmt: int = 0):
        frame = np.ascontiguousarray(frame, dtype=np.uint8)
        return lib().ao_detect(self.h, frame.ctypes.data, pixfmt)

    # ---- stage taps -------------------------------------------------------
    def _arr(self, fn, n, dtype):
        if n == 0:
            return np.zeros(0, dtype)
        return np.ctypeslib.as_array(getattr(lib(), fn)(self.h), shape=(n,)).astype(dtype, copy=True)

    def gray(self):
        return self._arr("ao_gray", self.W * self.H, np.uint8).reshape(self.H, self.W)

    def decimated(self):
        return self._arr("ao_decimated", self.W * self.H // 4, np.uint8).reshape(self.H // 2, self.W // 2)

    def thresholded(self):
        return self._arr("ao_thresholded", self.W * self.H // 4, np.uint8).reshape(self.H // 2, self.W // 2)

    def labels(self):
        return self._arr("ao_labels", self.W * self.H // 4, np.uint32).reshape(self.H // 2, self.W // 2)

    def sizes(self):
        return self._arr("ao_sizes", self.W * self.H // 4, np.uint32)

    def sorted_points(self):
        return self._arr("ao_sorted_points", lib().ao_num_points(self.h), np.uint64)

    def num_pairs(self):
        return lib().ao_num_pairs(self.h)

    def sorted_index_points(self):
        return self._arr("ao_sorted_index_points", lib().ao_num_selected_points(self.h), np.uint64)

    def filtered_errs(self):
        return self._arr("ao_filtered_errs", lib().ao_num_selected_points(self.h), np.float64)

    def errs(self):
        return self._arr("ao_errs", lib().ao_num_selected_points(self.h), np.float64)

    def num_peaks(self):
        return lib().ao_num_peaks(self.h)

    def fitquads(self):
        n = lib().ao_num_fitquads(self.h)
        ptr = lib().ao_fitquads(self.h)
        return [ptr[i] for i in range(n)]

    def quads(self):
        n = lib().ao_num_quads(self.h)
        ptr = lib().ao_quads(self.h)
        return [(np.array([[ptr[i].corners[k][j] for j in range(2)] for k in range(4)], np.float32),
                 int(ptr[i].blob_index)) for i in range(n)]

    def detections(self):
        n = lib().ao_num_detections(self.h)
        ptr = lib().ao_detections(self.h)
        out = []
        for i in range(n):
            d = ptr[i]
            out.append(dict(id=d.id, hamming=d.hamming, decision_margin=d.decision_margin,
                            H=np.array(list(d.H)).reshape(3, 3), c=np.array(list(d.c)),
                            p=np.array([[d.p[k][0], d.p[k][1]] for k in range(4)]),
                            blob_index=d.blob_index))
        return out

    def status(self):
        return lib().ao_status(self.h)


def estimate_tag_pose(H, corners, fx, fy, cx, cy, tagsize=0.1651):
    """estimate_tag_pose restatement (ao_pose.c): returns (R 3x3, t 3, err, (err1, err2), second_won)."""
    D = C.POINTER(C.c_double)
    H = np.ascontiguousarray(H, np.float64).reshape(9)
    P = np.ascontiguousarray(corners, np.float64).reshape(8)
    R = np.zeros(9)
    t = np.zeros(3)
    e = np.zeros(2)
    sec = lib().ao_estimate_tag_pose(H.ctypes.data_as(D), P.ctypes.data_as(D), fx, fy, cx, cy, tagsize,
                                     R.ctypes.data_as(D), t.ctypes.data_as(D), e.ctypes.data_as(D))
    err = e[0] if e[0] <= e[1] else e[1]
    return R.reshape(3, 3), t, err, (e[0], e[1]), bool(sec)


def set_fp_perturb(mask: int):
    """Sensitivity hook: bit k (0 atan2f, 1 hypotf, 2 cosf, 3 sinf) moves every result of
    that function 1 ulp (bit 8: towards -inf).  0 restores the exact restatement."""
    lib().ao_set_fp_perturb(int(mask))


def family_entries(family="tag36h11"):
    L = lib()
    f = family.encode()
    n = L.ao_family_ncodes(f)
    if n < 0:
        raise ValueError("oracle: unknown family %r" % family)
    return [(int(L.ao_family_id(f, i)), int(L.ao_family_code(f, i))) for i in range(n)]


def family_layout(family="tag36h11"):
    """(bit_x, bit_y) lists of the family's 3.x layout."""
    L = lib()
    f = family.encode()
    xs, ys = [], []
    for i in range(L.ao_family_nbits(f)):
        x, y = C.c_int(), C.c_int()
        L.ao_family_bit(f, i, C.byref(x), C.byref(y))
        xs.append(x.value)
        ys.append(y.value)
    return xs, ys


def gp_preprocess(bgr: np.ndarray, out_width=640, out_height=640, channels=3):
    """preprocess_image (game_piece_detection_node.cu:347-379) restated in ao_gp.c:
    (channels, out_height, out_width) float32."""
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    h, w, c = bgr.shape
    assert c == 3
    out = np.empty((channels, out_height, out_width), np.float32)
    rc = lib().ao_gp_preprocess(bgr.ctypes.data, w, h, out.ctypes.data, out_width, out_height, channels)
    if rc != 0:
        raise ValueError("ao_gp_preprocess: invalid arguments")
    return out
