"""CPU checks of the C-ABI library: it loads, exports every symbol
include/at_api.h declares, carries a gfx950 code object, and its host-only
entry points behave (no compute without a GPU)."""
import ctypes as C
import math
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "at_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(at_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = _declared()
    for n in ["at_create", "at_detect", "at_detect_batch", "at_detect_device", "at_debug_copy", "at_destroy",
              "at_strerror"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from ros_vision_amd import detector
    L = detector.load_library()
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert missing == []
    assert sorted(detector.EXPORTS) == _declared()


def test_library_contains_gfx950_code_object():
    data = open(os.path.join(ROOT, "ros_vision_amd", "libat_hip.so"), "rb").read()
    assert b"gfx950" in data


def test_config_defaults_match_reference():
    """apriltag_detector_create defaults + the node's overrides (apriltags_cuda_detector.cu:139-147)."""
    from ros_vision_amd import detector
    L = detector.load_library()
    cfg = detector.AtConfig()
    assert L.at_config_default(C.byref(cfg), 1280, 720) == 0
    assert cfg.family == b"tag36h11" and cfg.quad_decimate == 2.0 and cfg.refine_edges == 1
    assert cfg.decode_sharpening == 0.25 and cfg.min_white_black_diff == 5 and cfg.min_cluster_pixels == 5
    assert cfg.max_nmaxima == 10 and abs(cfg.max_line_fit_mse - 10.0) < 1e-6
    assert abs(cfg.cos_critical_rad - math.cos(math.radians(10))) < 1e-15


def test_invalid_geometry_rejected_before_any_gpu_call():
    from ros_vision_amd import detector
    L = detector.load_library()
    cam = detector.AtCamera()
    for w, h in [(1284, 720), (1280, 724), (2048, 2048), (8, 8)]:
        cfg = detector.AtConfig()
        L.at_config_default(C.byref(cfg), w, h)
        hnd = C.c_void_p()
        assert L.at_create(C.byref(cfg), C.byref(cam), C.byref(hnd)) == -1  # AT_E_INVALID
    cfg = detector.AtConfig()
    L.at_config_default(C.byref(cfg), 1280, 720)
    cfg.family = b"tagStandard41h12"  # named by setup_tag_family, no codebook offline
    assert L.at_create(C.byref(cfg), C.byref(cam), C.byref(C.c_void_p())) == -4  # AT_E_FAMILY
    assert L.at_strerror(-3) == b"frame exceeded a fixed capacity"


def test_family_matches_oracle(oracle_mod):
    from ros_vision_amd import detector
    assert detector.family_entries() == oracle_mod.family_entries()


def test_stage_names():
    from ros_vision_amd import detector
    L = detector.load_library()
    names = [L.at_stage_name(i).decode() for i in range(32)]
    names = names[:names.index("")]
    assert names[0] == "k_pre" and names[-1] == "k_pose" and L.at_stage_name(99) == b""
    assert {"k_extents", "k_blob_small", "k_blob", "k_decode"} <= set(names)


def test_product_library_ignores_the_environment():
    """The experiment knobs (AT_DIAG_PIPE_STOP, AT_DIAG_BLOB_STOP, AT_NO_GRAPH, grid and
    tile overrides, ...) are compiled in only with -DAT_EXPERIMENTS (`make exp`): the
    product library does not even import getenv, and names none of them."""
    import subprocess
    lib = os.path.join(ROOT, "ros_vision_amd", "libat_hip.so")
    nm = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True, check=True).stdout
    assert not re.search(r"\bgetenv\b|\bsecure_getenv\b", nm)
    data = open(lib, "rb").read()
    for knob in (b"AT_DIAG_PIPE_STOP", b"AT_DIAG_BLOB_STOP", b"AT_NO_GRAPH", b"AT_NO_FORK", b"AT_CCL_TILE",
                 b"AT_PHASE_PROBE", b"AT_BLOB_WG", b"AT_NLARGE", b"AT_BND_REGION", b"AT_WIDE_BLOB"):
        assert knob not in data, knob
