"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Integer / byte stages must be bit-identical; floats (homography, centre,
corners, decision margin) within 1e-4 and with identical integer pixel parts.
"""
import numpy as np
import pytest
from PIL import Image

from parity_util import compare_detections, compare_frame

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import ros_vision_amd as rva
    rva.GpuDetector.DEBUG_TAPS = True  # the IndexPoint tap (copy_blob_points) for every detector here
    yield rva
    rva.GpuDetector.DEBUG_TAPS = False


def _real(golden_dir, name):
    return np.asarray(Image.open(golden_dir + "/" + name + "_y.png"))


def test_reference_fixture_detects_554(gpu, oracle_mod, golden_dir):
    """gpu_detector_test.cu:84-92 + :122-157 -- one tag, id 554."""
    y = _real(golden_dir, "colorimage")
    H, W = y.shape
    det = gpu.GpuDetector(W, H)
    dets = det.detect(y, gpu.AT_FMT_GRAY8)
    assert [d.id for d in dets] == [554]
    orc = oracle_mod.Oracle(W, H)
    orc.detect(y, 2)
    assert compare_frame(det, orc) == []
    assert compare_detections(dets, orc.detections()) == []


def test_reference_fixture_grayimage_585(gpu, oracle_mod, golden_dir):
    """Reference fixture test/data/grayimage.jpg -- one tag, id 585."""
    y = _real(golden_dir, "grayimage")
    H, W = y.shape
    det = gpu.GpuDetector(W, H)
    dets = det.detect(y, gpu.AT_FMT_GRAY8)
    assert [d.id for d in dets] == [585]
    orc = oracle_mod.Oracle(W, H)
    orc.detect(y, 2)
    assert compare_frame(det, orc) == []
    assert compare_detections(dets, orc.detections()) == []


def test_reference_fixture_no_tags(gpu, oracle_mod, golden_dir):
    """gpu_detector_test.cu:94-102 -- zero detections."""
    y = _real(golden_dir, "colorimage_notags")
    H, W = y.shape
    det = gpu.GpuDetector(W, H)
    assert det.detect(y, gpu.AT_FMT_GRAY8) == []
    orc = oracle_mod.Oracle(W, H)
    orc.detect(y, 2)
    assert compare_frame(det, orc) == []


@pytest.mark.parametrize("frame", [0, 1, 2, 3])
def test_synthetic_720p_stage_parity(gpu, oracle_mod, frame):
    from ros_vision_amd import synth
    yuyv, gray, truth = synth.stream_frame(1280, 720, frame)
    det = gpu.GpuDetector(1280, 720)
    dets = det.detect(yuyv)
    orc = oracle_mod.Oracle(1280, 720)
    orc.detect(yuyv, 0)
    assert compare_frame(det, orc) == []
    assert compare_detections(dets, orc.detections()) == []
    assert sorted(d.id for d in dets) == sorted(t[0] for t in truth)


def test_batch_matches_single(gpu, oracle_mod):
    """Config C3: 4 cameras in one batched launch sequence == 4 single calls."""
    from ros_vision_amd import synth
    frames = [synth.stream_frame(1280, 720, 7, camera=c)[0] for c in range(4)]
    det = gpu.GpuDetector(1280, 720, max_batch=4)
    batch = det.detect_batch(frames)
    for c, f in enumerate(frames):
        orc = oracle_mod.Oracle(1280, 720)
        orc.detect(f, 0)
        assert compare_frame(det, orc, frame_idx=c) == []
        assert compare_detections(batch[c], orc.detections()) == []


def test_throughput_mode_matches_oracle(gpu, oracle_mod):
    """max_batch >= 8 selects the throughput-mode kernels (64-wide CCL tiles,
    k_ccl_merge + k_boundary<true>, k_extents for every candidate, k_blob_small
    without fused extents, 256-thread large-blob teams): per-frame stages and
    detections identical to the oracle, as in latency mode."""
    from ros_vision_amd import synth
    frames = [synth.stream_frame(1280, 720, f)[0] for f in (3, 17, 31, 45, 58, 5, 9, 12)]
    det = gpu.GpuDetector(1280, 720, max_batch=8)
    batch = det.detect_batch(frames)
    for c, f in enumerate(frames):
        orc = oracle_mod.Oracle(1280, 720)
        orc.detect(f, 0)
        assert compare_frame(det, orc, frame_idx=c) == []
        assert compare_detections(batch[c], orc.detections()) == []


def test_1080p_parity(gpu, oracle_mod):
    """Config C4 geometry (1920x1080, 24 tags)."""
    from ros_vision_amd import synth
    gray, truth = synth.render_board(1920, 1080, seed=4242, ntags=24)
    yuyv = synth.to_yuyv(gray)
    det = gpu.GpuDetector(1920, 1080)
    dets = det.detect(yuyv)
    orc = oracle_mod.Oracle(1920, 1080)
    orc.detect(yuyv, 0)
    assert compare_frame(det, orc) == []
    assert compare_detections(dets, orc.detections()) == []


@pytest.mark.parametrize("W,H", [(800, 600), (1000, 600), (648, 488), (1352, 760), (816, 616)])
@pytest.mark.parametrize("batch", [1, 8])
def test_partial_tile_geometries(gpu, oracle_mod, W, H, batch):
    """Decimated planes that are not a multiple of any tile (800x600 is the deployed
    camera of system_config.json:21-25: 400x300 against 32/64-wide CCL tiles, 32-row
    CCL tiles and 64x16 boundary tiles); tags and blobs flush against the right and
    bottom borders.  The reference's only geometry preconditions are W, H multiples of
    8 (threshold.cu:156-157) and even decimated sizes (labeling_allegretti_2019_BKE.cu:
    469-475).  Latency mode (batch 1: 32-wide CCL tiles, k_pre fused) and throughput
    mode (batch 8: 64-wide tiles, k_ccl_merge, k_extents): every stage bit-exact."""
    from ros_vision_amd import synth
    codes = dict(oracle_mod.family_entries())
    frames = [synth.render_edge_board(W, H, seed=W + H + 7 * k, codes=codes) for k in range(min(batch, 3))]
    fmt = gpu.AT_FMT_GRAY8 if W % 16 == 0 else gpu.AT_FMT_YUYV
    inputs = [g if fmt == gpu.AT_FMT_GRAY8 else synth.to_yuyv(g) for g, _ in frames]
    det = gpu.GpuDetector(W, H, max_batch=batch)
    res = det.detect_batch(inputs, fmt)
    ndet = 0
    for c, f in enumerate(inputs):
        orc = oracle_mod.Oracle(W, H)
        orc.detect(f, fmt)
        assert compare_frame(det, orc, frame_idx=c) == [], (W, H, batch, c)
        assert compare_detections(res[c], orc.detections()) == [], (W, H, batch, c)
        ndet += len(res[c])
    assert ndet >= 6 * len(inputs)


def test_bgr_and_gray_inputs(gpu, oracle_mod):
    from ros_vision_amd import synth
    gray, _ = synth.render_board(640, 480, seed=766, ntags=4)
    rng = np.random.default_rng(1)
    bgr = rng.integers(0, 256, size=(480, 640, 3), dtype=np.uint8)
    bgr[..., 1] = gray  # mostly-green-driven luma keeps the tags visible
    for fmt, frame in [(gpu.AT_FMT_GRAY8, gray), (gpu.AT_FMT_BGR8, bgr)]:
        det = gpu.GpuDetector(640, 480)
        dets = det.detect(frame, fmt)
        orc = oracle_mod.Oracle(640, 480)
        orc.detect(frame, fmt)
        assert compare_frame(det, orc) == []
        assert compare_detections(dets, orc.detections()) == []


def test_empty_and_flat_frames(gpu, oracle_mod):
    for val in (0, 128, 255):
        frame = np.full((720, 1280), val, np.uint8)
        det = gpu.GpuDetector(1280, 720)
        assert det.detect(frame, gpu.AT_FMT_GRAY8) == []
        orc = oracle_mod.Oracle(1280, 720)
        orc.detect(frame, 2)
        assert compare_frame(det, orc) == []


def test_device_resident_frames(gpu, oracle_mod):
    """Frames already in HBM (the bench path) give the same detections."""
    import torch
    from ros_vision_amd import synth
    frames = np.stack([synth.stream_frame(1280, 720, i)[0] for i in range(3)])
    t = torch.from_numpy(frames).cuda()
    det = gpu.GpuDetector(1280, 720, max_batch=3)
    res = det.detect_device(t.data_ptr(), frames[0].nbytes, 3)
    for i in range(3):
        orc = oracle_mod.Oracle(1280, 720)
        orc.detect(frames[i], 0)
        assert compare_detections(res[i], orc.detections()) == []


def _golden():
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return json.load(open(os.path.join(root, "tests", "golden", "vectors.json")))


@pytest.mark.parametrize("name", sorted(_golden()))
def test_gpu_matches_committed_golden(gpu, name):
    """HIP path vs the committed golden vectors: stage digests bit-exact,
    ids/hamming exact, floats within 1e-4."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import make_golden_vectors as mg
    want = _golden()[name]
    W, H, fmt, frame, family = {c[0]: c[1:] for c in mg.cases()}[name]
    det = gpu.GpuDetector(W, H, family=family)
    dets = det.detect(frame, fmt)
    assert mg.digest(det.copy_thresholded()) == want["thr"]
    assert mg.digest(det.copy_union_markers()) == want["labels"]
    assert mg.digest(det.copy_union_markers_size()) == want["sizes"]
    assert mg.digest(np.sort(det.copy_points())) == want["points_sorted"]
    assert det.num_pairs() == want["num_pairs"]
    assert mg.digest(det.copy_blob_points()) == want["index_points"]
    assert [d.id for d in dets] == [d["id"] for d in want["detections"]]
    for a, b in zip(dets, want["detections"]):
        assert a.hamming == b["hamming"]
        assert abs(a.decision_margin - b["decision_margin"]) <= 1e-4
        assert np.allclose(a.p, np.array(b["p"]), atol=1e-4) and np.allclose(a.c, np.array(b["c"]), atol=1e-4)
        assert np.allclose(a.H.ravel(), np.array(b["H"]), atol=1e-4)
        assert np.array_equal(np.floor(a.p), np.floor(np.array(b["p"])))


# ---- row A23: tag pose (k_pose) against the oracle's estimate_tag_pose -------

def _pose_close(a_R, a_t, b_R, b_t, tol):
    return np.abs(np.asarray(a_R) - np.asarray(b_R)).max() <= tol and np.abs(np.asarray(a_t) - np.asarray(b_t)).max() <= tol


@pytest.mark.parametrize("frame,batch", [(0, 1), (1, 1), (2, 8)])
def test_pose_parity_720p(gpu, oracle_mod, frame, batch):
    """GPU pose of every detection vs the oracle pose of the oracle's detection
    with the same id: within 1e-4 (north star float tolerance).  batch 1: the
    latency mode's k_pose (a wave per detection, parallel bracket search for the
    quartic's roots); batch 8: four lanes per detection (safeguarded Newton as
    upstream)."""
    from ros_vision_amd import synth
    cam = gpu.TEST_CAMERA
    yuyv, _, _ = synth.stream_frame(1280, 720, frame)
    det = gpu.GpuDetector(1280, 720, max_batch=batch)
    dets = det.detect(yuyv)
    poses = det.poses()
    assert len(poses) == len(dets) > 0
    orc = oracle_mod.Oracle(1280, 720)
    orc.detect(yuyv, 0)
    odets = {d["id"]: d for d in orc.detections()}
    worst = 0.0
    for d, p in zip(dets, poses):
        assert p.id == d.id
        od = odets[d.id]
        R, t, err, (e1, e2), _ = oracle_mod.estimate_tag_pose(od["H"], od["p"], cam.fx, cam.fy, cam.cx, cam.cy)
        if abs(e1 - e2) <= 1e-9 * max(e1, e2, 1e-30):
            continue  # two minima with equal error: either is the reference's answer
        worst = max(worst, np.abs(p.R - R).max(), np.abs(p.t - t).max())
        assert _pose_close(p.R, p.t, R, t, 1e-4), (d.id, p.R, R, p.t, t)
        assert abs(p.err - err) <= 1e-4 * max(1.0, abs(err))
    # same inputs (the GPU's own H and corners) agree far tighter
    for d, p in zip(dets, poses):
        R, t, _, _, _ = oracle_mod.estimate_tag_pose(d.H, d.p, cam.fx, cam.fy, cam.cx, cam.cy)
        assert _pose_close(p.R, p.t, R, t, 1e-9), d.id
    print("pose worst |diff| vs oracle detections: %.3g" % worst)


def test_wave_pose_matches_quad_pose(gpu):
    """The latency mode's k_pose (a wave per detection, parallel bracket search for
    the quartic's roots) equals the throughput mode's (four lanes per detection,
    upstream's safeguarded Newton) to 1e-9 on every detection of several frames."""
    import torch
    from ros_vision_amd import synth
    frames = np.stack([synth.stream_frame(1280, 720, f)[0] for f in range(3, 11)])
    t = torch.from_numpy(frames).cuda()
    quad = gpu.GpuDetector(1280, 720, max_batch=8)
    quad.detect_device(t.data_ptr(), frames[0].nbytes, 8)
    wave = gpu.GpuDetector(1280, 720, max_batch=1)
    n = 0
    for f in range(8):
        a = wave.detect(frames[f])
        assert [d.id for d in a] == [d.id for d in quad.detections(f)]
        for pa, pb in zip(wave.poses(), quad.poses(f)):
            assert _pose_close(pa.R, pa.t, pb.R, pb.t, 1e-9), (pa.id, pa.t, pb.t)
            assert pa.err == pytest.approx(pb.err, rel=1e-9, abs=1e-15)
            n += 1
    assert n >= 80


def test_pose_disabled_and_camera_to_robot(gpu):
    from ros_vision_amd import synth
    yuyv, _, _ = synth.stream_frame(1280, 720, 0)
    off = gpu.GpuDetector(1280, 720, tag_size=0.0)
    assert len(off.detect(yuyv)) > 0 and off.poses() == []
    on = gpu.GpuDetector(1280, 720)
    on.detect(yuyv)
    tags = gpu.tag_detections(on.poses(), np.eye(3), np.zeros(3))
    d = [t.distance for t in tags]
    assert d == sorted(d) and len(tags) == len(on.poses())
    for t in tags:
        assert np.allclose(t.camera, t.robot) and t.camera[2] > 0


@pytest.mark.parametrize("kind", ["white_noise", "block_noise_8", "block_noise_24", "checker_10",
                                  "vstripes_2", "diag_4", "tags_over_checker"])
def test_noise_frames(gpu, oracle_mod, kind):
    """Pathological inputs: pixel noise, blocky noise (thousands of rectangles -> many
    quads and decodes), and more blob pairs than the 12-bit blob index holds
    (checker_10, tags_over_checker): the reference overflows its 2048-entry extents
    buffer there (apriltag_gpu.cu:129,899-902, undefined); both sides keep the first
    4096 pairs in rank order, report AT_E_CAPACITY and return those pairs' detections."""
    from ros_vision_amd import synth
    rng = np.random.default_rng({"white_noise": 11, "block_noise_8": 12, "block_noise_24": 13, "checker_10": 14,
                                 "vstripes_2": 15, "diag_4": 16, "tags_over_checker": 17}[kind])
    if kind == "tags_over_checker":  # tags in the top rows (small labels: first ranks), ~5,000 dark squares below
        yy, xx = np.mgrid[0:720, 0:1280]
        frame = np.where(((yy % 12) < 10) & ((xx % 12) < 10), 25, 230).astype(np.uint8)
        frame[:200] = synth.render_board(1280, 200, seed=17, ntags=5, side_range=(70, 90))[0]
    elif kind == "white_noise":
        frame = rng.integers(0, 256, size=(720, 1280), dtype=np.uint8)
    elif kind == "checker_10":  # > 4096 blob pairs of >= 25 pixels
        yy, xx = np.mgrid[0:720, 0:1280]
        frame = np.where(((yy // 10) + (xx // 10)) & 1, 230, 25).astype(np.uint8)
    elif kind == "vstripes_2":  # ~2 boundary points per pixel: k_boundary tiles overflow their LDS stage
        yy, xx = np.mgrid[0:720, 0:1280]
        frame = np.where((xx // 2) & 1, 230, 25).astype(np.uint8)
    elif kind == "diag_4":
        yy, xx = np.mgrid[0:720, 0:1280]
        frame = np.where(((xx + yy) // 4) & 1, 230, 25).astype(np.uint8)
    else:
        s = int(kind.rsplit("_", 1)[1])
        small = rng.integers(0, 256, size=(720 // s + 1, 1280 // s + 1), dtype=np.uint8)
        frame = np.ascontiguousarray(np.kron(small, np.ones((s, s), np.uint8))[:720, :1280])
    det = gpu.GpuDetector(1280, 720)
    dets = det.detect(frame, gpu.AT_FMT_GRAY8)
    orc = oracle_mod.Oracle(1280, 720)
    rc = orc.detect(frame, 2)
    from ros_vision_amd.detector import AT_E_CAPACITY
    if kind in ("checker_10", "tags_over_checker"):
        assert orc.status() == AT_E_CAPACITY and orc.num_pairs() == 4096
    assert det.frame_status(0) == orc.status()
    if kind == "tags_over_checker":
        assert [d.id for d in dets] == [434, 435, 436, 437, 438]  # the tags' pairs rank first (smallest labels)
    assert rc >= 0
    assert compare_frame(det, orc) == []
    assert compare_detections(dets, orc.detections()) == []


@pytest.mark.parametrize("dist", [(0.0, 0.0, 0.0, 0.0, 0.0), (0.12, -0.21, 0.004, -0.002, 0.08),
                                  (-0.3, 0.09, 0.0, 0.0, -0.01)])
def test_distortion_variants(gpu, oracle_mod, dist):
    """RefineEdges' UnDistort/ReDistort (apriltag_detect.cu:307-402, incl. the :372
    p2 term) with other intrinsics and distortion coefficients, k3 != 0 included."""
    from ros_vision_amd import synth
    from ros_vision_amd.detector import CameraMatrix, DistCoeffs
    k1, k2, p1, p2, k3 = dist
    cam = CameraMatrix(fx=1010.5, cx=655.25, fy=1003.75, cy=371.5)
    yuyv, gray, truth = synth.stream_frame(1280, 720, 5)
    det = gpu.GpuDetector(1280, 720, camera_matrix=cam,
                          distortion_coefficients=DistCoeffs(k1=k1, k2=k2, p1=p1, p2=p2, k3=k3))
    dets = det.detect(yuyv)
    prm = oracle_mod.default_params(1280, 720)
    prm.fx, prm.fy, prm.cx, prm.cy = cam.fx, cam.fy, cam.cx, cam.cy
    prm.k1, prm.k2, prm.p1, prm.p2, prm.k3 = k1, k2, p1, p2, k3
    orc = oracle_mod.Oracle(1280, 720, prm)
    orc.detect(yuyv, 0)
    assert compare_frame(det, orc) == []
    assert compare_detections(dets, orc.detections()) == []
    assert sorted(d.id for d in dets) == sorted(t[0] for t in truth)


@pytest.mark.parametrize("batch,timed", [(8, "k_blob"), (8, "k_boundary"), (1, "k_blob_small"), (8, "k_pose"),
                                         (1, "k_decode"), (8, "k_thr_ccl"), (192, "k_thr_ccl")])
def test_timed_and_profiled_launches_match_graph(gpu, batch, timed):
    """The bench's launch modes give identical detections: hipGraph replay, the
    split graph around a timed kernel (fence-free events between three graphs; on
    the fork branch at B < 8 a direct launch), and stage profiling (direct
    launches with events between every kernel).  The timer reports every launch."""
    import torch
    from ros_vision_amd import synth
    distinct = np.stack([synth.stream_frame(1280, 720, 20 + i)[0] for i in range(min(batch, 8))])
    frames = np.concatenate([distinct] * (-(-batch // distinct.shape[0])))[:batch]
    t = torch.from_numpy(frames).cuda()
    det = gpu.GpuDetector(1280, 720, max_batch=batch)

    def run(n=2):
        out = None
        for _ in range(n):
            det.enqueue_device(t.data_ptr(), frames[0].nbytes, batch)
            det.collect(counts_only=True)
            out = [[(d.id, tuple(np.round(d.p.ravel(), 9))) for d in det._unpack(batch)[f]] for f in range(batch)]
        return out

    base = run()
    det.set_kernel_timer(timed)
    assert run(3) == base
    ms, launches = det.kernel_time()
    assert launches == 3 and ms > 0
    span, nspan = det.kernel_span()  # device-clock span: every launch of a stamped kernel
    if timed == "k_pose":
        assert nspan == 0
    else:
        assert nspan == 3 and 0 < span <= ms * 1.05 + 0.005, (span, ms)
    det.set_kernel_timer(None)
    det.set_profiling(True)
    assert run() == base
    stages, nb = det.stage_times()
    det.set_profiling(False)
    assert nb >= 2 and all(v > 0 for v in stages.values())
    assert run() == base


def test_mixed_geometries_keep_the_merge_lds_limit(gpu, oracle_mod):
    """k_ccl_merge's dynamic-LDS limit is a process-wide function attribute.
    A 1920x1080 throughput detector (153,600 B of merge LDS per launch), then an 800x600
    one created in the same process (78,400 B): the 1080p detector must still launch
    and detect like the oracle."""
    from ros_vision_amd import synth
    big = gpu.GpuDetector(1920, 1080, max_batch=8)
    small = gpu.GpuDetector(800, 600, max_batch=8)
    f1080 = synth.stream_frame(1920, 1080, 5)[0]
    res = big.detect_batch([f1080])
    orc = oracle_mod.Oracle(1920, 1080)
    orc.detect(f1080, 0)
    assert len(res[0]) > 0 and compare_detections(res[0], orc.detections()) == []
    g8, _ = synth.render_edge_board(800, 600, seed=1400, codes=dict(oracle_mod.family_entries()))
    res = small.detect_batch([g8], gpu.AT_FMT_GRAY8)
    orc = oracle_mod.Oracle(800, 600)
    orc.detect(g8, 2)
    assert compare_detections(res[0], orc.detections()) == []
    res = big.detect_batch([f1080])
    assert compare_detections(res[0], orc_1080(oracle_mod, f1080)) == []


def orc_1080(oracle_mod, frame):
    orc = oracle_mod.Oracle(1920, 1080)
    orc.detect(frame, 0)
    return orc.detections()


def test_environment_cannot_truncate_the_pipeline(oracle_mod):
    """A deployed detector with the former diagnostic knobs set (stage cut-offs, no
    graphs, other grids) still returns the oracle's detections: the product library
    ignores the environment (the reference either detects or aborts,
    cuda_frc971.h:14-17).  Run in a child process so the variables are seen from
    the first HIP call."""
    import json
    import os
    import subprocess
    import sys
    from ros_vision_amd import synth
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, AT_DIAG_PIPE_STOP="3", AT_DIAG_BLOB_STOP="2", AT_NO_GRAPH="1", AT_CCL_TILE="32",
               AT_BLOB_WG="16", AT_NLARGE="0", AT_BND_REGION="1")
    env.pop("AT_HIP_LIB", None)
    code = ("import json, sys; sys.path.insert(0, %r)\n"
            "import ros_vision_amd as rva\nfrom ros_vision_amd import synth\n"
            "out = []\n"
            "for b in (1, 8):\n"
            "    det = rva.GpuDetector(1280, 720, max_batch=b)\n"
            "    out.append([d.id for d in det.detect(synth.stream_frame(1280, 720, 4)[0])])\n"
            "print(json.dumps(out))\n" % root)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    orc = oracle_mod.Oracle(1280, 720)
    orc.detect(synth.stream_frame(1280, 720, 4)[0], 0)
    want = [d["id"] for d in orc.detections()]
    assert len(want) == 15 and got == [want, want]


@pytest.mark.parametrize("batch", [4, 8])
def test_dense_frames_keep_every_candidate(gpu, oracle_mod, batch):
    """Each frame owns its candidate slots (kMaxDets per frame in HBM, the first 128
    mirrored to the host; more copied at collect): a batch of frames with more than
    128 detections each returns every frame's detections, as the reference keeps every
    detection (apriltag_detect.cu:618-663), whatever the other frames hold."""
    from ros_vision_amd import synth
    codes = dict(oracle_mod.family_entries())
    frames = []
    for k in range(3):
        g, _ = synth.render_board(1920, 1080, seed=9160 + k, ntags=160, side_range=(50, 64),
                                  ids=[(400 + 3 * k + j) % 587 for j in range(160)], codes=codes)
        frames.append(synth.to_yuyv(g))
    frames.append(synth.stream_frame(1920, 1080, 3)[0])
    det = gpu.GpuDetector(1920, 1080, max_batch=batch)
    res = det.detect_batch(frames)
    for c, f in enumerate(frames):
        assert det.frame_status(c) == 0
        orc = oracle_mod.Oracle(1920, 1080)
        orc.detect(f, 0)
        assert compare_detections(res[c], orc.detections()) == [], c
        if c < 3:
            assert len(res[c]) > 128
        assert len(det.poses(c)) == len(res[c])


def test_ccl_merge_and_fallback_in_one_batch(gpu, oracle_mod):
    """Throughput mode merges each frame's listed local roots in one workgroup's LDS
    (k_ccl_merge); a frame with more (white noise: thousands of tile-border specks)
    is merged by the same workgroup in global memory (k_ccl_border's unions, k_ccl_roots'
    pass and the kept bits).
    Both kinds of frame in one batch: every stage bit-exact against the oracle
    (labels = the component's minimum node id, labeling_allegretti_2019_BKE.cu:340-462)."""
    from ros_vision_amd import synth
    rng = np.random.default_rng(99)
    yy, xx = np.mgrid[0:720, 0:1280]
    frames = [synth.stream_frame(1280, 720, 9)[1],
              rng.integers(0, 256, size=(720, 1280), dtype=np.uint8),
              synth.stream_frame(1280, 720, 10)[1],
              # a one-decimated-pixel checker: every border block its own background specks
              np.where(((xx // 2) + (yy // 2)) & 1, 230, 25).astype(np.uint8)]
    det = gpu.GpuDetector(1280, 720, max_batch=8)
    res = det.detect_batch(frames, gpu.AT_FMT_GRAY8)
    st = det.batch_stats()
    assert st["ccl_fallback_frames"] >= 1 and st["ccl_fallback_frames"] < len(frames), st
    for c, f in enumerate(frames):
        orc = oracle_mod.Oracle(1280, 720)
        orc.detect(f, 2)
        assert compare_frame(det, orc, frame_idx=c) == [], c
        assert compare_detections(res[c], orc.detections()) == [], c


def test_ccl_merge_lds_layouts_1080p(gpu, oracle_mod):
    """k_ccl_merge's two LDS layouts at 1080p (153,600 B): a 1080p stream frame lists
    ~11 k local roots, whose parent keys and pixel counts fit at 12 B per root; a frame
    with more than 12,799 (and at most 15,360) listed roots keeps the counts in the size
    plane at L2 (10 B per root).  Frames are a stream frame whose top rows are replaced
    by a one-decimated-pixel checker band of growing height (every background pixel of
    a tile border its own component); the band heights that land in the L2 range are
    found by running each frame alone.  No frame may fall back to the global merge,
    and every stage (labels, sizes, kept bits) stays bit-exact against the oracle."""
    from ros_vision_amd import synth
    base = synth.stream_frame(1920, 1080, 3)[1]
    yy, xx = np.mgrid[0:1080, 0:1920]
    chk = np.where(((xx // 2) + (yy // 2)) & 1, 230, 25).astype(np.uint8)
    frames, roots = [], []
    det = gpu.GpuDetector(1920, 1080, max_batch=8)
    for rows in (0, 64, 128, 192, 256, 320, 384, 448):
        f = base.copy()
        f[:rows] = chk[:rows]
        det.detect_batch([f], gpu.AT_FMT_GRAY8)
        st = det.batch_stats()
        frames.append(f)
        roots.append(st["ccl_listed_roots_max"])
        if st["ccl_listed_roots_max"] > 15360:
            break
    assert roots[0] * 12 + 4 <= 153600, roots  # the stream frame: counts in LDS
    picked = [0] + [i for i, r in enumerate(roots) if 12 * r + 4 > 153600 and r <= 15360][:2]
    assert len(picked) >= 2, roots  # (some band lands in the counts-at-L2 range)
    res = det.detect_batch([frames[i] for i in picked], gpu.AT_FMT_GRAY8)
    assert det.batch_stats()["ccl_fallback_frames"] == 0
    for c, i in enumerate(picked):
        orc = oracle_mod.Oracle(1920, 1080)
        orc.detect(frames[i], 2)
        assert compare_frame(det, orc, frame_idx=c) == [], (c, roots[i])
        assert compare_detections(res[c], orc.detections()) == [], (c, roots[i])


def test_ccl_adversarial_unions(gpu, oracle_mod):
    """k_thr_ccl runs no barrier between reading the union targets and
    the unions, nor between the finds and the root writes (unions and compressions only
    lower a parent within its component).  Frames built to race them (tests/ccl_patterns.py:
    serpentine backgrounds between interleaved combs, spirals, staircases -- components
    through every wave's block rows of a tile and across tile borders), at B = 1 (32-wide
    tiles, k_ccl_border / k_ccl_roots) and B = 192 (64-wide tiles, k_ccl_merge): labels
    (the component's minimum node id) and sizes bit-exact against the oracle for every
    frame, every later stage for the first frames of each batch."""
    import torch

    import ccl_patterns
    W, H, B = 1280, 720, 192
    variants = [ccl_patterns.frame(W, H, seed) for seed in range(8)]
    orcs = []
    for f in variants:
        o = oracle_mod.Oracle(W, H)
        o.detect(f, 2)
        orcs.append(o)
    want = [(o.labels().copy(), o.sizes().copy()) for o in orcs]
    det1 = gpu.GpuDetector(W, H)
    for v in range(4):
        det1.detect(variants[v], gpu.AT_FMT_GRAY8)
        assert compare_frame(det1, orcs[v]) == [], v
    batch = np.stack([variants[j % 8] for j in range(B)])
    t = torch.from_numpy(batch).cuda()
    det = gpu.GpuDetector(W, H, max_batch=B)
    det.detect_device(t.data_ptr(), batch[0].nbytes, B, gpu.AT_FMT_GRAY8)
    for j in range(B):
        assert np.array_equal(det.copy_union_markers(j), want[j % 8][0]), j
        assert np.array_equal(det.copy_union_markers_size(j), want[j % 8][1]), j
    for j in range(8):
        assert compare_frame(det, orcs[j], frame_idx=j) == [], j


@pytest.mark.parametrize("batch", [1, 8])
def test_debug_records_need_the_taps(batch):
    """The fitted-quad records (AT_STAGE_QUADS) are debug output the blob kernels and
    k_quad_fin write only while the taps are on: without them the copy is refused
    (AT_E_INVALID), never served stale; with them every detection has its accepted quad."""
    import ros_vision_amd as rva
    from ros_vision_amd import synth
    frame = synth.stream_frame(1280, 720, 2)[0]
    det = rva.GpuDetector(1280, 720, max_batch=batch, debug_taps=False)
    det.detect_batch([frame])
    with pytest.raises(RuntimeError):
        det.copy_quads(0)
    det.close()
    det = rva.GpuDetector(1280, 720, max_batch=batch, debug_taps=True)
    res = det.detect_batch([frame])
    quads = det.copy_quads(0)
    assert len(res[0]) > 0 and sum(q["accepted"] for q in quads) >= len(res[0])
    det.close()
