"""The compiled side of the boundary and the C++ node adapter.

CPU: node/abi_check (plain C11 consumer of include/at_api.h, struct layouts pinned by
_Static_assert) against the ctypes mirror; the ApriltagListProto bytes of the C++ core
parsed by google.protobuf against the reference schema (proto/apriltag.proto:6-17);
calibration / extrinsics loaders against the Python node; the outline drawing.
GPU: abi_check and at_mock_node detect through the C ABI and agree with the Python
binding, the Python node and the oracle.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = os.path.join(ROOT, "node")


@pytest.fixture(scope="module")
def built():
    import fcntl
    # one make at a time (pytest-xdist workers share the tree)
    with open(os.path.join(NODE, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", NODE, "-s"], check=True)
    return NODE


@pytest.fixture(scope="module")
def nodelib(built):
    from ros_vision_amd import detector
    detector.load_library()  # libat_hip first (torch owns the HIP runtime when present)
    L = C.CDLL(os.path.join(built, "libat_node.so"))
    L.at_node_encode_apriltag_list.restype = C.c_longlong
    L.at_node_encode_apriltag_list.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_void_p, C.c_size_t]
    L.at_node_load_camera_calibration.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(detector.AtCamera)]
    L.at_node_load_extrinsics.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                          C.c_char_p, C.c_size_t]
    L.at_node_draw_detection_outlines.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int]
    L.at_node_load_camera_config.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                             C.POINTER(C.c_int), C.c_char_p, C.c_size_t]
    L.at_node_package_share_directory.restype = C.c_longlong
    L.at_node_package_share_directory.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
    L.at_node_resolve_config.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.POINTER(detector.AtCamera),
                                         C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int)]
    return L


def make_share_tree(root, serial, width, height, location="center_front", extra_cameras=None):
    """An install prefix holding vision_config_data the way ament_index finds it:
    <prefix>/share/ament_index/resource_index/packages/vision_config_data (marker) and
    <prefix>/share/vision_config_data/data/{system_config.json, calibration/...}
    (the layout of src/vision_config_data, CMakeLists.txt installs data/)."""
    prefix = root / "install"
    (prefix / "share/ament_index/resource_index/packages").mkdir(parents=True)
    (prefix / "share/ament_index/resource_index/packages/vision_config_data").write_text("")
    data = prefix / "share/vision_config_data/data"
    (data / "calibration").mkdir(parents=True)
    cams = {serial: {"location": location, "format": "MJPG", "height": height, "width": width,
                     "frame_rate": 30, "api_preference": "V4L2"}}
    cams.update(extra_cameras or {})
    (data / "system_config.json").write_text(json.dumps({
        "camera_mounted_positions": cams,
        "extrinsics": {location: {"rotation": [[0, 0, 1], [-1, 0, 0], [0, -1, 0]], "offset": [0.25, -0.1, 0.4]}},
        "network_tables_config": {"table_address": "10.7.66.2", "table_name": "/SmartDashboard"}}))
    (data / "calibration" / ("calibrationmatrix_%s.json" % serial)).write_text(json.dumps(
        {"matrix": [[905.495617, 0, 609.916016], [0, 907.909470, 352.682645], [0, 0, 1]],
         "disto": [[0.059238, -0.075154, -0.003801, 0.001113, 0.0]]}))
    return prefix


def proto_classes():
    """ApriltagProto / ApriltagListProto built from the reference schema (proto2)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="apriltag.proto", package="com.team766.vision", syntax="proto2")
    m = fdp.message_type.add(name="ApriltagProto")
    for name, num, typ in [("collect_time", 1, F.TYPE_DOUBLE), ("tag_id", 2, F.TYPE_INT32), ("x", 3, F.TYPE_DOUBLE),
                           ("y", 4, F.TYPE_DOUBLE), ("z", 5, F.TYPE_DOUBLE)]:
        m.field.add(name=name, number=num, type=typ, label=F.LABEL_REQUIRED)
    ml = fdp.message_type.add(name="ApriltagListProto")
    ml.field.add(name="tags", number=1, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED,
                 type_name=".com.team766.vision.ApriltagProto")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = getattr(message_factory, "GetMessageClass", None)
    if get is None:
        get = message_factory.MessageFactory(pool).GetPrototype
    return get(pool.FindMessageTypeByName("com.team766.vision.ApriltagListProto"))


def test_abi_layout_matches_ctypes_mirror(built):
    from ros_vision_amd import detector as D
    lay = json.loads(subprocess.run([os.path.join(built, "abi_check"), "layout"], check=True, capture_output=True,
                                    text=True).stdout)
    assert lay["abi_version"] == lay["library_abi_version"] == D.load_library().at_abi_version()
    for cname, ct in [("at_config", D.AtConfig), ("at_camera", D.AtCamera), ("at_detection", D.AtDetection),
                      ("at_pose", D.AtPose), ("at_tag_detection", D.AtTagDetection),
                      ("at_quad_record", D.AtQuadRecord)]:
        assert lay["sizeof." + cname] == C.sizeof(ct), cname
        for fname, _ in ct._fields_:
            assert lay["%s.%s" % (cname, fname)] == getattr(ct, fname).offset, (cname, fname)


def test_apriltag_list_proto_bytes(nodelib):
    from ros_vision_amd import detector as D
    tags = (D.AtTagDetection * 3)()
    vals = [(7, (0.5, -1.25, 3.0)), (586, (1e-9, 2.5, -0.0)), (-3, (12.0, 0.1, 1.0))]
    for i, (tid, r) in enumerate(vals):
        tags[i].id = tid
        tags[i].robot[:] = list(r)
    buf = (C.c_uint8 * 1024)()
    n = nodelib.at_node_encode_apriltag_list(tags, 3, 1234.5678, buf, 1024)
    raw = bytes(buf[:n])
    Msg = proto_classes()
    msg = Msg()
    msg.ParseFromString(raw)
    assert [t.tag_id for t in msg.tags] == [7, 586, -3]
    for t, (tid, r) in zip(msg.tags, vals):
        assert t.collect_time == 1234.5678 and (t.x, t.y, t.z) == r
    assert msg.SerializeToString() == raw  # same bytes as the protobuf runtime writes
    assert nodelib.at_node_encode_apriltag_list(tags, 0, 0.0, buf, 1024) == 0  # no tags: empty message


def test_calibration_and_extrinsics_match_python_node(nodelib, tmp_path):
    from ros_vision_amd import detector as D
    from ros_vision_amd import node as N
    (tmp_path / "calibrationmatrix_CAM1.json").write_text(json.dumps(
        {"matrix": [[905.5, 0, 609.9], [0, 907.9, 352.7], [0, 0, 1]], "disto": [[0.05, -0.07, -0.003, 0.001, 0.02]]}))
    cam = D.AtCamera()
    assert nodelib.at_node_load_camera_calibration(str(tmp_path).encode(), b"CAM1", C.byref(cam)) == 0
    pc, pd = N.load_camera_calibration(str(tmp_path), "CAM1")
    assert (cam.fx, cam.fy, cam.cx, cam.cy) == (pc.fx, pc.fy, pc.cx, pc.cy)
    assert (cam.k1, cam.k2, cam.p1, cam.p2, cam.k3) == (pd.k1, pd.k2, pd.p1, pd.p2, pd.k3)
    assert nodelib.at_node_load_camera_calibration(str(tmp_path).encode(), b"NOPE", C.byref(cam)) != 0
    rot = [[0, -1, 0], [1, 0, 0], [0, 0, 1]]
    cfg = {"camera_mounted_positions": {"CAM1": "front", "CAM2": {"location": "back"}, "CAM3": "side"},
           "extrinsics": {"front": {"rotation": rot, "offset": [0.1, 0.2, 0.3]},
                          "back": {"rotation": sum(rot, []), "offset": [-1, 0, 2]}}}
    path = tmp_path / "system_config.json"
    path.write_text(json.dumps(cfg))
    for serial, ok in [("CAM1", 0), ("CAM2", 0), ("CAM3", -1), ("CAM9", -1)]:
        R, t = (C.c_double * 9)(), (C.c_double * 3)()
        loc = C.create_string_buffer(64)
        assert nodelib.at_node_load_extrinsics(str(path).encode(), serial.encode(), R, t, loc, 64) == ok
        pR, pt, ploc = N.load_extrinsics(str(path), serial)
        assert np.array_equal(np.array(list(R)).reshape(3, 3), pR) and np.array_equal(np.array(list(t)), pt)
        assert (loc.value.decode() or None) == ploc


def test_outlines_and_id_text(nodelib):
    from ros_vision_amd import detector as D
    W, H = 320, 240
    img = np.zeros((H, W, 3), np.uint8)
    det = (D.AtDetection * 1)()
    det[0].id = 42
    pts = [(100.7, 60.2), (220.3, 60.9), (220.9, 180.4), (100.1, 180.8)]
    for k, (x, y) in enumerate(pts):
        det[0].p[k][0], det[0].p[k][1] = x, y
    det[0].c[0], det[0].c[1] = 160.0, 120.0
    nodelib.at_node_draw_detection_outlines(img.ctypes.data, W, H, det, 1)
    assert tuple(img[60, 160]) == (0, 255, 0)      # p0-p1 green (BGR)
    assert tuple(img[120, 100]) == (0, 0, 255)     # p0-p3 red
    assert tuple(img[120, 220]) == (255, 0, 0)     # p1-p2 blue
    assert tuple(img[180, 160]) == (255, 0, 0)     # p2-p3 blue
    text = np.all(img[100:140, 130:190] == (255, 153, 0), axis=-1)
    assert text.sum() > 40                         # the id, centred on c


# ---- GPU: the compiled consumers detect through the C ABI --------------------

@pytest.mark.gpu
def test_abi_check_detects_reference_fixture(built, golden_dir, tmp_path):
    from PIL import Image
    y = np.asarray(Image.open(os.path.join(golden_dir, "colorimage_y.png")))
    f = tmp_path / "frame.raw"
    y.tofile(f)
    out = subprocess.run([os.path.join(built, "abi_check"), "detect", str(y.shape[1]), str(y.shape[0]), "2", str(f)],
                         check=True, capture_output=True, text=True, timeout=120).stdout
    dets = json.loads(out)
    assert [d["id"] for d in dets] == [554]


@pytest.mark.gpu
def test_mock_node_matches_python_node_and_oracle(built, oracle_mod, tmp_path):
    import ros_vision_amd as rva
    from ros_vision_amd import node as N
    from ros_vision_amd import synth
    W, H = 1280, 720
    frames = [synth.stream_frame(W, H, f)[1] for f in (3, 33)]
    bgr = np.stack([np.repeat(g[:, :, None], 3, axis=2) for g in frames])  # gray scene as bgr8
    path = tmp_path / "frames.raw"
    bgr.tofile(path)
    rot = [[0, 0, 1], [-1, 0, 0], [0, -1, 0]]
    cfg = tmp_path / "system_config.json"
    cfg.write_text(json.dumps({"camera_mounted_positions": {"S1": "front"},
                               "extrinsics": {"front": {"rotation": rot, "offset": [0.2, 0.0, 0.5]}}}))
    csv = tmp_path / "timing.csv"
    proto = tmp_path / "last.pb"
    out = subprocess.run([os.path.join(built, "at_mock_node"), "--width", str(W), "--height", str(H), "--format",
                          "bgr8", "--frames", str(path), "--camera-serial", "S1", "--system-config", str(cfg),
                          "--measurement-csv", str(csv), "--proto-out", str(proto)],
                         check=True, capture_output=True, text=True, timeout=180).stdout
    lines = [json.loads(l) for l in out.splitlines()][1:]  # after the set-up line
    assert len(lines) == 2
    node = N.ApriltagsDetectorNode(W, H, parameters={"camera_serial": "S1"}, system_config_path=str(cfg))
    Msg = proto_classes()
    for i, rec in enumerate(lines):
        assert rec["status"] == 0 and rec["location"] == "front" and rec["camera_pose_topic"] == "camera/pose_camera"
        orc = oracle_mod.Oracle(W, H)
        orc.detect(bgr[i], rva.AT_FMT_BGR8)
        want = orc.detections()
        assert [d["id"] for d in rec["detections"]] == [d["id"] for d in want] and len(want) == 15
        for a, b in zip(rec["detections"], want):
            assert np.allclose(a["p"], b["p"], atol=1e-4)
        res = node.image_callback(bgr[i], 1000.0 + 0.02 * i)
        assert [r[0] for r in rec["robot"]] == [r[0] for r in res.tag_detection_array]
        assert np.allclose(np.array(rec["robot"]), np.array(res.tag_detection_array), atol=1e-12)
        assert np.allclose(np.array(rec["camera"]), np.array(res.tag_detection_camera_array), atol=1e-12)
        assert np.allclose(rec["networktables"], res.networktables_pose_data, atol=1e-12)
        msg = Msg()
        msg.ParseFromString(bytes.fromhex(rec["proto_hex"]))
        assert [t.tag_id for t in msg.tags] == [r[0] for r in rec["robot"]]
        assert all(t.collect_time == 1000.0 + 0.02 * i for t in msg.tags)
    node.close()
    assert proto.read_bytes() == bytes.fromhex(lines[-1]["proto_hex"])
    rows = csv.read_text().splitlines()
    assert rows[0].startswith("latency_us,det_time_us") and len(rows) == 3


@pytest.mark.gpu
def test_gpu_outlines_match_cpu_drawing(nodelib):
    """at_draw_outlines_device draws the annotated image onto the
    BGR frame in HBM pixel-identically to the node's CPU drawing -- on a stream
    frame's real detections, and on hand-made overlapping ones (crossing sides,
    ids over edges: the last primitive in drawing order wins, as on the CPU)."""
    import torch
    from ros_vision_amd import detector as D
    from ros_vision_amd import synth
    L = D.load_library()
    W, H = 1280, 720
    _, gray, _ = synth.stream_frame(W, H, 9)
    bgr = np.ascontiguousarray(np.repeat(gray[:, :, None], 3, axis=2))
    det = D.GpuDetector(W, H)
    dets = det.detect(bgr, fmt=D.AT_FMT_BGR8)
    assert len(dets) > 10
    cpu = bgr.copy()
    nodelib.at_node_draw_detection_outlines(cpu.ctypes.data, W, H, det._out, len(dets))
    dev = torch.from_numpy(bgr).cuda()
    det.draw_outlines_device(dev.data_ptr())
    gpu_img = dev.cpu().numpy()
    assert not np.array_equal(cpu, bgr)
    assert np.array_equal(gpu_img, cpu), int((gpu_img != cpu).any(axis=-1).sum())
    # overlapping hand-made detections, multi-digit ids, corners partly off-image
    raw = (D.AtDetection * 4)()
    quads = [[(10.5, 10.2), (200.7, 30.1), (180.3, 190.9), (20.2, 170.4)],
             [(100.1, 50.8), (300.6, 60.2), (290.2, 230.7), (90.9, 220.3)],
             [(-20.0, 100.0), (60.0, 80.0), (70.0, 260.0), (-30.0, 250.0)],
             [(150.0, 100.0), (151.0, 100.5), (151.5, 101.0), (150.2, 101.2)]]
    for i, q in enumerate(quads):
        raw[i].id = [586, 12, 7, 100][i]
        for k, (x, y) in enumerate(q):
            raw[i].p[k][0], raw[i].p[k][1] = x, y
        raw[i].c[0] = sum(x for x, _ in q) / 4
        raw[i].c[1] = sum(y for _, y in q) / 4
    small = D.GpuDetector(320, 240)
    base = (np.arange(320 * 240 * 3) % 251).astype(np.uint8).reshape(240, 320, 3)
    cpu = base.copy()
    nodelib.at_node_draw_detection_outlines(cpu.ctypes.data, 320, 240, raw, 4)
    dev = torch.from_numpy(base).cuda()
    assert L.at_draw_outlines_device(small._h, raw, 4, dev.data_ptr()) == 0
    assert np.array_equal(dev.cpu().numpy(), cpu)
    # the scratch plane is left clear: drawing again on a fresh copy gives the same image
    dev2 = torch.from_numpy(base).cuda()
    assert L.at_draw_outlines_device(small._h, raw, 4, dev2.data_ptr()) == 0
    assert np.array_equal(dev2.cpu().numpy(), cpu)


def test_camera_config_records(nodelib, tmp_path):
    """ConfigLoader::getCameraConfig (vision_utils/config_loader.cpp:77-105, 158-170):
    complete records only, integer width / height / frame_rate."""
    cfg = tmp_path / "system_config.json"
    full = {"location": "left_front", "format": "MJPG", "height": 1080, "width": 1920, "frame_rate": 30,
            "api_preference": "V4L2"}
    cfg.write_text(json.dumps({"camera_mounted_positions": {
        "A": full, "B": dict(full, width=1280.0), "C": {k: v for k, v in full.items() if k != "format"},
        "D": "legacy_location"}}))
    w, h, fr = C.c_int(), C.c_int(), C.c_int()
    loc = C.create_string_buffer(64)
    assert nodelib.at_node_load_camera_config(str(cfg).encode(), b"A", w, h, fr, loc, 64) == 0
    assert (w.value, h.value, fr.value, loc.value) == (1920, 1080, 30, b"left_front")
    for serial in (b"B", b"C", b"D", b"missing"):  # skipped as the reference skips them
        assert nodelib.at_node_load_camera_config(str(cfg).encode(), serial, w, h, fr, loc, 64) == -1


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/vision_config_data/data"), reason="reference absent")
def test_camera_config_of_the_reference_system_config(nodelib):
    """The deployed records (src/vision_config_data/data/system_config.json:2-50):
    1920x1080, 800x600 and 1280x800 cameras."""
    path = b"/root/reference/src/vision_config_data/data/system_config.json"
    w, h, fr = C.c_int(), C.c_int(), C.c_int()
    loc = C.create_string_buffer(64)
    want = {b"HBVCAM": (1920, 1080, b"center_front"), b"12": (800, 600, b"left_front"),
            b"199": (1280, 800, b"left_back"), b"test_camera": (640, 480, b"center_front")}
    for serial, (ww, hh, ll) in want.items():
        assert nodelib.at_node_load_camera_config(path, serial, w, h, fr, loc, 64) == 0
        assert (w.value, h.value, loc.value) == (ww, hh, ll)


def test_resolve_node_config_through_ament_prefix(nodelib, tmp_path, monkeypatch):
    """setup_apriltags (apriltags_cuda_detector.cu:137-193): vision_config_data found
    through AMENT_PREFIX_PATH as ament_index_cpp does; W x H from the camera record,
    intrinsics from data/calibration, extrinsics from data/system_config.json."""
    from ros_vision_amd import detector as D
    prefix = make_share_tree(tmp_path, "CAMX", 1920, 1080)
    monkeypatch.setenv("AMENT_PREFIX_PATH", "/nonexistent:" + str(prefix))
    buf = C.create_string_buffer(512)
    assert nodelib.at_node_package_share_directory(b"vision_config_data", buf, 512) > 0
    assert buf.value.decode() == str(prefix / "share/vision_config_data")
    wh, cam, R, t, have = (C.c_int * 2)(), D.AtCamera(), (C.c_double * 9)(), (C.c_double * 3)(), C.c_int()
    assert nodelib.at_node_resolve_config(b"CAMX", None, wh, C.byref(cam), R, t, C.byref(have)) == 0
    assert list(wh) == [1920, 1080] and cam.fx == 905.495617 and cam.k2 == -0.075154 and have.value == 1
    assert list(R) == [0, 0, 1, -1, 0, 0, 0, -1, 0] and list(t) == [0.25, -0.1, 0.4]
    # the reference throws without the camera record or the calibration file
    assert nodelib.at_node_resolve_config(b"UNKNOWN", None, wh, C.byref(cam), R, t, C.byref(have)) == -1
    monkeypatch.setenv("AMENT_PREFIX_PATH", "/nonexistent")
    assert nodelib.at_node_resolve_config(b"CAMX", None, wh, C.byref(cam), R, t, C.byref(have)) == -1
    share = str(prefix / "share/vision_config_data").encode()  # explicit directory (fallback parameter)
    assert nodelib.at_node_resolve_config(b"CAMX", share, wh, C.byref(cam), R, t, C.byref(have)) == 0


def test_cpu_pinning_and_scheduling(built):
    """ProcessScheduler::applyCpuPinningAndScheduling (process_scheduler.cpp:23-121) in a
    child process: -1 disables; an out-of-range core fails; a valid core pins the
    thread (SCHED_FIFO succeeds only with CAP_SYS_NICE, reported either way)."""
    code = r"""
import ctypes as C, os, sys, json
sys.path.insert(0, %r)
from ros_vision_amd import detector
detector.load_library()
L = C.CDLL(%r)
L.at_node_apply_cpu_pinning.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_size_t]
log = C.create_string_buffer(4096)
out = {"off": L.at_node_apply_cpu_pinning(-1, 80, log, 4096)}
out["bad_core"] = L.at_node_apply_cpu_pinning(10 ** 6, 80, log, 4096)
core = sorted(os.sched_getaffinity(0))[0]
out["pin"] = L.at_node_apply_cpu_pinning(core, 10, log, 4096)
out["affinity"] = sorted(os.sched_getaffinity(0))
out["core"] = core
out["log"] = log.value.decode()
print(json.dumps(out))
""" % (ROOT, os.path.join(built, "libat_node.so"))
    r = json.loads(subprocess.run([sys.executable, "-c", code], check=True, capture_output=True, text=True,
                                  timeout=120).stdout.strip().splitlines()[-1])
    assert r["off"] == 1 and r["bad_core"] == 0
    assert r["affinity"] == [r["core"]]  # the calling thread is pinned whatever SCHED_FIFO did
    assert ("SCHED_FIFO priority 10" in r["log"]) == (r["pin"] == 1)


@pytest.mark.gpu
def test_mock_node_from_camera_serial_1080p(built, oracle_mod, tmp_path, nodelib):
    """given only --camera-serial (the launch file's parameters,
    launch_vision.py:283-305) the node takes 1920x1080, the intrinsics and the extrinsics
    from vision_config_data, detects like the oracle, and publishes the outlined image
    drawn on the GPU on the staged frame -- pixel-identical to the CPU drawing."""
    import ros_vision_amd as rva
    from ros_vision_amd import synth
    W, H = 1920, 1080
    prefix = make_share_tree(tmp_path, "HBVCAM", W, H)
    gray, _ = synth.render_board(W, H, seed=4300, ntags=24)
    bgr = np.ascontiguousarray(np.repeat(gray[:, :, None], 3, axis=2))
    path = tmp_path / "frames.raw"
    bgr.tofile(path)
    img_out = tmp_path / "annotated.raw"
    env = dict(os.environ, AMENT_PREFIX_PATH=str(prefix))
    out = subprocess.run([os.path.join(built, "at_mock_node"), "--camera-serial", "HBVCAM", "--format", "bgr8",
                          "--frames", str(path), "--image-out", str(img_out), "--pin-to-core", "-1"],
                         check=True, capture_output=True, text=True, timeout=180, env=env).stdout
    lines = [json.loads(l) for l in out.splitlines()]
    assert lines[0]["width"] == W and lines[0]["height"] == H and lines[0]["location"] == "center_front"
    rec = lines[1]
    orc = oracle_mod.Oracle(W, H)
    orc.detect(bgr, rva.AT_FMT_BGR8)
    want = orc.detections()
    assert rec["status"] == 0 and len(want) >= 15
    assert [d["id"] for d in rec["detections"]] == [d["id"] for d in want]
    for a, b in zip(rec["detections"], want):
        assert np.allclose(a["p"], b["p"], atol=1e-4) and np.array_equal(np.floor(a["p"]), np.floor(b["p"]))
    # robot frame = R_ext t + t_ext of the camera-frame position
    R = np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], float)
    for r, c in zip(rec["robot"], rec["camera"]):
        assert r[0] == c[0] and np.allclose(R @ np.array(c[1:]) + [0.25, -0.1, 0.4], r[1:], atol=1e-12)
    # the GPU-annotated image == the node's CPU drawing of the same detections
    dets = (rva.detector.AtDetection * len(want))()
    for i, d in enumerate(rec["detections"]):
        dets[i].id = d["id"]
        for k in range(4):
            dets[i].p[k][0], dets[i].p[k][1] = d["p"][k]
        dets[i].c[0], dets[i].c[1] = d["c"]
    cpu = bgr.copy()
    nodelib.at_node_draw_detection_outlines(cpu.ctypes.data, W, H, dets, len(want))
    gpu_img = np.fromfile(img_out, np.uint8).reshape(H, W, 3)
    assert not np.array_equal(cpu, bgr) and np.array_equal(gpu_img, cpu)


def test_ros2_node_type_checks():
    """node/ros2_apriltags_node.cpp (the rclcpp binding; ROS 2 is absent here) compiles
    against type-check stand-ins of the rclcpp / sensor_msgs / ament_index API it uses
    and the reference's message layouts (msg/TagDetection.msg: int32 id, float64 x y z)."""
    stub = os.path.join(ROOT, "tests", "ros_stub")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I" + stub,
                        "-I" + NODE, os.path.join(NODE, "ros2_apriltags_node.cpp")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]


def test_mock_node_rejects_timing_without_frames(built, tmp_path):
    """`--time` over zero frames (--count 0 or an empty frames file) exits 2
    with a message before the timed loop (its `% count` would divide by zero)."""
    empty = tmp_path / "empty.bgr"
    empty.write_bytes(b"")
    for extra in ([], ["--count", "0"]):
        r = subprocess.run([os.path.join(built, "at_mock_node"), "--width", "64", "--height", "64", "--format",
                            "gray", "--frames", str(empty), "--time", "5"] + extra,
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 2 and "--time needs at least one frame" in r.stderr, (r.returncode, r.stderr)
