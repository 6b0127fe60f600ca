"""Node adapter (ros_vision_amd/node.py): configuration loading and per-frame
outputs of the reference node's imageCallback.  The config files are written
here: only their schema (key names and nesting of
calibrationmatrix_<serial>.json and system_config.json, read by
apriltags_cuda_detector.cu:196-371) follows the reference; every value is
synthetic."""
import json
import math
import types

import numpy as np
import pytest


def _rz(deg):
    a = math.radians(deg)
    return np.array([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]])


def _write_calibration(d, serial, fx=800.0, fy=810.0, cx=640.0, cy=360.0, disto=(0.01, -0.02, 0.001, 0.002, 0.0)):
    path = d / ("calibrationmatrix_%s.json" % serial)
    path.write_text(json.dumps({"matrix": [[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]],
                                "disto": [list(disto)]}))
    return path


def _write_system_config(d):
    rot = _rz(30.0)
    cfg = {"camera_mounted_positions": {"CAM_A": {"location": "mount_a"},
                                        "CAM_B": "mount_b",
                                        "CAM_C": {"width": 640},
                                        "CAM_D": {"location": "mount_missing"}},
           "extrinsics": {"mount_a": {"rotation": rot.tolist(), "offset": [0.1, -0.2, 0.5]},
                          "mount_b": {"rotation": np.eye(3).tolist(), "offset": [1.0, 2.0, 3.0]}}}
    path = d / "system_config.json"
    path.write_text(json.dumps(cfg))
    return path, rot


def test_calibration_loader(tmp_path):
    from ros_vision_amd.node import load_camera_calibration
    _write_calibration(tmp_path, "S1")
    cam, dist = load_camera_calibration(str(tmp_path), "S1")
    assert (cam.fx, cam.fy, cam.cx, cam.cy) == (800.0, 810.0, 640.0, 360.0)
    assert (dist.k1, dist.k2, dist.p1, dist.p2, dist.k3) == (0.01, -0.02, 0.001, 0.002, 0.0)
    (tmp_path / "calibrationmatrix_BAD.json").write_text(json.dumps({"matrix": [[1, 0, 0]]}))
    with pytest.raises(KeyError):
        load_camera_calibration(str(tmp_path), "BAD")


def test_extrinsics_loader_formats(tmp_path):
    from ros_vision_amd.node import load_extrinsics
    path, rot = _write_system_config(tmp_path)
    R, t, loc = load_extrinsics(str(path), "CAM_A")              # {"location": ...} object
    assert loc == "mount_a" and np.allclose(R, rot) and np.allclose(t, [0.1, -0.2, 0.5])
    R, t, loc = load_extrinsics(str(path), "CAM_B")              # legacy string
    assert loc == "mount_b" and np.array_equal(R, np.eye(3)) and np.allclose(t, [1.0, 2.0, 3.0])
    for serial in ("CAM_C", "CAM_D", "UNKNOWN"):
        R, t, _ = load_extrinsics(str(path), serial)
        assert np.array_equal(R, np.eye(3)) and np.array_equal(t, np.zeros(3))
    R, t, loc = load_extrinsics(str(tmp_path / "absent.json"), "CAM_A")
    assert loc is None and np.array_equal(R, np.eye(3))


def test_parameter_defaults_and_qos():
    from ros_vision_amd.node import PARAMETER_DEFAULTS, SUBSCRIPTION_QOS
    assert PARAMETER_DEFAULTS["topic_name"] == "camera/image_raw"
    assert PARAMETER_DEFAULTS["publish_pose_to_topic"] == "camera/pose"
    assert PARAMETER_DEFAULTS["publish_images_to_topic"] == "apriltags/images"
    assert PARAMETER_DEFAULTS["priority"] == 80 and PARAMETER_DEFAULTS["pin_to_core"] == -1
    assert SUBSCRIPTION_QOS == {"depth": 1, "reliability": "best_effort", "durability": "volatile",
                                "deadline_ms": 50}


def test_draw_detection_outlines_colors():
    from ros_vision_amd.node import draw_detection_outlines
    img = np.zeros((40, 40, 3), np.uint8)
    d = types.SimpleNamespace(p=np.array([[5.0, 30.0], [30.0, 30.0], [30.0, 5.0], [5.0, 5.0]]))
    draw_detection_outlines(img, [d])
    assert tuple(img[30, 15]) == (0, 255, 0)     # p0-p1 green
    assert tuple(img[15, 5]) == (0, 0, 255)      # p0-p3 red
    assert tuple(img[15, 30]) == (255, 0, 0)     # p1-p2 blue
    assert tuple(img[20, 20]) == (0, 0, 0)


@pytest.mark.gpu
def test_node_frame_outputs(tmp_path):
    """imageCallback on a synthetic bgr8 frame: tag set, distance order, camera/robot
    arrays, NetworkTables vector layout, CSV row."""
    from ros_vision_amd import synth
    from ros_vision_amd.node import CSV_HEADER, ApriltagsDetectorNode
    _write_calibration(tmp_path, "CAM_A")
    cfg, rot = _write_system_config(tmp_path)
    got = {}
    csv = tmp_path / "timing.csv"
    node = ApriltagsDetectorNode(1280, 720, {"camera_serial": "CAM_A", "measurement_mode": True,
                                             "timing_csv_path": str(csv)},
                                 calibration_dir=str(tmp_path), system_config_path=str(cfg),
                                 publishers={"camera/pose": lambda m: got.setdefault("pose", m),
                                             "camera/pose_camera": lambda m: got.setdefault("cam", m),
                                             "networktables": lambda m: got.setdefault("nt", m),
                                             "apriltags/images": lambda m: got.setdefault("img", m)})
    _, gray, truth = synth.stream_frame(1280, 720, 0)
    bgr = np.repeat(gray[:, :, None], 3, axis=2)
    res = node.image_callback(bgr, stamp_s=123.5)
    node.close()
    ids = sorted(t[0] for t in truth)
    assert sorted(t[0] for t in res.tag_detection_array) == ids
    cam = res.tag_detection_camera_array
    dist = [math.sqrt(x * x + y * y + z * z) for _, x, y, z in cam]
    assert dist == sorted(dist)
    for (i0, x, y, z), (i1, rx, ry, rz) in zip(cam, res.tag_detection_array):
        assert i0 == i1
        assert np.allclose(rot @ np.array([x, y, z]) + [0.1, -0.2, 0.5], [rx, ry, rz])
    nt = res.networktables_pose_data
    assert len(nt) == 5 * len(ids) and nt[0] == 123.5 and nt[1] == float(res.tag_detection_array[0][0])
    assert got["pose"] is res.tag_detection_array and got["cam"] is cam and got["img"].shape == bgr.shape
    lines = csv.read_text().splitlines()
    assert lines[0] == CSV_HEADER and len(lines) == 2 and len(lines[1].split(",")) == 7
