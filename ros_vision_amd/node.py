"""Node-side adapter: the per-frame logic of the reference ROS 2 node over this
detector (reference src/apriltags_cuda/src/apriltags_cuda_detector.cu).

ROS 2 (rclpy / rclcpp, cv_bridge, image_transport) is not installed in this
image, so the adapter is transport-free: `ApriltagsDetectorNode` owns the
detector, the calibration, the extrinsics and the measurement CSV, and hands
each frame's outputs to injected publisher callables.  A ROS 2 wrapper binds
those callables to the node's publishers.  What it keeps
from the reference:

* parameters and defaults (`setup_topics`, `setup_measurement_params`,
  apriltags_cuda_detector.cu:93-133, 558-593) and the subscription QoS
  (depth 1, best effort, volatile, 50 ms deadline);
* camera calibration from ``calibrationmatrix_<serial>.json`` (`matrix`,
  `disto`, :315-371) and extrinsics from ``system_config.json``
  (`camera_mounted_positions` legacy string or ``{"location": ...}`` object,
  `extrinsics[location].rotation/offset`, :196-300);
* per frame (`imageCallback`, :382-557): detect (BGR input goes straight to the
  GPU, no CPU cvtColor), pose of every tag (GPU), camera->robot transform,
  sort by distance, the two TagDetectionArray messages (robot frame on
  `publish_pose_to_topic`, camera frame on `..._camera`), the NetworkTables
  vector ``[t, id, x, y, z] * n`` and the ``ApriltagListProto`` tag list, the
  outlined image (`draw_detection_outlines`, apriltag_utils.cu:54-79, without
  the id text), and the measurement CSV row.
"""
import json
import os
import time
from dataclasses import dataclass, field

import numpy as np

from .detector import (AT_FMT_BGR8, AT_FMT_YUYV, TAG_SIZE, CameraMatrix, DistCoeffs, GpuDetector,
                       tag_detections)

PARAMETER_DEFAULTS = {
    "topic_name": "camera/image_raw",
    "camera_serial": "N/A",
    "publish_images_to_topic": "apriltags/images",
    "publish_pose_to_topic": "camera/pose",
    "pin_to_core": -1,
    "priority": 80,
    "measurement_mode": False,
    "timing_csv_path": "",
}

# rclcpp::QoS(1).best_effort().durability_volatile().deadline(50 ms)
SUBSCRIPTION_QOS = {"depth": 1, "reliability": "best_effort", "durability": "volatile", "deadline_ms": 50}

CSV_HEADER = ("latency_us,det_time_us,publish_pose_us,publish_camera_pose_us,"
              "publish_image_us,networktables_us,processing_time_us")


def load_camera_calibration(calibration_dir, camera_serial):
    """calibrationmatrix_<serial>.json -> (CameraMatrix, DistCoeffs)."""
    path = os.path.join(calibration_dir, "calibrationmatrix_%s.json" % camera_serial)
    with open(path) as f:
        data = json.load(f)
    if "matrix" not in data or "disto" not in data:
        raise KeyError("calibration file %s needs 'matrix' and 'disto'" % path)
    m, d = data["matrix"], data["disto"][0]
    cam = CameraMatrix(fx=float(m[0][0]), cx=float(m[0][2]), fy=float(m[1][1]), cy=float(m[1][2]))
    dist = DistCoeffs(k1=float(d[0]), k2=float(d[1]), p1=float(d[2]), p2=float(d[3]), k3=float(d[4]))
    return cam, dist


def load_extrinsics(system_config_path, camera_serial):
    """system_config.json -> (3x3 rotation, 3 offset, location).  Identity / zero when the
    camera or its location is missing (the reference logs an error and keeps its defaults)."""
    R, t = np.eye(3), np.zeros(3)
    try:
        with open(system_config_path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        return R, t, None
    pos = data.get("camera_mounted_positions", {}).get(camera_serial)
    if isinstance(pos, str):
        location = pos                      # legacy format
    elif isinstance(pos, dict) and "location" in pos:
        location = pos["location"]
    else:
        return R, t, None
    extr = data.get("extrinsics", {}).get(location)
    if not extr or "rotation" not in extr or "offset" not in extr:
        return R, t, location
    return (np.array(extr["rotation"], np.float64).reshape(3, 3), np.array(extr["offset"], np.float64).reshape(3),
            location)


def draw_detection_outlines(bgr, dets):
    """Outline every tag on a BGR image in place: p0-p1 green, p0-p3 red, p1-p2 and p2-p3
    blue, 2 px (apriltag_utils.cu:54-79; the id text is not drawn)."""
    h, w = bgr.shape[:2]

    def line(a, b, color):
        n = int(max(abs(b[0] - a[0]), abs(b[1] - a[1]))) + 1
        xs = np.rint(np.linspace(a[0], b[0], n)).astype(int)
        ys = np.rint(np.linspace(a[1], b[1], n)).astype(int)
        for dx in (0, 1):
            for dy in (0, 1):
                x, y = xs + dx, ys + dy
                ok = (x >= 0) & (x < w) & (y >= 0) & (y < h)
                bgr[y[ok], x[ok]] = color

    for d in dets:
        p = np.asarray(d.p)
        line(p[0], p[1], (0, 255, 0))
        line(p[0], p[3], (0, 0, 255))
        line(p[1], p[2], (255, 0, 0))
        line(p[2], p[3], (255, 0, 0))
    return bgr


@dataclass
class FrameResult:
    """Everything one imageCallback publishes."""
    tag_detection_array: list = field(default_factory=list)          # robot frame: (id, x, y, z)
    tag_detection_camera_array: list = field(default_factory=list)   # camera frame
    networktables_pose_data: list = field(default_factory=list)      # [t, id, x, y, z] * n
    proto_tags: list = field(default_factory=list)                    # ApriltagListProto.tags
    image: np.ndarray = None


class ApriltagsDetectorNode:
    """ApriltagsDetector (apriltags_cuda_detector.cu) without the ROS transport."""

    def __init__(self, width, height, parameters=None, calibration_dir=None, system_config_path=None,
                 publishers=None, device=0):
        self.params = dict(PARAMETER_DEFAULTS)
        self.params.update(parameters or {})
        serial = self.params["camera_serial"]
        if calibration_dir is not None:
            cam, dist = load_camera_calibration(calibration_dir, serial)
        else:
            from .detector import TEST_CAMERA, TEST_DIST
            cam, dist = TEST_CAMERA, TEST_DIST
        self.camera, self.distortion = cam, dist
        self.extrinsic_rotation, self.extrinsic_offset, self.location = (
            load_extrinsics(system_config_path, serial) if system_config_path else (np.eye(3), np.zeros(3), None))
        self.detector = GpuDetector(width, height, cam, dist, device=device, tag_size=TAG_SIZE)
        self.publishers = publishers or {}
        self.pose_topic = self.params["publish_pose_to_topic"]
        self.camera_pose_topic = self.pose_topic + "_camera"
        self.image_topic = self.params["publish_images_to_topic"]
        self.csv = None
        if self.params["measurement_mode"]:
            path = self.params["timing_csv_path"] or time.strftime("apriltags_timing_%Y%m%d_%H%M%S.csv")
            self.csv = open(path, "w")
            self.csv.write(CSV_HEADER + "\n")
            self.csv.flush()

    def close(self):
        if self.csv:
            self.csv.close()
            self.csv = None
        self.detector.close()

    def _publish(self, topic, payload):
        fn = self.publishers.get(topic)
        if fn is not None:
            fn(payload)

    def image_callback(self, image, stamp_s, encoding="bgr8", receive_time_s=None):
        """One frame: `image` is bgr8 [H, W, 3] (what cv_bridge hands the reference) or
        yuyv [H, 2W]."""
        start = time.perf_counter()
        latency_s = (receive_time_s if receive_time_s is not None else time.time()) - stamp_s
        fmt = AT_FMT_BGR8 if encoding == "bgr8" else AT_FMT_YUYV
        det0 = time.perf_counter()
        dets = self.detector.detect(np.ascontiguousarray(image), fmt)
        det1 = time.perf_counter()
        poses = self.detector.poses()
        res = FrameResult()
        for tag in tag_detections(poses, self.extrinsic_rotation, self.extrinsic_offset):
            rx, ry, rz = (float(v) for v in tag.robot)
            res.networktables_pose_data += [stamp_s, tag.id * 1.0, rx, ry, rz]
            res.proto_tags.append({"collect_time": stamp_s, "tag_id": tag.id, "x": rx, "y": ry, "z": rz})
            res.tag_detection_camera_array.append((tag.id, *(float(v) for v in tag.camera)))
            res.tag_detection_array.append((tag.id, rx, ry, rz))
        if encoding == "bgr8":
            res.image = draw_detection_outlines(np.array(image, copy=True), dets)
        nt0 = time.perf_counter()
        self._publish("networktables", res.networktables_pose_data)
        self._publish("networktables_proto", res.proto_tags)
        nt1 = time.perf_counter()
        self._publish(self.pose_topic, res.tag_detection_array)
        pp1 = time.perf_counter()
        self._publish(self.camera_pose_topic, res.tag_detection_camera_array)
        pc1 = time.perf_counter()
        if res.image is not None:
            self._publish(self.image_topic, res.image)
        pi1 = time.perf_counter()
        if self.csv:
            us = lambda a, b: int(round((b - a) * 1e6))  # noqa: E731
            self.csv.write("%d,%d,%d,%d,%d,%d,%d\n" % (int(latency_s * 1e6), us(det0, det1), us(nt1, pp1),
                                                       us(pp1, pc1), us(pc1, pi1), us(nt0, nt1), us(start, pi1)))
            self.csv.flush()
        return res
