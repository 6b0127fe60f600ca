"""MI355X-native AprilTag detection stage (drop-in for ros_vision's apriltags_cuda detector).

Product code: HIP kernels + C ABI in ``csrc/`` (built into ``libat_hip.so``),
the Python mirror of the reference GpuDetector interface in ``detector.py``
and the synthetic tag-board generator in ``synth.py``.
"""
from .detector import (AT_FMT_BGR8, AT_FMT_GRAY8, AT_FMT_YUYV, TAG_SIZE, TEST_CAMERA, TEST_DIST,  # noqa: F401
                       CameraMatrix, Detection, DistCoeffs, GpuDetector, Pose, TagDetection, family_entries,
                       game_piece_preprocess_device, load_library, tag_detections)

__all__ = ["GpuDetector", "CameraMatrix", "DistCoeffs", "Detection", "Pose", "TagDetection", "load_library",
           "family_entries", "tag_detections", "game_piece_preprocess_device", "TAG_SIZE", "TEST_CAMERA", "TEST_DIST",
           "AT_FMT_YUYV", "AT_FMT_BGR8", "AT_FMT_GRAY8"]
