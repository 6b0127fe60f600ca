"""MI355X-native AprilTag detection stage (drop-in for ros_vision's apriltags_cuda detector).

Product code: HIP kernels + C ABI in ``csrc/`` (built into ``libat_hip.so``),
the Python mirror of the reference GpuDetector interface in ``detector.py``
and the synthetic tag-board generator in ``synth.py``.
"""
from .detector import (AT_FMT_BGR8, AT_FMT_GRAY8, AT_FMT_YUYV, CameraMatrix, Detection,  # noqa: F401
                       DistCoeffs, GpuDetector, family_entries, load_library)

__all__ = ["GpuDetector", "CameraMatrix", "DistCoeffs", "Detection", "load_library", "family_entries",
           "AT_FMT_YUYV", "AT_FMT_BGR8", "AT_FMT_GRAY8"]
