"""Kernel-trace companion of tools/lat_stages.py: B=1 detections from HBM in graph
mode, N frames (run under rocprofv3 --kernel-trace; tools/gap_report.py then
reports the per-kernel durations and the idle gaps between them)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ros_vision_amd as rva  # noqa: E402
from ros_vision_amd import synth  # noqa: E402

W, H = 1280, 720
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
pool = 16
frames = np.stack([synth.stream_frame(W, H, f)[0] for f in range(pool)])
d_frames = torch.from_numpy(frames).cuda()
stride = frames[0].nbytes
det = rva.GpuDetector(W, H, max_batch=1)
for i in range(N):
    det.detect_device(d_frames.data_ptr() + (i % pool) * stride, stride, 1, counts_only=True)
print("ok", N)
