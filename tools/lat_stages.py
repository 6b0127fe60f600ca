"""B=1 latency breakdown: serialized per-stage GPU time of the latency-mode
detector (HIP events between the kernels, direct launches) over N stream frames,
next to the end-to-end wall time from HBM (graph replay, no events).
Usage: python tools/lat_stages.py [N]"""
import os
import sys
import time

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
for i in range(20):
    det.detect_device(d_frames.data_ptr() + (i % pool) * stride, stride, 1, counts_only=True)
lat = []
for i in range(N):
    t = time.perf_counter()
    det.detect_device(d_frames.data_ptr() + (i % pool) * stride, stride, 1, counts_only=True)
    lat.append(time.perf_counter() - t)
print("wall p50 %.1f us  p10 %.1f us" % (np.percentile(lat, 50) * 1e6, np.percentile(lat, 10) * 1e6))
det.set_profiling(True)
for i in range(N):
    det.detect_device(d_frames.data_ptr() + (i % pool) * stride, stride, 1, counts_only=True)
st, nb = det.stage_times()
print("stage us:", " ".join("%s=%.1f" % (k, v * 1e3) for k, v in st.items()), " sum %.1f" % (sum(st.values()) * 1e3))
