"""B=1 host-side latency split: at_enqueue_device (graph launch) and at_collect (wait +
host tail) timed apart around the same call the bench's p50_latency_hbm_ms times.
Usage: python tools/lat_host.py [N]"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ros_vision_amd as rva  # noqa: E402
from ros_vision_amd import synth  # noqa: E402

W, H = 1280, 720
N = int(sys.argv[1]) if len(sys.argv) > 1 else 500
pool = 16
frames = np.stack([synth.stream_frame(W, H, f)[0] for f in range(pool)])
d_frames = torch.from_numpy(frames).cuda()
stride = frames[0].nbytes
det = rva.GpuDetector(W, H, max_batch=1)
L = rva.detector.load_library()
for i in range(50):
    det.detect_device(d_frames.data_ptr() + (i % pool) * stride, stride, 1, counts_only=True)
enq, col, tot = [], [], []
for i in range(N):
    p = C.c_void_p(d_frames.data_ptr() + (i % pool) * stride)
    t0 = time.perf_counter()
    L.at_enqueue_device(det._h, p, stride, 1, 0)
    t1 = time.perf_counter()
    L.at_collect(det._h, det._out, det._cap, det._n)
    t2 = time.perf_counter()
    enq.append(t1 - t0)
    col.append(t2 - t1)
    tot.append(t2 - t0)
    det._pending = 1
f = lambda v: np.percentile(np.array(v) * 1e6, 50)
print("p50 us: enqueue %.1f  collect %.1f  total %.1f   (python detect_device adds the ctypes/unpack overhead)"
      % (f(enq), f(col), f(tot)))
