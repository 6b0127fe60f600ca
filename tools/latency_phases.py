"""Per-phase average time of the blob and decode kernels (AT_PHASE_PROBE=1) at a
given batch size: ticks accumulated per phase over every item (wall_clock64,
100 MHz) divided by the item count of the phase.  Usage: python tools/latency_phases.py [B]"""
import os
import sys

import numpy as np

os.environ.setdefault("AT_PHASE_PROBE", "1")
# the phase probes exist only in the experiment build (make -C ros_vision_amd/csrc exp)
os.environ.setdefault("AT_HIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "ros_vision_amd/ab/libat_hip_exp.so"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ros_vision_amd as rva  # noqa: E402
from ros_vision_amd import synth  # noqa: E402

W, H = int(os.environ.get("LP_W", 1280)), int(os.environ.get("LP_H", 720))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
NT = int(os.environ.get("LP_TAGS", 15))
frames = np.stack([synth.stream_frame(W, H, f, ntags=NT)[0] for f in range(min(B, 16))])
frames = frames[np.arange(B) % frames.shape[0]]
d_frames = torch.from_numpy(frames).cuda()
det = rva.GpuDetector(W, H, max_batch=B)
for rep in range(3):
    det.detect_device(d_frames.data_ptr(), frames[0].nbytes, B)
p = det.copy_probe().astype(np.int64)
for name, base in (("k_blob_small", 64), ("k_blob", 80), ("k_decode", 128)):
    row = []
    for k in range(0, 10):
        t, n = p[base + k], p[base + 32 + k]
        if n:
            row.append("%d:%.2fus(x%d)" % (k, t / n / 100.0, n))
    print(name, " ".join(row))
for name, idx in (("small", 200), ("large", 201)):
    v = int(p[idx])
    print("slowest %s item: %.2f us, %d points" % (name, (v >> 20) / 100.0, v & 0xfffff))
nbig = max(1, int(p[220]))
print("large blobs > 2048 points (%d): mean phase us" % int(p[220]), [round(p[208 + k] / 100.0 / nbig, 2) for k in range(10)])
if B >= 8 and p[63]:
    nw = float(p[63])
    print("k_thr_ccl phases (us per workgroup, %d workgroups): loads %.2f  filter %.2f  threshold %.2f  runs %.2f  targets %.2f  "
          "unions %.2f  finds %.2f  counts %.2f  publish %.2f" % ((int(nw),) + tuple(p[48 + k] / nw / 100.0 for k in range(9))))
if B >= 8:
    print("k_ccl_merge phases (us, frame 0): base %.2f  roots %.2f  links %.2f  sizes %.2f  words %.2f" % tuple(np.diff(p[40:46]) / 100.0))
print("k_pairs phases (us): merge %.2f  list %.2f  rank %.2f  scan %.2f  work+bases %.2f" % tuple(np.diff(p[0:6]) / 100.0))
print("pose phases (us): polar3 %.2f  OI-1 %.2f  ambiguity %.2f  OI-2 %.2f" % tuple(np.diff(p[16:21]) / 100.0))
a = p[16 + 2]
print("ambiguity detail (us): setup %.2f  deg2 %.2f  deg3 %.2f  deg4 %.2f  minima %.2f  rest %.2f" % (
    (p[26] - a) / 100.0, (p[27] - p[26]) / 100.0, (p[28] - p[27]) / 100.0, (p[29] - p[28]) / 100.0,
    (p[30] - p[29]) / 100.0, (p[19] - p[30]) / 100.0))
