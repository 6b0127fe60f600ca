"""Accumulated per-phase time of the blob and decode kernels (AT_PHASE_PROBE=1): phase k
of blob_item = time from marker k-1 to marker k summed over all work items
(microseconds of wave time), for the wave-per-blob (small) and the
workgroup-per-blob (large) variants."""
import os
import sys
import numpy as np

os.environ.setdefault("AT_PHASE_PROBE", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ros_vision_amd as rva
from ros_vision_amd import synth

W, H, B = 1280, 720, int(sys.argv[1]) if len(sys.argv) > 1 else 32
codes = dict(rva.family_entries())
frames = np.stack([synth.to_yuyv(synth.render_board(W, H, seed=766000 + i, ntags=15, codes=codes)[0])
                   for i in range(B)])
d_frames = torch.from_numpy(frames).cuda()
det = rva.GpuDetector(W, H, max_batch=B)
det.detect_device(d_frames.data_ptr(), frames[0].nbytes, B)
p0 = det.copy_probe().astype(np.int64)
det.detect_device(d_frames.data_ptr(), frames[0].nbytes, B)
p = det.copy_probe().astype(np.int64) - p0
names = {0: "select check", 1: "load keys", 2: "theta sort", 3: "compact+scan", 4: "errors",
         5: "filter+peaks", 6: "top10+prefix", 7: "segment fits", 8: "combinations", 9: "update+emit"}
dnames = {1: "refine samples", 2: "edge fits", 3: "corners", 4: "homography", 5: "gray samples",
          6: "gray models", 7: "bit samples", 8: "sharpen+score", 9: "codebook+emit"}
for kind, base in (("small", 64), ("large", 80), ("decode", 128)):
    if kind == "decode":
        names = dnames
    print(kind)
    for k in range(16):
        if p[base + k] or p[base + 32 + k]:
            print("  phase %d %-16s total %9.1f us  count %6d  mean %7.2f us" % (
                k, names.get(k, ""), p[base + k] / 100.0, p[base + 32 + k], p[base + k] / 100.0 / max(1, p[base + 32 + k])))

for name, idx in (("small", 200), ("large", 201)):
    v = int(det.copy_probe().astype(np.int64)[idx])
    print("slowest %s item: %.2f us, %d points" % (name, (v >> 20) / 100.0, v & 0xfffff))
pp = det.copy_probe().astype(np.int64)
nbig = max(1, int(pp[220]) // 2)
print("large blobs > 2048 points (%d per batch): mean phase us" % nbig,
      [round(pp[208 + k] / 100.0 / 2 / nbig, 2) for k in range(10)])
nslow = max(1, int(pp[234]))
print("slowest small item per wave team (%d teams): mean phase us" % int(pp[234]),
      [round(pp[224 + k] / 100.0 / nslow, 2) for k in range(10)])
