"""Phase clock stamps of an instrumented kernel (AT_PHASE_PROBE=1): runs one
batch of the bench stream and prints the deltas between stamps in microseconds
(wall_clock64 ticks at 100 MHz)."""
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
for rep in range(3):
    det.detect_device(d_frames.data_ptr(), frames[0].nbytes, B)
    p = det.copy_probe().astype(np.int64)
    nz = [i for i in range(64) if p[i] and i not in (24, 25)]
    print("  oi steps", p[24], p[25])
    t0 = p[nz[0]]
    print("rep %d:" % rep, " ".join("%d:%.2fus" % (i, (p[i] - t0) / 100.0) for i in nz))
