"""k_pose time per batch (HIP events) at B=32 and B=1 on the bench stream."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ros_vision_amd as rva
from ros_vision_amd import synth
W, H = 1280, 720
codes = dict(rva.family_entries())
frames = np.stack([synth.to_yuyv(synth.render_board(W, H, seed=766000 + i, ntags=15, codes=codes)[0]) for i in range(32)])
d_frames = torch.from_numpy(frames).cuda()
for B in (32, 1):
    det = rva.GpuDetector(W, H, max_batch=B)
    det.set_profiling(True)
    for _ in range(10):
        det.detect_device(d_frames.data_ptr(), frames[0].nbytes, B)
    st, n = det.stage_times()
    print("B=%d" % B, {k: round(v, 4) for k, v in st.items()})

# phase stamps of detection 0 of frame 0 (AT_PHASE_PROBE=1): probe[16 + k]
if os.environ.get("AT_PHASE_PROBE"):
    det = rva.GpuDetector(W, H, max_batch=1)
    for _ in range(3):
        det.detect_device(d_frames.data_ptr(), frames[0].nbytes, 1)
    p = det.copy_probe().astype(np.int64)
    st = p[16:21]
    print("pose phases (us): polar3 %.2f  OI-1 %.2f  ambiguity %.2f  OI-2 %.2f   steps k1=%d k2=%d" % tuple(
        list(np.diff(st) / 100.0) + [p[24], p[25]]))
