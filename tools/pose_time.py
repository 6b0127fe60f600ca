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
