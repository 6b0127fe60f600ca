import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # loads torch's bundled libamdhip64.so.7 first
import numpy as np
import ros_vision_amd as rva
from ros_vision_amd import synth
x = torch.zeros(4, device="cuda"); print("torch ok", x.device)
frames = np.stack([synth.stream_frame(1280, 720, i)[0] for i in range(3)])
t = torch.from_numpy(frames).cuda()
det = rva.GpuDetector(1280, 720, max_batch=3)
res = det.detect_device(t.data_ptr(), frames[0].nbytes, 3)
print([[d.id for d in r] for r in res])
print(det.detect(frames[0]) and "host ok")
