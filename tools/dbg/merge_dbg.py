import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'oracle'))
import numpy as np
import ao
import ros_vision_amd as rva
from ros_vision_amd import synth
rva.GpuDetector.DEBUG_TAPS = True
frames = [synth.stream_frame(1280, 720, f)[0] for f in (3, 17, 31, 45, 58, 5, 9, 12)]
det = rva.GpuDetector(1280, 720, max_batch=8)
det.detect_batch(frames)
print(det.batch_stats())
for c, f in enumerate(frames):
    orc = ao.Oracle(1280, 720); orc.detect(f, 0)
    gl = det.copy_union_markers(c); ol = orc.labels(); t = orc.thresholded()
    bad = np.argwhere(gl != ol)
    print("frame", c, "bad", len(bad))
    for (y, x) in bad[:10]:
        print("  at", y, x, "gpu", gl[y, x], divmod(int(gl[y, x]), 640), "orc", ol[y, x], divmod(int(ol[y, x]), 640), "thr", t[y, x],
              "tile", y // 32, x // 64, "in-tile", y % 32, x % 64)
        comp = (ol == ol[y, x]); print("   comp size(orc)", comp.sum(), "gpu labels in comp", np.unique(gl[comp])[:10])
        gcomp = (gl == gl[y, x]); print("   gpu comp size", gcomp.sum())
        print(t[max(0,y-3):y+4, max(0,x-3):x+4])
