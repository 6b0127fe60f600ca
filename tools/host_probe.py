"""Host-side cost of the bench loop: time spent in enqueue (graph launch) and in
collect (wait + host tail) per step, 4 detector instances, B=32 (bench defaults)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch  # noqa: E402

import ros_vision_amd as rva  # noqa: E402
from ros_vision_amd import synth  # noqa: E402

W, H, B, NI, STEPS = 1280, 720, int(sys.argv[1]) if len(sys.argv) > 1 else 32, 4, 60
codes = dict(rva.family_entries())
frames = np.stack([synth.to_yuyv(synth.render_board(W, H, seed=766000 + i, ntags=15, codes=codes)[0])
                   for i in range(64)])
d_frames = torch.from_numpy(frames).to("cuda")
stride, base = frames[0].nbytes, d_frames.data_ptr()
dets = [rva.GpuDetector(W, H, max_batch=B) for _ in range(NI)]


def loop(n):
    te = tc = 0.0
    inflight = []
    t0 = time.perf_counter()
    for s in range(n):
        d = dets[s % NI]
        t1 = time.perf_counter()
        d.enqueue_device(base + ((s * B) % 64) * stride, stride, B)
        te += time.perf_counter() - t1
        inflight.append(d)
        if len(inflight) == NI:
            t1 = time.perf_counter()
            inflight.pop(0).collect(counts_only=True)
            tc += time.perf_counter() - t1
    for d in inflight:
        d.collect(counts_only=True)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, te, tc


loop(8)
tot, te, tc = loop(STEPS)
print("B=%d step %.3f ms  enqueue %.3f ms/step  collect %.3f ms/step  fps %.0f" %
      (B, 1e3 * tot / STEPS, 1e3 * te / STEPS, 1e3 * tc / STEPS, STEPS * B / tot))
# host tail alone: collect of a batch that is already complete
d = dets[0]
d.enqueue_device(base, stride, B)
torch.cuda.synchronize()
time.sleep(0.01)
t1 = time.perf_counter()
d.collect(counts_only=True)
print("collect of a finished batch (host tail only): %.3f ms" % (1e3 * (time.perf_counter() - t1)))
