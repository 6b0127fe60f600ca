# throughput with and without k_pose (tag_size 0 skips it): does the pose kernel's
# long low-occupancy tail limit the concurrent pipeline?
import os, sys, time, json
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import ros_vision_amd as rva
from ros_vision_amd import synth
W, H, B, NI = 1280, 720, 128, 4
frames = np.stack([synth.stream_frame(W, H, f)[0] for f in range(64)])
pool = torch.from_numpy(np.concatenate([frames, frames])).cuda()
stride = frames[0].nbytes
for rep in range(3):
    for ts in (0.1651, 0.0):
        dets = [rva.GpuDetector(W, H, max_batch=B, tag_size=ts) for _ in range(NI)]
        def run(n):
            inflight = []
            for s in range(n):
                d = dets[s % NI]
                d.enqueue_device(pool.data_ptr() + (s % 2) * 64 * stride // 2 * 0, stride, B)
                inflight.append(d)
                if len(inflight) == NI:
                    inflight.pop(0).collect(counts_only=True)
            for d in inflight: d.collect(counts_only=True)
        run(10); torch.cuda.synchronize()
        t0 = time.perf_counter(); run(200); torch.cuda.synchronize(); dt = time.perf_counter() - t0
        print("tag_size %.4f: %.0f frames/s" % (ts, 200 * B / dt), flush=True)
        for d in dets: d.close()
