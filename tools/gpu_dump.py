"""Run the HIP path on a few inputs and dump every parity tap to gpurun_out/dump_*.npz
(analysed on the CPU side against the oracle)."""
import os
import sys
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ros_vision_amd as rva
from ros_vision_amd import synth

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
os.makedirs(out, exist_ok=True)
cases = [("syn1080", 1920, 1080, synth.to_yuyv(synth.render_board(1920, 1080, seed=4242, ntags=24)[0]), 0)]
for name, W, H, frame, fmt in cases:
    det = rva.GpuDetector(W, H, debug_taps=True)
    dets = det.detect(frame, fmt)
    np.savez_compressed(os.path.join(out, "dump_%s.npz" % name),
                        blob_points=det.copy_blob_points(), points=det.copy_points(),
                        quads=np.array([(q["blob_index"], q["valid"], q["accepted"], *q["indices"],
                                         *q["corners"].ravel()) for q in det.copy_quads()], np.float64),
                        ids=np.array([d.id for d in dets]), npairs=det.num_pairs())
    print(name, "dets", [d.id for d in dets], "pairs", det.num_pairs())

