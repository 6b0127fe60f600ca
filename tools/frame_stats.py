"""Per-frame workload statistics of the bench stream (boundary points, blob
pairs, per-tile pair entries, selected blobs by size) -- sizing data for the
k_boundary / k_pairs / k_blob launch shapes."""
import os
import sys
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (owns the HIP runtime)
import ros_vision_amd as rva
from ros_vision_amd import synth

W, H, N = 1280, 720, 8
codes = dict(rva.family_entries())
det = rva.GpuDetector(W, H, debug_taps=True)
for i in range(N):
    gray, _ = synth.render_board(W, H, seed=766000 + i, ntags=15, codes=codes)
    det.detect(synth.to_yuyv(gray))
    bp = det.copy_blob_points()
    qs = det.copy_quads()
    print("frame %d: points %d pairs %d pair_entries %d selected_points %d quads %d" % (
        i, det.num_points(), det.num_pairs(), det.num_pair_entries(), bp.size, len(qs)))
