"""Blob-size histogram and lane occupancy of the blob kernels on the bench workload.

Runs the product library in throughput mode (max_batch 64) over the bench's C2 pool
(stream_pool: 1280x720, 15 tags), reads the selected blobs' sorted IndexPoint keys
(AT_STAGE_BLOB_POINTS: blob index in bits 63:52) and the FitQuads records, and
reports per size class (the work-list classes of k_group, size_class()):
  - blobs and points;
  - the lane occupancy of the one-wave small-blob kernel's per-point phases: a blob of
    n points runs c = ceil(n / 64) points per lane, so n / (64 c) of the lane slots work;
  - for the large-blob teams (NT = 256 / 128 threads) the same with their NT.
Usage (GPU): python3 tools/blob_hist.py [out.json]
"""
import json
import torch  # noqa: F401  (one HIP runtime: torch first, as the library loader does)
import sys

import numpy as np

sys.path.insert(0, ".")
from ros_vision_amd.detector import GpuDetector, AT_FMT_YUYV  # noqa: E402
from ros_vision_amd.stream import stream_pool  # noqa: E402

W, H, POOL = 1280, 720, 64
EDGES = [(0, 64, "<=64"), (65, 128, "65-128"), (129, 256, "129-256"), (257, 512, "257-512"),
         (513, 1024, "513-1024"), (1025, 2048, "1025-2048"), (2049, 1 << 30, ">2048")]


def team_threads(n):
    """Threads of the team that fits an n-point blob (throughput-mode launches)."""
    if n <= 512:
        return 64
    if n <= 1024:
        return 128
    if n <= 4096:
        return 256
    return 512


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    frames = stream_pool(W, H, POOL, 15, 0)
    det = GpuDetector(W, H, max_batch=POOL, debug_taps=True)
    det.detect_batch(list(frames), AT_FMT_YUYV)
    sizes, records = [], 0
    for f in range(POOL):
        keys = det.copy_blob_points(f)
        bi = (keys >> np.uint64(52)).astype(np.int64)
        if bi.size:
            sizes.extend(np.bincount(bi)[np.unique(bi)].tolist())
        records += len(det.copy_quads(f))
    det.close()
    n = np.array(sizes, np.int64)
    rows = []
    for lo, hi, name in EDGES:
        m = n[(n >= lo) & (n <= hi)]
        if m.size == 0:
            rows.append(dict(cls=name, blobs=0, points=0))
            continue
        nt = np.array([team_threads(int(v)) for v in m])
        c = -(-m // nt)
        occ = m / (nt * c)
        rows.append(dict(cls=name, blobs=int(m.size), points=int(m.sum()), mean_points=round(float(m.mean()), 1),
                         team_threads=int(nt[0]), lane_occupancy_mean=round(float(occ.mean()), 3),
                         lane_occupancy_point_weighted=round(float((occ * m).sum() / m.sum()), 3)))
    small = n[n <= 512]
    occ_s = small / (64 * -(-small // 64))
    res = dict(workload="C2 stream pool 1280x720, 15 tags, %d frames, throughput mode" % POOL,
               frames=POOL, selected_blobs=int(n.size), fitquads_records=records,
               blobs_per_frame=round(n.size / POOL, 1), points_per_frame=round(float(n.sum()) / POOL, 1),
               small_blobs=int(small.size), small_mean_points=round(float(small.mean()), 1),
               small_lane_occupancy_mean=round(float(occ_s.mean()), 3),
               small_lane_occupancy_point_weighted=round(float((occ_s * small).sum() / small.sum()), 3),
               classes=rows,
               fine_histogram=dict(zip([str(int(e)) for e in np.arange(0, 544, 32)],
                                       np.histogram(small, bins=np.arange(0, 576, 32))[0].tolist())))
    text = json.dumps(res, indent=1)
    print(text)
    if out:
        with open(out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
