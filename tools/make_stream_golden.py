"""Generate the oracle goldens of the bench's own workloads (tests/golden/stream_*.npz).

stream_c2.npz   -- the 64-frame config C2 pool bench.py renders on rank 0
                   (ros_vision_amd.stream.stream_pool: 1280x720, 15 tags, YUYV)
stream_c4.npz   -- 8 config C4 frames (1920x1080, 24 tags, seeds 4300 + i)

Per frame: a digest of the frame bytes (the GPU test re-renders the pool and
checks it is the same input), of the threshold and label planes, the pair count
and the oracle's detections {id, hamming, decision_margin, H, c, p} with the
oracle pose of each (estimate_tag_pose; e1/e2 are the errors of the two minima,
equal ones make the choice ambiguous).  tests/test_stream_golden.py (CPU)
re-derives them with the oracle; tests/test_stream_parity.py (GPU) compares the
HIP path, run exactly as the bench runs it, with them.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ao  # noqa: E402
from ros_vision_amd import synth  # noqa: E402
from ros_vision_amd.detector import TEST_CAMERA  # noqa: E402
from ros_vision_amd.stream import stream_pool  # noqa: E402

C2 = dict(width=1280, height=720, pool=64, tags=15)
C4 = dict(width=1920, height=1080, frames=8, tags=24)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:24]


def c2_frames(codes=None):
    codes = codes if codes is not None else dict(ao.family_entries())
    return stream_pool(C2["width"], C2["height"], C2["pool"], C2["tags"], 0, codes=codes)


def c4_frames(codes=None):
    codes = codes if codes is not None else dict(ao.family_entries())
    out = np.empty((C4["frames"], C4["height"], 2 * C4["width"]), np.uint8)
    for i in range(C4["frames"]):
        out[i] = synth.to_yuyv(synth.render_board(C4["width"], C4["height"], seed=4300 + i, ntags=C4["tags"],
                                                  codes=codes)[0])
    return out


def oracle_golden(frames, W, H):
    cam = TEST_CAMERA
    o = ao.Oracle(W, H)
    g = {k: [] for k in ("frame_digest", "thr_digest", "labels_digest", "num_pairs", "status", "ndet")}
    dets = {k: [] for k in ("frame", "id", "hamming", "margin", "H", "c", "p", "R", "t", "err", "e1", "e2")}
    for f in range(frames.shape[0]):
        o.detect(frames[f], 0)
        g["frame_digest"].append(digest(frames[f]))
        g["thr_digest"].append(digest(o.thresholded()))
        g["labels_digest"].append(digest(o.labels()))
        g["num_pairs"].append(o.num_pairs())
        g["status"].append(o.status())
        dl = o.detections()
        g["ndet"].append(len(dl))
        for d in dl:
            R, t, err, (e1, e2), _ = ao.estimate_tag_pose(d["H"], d["p"], cam.fx, cam.fy, cam.cx, cam.cy)
            for k, v in (("frame", f), ("id", d["id"]), ("hamming", d["hamming"]),
                         ("margin", d["decision_margin"]), ("H", np.ravel(d["H"])), ("c", d["c"]),
                         ("p", np.ravel(d["p"])), ("R", np.ravel(R)), ("t", np.ravel(t)), ("err", err),
                         ("e1", e1), ("e2", e2)):
                dets[k].append(v)
    out = {k: np.array(v) for k, v in g.items()}
    out.update({"det_" + k: np.array(v) for k, v in dets.items()})
    out["width"], out["height"] = np.int32(W), np.int32(H)
    return out


def build(name):
    ao.build()
    if name == "c2":
        return oracle_golden(c2_frames(), C2["width"], C2["height"])
    return oracle_golden(c4_frames(), C4["width"], C4["height"])


def path(name):
    return os.path.join(ROOT, "tests", "golden", "stream_%s.npz" % name)


if __name__ == "__main__":
    for name in sys.argv[1:] or ["c2", "c4"]:
        g = build(name)
        np.savez_compressed(path(name), **g)
        print(name, "frames", g["frame_digest"].size, "detections", g["det_id"].size,
              "bytes", os.path.getsize(path(name)))
