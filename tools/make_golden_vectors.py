"""Generate tests/golden/vectors.json: oracle outputs on the committed inputs.

Inputs are the reference's own fixtures (tests/golden/*_y.png, decoded from
test/data/*.jpg by tools/make_golden_images.py) and seeded synthetic boards
(ros_vision_amd/synth.py).  Per case we store per-stage digests (threshold
plane, labels, sizes, sorted boundary points, sorted index points), counts and
the final detections.  tests/test_golden.py checks the oracle still reproduces
them and tests/test_gpu_parity.py checks the HIP path against them.
"""
import hashlib
import json
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ao  # noqa: E402
from ros_vision_amd import synth  # noqa: E402


def cases():
    codes = dict(ao.family_entries())
    g = os.path.join(ROOT, "tests", "golden")
    T = "tag36h11"
    yield "colorimage", 1920, 1080, 2, np.asarray(Image.open(g + "/colorimage_y.png")), T
    yield "colorimage_notags", 1920, 1080, 2, np.asarray(Image.open(g + "/colorimage_notags_y.png")), T
    yield "grayimage", 1280, 800, 2, np.asarray(Image.open(g + "/grayimage_y.png")), T
    yield "frc_rebuilt_frame1", 1920, 1080, 2, np.asarray(Image.open(g + "/frc_rebuilt_frame1_y.png")), T
    yield "frc_reefscape_frame6141", 640, 640, 2, np.asarray(Image.open(g + "/frc_reefscape_frame6141_y.png")), T
    yield "c1_640x480", 640, 480, 0, synth.to_yuyv(synth.render_board(640, 480, seed=766, ntags=4,
                                                                       ids=[0, 1, 2, 554], codes=codes)[0]), T
    for f in (0, 1, 2, 30, 44, 58):  # ids 10f..10f+14 mod 587 across the family
        yield "c2_720p_f%d" % f, 1280, 720, 0, synth.stream_frame(1280, 720, f, codes=codes)[0], T
    yield "c4_1080p", 1920, 1080, 0, synth.to_yuyv(synth.render_board(1920, 1080, seed=4242, ntags=24,
                                                                       codes=codes)[0]), T
    # more tags than the former 128-detection cap, ids 400.. across the wrap to 0..
    yield "dense_1080p_160tags", 1920, 1080, 0, synth.to_yuyv(synth.render_board(
        1920, 1080, seed=9160, ntags=160, side_range=(50, 64), ids=[(400 + j) % 587 for j in range(160)],
        codes=codes)[0]), T
    # more accepted quads than the former 512-quad decode queue
    yield "dots_1080p", 1920, 1080, 2, synth.render_dots(1920, 1080, seed=9512)[0], T
    # geometries whose decimated plane is not a multiple of the CCL / boundary tiles
    # (800x600: the deployed camera of system_config.json:21-25, W/2 = 400, H/2 = 300),
    # with tags and blobs flush against the right and bottom borders
    for (W, H, fmt) in ((800, 600, 2), (1000, 600, 0), (648, 488, 0), (1352, 760, 2)):
        g8 = synth.render_edge_board(W, H, seed=W + H, codes=codes)[0]
        yield "edge_%dx%d" % (W, H), W, H, fmt, (g8 if fmt == 2 else synth.to_yuyv(g8)), T
    # the other classic families (apriltag_utils.cu:13-16): every code of the family on
    # two 720p boards (tag16h5 also decodes texture quads, as upstream does)
    for fam, n in (("tag25h9", 35), ("tag16h5", 30)):
        fc = dict(ao.family_entries(fam))
        for k, ids in enumerate((list(range(0, 18)), list(range(18, n)))):
            yield "%s_720p_%d" % (fam, k), 1280, 720, 0, synth.to_yuyv(synth.render_board(
                1280, 720, seed=7250 + 10 * len(fam) + k, ntags=len(ids), ids=ids, codes=fc, family=fam)[0]), fam


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:24]


def run_case(W, H, fmt, frame, family="tag36h11"):
    o = ao.Oracle(W, H, family=family)
    o.detect(frame, fmt)
    pts = o.sorted_points()
    return {
        "thr": digest(o.thresholded()), "labels": digest(o.labels()), "sizes": digest(o.sizes()),
        "points_sorted": digest(np.sort(pts)), "num_points": int(pts.size), "num_pairs": o.num_pairs(),
        "index_points": digest(o.sorted_index_points()), "num_index_points": int(o.sorted_index_points().size),
        "valid_fitquads": sum(int(f.valid) for f in o.fitquads()), "quads": len(o.quads()),
        "detections": [{"id": d["id"], "hamming": d["hamming"], "decision_margin": float(d["decision_margin"]),
                        "c": d["c"].tolist(), "p": d["p"].tolist(), "H": d["H"].ravel().tolist()}
                       for d in o.detections()],
    }


if __name__ == "__main__":
    out = {}
    for name, W, H, fmt, frame, family in cases():
        out[name] = dict(width=W, height=H, fmt=fmt, family=family, **run_case(W, H, fmt, frame, family))
        print(name, [d["id"] for d in out[name]["detections"]])
    json.dump(out, open(os.path.join(ROOT, "tests", "golden", "vectors.json"), "w"), indent=1)
