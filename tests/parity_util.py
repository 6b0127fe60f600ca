"""Helpers comparing the HIP path (C ABI) with the CPU oracle stage by stage."""
import numpy as np


def compare_frame(det, orc, frame_idx=0, check_points=True):
    """Returns a list of mismatch descriptions (empty == bit-identical)."""
    bad = []
    for name, a, b in [("gray", det.copy_gray(frame_idx), orc.gray()),
                       ("decimated", det.copy_decimated(frame_idx), orc.decimated()),
                       ("threshold", det.copy_thresholded(frame_idx), orc.thresholded()),
                       ("labels", det.copy_union_markers(frame_idx), orc.labels()),
                       ("sizes", det.copy_union_markers_size(frame_idx), orc.sizes())]:
        if a.shape != b.shape or not np.array_equal(a, b):
            nd = int(np.count_nonzero(a != b)) if a.shape == b.shape else -1
            bad.append("%s differs at %d positions" % (name, nd))
            return bad  # later stages depend on these
    if check_points:
        gp = np.sort(det.copy_points(frame_idx))
        op = np.sort(orc.sorted_points())
        if not np.array_equal(gp, op):
            bad.append("boundary points differ: gpu %d oracle %d" % (gp.size, op.size))
            return bad
    if det.num_pairs(frame_idx) != orc.num_pairs():
        bad.append("pairs %d vs %d" % (det.num_pairs(frame_idx), orc.num_pairs()))
    gb = det.copy_blob_points(frame_idx)
    ob = orc.sorted_index_points()
    if gb.shape != ob.shape or not np.array_equal(gb, ob):
        nd = int(np.count_nonzero(gb != ob)) if gb.shape == ob.shape else -1
        bad.append("selected blob points differ (gpu %d oracle %d, %d mismatches)" % (gb.size, ob.size, nd))
    gq = [q for q in det.copy_quads(frame_idx) if q["valid"]]
    oq = [f for f in orc.fitquads() if f.valid]
    gqi = [(q["blob_index"], tuple(q["indices"])) for q in gq]
    oqi = [(int(f.blob_index), tuple(int(v) for v in f.indices)) for f in oq]
    if gqi != oqi:
        bad.append("valid fit quads differ: %s vs %s" % (gqi[:5], oqi[:5]))
    # corners bit for bit; a NaN corner (a degenerate line fit: both sides accept the
    # quad, UpdateFitQuads' area test is false on NaN) compares by NaN-ness, not by
    # its payload (the GPU's default NaN is positive, x86's negative)
    def canon(c):
        c = np.asarray(c, np.float32)
        return np.where(np.isnan(c), np.float32(np.nan), c).tobytes()
    ga = [(q["blob_index"], canon(q["corners"])) for q in det.copy_quads(frame_idx) if q["accepted"]]
    oa = [(b, canon(c)) for c, b in orc.quads()]
    if ga != oa:
        bad.append("accepted quad corners differ (%d vs %d)" % (len(ga), len(oa)))
    return bad


def compare_detections(gd, od, tol=1e-4):
    bad = []
    if [d.id for d in gd] != [d["id"] for d in od]:
        return ["ids differ: %s vs %s" % ([d.id for d in gd], [d["id"] for d in od])]
    for a, b in zip(gd, od):
        if a.hamming != b["hamming"]:
            bad.append("hamming id %d" % a.id)
        if abs(a.decision_margin - b["decision_margin"]) > tol:
            bad.append("margin id %d %r vs %r" % (a.id, a.decision_margin, b["decision_margin"]))
        for nm, x, y in [("H", a.H, b["H"]), ("c", a.c, b["c"]), ("p", a.p, b["p"])]:
            if not np.allclose(x, y, rtol=0, atol=tol):
                bad.append("%s id %d max diff %g" % (nm, a.id, float(np.max(np.abs(x - y)))))
            if not np.array_equal(np.floor(x), np.floor(y)) and nm != "H":
                bad.append("integer %s id %d differ" % (nm, a.id))
    return bad


# ---- goldens of the bench's own workloads (tools/make_stream_golden.py) --------

def load_stream_golden(name):
    """tests/golden/stream_<name>.npz as a dict of arrays, plus per-frame slices."""
    import os
    g = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "stream_%s.npz" % name)))
    starts = np.concatenate([[0], np.cumsum(g["ndet"])])
    g["_start"] = starts
    return g


def compare_with_stream_golden(g, f, dets, poses=None, tol=1e-4):
    """Detections (and poses) of golden frame f: ids / hamming exact, integer parts of
    c and p equal, margin / H / c / p (and pose R, t) within tol.  Poses whose two
    minima have equal error are skipped (either is estimate_tag_pose's answer)."""
    bad = []
    a, b = int(g["_start"][f]), int(g["_start"][f + 1])
    ids = [int(v) for v in g["det_id"][a:b]]
    if [d.id for d in dets] != ids:
        return ["frame %d ids differ: %s vs %s" % (f, [d.id for d in dets], ids)]
    for k, d in enumerate(dets):
        i = a + k
        if d.hamming != int(g["det_hamming"][i]):
            bad.append("frame %d id %d hamming" % (f, d.id))
        if abs(d.decision_margin - float(g["det_margin"][i])) > tol:
            bad.append("frame %d id %d margin %r vs %r" % (f, d.id, d.decision_margin, float(g["det_margin"][i])))
        for nm, x, y in (("H", d.H.ravel(), g["det_H"][i]), ("c", d.c, g["det_c"][i]),
                         ("p", d.p.ravel(), g["det_p"][i])):
            if not np.allclose(x, y, rtol=0, atol=tol):
                bad.append("frame %d id %d %s max diff %g" % (f, d.id, nm, float(np.max(np.abs(x - y)))))
            if nm != "H" and not np.array_equal(np.floor(x), np.floor(y)):
                bad.append("frame %d id %d integer %s differ" % (f, d.id, nm))
    if poses is not None:
        if [p.id for p in poses] != ids:
            return bad + ["frame %d pose ids differ" % f]
        for k, p in enumerate(poses):
            i = a + k
            e1, e2 = float(g["det_e1"][i]), float(g["det_e2"][i])
            if abs(e1 - e2) <= 1e-9 * max(e1, e2, 1e-30):
                continue
            if (np.abs(p.R.ravel() - g["det_R"][i]).max() > tol or np.abs(p.t - g["det_t"][i]).max() > tol):
                bad.append("frame %d id %d pose differs" % (f, p.id))
    return bad
