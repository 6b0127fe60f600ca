"""CPU tests of the oracle itself: pinned against the reference's own fixtures
and against independent re-derivations of the reference arithmetic."""
import math

import numpy as np
import pytest
from PIL import Image


def _real(golden_dir, name):
    return np.asarray(Image.open(golden_dir + "/" + name + "_y.png"))


def test_colorimage_detects_554(oracle_mod, golden_dir):
    """gpu_detector_test.cu:84-92 / :122-157: one detection, the printed id 554."""
    y = _real(golden_dir, "colorimage")
    o = oracle_mod.Oracle(y.shape[1], y.shape[0])
    assert o.detect(y, 2) == 1
    d = o.detections()[0]
    assert d["id"] == 554 and d["hamming"] == 0 and d["decision_margin"] > 50
    # outer black border seen in the image: TL(632,360) TR(914,345) BR(937,618) BL(659,642)
    expect = np.array([[659, 642], [937, 618], [914, 345], [632, 360]], float)
    assert np.max(np.abs(d["p"] - expect)) < 3.0


def test_grayimage_detects_585(oracle_mod, golden_dir):
    """Reference fixture test/data/grayimage.jpg: one printed tag captioned id 585."""
    y = _real(golden_dir, "grayimage")
    o = oracle_mod.Oracle(y.shape[1], y.shape[0])
    assert o.detect(y, 2) == 1
    d = o.detections()[0]
    assert d["id"] == 585 and d["hamming"] == 0 and d["decision_margin"] > 50
    # outer black border in the photograph: TL(432,170) TR(772,158) BR(787,504) BL(430,509)
    expect = np.array([[430, 509], [787, 504], [772, 158], [432, 170]], float)
    assert np.max(np.abs(d["p"] - expect)) < 3.0


def test_colorimage_notags(oracle_mod, golden_dir):
    """gpu_detector_test.cu:94-102: zero detections."""
    y = _real(golden_dir, "colorimage_notags")
    o = oracle_mod.Oracle(y.shape[1], y.shape[0])
    assert o.detect(y, 2) == 0


def _ref_unrank(i):
    """Literal transcription of Unrank/FindM0/FindM1/FindM2 (line_fit_filter.cu:613-728)."""
    def binom(n, k):
        return math.comb(n, k) if n >= k else 0
    cum = [sum(binom(10 - m0 - 1, 3) for m0 in range(0, j + 1)) for j in range(7)]
    bm1 = [binom(10 - 2 - j, 2) for j in range(7)]
    m0, last = 0, 0
    while True:
        nxt = cum[m0]
        if i < nxt:
            i -= last
            break
        last = nxt
        m0 += 1
    m1 = m0
    while True:
        nxt = bm1[m1]
        if i < nxt or m1 == 10 - 4:
            break
        i -= nxt
        m1 += 1
    m1 += 1
    m2 = m1
    while True:
        nxt = 10 - m2 - 1 - 1
        if i < nxt or m2 == 10 - 3:
            break
        i -= nxt
        m2 += 1
    m3 = m2 + i + 2
    return m0, m1, m2 + 1, m3


def test_unrank_is_lexicographic(oracle_mod):
    import ctypes as C
    L = oracle_mod.lib()
    combos = [(a, b, c, d) for a in range(10) for b in range(a + 1, 10) for c in range(b + 1, 10)
              for d in range(c + 1, 10)]
    assert len(combos) == 210
    for i, want in enumerate(combos):
        assert _ref_unrank(i) == want
        m = [C.c_int() for _ in range(4)]
        L.ao_unrank(i, *[C.byref(v) for v in m])
        assert tuple(v.value for v in m) == want


def test_deterministic_math_close_to_libm(oracle_mod):
    L = oracle_mod.lib()
    rng = np.random.default_rng(0)
    for _ in range(20000):
        y, x = (rng.normal(size=2) * 10 ** rng.uniform(-3, 3)).astype(np.float32)
        a = L.ao_det_atan2f(float(y), float(x))
        ref = math.atan2(float(y), float(x))
        assert abs(a - ref) <= 2.5e-7 * max(1.0, abs(ref))
    for _ in range(20000):
        t = float(np.float32(rng.uniform(-1.6, 1.6)))
        assert abs(L.ao_det_cosf(t) - math.cos(t)) < 1.2e-7
        assert abs(L.ao_det_sinf(t) - math.sin(t)) < 1.2e-7
    # hypot of integer gradients: truncation equals isqrt (W weights, apriltag_gpu.cu:656)
    for gx in range(-255, 256, 3):
        for gy in range(-255, 256, 7):
            assert int(L.ao_det_hypotf(float(gx), float(gy)) + np.float32(1.0)) == math.isqrt(gx * gx + gy * gy) + 1


def test_rotate90_matches_layout(oracle_mod):
    """rotate90 on the 3.x spiral layout == rotating the 6x6 cell grid by 90 degrees."""
    L = oracle_mod.lib()
    from ros_vision_amd.synth import BIT_X, BIT_Y
    rng = np.random.default_rng(3)
    for _ in range(50):
        code = int(rng.integers(0, 1 << 36))
        grid = np.zeros((8, 8), int)
        for i in range(36):
            grid[BIT_Y[i], BIT_X[i]] = (code >> (35 - i)) & 1
        r = L.ao_rotate90(code)
        g2 = np.zeros((8, 8), int)
        for i in range(36):
            g2[BIT_Y[i], BIT_X[i]] = (r >> (35 - i)) & 1
        assert any(np.array_equal(np.rot90(grid, k), g2) for k in (1, 3))


@pytest.mark.parametrize("family", ["tag25h9", "tag16h5"])
def test_rotate90_matches_layout_small_families(oracle_mod, family):
    """rotate90 (3.x, odd nbits keep the centre bit) == rotating the d x d grid."""
    L = oracle_mod.lib()
    from ros_vision_amd.synth import FAMILY_D, family_layout
    bx, by = family_layout(family)
    assert (bx, by) == oracle_mod.family_layout(family)
    d = FAMILY_D[family]
    n = d * d
    rng = np.random.default_rng(4)
    for _ in range(50):
        code = int(rng.integers(0, 1 << n))
        grid = np.zeros((d + 2, d + 2), int)
        for i in range(n):
            grid[by[i], bx[i]] = (code >> (n - 1 - i)) & 1
        r = L.ao_rotate90_n(code, n)
        g2 = np.zeros((d + 2, d + 2), int)
        for i in range(n):
            g2[by[i], bx[i]] = (r >> (n - 1 - i)) & 1
        assert any(np.array_equal(np.rot90(grid, k), g2) for k in (1, 3))


@pytest.mark.parametrize("family,frame", [("tag36h11", 0), ("tag36h11", 1), ("tag25h9", 0), ("tag16h5", 0)])
def test_synthetic_board_all_tags_found(oracle_mod, family, frame):
    from ros_vision_amd import synth
    codes = dict(oracle_mod.family_entries(family))
    yuyv_gray = synth.render_board(1280, 720, seed=766000 + frame, codes=codes, family=family)
    gray, truth = yuyv_gray
    o = oracle_mod.Oracle(1280, 720, family=family)
    o.detect(synth.to_yuyv(gray), 0)
    dets = o.detections()

    def dist(d, tc):
        # detection corners (p[0] = tag (-1, 1)) vs the rendered border corners (order-free;
        # apriltag corners wind the other way round from the renderer's)
        return min(np.max(np.abs(np.roll(pp, k, axis=0) - tc)) for k in range(4) for pp in (d["p"], d["p"][::-1]))

    if family != "tag16h5":
        assert sorted(d["id"] for d in dets) == sorted(t[0] for t in truth)
        for d in dets:
            assert dist(d, dict((t[0], t[1]) for t in truth)[d["id"]]) < 1.5
    else:
        # tag16h5 (minimum distance 5, 2 bits corrected) also decodes some quads of the
        # texture around the tags, as upstream does: every rendered tag is found at its
        # place, and the extra detections lie elsewhere
        for tid, tc in truth:
            assert any(d["id"] == tid and dist(d, tc) < 1.5 for d in dets)
        extra = [d for d in dets if not any(d["id"] == t and dist(d, tc) < 1.5 for t, tc in truth)]
        assert len(extra) == len(dets) - len(truth)


def test_cpu_oracle_stage_invariants(oracle_mod):
    """Structural invariants the reference guarantees at each stage."""
    from ros_vision_amd import synth
    codes = dict(oracle_mod.family_entries())
    gray, _ = synth.render_board(1280, 720, seed=5, codes=codes)
    o = oracle_mod.Oracle(1280, 720)
    o.detect(gray, 2)
    thr = o.thresholded()
    assert set(np.unique(thr)) <= {0, 127, 255}
    lab = o.labels()
    sizes = o.sizes()
    # labels are component roots: every live pixel's label carries the component's pixel count,
    # and a root label is the min node id, so it never exceeds the pixel's own node id
    # (fg node = top-left pixel of the 2x2 block, bg nodes = bottom-left / bottom-right pixel)
    live = thr != 127
    assert sizes.sum() == np.count_nonzero(live)
    assert np.all(sizes[lab[live]] > 0)
    H2, W2 = thr.shape
    rr, cc = np.mgrid[0:H2, 0:W2]
    fg_node = (rr // 2 * 2) * W2 + (cc // 2 * 2)
    bg_node = (rr // 2 * 2 + 1) * W2 + (cc // 2 * 2) + (cc % 2)
    node = np.where(thr == 255, fg_node, bg_node)
    assert np.all(lab[live] <= node[live])
    # sorted boundary points: rep01 non-decreasing (P2), rep0 < rep1
    p = o.sorted_points()
    r01 = p >> np.uint64(24)
    assert np.all(np.diff(r01.astype(np.int64)) >= 0)
    rep0 = (p >> np.uint64(24)) & np.uint64(0xfffff)
    rep1 = (p >> np.uint64(44)) & np.uint64(0xfffff)
    assert np.all(rep0 < rep1)
    # index points sorted by (blob, theta) (P6)
    ip = o.sorted_index_points() >> np.uint64(24)
    assert np.all(np.diff(ip.astype(np.int64)) >= 0)


def test_pair_capacity_keeps_the_first_4096_pairs(oracle_mod):
    """More blob pairs than the 12-bit blob index holds (points.h:183-193; the
    reference overflows its 2048-entry extents buffer, apriltag_gpu.cu:129,899-902):
    the first 4096 pairs in P2 rank order are processed, the rest dropped, the status
    is AT_E_CAPACITY and the kept pairs' tags are still detected."""
    from ros_vision_amd import synth
    codes = dict(oracle_mod.family_entries())
    yy, xx = np.mgrid[0:720, 0:1280]
    frame = np.where(((yy % 12) < 10) & ((xx % 12) < 10), 25, 230).astype(np.uint8)  # ~5,000 dark squares
    frame[:200] = synth.render_board(1280, 200, seed=17, ntags=5, side_range=(70, 90), codes=codes)[0]
    o = oracle_mod.Oracle(1280, 720)
    o.detect(frame, 2)
    assert o.status() == -3 and o.num_pairs() == 4096
    assert [d["id"] for d in o.detections()] == [434, 435, 436, 437, 438]
    ip = o.sorted_index_points()
    assert ip.size and int(ip.max() >> 52) <= 4095  # blob indices of the kept pairs only
    assert len(o.quads()) > 3000  # the kept squares still go through quad fitting
