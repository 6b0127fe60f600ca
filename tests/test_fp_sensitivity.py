"""Sensitivity of the integer decisions to one-ulp differences in atan2f / hypotf /
cosf / sinf (tools/fp_sensitivity.py, committed counts in
tests/golden/fp_sensitivity.json).

The HIP kernels and the oracle share one fixed sequence for these functions
(at_detmath.h), so GPU-vs-oracle parity is bit-exact by construction; the
reference uses CUDA's libdevice.  Under a faithful-libm model (inexact results
within one ulp, exact ones exact) no FitQuad argmin and no integer corner pixel
changes on any golden case; detection corners move by at most one float ulp.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

CASES = ["colorimage", "c2_720p_f0", "dense_1080p_160tags"]


@pytest.fixture(scope="module")
def committed():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "fp_sensitivity.json")))


def test_counts_reproduce(oracle_mod, committed):
    import fp_sensitivity as fs
    import make_golden_vectors as mg
    cases = {c[0]: c[1:5] for c in mg.cases() if c[0] in CASES}
    try:
        for name in CASES:
            W, H, fmt, frame = cases[name]
            oracle_mod.set_fp_perturb(0)
            base = fs.snapshot(W, H, fmt, frame)
            for cname, mask in fs.CONFIGS:
                oracle_mod.set_fp_perturb(mask)
                got = fs.diff(base, fs.snapshot(W, H, fmt, frame))
                want = committed["cases"][name][cname]
                for k, v in want.items():
                    assert got[k] == pytest.approx(v, rel=0, abs=1e-12), (name, cname, k)
    finally:
        oracle_mod.set_fp_perturb(0)


def test_faithful_libm_keeps_integer_outputs(committed):
    tot = committed["totals"]
    for cname in [c for c in tot if c.endswith("_inexact")]:
        assert tot[cname]["quad_indices"] == 0, cname
        assert tot[cname]["det_integer_corner_changes"] == 0, cname
        assert tot[cname]["det_corner_max_px"] < 2.5e-4, cname  # <= 2 float ulps at x < 2048
        assert tot[cname]["theta_order"] <= 1e-4 * tot["index_points"], cname


def test_line_fit_weight_is_integer_sqrt_plus_one():
    """k_extents / the fused blob paths compute TransformLineFitPoint's weight
    (int)(hypotf(gx, gy) + 1) -- hypotf as (float)sqrt((double)gx^2 + (double)gy^2), the
    oracle's det_hypotf -- as floor(sqrt(gx^2 + gy^2)) + 1 with an integer square root
    (lf_weight, at_kernels.hip).  Exhaustive over the byte differences the gradient takes."""
    import numpy as np
    g = np.arange(-255, 256, dtype=np.int64)
    s = (g[:, None] ** 2 + g[None, :] ** 2).ravel()
    ref = np.trunc(np.sqrt(s.astype(np.float64)).astype(np.float32) + np.float32(1.0)).astype(np.int64)
    r = np.floor(np.sqrt(s.astype(np.float64))).astype(np.int64)
    r -= (r * r > s)
    r += ((r + 1) * (r + 1) <= s)
    assert np.array_equal(ref, r + 1)
