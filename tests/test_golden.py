"""The oracle reproduces the committed golden vectors (tools/make_golden_vectors.py)."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VEC = json.load(open(os.path.join(ROOT, "tests", "golden", "vectors.json")))


@pytest.mark.parametrize("name", sorted(VEC))
def test_oracle_reproduces_golden(name):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_golden_vectors as mg
    case = {c[0]: c[1:] for c in mg.cases()}[name]
    got = mg.run_case(*case)
    assert VEC[name].get("family", "tag36h11") == case[4]
    want = VEC[name]
    for k in got:
        assert got[k] == want[k], k


def test_reference_fixture_expectations():
    """gpu_detector_test.cu:84-102: id 554 on colorimage, nothing on colorimage_notags."""
    assert [d["id"] for d in VEC["colorimage"]["detections"]] == [554]
    assert VEC["colorimage_notags"]["detections"] == []
    assert [d["id"] for d in VEC["grayimage"]["detections"]] == [585]
    # natural outdoor frames of the reference's game-piece data: quads, no tags
    for name in ("frc_rebuilt_frame1", "frc_reefscape_frame6141"):
        assert VEC[name]["detections"] == [] and VEC[name]["quads"] > 0
    assert [d["id"] for d in VEC["c1_640x480"]["detections"]] == [0, 1, 2, 554]
