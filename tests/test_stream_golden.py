"""CPU: the committed goldens of the bench's workloads (tests/golden/stream_*.npz)
are what the oracle gives on the frames the bench renders (re-rendered and
re-detected here, tools/make_stream_golden.py)."""
import numpy as np
import pytest


@pytest.mark.parametrize("name", ["c2", "c4"])
def test_stream_golden_reproduces(oracle_mod, name):
    import make_stream_golden as mg
    from parity_util import load_stream_golden
    want = load_stream_golden(name)
    got = mg.build(name)
    for k, v in got.items():
        if k.startswith("det_") and v.dtype.kind == "f":
            assert np.array_equal(v, want[k]), k  # same oracle, same inputs: bit-identical
        else:
            assert np.array_equal(np.asarray(v), want[k]), k
    # the stream is what the bench claims: 15 detections per C2 frame, ids 10f..10f+14 mod 587
    if name == "c2":
        assert list(want["ndet"]) == [15] * 64
        for f in range(64):
            a, b = want["_start"][f], want["_start"][f + 1]
            assert sorted(want["det_id"][a:b]) == sorted((10 * f + j) % 587 for j in range(15))
