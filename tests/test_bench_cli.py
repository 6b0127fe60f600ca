"""bench.py's command line on the CPU: the headline defaults the GPU parity test of the
headline configuration imports (tests/test_stream_parity.py), and the helpers the
roofline and multi-GPU legs use."""
import bench


def test_headline_defaults():
    a = bench.parse([])
    assert (a.width, a.height, a.tags, a.pool) == (1280, 720, 15, 64)
    assert a.batch >= 1 and a.instances >= 1
    # at least 4 copies and two batches' worth of frames resident in HBM
    c = bench.pool_copies(a)
    assert c >= 4 and a.pool * c >= 2 * a.batch
    assert bench.pool_copies(bench.parse(["--hbm-copies", "2"])) == 2
    assert bench.DOMINANT in ("k_thr_ccl", "k_boundary", "k_blob_small", "k_blob", "k_extents", "k_decode")


def test_isolated_table_orders_by_span():
    st = {"frames": 2, "boundary_points": 1000, "ccl_listed_roots": 10, "small_blob_points": 500,
          "large_blob_points": 100}
    iso = {"k_thr_ccl": (0.2, 0.25, 10, st), "k_boundary": (0.3, 0.31, 10, st), "k_pairs": (0.01, 0.02, 10, st)}
    rows = bench.isolated_table(iso, 1280, 720)
    assert [r["kernel"] for r in rows] == ["k_boundary", "k_thr_ccl", "k_pairs"]
    kb = bench.kernel_algorithmic_bytes("k_boundary", st, 1280, 720)
    assert rows[0]["algorithmic_bytes_per_launch"] == kb
    assert abs(rows[0]["achieved"] - kb / 0.3e-3 / 1e9) < 1e-3
    assert rows[2]["frac"] is None  # (no algorithmic byte model for k_pairs)


def test_dominant_matches_committed_ablation():
    """DOMINANT is the top stage of the stage-cut ablation committed
    at bench.ABLATION (marginal ms per step of each stage at the bench configuration)."""
    marg, top = bench.ablation_marginals()
    assert top == bench.DOMINANT, marg
    assert set(marg) >= {"k_pre", "k_thr_ccl", "k_boundary", "k_blob_small", "k_blob", "k_decode"}
    assert all(v > -0.05 for v in marg.values()), marg


def test_ablation_marginals_parse(tmp_path):
    p = tmp_path / "abl.txt"
    p.write_text("pipe_stop=0 100 2.0 15\npipe_stop=1 9 0.1 0\npipe_stop=2 8 0.5 0\npipe_stop=3 7 0.6 0\n"
                 "pipe_stop=5 6 1.2 0\n")
    marg, top = bench.ablation_marginals(str(p))
    assert marg == {"k_pre": 0.1, "k_thr_ccl": 0.4, "k_ccl_merge": 0.1, "k_boundary": 0.6}
    assert top == "k_boundary"
