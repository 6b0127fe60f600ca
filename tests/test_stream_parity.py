"""GPU parity of the exact configurations the bench reports.

* C2 headline: bench.py's own loop (ros_vision_amd.stream.StreamRunner) with
  its defaults imported from bench.py (instances, batch, HBM pool copies,
  DOMINANT) -- enqueue_device / collect round-robin over the 64-frame C2 pool in
  HBM, hipGraph replay, then again with the live kernel timer on the dominant
  kernel (the split graphs of the timed region).
  Every frame of every batch is compared with the committed oracle goldens.
* C4 geometry in throughput mode: 8 1920x1080 frames, max_batch 8 (the
  throughput-mode kernels), stage-by-stage against the live oracle and against
  the goldens.

Reference test this mirrors: test/gpu_detector_test.cu:122-157 (CpuAndGpuEqual),
tightened to bit-exact ids / integer corners and 1e-4 on floats.
"""
import numpy as np
import pytest

from parity_util import compare_detections, compare_frame, compare_with_stream_golden, load_stream_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2():
    import make_stream_golden as mg
    g = load_stream_golden("c2")
    frames = mg.c2_frames(dict(__import__("ros_vision_amd").family_entries()))
    assert [mg.digest(f) for f in frames] == list(g["frame_digest"]), "C2 pool renders differently"
    return g, frames


def test_bench_headline_configuration(c2):
    """bench.py's headline configuration exactly: its defaults (instances, batch, the HBM
    pool copies, the kernel timer on DOMINANT) are imported from bench.py, so a changed
    bench default changes what this test runs.  8 batches with graph replay, then 8
    under the live kernel timer (the launch sequence as three graphs cut around the
    timed kernel -- the bench's timed region); every frame of every batch against the
    oracle goldens."""
    import torch

    import bench
    import make_stream_golden as mg
    import ros_vision_amd as rva
    from ros_vision_amd.stream import StreamRunner
    g, frames = c2
    args = bench.parse([])
    instances, B, copies, timed = args.instances, args.batch, bench.pool_copies(args), bench.DOMINANT
    assert (args.width, args.height, args.tags, args.pool) == (1280, 720, 15, frames.shape[0])
    pool = frames.shape[0]
    d_frames = torch.from_numpy(frames).to("cuda").repeat(copies, 1, 1).contiguous()
    stride = frames[0].nbytes
    dets = [rva.GpuDetector(1280, 720, max_batch=B) for _ in range(instances)]
    runner = StreamRunner(dets, d_frames.data_ptr(), stride, pool * copies, B)
    seen = {"frames": 0, "dets": 0}
    bad = []

    def check(det, step, off):
        res = det.results()
        for j in range(B):
            f = (off + j) % pool
            assert det.frame_status(j) == 0
            bad.extend(compare_with_stream_golden(g, f, res[j], det.poses(j)))
            seen["dets"] += len(res[j])
        seen["frames"] += B

    n = runner.run(8, 0, on_batch=check)
    assert bad == [], bad[:10]
    assert seen["frames"] == 8 * B and n == seen["dets"] == 8 * B * 15
    # the timed region of the bench: the kernel timer splits the graph around its kernel
    for d in dets:
        d.set_kernel_timer(timed)
    n = runner.run(8, 8, on_batch=check)
    assert bad == [], bad[:10]
    assert seen["frames"] == 16 * B and n == 8 * B * 15
    per = 8 // instances
    assert all(ms > 0 and launches == per for ms, launches in (d.kernel_time() for d in dets))
    assert all(ms > 0 and launches == per for ms, launches in (d.kernel_span() for d in dets))
    for d in dets:
        d.set_kernel_timer(None)
    # intermediate planes of each instance's last batch: threshold + labels bit-exact
    for d in dets[:2]:
        off = runner.offset(12 + dets.index(d))
        for j in (0, 1, B - 1):
            f = (off + j) % pool
            assert mg.digest(d.copy_thresholded(j)) == g["thr_digest"][f]
            assert mg.digest(d.copy_union_markers(j)) == g["labels_digest"][f]
            assert d.num_pairs(j) == g["num_pairs"][f]


def test_c4_1080p_throughput_mode(oracle_mod):
    """1920x1080, 24 tags, max_batch 8 (throughput-mode kernels: 64-wide CCL tiles,
    k_ccl_merge + k_boundary<true>, k_extents for every candidate, 256-thread
    large-blob teams), frames resident in HBM."""
    import torch

    import make_stream_golden as mg
    import ros_vision_amd as rva
    g = load_stream_golden("c4")
    frames = mg.c4_frames(dict(rva.family_entries()))
    assert [mg.digest(f) for f in frames] == list(g["frame_digest"])
    t = torch.from_numpy(frames).cuda()
    det = rva.GpuDetector(1920, 1080, max_batch=8, debug_taps=True)
    res = det.detect_device(t.data_ptr(), frames[0].nbytes, 8)
    for f in range(8):
        assert compare_with_stream_golden(g, f, res[f], det.poses(f)) == []
        orc = oracle_mod.Oracle(1920, 1080)
        orc.detect(frames[f], 0)
        assert compare_frame(det, orc, frame_idx=f) == []
        assert compare_detections(res[f], orc.detections()) == []


def test_bench_1080p_configuration():
    """configs[3]'s per-GPU workload at the bench's own settings:
    1920x1080, the batch, instances, HBM pool copies and DOMINANT kernel timer that
    `bench.py --width 1920 --height 1080 --tags 24` uses (imported from bench.py), so
    the 1080p throughput kernels (CAP-8192 teams for the blobs over 4096 points, the
    mid-size 128-thread teams, k_ccl_merge at 1080p) run at B = 192 with four batches
    in flight, graph replay then the split timer graphs.  The 8 C4 golden frames are
    tiled to a 64-frame pool; every frame of every batch against the goldens."""
    import torch

    import bench
    import make_stream_golden as mg
    import ros_vision_amd as rva
    from ros_vision_amd.stream import StreamRunner
    g = load_stream_golden("c4")
    frames8 = mg.c4_frames(dict(rva.family_entries()))
    assert [mg.digest(f) for f in frames8] == list(g["frame_digest"])
    args = bench.parse(["--width", "1920", "--height", "1080", "--tags", "24"])
    instances, B, copies, timed = args.instances, args.batch, bench.pool_copies(args), bench.DOMINANT
    assert B >= 128 and instances >= 2
    pool = args.pool
    frames = np.concatenate([frames8] * (pool // 8))
    d_frames = torch.from_numpy(frames).to("cuda").repeat(copies, 1, 1).contiguous()
    stride = frames[0].nbytes
    dets = [rva.GpuDetector(1920, 1080, max_batch=B) for _ in range(instances)]
    runner = StreamRunner(dets, d_frames.data_ptr(), stride, pool * copies, B)
    bad, seen = [], {"frames": 0, "dets": 0}
    want = int(np.sum(g["ndet"][:8]))

    def check(det, step, off):
        res = det.results()
        for j in range(B):
            f = (off + j) % 8
            assert det.frame_status(j) == 0
            bad.extend(compare_with_stream_golden(g, f, res[j], det.poses(j)))
            seen["dets"] += len(res[j])
        seen["frames"] += B

    n1 = runner.run(instances, 0, on_batch=check)
    assert bad == [], bad[:10]
    for d in dets:
        d.set_kernel_timer(timed)
    n2 = runner.run(instances, instances, on_batch=check)
    assert bad == [], bad[:10]
    assert all(launches == 1 for _, launches in (d.kernel_span() for d in dets))
    for d in dets:
        d.set_kernel_timer(None)
    assert seen["frames"] == 2 * instances * B and n1 + n2 == seen["dets"] == 2 * instances * B // 8 * want > 0


def test_host_ingest_loop(c2):
    """bench.py's host_ingest leg: the same round-robin loop fed from page-locked
    host frames through at_enqueue_host (H2D copies on the detector streams, runs of
    back-to-back frames in one 2-D copy, batches wrapping the pool)."""
    import torch

    import ros_vision_amd as rva
    from ros_vision_amd.stream import StreamRunner
    g, frames = c2
    pinned = torch.from_numpy(frames).pin_memory()
    B = 48  # batches wrap the 64-frame pool: two copy runs per batch
    dets = [rva.GpuDetector(1280, 720, max_batch=B) for _ in range(3)]
    runner = StreamRunner(dets, pinned.data_ptr(), frames[0].nbytes, frames.shape[0], B, host=True)
    bad, seen = [], []

    def check(det, step, off):
        res = det.results()
        for j in range(B):
            bad.extend(compare_with_stream_golden(g, (off + j) % frames.shape[0], res[j], det.poses(j)))
        seen.append(step)

    runner.run(5, 0, on_batch=check)
    assert bad == [] and seen == [0, 1, 2, 3, 4]
