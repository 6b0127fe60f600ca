"""world_size-2 gloo tests of the multi-GPU data path (CPU, no GPU needed).

The detector on each rank is stood in for by the CPU oracle (test harness
only); what is under test is the sharding, the frame scatter from rank 0, the
fixed-size detection records and the gather back to rank 0, plus the bench's
max/sum timing reduction.
"""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, nper, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist
    import ao
    from ros_vision_amd import multigpu, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    codes = dict(ao.family_entries())
    src = None
    if rank == 0:
        frames = np.stack([synth.to_yuyv(synth.render_board(W, H, seed=100 + i, ntags=4, codes=codes)[0])
                           for i in range(world * nper)])
        src = torch.from_numpy(frames)
    mine = multigpu.scatter_frames(dist, src, nper, (H, 2 * W), "cpu").numpy()
    o = ao.Oracle(W, H)
    recs = []
    for f in mine:
        o.detect(f, 0)
        recs.append(multigpu.detection_records(o.detections()))
    # the bench's record path: 2 records per frame in the fixed-size row, the rest overflow
    rows, counts, over = multigpu.split_records(recs, 2)
    g = multigpu.RecordGather(dist, nper, 2 * multigpu._rec_size(), "cpu")
    g.post(0, torch.from_numpy(rows), torch.from_numpy(counts), over)
    allp = None
    if rank == 0:
        allp = recs + [b for r in range(1, world) for b in g.frames(0)[r]]
    g.drain()
    el, cnt = multigpu.reduce_max_sum(dist, 1.0 + rank, float(counts.sum()), "cpu")
    if rank == 0:
        q.put((allp, el, cnt))
    dist.barrier()
    dist.destroy_process_group()


def test_scatter_detect_gather_world2(oracle_mod):
    from ros_vision_amd import multigpu, synth
    W, H, nper, world = 320, 240, 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, nper, q)) for r in range(world)]
    for p in procs:
        p.start()
    allp, el, cnt = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert el == 2.0  # max over ranks
    codes = dict(oracle_mod.family_entries())
    o = oracle_mod.Oracle(W, H)
    total = 0
    for i in range(world * nper):
        o.detect(synth.to_yuyv(synth.render_board(W, H, seed=100 + i, ntags=4, codes=codes)[0]), 0)
        want = o.detections()
        got = multigpu.records_to_dicts(allp[i])
        total += len(want)
        assert len(want) > 2  # (every frame goes through the overflow message)
        assert [d["id"] for d in got] == [d["id"] for d in want]
        for a, b in zip(got, want):
            assert np.array_equal(a["p"], b["p"]) and np.array_equal(a["H"], b["H"])
    assert cnt == total


def test_shard_range_covers_all():
    from ros_vision_amd.multigpu import shard_range
    for world in (1, 2, 4, 8):
        for n in (1, 7, 8, 64):
            seen = []
            for r in range(world):
                lo, hi = shard_range(r, world, n)
                seen.extend(range(lo, hi))
            assert seen == list(range(n))


def _ingest_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from ros_vision_amd import multigpu
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, npool, shape = 2, 6, (4, 8)
    pool = None
    if rank == 0:  # frame (r, i) is filled with 16*r + i
        pool = torch.stack([torch.stack([torch.full(shape, 16 * r + i, dtype=torch.uint8) for i in range(npool)])
                            for r in range(world)])
    ing = multigpu.ScatterIngest(dist, pool, B, shape, "cpu")
    got = []
    ing.start(0)
    for s in range(5):
        buf = ing.ready(s)
        got.append([int(buf[k, 0, 0]) for k in range(B)])
        if s + 1 < 5:
            ing.start(s + 1)
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_scatter_ingest_double_buffer_world2():
    """bench.py --ingest scatter: step s delivers rank r the frames (r, s*B mod npool ...)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ingest_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    B, npool = 2, 6
    for r in range(world):
        want = []
        for s in range(5):
            off = (s * B) % npool
            want.append([16 * r + off + k for k in range(B)])
        assert res[r] == want


def _gather_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from ros_vision_amd import multigpu
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, cap = 3, 2
    g = multigpu.RecordGather(dist, B, cap * multigpu._rec_size(), "cpu")
    got = []
    for s in range(5):  # step s: frame f of rank r has r + s + f detections, ids 1000 r + 100 s + k
        recs = [multigpu.detection_records(_fake_dets(rank, s, f)) for f in range(B)]
        rows, counts, over = multigpu.split_records(recs, cap)
        g.post(s, torch.from_numpy(rows), torch.from_numpy(counts), over)
        if s >= 1 and rank == 0:  # results of the previous step (double buffered)
            got.append({r: [[d["id"] for d in multigpu.records_to_dicts(b)] for b in fr]
                        for r, fr in g.frames(s - 1).items()})
    if rank == 0:
        got.append({r: [[d["id"] for d in multigpu.records_to_dicts(b)] for b in fr] for r, fr in g.frames(4).items()})
    g.drain()
    q.put((rank, got, g.records_received))
    dist.barrier()
    dist.destroy_process_group()


def _fake_dets(rank, step, frame):
    n = rank + step + frame
    return [dict(id=1000 * rank + 100 * step + k, hamming=k % 3, decision_margin=50.0 + k, H=np.eye(3) * k,
                 c=np.array([k, 2.0 * k]), p=np.full((4, 2), 0.5 * k)) for k in range(n)]


def test_record_gather_world3():
    """bench.py --ingest scatter: detection records of ranks 1..N-1 reach rank 0 by
    point-to-point sends (rank 0's own never move), double-buffered over steps; frames
    with more records than the fixed-size row holds send the rest in the overflow
    message (0 .. 8 records per frame against a row of 2)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (got, n) for r, got, n in (q.get(timeout=300) for _ in range(world))}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    got, nrec = res[0]
    assert len(got) == 5
    for s, step in enumerate(got):
        assert sorted(step) == [1, 2]
        for r in (1, 2):
            assert step[r] == [[d["id"] for d in _fake_dets(r, s, f)] for f in range(3)]
    assert nrec == sum(r + s + f for r in (1, 2) for s in range(5) for f in range(3))


def _dense_worker(rank, world, port, q):
    """Rank 1 holds a batch of the oracle's detections of the 160-tag 1080p board (131
    per frame) and of a 15-tag C2 frame, packed as bench.py packs them (rec_cap 32 in
    the fixed-size row, overflow_from for the rest of the frame's records)."""
    sys.path.insert(0, ROOT)
    import json
    import torch
    import torch.distributed as dist
    from ros_vision_amd import multigpu
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    v = json.load(open(os.path.join(ROOT, "tests", "golden", "vectors.json")))
    batch = [v["dense_1080p_160tags"]["detections"], v["c2_720p_f0"]["detections"],
             v["dense_1080p_160tags"]["detections"], []]
    B, rec_cap = len(batch), 32
    g = multigpu.RecordGather(dist, B, rec_cap * multigpu._rec_size(), "cpu")
    out = None
    for s in range(3):
        if rank == 0:
            g.post(s)
        else:
            recs = [multigpu.detection_records(batch[(f + s) % B]) for f in range(B)]
            counts = [len(r) // multigpu._rec_size() for r in recs]
            rows = np.zeros((B, rec_cap * multigpu._rec_size()), np.uint8)
            for f, r in enumerate(recs):
                head = r[:rec_cap * multigpu._rec_size()]
                rows[f, :len(head)] = np.frombuffer(head, np.uint8)
            g.post(s, torch.from_numpy(rows), torch.tensor(counts, dtype=torch.int32),
                   multigpu.overflow_from(counts, rec_cap, lambda f: recs[f]))
    if rank == 0:
        out = [[multigpu.records_to_dicts(b) for b in g.frames(s)[1]] for s in (1, 2)]
    g.drain()
    if rank == 0:
        q.put((out, g.records_received))
    dist.barrier()
    dist.destroy_process_group()


def test_record_gather_keeps_dense_frames_world2():
    """a peer frame with more detections than the fixed-size record
    row (131 on the 160-tag 1080p golden board vs 32) reaches rank 0 whole, with every
    field of every record (the reference publishes every detection,
    apriltags_cuda_detector.cu:420-465)."""
    import json
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dense_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out, nrec = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    v = json.load(open(os.path.join(ROOT, "tests", "golden", "vectors.json")))
    batch = [v["dense_1080p_160tags"]["detections"], v["c2_720p_f0"]["detections"],
             v["dense_1080p_160tags"]["detections"], []]
    assert len(batch[0]) == 131
    for k, s in enumerate((1, 2)):
        for f in range(4):
            want = batch[(f + s) % 4]
            got = out[k][f]
            assert len(got) == len(want)
            for a, b in zip(got, want):
                assert a["id"] == b["id"] and a["hamming"] == b["hamming"]
                assert np.float32(a["decision_margin"]) == np.float32(b["decision_margin"])
                for key in ("H", "c", "p"):
                    assert np.array_equal(np.asarray(a[key]).ravel(), np.asarray(b[key], np.float64).ravel())
    assert nrec == 3 * (2 * 131 + 15)


def _leg_dets(v):
    """What the stand-in detector finds in a frame filled with byte v: (v % 3) records,
    plus 40 more when v % 4 == 1 (above the 32-record row: the overflow message)."""
    n = v % 3 + (40 if v % 4 == 1 else 0)
    return [dict(id=100 * v + k, hamming=k % 3, decision_margin=float(k), H=np.eye(3) * v, c=np.array([v, k]),
                 p=np.full((4, 2), 0.25 * k)) for k in range(n)]


class _CpuDetector:
    """GpuDetector's interface as multigpu.ScatterLoop drives it (enqueue_device on a
    frame buffer's address, collect, the page-locked record buffer _out_t with 64
    records per frame, _n, frame_record_bytes), detecting on the CPU by _leg_dets."""

    def __init__(self, batch, rs):
        import torch
        self.batch, self.rs, self.cap = batch, rs, 64
        self._out_t = torch.zeros(batch * self.cap * rs, dtype=torch.uint8)
        self._n = [0] * batch
        self.seen = []

    def enqueue_device(self, ptr, stride, n):
        import ctypes
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * (stride * n)).from_address(ptr)).reshape(n, stride)
        self._pending = [int(buf[f, 0]) for f in range(n)]
        assert all((buf[f] == buf[f, 0]).all() for f in range(n))

    def collect(self, counts_only=True):
        import torch
        from ros_vision_amd import multigpu
        for f, v in enumerate(self._pending):
            dets = _leg_dets(v)
            rec = multigpu.detection_records(dets)[:len(dets) * self.rs]
            o = f * self.cap * self.rs
            if rec:
                self._out_t[o:o + len(rec)] = torch.frombuffer(bytearray(rec), dtype=torch.uint8)
            self._n[f] = len(dets)
            self.seen.append(v)
        return list(self._n)

    def frame_record_bytes(self, f):
        o = f * self.cap * self.rs
        return bytes(self._out_t[o:o + self._n[f] * self.rs].numpy())


def _leg_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from ros_vision_amd import multigpu
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, npool, shape, ni, steps = 3, 9, (4, 8), 2, 7
    pool = None
    if rank == 0:  # frame (r, i) is filled with 16 r + i
        pool = torch.stack([torch.stack([torch.full(shape, 16 * r + i, dtype=torch.uint8) for i in range(npool)])
                            for r in range(world)])
    ingest = multigpu.ScatterIngest(dist, pool, B, shape, "cpu", nbuf=ni)
    gather = multigpu.RecordGather(dist, B, 32 * multigpu._rec_size(), "cpu")
    dets = [_CpuDetector(B, multigpu._rec_size()) for _ in range(ni)]
    loop = multigpu.ScatterLoop(dist, dets, ingest, gather, B, shape[0] * shape[1], 32)
    loop.run(ni, 0)  # warm-up, as bench.py's leg
    recv0 = gather.records_received
    nd = loop.run(steps, step0=ni)
    at_root = nd + gather.records_received - recv0 if rank == 0 else None
    el, tot = multigpu.reduce_max_sum(dist, 0.5 + rank, nd, "cpu")
    leg = multigpu.scatter_leg_summary(world, steps, B, shape[0] * shape[1], el, tot, at_root)
    q.put((rank, leg, sorted(v for d in dets for v in d.seen)))
    dist.barrier()
    dist.destroy_process_group()


def test_scatter_leg_world2():
    """the N > 1 bench line's scatter leg (multigpu.ScatterLoop, the
    loop bench.py --ingest scatter runs): every rank detects exactly the frames rank 0
    holds for it, step after step, and rank 0 ends with every record of every rank
    (frames above the 32-record row included); the sub-object's fields."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_leg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (leg, seen) for r, leg, seen in (q.get(timeout=300) for _ in range(world))}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    B, npool, ni, steps = 3, 9, 2, 7
    want_total = 0
    for r in range(world):
        want = []
        for s in list(range(ni)) + list(range(ni, ni + steps)):
            off = (s * B) % npool
            off = 0 if off + B > npool else off
            want += [16 * r + off + k for k in range(B)]
        assert res[r][1] == sorted(want)
        want_total += sum(len(_leg_dets(16 * r + ((s * B) % npool) + k)) for s in range(ni, ni + steps) for k in range(B))
    leg = res[0][0]
    assert leg["records_at_rank0"] == leg["detections"] == want_total
    assert any(v % 4 == 1 for v in res[1][1])  # (a peer frame went through the overflow message)
    assert leg["steps"] == steps and leg["peers"] == 1 and leg["unit"] == "frames/s"
    assert leg["bytes_scattered_per_peer_per_step"] == B * 32
    assert leg["bytes_scattered_per_peer"] == steps * B * 32
    assert abs(leg["value"] - world * steps * B / 1.5) < 0.01  # max elapsed over ranks (1.5 s)
    assert res[1][0]["records_at_rank0"] is None
