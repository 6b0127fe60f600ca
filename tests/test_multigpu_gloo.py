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
    dets = []
    for f in mine:
        o.detect(f, 0)
        dets.append(o.detections())
    packed = multigpu.pack_detections(dets, 16)
    allp = multigpu.gather_detections(dist, packed, "cpu")
    el, cnt = multigpu.reduce_max_sum(dist, 1.0 + rank, float(sum(len(d) for d in dets)), "cpu")
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
    got = multigpu.unpack_detections(allp)
    codes = dict(oracle_mod.family_entries())
    o = oracle_mod.Oracle(W, H)
    total = 0
    for i in range(world * nper):
        o.detect(synth.to_yuyv(synth.render_board(W, H, seed=100 + i, ntags=4, codes=codes)[0]), 0)
        want = o.detections()
        total += len(want)
        assert [d["id"] for d in got[i]] == [d["id"] for d in want]
        for a, b in zip(got[i], want):
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
    B, rb = 3, 8
    g = multigpu.RecordGather(dist, B, rb, "cpu")
    got = []
    for s in range(5):  # step s: rank r's record bytes = 10*r + s, counts = r + s + frame
        recs = torch.full((B, rb), 10 * rank + s, dtype=torch.uint8)
        cnt = torch.tensor([rank + s + f for f in range(B)], dtype=torch.int32)
        g.post(s, recs, cnt)
        if s >= 1 and rank == 0:  # results of the previous step (double buffered)
            res = g.result(s - 1)
            got.append({r: (int(t[0, 4]), t[:, :4].contiguous().view(torch.int32).ravel().tolist()) for r, t in res.items()})
    if rank == 0:
        res = g.result(4)
        got.append({r: (int(t[0, 4]), t[:, :4].contiguous().view(torch.int32).ravel().tolist()) for r, t in res.items()})
    g.drain()
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_record_gather_world3():
    """bench.py --ingest scatter: detection records of ranks 1..N-1 reach rank 0 by
    point-to-point sends (rank 0's own never move), double-buffered over steps."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(res[0]) == 5
    for s, step in enumerate(res[0]):
        assert sorted(step) == [1, 2]
        for r in (1, 2):
            assert step[r] == (10 * r + s, [r + s + f for f in range(3)])
