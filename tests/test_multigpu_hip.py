"""The HIP detector inside a process group (world_size 2 on one GPU, gloo).

Frames originate on rank 0 and are scattered (gloo, CPU), each rank moves its
shard into HBM on torch's stream, hands that stream to its detector with
at_stream_wait (no host synchronize), detects through the C ABI, and every
detection record is gathered to rank 0 (multigpu.RecordGather: fixed-size rows plus
the overflow message) and compared with the oracle.
The RCCL variant of the same flow is bench.py --ingest scatter.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, nper, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from ros_vision_amd import GpuDetector, multigpu, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    src = None
    if rank == 0:
        frames = np.stack([synth.stream_frame(W, H, 40 + i)[0] for i in range(world * nper)])
        src = torch.from_numpy(frames)
    mine = multigpu.scatter_frames(dist, src, nper, (H, 2 * W), "cpu")
    d_frames = mine.pin_memory().to("cuda", non_blocking=True)  # async on torch's stream
    det = GpuDetector(W, H, max_batch=nper)
    det.wait_stream(torch.cuda.current_stream().cuda_stream)
    det.enqueue_device(d_frames.data_ptr(), d_frames[0].numel(), nper)
    counts = det.collect(counts_only=True)
    # the bench's record path (rows of the first rec_cap records + the true counts, the
    # rest of each frame in the overflow message); rec_cap 4 < 15 detections per frame
    rec_cap = 4
    rows, cnt, over = multigpu.split_records([det.frame_record_bytes(f) for f in range(nper)], rec_cap)
    assert list(cnt) == counts
    g = multigpu.RecordGather(dist, nper, rec_cap * multigpu._rec_size(), "cpu")
    g.post(0, torch.from_numpy(rows), torch.from_numpy(cnt), over)
    if rank == 0:
        allp = [det.frame_record_bytes(f) for f in range(nper)] + g.frames(0)[1]
        q.put(allp)
    g.drain()
    dist.barrier()
    det.close()
    dist.destroy_process_group()


def test_hip_detector_in_process_group(oracle_mod):
    from ros_vision_amd import multigpu, synth
    W, H, nper, world = 1280, 720, 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, nper, q)) for r in range(world)]
    for p in procs:
        p.start()
    allp = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    o = oracle_mod.Oracle(W, H)
    for i in range(world * nper):
        o.detect(synth.stream_frame(W, H, 40 + i)[0], 0)
        want = o.detections()
        got = multigpu.records_to_dicts(allp[i])
        assert len(want) == 15
        assert [d["id"] for d in got] == [d["id"] for d in want]
        for a, b in zip(got, want):
            assert np.allclose(a["p"], b["p"], atol=1e-4) and np.allclose(a["H"], b["H"], atol=1e-4)
