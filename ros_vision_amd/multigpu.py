"""Frame sharding across GPUs.

Frames are independent, so the path shards one frame per GPU with no
exchange between frames.  Two modes:

* local (default bench mode): every rank owns its own frames, nothing crosses
  xGMI on the data path; only timing/counters are reduced.
* scatter/gather (the north-star multi-camera topology): frames originate on
  rank 0, which sends each other rank its fixed-size YUYV slots (``ScatterIngest``:
  RCCL point-to-point sends over xGMI with backend "nccl", one peer per link;
  ``scatter_frames``: torch.distributed.scatter; gloo on CPU), each rank detects,
  and ``RecordGather`` returns every detection record to rank 0 (a fixed-capacity
  row per frame plus an overflow message for frames with more).

The helpers are backend-agnostic (CPU tensors + gloo in the tests, HBM
tensors + RCCL on the node).
"""
import numpy as np


def shard_range(rank: int, world: int, nframes: int):
    """Contiguous frame range [lo, hi) owned by `rank` (frame k -> GPU k*world//n)."""
    per = (nframes + world - 1) // world
    lo = min(nframes, rank * per)
    return lo, min(nframes, lo + per)


def scatter_frames(dist, frames_on_root, frames_per_rank: int, frame_shape, device, dtype=None):
    """Rank 0 holds [world * frames_per_rank, *frame_shape] frames; every rank
    receives its [frames_per_rank, *frame_shape] slice (one collective)."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    out = torch.empty((frames_per_rank,) + tuple(frame_shape), dtype=dtype or torch.uint8, device=device)
    chunks = list(frames_on_root.chunk(world, dim=0)) if rank == 0 else None
    dist.scatter(out, scatter_list=chunks, src=0)
    return out


class ScatterIngest:
    """Multi-buffered frame ingest from rank 0 (north-star topology).

    Rank 0 holds every rank's frames in device memory.  ``start(step)`` sends step
    `step`'s batch to every other rank -- one point-to-point RCCL send per peer
    (``batch_isend_irecv``; gloo on CPU), i.e. the sends a scatter is made of, each
    peer on its own xGMI link -- into that rank's buffer step % nbuf; ``ready(step)``
    hands the arrival to the detector's stream and returns the buffer.  Rank 0's
    own share never moves: its batch is read in place from the pool (a scatter
    would copy it into a buffer of its own, 2 x 236 MB of HBM traffic per
    128-frame step at 720p, by an RCCL kernel on the CUs the detector uses).
    The caller must have finished reading buffer (step % nbuf) -- i.e. collected
    step - nbuf -- before ``start(step)``; nbuf = the batches in flight keeps the
    same depth as the local-ingest pipeline.
    """

    def __init__(self, dist, root_pool, batch: int, frame_shape, device, nbuf: int = 2):
        import torch
        self.dist, self.batch, self.device = dist, batch, device
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.pool = root_pool  # rank 0: [world, npool, *frame_shape] (None elsewhere)
        self.npool = int(root_pool.shape[1]) if root_pool is not None else 0
        self.nbuf = max(2, int(nbuf))
        self.buf = ([torch.empty((batch,) + tuple(frame_shape), dtype=torch.uint8, device=device)
                     for _ in range(self.nbuf)] if self.rank != 0 else None)
        self.work = [None] * self.nbuf

    def _offset(self, step):
        off = (step * self.batch) % self.npool if self.npool else 0
        return 0 if off + self.batch > self.npool else off

    def start(self, step):
        i = step % self.nbuf
        if self.world == 1:
            self.work[i] = None
            return
        d = self.dist
        for w in (self.work[i] or []):  # the slot's previous transfer (at most nbuf in flight)
            w.wait()
        if self.rank == 0:
            off = self._offset(step)
            ops = [d.P2POp(d.isend, self.pool[r, off:off + self.batch], r) for r in range(1, self.world)]
        else:
            ops = [d.P2POp(d.irecv, self.buf[i], 0)]
        self.work[i] = d.batch_isend_irecv(ops)

    def ready(self, step, detector=None):
        """Buffer of step `step` (rank 0: its slice of the pool).  On the GPU the
        arrival is handed to `detector`'s stream as a stream dependency
        (at_stream_wait), not a host wait; without a detector the host
        synchronizes torch's stream."""
        import torch
        i = step % self.nbuf
        if self.rank == 0:  # (its sends read the pool, which nothing writes: no wait)
            off = self._offset(step)
            return self.pool[0, off:off + self.batch]
        for w in self.work[i]:
            w.wait()  # torch's current stream now waits for the receive
        self.work[i] = None
        if self.buf[i].is_cuda:
            stream = torch.cuda.current_stream(self.buf[i].device)
            if detector is not None:
                detector.wait_stream(stream.cuda_stream)
            else:
                stream.synchronize()
        return self.buf[i]

    def drain(self):
        """Completes every outstanding send / receive (end of a timed run)."""
        for ws in self.work:
            for w in (ws or []):
                w.wait()
        self.work = [None] * self.nbuf


def _rec_size():
    import ctypes
    from .detector import AtDetection
    return ctypes.sizeof(AtDetection)


def detection_records(dets) -> bytes:
    """at_detection records (include/at_api.h) of a list of detections (dicts with the
    oracle's keys or Detection objects), as the C ABI lays them out."""
    from .detector import AtDetection
    arr = (AtDetection * max(1, len(dets)))()
    for i, d in enumerate(dets):
        get = (lambda k: d[k]) if isinstance(d, dict) else (lambda k: getattr(d, k))
        arr[i].id, arr[i].hamming, arr[i].decision_margin = int(get("id")), int(get("hamming")), \
            float(get("decision_margin"))
        arr[i].H[:] = [float(x) for x in np.asarray(get("H"), np.float64).ravel()]
        arr[i].c[:] = [float(x) for x in np.asarray(get("c"), np.float64).ravel()]
        p = np.asarray(get("p"), np.float64).reshape(4, 2)
        for k in range(4):
            arr[i].p[k][0], arr[i].p[k][1] = float(p[k, 0]), float(p[k, 1])
    return bytes(arr)[:len(dets) * _rec_size()]


def records_to_dicts(buf) -> list:
    """Inverse of detection_records: at_detection bytes -> detections as dicts."""
    from .detector import AtDetection
    rs = _rec_size()
    buf = bytes(buf)
    out = []
    for i in range(len(buf) // rs):
        r = AtDetection.from_buffer_copy(buf[i * rs:(i + 1) * rs])
        out.append(dict(id=r.id, hamming=r.hamming, decision_margin=r.decision_margin,
                        H=np.array(list(r.H)).reshape(3, 3), c=np.array(list(r.c)),
                        p=np.array([[r.p[k][0], r.p[k][1]] for k in range(4)])))
    return out


def overflow_from(counts, cap: int, frame_records) -> np.ndarray:
    """The records past `cap` of every frame that has more, in frame order (uint8,
    possibly empty); frame_records(f) gives frame f's full at_detection bytes and is
    called only for those frames."""
    rs = _rec_size()
    over = [bytes(frame_records(f))[cap * rs:int(n) * rs] for f, n in enumerate(counts) if n > cap]
    return np.frombuffer(b"".join(over), np.uint8).copy()


def split_records(frame_records, cap: int):
    """Per-frame at_detection bytes -> what a peer sends rank 0 for one batch: the
    fixed-capacity rows [nframes, cap * rec] (the first `cap` records of each frame),
    the TRUE counts [nframes] int32 and the overflow (overflow_from).  Nothing is
    dropped: join_records restores every frame's full list."""
    rs = _rec_size()
    nf = len(frame_records)
    rows = np.zeros((nf, cap * rs), np.uint8)
    counts = np.zeros(nf, np.int32)
    for f, b in enumerate(frame_records):
        b = bytes(b)
        counts[f] = len(b) // rs
        head = b[:min(int(counts[f]), cap) * rs]
        rows[f, :len(head)] = np.frombuffer(head, np.uint8)
    return rows, counts, overflow_from(counts, cap, lambda f: frame_records[f])


def overflow_bytes(counts, cap: int) -> int:
    """Size of the overflow message of a batch with these true per-frame counts."""
    c = np.asarray(counts, np.int64)
    return int(np.maximum(c - cap, 0).sum()) * _rec_size()


def join_records(rows, counts, overflow, cap: int):
    """Inverse of split_records: every frame's full at_detection bytes."""
    rs = _rec_size()
    rows = np.asarray(rows, np.uint8)
    overflow = np.asarray(overflow, np.uint8)
    out, pos = [], 0
    for f, n in enumerate(np.asarray(counts, np.int64)):
        n = int(n)
        b = rows[f, :min(n, cap) * rs].tobytes()
        if n > cap:
            m = (n - cap) * rs
            b += overflow[pos:pos + m].tobytes()
            pos += m
        out.append(b)
    if pos != overflow.size:
        raise ValueError("overflow holds %d bytes, the counts name %d" % (overflow.size, pos))
    return out


class RecordGather:
    """Detection records of every rank's batch -> rank 0 (north-star topology), every
    detection of every frame (the reference publishes all of them,
    apriltags_cuda_detector.cu:420-465): one point-to-point message per peer and step
    holds a fixed-capacity row per frame (its first `cap` records) and the frame's true
    count; the records of frames with more than `cap` follow in a second message sized
    by those counts.  RCCL with backend "nccl", gloo on CPU.  Double-buffered: the
    transfer of step s overlaps the detection of the next steps.  Rank 0's own records
    never move (they are already in its host buffer), so at world size 1 nothing is sent.

    A peer's ``post(step, records, counts, overflow)``: `records` [batch, rec_bytes]
    and `counts` [batch] int32 (host tensors; `records` page-locked, read by an async
    copy -- the caller keeps it intact until ``copied`` of that step has completed),
    `overflow` the bytes of split_records (None or empty: no frame above `cap`).
    Rank 0's ``post(step)`` posts the receives; ``result(step)`` returns, per peer, the
    [batch, 4 + rec_bytes] tensor (count, records) and the overflow bytes once arrived
    (``frames(step)``: every frame's full record bytes).

    Message order per peer (point-to-point order is the matching order): header(s),
    overflow(s) if any, header(s + 1) ...  Rank 0 learns the size of overflow(s) from
    header(s), so before posting header(s + 1) it waits for header(s) (one step behind
    the detector) and posts the overflow receive first.

    The gather runs in a process group of its own (``dist.new_group``, created
    collectively by every rank in the constructor): with backend "nccl" that is an RCCL
    communicator, and so a stream, separate from ScatterIngest's.  On one shared
    communicator a peer's queue [header(s)][overflow(s)][receive frames(s + n)] and rank
    0's [receive header(s)][send frames(s + n)][receive overflow(s)] each wait on a
    transfer the other side queued behind its own, which only progresses while RCCL can
    buffer the overflow (a dense frame's overflow exceeds that).  Rank 0 reads the
    headers' counts on a side stream (copy to page-locked memory, event), not by
    synchronizing torch's current stream."""

    def __init__(self, dist, batch: int, rec_bytes: int, device, group=None):
        import torch
        self.dist, self.world, self.rank = dist, dist.get_world_size(), dist.get_rank()
        self.device = device
        self.cuda = str(device).startswith("cuda")
        # the gather's own communicator (every rank constructs RecordGather, so the
        # collective new_group call matches on all of them)
        self.group = group if group is not None else (dist.new_group(list(range(self.world)))
                                                      if self.world > 1 else None)
        self.side = torch.cuda.Stream(device) if (self.cuda and self.world > 1) else None
        self.batch, self.rec_bytes = batch, rec_bytes
        self.cap = rec_bytes // _rec_size()
        row = rec_bytes + 4
        self.send = [torch.empty((batch, row), dtype=torch.uint8, device=device) for _ in range(2)]
        self.cnt = [torch.empty((batch,), dtype=torch.int32) for _ in range(2)]
        # rank 0: the peers' counts of a header, read back to the host
        self.hcnt = torch.empty((max(1, self.world - 1), batch), dtype=torch.int32)
        if self.cuda:
            self.cnt = [c.pin_memory() for c in self.cnt]
            self.hcnt = self.hcnt.pin_memory()
        self.recv = ([{r: torch.empty((batch, row), dtype=torch.uint8, device=device) for r in range(1, self.world)}
                      for _ in range(2)] if self.rank == 0 else None)
        self.ovf = [None, None]      # peer: overflow send buffer; rank 0: {peer: receive buffer}
        self.work = [None, None]     # header transfers of the slot
        self.owork = [None, None]    # overflow transfers of the slot
        self.unresolved = []         # rank 0: steps whose overflow receives are not posted yet
        self.records_received = 0    # rank 0: records of the peers received (true counts)
        self.copied = [None, None]   # event after step's copies out of the caller's host buffers

    def _wait(self, i):
        for w in (self.work[i] or []) + (self.owork[i] or []):
            w.wait()
        self.work[i] = self.owork[i] = None

    def _p2p(self, op, tensor, peer):
        return self.dist.P2POp(op, tensor, peer, group=self.group)

    def _resolve(self, step):
        """Rank 0: header(step) has to have arrived; post its overflow receives."""
        import torch
        i = step % 2
        if self.cuda:
            # the headers are in HBM: a side stream waits for their arrival and copies the
            # count columns to page-locked memory; the host waits for that copy only
            with torch.cuda.stream(self.side):
                for w in (self.work[i] or []):
                    w.wait()
                for r in range(1, self.world):
                    self.hcnt[r - 1].view(torch.uint8).view(-1, 4).copy_(self.recv[i][r][:, :4], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            ev.synchronize()
        else:
            for w in (self.work[i] or []):
                w.wait()
            for r in range(1, self.world):
                self.hcnt[r - 1].copy_(self.recv[i][r][:, :4].contiguous().view(torch.int32).ravel())
        self.work[i] = None
        ovf, ops = {}, []
        for r in range(1, self.world):
            counts = self.hcnt[r - 1].numpy().copy()
            self.records_received += int(counts.sum())
            m = overflow_bytes(counts, self.cap)
            if m:
                ovf[r] = torch.empty((m,), dtype=torch.uint8, device=self.device)
                ops.append(self._p2p(self.dist.irecv, ovf[r], r))
        self.ovf[i] = ovf
        self.owork[i] = self.dist.batch_isend_irecv(ops) if ops else None

    def post(self, step, records=None, counts=None, overflow=None):
        import torch
        if self.world == 1:
            return
        d, i = self.dist, step % 2
        if self.rank == 0:
            while self.unresolved:  # overflow(s) precedes header(s + 1) on every link
                self._resolve(self.unresolved.pop(0))
            self._wait(i)  # the buffer's previous transfer (step - 2)
            self.work[i] = d.batch_isend_irecv([self._p2p(d.irecv, self.recv[i][r], r) for r in range(1, self.world)])
            self.unresolved.append(step)
            return
        self._wait(i)  # the buffer's previous transfer (step - 2)
        if self.copied[i] is not None:
            self.copied[i].synchronize()  # (step - 2's copy of cnt[i]: long done)
        self.cnt[i].copy_(counts)
        self.send[i][:, 4:].copy_(records, non_blocking=True)
        self.send[i][:, :4].copy_(self.cnt[i].view(torch.uint8).view(-1, 4), non_blocking=True)
        n_over = 0 if overflow is None else int(overflow.numel() if hasattr(overflow, "numel") else len(overflow))
        if n_over != overflow_bytes(self.cnt[i].numpy(), self.cap):
            raise ValueError("overflow of %d bytes does not match the counts" % n_over)
        self.ovf[i] = None
        if n_over:
            o = overflow if hasattr(overflow, "numel") else torch.from_numpy(np.asarray(overflow, np.uint8))
            self.ovf[i] = o.to(self.device, non_blocking=False) if self.cuda else o.clone()
        if self.cuda:
            self.copied[i] = torch.cuda.Event()
            self.copied[i].record()
        self.work[i] = d.batch_isend_irecv([self._p2p(d.isend, self.send[i], 0)])
        if n_over:
            self.owork[i] = d.batch_isend_irecv([self._p2p(d.isend, self.ovf[i], 0)])

    def result(self, step):
        """Rank 0: {peer: (header [batch, 4 + rec_bytes], overflow bytes or None)}."""
        i = step % 2
        if step in self.unresolved:
            while self.unresolved and self.unresolved[0] <= step:
                self._resolve(self.unresolved.pop(0))
        for w in (self.owork[i] or []):
            w.wait()
        self.owork[i] = None
        if self.rank != 0:
            return None
        return {r: (self.recv[i][r], self.ovf[i].get(r)) for r in range(1, self.world)}

    def frames(self, step):
        """Rank 0: {peer: [full at_detection bytes of each frame of its batch]}."""
        import torch
        out = {}
        for r, (hdr, ovf) in self.result(step).items():
            h = hdr.cpu()
            counts = h[:, :4].contiguous().view(torch.int32).ravel().numpy()
            o = ovf.cpu().numpy() if ovf is not None else np.zeros(0, np.uint8)
            out[r] = join_records(h[:, 4:].numpy(), counts, o, self.cap)
        return out

    def drain(self):
        if self.rank == 0:
            while self.unresolved:
                self._resolve(self.unresolved.pop(0))
        self._wait(0)
        self._wait(1)


class ScatterLoop:
    """The north-star loop (bench.py ``--ingest scatter``, and the scatter leg of every
    N > 1 line): frames leave rank 0 by ScatterIngest, every rank detects its batch on
    detector instances used round-robin (batch k enqueued on instance k mod n, collected
    n - 1 enqueues later: the local loop's in-flight depth), and each peer's records
    return to rank 0 by RecordGather -- the first `rec_cap` records of every frame in the
    fixed-size row plus an overflow message.  The scatter of step k + 1 overlaps the
    detection of steps k - n + 2 .. k (one frame buffer per instance; a buffer is sent
    again only after the batch that read it is collected).

    A detector here is anything with GpuDetector's ``enqueue_device(ptr, stride, n)``,
    ``collect(counts_only=True)``, ``wait_stream``, the page-locked record buffer
    ``_out_t``, the per-frame counts ``_n`` and ``frame_record_bytes(f)`` (the gloo test
    stands a CPU detector in)."""

    def __init__(self, dist, dets, ingest, gather, batch: int, stride: int, rec_cap: int):
        self.dist, self.dets, self.ingest, self.gather = dist, list(dets), ingest, gather
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.batch, self.stride, self.rec_cap = batch, stride, rec_cap
        self.rec_bytes = rec_cap * _rec_size()
        self.copied = {}  # detector -> event after the async copy out of its record buffer

    def _gather(self, d, step):
        import torch
        if self.world == 1:
            return
        if self.rank == 0:
            self.gather.post(step)
            return
        counts = [int(d._n[f]) for f in range(self.batch)]
        self.gather.post(step, d._out_t.view(self.batch, -1)[:, :self.rec_bytes], torch.tensor(counts, dtype=torch.int32),
                         overflow_from(counts, self.rec_cap, d.frame_record_bytes))
        self.copied[id(d)] = self.gather.copied[step % 2]

    def run(self, nsteps: int, step0: int = 0) -> int:
        """Runs nsteps batches from step step0; returns this rank's detections."""
        ndet, ni, inflight = 0, len(self.dets), []

        def drain():
            pd, ps = inflight.pop(0)
            ev = self.copied.pop(id(pd), None)
            if ev is not None:  # its record buffer may still be copied from
                ev.synchronize()
            n = sum(pd.collect(counts_only=True))
            self._gather(pd, ps)
            return n

        self.ingest.start(step0)
        for s in range(step0, step0 + nsteps):
            d = self.dets[(s - step0) % ni]
            buf = self.ingest.ready(s, detector=d)  # stream dependency, no host wait
            d.enqueue_device(buf.data_ptr(), self.stride, self.batch)
            inflight.append((d, s))
            if len(inflight) == ni:
                ndet += drain()
            if s + 1 < step0 + nsteps:
                self.ingest.start(s + 1)  # its buffer was read by step s+1-instances, collected above
        while inflight:
            ndet += drain()
        self.gather.drain()
        self.ingest.drain()
        return ndet


def scatter_leg_summary(world: int, steps: int, batch: int, frame_bytes: int, elapsed: float, detections: int,
                        records_at_rank0):
    """The scatter topology's sub-object of an N > 1 bench line: whole-job frames/s over
    the leg's timed steps (max elapsed over ranks), what rank 0 holds afterwards, and the
    bytes each peer received from rank 0 over its xGMI link."""
    per_step = batch * frame_bytes
    return {"value": round(world * steps * batch / elapsed, 2), "unit": "frames/s", "steps": steps,
            "ms_per_step": round(1e3 * elapsed / steps, 4), "detections": int(detections),
            "records_at_rank0": None if records_at_rank0 is None else int(records_at_rank0),
            "peers": world - 1, "bytes_scattered_per_peer_per_step": per_step,
            "bytes_scattered_per_peer": per_step * steps,
            "GBps_per_peer": round(per_step * steps / elapsed / 1e9, 3),
            "note": "north-star topology (SURVEY.md 8(e)): frames resident on rank 0, each step's batch sent to "
                    "every peer by RCCL point-to-point (multigpu.ScatterIngest), detection records gathered to "
                    "rank 0 (multigpu.RecordGather: a 32-record row per frame + overflow); rank 0's own share "
                    "read in place"}


def reduce_max_sum(dist, elapsed: float, count: float, device):
    """(max elapsed over ranks, sum of counts) -- the bench's timing reduction."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([count], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), float(c.item())
