"""Frame sharding across GPUs.

Frames are independent, so the path shards one frame per GPU with no
exchange between frames.  Two modes:

* local (default bench mode): every rank owns its own frames, nothing crosses
  xGMI on the data path; only timing/counters are reduced.
* scatter/gather (the north-star multi-camera topology): frames originate on
  rank 0, which sends each other rank its fixed-size YUYV slots (``ScatterIngest``:
  RCCL point-to-point sends over xGMI with backend "nccl", one peer per link;
  ``scatter_frames``: torch.distributed.scatter; gloo on CPU), each rank detects,
  and ``gather_detections`` returns fixed-capacity detection records to rank 0.

The helpers are backend-agnostic (CPU tensors + gloo in the tests, HBM
tensors + RCCL on the node).
"""
import numpy as np

REC = 22  # id, hamming, margin, H[9], c[2], p[4][2]


def shard_range(rank: int, world: int, nframes: int):
    """Contiguous frame range [lo, hi) owned by `rank` (frame k -> GPU k*world//n)."""
    per = (nframes + world - 1) // world
    lo = min(nframes, rank * per)
    return lo, min(nframes, lo + per)


def pack_detections(dets_per_frame, cap: int) -> np.ndarray:
    """[nframes, cap + 1, REC] float64; row 0 holds the count."""
    out = np.zeros((len(dets_per_frame), cap + 1, REC), np.float64)
    for f, dets in enumerate(dets_per_frame):
        out[f, 0, 0] = min(len(dets), cap)
        for i, d in enumerate(dets[:cap]):
            get = (lambda k: d[k]) if isinstance(d, dict) else (lambda k: getattr(d, k))
            out[f, i + 1, 0] = get("id")
            out[f, i + 1, 1] = get("hamming")
            out[f, i + 1, 2] = get("decision_margin")
            out[f, i + 1, 3:12] = np.asarray(get("H"), np.float64).ravel()
            out[f, i + 1, 12:14] = np.asarray(get("c"), np.float64)
            out[f, i + 1, 14:22] = np.asarray(get("p"), np.float64).ravel()
    return out


def unpack_detections(arr: np.ndarray):
    res = []
    for f in range(arr.shape[0]):
        n = int(arr[f, 0, 0])
        res.append([dict(id=int(r[0]), hamming=int(r[1]), decision_margin=float(r[2]), H=r[3:12].reshape(3, 3),
                         c=r[12:14].copy(), p=r[14:22].reshape(4, 2)) for r in arr[f, 1:n + 1]])
    return res


def scatter_frames(dist, frames_on_root, frames_per_rank: int, frame_shape, device, dtype=None):
    """Rank 0 holds [world * frames_per_rank, *frame_shape] frames; every rank
    receives its [frames_per_rank, *frame_shape] slice (one collective)."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    out = torch.empty((frames_per_rank,) + tuple(frame_shape), dtype=dtype or torch.uint8, device=device)
    chunks = list(frames_on_root.chunk(world, dim=0)) if rank == 0 else None
    dist.scatter(out, scatter_list=chunks, src=0)
    return out


def gather_detections(dist, packed: np.ndarray, device):
    """Every rank's packed [frames_per_rank, cap+1, REC] records -> rank 0 (list per rank)."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.from_numpy(packed).to(device)
    gl = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gather_list=gl, dst=0)
    if rank != 0:
        return None
    return np.concatenate([g.cpu().numpy() for g in gl], axis=0)


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


class RecordGather:
    """Fixed-capacity detection records of every rank's batch -> rank 0 (north-star
    topology): one point-to-point receive per peer on rank 0, one send on each peer
    (RCCL with backend "nccl", gloo on CPU), double-buffered so the transfer of step
    s overlaps the detection of the next steps.  Rank 0's own records never move
    (they are already in its host buffer), so at world size 1 nothing is sent.

    A peer's ``post(step, records, counts)``: `records` [batch, rec_bytes] and
    `counts` [batch] int32 (host tensors; `records` page-locked, read by an async
    copy -- the caller keeps it intact until ``copied`` of that step has completed);
    rank 0's ``post(step)`` posts the receives and ``result(step)`` returns the
    peers' [batch, 4 + rec_bytes] tensors (count, records) once they have arrived."""

    def __init__(self, dist, batch: int, rec_bytes: int, device):
        import torch
        self.dist, self.world, self.rank = dist, dist.get_world_size(), dist.get_rank()
        self.cuda = str(device).startswith("cuda")
        row = rec_bytes + 4
        self.send = [torch.empty((batch, row), dtype=torch.uint8, device=device) for _ in range(2)]
        self.cnt = [torch.empty((batch,), dtype=torch.int32) for _ in range(2)]
        if self.cuda:
            self.cnt = [c.pin_memory() for c in self.cnt]
        self.recv = ([{r: torch.empty((batch, row), dtype=torch.uint8, device=device) for r in range(1, self.world)}
                      for _ in range(2)] if self.rank == 0 else None)
        self.work = [None, None]
        self.copied = [None, None]  # event after step's copies out of the caller's host buffers

    def _wait(self, i):
        for w in (self.work[i] or []):
            w.wait()
        self.work[i] = None

    def post(self, step, records=None, counts=None):
        import torch
        if self.world == 1:
            return
        d, i = self.dist, step % 2
        self._wait(i)  # the buffer's previous transfer (step - 2)
        if self.rank == 0:
            ops = [d.P2POp(d.irecv, self.recv[i][r], r) for r in range(1, self.world)]
        else:
            if self.copied[i] is not None:
                self.copied[i].synchronize()  # (step - 2's copy of cnt[i]: long done)
            self.cnt[i].copy_(counts)
            self.send[i][:, 4:].copy_(records, non_blocking=True)
            self.send[i][:, :4].copy_(self.cnt[i].view(torch.uint8).view(-1, 4), non_blocking=True)
            if self.cuda:
                self.copied[i] = torch.cuda.Event()
                self.copied[i].record()
            ops = [d.P2POp(d.isend, self.send[i], 0)]
        self.work[i] = d.batch_isend_irecv(ops)

    def result(self, step):
        i = step % 2
        self._wait(i)
        return self.recv[i] if self.rank == 0 else None

    def drain(self):
        self._wait(0)
        self._wait(1)


def reduce_max_sum(dist, elapsed: float, count: float, device):
    """(max elapsed over ranks, sum of counts) -- the bench's timing reduction."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([count], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), float(c.item())
