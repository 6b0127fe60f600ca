"""Frame sharding across GPUs.

Frames are independent, so the path shards one frame per GPU with no
exchange between frames.  Two modes:

* local (default bench mode): every rank owns its own frames, nothing crosses
  xGMI on the data path; only timing/counters are reduced.
* scatter/gather (the north-star multi-camera topology): frames originate on
  rank 0, ``scatter_frames`` sends each rank its fixed-size YUYV slots
  (torch.distributed.scatter -> ncclScatter-style RCCL sends over xGMI with
  backend "nccl", gloo on CPU), each rank detects, and ``gather_detections``
  returns fixed-capacity detection records to rank 0.

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

    Rank 0 holds every rank's frames in device memory; ``start(step)`` launches
    the scatter of step `step`'s batch (async RCCL/gloo collective) into buffer
    step % nbuf, ``ready(step)`` waits for it and returns that buffer.  The caller
    must have finished reading buffer (step % nbuf) -- i.e. collected step - nbuf --
    before ``start(step)``; nbuf = the batches in flight keeps the same depth as
    the local-ingest pipeline.
    """

    def __init__(self, dist, root_pool, batch: int, frame_shape, device, nbuf: int = 2):
        import torch
        self.dist, self.batch, self.device = dist, batch, device
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.pool = root_pool  # rank 0: [world, npool, *frame_shape] (None elsewhere)
        self.npool = int(root_pool.shape[1]) if root_pool is not None else 0
        self.nbuf = max(2, int(nbuf))
        self.buf = [torch.empty((batch,) + tuple(frame_shape), dtype=torch.uint8, device=device)
                    for _ in range(self.nbuf)]
        self.work = [None] * self.nbuf

    def _chunks(self, step):
        if self.rank != 0:
            return None
        off = (step * self.batch) % self.npool
        if off + self.batch > self.npool:
            off = 0
        return [self.pool[r, off:off + self.batch] for r in range(self.world)]

    def start(self, step):
        i = step % self.nbuf
        self.work[i] = self.dist.scatter(self.buf[i], scatter_list=self._chunks(step), src=0, async_op=True)

    def ready(self, step, detector=None):
        """Buffer of step `step`.  On the GPU the collective's completion is handed to
        `detector`'s stream as a stream dependency (at_stream_wait), not a host wait;
        without a detector the host synchronizes torch's stream."""
        import torch
        i = step % self.nbuf
        self.work[i].wait()  # torch's current stream now waits for the collective
        if self.buf[i].is_cuda:
            stream = torch.cuda.current_stream(self.buf[i].device)
            if detector is not None:
                detector.wait_stream(stream.cuda_stream)
            else:
                stream.synchronize()
        return self.buf[i]


def reduce_max_sum(dist, elapsed: float, count: float, device):
    """(max elapsed over ranks, sum of counts) -- the bench's timing reduction."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([count], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), float(c.item())
