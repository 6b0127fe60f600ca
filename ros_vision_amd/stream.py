"""The throughput configuration of the bench, as one reusable loop.

Config C2: a 1280x720 synthetic tag36h11 stream whose frames
are already resident in HBM.  ``StreamRunner`` drives several detector
instances (one HIP stream each) round-robin: batch k is enqueued on instance
k mod n and collected n-1 enqueues later, so up to n batches are in flight and
the host tail of one batch overlaps the kernels of the next ones.  bench.py
times exactly this loop and tests/test_stream_parity.py checks every frame it
returns against the oracle goldens, so the headline number and its parity
evidence come from the same code.
"""
import numpy as np

from .detector import AT_FMT_YUYV


def stream_pool(width: int, height: int, pool: int, tags: int = 15, rank: int = 0, codes=None):
    """The C2 frames one rank renders into its HBM: frame f = rank*pool + i, seed
    766000 + f, ids 10f .. 10f+tags-1 mod 587, packed YUYV [pool, H, 2W]."""
    from . import synth
    codes = codes if codes is not None else synth._codes()
    frames = np.empty((pool, height, 2 * width), np.uint8)
    for i in range(pool):
        f = rank * pool + i
        gray, _ = synth.render_board(width, height, seed=766000 + f, ntags=tags,
                                     ids=synth.stream_ids(f, tags, len(codes)), codes=codes)
        frames[i] = synth.to_yuyv(gray)
    return frames


class StreamRunner:
    """Round-robin enqueue/collect over detector instances on a frame pool in HBM.

    ``base``/``stride``/``npool``: device address of the pool, bytes per frame,
    frames in it.  Step s reads the `batch` frames at offset
    ``offset(s)`` (consecutive batches walk the pool and wrap)."""

    def __init__(self, detectors, base: int, stride: int, npool: int, batch: int, fmt: int = AT_FMT_YUYV,
                 host: bool = False):
        """host=True: `base` is a host (page-locked) pool and the frames go through
        at_enqueue_host (H2D copies on the detector's stream); a batch may then be
        larger than the pool (frames taken modulo the pool)."""
        self.dets = list(detectors)
        self.base, self.stride, self.npool, self.batch, self.fmt = base, stride, npool, batch, fmt
        self.host = host

    def offset(self, step: int) -> int:
        off = (step * self.batch) % self.npool
        if self.host:
            return off
        return 0 if off + self.batch > self.npool else off

    def _enqueue(self, d, step):
        off = self.offset(step)
        if self.host:
            d.enqueue_host([self.base + ((off + j) % self.npool) * self.stride for j in range(self.batch)], self.fmt)
        else:
            d.enqueue_device(self.base + off * self.stride, self.stride, self.batch, self.fmt)

    def run(self, nsteps: int, step0: int = 0, on_batch=None) -> int:
        """Runs nsteps batches; returns the number of detections.  on_batch(det,
        step, offset) is called right after each batch is collected (its results
        are then in det's output buffer: det.results())."""
        ndet = 0
        ni = len(self.dets)
        inflight = []

        def drain():
            d, s = inflight.pop(0)
            n = sum(d.collect(counts_only=True))
            if on_batch is not None:
                on_batch(d, s, self.offset(s))
            return n

        for s in range(step0, step0 + nsteps):
            d = self.dets[(s - step0) % ni]
            self._enqueue(d, s)
            inflight.append((d, s))
            if len(inflight) == ni:
                ndet += drain()
        while inflight:
            ndet += drain()
        return ndet
