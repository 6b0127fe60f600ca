#!/usr/bin/env python3
"""bench.py -- frames/s and p50 per-frame latency of 1280x720 AprilTag detection
on N MI355X (BASELINE.json metric; workload = configs[1], a single-camera
1280x720 tag36h11 synthetic stream).

A *step* is one launch sequence over a batch of B frames that are already
resident in HBM (see DESIGN.md "Measurement").  Each rank owns its own shard of
the stream (weak scaling, no data-path collective: frames are independent).
Four detector instances (one HIP stream and hardware queue each) are used
round-robin, so up to four batches are in flight: the latency-bound kernels of
one batch overlap those of the others, and the host tail (reconcile + sort by
id) of batch k overlaps the kernels of the later ones.

    python bench.py [--gpus N --steps K --warmup W --batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.  Latency: frames fed one at a time (B = 1) from
HBM to detections in host memory.  cpu_baseline: the C oracle
(oracle/ao_bench, restatement of the reference pipeline) on host cores.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec + p50 per-frame latency, 1280x720 AprilTag detect at 1/2/4/8 MI355X"
# The roofline's kernel, by a fixed rule rather than by the stage profile of the box
# (the top serialized stages are within ~10 % of each other and swap places between
# boxes): the kernel with the largest marginal cost in the concurrent bench loop --
# throughput with the launch sequence cut after each stage (AT_DIAG_PIPE_STOP,
# tools/r06_call.sh ABL=1), re-derived at HEAD and committed as ABLATION; every line
# reports that file's marginal costs and flags a DOMINANT that no longer matches it
# (tests/test_bench_cli.py checks the pair).
DOMINANT = "k_boundary"
ABLATION = "profiles/r06/ablation_720p.txt"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse(argv=None):
    """The bench's options; parse([]) gives the headline defaults (the parity test of the
    headline configuration, tests/test_stream_parity.py, takes them from here)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    # 192 frames per step: +3 % frames/s over 128 with four batches in flight (profiles/r04s,
    # r04t sweeps: 160 / 224 / 256 and 3 or 5 instances are not better)
    ap.add_argument("--batch", type=int, default=192, help="frames per step per GPU")
    ap.add_argument("--pool", type=int, default=64, help="distinct synthetic frames per GPU")
    ap.add_argument("--hbm-copies", type=int, default=None,
                    help="copies of the frame pool in HBM (default: at least 4 and two batches' worth, "
                         "6 x 64 frames = 0.71 GB at 720p and batch 192: more than the 256 MB Infinity "
                         "Cache, and consecutive steps read different frames, all from HBM)")
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--tags", type=int, default=15)
    ap.add_argument("--latency-frames", type=int, default=1000)
    ap.add_argument("--instances", type=int, default=4,
                    help="detector instances (one HIP stream each) used round-robin, i.e. batches in flight")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (HIP default 4): one hardware queue per "
                         "detector stream so the batches in flight run concurrently")
    ap.add_argument("--host-ingest-steps", type=int, default=20,
                    help="steps of the same loop fed from page-locked host frames (at_enqueue_host: H2D on the "
                         "detector streams), reported as host_ingest; 0 = skip")
    ap.add_argument("--c3-latency-iters", type=int, default=300,
                    help="config C3 latency: one batch of 4 camera frames (pageable host memory) -> detections, "
                         "p50 over this many batches; 0 = skip")
    ap.add_argument("--node-path-calls", type=int, default=300,
                    help="the deployed node's per-frame path, B=1: DetectorCore::process on bgr8 host frames "
                         "at 1920x1080 and 800x600 (node/at_mock_node --time), p50/p99 per call; 0 = skip")
    ap.add_argument("--isolated-batches", type=int, default=10,
                    help="batches per kernel of the isolated roofline pass (one batch in flight, each kernel of "
                         "the sequence timed on its own stream in turn); 0 = skip")
    ap.add_argument("--isolated-only", action="store_true",
                    help="only the isolated roofline pass (no concurrent loop): the command profiled by "
                         "rocprofv3 --kernel-trace for profiles/, every launch in the process serialized")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-profile", action="store_true")
    ap.add_argument("--timed-kernel", default=None,
                    help="kernel timed live for the roofline (default: the dominant one of the stage profile; "
                         "lets a traced run without the stage-profile pass time the same kernel)")
    ap.add_argument("--no-kernel-timer", action="store_true",
                    help="no HIP events around the dominant kernel (graph replay in the timed region)")
    ap.add_argument("--ingest", choices=["local", "scatter"], default="local",
                    help="local: every rank renders its own frames into its HBM (weak scaling, no data-path "
                         "collective); scatter: frames live on rank 0 and are scattered each step over RCCL "
                         "(north-star topology), detection records gathered back to rank 0")
    ap.add_argument("--scatter-leg-steps", type=int, default=None,
                    help="N > 1 with --ingest local: steps of the scatter leg run after the timed region (the "
                         "north-star topology, reported as scatter_leg; default = --steps; 0 = skip)")
    return ap.parse_args(argv)


def pool_copies(args):
    """Copies of the --pool frames resident per GPU: at least 4 and two batches' worth,
    so consecutive steps read different frames, all from HBM (rank 0's scatter pool per
    rank follows the same rule)."""
    if args.hbm_copies:
        return max(1, args.hbm_copies)
    return max(4, -(-2 * args.batch // args.pool))


STAGE_NAMES = ["k_pre", "k_thr_ccl", "k_ccl_merge", "k_ccl_roots", "k_boundary", "k_pairs", "k_group", "k_extents",
               "k_blob_small", "k_blob", "k_decode", "k_pose"]  # (at_common.h kStageNames)


def ablation_marginals(path=None):
    """Marginal ms per step of each stage from a stage-cut ablation file (lines
    `pipe_stop=N frames/s ms_per_step ...`: only the stages < N launched): the stage
    added by a cut at N over the previous cut is STAGE_NAMES[N - 1] (the stages between
    them are not launched in throughput mode: k_ccl_roots).  Returns ({stage: ms}, top)."""
    path = os.path.join(ROOT, path or ABLATION)
    ms = {}
    for line in open(path):
        f = line.split()
        if f and f[0].startswith("pipe_stop=") and len(f) >= 3:
            n = int(f[0].split("=")[1])
            if n > 0:
                ms[n] = float(f[2])
    out, prev = {}, 0.0
    for n in sorted(ms):
        out[STAGE_NAMES[n - 1]] = round(ms[n] - prev, 4)
        prev = ms[n]
    return out, max(out, key=out.get)


def kernel_algorithmic_bytes(kernel, stats, W, H):
    """Algorithmic bytes one launch of `kernel` must move, from the
    batch's work counts."""
    nf = stats.get("frames", 0)
    Wd, Hd = W // 2, H // 2
    if kernel == "k_pre":
        return nf * (2 * W * H + W * H + Wd * Hd)           # YUYV in, gray + decimated out
    if kernel == "k_boundary":
        # thr (1 B per decimated pixel) + the parent words (3 words per 2x2 block: 3 B per
        # pixel) in; points out as the 4-B (pair entry, point bits) words of narrow tiles
        return nf * 4 * Wd * Hd + 4 * stats.get("boundary_points", 0)
    if kernel == "k_blob":  # kept blobs: the 8-B sort key of every point (the line-fit weight W rides in it)
        return 8 * stats.get("large_blob_points", 0)
    if kernel == "k_blob_small":
        return 8 * stats.get("small_blob_points", 0)
    if kernel == "k_extents":  # candidate points read (bounded by all boundary points), kept points' keys written
        return 8 * stats.get("boundary_points", 0) + 8 * (stats.get("small_blob_points", 0) +
                                                          stats.get("large_blob_points", 0))
    if kernel == "k_thr_ccl":  # dec in; thr and parent words (3 per 2x2 block) out; lists (id, count), descriptors out
        tiles = ((Wd + 63) // 64) * ((Hd + 31) // 32)
        return nf * 5 * Wd * Hd + 8 * stats.get("ccl_listed_roots", 0) + nf * tiles * 704
    if kernel == "k_ccl_border":  # per 32x32 tile: 47 border blocks, thr bytes + parent words
        return nf * ((Wd + 31) // 32) * ((Hd + 31) // 32) * 47 * 16
    if kernel == "k_ccl_merge":  # border descriptors (704 B per 64x32 tile) + listed roots (id, count) in, words out
        return nf * ((Wd + 63) // 64) * ((Hd + 31) // 32) * 704 + 12 * stats.get("ccl_listed_roots", 0)
    if kernel == "k_pose":  # per candidate detection: H + corners in, R, t, errors out
        return stats.get("candidates", 0) * (72 + 64 + 112)
    return None


def isolated_kernel_times(det, batch_ptr, stride, B, nbatches):
    """Every kernel of the launch sequence on its own: one batch in flight (enqueue,
    collect), the kernel timer on one kernel at a time (the sequence as three graphs
    cut around it), two warm-up batches, then `nbatches` timed.  {kernel: (device-clock
    span ms, HIP-event ms, launches, batch stats)} -- the kernel's duration when it
    has the chip, which a rocprofv3 kernel trace reproduces (tracing does not change
    a serialized launch; it does change how concurrent batches interleave)."""
    from ros_vision_amd import detector
    L = detector.load_library()
    names = []
    for i in range(32):
        nm = L.at_stage_name(i)
        if not nm:
            break
        names.append(nm.decode())
    out = {}
    s = 0
    for k in names:
        try:
            det.set_kernel_timer(k)
        except Exception:
            continue
        for _ in range(2):
            det.enqueue_device(batch_ptr(s), stride, B)
            det.collect(counts_only=True)
            s += 1
        det.set_kernel_timer(k)  # reset the accumulators
        for _ in range(nbatches):
            det.enqueue_device(batch_ptr(s), stride, B)
            det.collect(counts_only=True)
            s += 1
        span, nspan = det.kernel_span()
        ev, nev = det.kernel_time()
        if nspan > 0 and span > 0:
            out[k] = (span, ev, nspan, det.batch_stats())
    det.set_kernel_timer(None)
    return out


def isolated_table(iso, W, H):
    """isolated_kernel_times -> [{kernel, ms, algorithmic bytes, achieved, frac}], longest first."""
    rows = []
    for k, (span, ev, n, st) in sorted(iso.items(), key=lambda kv: -kv[1][0]):
        kb = kernel_algorithmic_bytes(k, st, W, H)
        gbs = kb / (span * 1e-3) / 1e9 if kb else None
        rows.append({"kernel": k, "avg_launch_ms_device_clock": round(span, 5), "avg_launch_ms_hip_events": round(ev, 5),
                     "launches": n, "algorithmic_bytes_per_launch": kb,
                     "achieved": round(gbs, 3) if gbs else None,
                     "frac": round(gbs / HBM_PEAK_GBS, 6) if gbs else None})
    return rows


def pmc_traffic(W, H):
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        tj = json.load(open(tpath))
        if tj.get("width") == W and tj.get("height") == H:
            return tj
    except Exception:
        pass
    return None


def render_pool(args, rank):
    from ros_vision_amd.stream import stream_pool
    return stream_pool(args.width, args.height, args.pool, args.tags, rank)


def host_cpus():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(period))))
    except Exception:
        pass
    return (min(affinity, quota) if quota else affinity), affinity, quota


def cpu_baseline(frames, width, height):
    """Time the C oracle on this host (rank 0, N=1 only): ~20-30 s of CPU work.

    Built here with -O3 -march=native (the host's own ISA), one frame
    stream per usable host CPU for throughput, 1,000 frames single-threaded for
    latency (p50)."""
    threads, affinity, quota = host_cpus()
    nf = min(16, frames.shape[0])
    tmpdir = tempfile.mkdtemp(prefix="ao_bench_")
    exe = os.path.join(tmpdir, "ao_bench")
    od = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-O3", "-march=native", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-D_GNU_SOURCE",
                    "-o", exe, os.path.join(od, "ao_bench.c"), os.path.join(od, "ao_oracle.c"),
                    os.path.join(od, "ao_pose.c"), "-lm", "-lpthread"], check=True, timeout=300)
    path = os.path.join(tmpdir, "frames.raw")
    frames[:nf].tofile(path)
    try:
        lat_iters, thr_iters = 1000, 30
        out = subprocess.run([exe, path, str(width), str(height), str(nf), str(lat_iters), str(thr_iters),
                              str(threads)], check=True, capture_output=True, text=True, timeout=900).stdout
    finally:
        for f in (path, exe):
            if os.path.exists(f):
                os.unlink(f)
        os.rmdir(tmpdir)
    r = json.loads(out.strip().splitlines()[-1])
    return {"value": round(r["throughput_fps"], 3), "unit": "frames/s", "cores": r["threads"],
            "kind": "port", "p50_ms_1thread": round(r["p50_ms"], 3), "p99_ms_1thread": round(r["p99_ms"], 3),
            "host_cpus_affinity": affinity, "host_cpu_quota": quota, "build": "gcc -O3 -march=native",
            "sample": "C oracle (restatement of the reference pipeline incl. decode), %d distinct 1280x720 "
                      "synthetic frames: %d frames single-thread for latency, %d threads x %d frames for "
                      "throughput (threads = affinity mask %d capped by the cgroup CPU quota %s)"
                      % (nf, lat_iters, r["threads"], thr_iters, affinity, quota)}


def node_path_latency(calls):
    """The path the ROS 2 node runs per image (apriltags_cuda_detector.cu:382-557, what
    its measurement_mode CSV times): DetectorCore::process on a bgr8 host frame --
    at_detect (the frame to HBM, BGR -> luma on the GPU, detection, poses), robot frame,
    distance sort, TagDetectionArray / NetworkTables / ApriltagListProto payloads, and the
    outlined image drawn on the GPU and copied out (at_annotate_staged) -- at the
    deployed geometries of system_config.json (1920x1080; 800x600: 400x300 decimated,
    partial tiles).  Runs node/at_mock_node (a child process) on 4 rendered frames."""
    from ros_vision_amd import synth
    exe = os.path.join(ROOT, "node", "at_mock_node")
    if not os.path.exists(exe) or calls <= 0:
        return None
    out = {}
    for (W, H, ntags) in ((1920, 1080, 24), (800, 600, 8)):
        frames = []
        for k in range(4):
            g, _ = synth.render_board(W, H, seed=5150 + 7 * k + W, ntags=ntags, side_range=(48, 96))
            frames.append(np.repeat(g[:, :, None], 3, axis=2))  # bgr8 (gray board in every channel)
        fd, path = tempfile.mkstemp(prefix="node_frames_", suffix=".bgr")
        os.close(fd)
        try:
            np.stack(frames).tofile(path)
            r = subprocess.run([exe, "--width", str(W), "--height", str(H), "--format", "bgr8", "--frames", path,
                                "--time", str(calls)], capture_output=True, text=True, timeout=300)
            lines = [l for l in r.stdout.splitlines() if l.startswith('{"timing"')]
            if r.returncode == 0 and lines:
                out["%dx%d" % (W, H)] = json.loads(lines[-1])["timing"]
            else:
                out["%dx%d" % (W, H)] = {"error": (r.stderr or "no output")[-200:]}
        finally:
            os.unlink(path)
    return out


def main():
    args = parse()
    # several detector instances (batches in flight) each own a HIP stream: give the
    # process one hardware queue per stream; must precede HIP runtime initialisation
    os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    # stdout carries exactly one JSON line: libraries that print banners to fd 1
    # (RCCL prints its version block at communicator init) are sent to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch  # device memory + torch.distributed; loads the HIP runtime first
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    if world > 1 or args.ingest == "scatter":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local_rank))

    import ros_vision_amd as rva
    from ros_vision_amd import multigpu
    from ros_vision_amd.stream import StreamRunner
    W, H, B = args.width, args.height, args.batch
    scatter = args.ingest == "scatter"
    frames = render_pool(args, rank)
    copies = pool_copies(args)
    d_frames = torch.from_numpy(frames).to("cuda").repeat(copies, 1, 1).contiguous()
    stride = frames[0].nbytes
    base = d_frames.data_ptr()
    npool = args.pool * copies
    assert npool >= B, "the frames resident per GPU (--pool x --hbm-copies) must hold one batch"
    # (peers of a scatter run, or of the N > 1 line's scatter leg, send their records
    # from a page-locked output buffer)
    dets = [rva.GpuDetector(W, H, max_batch=B, device=local_rank, pinned_out=scatter or world > 1)
            for _ in range(args.instances)]
    rec_cap = 32  # detection records per frame in the fixed-size message; more follow in the overflow one
    rec_bytes = rec_cap * ctypes.sizeof(rva.detector.AtDetection)
    topo = {}    # the scatter topology's ingest / gather (set up on first use)

    def setup_scatter():
        """rank 0 holds every rank's frame pool in its HBM; each step sends B frames to
        every peer (multigpu.ScatterIngest), records return by multigpu.RecordGather"""
        if topo:
            return topo["ingest"], topo["gather"]
        root_pool = None
        mine = torch.from_numpy(frames).to("cuda")
        # every rank's rendered pool to rank 0 (set-up, untimed: one send per peer instead
        # of rank 0 rendering them all)
        if rank == 0:
            root_pool = torch.empty((world, npool) + frames.shape[1:], dtype=torch.uint8, device="cuda")
            root_pool[0] = mine.repeat(copies, 1, 1)
            for r in range(1, world):
                dist.recv(mine, src=r)
                root_pool[r] = mine.repeat(copies, 1, 1)
        else:
            dist.send(mine, dst=0)
        del mine
        topo["ingest"] = multigpu.ScatterIngest(dist, root_pool, B, frames.shape[1:], "cuda", nbuf=args.instances)
        topo["gather"] = multigpu.RecordGather(dist, B, rec_bytes, "cuda")
        return topo["ingest"], topo["gather"]

    ingest = gather = None
    if scatter:
        ingest, gather = setup_scatter()

    runner = StreamRunner(dets, base, stride, npool, B)

    def batch_ptr(step):
        return base + runner.offset(step) * stride

    def run(nsteps, step0=0):
        """Round-robin over the detector instances: enqueue k, collect k-(instances-1)
        (ros_vision_amd/stream.py; tests/test_stream_parity.py checks this loop's output)."""
        if scatter:
            return run_scatter(nsteps, step0)
        return runner.run(nsteps, step0)

    def run_scatter(nsteps, step0):
        """multigpu.ScatterLoop: frames from rank 0, records back to rank 0."""
        ingest, gather = setup_scatter()
        if "loop" not in topo:
            topo["loop"] = multigpu.ScatterLoop(dist, dets, ingest, gather, B, stride, rec_cap)
        return topo["loop"].run(nsteps, step0)

    if args.isolated_only:  # (the rocprofv3 command of profiles/: every launch serialized)
        iso = isolated_kernel_times(dets[0], batch_ptr, stride, B, max(1, args.isolated_batches))
        if rank == 0:
            print(json.dumps({"mode": "isolated-only", "batch": B, "width": W, "height": H,
                              "isolated": isolated_table(iso, W, H)}), file=json_out, flush=True)
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
        return

    run(max(1, args.warmup))

    # per-stage GPU time (HIP events between the kernels, serialized launch
    # sequence) -- identifies the dominant kernel before the timed region
    stages, stage_batches = {}, 0
    if not args.no_stage_profile:
        prof = dets[0]
        prof.set_profiling(True)
        for s in range(10):
            prof.enqueue_device(batch_ptr(s), stride, B)
            prof.collect()
        stages, stage_batches = prof.stage_times()
        prof.set_profiling(False)
    dominant = args.timed_kernel or DOMINANT
    # live per-launch time of the dominant kernel inside the timed region
    ktimer = None if args.no_kernel_timer else dominant
    for d in dets:
        d.set_kernel_timer(ktimer)
    run(1)
    for d in dets:
        d.set_kernel_timer(ktimer)  # reset the accumulators

    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host0 = [d.batch_stats() for d in dets]
    gathered0 = gather.records_received if scatter else 0
    ndet = run(args.steps, step0=args.warmup)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    host1 = [d.batch_stats() for d in dets]
    kt = [d.kernel_time() for d in dets] if ktimer else [(0.0, 0)]
    k_launches = sum(n for _, n in kt)
    k_ms_events = sum(ms * n for ms, n in kt) / max(1, k_launches)
    ks = [d.kernel_span() for d in dets] if ktimer else [(0.0, 0)]
    k_spans = sum(n for _, n in ks)
    k_ms_span = sum(ms * n for ms, n in ks) / max(1, k_spans)
    # the kernel's execution span on the device clock (what rocprofv3's kernel trace
    # reports); the HIP-event bracket also holds the launch's wait for free CUs
    # behind the other batches in flight
    k_ms = k_ms_span if k_spans else k_ms_events
    # scatter: the detection records rank 0 holds after the timed region (its own + every
    # peer's, overflow included) -- equal to the detections of all ranks
    records_at_root = (ndet + gather.records_received - gathered0) if (scatter and rank == 0) else None
    stats = dets[0].batch_stats()
    for d in dets:
        d.set_kernel_timer(None)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nd = torch.tensor([ndet], dtype=torch.float64, device="cuda")
        dist.all_reduce(nd, op=dist.ReduceOp.SUM)
        ndet = int(nd.item())
    total_frames = world * args.steps * B
    fps = total_frames / elapsed

    # N > 1 with local ingest: the north-star topology beside the headline, so a 1->8
    # run measures it too -- frames from rank 0 over RCCL, records back to rank 0
    scatter_leg = None
    leg_steps = args.steps if args.scatter_leg_steps is None else args.scatter_leg_steps
    if world > 1 and not scatter and leg_steps > 0:
        _, leg_gather = setup_scatter()
        run_scatter(len(dets), 0)  # warm-up: buffers, the gather's communicator
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        recv0 = leg_gather.records_received
        nd_leg = run_scatter(leg_steps, step0=len(dets))
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        leg_el = time.perf_counter() - t1
        at_root = nd_leg + leg_gather.records_received - recv0 if rank == 0 else None
        leg_el, leg_det = multigpu.reduce_max_sum(dist, leg_el, nd_leg, "cuda")
        scatter_leg = multigpu.scatter_leg_summary(world, leg_steps, B, stride, leg_el, leg_det, at_root)

    # every kernel on its own (one batch in flight): the headline roofline kernel is
    # the one with the longest isolated launch
    iso = isolated_kernel_times(dets[0], batch_ptr, stride, B, args.isolated_batches) \
        if (args.isolated_batches > 0 and not args.no_kernel_timer) else {}

    # per-frame latency, one frame at a time (B = 1), detections in host memory:
    # from a (pageable) host frame as the node feeds it, and from
    # a frame already resident in HBM
    lat_h, lat_d = [], []
    if args.latency_frames > 0:
        lat_det = rva.GpuDetector(W, H, max_batch=1, device=local_rank)
        for i in range(10):
            lat_det.detect_count(frames[i % args.pool])
            lat_det.detect_device(base + (i % npool) * stride, stride, 1, counts_only=True)
        for i in range(args.latency_frames):
            fr = frames[i % args.pool]
            t1 = time.perf_counter()
            lat_det.detect_count(fr)
            lat_h.append(time.perf_counter() - t1)
            t1 = time.perf_counter()
            lat_det.detect_device(base + (i % npool) * stride, stride, 1, counts_only=True)
            lat_d.append(time.perf_counter() - t1)
    lat_h = np.array(lat_h or [0.0]) * 1e3
    lat_d = np.array(lat_d or [0.0]) * 1e3

    # config C3 (4 cameras, one batch per launch sequence): 4 host frames -> detections
    lat_c3 = []
    if args.c3_latency_iters > 0:
        c3 = rva.GpuDetector(W, H, max_batch=4, device=local_rank)
        cams = [np.ascontiguousarray(frames[(7 * c) % args.pool]) for c in range(4)]
        for i in range(10):
            c3.detect_batch(cams)
        for i in range(args.c3_latency_iters):
            t1 = time.perf_counter()
            c3.detect_batch(cams)
            lat_c3.append(time.perf_counter() - t1)
        c3.close()
    lat_c3 = np.array(lat_c3 or [0.0]) * 1e3

    # the same loop fed from page-locked host frames: what a camera-fed GPU sustains
    host_ingest = None
    if args.host_ingest_steps > 0 and not scatter:
        pinned = torch.from_numpy(frames).pin_memory()
        hrun = StreamRunner(dets, pinned.data_ptr(), stride, args.pool, B, host=True)
        hrun.run(len(dets))
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
        t1 = time.perf_counter()
        hrun.run(args.host_ingest_steps)
        torch.cuda.synchronize()
        h_el = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([h_el], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            h_el = float(t.item())
        h_fps = world * args.host_ingest_steps * B / h_el
        host_ingest = {"value": round(h_fps, 2), "unit": "frames/s", "steps": args.host_ingest_steps,
                       "h2d_GBps_per_gpu": round(h_fps / world * stride / 1e9, 2),
                       "note": "frames in page-locked host memory, copied H2D on the detector streams "
                               "(at_enqueue_host) while other batches compute; bounded by the host-to-device link"}
        del pinned

    if rank != 0:
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
        return

    per_gpu_fps = fps / world
    pipe_ms = sum(stages.values()) if stages else None
    pmc = pmc_traffic(W, H)

    def traffic_per_launch(kernel):
        """PMC bytes of one launch of `kernel` (FETCH x2 (gfx950 correction) + WRITE per
        frame, profiles/pmc_traffic.json, x the batch)."""
        kk = [v for k, v in (pmc or {}).get("kernels", {}).items() if k.split("<")[0] == kernel]
        return round(B * sum(2 * v["fetch_bytes_per_frame"] + v["write_bytes_per_frame"] for v in kk)) if kk else None

    # headline roofline: the DOMINANT kernel (fixed rule: the largest marginal cost in
    # the concurrent loop) with its launch measured in isolation (one batch in flight),
    # its device-clock span in this run; the longest isolated kernel is named beside it
    iso_rows = isolated_table(iso, W, H)
    try:
        marg, abl_top = ablation_marginals()
        ablation = {"file": ABLATION, "marginal_ms_per_step": marg, "top_stage": abl_top,
                    "dominant_changed": abl_top != DOMINANT,
                    "note": "stage-cut ablation at the bench configuration (%d instances x %d frames, 720p): "
                            "ms per step added by each stage; DOMINANT is its top stage" % (4, 192)}
    except OSError:
        ablation = None
    head = next((r for r in iso_rows if r["kernel"] == dominant), None)
    longest = iso_rows[0]["kernel"] if iso_rows else None
    # concurrent: the DOMINANT kernel timed inside the timed region (four batches in flight)
    kbytes = kernel_algorithmic_bytes(dominant, stats, W, H)
    k_achieved = kbytes / (k_ms * 1e-3) / 1e9 if (kbytes and k_ms > 0) else None
    pipe_bytes = 3 * W * H  # read YUYV 2WH + write gray WH
    top_stage = max(stages, key=stages.get) if stages else None
    if head:
        roofline = {"bound": "hbm", "kernel": head["kernel"], "achieved": head["achieved"], "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": head["frac"], "traffic": traffic_per_launch(head["kernel"]),
                    "algorithmic_bytes_per_launch": head["algorithmic_bytes_per_launch"],
                    "avg_launch_ms": head["avg_launch_ms_device_clock"],
                    "avg_launch_ms_hip_events": head["avg_launch_ms_hip_events"], "launches_timed": head["launches"],
                    "longest_isolated_kernel": longest, "differs_from_longest_isolated": longest != head["kernel"],
                    "isolated": iso_rows,
                    "note": "DOMINANT (fixed rule: the largest marginal cost in the concurrent loop, "
                            "%s, see `ablation`) measured in isolation in this run: one batch of "
                            "%d frames in flight (enqueue, collect), the kernel timer on one kernel at a time, "
                            "avg_launch_ms = its execution span on the device wall clock (first workgroup start "
                            "to last workgroup end, at_kernel_span: what a rocprofv3 kernel trace reports; "
                            "`bench.py --isolated-only` under rocprofv3 --kernel-trace reproduces it, "
                            "profiles/); algorithmic bytes per DESIGN.md section 4; traffic = PMC "
                            "(2*FETCH_SIZE+WRITE_SIZE) per launch from profiles/pmc_traffic.json; `isolated`: "
                            "every kernel the same way, longest first (the top three are within ~10 %% of each "
                            "other and change places between boxes)" % (ABLATION, B)}
    else:
        roofline = None
    roofline_concurrent = {
        "bound": "hbm", "kernel": dominant, "achieved": round(k_achieved, 3) if k_achieved else None,
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(k_achieved / HBM_PEAK_GBS, 6) if k_achieved else None,
        "traffic": traffic_per_launch(dominant), "algorithmic_bytes_per_launch": kbytes,
        "avg_launch_ms": round(k_ms, 5), "launches_timed": k_launches,
        "avg_launch_ms_device_clock": round(k_ms_span, 5), "launches_device_clock": k_spans,
        "avg_launch_ms_hip_events": round(k_ms_events, 5),
        "frac_hip_events": round(kbytes / (k_ms_events * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)
        if (kbytes and k_ms_events > 0) else None,
        "top_serialized_stage": top_stage, "differs_from_top_serialized_stage": bool(top_stage and top_stage != dominant),
        "note": "DOMINANT (fixed rule: the largest marginal cost in the concurrent loop, " + ABLATION + ") "
                "timed on every launch of the timed region with %d batches in flight: its span there holds the "
                "other batches' kernels sharing the CUs (co-residency), and a tracer changes how the batches "
                "interleave, so this figure is not reproducible under rocprofv3; top_serialized_stage = the "
                "largest stage of this run's stage profile" % args.instances}
    out = {
        "metric": METRIC,
        "value": round(fps, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": ("configs[1]: 1280x720 single-camera synthetic tag36h11 stream "
                                "(%d tags/frame, YUYV, frames resident in HBM)" % args.tags)
                               if (W, H) == (1280, 720) else
                               ("configs[3] geometry: %dx%d synthetic tag36h11 frames (%d tags/frame, YUYV, "
                                "frames resident in HBM), one GPU" % (W, H, args.tags)),
                   "width": W, "height": H, "batch_per_gpu": B, "distinct_frames_per_gpu": args.pool,
                   "frames_resident_per_gpu": npool,
                   "parallelism": ("frame-sharded x%d, frames scattered from rank 0 over RCCL, records gathered "
                                   "to rank 0" % world) if scatter else
                                  "frame-sharded x%d (no data-path collective)" % world,
                   "ingest": "scatter" if scatter else "local"},
        "p50_latency_ms": round(float(np.percentile(lat_h, 50)), 4),
        "p99_latency_ms": round(float(np.percentile(lat_h, 99)), 4),
        "latency_note": "B=1, pageable host YUYV frame -> detections + poses in host memory",
        "p50_latency_hbm_ms": round(float(np.percentile(lat_d, 50)), 4),
        "p99_latency_hbm_ms": round(float(np.percentile(lat_d, 99)), 4),
        "p50_latency_c3_ms": round(float(np.percentile(lat_c3, 50)), 4),
        "p99_latency_c3_ms": round(float(np.percentile(lat_c3, 99)), 4),
        "latency_c3_note": "config C3: one batch of 4 camera frames (pageable host YUYV) -> detections + poses",
        "host_ingest": host_ingest,
        "detections_per_frame": round(ndet / total_frames, 3),
        "records_at_rank0": records_at_root,
        "scatter_leg": scatter_leg,
        "roofline": roofline,
        "roofline_concurrent": roofline_concurrent,
        "roofline_pipeline": {"bound": "hbm", "achieved": round(per_gpu_fps * pipe_bytes / 1e9, 3),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(per_gpu_fps * pipe_bytes / 1e9 / HBM_PEAK_GBS, 6),
                              "traffic": pmc.get("hbm_bytes_per_frame") if pmc else None,
                              "bytes_per_frame": pipe_bytes,
                              "note": "SURVEY.md 8(d): per-GPU frames/s x 3*W*H; traffic = PMC bytes per frame"},
        "batch_stats": stats,
        "host_us_per_step": {k: round(sum(b[k] - a[k] for a, b in zip(host0, host1)) / args.steps, 1)
                             for k in ("host_wait_us_total", "host_tail_us_total")},
        "stage_ms_per_batch": {k: round(v, 4) for k, v in stages.items()},
        "dominant_kernel": dominant,
        "ablation": ablation,
        "pipeline_gpu_ms_per_batch": round(pipe_ms, 4) if pipe_ms else None,
        "cpu_baseline": None,
    }
    if world == 1 and args.node_path_calls > 0:
        try:
            out["node_path_latency"] = node_path_latency(args.node_path_calls)
        except Exception as e:  # reported, never fatal for the GPU number
            out["node_path_latency"] = {"error": str(e)[:200]}
    if world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(frames, W, H)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": str(e)[:200]}
    print(json.dumps(out), file=json_out, flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
