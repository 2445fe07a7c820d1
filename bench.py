#!/usr/bin/env python3
"""bench.py — TULIPS checksum path on MI355X: device-resident GiB/s.

Metric (BASELINE.json): "GiB/s checksummed (device-resident), batched 1500 B
and 9000 B segments". Algorithmic bytes = sum of segment lengths.

Workload (one "step" = one pass of the hot path over one batch):
  configs[1] of BASELINE.json — a 65,536-segment batch of fixed 1500 B
  segments, device-resident, checksummed by the gfx950 kernel through the
  C ABI (tulips_csum_batch_fixed). Each rank holds 16 such batches
  (1,048,576 segments = 1.57 GB, i.e. shard <rank> of the M8x1500 config,
  configs[4]) and steps rotate through them, so every step streams from HBM
  rather than from the 256 MB Infinity Cache. Per-rank work is fixed as N
  grows (weak scaling); no data-path collective: segments are independent.

Also reported (N=1, rank 0): F9000 (configs[2]) and ZIPF (configs[3]) rates,
the plain streaming-read ceiling on the same buffer, the end-to-end host path
(pinned H2D + kernel + D2H), and the reference CPU checksum timed on this
box's cores (cpu_baseline).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N>1 runs one rank per GPU: under `python -m torch.distributed.run
       --nproc-per-node N ...`, or, with no launcher (WORLD_SIZE unset), this
       script starts that launcher itself as a child process (before any GPU
       call), relays its output and exits with its status.

Parity of the measured work: the result buffers are poisoned (0xA5 bytes)
before every timed replay and the digests of what the replay wrote are
compared with the reference's afterwards (per batch, tests/golden).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s checksummed (device-resident), batched 1500 B and 9000 B segments"
GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E nameplate, GB/s (MI355X_MICROARCH.md)
SEG, NSEG = 1500, 65536        # configs[1]
NBATCH = 16                    # batches per rank = one M8x1500 shard
DATA_SEED = 0x54554C495053
ZIPF_SEED, ZIPF_RMAX = 0x5A495046, 8937


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1024)
    p.add_argument("--warmup", type=int, default=32)
    p.add_argument("--no-extras", action="store_true",
                   help="skip F9000/ZIPF/e2e/ceiling side measurements")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=1.5,
                   help="wall seconds per CPU-baseline leg")
    p.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                   help="torch.distributed backend for N>1 (nccl = RCCL)")
    p.add_argument("--one-device", action="store_true",
                   help="rehearsal only: every rank uses cuda:0 (use with gloo)")
    p.add_argument("--extras-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--mctx-child", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--streams", type=int, default=0,
                   help="independent graph branches the timed steps round-robin over "
                        "(batches are independent). 0 = by step count (branches_for): "
                        "2 below 128 steps, else 16 (four per hardware queue, "
                        "GPU_MAX_HW_QUEUES being 4 on the box; "
                        "profiles/probe_branches_r03.txt, profiles/probe_graph_k_r04.txt)")
    p.add_argument("--main-branch", type=int, default=0, choices=(0, 1),
                   help="1: the timed graph's capture stream carries one of its branches "
                        "(one fork and join fewer per replay)")
    p.add_argument("--start-delay-us", type=int, default=200,
                   help="a one-wave GPU sleep queued before every timed region's start "
                        "event (not timed), so the region starts on the GPU only once the "
                        "host has submitted its graph: host launch latency is not counted "
                        "as checksum time (0 = off)")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher and process-group check only (no GPU work): ranks form "
                        "the group, assert its size and rank 0 prints the JSON line "
                        "without measurements")
    p.add_argument("--eager", action="store_true",
                   help="launch every step from Python instead of replaying a "
                        "captured HIP graph of one shard rotation (16 launches); "
                        "eager Python launches (~19 us each) cannot keep up "
                        "with a ~17 us kernel")
    return p.parse_args()


def zipf_lengths(n, seed=ZIPF_SEED, rmax=ZIPF_RMAX):
    """SURVEY.md §8c Zipf lengths (data generation for the ZIPF side run)."""
    golden = 0x9E3779B97F4A7C15
    mask = (1 << 64) - 1
    c = np.cumsum(np.arange(1, rmax + 1, dtype=np.float64) ** -1.1)
    # sequential summation as in the spec (np.cumsum is sequential)
    s = np.uint64(seed)
    k = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = s + k * np.uint64(golden)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    del mask
    u = (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    r = np.searchsorted(c, u * c[-1], side="left") + 1
    return (63 + r).astype(np.uint16)


def fnv1a_u16(v: np.ndarray) -> str:
    h = 0xCBF29CE484222325
    b = np.ascontiguousarray(v, dtype="<u2").view(np.uint8)
    prime = 0x100000001B3
    mask = (1 << 64) - 1
    for x in b.tobytes():
        h = ((h ^ x) * prime) & mask
    return f"{h:016x}"


def golden_rotations():
    """Reference digests of the distinct batches the side measurements
    rotate over (tests/golden/make_golden.py rotation_digests)."""
    path = os.path.join(ROOT, "tests", "golden", "digests.json")
    try:
        with open(path) as f:
            return json.load(f).get("rotations", {})
    except OSError:
        return {}


def golden_digests():
    path = os.path.join(ROOT, "tests", "golden", "digests.json")
    try:
        with open(path) as f:
            return json.load(f)["batches"]
    except OSError:
        return {}


START_DELAY_US = 200   # bench --start-delay-us
# launches in the serial chain the roofline's per-launch duration comes from,
# whatever --steps is: one graph replay costs ~10 us on top of its launches
# (profiles/probe_graph_k_r04.txt), 0.5 us per launch over the driver's 20.
# The median of 5 timed replays of that chain is taken: right after a short
# run (the driver's 20 steps) the first replay measured 16.5-16.6 us per
# launch where the steady state, and rocprofv3's serial bursts, give 16.1-16.3
SERIAL_LAUNCHES = 256


def branches_for(steps):
    """Graph branches for a K-step timed replay. A replay costs about a + b K
    (tools/sessions/probes/probe_graph_k.py, profiles/probe_graph_k_r04.txt, one box; b from
    K = 4..64): 1 branch a = 10 us, b = 15.6 us; 2 branches a = 24 us,
    b = 13.47 us; 4-16 branches a = 39-40 us, b = 13.36-13.41 us. The
    per-replay cost grows with the hardware queues the graph spans, so 2
    branches win the short replays: the driver's K = 20 at 6,224-6,268 GiB/s
    against 5,860-5,955 with 16 (3 alternations, profiles/ab_branches_k_r04.txt),
    and K = 64 at 6,608 against 6,538. Long chains on 2 branches lose pace
    (K = 1,024: 6,368 against 6,743 with 16), so 16 from K = 128 on."""
    return 2 if steps < 128 else 16


def gate(stream):
    """Queue the untimed start delay (tulips_csum_gpu_sleep) on `stream`."""
    if START_DELAY_US > 0:
        from tulips_amd import csum
        rc = _bench().lib.tulips_csum_gpu_sleep(START_DELAY_US, stream.cuda_stream)
        if rc:
            raise csum.CsumError(rc, "tulips_csum_gpu_sleep")


def _bench():
    """The measurement library (benchlib/, include/tulips_csum_bench.h): the
    device data fill, the ceiling kernels, the start-delay sleep."""
    import benchlib
    return benchlib


class CheckedLib:
    """csum.lib with every status-returning call checked: a non-zero status
    raises CsumError at the call, which also ends a graph capture in progress
    (torch.cuda.graph's exit), so no capture can silently miss a launch.
    Names the product does not export (the ceiling kernels) resolve in the
    measurement library."""

    def __init__(self, csum):
        self._csum = csum

    def __getattr__(self, name):
        try:
            f = getattr(self._csum.lib, name)
        except AttributeError:
            f = getattr(_bench().lib, name)
        err = self._csum.CsumError

        def call(*a):
            rc = f(*a)
            if rc:
                raise err(rc, name)
            return rc
        setattr(self, name, call)
        return call


_CHECKED = None


def checked_lib(csum):
    global _CHECKED
    if _CHECKED is None:
        _CHECKED = CheckedLib(csum)
    return _CHECKED


class Timer:
    """Seconds per launch, from HIP events on the stream the kernels run on.

    With graph=True the `reps` launches are first captured into one HIP graph
    and the replay is timed, so host-side launch cost (ctypes + hipLaunch,
    several us) cannot leave the GPU idle between short kernels; the events
    still bracket exactly the kernels' execution on that stream.
    fn(i, stream_handle) must enqueue launch i on stream_handle.
    """

    def __init__(self, torch, stream, graph=True):
        self.torch, self.stream, self.graph = torch, stream, graph
        # the capture stream and the branch streams, made once and reused by
        # every call (not drawn again from torch's recycled pool per call)
        self._streams = []
        # every graph this timer captured, kept alive until the process ends:
        # the HIP runtime torch bundles can crash in hipGraphLaunch after a
        # multi-branch graph was destroyed (DESIGN.md §8,
        # tools/probe_graph_churn.py), and no launch follows the teardown
        self._kept = []

    def streams(self, k):
        while len(self._streams) < k:
            self._streams.append(self.torch.cuda.Stream())
        return self._streams[:k]

    def __call__(self, fn, reps, branches=1, replays=1, poison=None):
        """branches > 1: launch i goes to graph branch i % branches (independent
        launches overlap); the result is then time per launch of the pipeline.
        replays > 1 (graph only): the captured graph is replayed that many
        times, each timed on its own, and the median is returned.
        poison(): overwrites the launches' outputs after every untimed launch
        (capture warm-up, warm replay) and before the timed replay(s), so what
        the caller checks afterwards was written inside the timed region."""
        t = self.torch
        a, b = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        g = None
        if self.graph:
            g = t.cuda.CUDAGraph()
            ss = self.streams(1 + (branches if branches > 1 else 0))
            cap, side = ss[0], ss[1:]
            # one eager launch on every stream the capture uses first (the
            # library needs none: a captured call gets state of its own)
            for j, sd in enumerate([cap] + side):
                fn(j, sd.cuda_stream)
            t.cuda.synchronize()
            with t.cuda.graph(g, stream=cap):
                main = t.cuda.current_stream()
                for sd in side:
                    sd.wait_stream(main)
                for i in range(reps):
                    fn(i, side[i % branches].cuda_stream if side else main.cuda_stream)
                for sd in side:
                    main.wait_stream(sd)
            g.replay()                      # warm replay
            self._kept.append(g)
        t.cuda.synchronize()
        if poison is not None:
            poison()
            t.cuda.synchronize()
        if g is not None and replays > 1:
            times = []
            for _ in range(replays):
                gate(self.stream)
                a.record(self.stream)
                g.replay()
                b.record(self.stream)
                b.synchronize()
                times.append(a.elapsed_time(b) / 1e3 / reps)
            return float(np.median(times))
        gate(self.stream)
        a.record(self.stream)
        if g is not None:
            g.replay()
        else:
            for i in range(reps):
                fn(i, self.stream.cuda_stream)
        b.record(self.stream)
        b.synchronize()
        return a.elapsed_time(b) / 1e3 / reps  # seconds per launch


def self_launch(args):
    """--gpus N > 1 without a launcher: run this script under
    torch.distributed.run with N ranks as a CHILD process (no exec: nothing
    here has touched the GPU, and the child owns its own HIP state), stream
    its output through and return its exit status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def progress(stage):
    """One stderr line per bench stage (stdout carries only the JSON line):
    where a long run is, and where it stopped if it dies."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {stage}", file=sys.stderr, flush=True)


def main():
    global START_DELAY_US
    import faulthandler
    faulthandler.enable(file=sys.stderr, all_threads=True)
    args = parse()
    START_DELAY_US = max(0, args.start_delay_us)
    if args.extras_child:
        return extras_child()
    if args.mctx_child:
        return mctx_child(args.mctx_child, args.one_device)
    if args.streams <= 0:
        args.streams = branches_for(args.steps)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.one_device:
        local = 0
    if args.dry_run:
        return dry_run(args, world, rank)
    from tulips_amd import csum
    from tulips_amd.shard import (all_ranks_ok, gather_results, gather_strings,
                                  max_over_ranks, shard_for)
    # a native crash names its frames before faulthandler prints Python's
    _bench().crash_backtrace()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # control-plane reductions live on the GPU under RCCL, on the CPU under gloo
    cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        check_world(dist, args)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    lib = checked_lib(csum)

    progress("data")
    # ---- data: M8x1500 shard <rank>, 16 batches of 65,536 x 1500 B -------------
    shard = shard_for(rank, world)
    batch_bytes = NSEG * SEG
    arena = torch.empty(shard.nbytes + 256, dtype=torch.uint8, device=dev)
    _bench().fill_splitmix(arena, shard.nbytes, seed=DATA_SEED, byte_off=shard.byte_offset)
    outs = torch.empty(NBATCH * NSEG, dtype=torch.uint16, device=dev)
    base = arena.data_ptr()
    optr = outs.data_ptr()
    fixed = lib.tulips_csum_batch_fixed

    def step(i):
        b = i % NBATCH
        rc = fixed(base + b * batch_bytes, SEG, SEG, None, None, None,
                   optr + b * NSEG * 2, NSEG, 0, sh)
        if rc:
            raise csum.CsumError(rc, "tulips_csum_batch_fixed")

    for i in range(max(args.warmup, NBATCH)):
        step(i)
    torch.cuda.synchronize()

    # The K timed steps (batch i % 16 at step i) captured as ONE HIP graph and
    # replayed once: each step is still one kernel launch over one 98 MB
    # batch; the graph only removes Python's per-launch cost (~19 us, more
    # than the ~17 us kernel) and the inter-replay gap. Steps round-robin over
    # `streams` independent branches, as a receive pipeline would overlap
    # independent bursts: a launch's ramp-up and drain (~2 us each) then
    # overlap the neighbouring launch's steady state.
    graph = None
    if not args.eager:
        graph = torch.cuda.CUDAGraph()
        # --main-branch: the capture stream itself is one of the branches, so
        # the graph forks to and joins from streams - 1 side streams
        nside = args.streams - 1 if args.main_branch else args.streams
        side = [torch.cuda.Stream() for _ in range(nside)]
        with torch.cuda.graph(graph):
            main = torch.cuda.current_stream()
            # Steps round-robin over `streams` independent branches of the
            # graph (batches are independent), so step i+1's waves can fill
            # the drain of step i; each step is still one launch over one
            # whole batch. streams=1 is a single serial chain.
            for sd in side:
                sd.wait_stream(main)
            lanes = ([main] if args.main_branch else []) + side
            for i in range(args.steps):
                b = i % NBATCH
                fixed(base + b * batch_bytes, SEG, SEG, None, None, None,
                      optr + b * NSEG * 2, NSEG, 0, lanes[i % len(lanes)].cuda_stream)
            for sd in side:
                main.wait_stream(sd)
        graph.replay()
        torch.cuda.synchronize()

    progress("timed region")
    # ---- timed region ------------------------------------------------------
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    # every result word overwritten first: what is checked after the timed
    # replay was written by it (outside the timed region)
    outs.view(torch.uint8).fill_(0xA5)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_wall0 = time.perf_counter()
    gate(stream)
    ev0.record(stream)
    if graph is not None:
        graph.replay()
        steps_done = args.steps
    else:
        for i in range(args.steps):
            step(i)
        steps_done = args.steps
    ev1.record(stream)
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t_wall0
    if world > 1:
        dist.barrier()
    t_gpu = ev0.elapsed_time(ev1) / 1e3
    t_local = max(t_gpu, 0.0)
    t_max = max_over_ranks(t_local, dist, cdev)

    total_bytes = float(world) * steps_done * batch_bytes
    value = total_bytes / t_max / GIB
    per_launch_s = t_local / steps_done

    # ---- parity of what the timed replay wrote: per-batch digests vs the
    # reference's (shard <rank> of M8x1500, batch b = steps i with i % 16 == b)
    gold = golden_digests().get("M8x1500", {})
    written = sorted({i % NBATCH for i in range(steps_done)})
    got_b = row_digests(outs, NBATCH, NSEG)
    ok = False
    if rank < 8 and gold.get("shards") and "batches" in gold["shards"][rank]:
        want_b = gold["shards"][rank]["batches"]
        ok = all(got_b[b] == want_b[b] for b in written)
    parity = "ok" if all_ranks_ok(ok, dist, cdev) else "MISMATCH"
    parity_checked = (f"result words poisoned (0xA5A5) before the timed replay; the "
                      f"{len(written)} batches it wrote per rank checked against the "
                      "reference's per-batch digests of M8x1500 shard <rank>")
    if len(written) < NBATCH:
        # the later legs use the whole shard's results
        for b in range(NBATCH):
            step(b)
        torch.cuda.synchronize()

    # the same graph replayed again, each replay timed alone (HIP events on
    # the replay stream, max over ranks): the spread of `value` within one
    # session (make the headline reproducible)
    replays = []
    if graph is not None:
        for _ in range(7):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            gate(stream)
            ev0.record(stream)
            graph.replay()
            ev1.record(stream)
            torch.cuda.synchronize()
            tr = max_over_ranks(ev0.elapsed_time(ev1) / 1e3, dist, cdev)
            replays.append(total_bytes / tr / GIB)
    # ... and without the start gate: the start event then runs
    # as soon as it is queued, so the host's submission of the graph counts,
    # as it did in the rounds before the gate
    ungated = []
    if graph is not None:
        for _ in range(3):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            ev0.record(stream)
            graph.replay()
            ev1.record(stream)
            torch.cuda.synchronize()
            tr = max_over_ranks(ev0.elapsed_time(ev1) / 1e3, dist, cdev)
            ungated.append(total_bytes / tr / GIB)

    digest = fnv1a_u16(outs.cpu().numpy().view(np.uint16))
    shard_digests = gather_strings(digest, dist)

    # the kernel alone, as one serial chain of the same launches (the figure
    # rocprofv3 --stats averages), measured after the timed region so that
    # nothing but the warm replay precedes it
    serial_s = None
    if graph is not None and args.streams > 1:
        def serial(i, st):
            b = i % NBATCH
            fixed(base + b * batch_bytes, SEG, SEG, None, None, None,
                  optr + b * NSEG * 2, NSEG, 0, st)
        serial_s = Timer(torch, stream)(serial, SERIAL_LAUNCHES, replays=5)

    # exchange-inclusive figures (N>1, reported beside `value`, never as it):
    # the results all-gathered after the compute (sequential) and overlapped
    # with it, the golden ZIPF batch split byte-balanced over the ranks, and
    # data starting on GPU 0 scattered over xGMI
    exchange = None
    multi = None
    if world > 1:
        exchange = exchange_sequential(torch, dist, cdev, outs, total_bytes, t_max,
                                       shard_digests, rank, world)
        multi = multi_rank_legs(torch, dist, csum, dev, cdev, stream, arena, outs,
                                rank, world, args, shard_digests, total_bytes)

    # the same shards starting in host memory, every rank over its own PCIe
    # link (§8e; beside `value`, never as it)
    host_start = _leg(host_start_leg, torch, dist, csum, cdev, arena, rank, world)

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "value_kind": "overlapped pipeline rate: the K launches replayed as one graph over "
                      "`config.streams` independent branches (bursts overlap); one launch "
                      "at a time is roofline.avg_launch_us / roofline.frac",
        "unit": "GiB/s",
        "n_gpus": dist.get_world_size() if dist.is_initialized() else 1,
        "steps": steps_done,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / steps_done * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (SplitMix64 bytes, SURVEY.md §8c spec), device-resident",
        "config": {
            "workload": "F1500: 65,536 x 1500 B fixed-stride segments per step "
                        "(BASELINE configs[1]); each rank rotates 16 batches = "
                        "M8x1500 shard <rank> (1,048,576 segments, 1.57 GB)",
            "global_batch": world * NSEG,
            "segment_bytes": SEG,
            "parallelism": f"shard{world}",
            "launch": "graph" if graph is not None else "eager",
            "streams": args.streams if graph is not None else 1,
            "main_branch": bool(args.main_branch),
        },
        "parity": parity,
        "parity_checked": parity_checked,
        "dist": dist_info(torch, dist, world, local, args),
        "shard_digests": shard_digests,
        "exchange": exchange,
        "multi_gpu": multi,
        "host_start": host_start,
        "wall_s_timed": round(t_wall, 4),
        "timing": "HIP events on the launch stream around the timed graph replay; a "
                  f"{START_DELAY_US} us one-wave GPU sleep queued before the start event "
                  "(untimed: the region starts when its launches are on the GPU)",
    }
    if replays:
        result["value_replays"] = {
            "what": "the timed graph (all K steps) replayed 7 more times in this session, "
                    "each replay timed on its own; GiB/s",
            "median": round(float(np.median(replays)), 2),
            "min": round(min(replays), 2), "max": round(max(replays), 2),
            "all": [round(x, 1) for x in replays]}
        result["value_replays_ungated"] = {
            "what": "the same graph replayed 3 more times with no start gate (host "
                    "submission inside the timed region, as before round 4); GiB/s",
            "median": round(float(np.median(ungated)), 2),
            "all": [round(x, 1) for x in ungated]}

    tun = csum.default_tuning(SEG)
    # Roofline of the kernel itself: bytes per launch / one launch's duration,
    # from HIP events around a serial chain of the same launches (the figure
    # rocprofv3 --stats averages). With several graph branches the timed
    # region's per-launch time is shorter than any one dispatch (launches
    # overlap), so it is reported separately as "pipeline".
    serial_s = per_launch_s if serial_s is None else serial_s
    achieved = batch_bytes / serial_s / 1e9
    result["roofline"] = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": read_traffic("F1500"),
        "kernel": f"csum_kernel<G={tun.group},U={tun.unroll},FixedSegs>",
        "bytes_per_launch": batch_bytes,
        "avg_launch_us": round(serial_s * 1e6, 3),
        "pipeline": {
            "branches": args.streams if graph is not None else 1,
            "us_per_launch": round(per_launch_s * 1e6, 3),
            "achieved": round(batch_bytes / per_launch_s / 1e9, 1),
            "frac": round(batch_bytes / per_launch_s / 1e9 / HBM_PEAK_GBS, 4),
        },
    }

    if world == 1 and rank == 0 and not args.no_extras:
        progress("extras (child process)")
        result["extras"] = extras_in_child()

    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        progress("cpu baseline")
        result["cpu_baseline"] = cpu_baseline(arena, batch_bytes, args.cpu_seconds)

    # the figures north_star is judged on, last in the line so a reader of
    # its tail (the driver keeps the tail) sees them: serial, 4-branch and
    # read-ceiling fractions of 8 TB/s with parity
    result["summary"] = summary_of(result)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def summary_of(result):
    """Compact per-config fractions of the 8 TB/s HBM peak (serial launch,
    4 graph branches, the plain read of the same bytes) and parity."""
    ex = result.get("extras") or {}

    def pick(e, serial=None):
        if not isinstance(e, dict) or "error" in e:
            return None
        rd = e.get("read_same_bytes", {})
        return {"serial_frac": serial if serial is not None else e.get("frac_of_peak"),
                "branches4_frac": (e.get("pipeline") or {}).get("frac_of_peak"),
                "read_same_bytes_frac": rd.get("frac_of_peak"),
                "parity": e.get("parity")}
    f15 = pick(ex.get("F1500"), serial=result.get("roofline", {}).get("frac"))
    if f15 is not None:
        # the plain contiguous read of the batch, and the kernel's own load pattern
        f15["read_same_bytes_frac"] = ex.get("stream_read_F1500_batch", {}).get("frac_of_peak")
        f15["read_same_pattern_frac"] = (ex.get("F1500", {}).get("read_same_bytes") or {}).get(
            "frac_of_peak")
        f15["parity"] = "ok" if (result.get("parity") == "ok" and
                                 ex.get("F1500", {}).get("parity") == "ok") else "MISMATCH"
    out = {"F1500": f15, "F9000": pick(ex.get("F9000")), "ZIPF": pick(ex.get("ZIPF"))}
    seg = ex.get("segment_TSO_64K_mss1460")
    if isinstance(seg, dict) and "frac_of_peak" in seg:
        out["segment_serial_frac"] = seg.get("frac_of_peak")
        out["segment_copy_same_bytes_frac"] = (seg.get("copy_same_bytes") or {}).get(
            "frac_of_peak")
    hs = result.get("host_start")
    if isinstance(hs, dict) and "aggregate_GiBps" in hs:
        out["host_start_GiBps"] = hs["aggregate_GiBps"]
    out["value"] = result.get("value")
    return out


def extras_in_child():
    """The side measurements, run in a child process after the timed region
    (no exec: a fresh interpreter started by subprocess, which touches the GPU
    on its own), so that a failure there - an exception or a crash - costs
    the extras, never the headline line. Returns the child's extras dict, or
    an error entry with its exit status."""
    import subprocess
    # the child's progress lines and native/faulthandler stacks are kept and
    # shown only if it fails (the driver keeps the tail of the output, where
    # the JSON line's summary should be)
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--extras-child"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode == 0 and lines:
        return json.loads(lines[-1])["extras"]
    sys.stderr.write(r.stderr[-4000:])
    return {"error": f"extras process exited with status {r.returncode}",
            "stdout_tail": r.stdout[-500:], "stderr_tail": r.stderr[-1500:]}


def extras_child():
    """bench.py --extras-child: rank 0's data (M8x1500 shard 0, the same
    bytes as the headline's) and every side measurement; one JSON line."""
    import torch
    from tulips_amd import csum
    from tulips_amd.shard import shard_for
    _bench().crash_backtrace()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    shard = shard_for(0, 1)
    arena = torch.empty(shard.nbytes + 256, dtype=torch.uint8, device=dev)
    _bench().fill_splitmix(arena, shard.nbytes, seed=DATA_SEED, byte_off=shard.byte_offset)
    torch.cuda.synchronize()
    ex = extras(torch, csum, dev, torch.cuda.current_stream(), arena, NSEG * SEG)
    print(json.dumps({"extras": ex}), flush=True)


def check_world(dist, args):
    """Every rank: the process group holds exactly --gpus ranks."""
    if dist.get_world_size() != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has "
                         f"{dist.get_world_size()} ranks")


def dry_run(args, world, rank):
    """The launcher/process-group half of a run, with no GPU call: ranks
    form the group over gloo, check its size against --gpus, gather their
    ranks and rank 0 prints one JSON line (tests/test_bench_launch.py)."""
    import torch.distributed as dist
    from tulips_amd.shard import gather_strings
    ranks = [0]
    if world > 1:
        dist.init_process_group("gloo")
        check_world(dist, args)
        ranks = [int(x) for x in gather_strings(str(rank), dist)]
        dist.barrier()
        n = dist.get_world_size()
        dist.destroy_process_group()
    else:
        n = 1
        if args.gpus != 1:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has 1 rank")
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": n,
                          "dry_run": True, "parity": "not run (dry run)",
                          "config": {"streams": args.streams},
                          "dist": {"world_size": n, "backend": "gloo" if n > 1 else None,
                                   "ranks": ranks}}), flush=True)


def dist_info(torch, dist, world, local, args):
    """What the process group saw: its size and backend, and each rank's
    device (index and PCI bus id), so a reader can confirm N ranks on N
    distinct GPUs."""
    from tulips_amd.shard import gather_strings
    props = torch.cuda.get_device_properties(local)
    me = {"device": local, "name": props.name,
          "pci_bus_id": getattr(props, "pci_bus_id", None),
          "pci_device_id": getattr(props, "pci_device_id", None)}
    if world == 1 or not dist.is_initialized():
        return {"world_size": 1, "backend": None, "ranks": [me]}
    ranks = [json.loads(x) for x in gather_strings(json.dumps(me), dist)]
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
            "one_device_rehearsal": bool(args.one_device),
            "distinct_devices": len({(r["device"], r["pci_bus_id"]) for r in ranks}),
            "ranks": ranks}


def exchange_sequential(torch, dist, cdev, outs, total_bytes, t_max, shard_digests, rank,
                        world):
    """The K steps' results gathered to every rank after the compute - 16
    batches x 65,536 x 2 B = 2 MiB per rank - timed on its own and added to
    the compute time."""
    from tulips_amd.shard import gather_results, max_over_ranks
    dist.barrier()
    torch.cuda.synchronize()
    tg0 = time.perf_counter()
    gathered = gather_results(outs, dist, cdev)
    torch.cuda.synchronize()
    tg = max_over_ranks(time.perf_counter() - tg0, dist, cdev)
    g_ok = all(fnv1a_u16(gathered[r * outs.numel():(r + 1) * outs.numel()]
                         .cpu().numpy().view(np.uint16)) == shard_digests[r]
               for r in range(world)) if rank == 0 else True
    return {"op": "all_gather of the result words, after the compute",
            "bytes_per_rank": outs.numel() * 2, "ms": round(tg * 1e3, 3),
            "value_exchange_inclusive": round(total_bytes / (t_max + tg) / GIB, 2),
            "parity": "ok" if g_ok else "MISMATCH"}


def _leg(fn, *a):
    """Run one multi-rank side measurement; an exception becomes an error
    entry (every rank runs the same code, so they fail alike)."""
    try:
        return fn(*a)
    except Exception as e:  # noqa: BLE001 - reported, never hidden
        return {"error": f"{type(e).__name__}: {e}"}


def multi_rank_legs(torch, dist, csum, dev, cdev, stream, arena, outs, rank, world, args,
                    shard_digests, total_bytes):
    # (under gloo, the one-GPU rehearsal, the collectives take the same CUDA
    # tensors through host memory)
    res = {"backend": args.dist_backend}
    res["library_scatter_from_gpu0"] = _leg(mctx_device_leg, torch, dist, csum, cdev, rank,
                                            world, args)
    res["exchange_overlapped"] = _leg(exchange_overlapped, torch, dist, csum, cdev,
                                      stream, arena, rank, world, args, shard_digests)
    res["scatter_from_gpu0"] = _leg(scatter_leg, torch, dist, csum, dev, cdev, arena,
                                    outs, rank, world)
    res["zipf_byte_balanced"] = _leg(zipf_sharded_leg, torch, dist, csum, dev, cdev, stream,
                                     rank, world)
    return res


def host_start_leg(torch, dist, csum, cdev, arena, rank, world):
    """SURVEY.md §8e / north_star's host-start form (the path starts and ends
    in host memory, src/transport hands over pipe/NIC buffers): rank r's M8
    shard (16 x 65,536 x 1500 B = 1.57 GB) lies in page-locked host memory
    allocated after the rank's GPU was selected (tulips_csum_host_alloc =
    hipHostMalloc with default flags: placed on the NUMA node nearest that
    GPU), and every rank checksums it through its own H2D -> kernel -> D2H
    pipeline over its own PCIe link (tulips_csum_batch_host, one call for the
    whole shard: pinned, so the staging DMAs straight from it). No data-path
    collective. Timed end to end, median of 3, max over ranks; aggregate =
    all ranks' bytes / that time. Parity: the 16 per-batch digests of every
    rank's results against the reference's M8x1500 shard digests. Reference
    analogue: per-queue RX spreading, src/transport/ena/RedirectionTable.cpp:
    74-98."""
    import ctypes as C
    from tulips_amd.shard import all_ranks_ok, max_over_ranks
    nbytes = NBATCH * NSEG * SEG
    lib = checked_lib(csum)
    ptr = C.c_void_p()
    ctx = None
    err = None
    times = []
    ok = False
    # every rank takes part in every barrier and reduction below whatever
    # fails locally (a failure becomes this rank's error and parity MISMATCH),
    # so no rank is left waiting in a collective
    try:
        lib.tulips_csum_host_alloc(nbytes, C.byref(ptr))
        host = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(nbytes,))
        torch.from_numpy(host).copy_(arena[:nbytes])     # the shard's bytes, D2H once
        torch.cuda.synchronize()
        offs = np.arange(NBATCH * NSEG, dtype=np.uint64) * np.uint64(SEG)
        lens = np.full(NBATCH * NSEG, SEG, dtype=np.uint16)
        out = np.empty(NBATCH * NSEG, dtype=np.uint16)
        ctx = csum.HostContext(torch.cuda.current_device())
        ctx.batch(ptr.value, offs, lens, out=out)          # staging made
    except Exception as e:  # noqa: BLE001 - reported, never hidden
        err = f"{type(e).__name__}: {e}"
    for _ in range(3):
        if world > 1:
            dist.barrier()
        if err is None:
            try:
                out.fill(0xA5A5)
                t0 = time.perf_counter()
                ctx.batch(ptr.value, offs, lens, out=out)
                times.append(time.perf_counter() - t0)
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
    if err is None:
        gold = golden_digests().get("M8x1500", {}).get("shards", [])
        ok = rank < len(gold) and "batches" in gold[rank] and all(
            fnv1a_u16(out[b * NSEG:(b + 1) * NSEG]) == gold[rank]["batches"][b]
            for b in range(NBATCH))
    if ctx is not None:
        ctx.close()
    if ptr.value:
        lib.tulips_csum_host_free(ptr)
    t_local = float(np.median(times)) if times and err is None else float("inf")
    t_max = max_over_ranks(t_local, dist, cdev) if world > 1 else t_local
    t_min = -max_over_ranks(-t_local, dist, cdev) if world > 1 else t_local
    ok = all_ranks_ok(ok and err is None, dist, cdev) if world > 1 else (ok and err is None)
    res = {"what": "each rank's M8x1500 shard from page-locked host memory near its GPU: "
                   "tulips_csum_batch_host (H2D -> kernel -> D2H pipeline, one call per "
                   "1.57 GB shard), median of 3, max over ranks",
           "bytes_per_rank": nbytes,
           "parity": "ok" if ok else "MISMATCH"}
    if err is not None or t_max == float("inf"):
        res["error"] = err or "another rank failed"
        return res
    res.update({"ms_max": round(t_max * 1e3, 3), "ms_min": round(t_min * 1e3, 3),
                "per_gpu_GiBps": round(nbytes / t_max / GIB, 2),
                "aggregate_GiBps": round(world * nbytes / t_max / GIB, 2)})
    return res


def mctx_device_leg(torch, dist, csum, cdev, rank, world, args):
    """configs[4] with the data starting on GPU 0, through the LIBRARY
    (tulips_csum_mctx_batch_fixed_device): rank 0 holds the
    whole world x 1,048,576 x 1500 B batch (at N = 8: M8x1500, 12.6 GB) in
    GPU 0's HBM and spreads it over every GPU of the node from one process -
    each peer pulls its ~32 MiB pieces over xGMI while checksumming the
    previous ones, results come back to GPU 0 in segment order. Rank 0 runs
    it in a child process (bench.py --mctx-child: one process driving every
    device, as an integrator's would), so that a failure on real peers - an
    exception or a crash - costs this entry, never the line; the other ranks
    wait at a barrier. Timed end to end on GPU 0's stream (best of 3;
    exchange-inclusive). Parity: every shard's digest equals the reference's
    M8 shard digest, and at N = 8 the whole batch's digest equals M8x1500's."""
    from tulips_amd.shard import gather_strings
    res = {}
    if rank == 0:
        # rank 0 alone works here: an error must still reach the barrier below,
        # or the other ranks would meet rank 0's next collective there
        import subprocess
        cmd = [sys.executable, "-u", os.path.abspath(__file__), "--mctx-child", str(world)]
        if args.one_device:
            cmd.append("--one-device")
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                               cwd=ROOT, timeout=600)
            lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode == 0 and lines:
                res = json.loads(lines[-1])["mctx"]
            else:
                sys.stderr.write(r.stderr[-4000:])
                res = {"error": f"mctx process exited with status {r.returncode}",
                       "stderr_tail": r.stderr[-1500:]}
        except Exception as e:  # noqa: BLE001 - reported, never hidden
            res = {"error": f"{type(e).__name__}: {e}"}
    dist.barrier()
    return json.loads(gather_strings(json.dumps(res), dist)[0])


def mctx_child(world, one_device):
    """bench.py --mctx-child WORLD: mctx_device_leg's work in its own process;
    one JSON line {"mctx": ...}."""
    import torch
    from tulips_amd import csum
    from tulips_amd.shard import SHARD_SEGMENTS
    _bench().crash_backtrace()
    devs = [0] * world if one_device else list(range(world))
    res = {}
    try:
        n = world * SHARD_SEGMENTS
        d0 = torch.device("cuda", 0)
        with torch.cuda.device(d0):
            arena = torch.empty(n * SEG + 64, dtype=torch.uint8, device=d0)
            _bench().fill_splitmix(arena, n * SEG, seed=DATA_SEED)
            out = torch.empty(n, dtype=torch.uint16, device=d0)
            st = torch.cuda.current_stream(d0)
            with csum.MultiContext(devs, chunk_bytes=1 << 20) as m:
                m.batch_fixed_device(arena, SEG, SEG, n, out=out, stream=st)   # buffers made
                st.synchronize()
                best = None
                for _ in range(3):
                    st.synchronize()
                    t0 = time.perf_counter()
                    m.batch_fixed_device(arena, SEG, SEG, n, out=out, stream=st)
                    st.synchronize()
                    t = time.perf_counter() - t0
                    best = t if best is None else min(best, t)
                bounds = m.bounds().tolist()
            o = out.cpu().numpy().view(np.uint16)
        gold = golden_digests().get("M8x1500", {})
        shards = gold.get("shards", [])
        ok = all(fnv1a_u16(o[k * SHARD_SEGMENTS:(k + 1) * SHARD_SEGMENTS]) ==
                 shards[k]["fnv1a64"] for k in range(min(world, len(shards))))
        if world == 8:
            ok = ok and fnv1a_u16(o) == gold.get("fnv1a64")
        nbytes = float(n) * SEG
        res = {"entry": "tulips_csum_mctx_batch_fixed_device (one process, devices "
                        f"{devs})",
               "workload": f"{n:,} x 1500 B resident on GPU 0 ({nbytes / 1e9:.2f} GB)",
               "bytes_pulled_by_peers": int(nbytes * (world - 1) / world),
               "ms": round(best * 1e3, 3),
               "value_exchange_inclusive_GiBps": round(nbytes / best / GIB, 2),
               "shard_bounds": bounds,
               "parity": "ok" if ok else "MISMATCH"}
        del arena, out
        res["kernel_only"] = single_process_kernel_only(torch, csum, devs)
    except Exception as e:  # noqa: BLE001 - reported, never hidden
        res = {"error": f"{type(e).__name__}: {e}"}
    print(json.dumps({"mctx": res}), flush=True)


def single_process_kernel_only(torch, csum, devs, rotations=4):
    """The kernel-only half of the one-process form: device k of `devs`
    holds M8x1500 shard k resident in its own HBM; one process replays, on
    every device, a captured graph of `rotations` passes over the shard's 16
    batches (graph replays, so the host's launch rate is not what is timed),
    and the wall time from the first replay to the last device's completion
    gives the aggregate. Parity: every device's results poisoned before the
    timed replays, then its shard digest vs the reference's."""
    from tulips_amd.shard import SHARD_SEGMENTS
    gold = golden_digests().get("M8x1500", {}).get("shards", [])
    fixed = checked_lib(csum).tulips_csum_batch_fixed
    per = []
    for k, d in enumerate(devs):
        dv = torch.device("cuda", d)
        with torch.cuda.device(dv):
            a = torch.empty(SHARD_SEGMENTS * SEG + 256, dtype=torch.uint8, device=dv)
            _bench().fill_splitmix(a, SHARD_SEGMENTS * SEG, seed=DATA_SEED,
                               byte_off=k * SHARD_SEGMENTS * SEG)
            o = torch.empty(SHARD_SEGMENTS, dtype=torch.uint16, device=dv)
            st = torch.cuda.Stream(device=dv)

            def one(stream_h, a=a, o=o):
                for _ in range(rotations):
                    for b in range(NBATCH):
                        rc = fixed(a.data_ptr() + b * NSEG * SEG, SEG, SEG, None, None, None,
                                   o.data_ptr() + b * NSEG * 2, NSEG, 0, stream_h)
                        if rc:
                            raise csum.CsumError(rc, "tulips_csum_batch_fixed")
            one(st.cuda_stream)
            torch.cuda.synchronize(dv)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                one(st.cuda_stream)
        per.append((dv, a, o, st, g))

    def sync_all():
        for dv, *_ in per:
            torch.cuda.synchronize(dv)
    best = None
    for _ in range(3):
        for dv, a, o, st, g in per:
            with torch.cuda.device(dv):
                o.view(torch.uint8).fill_(0xA5)
        sync_all()
        t0 = time.perf_counter()
        for dv, a, o, st, g in per:
            with torch.cuda.device(dv):
                g.replay()
        sync_all()
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    ok = all(k < len(gold) and fnv1a_u16(o.cpu().numpy().view(np.uint16)) ==
             gold[k]["fnv1a64"] for k, (dv, a, o, st, g) in enumerate(per))
    nbytes = float(len(devs)) * rotations * SHARD_SEGMENTS * SEG
    del per
    return {"what": "one process, every device checksumming its own resident shard: "
                    f"a captured graph of {rotations} x 16 F1500 launches replayed per "
                    "device, wall time first replay -> last device done (best of 3)",
            "devices": list(devs), "ms": round(best * 1e3, 3),
            "value_GiBps": round(nbytes / best / GIB, 2),
            "parity": "ok" if ok else "MISMATCH"}


def exchange_overlapped(torch, dist, csum, cdev, stream, arena, rank, world, args,
                        shard_digests):
    """Results all-gathered WHILE the next rotation computes: rotation r (16
    launches, one per batch of the shard) writes result buffer r % 2, and the
    all-gather of buffer r runs on a communication stream behind an event,
    overlapping rotation r + 1; rotation r + 2 waits for that gather before
    overwriting its buffer. Timed end to end (max over ranks) beside the same
    rotations without the gathers."""
    from tulips_amd.shard import max_over_ranks
    fixed = checked_lib(csum).tulips_csum_batch_fixed
    batch_bytes = NSEG * SEG
    base = arena.data_ptr()
    bufs = [torch.empty(NBATCH * NSEG, dtype=torch.uint16, device=arena.device)
            for _ in range(2)]
    gath = [torch.empty(world * NBATCH * NSEG * 2, dtype=torch.uint8, device=arena.device)
            for _ in range(2)]
    side = [torch.cuda.Stream() for _ in range(PIPE)]
    graphs = []
    for k in range(2):
        for b in range(NBATCH):     # warm (per-stream state outside the capture)
            fixed(base + b * batch_bytes, SEG, SEG, None, None, None,
                  bufs[k].data_ptr() + b * NSEG * 2, NSEG, 0, stream.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            main = torch.cuda.current_stream()
            for sd in side:
                sd.wait_stream(main)
            for b in range(NBATCH):
                fixed(base + b * batch_bytes, SEG, SEG, None, None, None,
                      bufs[k].data_ptr() + b * NSEG * 2, NSEG, 0,
                      side[b % PIPE].cuda_stream)
            for sd in side:
                main.wait_stream(sd)
        graphs.append(g)
    comm = torch.cuda.Stream()
    rot = max(4, args.steps // NBATCH)

    def run(with_gather):
        done = [None, None]
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(rot):
            k = r % 2
            if done[k] is not None:
                stream.wait_event(done[k])
            graphs[k].replay()
            if with_gather:
                ev = torch.cuda.Event()
                ev.record(stream)
                with torch.cuda.stream(comm):
                    comm.wait_event(ev)
                    dist.all_gather_into_tensor(gath[k], bufs[k].view(torch.uint8))
                    de = torch.cuda.Event()
                    de.record(comm)
                done[k] = de if with_gather else None
        torch.cuda.synchronize()
        return max_over_ranks(time.perf_counter() - t0, dist, cdev)

    t_compute = run(False)
    t_both = run(True)
    last = gath[(rot - 1) % 2].view(torch.uint16).cpu().numpy()
    per = NBATCH * NSEG
    ok = all(fnv1a_u16(last[r * per:(r + 1) * per]) == shard_digests[r]
             for r in range(world)) if rank == 0 else True
    from tulips_amd.shard import all_ranks_ok
    ok = all_ranks_ok(ok, dist, cdev)
    nbytes = float(world) * rot * NBATCH * batch_bytes
    return {"op": "all_gather of each rotation's 2 MiB of result words on a comm stream, "
                  "overlapping the next rotation's 16 launches (double-buffered results)",
            "rotations": rot, "ms_compute_only": round(t_compute * 1e3, 3),
            "ms_with_exchange": round(t_both * 1e3, 3),
            "value_compute_only": round(nbytes / t_compute / GIB, 2),
            "value_exchange_inclusive": round(nbytes / t_both / GIB, 2),
            "exchange_hidden_frac": round(min(1.0, t_compute / t_both), 4),
            "parity": "ok" if ok else "MISMATCH"}


def scatter_leg(torch, dist, csum, dev, cdev, arena, outs, rank, world):
    """Data starting on GPU 0: rank 0 holds `world` F1500
    batches, RCCL scatters batch r to rank r over xGMI, every rank checksums
    what it received; timed scatter + kernel (max over ranks). Parity: rank
    r's results equal rank 0's own results for batch r of its shard."""
    from tulips_amd.shard import all_ranks_ok, gather_strings, max_over_ranks
    batch_bytes = NSEG * SEG
    if world > NBATCH:
        return {"skipped": "more ranks than batches per shard"}
    recv = torch.empty(batch_bytes + 256, dtype=torch.uint8, device=dev)
    out = torch.empty(NSEG, dtype=torch.uint16, device=dev)
    chunks = [arena[b * batch_bytes:(b + 1) * batch_bytes] for b in range(world)] \
        if rank == 0 else None
    fixed = checked_lib(csum).tulips_csum_batch_fixed
    best = None
    for _ in range(3):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.scatter(recv[:batch_bytes], chunks, src=0)
        rc = fixed(recv.data_ptr(), SEG, SEG, None, None, None, out.data_ptr(), NSEG, 0,
                   torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        t = max_over_ranks(time.perf_counter() - t0, dist, cdev)
        if rc:
            raise csum.CsumError(rc, "tulips_csum_batch_fixed")
        best = t if best is None else min(best, t)
    digs = gather_strings(fnv1a_u16(out.cpu().numpy().view(np.uint16)), dist)
    ok = True
    if rank == 0:
        own = outs.cpu().numpy().view(np.uint16)
        ok = all(digs[r] == fnv1a_u16(own[r * NSEG:(r + 1) * NSEG]) for r in range(world))
    ok = all_ranks_ok(ok, dist, cdev)
    return {"op": "dist.scatter (RCCL send/recv over xGMI) of one 98.3 MB F1500 batch per "
                  "rank from GPU 0, then the kernel on each rank",
            "bytes_moved": (world - 1) * batch_bytes, "ms": round(best * 1e3, 3),
            "value_scatter_inclusive": round(world * batch_bytes / best / GIB, 2),
            "parity": "ok" if ok else "MISMATCH"}


def zipf_sharded_leg(torch, dist, csum, dev, cdev, stream, rank, world):
    """A Zipf batch of world x 65,536 segments (the §8c length sequence,
    continued: its first 65,536 segments and their bytes ARE the golden ZIPF
    batch, configs[3]) split over the ranks by BYTES (tulips_csum_shard_plan):
    each rank fills and checksums its contiguous shard of the global packed
    arena (serial chain of launches, HIP events). Aggregate = all bytes /
    slowest rank. Parity: the gathered results of the first 65,536 segments
    equal the reference's ZIPF digest."""
    from tulips_amd.shard import all_ranks_ok, byte_shard_for, max_over_ranks
    lens = zipf_lengths(world * NSEG)
    zb = int(lens.astype(np.int64).sum()) / world    # mean bytes per rank
    bs = byte_shard_for(rank, world, lens)
    ll = lens[bs.seg_begin:bs.seg_begin + bs.seg_count]
    offs = np.zeros(len(ll), dtype=np.uint64)
    if len(ll) > 1:
        np.cumsum(ll[:-1], dtype=np.uint64, out=offs[1:])
    az = torch.empty(bs.nbytes + 256, dtype=torch.uint8, device=dev)
    _bench().fill_splitmix(az, bs.nbytes, byte_off=bs.byte_offset)
    doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
    dlens = torch.from_numpy(ll.view(np.int16).copy()).to(dev)
    out = torch.empty(max(1, len(ll)), dtype=torch.uint16, device=dev)
    batch = checked_lib(csum).tulips_csum_batch_arena   # a shard is a packed, in-order arena

    def fz(i, st):
        rc = batch(az.data_ptr(), bs.nbytes, doffs.data_ptr(), dlens.data_ptr(), None, None,
                   None, out.data_ptr(), len(ll), 0, st)
        if rc:
            raise csum.CsumError(rc, "tulips_csum_batch_arena")
    fz(0, stream.cuda_stream)
    torch.cuda.synchronize()
    dist.barrier()
    t = Timer(torch, stream)(fz, 40)
    t_max = max_over_ranks(t, dist, cdev)
    t_min = -max_over_ranks(-t, dist, cdev)
    # per-rank byte spread of this plan vs a split by segment count
    cnt_b = np.add.reduceat(lens.astype(np.int64), np.arange(0, len(lens), len(lens) // world))
    plan = csum.shard_plan(lens, world)
    byt_b = np.add.reduceat(lens.astype(np.int64), plan[:-1].astype(np.int64))
    # parity over the golden arena: results of global segments [0, 65536)
    cmax = int(max_over_ranks(float(len(ll)), dist, cdev))
    pad = torch.zeros(cmax, dtype=torch.uint16, device=dev)
    pad[:len(ll)] = out[:len(ll)]
    from tulips_amd.shard import gather_results
    allw = gather_results(pad, dist, cdev).cpu().numpy().view(np.uint16)
    glob = np.concatenate([allw[r * cmax:r * cmax + int(plan[r + 1] - plan[r])]
                           for r in range(world)])
    gold = golden_digests().get("ZIPF", {}).get("fnv1a64")
    ok = all_ranks_ok(fnv1a_u16(glob[:NSEG]) == gold, dist, cdev)
    return {"workload": f"Zipf batch of {world} x 65,536 segments ({int(world * zb)} B), "
                        "byte-balanced shards",
            "entry": "tulips_csum_batch_arena (each shard is a packed in-order arena)",
            "shard_segments": int(bs.seg_count), "shard_bytes": int(bs.nbytes),
            "us_per_launch_max": round(t_max * 1e6, 2),
            "us_per_launch_min": round(t_min * 1e6, 2),
            "value_GiBps": round(world * zb / t_max / GIB, 2),
            "bytes_spread_byte_plan": int(byt_b.max() - byt_b.min()),
            "bytes_spread_count_split": int(cnt_b.max() - cnt_b.min()),
            "parity": "ok" if ok else "MISMATCH"}


PIPE = 4    # graph branches for the "pipeline" figures: one per hardware queue
PIPE_WIDE = 8   # two per hardware queue (the bench --streams default)


PIPE_LAUNCHES = 4   # a pipeline graph holds this many times the serial launches


def pipe_times(timer, fn, reps, poison=None):
    """Seconds per launch of `fn` over PIPE and over PIPE_WIDE graph branches:
    PIPE_LAUNCHES x reps launches per graph, so its fork and join are spread
    thin (profiles/probe_branches_r03.txt: ZIPF over 160 launches on 4
    branches 7.5-8.8 us, over 640 7.5-7.9), median of 3 replays."""
    n = PIPE_LAUNCHES * reps
    return (timer(fn, n, branches=PIPE, replays=3, poison=poison),
            timer(fn, n, branches=PIPE_WIDE, replays=3, poison=poison))


POISON = 0xA5   # byte the outputs are overwritten with before a timed replay


def poisoner(*tensors):
    """A poison() for Timer: every byte of the tensors set to POISON (0xA5A5
    as a u16 result, 0xA5 as a frame flag byte, which no valid flag set is)."""
    import torch

    def run():
        for x in tensors:
            x.view(torch.uint8).fill_(POISON)
    return run


def row_digests(t, rows, per):
    """FNV-1a-64 of rows [0, rows) of a flat u16 device tensor, `per` each."""
    o = t[:rows * per].cpu().numpy().view(np.uint16)
    return [fnv1a_u16(o[r * per:(r + 1) * per]) for r in range(rows)]


def pipe_entry(nbytes, tt):
    """Rates of overlapped graph branches: (t at PIPE, t at PIPE_WIDE) in seconds."""
    def one(b, t):
        return {"branches": b, "us_per_launch": round(t * 1e6, 2),
                "GiBps": round(nbytes / t / GIB, 1),
                "frac_of_peak": round(nbytes / t / 1e9 / HBM_PEAK_GBS, 4)}
    e = one(PIPE, tt[0])
    e["wide"] = one(PIPE_WIDE, tt[1])
    return e


def read_traffic(workload):
    """HBM bytes per launch from the committed PMC summary (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d[workload]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def extras(torch, csum, dev, stream, arena, batch_bytes):
    timer = Timer(torch, stream)
    sh = stream.cuda_stream
    lib = checked_lib(csum)
    ex = {}

    # plain streaming read of the whole 1.57 GB shard: the measured ceiling
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    nbytes = NBATCH * batch_bytes
    t = timer(lambda i, st: lib.tulips_csum_stream_read(arena.data_ptr(), nbytes,
                                                        sink.data_ptr(), 0, st), 10)
    ex["stream_read_ceiling_GBps"] = round(nbytes / t / 1e9, 1)
    # ... and of one 98.3 MB batch per launch, rotated like the F1500 steps:
    # what a single launch of that size can read (ramp and drain included)
    def one(i, st):
        b = i % NBATCH
        lib.tulips_csum_stream_read(arena.data_ptr() + b * batch_bytes, batch_bytes,
                                    sink.data_ptr(), 0, st)
    for i in range(NBATCH):
        one(i, sh)
    t1 = timer(one, 64)
    tp1 = pipe_times(timer, one, 64)
    ex["stream_read_F1500_batch"] = {
        "what": "plain 16-byte streaming read of one F1500 batch per launch (98.3 MB), "
                "batches rotated: the single-launch ceiling roofline.frac compares with",
        "avg_launch_us": round(t1 * 1e6, 2),
        "frac_of_peak": round(batch_bytes / t1 / 1e9 / HBM_PEAK_GBS, 4),
        "pipeline": pipe_entry(batch_bytes, tp1)}

    gold = golden_digests()
    rot = golden_rotations()

    # F1500 (configs[1]) itself in the extras' forms: serial and on 4 / 8
    # graph branches over the shard's 16 batches, each replay's outputs
    # poisoned first and the 16 batch digests checked after
    o15 = torch.empty(NBATCH * NSEG, dtype=torch.uint16, device=dev)
    fixed15 = lib.tulips_csum_batch_fixed

    def f15(i, st):
        b = i % NBATCH
        fixed15(arena.data_ptr() + b * batch_bytes, SEG, SEG, None, None, None,
                o15.data_ptr() + b * NSEG * 2, NSEG, 0, st)
    want15 = golden_digests().get("M8x1500", {}).get("shards", [{}])[0].get("batches")

    def ok15():
        return want15 is not None and row_digests(o15, NBATCH, NSEG) == want15
    t15 = timer(f15, 64, poison=poisoner(o15))
    okf = ok15()
    tp15 = pipe_times(timer, f15, 64, poison=poisoner(o15))
    okf = okf and ok15()
    ex["F1500"] = {"avg_launch_us": round(t15 * 1e6, 2),
                   "frac_of_peak": round(batch_bytes / t15 / 1e9 / HBM_PEAK_GBS, 4),
                   "pipeline": pipe_entry(batch_bytes, tp15),
                   "parity": "ok" if okf else "MISMATCH"}
    del o15

    # the F1500 kernel's exact load pattern without its arithmetic (32-lane
    # subgroup per 1500 B segment at stride 1500, 3 clamped loads per lane),
    # over the same rotated batches: that kernel's own ceiling
    def f15read(i, st):
        b = i % NBATCH
        lib.tulips_csum_stream_read_slots_geom(arena.data_ptr() + b * batch_bytes, SEG, SEG,
                                               NSEG, 32, 3, sink.data_ptr(), st)
    t = timer(f15read, 64)
    tp = pipe_times(timer, f15read, 64)
    ex["F1500"]["read_same_bytes"] = {
        "what": "tulips_csum_stream_read_slots_geom(32, 3): the kernel's loads (one 32-lane "
                "subgroup per 1500 B segment, 3 clamped loads per lane), no arithmetic",
        "avg_launch_us": round(t * 1e6, 2),
        "frac_of_peak": round(batch_bytes / t / 1e9 / HBM_PEAK_GBS, 4),
        "pipeline": pipe_entry(batch_bytes, tp)}

    # F9000 (configs[2]): 4 distinct 590 MB batches (2.36 GB, 9x the 256 MB
    # Infinity Cache) rotated, so every launch streams from HBM; the 2-batch
    # rotation (1.18 GB) of earlier rounds beside it as `mall_assisted`.
    # Outputs are poisoned before the timed replay and every batch's digest
    # is checked against the reference's after it.
    L9, NB9 = 9000, 4
    b9 = NSEG * L9
    a9 = torch.empty(NB9 * b9 + 256, dtype=torch.uint8, device=dev)
    _bench().fill_splitmix(a9, NB9 * b9)
    o9 = torch.empty(NB9 * NSEG, dtype=torch.uint16, device=dev)
    fixed = lib.tulips_csum_batch_fixed
    p9 = poisoner(o9)

    def f9_over(nb):
        def f9(i, st):
            b = i % nb
            fixed(a9.data_ptr() + b * b9, L9, L9, None, None, None,
                  o9.data_ptr() + b * NSEG * 2, NSEG, 0, st)
        return f9

    def f9_ok(nb):
        want = rot.get("F9000", [])[:nb]
        return len(want) == nb and row_digests(o9, nb, NSEG) == want
    f9 = f9_over(NB9)
    for i in range(NB9):
        f9(i, sh)
    t = timer(f9, 40, poison=p9)
    ok9 = f9_ok(NB9)
    tp = pipe_times(timer, f9, 40, poison=p9)
    ok9 = ok9 and f9_ok(NB9)
    t2 = timer(f9_over(2), 40, poison=p9)
    ok9_2 = f9_ok(2)
    # the F9000 kernel's own read pattern without the arithmetic, over the
    # same rotated batches: the ceiling that kernel is held against
    sink9 = torch.zeros(4, dtype=torch.int32, device=dev)

    def f9r_over(nb):
        def f9r(i, st):
            b = i % nb
            lib.tulips_csum_stream_read_tiles(a9.data_ptr() + b * b9, L9, NSEG,
                                              sink9.data_ptr(), st)
        return f9r
    t9r = timer(f9r_over(NB9), 40)
    t9r2 = timer(f9r_over(2), 40)
    tun = csum.default_tuning(L9)
    ex["F9000"] = {"GiBps": round(b9 / t / GIB, 1), "GBps": round(b9 / t / 1e9, 1),
                   "frac_of_peak": round(b9 / t / 1e9 / HBM_PEAK_GBS, 4),
                   "avg_launch_us": round(t * 1e6, 2),
                   "rotation": f"{NB9} distinct batches of 65,536 x 9000 B "
                               f"({NB9 * b9 / 1e9:.2f} GB), HBM-resident working set",
                   "pipeline": pipe_entry(b9, tp),
                   "geometry": f"G={tun.group},U={tun.unroll}",
                   "traffic": read_traffic("F9000"),
                   "read_same_bytes": {
                       "what": "tulips_csum_stream_read_tiles: the kernel's loads (one wave per "
                               "9000 B tile, 64 lanes x 12 clamped loads), no arithmetic",
                       "avg_launch_us": round(t9r * 1e6, 2),
                       "frac_of_peak": round(b9 / t9r / 1e9 / HBM_PEAK_GBS, 4)},
                   "mall_assisted": {
                       "rotation": f"2 batches ({2 * b9 / 1e9:.2f} GB)",
                       "avg_launch_us": round(t2 * 1e6, 2),
                       "frac_of_peak": round(b9 / t2 / 1e9 / HBM_PEAK_GBS, 4),
                       "read_same_bytes_frac": round(b9 / t9r2 / 1e9 / HBM_PEAK_GBS, 4),
                       "parity": "ok" if ok9_2 else "MISMATCH"},
                   "parity": "ok" if ok9 else "MISMATCH",
                   "parity_checked": "outputs poisoned before the timed replays; the "
                                     f"{NB9} batch digests after them vs the reference's"}
    del a9, o9

    # SURVEY.md §8d's aligned-stride layouts: F1500 at stride 2048 (the OFED
    # RX slots, include/tulips/transport/ofed/Device.h:25) and F9000 at
    # stride 9216, each as 4 copies of the golden arena at different addresses
    # (537 MB and 2.42 GB rotated: HBM-resident); rate over the segment bytes
    # only (65,536 x L), every copy's digest vs the reference's
    progress("extras: aligned strides")
    ex["aligned_strides"] = {}
    # (BENCH_EXTRAS_SKIP=aligned_strides: a profiling pass leaves them out -
    # their launches are the F1500 / F9000 kernels with the same grids, which
    # tools/pmc_traffic.py could not tell apart from the rotated batches')
    skip = os.environ.get("BENCH_EXTRAS_SKIP", "").split(",")
    for name, L, S in (() if "aligned_strides" in skip else
                       (("F1500s2048", 1500, 2048), ("F9000s9216", 9000, 9216))):
        ncp = 4
        cb = NSEG * S
        ac = torch.empty(ncp * cb + 256, dtype=torch.uint8, device=dev)
        _bench().fill_splitmix(ac, cb)
        for c in range(1, ncp):
            ac[c * cb:(c + 1) * cb].copy_(ac[:cb])
        oc = torch.empty(ncp * NSEG, dtype=torch.uint16, device=dev)
        pc = poisoner(oc)

        def fs(i, st, ac=ac, oc=oc, L=L, S=S, cb=cb, ncp=ncp):
            c = i % ncp
            fixed(ac.data_ptr() + c * cb, S, L, None, None, None,
                  oc.data_ptr() + c * NSEG * 2, NSEG, 0, st)
        for i in range(ncp):
            fs(i, sh)
        want = gold.get(name, {}).get("fnv1a64")
        ts = timer(fs, 40, poison=pc)
        okc = want is not None and row_digests(oc, ncp, NSEG) == [want] * ncp
        tps = pipe_times(timer, fs, 40, poison=pc)
        okc = okc and row_digests(oc, ncp, NSEG) == [want] * ncp
        alg = NSEG * L
        ex["aligned_strides"][name] = {
            "avg_launch_us": round(ts * 1e6, 2), "GiBps": round(alg / ts / GIB, 1),
            "frac_of_peak": round(alg / ts / 1e9 / HBM_PEAK_GBS, 4),
            "pipeline": pipe_entry(alg, tps),
            "rotation": f"{ncp} copies ({ncp * cb / 1e9:.2f} GB)",
            "parity": "ok" if okc else "MISMATCH"}
        del ac, oc

    # ZIPF (configs[3]): 24 copies with the same lengths, different bytes
    # (1.05 GB rotated: HBM-resident), the 8-copy rotation (350 MB) beside it
    # as `mall_assisted`. Copy c = stream bytes [c * zb, (c + 1) * zb); copy 0
    # is the golden ZIPF arena.
    progress("extras: ZIPF")
    lens = zipf_lengths(NSEG)
    offs = np.zeros(NSEG, dtype=np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    zb = int(lens.astype(np.int64).sum())
    nz = 24
    az = torch.empty(nz * zb + 256, dtype=torch.uint8, device=dev)
    _bench().fill_splitmix(az, nz * zb)
    doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
    dlens = torch.from_numpy(lens).to(dev)
    oz = torch.empty(nz * NSEG, dtype=torch.uint16, device=dev)
    batch = lib.tulips_csum_batch
    arena_batch = lib.tulips_csum_batch_arena
    batch_tuned = lib.tulips_csum_batch_tuned
    pz = poisoner(oz)

    def z_ok(ncopies):
        want = rot.get("ZIPF", [])[:ncopies]
        return len(want) == ncopies and row_digests(oz, ncopies, NSEG) == want

    # the batch is one in-order arena (segments back to back): the arena
    # entry point cuts the work by bytes (KIND_SPAN)
    def fz_over(nc):
        def fz(i, st):
            b = i % nc
            assert arena_batch(az.data_ptr() + b * zb, zb, doffs.data_ptr(), dlens.data_ptr(),
                               None, None, None, oz.data_ptr() + b * NSEG * 2, NSEG, 0, st) == 0
        return fz

    # the same batch through the any-layout entry point (offsets alone)
    def fz_any(i, st):
        b = i % nz
        assert batch(az.data_ptr() + b * zb, doffs.data_ptr(), dlens.data_ptr(), None, None,
                     None, oz.data_ptr() + b * NSEG * 2, NSEG, 0, st) == 0

    # configs[3] as written: one wave (64 lanes) per segment
    wave_t = csum.Tuning(kind=csum.KIND_SUBGROUP, group=64, unroll=4, sps=1)

    def fz_wave(i, st):
        b = i % nz
        assert batch_tuned(az.data_ptr() + b * zb, doffs.data_ptr(), dlens.data_ptr(), None,
                           None, None, oz.data_ptr() + b * NSEG * 2, NSEG, 0,
                           __import__("ctypes").byref(wave_t), st) == 0
    for i in range(nz):
        fz_any(i, sh)
    ta = timer(fz_any, 80, poison=pz)
    ok_any = z_ok(nz)
    tpa = pipe_times(timer, fz_any, 80, poison=pz)
    ok_any = ok_any and z_ok(nz)
    tw = timer(fz_wave, 80, poison=pz)
    ok_wave = z_ok(nz)
    fz = fz_over(nz)
    t = timer(fz, 80, poison=pz)
    okz = z_ok(nz)
    tp = pipe_times(timer, fz, 80, poison=pz)
    okz = okz and z_ok(nz)
    t8 = timer(fz_over(8), 80, poison=pz)
    okz8 = z_ok(8)
    # the single-launch read ceiling for these bytes: a plain streaming read
    # of one ZIPF arena per launch, the copies rotated
    zsink = torch.zeros(4, dtype=torch.int32, device=dev)
    zr = zb & ~15

    def fzr_over(nc):
        def fzr(i, st):
            b = i % nc
            lib.tulips_csum_stream_read(az.data_ptr() + b * zr, zr, zsink.data_ptr(), 0, st)
        return fzr
    tr = timer(fzr_over(nz), 80)
    trp = pipe_times(timer, fzr_over(nz), 80)
    tr8 = timer(fzr_over(8), 80)
    ex["ZIPF"] = {"GiBps": round(zb / t / GIB, 1), "Mseg_per_s": round(NSEG / t / 1e6, 1),
                  "frac_of_peak": round(zb / t / 1e9 / HBM_PEAK_GBS, 4),
                  "avg_launch_us": round(t * 1e6, 2),
                  "rotation": f"{nz} copies of the golden Zipf batch ({nz * zb / 1e9:.2f} GB), "
                              "HBM-resident working set",
                  "pipeline": pipe_entry(zb, tp),
                  "entry": "tulips_csum_batch_arena (segments in order in one arena)",
                  "geometry": "span, split form: a workgroup per 28 KiB of arena bytes, "
                              "no halo, chunk prefixes in LDS, boundary chunks loaded by "
                              "the entry holders ahead of the range's last rows; a segment "
                              "crossing ranges is summed in parts that meet in a per-range "
                              "word (one returning atomic per part)",
                  "traffic": read_traffic("ZIPF"),
                  "parity": "ok" if okz else "MISMATCH",
                  "parity_checked": "outputs poisoned before the timed replays; the "
                                    f"{nz} copy digests after them vs the reference's",
                  "read_same_bytes": {"avg_launch_us": round(tr * 1e6, 2),
                                      "frac_of_peak": round(zr / tr / 1e9 / HBM_PEAK_GBS, 4),
                                      "pipeline": pipe_entry(zr, trp)},
                  "mall_assisted": {"rotation": f"8 copies ({8 * zb / 1e6:.0f} MB)",
                                    "avg_launch_us": round(t8 * 1e6, 2),
                                    "frac_of_peak": round(zb / t8 / 1e9 / HBM_PEAK_GBS, 4),
                                    "read_same_bytes_frac": round(
                                        zr / tr8 / 1e9 / HBM_PEAK_GBS, 4),
                                    "parity": "ok" if okz8 else "MISMATCH"},
                  "one_wave_per_segment": {
                      "what": "BASELINE configs[3] as written: tulips_csum_batch with one "
                              "64-lane wave per segment (KIND_SUBGROUP, group 64, unroll 4)",
                      "GBps": round(zb / tw / 1e9, 1),
                      "frac_of_peak": round(zb / tw / 1e9 / HBM_PEAK_GBS, 4),
                      "avg_launch_us": round(tw * 1e6, 2),
                      "parity": "ok" if ok_wave else "MISMATCH"},
                  "any_layout": {
                      "entry": "tulips_csum_batch (offsets only)",
                      "geometry": "packed: one wave per 8 segments, chunks packed end to "
                                  "end, 4 x 64-chunk windows in flight, double-buffered",
                      "GBps": round(zb / ta / 1e9, 1),
                      "frac_of_peak": round(zb / ta / 1e9 / HBM_PEAK_GBS, 4),
                      "avg_launch_us": round(ta * 1e6, 2),
                      "pipeline": pipe_entry(zb, tpa),
                      "parity": "ok" if ok_any else "MISMATCH"}}
    del az, oz

    progress("extras: end-to-end host path")
    # end-to-end host path: F1500 batch from host memory, results back to host
    host = arena[:batch_bytes].cpu().numpy()
    pinned = torch.from_numpy(host.copy()).pin_memory()
    hoffs = (np.arange(NSEG, dtype=np.uint64) * np.uint64(SEG))
    hlens = np.full(NSEG, SEG, dtype=np.uint16)
    e2e = {}
    with csum.HostContext(torch.cuda.current_device()) as ctx:
        for name, src in (("pinned", pinned.data_ptr()), ("pageable", host)):
            ctx.batch(src, hoffs, hlens)
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < 1.0 or reps < 3:
                out = ctx.batch(src, hoffs, hlens)
                reps += 1
            t = (time.perf_counter() - t0) / reps
            e2e[name] = {"GiBps": round(batch_bytes / t / GIB, 2),
                         "ms_per_batch": round(t * 1e3, 3),
                         "parity": "ok" if fnv1a_u16(out) == gold.get("F1500", {}).get(
                             "fnv1a64") else "MISMATCH"}
    ex["e2e_host_F1500"] = e2e
    progress("extras: multi-device host context")
    try:  # every visible device: on a multi-GPU node a failure here must not cost the line
        ex["mctx_host_F1500"] = mctx_leg(torch, csum, pinned, hoffs, hlens, batch_bytes, gold)
    except Exception as e:  # noqa: BLE001
        ex["mctx_host_F1500"] = {"error": repr(e)}
    progress("extras: burst latency")
    ex["burst_latency_host"] = burst_latency(torch, csum)
    progress("extras: beside the resident server")
    ex["F1500_beside_resident_server"] = beside_server(torch, csum, timer, arena, batch_bytes)
    progress("extras: frames, segmentation, RSS")
    ex.update(frame_extras(torch, csum, dev, timer))
    return ex


def mctx_leg(torch, csum, pinned, hoffs, hlens, batch_bytes, gold, ndev=1):
    """The multi-device host context (tulips_csum_mctx) over the run's
    --gpus devices (the extras run at N = 1: device 0): one pinned F1500
    host batch split byte-balanced, each device's shard through its own
    H2D -> kernel -> D2H pipeline at once (PCIe-bound). The N > 1 host-start
    figure is the top-level `host_start` (one rank per GPU)."""
    with csum.MultiContext(list(range(ndev))) as m:
        out = m.batch(pinned.data_ptr(), hoffs, hlens)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 1.0 or reps < 3:
            out = m.batch(pinned.data_ptr(), hoffs, hlens)
            reps += 1
        t = (time.perf_counter() - t0) / reps
        bounds = m.bounds().tolist()
    return {"devices": ndev, "GiBps": round(batch_bytes / t / GIB, 2),
            "ms_per_batch": round(t * 1e3, 3), "shard_bounds": bounds,
            "workload": "F1500 batch 0 from pinned host memory, one tulips_csum_mctx_batch_host "
                        "call per batch",
            "parity": "ok" if fnv1a_u16(out) == gold.get("F1500", {}).get("fnv1a64")
            else "MISMATCH"}


BURSTS = (1, 8, 64, 256, 1024)


def burst_frames(nf):
    """nf TCP frames of 1514 B (checksums generated, so they verify) in 2 KiB
    host slots, as one receive poll burst: (arena, offsets, lengths)."""
    from tulips_amd import csum
    slot = 2048
    rng = np.random.default_rng(nf)
    ar = rng.integers(0, 256, nf * slot, dtype=np.uint8)
    v = ar.reshape(nf, slot)
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, SEG >> 8),
                     (17, SEG & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        v[:, off] = val
    offs = np.arange(nf, dtype=np.uint64) * np.uint64(slot)
    lens = np.full(nf, SEG + 14, np.uint16)
    with csum.HostContext(0) as ctx:
        ctx.generate_frames(ar, offs, lens)
    return ar, offs, lens


def burst_latency(torch, csum):
    """What one receive poll burst costs on the two GPU paths the gpucsum
    decorator takes, timed in C around each library call
    (tulips_csum_time_validate: no interpreter in the loop), frames in a
    page-locked 2 KiB-slot arena as the decorator stages them:
      staged: tulips_csum_validate_frames_host (pinned DMA, launch, D2H);
      zero_copy: tulips_csum_validate_frames_zc, one launch per burst (the
      kernel reads the frames in place over PCIe, descriptors in its
      arguments, flags written to a page-locked mailbox the host spins on);
      zero_copy_resident: the same with resident workgroups polling a
      doorbell (tulips_csum_ctx_set_lowlat); gpu_service_us is the kernel's
      own request-to-flags time from its realtime clock.
    The reference verifies each frame on the CPU as it arrives
    (ipv4/Processor.cpp:94-103, tcpv4/Processor.cpp:121-131); its C-timed
    cost for the same bursts is cpu_baseline.burst_latency."""
    import ctypes as C
    res = {}
    out = (C.c_double * 5)()
    with csum.HostContext(torch.cuda.current_device(), chunk_bytes=4 << 20) as ctx:
        for nf in BURSTS:
            ar, offs, lens = burst_frames(nf)
            pinned = torch.from_numpy(ar).pin_memory()
            flags = np.empty(nf, np.uint8)
            ent = {}
            for name, path, resident in (("staged", 0, False), ("zero_copy", 1, False),
                                         ("zero_copy_resident", 1, True),
                                         ("cpu_product", 2, False), ("decorator", 3, False)):
                ctx.set_lowlat(resident)
                reps = 2000 if nf <= 64 else 300
                rc = _bench().lib.tulips_csum_time_validate(
                    ctx._h, path, pinned.data_ptr(), offs.ctypes.data, lens.ctypes.data, nf,
                    reps, flags.ctypes.data, out)
                if rc:
                    ent[name] = {"error": rc}
                    continue
                ent[name] = {"us_median": round(out[0], 2), "us_p99": round(out[1], 2),
                             "us_min": round(out[2], 2), "reps": reps,
                             "parity": "ok" if bool((flags == 0x0F).all()) else "MISMATCH"}
                if path == 1:
                    ent[name]["gpu_service_us"] = round(out[4], 2)
            res[str(nf)] = ent
    # the same bursts cold: a 256 MB page-locked ring of copies of the
    # burst, one copy per call, so the host code meets frames outside the
    # CPU caches (as frames a NIC has just written by DMA would be)
    cold = {}
    ring_bytes = 256 << 20
    with csum.HostContext(torch.cuda.current_device(), chunk_bytes=4 << 20) as ctx:
        for nf in (1, 8, 64, 96, 128, 256, 1024):
            ar, offs, lens = burst_frames(nf)
            nb = ring_bytes // len(ar)
            ring = torch.from_numpy(np.tile(ar, nb)).pin_memory()
            flags = np.empty(nf, np.uint8)
            ent = {}
            for name, path in (("zero_copy", 1), ("cpu_product", 2), ("decorator", 3)):
                ctx.set_lowlat(False)
                reps = int(min(nb, 2000))
                rc = _bench().lib.tulips_csum_time_validate_ring(
                    ctx._h, path, ring.data_ptr(), len(ar), nb, offs.ctypes.data,
                    lens.ctypes.data, nf, reps, flags.ctypes.data, out)
                ent[name] = ({"error": rc} if rc else
                             {"us_median": round(out[0], 2), "us_p99": round(out[1], 2),
                              "reps": reps, "parity": "ok" if bool((flags == 0x0F).all())
                              else "MISMATCH"})
            cold[str(nf)] = ent
            del ring
    # the burst size from which the zero-copy launch beats the host code
    cross = None
    for nf in BURSTS:
        e = res[str(nf)]
        if "us_median" in e.get("zero_copy", {}) and "us_median" in e.get("cpu_product", {}) \
                and e["zero_copy"]["us_median"] < e["cpu_product"]["us_median"]:
            cross = nf
            break
    return {"workload": "TCP frames of 1514 B in 2 KiB page-locked host slots, one "
                        "validation call per burst, C-timed (tulips_csum_time_validate); "
                        "cpu_product = tulips_csum_validate_frames_cpu, the library's host "
                        "code the gpucsum decorator uses below its crossover; decorator = "
                        "the decorator's default choice per burst "
                        "(tulips_csum_burst_prefers_cpu: CPU below 96 frames and 96 x 1514 B)",
            "gpu_beats_cpu_from_burst": cross,
            "bursts": res,
            "cold_ring": {"what": "the same bursts from a 256 MB page-locked ring, a "
                                  "different copy per call (tulips_csum_time_validate_ring)",
                          "bursts": cold}}


def beside_server(torch, csum, timer, arena, batch_bytes):
    """What the resident low-latency server (8 workgroups of 1,024 threads
    polling the mailbox, tulips_csum_ctx_set_lowlat) costs a bulk kernel
    sharing the GPU: the F1500 serial launch rate with the server idle-
    polling beside it, against the same launches without it."""
    fixed = checked_lib(csum).tulips_csum_batch_fixed
    outs = torch.empty(NBATCH * NSEG, dtype=torch.uint16, device=arena.device)

    def f(i, st):
        b = i % NBATCH
        fixed(arena.data_ptr() + b * batch_bytes, SEG, SEG, None, None, None,
              outs.data_ptr() + b * NSEG * 2, NSEG, 0, st)
    t_alone = timer(f, 64)
    ar, offs, lens = burst_frames(8)
    pinned = torch.from_numpy(ar).pin_memory()
    with csum.HostContext(torch.cuda.current_device()) as ctx:
        ctx.set_lowlat(True)
        fl = ctx.validate_frames(pinned.numpy(), offs, lens, low_latency=True)
        # the server idles out 100 ms after its last burst: the capture,
        # warm replay and timed replay of 64 launches take a few ms
        t_srv = timer(f, 64)
        fl2 = ctx.validate_frames(pinned.numpy(), offs, lens, low_latency=True)
    ok = bool((fl == 0x0F).all()) and bool((fl2 == 0x0F).all())
    return {"what": "F1500 serial launches with the resident zero-copy server idle-polling "
                    "on the same GPU (8 x 1,024-thread workgroups) vs without",
            "avg_launch_us_alone": round(t_alone * 1e6, 2),
            "avg_launch_us_with_server": round(t_srv * 1e6, 2),
            "slowdown": round(t_srv / t_alone, 4),
            "parity": "ok" if ok else "MISMATCH"}


def rate_entry(alg_bytes, t, **kw):
    gbs = alg_bytes / t / 1e9
    d = {"GBps": round(gbs, 1), "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4),
         "avg_launch_us": round(t * 1e6, 2), "bytes_per_launch": int(alg_bytes)}
    d.update(kw)
    return d


def frame_extras(torch, csum, dev, timer):
    """§8f rows: frame validation / generation (receive and send sides),
    segmentation offload and the Toeplitz RSS batch, each on device-resident
    synthetic frames with its own parity check."""
    lib = checked_lib(csum)
    ex = {}
    # 8 bursts x 65,536 TCP frames of 1514 B (MTU 1500) in 2 KiB receive
    # slots (the OFED RX layout, include/tulips/transport/ofed/Device.h:25),
    # 1.07 GB in all so the rotation streams from HBM.
    nf, slot, flen, nb = NSEG, 2048, SEG + 14, 8
    ar = torch.empty(nb * nf * slot, dtype=torch.uint8, device=dev)
    _bench().fill_splitmix(ar, seed=0xF4A3E5)
    v = ar.view(nb * nf, slot)
    for off, val in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, SEG >> 8),
                     (17, SEG & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        v[:, off] = val
    offs = torch.arange(nf, dtype=torch.int64, device=dev) * slot
    lens = torch.full((nf,), flen, dtype=torch.int16, device=dev)
    flags = torch.empty(nb * nf, dtype=torch.uint8, device=dev)
    burst = nf * slot
    alg = nf * flen
    gen, val = lib.tulips_csum_generate_frames, lib.tulips_csum_validate_frames

    def fgen(i, st):
        b = i % nb
        gen(ar.data_ptr() + b * burst, offs.data_ptr(), lens.data_ptr(), nf, None, st)

    def fval(i, st):
        b = i % nb
        val(ar.data_ptr() + b * burst, offs.data_ptr(), lens.data_ptr(), nf,
            flags.data_ptr() + b * nf, None, st)
    def gen_poison():
        # both checksum fields of every frame: what the timed replay must write
        # (checked below by the fields comparison and by validation == 0x0F)
        v[:, 24:26].fill_(POISON)
        v[:, 50:52].fill_(POISON)
    for i in range(nb):
        fgen(i, torch.cuda.current_stream().cuda_stream)
    t = timer(fgen, 64, poison=gen_poison)
    tp = pipe_times(timer, fgen, 64, poison=gen_poison)
    ex["frames_generate_F1514"] = rate_entry(
        alg, t, kernel="frame_kernel<GENERATE, 16 lanes x 6 chunks per frame>",
        workload="65,536 x 1514 B TCP frames per launch, 2 KiB slots, 8 bursts rotated",
        pipeline=pipe_entry(alg, tp), traffic=read_traffic("frames_generate_F1514"))
    # compact-field generation: the same two values per frame, returned as
    # one u32 instead of patched in place (frames only read); algorithmic
    # bytes = the frames read + 4 B written per frame. Parity: the values
    # equal the fields the in-place generation wrote (bytes 24-25, 50-51)
    fields = torch.empty(nb * nf, dtype=torch.int32, device=dev)
    gfl = lib.tulips_csum_generate_fields

    def ffld(i, st):
        b = i % nb
        gfl(ar.data_ptr() + b * burst, offs.data_ptr(), lens.data_ptr(), nf,
            fields.data_ptr() + b * nf * 4, None, st)
    for i in range(nb):
        ffld(i, torch.cuda.current_stream().cuda_stream)
    t = timer(ffld, 64, poison=poisoner(fields))
    tp = pipe_times(timer, ffld, 64, poison=poisoner(fields))
    fv = v.view(nb * nf, slot)
    want = (fv[:, 24].int() | (fv[:, 25].int() << 8) | (fv[:, 50].int() << 16) |
            (fv[:, 51].int() << 24))
    ok = bool((fields == want).all().item())
    ex["frames_generate_fields_F1514"] = rate_entry(
        alg + 4 * nf, t, kernel="frame_kernel<FIELDS, 16 lanes x 6 chunks per frame>",
        workload="same frames: tulips_csum_generate_fields, one u32 per frame out",
        pipeline=pipe_entry(alg + 4 * nf, tp), parity="ok" if ok else "MISMATCH",
        traffic=read_traffic("frames_generate_fields_F1514"))
    del fields, fv, want
    t = timer(fval, 64, poison=poisoner(flags))
    ok = bool((flags == 0x0F).all().item())
    tp = pipe_times(timer, fval, 64, poison=poisoner(flags))
    ok = ok and bool((flags == 0x0F).all().item())
    ex["frames_validate_F1514"] = rate_entry(
        alg, t, kernel="frame_kernel<VALIDATE, 16 lanes x 6 chunks per frame>",
        workload="same frames: generated checksums verified (flags == 0x0F)",
        pipeline=pipe_entry(alg, tp), parity="ok" if ok else "MISMATCH",
        traffic=read_traffic("frames_validate_F1514"))
    # the frame kernels' read pattern without the arithmetic, over the same
    # rotated bursts: the ceiling those kernels are held against
    fsink = torch.zeros(4, dtype=torch.int32, device=dev)

    def frd(i, st):
        b = i % nb
        lib.tulips_csum_stream_read_slots(ar.data_ptr() + b * burst, slot, flen, nf,
                                          fsink.data_ptr(), st)
    t = timer(frd, 64)
    tp = pipe_times(timer, frd, 64)
    ex["frames_validate_F1514"]["read_same_bytes"] = {
        "what": "tulips_csum_stream_read_slots: the frame kernels' loads (one 16-lane "
                "subgroup per 1514 B frame in its 2 KiB slot, 6 clamped loads per lane), "
                "no arithmetic",
        "avg_launch_us": round(t * 1e6, 2),
        "frac_of_peak": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
        "pipeline": pipe_entry(alg, tp)}
    del ar, v, flags

    # Segmentation offload: 4 batches x 1024 super-frames of 64,294 B (44 x
    # 1460 B payload) -> 45,056 segments of <= 1514 B in 1536 B slots.
    nsf, pay, mss = 1024, 44 * 1460, 1460
    sflen = 54 + pay
    sslot = 65536
    sb = 4
    sa = torch.empty(sb * nsf * sslot, dtype=torch.uint8, device=dev)
    _bench().fill_splitmix(sa, seed=0x7505)
    sv = sa.view(sb * nsf, sslot)
    tot = sflen - 14
    for off, val_ in ((12, 0x08), (13, 0), (14, 0x45), (15, 0), (16, tot >> 8),
                      (17, tot & 0xFF), (20, 0x40), (21, 0), (23, 6), (46, 0x50)):
        sv[:, off] = val_
    soffs = torch.arange(nsf, dtype=torch.int64, device=dev) * sslot
    slens = torch.full((nsf,), sflen - 65536 if sflen > 32767 else sflen,  # u16 bits
                       dtype=torch.int16, device=dev)
    nseg = nsf * (pay // mss)
    ostride = 1536
    sout = torch.empty(sb * nseg * ostride, dtype=torch.uint8, device=dev)
    solen = torch.zeros(sb * nseg, dtype=torch.int16, device=dev)
    sfirst = torch.empty(sb * (nsf + 1), dtype=torch.int32, device=dev)
    seg = lib.tulips_csum_segment_frames

    def fseg(i, st):
        b = i % sb
        seg(sa.data_ptr() + b * nsf * sslot, soffs.data_ptr(), slens.data_ptr(), nsf, mss,
            sout.data_ptr() + b * nseg * ostride, ostride, nseg,
            solen.data_ptr() + b * nseg * 2, sfirst.data_ptr() + b * (nsf + 1) * 4, st)
    for i in range(sb):
        fseg(i, torch.cuda.current_stream().cuda_stream)
    t = timer(fseg, 32, replays=3, poison=poisoner(sout, solen, sfirst))
    tp = pipe_times(timer, fseg, 32, poison=poisoner(sout, solen, sfirst))
    moved = nsf * sflen + nseg * (54 + mss)       # read super-frames + write segments
    so = torch.arange(nseg, dtype=torch.int64, device=dev) * ostride
    ok = True
    for b in range(sb):     # every rotated call's segments, written in the timed replays
        sfl = csum.validate_frames(sout[b * nseg * ostride:(b + 1) * nseg * ostride], so,
                                   solen[b * nseg:(b + 1) * nseg])
        ok = ok and bool((sfl == 0x0F).all().item()) and \
            int(sfirst[b * (nsf + 1) + nsf].item()) == nseg
    counted = rate_entry(
        moved, t, kernel="seg_prologue_small_kernel + segment_kernel<16,6> "
                         "(16-lane subgroup per output segment)",
        entry="tulips_csum_segment_frames (segment counts computed on the device)",
        segments_per_s=round(nseg / t / 1e6, 2) * 1e6, pipeline=pipe_entry(moved, tp),
        traffic=read_traffic("segment_TSO_64K_mss1460_device_counted"),
        parity="ok" if ok else "MISMATCH")
    # the same calls with the caller's plan (tulips_csum_segment_frames_planned:
    # first[] from the host, as the reference's transport decides the TSO
    # split on the host, src/stack/Utils.cpp:67-84, src/transport/ofed/
    # Device.cpp:688-700): the segment kernel alone, no prologue. The plan is
    # tulips_csum_segment_plan_host over the super-frames' headers; parity:
    # it equals the device prologue's first[], and every rotated call's
    # output bytes and lengths equal the prologue form's
    hdr = sv[:nsf, :64].cpu().numpy().reshape(-1)
    plan = csum.segment_plan(hdr, np.arange(nsf, dtype=np.uint64) * np.uint64(64),
                             np.full(nsf, sflen, dtype=np.uint16), mss)
    plan_ok = bool(np.array_equal(plan.view(np.int32), sfirst[:nsf + 1].cpu().numpy()))
    dplan = torch.from_numpy(plan.view(np.int32).copy()).to(dev)
    ref_out, ref_len = sout.clone(), solen.clone()
    segp = lib.tulips_csum_segment_frames_planned

    def fsegp(i, st):
        b = i % sb
        segp(sa.data_ptr() + b * nsf * sslot, soffs.data_ptr(), slens.data_ptr(), nsf, mss,
             dplan.data_ptr(), sout.data_ptr() + b * nseg * ostride, ostride, nseg,
             solen.data_ptr() + b * nseg * 2, st)
    t = timer(fsegp, 32, replays=3, poison=poisoner(sout, solen))
    okp = plan_ok and bool(torch.equal(sout, ref_out)) and bool(torch.equal(solen, ref_len))
    tp = pipe_times(timer, fsegp, 32, poison=poisoner(sout, solen))
    okp = okp and bool(torch.equal(sout, ref_out)) and bool(torch.equal(solen, ref_len))
    # the TSO path as the product runs it (the decorator's transmit side and
    # tulips_csum_segment_frames_host plan on the host): the planned entry;
    # the device-counted form beside it
    ex["segment_TSO_64K_mss1460"] = rate_entry(
        moved, t, kernel="segment_planned_kernel<16,6> (frames found from the caller's "
                         "first[], headers parsed in the segment kernel, no prologue)",
        entry="tulips_csum_segment_frames_planned (plan from tulips_csum_segment_plan_host)",
        workload="1024 super-frames of 64,294 B -> 45,056 segments of 1514 B per call",
        traffic=read_traffic("segment_TSO_64K_mss1460"),
        segments_per_s=round(nseg / t / 1e6, 2) * 1e6, pipeline=pipe_entry(moved, tp),
        parity="ok" if okp else "MISMATCH", device_counted=counted)
    # the segment kernel's loads and stores without its header work, over the
    # same rotated source: slot k copies [frame + (k % 44) * 1460, + 1514) to
    # its 1536 B slot (tulips_csum_stream_copy_slots); the ceiling the
    # segmentation figure is held against. Parity: every slot's payload bytes
    # equal the planned segmentation's
    cout = torch.empty_like(sout)

    def fcopy(i, st):
        b = i % sb
        lib.tulips_csum_stream_copy_slots(sa.data_ptr() + b * nsf * sslot, sslot, pay // mss,
                                          mss, 54 + mss, nseg,
                                          cout.data_ptr() + b * nseg * ostride, ostride, st)
    t = timer(fcopy, 32, replays=3)
    tp = pipe_times(timer, fcopy, 32)
    okc = bool(torch.equal(cout.view(-1, ostride)[:, 54:54 + mss],
                           sout.view(-1, ostride)[:, 54:54 + mss]))
    ex["segment_TSO_64K_mss1460"]["copy_same_bytes"] = {
        "what": "tulips_csum_stream_copy_slots: the segment kernel's loads and stores (one "
                "16-lane subgroup per 1514 B slot, dword-aligned loads, funnel shift, "
                "nontemporal stores), no header parse, patch or sums",
        "avg_launch_us": round(t * 1e6, 2),
        "frac_of_peak": round(moved / t / 1e9 / HBM_PEAK_GBS, 4),
        "pipeline": pipe_entry(moved, tp),
        "parity": "ok" if okc else "MISMATCH"}
    del sa, sv, sout, cout, ref_out, ref_len

    # Toeplitz RSS over 16M tuples (12 B in, 4 B out per tuple)
    nt = 1 << 24
    g = torch.Generator(device="cpu").manual_seed(5)
    tup = torch.randint(0, 2**31 - 1, (4, nt), generator=g, dtype=torch.int64)
    sa_, da_ = tup[0].to(torch.int32).to(dev), tup[1].to(torch.int32).to(dev)
    sp_, dp_ = tup[2].to(torch.int16).to(dev), tup[3].to(torch.int16).to(dev)
    key = bytes(range(1, 41))
    rout = torch.empty(nt, dtype=torch.int32, device=dev)
    kb = (np.frombuffer(key, dtype=np.uint8)).copy()
    kp = kb.ctypes.data_as(__import__("ctypes").POINTER(__import__("ctypes").c_uint8))
    rss = lib.tulips_rss_toeplitz_batch

    def frss(i, st):
        rss(sa_.data_ptr(), da_.data_ptr(), sp_.data_ptr(), dp_.data_ptr(), nt, kp, len(key),
            0, rout.data_ptr(), st)
    frss(0, torch.cuda.current_stream().cuda_stream)
    t = timer(frss, 32, poison=poisoner(rout))
    tp = pipe_times(timer, frss, 32, poison=poisoner(rout))
    # parity: 2,048 tuples spread over the batch against the host symbol
    js = torch.arange(0, nt, nt // 2048)
    cols = [x.cpu().numpy() for x in (sa_[js], da_[js], sp_[js], dp_[js], rout[js])]
    ok = all((int(cols[4][k]) & 0xFFFFFFFF) ==
             csum.toeplitz(int(cols[0][k]) & 0xFFFFFFFF, int(cols[1][k]) & 0xFFFFFFFF,
                           int(cols[2][k]) & 0xFFFF, int(cols[3][k]) & 0xFFFF, key, 0)
             for k in range(len(js)))
    ex["rss_toeplitz_16M"] = rate_entry(
        nt * 16, t, kernel="rss_kernel<VEC> (4 byte + 16 nibble LDS tables, 4 tuples per thread)", Mtuples_per_s=round(nt / t / 1e6, 1),
        pipeline=pipe_entry(nt * 16, tp), parity="ok" if ok else "MISMATCH",
        traffic=read_traffic("rss_toeplitz_16M"))
    return ex


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(arena, batch_bytes, seconds):
    """The reference CPU checksum (oracle/_ref: the reference's own src/stack
    compiled with -O3 -mssse3), else the C restatement, on this box's cores,
    over the first F1500 batch of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import REF_CLANG_SO, Oracle, Reference  # noqa: E402 (cpu_baseline leg only)
    if Reference.available():
        impl, kind = Reference(), "reference"
    else:
        impl, kind = Oracle(), "port"
    host = arena[:batch_bytes].cpu().numpy()
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    threads = max(1, min(16, ncpu))

    def rate(nt, impl=impl):
        impl.batch(host, stride=SEG, fixed_len=SEG, n=NSEG, nthreads=nt)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            impl.batch(host, stride=SEG, fixed_len=SEG, n=NSEG, nthreads=nt)
            reps += 1
        return reps * batch_bytes / (time.perf_counter() - t0) / GIB, reps

    r1, n1 = rate(1)
    rN, nN = rate(threads)
    res = {"value": round(rN, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
           "value_1core": round(r1, 3),
           "sample": f"F1500 batch 0 (65,536 x 1500 B = 98.3 MB) copied to host; "
                     f"{nN} passes on {threads} pinned threads + {n1} passes on 1 "
                     f"thread, ~{seconds:.1f} s wall each; g++ -O3 -mssse3"}
    res["cpu_model"] = cpu_model()
    # the reference's per-frame receive verification over the same bursts as
    # extras.burst_latency_host: ipv4::checksum of each header and the tcpv4
    # checksum of each segment (its own build), one thread, as the stack's
    # poll loop runs it, timed in C (oracle/ref_harness.cpp
    # ref_time_verify_burst)
    lat = {}
    if kind == "reference":
        import ctypes as C
        f = impl.lib.ref_time_verify_burst
        f.restype = C.c_uint32
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                      C.c_void_p]
        out = (C.c_double * 4)()
        for nf in BURSTS:
            far, foffs, flens = burst_frames(nf)
            reps = 20000 if nf <= 64 else 2000
            good = f(far.ctypes.data, foffs.ctypes.data, flens.ctypes.data, nf, reps,
                     C.addressof(out))
            lat[str(nf)] = {"us_median": round(out[0], 3), "us_p99": round(out[1], 3),
                            "ns_per_frame": round(out[0] * 1e3 / nf, 1), "reps": reps,
                            "parity": "ok" if good == nf else "MISMATCH"}
    res["burst_latency"] = {"what": "reference ipv4 + tcpv4 checksum verification of each "
                                    "frame of the burst, 1 thread, C-timed "
                                    "(oracle/ref_harness.cpp ref_time_verify_burst)",
                            "bursts": lat}
    if kind == "reference" and Reference.available(REF_CLANG_SO):
        # the same reference sources built with clang, the compiler the
        # reference's CMake prefers (CMakeLists.txt:20-21)
        clang = Reference(REF_CLANG_SO)
        c1, _ = rate(1, clang)
        cN, _ = rate(threads, clang)
        res["clang"] = {"value": round(cN, 3), "value_1core": round(c1, 3),
                        "build": "clang++ (ROCm LLVM) -O3 -mssse3"}
    return res


if __name__ == "__main__":
    main()
