#!/usr/bin/env python3
"""The captured-graph churn of tests/test_fuzz.py::test_fuzz_captured_graphs
with TORCH kernels only (no library call): graphs of 1-6 calls (x_k.add_)
round-robin over 1-4 side streams forked from and joined to the capture
stream, at most 8 live, replayed on fresh pool streams, direct ops beside
them, random drops. If this crashes in hipGraphLaunch as the library's fuzz
does, the fault is the runtime's, not the library's. Variants (env):
NOEMPTY=1 never forks a side stream that gets no work; SAME=1 replays on the
current stream instead of a fresh pool stream; NODROP=1 never destroys a
graph while others live (at most 8 are made); MAXLIVE=k keeps at most k
graphs (a new capture drops one); KEEPALL=1 never destroys a graph and
keeps capturing; SYNCDROP=1 synchronises the device and collects garbage
before and after every graph destruction (the teardown-order test ADVICE r05
asked for). Prints progress; a crash ends the process (exit 139).

The fault (profiles/graph_crash_r05.txt): hip::Graph::UpdateStreams, called
from hip::GraphExec::Run, reads a NULL or stale entry of the launched
executable's parallel-stream list."""
import gc
import os
import time

import numpy as np
import torch

rng = np.random.default_rng(int(os.environ.get("SEED", "1")))
budget = float(os.environ.get("SECS", "60"))
xs = [torch.zeros(1 << 16, device="cuda:0") for _ in range(6)]
graphs = []


def drop(k):
    if os.environ.get("SYNCDROP"):
        torch.cuda.synchronize()
        graphs.pop(k)
        gc.collect()
        torch.cuda.synchronize()
    else:
        graphs.pop(k)


t0 = last = time.monotonic()
steps = 0
while time.monotonic() - t0 < budget:
    op = rng.random()
    if (op < 0.3 or not graphs) and not (os.environ.get("NODROP") and len(graphs) >= 8):
        ncalls = int(rng.integers(1, 7))
        outs = [torch.zeros(1 << 16, device="cuda:0") for _ in range(ncalls)]
        cap = torch.cuda.Stream()
        nside = int(rng.integers(1, 5))
        if os.environ.get("NOEMPTY"):
            nside = min(nside, ncalls)
        side = [torch.cuda.Stream() for _ in range(nside)]
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            main = torch.cuda.current_stream()
            for sd in side:
                sd.wait_stream(main)
            for i in range(ncalls):
                with torch.cuda.stream(side[i % len(side)]):
                    outs[i].add_(xs[i])
            for sd in side:
                main.wait_stream(sd)
        graphs.append((g, outs))
        if not os.environ.get("KEEPALL") and len(graphs) > int(os.environ.get("MAXLIVE", "8")):
            drop(int(rng.integers(0, len(graphs))))
    elif op < 0.75:
        g, outs = graphs[int(rng.integers(0, len(graphs)))]
        for o in outs:
            o.fill_(0)
        torch.cuda.synchronize()
        if os.environ.get("SAME"):
            g.replay()
        else:
            with torch.cuda.stream(torch.cuda.Stream()):
                g.replay()
        torch.cuda.synchronize()
    elif op < 0.95:
        o = torch.zeros(1 << 16, device="cuda:0")
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            o.add_(xs[0])
        torch.cuda.synchronize()
    elif not os.environ.get("NODROP") and not os.environ.get("KEEPALL"):
        drop(int(rng.integers(0, len(graphs))))
    steps += 1
    if time.monotonic() - last > 10:
        last = time.monotonic()
        print(f"torch churn: {steps} steps, {last - t0:.0f} s", flush=True)
print(f"torch churn: {steps} steps, no crash", flush=True)
