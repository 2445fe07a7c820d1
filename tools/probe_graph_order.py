#!/usr/bin/env python3
"""Does a multi-branch HIP graph launched on a stream start only after the
stream's earlier work? Torch kernels only, on the runtime
torch bundles: 16 graphs of 1-6 `out_k.copy_(x_k)` kernels round-robin over
1-4 side streams forked from and joined to the capture stream, kept alive
(no graph is destroyed: that is the other runtime fault); then, repeatedly,
on one of 4 non-default streams: every output of a graph poisoned by a fill
kernel, the graph replayed on the same stream with no host synchronisation
in between, the stream synchronised, the outputs checked. A poisoned word
after the replay means a branch ran before (or beside) the fill queued ahead
of it. SECS (default 30) bounds the run; prints one JSON line."""
import json
import os
import time

import numpy as np
import torch

rng = np.random.default_rng(int(os.environ.get("SEED", "1")))
budget = float(os.environ.get("SECS", "30"))
n = 1 << 14
xs = [torch.arange(n, device="cuda:0", dtype=torch.float32) + k for k in range(6)]
graphs = []
for _ in range(16):
    ncalls = int(rng.integers(1, 7))
    nside = int(rng.integers(1, 5))
    outs = [torch.zeros(n, device="cuda:0") for _ in range(ncalls)]
    cap = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(nside)]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        main = torch.cuda.current_stream()
        for sd in side:
            sd.wait_stream(main)
        for i in range(ncalls):
            with torch.cuda.stream(side[i % nside]):
                outs[i].copy_(xs[i])
        for sd in side:
            main.wait_stream(sd)
    graphs.append((g, outs, nside))
pool = [torch.cuda.Stream() for _ in range(4)]
torch.cuda.synchronize()
t0 = time.monotonic()
replays = bad = 0
examples = []
while time.monotonic() - t0 < budget:
    gi = int(rng.integers(0, len(graphs)))
    g, outs, nside = graphs[gi]
    s = pool[int(rng.integers(0, len(pool)))]
    with torch.cuda.stream(s):
        for o in outs:
            o.fill_(-1.0)
        g.replay()
    s.synchronize()
    for i, o in enumerate(outs):
        poisoned = int((o == -1.0).sum())
        if poisoned:
            bad += 1
            if len(examples) < 8:
                examples.append({"replay": replays, "graph": gi, "call": i, "calls": len(outs),
                                 "branches": nside, "poison_words": poisoned})
    replays += 1
print(json.dumps({"graph_order_s": budget, "replays": replays, "mismatches": bad,
                  "examples": examples, "torch": torch.__version__,
                  "hip": torch.version.hip}), flush=True)
