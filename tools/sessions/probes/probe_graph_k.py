#!/usr/bin/env python3
"""Replay time of the headline graph against its step count K: the bench's
F1500 launches (batch i % 16) captured as one graph on B branches, each K
timed over REPS replays (median) behind the bench's 200 us start gate, for
each B in $BRANCHES (default 16 and 1). A straight-line fit t = a + b K
separates the per-replay cost a from the per-step cost b. Measurement only; prints JSON lines."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from tulips_amd import csum  # noqa: E402


def main():
    ks = [int(x) for x in os.environ.get("KS", "1 2 4 8 16 20 32 64 128").split()]
    reps = int(os.environ.get("REPS", "7"))
    mainb = os.environ.get("MAIN_BRANCH", "0") == "1"
    dev = torch.device("cuda", 0)
    lib = csum.lib
    SEG, NSEG, NB = bench.SEG, bench.NSEG, bench.NBATCH
    bb = SEG * NSEG
    arena = torch.empty(NB * bb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(arena, NB * bb, seed=bench.DATA_SEED, byte_off=0)
    outs = torch.empty(NB * NSEG, dtype=torch.uint16, device=dev)
    base, optr = arena.data_ptr(), outs.data_ptr()
    main_s = torch.cuda.current_stream()

    def launch(i, st):
        b = i % NB
        rc = lib.tulips_csum_batch_fixed(base + b * bb, SEG, SEG, None, None, None,
                                         optr + b * NSEG * 2, NSEG, 0, st)
        assert rc == 0, rc

    for i in range(32):
        launch(i, main_s.cuda_stream)
    torch.cuda.synchronize()
    for nbr in [int(x) for x in os.environ.get("BRANCHES", "16 1").split()]:
        side = [torch.cuda.Stream() for _ in range(nbr)]
        rows = []
        for k in ks:
            g = torch.cuda.CUDAGraph()
            used = min(nbr, k)
            with torch.cuda.graph(g):
                m = torch.cuda.current_stream()
                # MAIN_BRANCH=1: branch 0 is the capture stream itself (its
                # launches need no fork edge), the others fork from it
                br = ([m] + side[:used - 1]) if mainb else side[:used]
                for sd in br:
                    if sd is not m:
                        sd.wait_stream(m)
                for i in range(k):
                    launch(i, br[i % used].cuda_stream)
                for sd in br:
                    if sd is not m:
                        m.wait_stream(sd)
            g.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                bench.gate(main_s)
                a.record(main_s)
                g.replay()
                b.record(main_s)
                b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            t = float(np.median(ts))
            rows.append((k, t))
            print(json.dumps({"branches": nbr, "main_branch": mainb, "steps": k, "us_median": round(t, 2),
                              "us_min": round(min(ts), 2),
                              "gib_s": round(k * bb / (t * 1e-6) / bench.GIB, 1)}), flush=True)
            del g
        x = np.array([r[0] for r in rows], float)
        y = np.array([r[1] for r in rows], float)
        sel = x >= 4
        bfit, afit = np.polyfit(x[sel], y[sel], 1)
        print(json.dumps({"branches": nbr, "fit_K_ge_4": {"per_replay_us": round(afit, 2),
                                                          "per_step_us": round(bfit, 3)}}),
              flush=True)


if __name__ == "__main__":
    main()
