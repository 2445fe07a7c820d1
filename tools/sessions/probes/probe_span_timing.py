#!/usr/bin/env python3
"""Where do the ~35 us that separate bench.py's 20-step figure from its
1,024-step figure go? The same K launches of the headline (F1500, batch i % 16,
16 branches) timed four ways, ROUNDS alternations, results poisoned before each
timed region and digested after:

  graph_main  the bench's current region: gate + start event on the launch
              stream, one graph replay (fork -> 16 branches -> join), end event
  eager_main  the same fork/join issued eagerly behind the gate, events on the
              launch stream (so the fork and join barriers are inside)
  eager_span  eager launches behind the gate, a start event on every branch
              after its fork wait and an end event after its last launch;
              region = earliest branch start .. latest branch end
  graph_span  the graph with the per-branch start/end events captured into it
              (external events), same region rule; skipped if unsupported

Measurement only; prints JSON lines."""
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
    steps_list = [int(x) for x in os.environ.get("STEPS", "20 1024").split()]
    rounds = int(os.environ.get("ROUNDS", "3"))
    nbr = int(os.environ.get("BRANCHES", "16"))
    gate_us = int(os.environ.get("GATE_US", "0"))
    dev = torch.device("cuda", 0)
    lib = csum.lib
    SEG, NSEG, NB = bench.SEG, bench.NSEG, bench.NBATCH
    bb = SEG * NSEG
    arena = torch.empty(NB * bb + 256, dtype=torch.uint8, device=dev)
    csum.fill_splitmix(arena, NB * bb, seed=bench.DATA_SEED, byte_off=0)
    outs = torch.empty(NB * NSEG, dtype=torch.uint16, device=dev)
    base, optr = arena.data_ptr(), outs.data_ptr()
    main_s = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(nbr)]

    def launch(i, st):
        b = i % NB
        rc = lib.tulips_csum_batch_fixed(base + b * bb, SEG, SEG, None, None, None,
                                         optr + b * NSEG * 2, NSEG, 0, st)
        assert rc == 0, rc

    for i in range(32):
        launch(i, main_s.cuda_stream)
    torch.cuda.synchronize()
    want = bench.fnv1a_u16(outs.cpu().numpy().view(np.uint16))

    def sleep(us):
        rc = lib.tulips_csum_gpu_sleep(us, main_s.cuda_stream)
        assert rc == 0

    def poison():
        outs.view(torch.uint8).fill_(0xA5)
        torch.cuda.synchronize()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def check(k):
        if k >= NB:
            got = bench.fnv1a_u16(outs.cpu().numpy().view(np.uint16))
            assert got == want, "digest mismatch"

    def eager_issue(k, starts=None, ends=None):
        fork = torch.cuda.Event()
        fork.record(main_s)
        used = min(nbr, k)
        for j in range(used):
            side[j].wait_event(fork)
            if starts is not None:
                starts[j].record(side[j])
        for i in range(k):
            launch(i, side[i % used].cuda_stream)
        for j in range(used):
            if ends is not None:
                ends[j].record(side[j])
            main_s.wait_stream(side[j])

    def capture(k, with_events):
        g = torch.cuda.CUDAGraph()
        used = min(nbr, k)
        starts = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(used)]
        ends = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(used)]
        with torch.cuda.graph(g):
            m = torch.cuda.current_stream()
            for j in range(used):
                side[j].wait_stream(m)
                if with_events:
                    starts[j].record(side[j])
            for i in range(k):
                launch(i, side[i % used].cuda_stream)
            for j in range(used):
                if with_events:
                    ends[j].record(side[j])
                m.wait_stream(side[j])
        g.replay()
        torch.cuda.synchronize()
        return g, starts, ends

    def span(ref, starts, ends):
        t0 = min(ref.elapsed_time(s) for s in starts)
        t1 = max(ref.elapsed_time(e) for e in ends)
        return (t1 - t0) / 1e3

    for k in steps_list:
        gus = gate_us or max(200, 30 * k)
        g_main, _, _ = capture(k, False)
        try:
            g_span, gs, ge = capture(k, True)
        except Exception as e:  # noqa: BLE001
            g_span = None
            print(json.dumps({"graph_span": "unsupported", "error": str(e)[:200]}), flush=True)
        res = {"graph_main": [], "eager_main": [], "eager_span": [], "graph_span": []}
        for r in range(rounds):
            # graph_main
            poison()
            a, b = ev(), ev()
            sleep(200)
            a.record(main_s)
            g_main.replay()
            b.record(main_s)
            torch.cuda.synchronize()
            check(k)
            res["graph_main"].append(a.elapsed_time(b) / 1e3)
            # eager_main
            poison()
            a, b = ev(), ev()
            sleep(gus)
            a.record(main_s)
            eager_issue(k)
            b.record(main_s)
            torch.cuda.synchronize()
            check(k)
            res["eager_main"].append(a.elapsed_time(b) / 1e3)
            # eager_span
            poison()
            used = min(nbr, k)
            ref = ev()
            starts = [ev() for _ in range(used)]
            ends = [ev() for _ in range(used)]
            ref.record(main_s)
            sleep(gus)
            eager_issue(k, starts, ends)
            torch.cuda.synchronize()
            check(k)
            res["eager_span"].append(span(ref, starts, ends))
            # graph_span
            if g_span is not None:
                poison()
                ref = ev()
                ref.record(main_s)
                sleep(200)
                g_span.replay()
                torch.cuda.synchronize()
                check(k)
                try:
                    res["graph_span"].append(span(ref, gs, ge))
                except Exception as e:  # noqa: BLE001
                    res["graph_span"] = ["error: " + str(e)[:200]]
                    g_span = None
        out = {"steps": k, "branches": nbr, "gate_us_eager": gus}
        for name, ts in res.items():
            ts = [t for t in ts if isinstance(t, float)]
            if ts:
                out[name] = {"gib_s": [round(k * bb / t / bench.GIB, 1) for t in ts],
                             "median_gib_s": round(k * bb / float(np.median(ts)) / bench.GIB, 1)}
        out["parity"] = "ok"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
