#!/usr/bin/env python3
"""Does a captured graph with an EMPTY forked branch (a side stream forked
from the capture stream and joined back with no work on it) crash
hipGraphLaunch? Torch-only work (no library call): MODE=empty captures
graphs whose work lands on side stream 0 of 4 (branches 1-3 empty), MODE=full
puts work on every branch. Each graph is replayed on a fresh pool stream a
few times. Prints one line per 50 graphs; a crash ends the process (exit
139)."""
import os
import sys

import torch

mode = os.environ.get("MODE", "empty")
n_graphs = int(os.environ.get("GRAPHS", "400"))
x = torch.zeros(1 << 20, device="cuda:0")
keep = []
for it in range(n_graphs):
    cap = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(4)]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        main = torch.cuda.current_stream()
        for sd in side:
            sd.wait_stream(main)
        for k, sd in enumerate(side):
            if mode == "full" or k == 0:
                with torch.cuda.stream(sd):
                    x.add_(1.0)
        for sd in side:
            main.wait_stream(sd)
    keep.append(g)
    if len(keep) > 8:
        keep.pop(0)
    for r in range(3):
        with torch.cuda.stream(torch.cuda.Stream()):
            keep[(it * 7 + r) % len(keep)].replay()
        torch.cuda.synchronize()
    if it % 50 == 0:
        print(f"{mode}: {it} graphs ok", flush=True)
print(f"{mode}: all {n_graphs} graphs replayed", flush=True)
