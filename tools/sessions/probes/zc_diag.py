"""Diagnose a zero-copy validation mismatch: the test's burst sequence on the
frames fixture, and on the first mismatch the frame's details and three
repeats of the same call."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from oracle import Oracle  # noqa: E402
from test_frames import frames_fixture, mutate  # noqa: E402
from tulips_amd import csum  # noqa: E402

oracle = Oracle()
fx = frames_fixture()
rng = np.random.default_rng(77)
buf = torch.empty(len(fx["arena"]), dtype=torch.uint8).pin_memory()
arena = buf.numpy()
n = len(fx["offsets"])
bad = 0
with csum.HostContext(0, chunk_bytes=1 << 17) as ctx:
    for rnd in range(3):
        arena[:] = mutate(fx, rng, 1500)
        exp = oracle.validate_frames(arena, fx["offsets"], fx["lengths"])
        i = 0
        for b in (1, 1, 7, 64, 200, 1024, 1, 1025, 3, 62, 63, 64, 65):
            if i + b > n:
                i = 0
            o, ln = fx["offsets"][i:i + b], fx["lengths"][i:i + b]
            got = ctx.validate_frames(arena, o, ln, low_latency=True)
            w = np.nonzero(got != exp[i:i + b])[0]
            if len(w):
                bad += 1
                k = int(w[0])
                print(f"round {rnd} burst {b} at {i}: {len(w)} wrong, first k={k} frame "
                      f"{i + k} off {int(o[k])} len {int(ln[k])} got {got[k]} exp "
                      f"{exp[i + k]}; wrong ks {w[:8].tolist()}", flush=True)
                for r in range(3):
                    g2 = ctx.validate_frames(arena, o, ln, low_latency=True)
                    print(f"   repeat {r}: wrong {np.nonzero(g2 != exp[i:i + b])[0][:8].tolist()}")
                g3 = ctx.validate_frames(arena, o, ln)
                print(f"   staged path: wrong {np.nonzero(g3 != exp[i:i + b])[0][:8].tolist()}")
            i += b
print("mismatching calls:", bad)
