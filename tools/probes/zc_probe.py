"""Probe of the low-latency validation path: one context, bursts of 1 and
64 frames from pinned (or, with argv[1] == 'pageable', pageable) memory,
timing and status of each call. Exits hard after the first failure (a
server that never answered cannot be stopped)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402
from tulips_amd import csum  # noqa: E402

nf, slot, seg = 256, 2048, 1500
t = torch.zeros(nf * slot, dtype=torch.uint8)
pageable = len(sys.argv) > 1 and sys.argv[1] == "pageable"
ar = t.numpy() if pageable else t.pin_memory().numpy()
offs = np.arange(nf, dtype=np.uint64) * np.uint64(slot)
lens = np.full(nf, seg + 14, np.uint16)
ctx = csum.HostContext(0)
res = {}
for b in (1, 1, 64, 1, 64) + (1,) * 200 + (64,) * 200 + (256,) * 50:
    t0 = time.perf_counter()
    try:
        fl = ctx.validate_frames(ar, offs[:b], lens[:b], low_latency=True)
        res.setdefault(b, []).append(1e6 * (time.perf_counter() - t0))
    except Exception as e:  # noqa: BLE001
        print(f"burst {b}: {e!r} after {time.perf_counter() - t0:.2f} s", flush=True)
        os._exit(3)
ctx.close()
mode = os.environ.get("TULIPS_ZC_MODE", "launch")
for b, ts in res.items():
    print(f"{mode} {'pageable' if pageable else 'pinned'} burst {b}: median "
          f"{np.median(ts):.1f} us p99 {np.percentile(ts, 99):.1f} us (n={len(ts)})", flush=True)
