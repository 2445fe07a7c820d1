#!/usr/bin/env python3
"""Tiny crafted batches through the PACKED kernel vs the restatement (debug)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tulips_amd  # noqa: E402
from tulips_amd import csum  # noqa: E402
from oracle import Oracle, MODE_RAW  # noqa: E402

orc = Oracle()
rng = np.random.default_rng(5)
arena = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
da = torch.from_numpy(arena).cuda()
cases = {
    "1x16": [(0, 16)], "8x16": [(16 * i, 16) for i in range(8)],
    "1x1024": [(0, 1024)], "1x1040": [(0, 1040)], "8x160": [(160 * i, 160) for i in range(8)],
    "1x5@3": [(3, 5)], "2x(5@3,17@40)": [(3, 5), (40, 17)],
    "9x100": [(100 * i, 100) for i in range(9)], "8x2000": [(2000 * i, 2000) for i in range(8)],
}
for geo in ((8, 2), (16, 4), (64, 8)):
    t = csum.Tuning(kind=csum.KIND_PACKED, group=geo[0], unroll=geo[1], nontemporal=1)
    for name, segs in cases.items():
        offs = np.array([o for o, _ in segs], np.uint64)
        lens = np.array([L for _, L in segs], np.uint16)
        exp = orc.batch(arena, offs, lens, mode=MODE_RAW)
        got = tulips_amd.batch(da, torch.from_numpy(offs.view(np.int64)).cuda(),
                               torch.from_numpy(lens).cuda(), tuning=t)
        torch.cuda.synchronize()
        got = got.cpu().numpy().view(np.uint16)
        ok = np.array_equal(got, exp)
        print(geo, name, "ok" if ok else f"BAD got={got.tolist()} exp={exp.tolist()}")

# adversarial fixture: which segments go wrong
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_util as gu  # noqa: E402
adv = gu.adversarial()
ar = torch.from_numpy(adv["arena"]).cuda()
offs, lens = adv["offsets"], adv["lengths"]
exp = orc.batch(adv["arena"], offs, lens, mode=MODE_RAW)
for geo in ((8, 2), (64, 8)):
    t = csum.Tuning(kind=csum.KIND_PACKED, group=geo[0], unroll=geo[1], nontemporal=1)
    got = tulips_amd.batch(ar, torch.from_numpy(offs.view(np.int64)).cuda(),
                           torch.from_numpy(lens).cuda(), tuning=t)
    got = got.cpu().numpy().view(np.uint16)
    bad = np.nonzero(got != exp)[0]
    print(geo, "adversarial bad", len(bad), "of", len(lens))
    for i in bad[:12]:
        w0 = (i // geo[0]) * geo[0]
        print("  seg", i, "lane", i - w0, "off", int(offs[i]), "len", int(lens[i]),
              "wave lens", lens[w0:w0 + geo[0]].tolist(), "got", hex(got[i]), "exp", hex(exp[i]))
    bad_w = sorted(set(int(i) // geo[0] for i in bad))
    good_w = [w for w in range(len(lens) // geo[0]) if w not in set(bad_w)]
    print("  bad waves", len(bad_w), "good waves", len(good_w))
    tw = lambda w: sum(((int(offs[k]) % 16 + int(lens[k]) + 15) // 16) if lens[k] else 0
                       for k in range(w * geo[0], min((w + 1) * geo[0], len(lens))))
    print("  T of bad waves (first 10)", [tw(w) for w in bad_w[:10]])
    print("  T of good waves (first 10)", [tw(w) for w in good_w[:10]])
