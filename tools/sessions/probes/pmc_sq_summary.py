#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc counter CSV (run on the box, so
only this small summary comes back): python tools/pmc_sq_summary.py <csv>"""
import csv
import json
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"]
        for key in ("frame_kernel", "csum_kernel", "csum_span_kernel", "stream_slots_kernel",
                    "fill_splitmix"):
            if key in name:
                name = name[:120]
                break
        else:
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in acc.items():
    out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    out[k]["dispatches"] = max(len(v) for v in cs.values())
    w = out[k].get("SQ_WAVES")
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
            if c in out[k]:
                out[k][c + "_per_wave"] = out[k][c] / w
    wc = out[k].get("SQ_WAVE_CYCLES")
    if wc:
        # shares of the waves' lifetime (disjoint: waiting on a counter or
        # barrier, stalled at issue, issuing)
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in out[k]:
                out[k][c + "_share"] = out[k][c] / wc
        if "SQ_BUSY_CYCLES" in out[k]:
            out[k]["resident_waves_avg"] = wc / out[k]["SQ_BUSY_CYCLES"]
print(json.dumps(out, indent=1))
