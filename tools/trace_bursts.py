#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace into launch bursts and summarise each.

usage: trace_bursts.py <run_kernel_trace.csv> [kernel-substring] [--gap-us G]
       trace_bursts.py <run_kernel_trace.csv> --all [--gap-us G]

A burst is a run of dispatches of the selected kernel with less than G us
(default 50) between one dispatch's end and the next one's start. For each
burst: dispatch count, mean per-dispatch duration (what `--stats` averages),
and the busy span (union of dispatch intervals) per dispatch — the effective
time per launch when a graph overlaps launches on several branches, i.e. the
quantity bench.py's HIP events measure over its timed region.

--all labels every dispatch with its bench.py workload (kernel + grid, the
table in tools/pmc_traffic.py), prints every burst of every workload, and
ends with one summary line per workload:
  serial      the largest burst whose dispatches never overlap (bench.py's
              one-launch-at-a-time chain): mean dispatch duration, and the
              fraction of 8 TB/s its algorithmic bytes per launch give;
  overlapped  the largest burst whose dispatches overlap (the 4-branch
              pipeline): busy span per dispatch and its fraction.
so that every roofline figure bench.py reports can be recomputed from the
committed trace summary (profiles/rocprof_<tag>_bursts.jsonl).
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import ALGO_BYTES, label  # noqa: E402

HBM_PEAK = 8.0e12


def read(path, keep):
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            tag = keep(r)
            if tag:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r["Kernel_Name"], tag))
    rows.sort()
    return rows


def split(rows, gap_ns):
    out, cur, cur_end = [], [], None
    for s, e, name, tag in rows:
        if cur and s - cur_end > gap_ns:
            out.append(cur)
            cur, cur_end = [], None
        cur.append((s, e, name, tag))
        cur_end = e if cur_end is None else max(cur_end, e)
    if cur:
        out.append(cur)
    return out


def summarise(b):
    busy, last = 0, None
    for s, e, _, _ in b:                         # union of sorted intervals
        if last is None or s > last:
            busy += e - s
            last = e
        elif e > last:
            busy += e - last
            last = e
    n = len(b)
    total = sum(e - s for s, e, _, _ in b)
    return {
        "dispatches": n,
        "mean_dispatch_us": round(total / n / 1e3, 3),
        "busy_span_per_dispatch_us": round(busy / n / 1e3, 3),
        "wall_span_per_dispatch_us": round((max(e for _, e, _, _ in b) - b[0][0]) / n / 1e3, 3),
        "overlap": round(total / busy, 3) if busy else None,
        "kernel": b[0][2].replace("(anonymous namespace)::", "").split("(")[0],
    }


def bursts(path, needle, gap_ns):
    rows = read(path, lambda r: needle if needle in r["Kernel_Name"] else None)
    return [summarise(b) for b in split(rows, gap_ns)]


def all_workloads(path, gap_ns):
    rows = read(path, lambda r: label(r["Kernel_Name"], r.get("Grid_Size_X", 0)))
    by = {}
    for row in rows:
        by.setdefault(row[3], []).append(row)
    lines, summary = [], {}
    for wl, rs in sorted(by.items()):
        bs = [dict(summarise(b), workload=wl) for b in split(rs, gap_ns)]
        lines += bs
        nbytes = ALGO_BYTES.get(wl)
        ser = [b for b in bs if b["overlap"] is not None and b["overlap"] < 1.02 and
               b["dispatches"] >= 8]
        ovl = [b for b in bs if b["overlap"] is not None and b["overlap"] >= 1.02 and
               b["dispatches"] >= 8]
        s = {"workload": wl, "bytes_per_launch": nbytes}
        if ser:
            b = max(ser, key=lambda x: x["dispatches"])
            s["serial"] = {"dispatches": b["dispatches"], "mean_dispatch_us": b["mean_dispatch_us"],
                           "frac": round(nbytes / (b["mean_dispatch_us"] * 1e-6) / HBM_PEAK, 4)
                           if nbytes else None}
        if ovl:
            b = max(ovl, key=lambda x: x["dispatches"])
            s["overlapped"] = {"dispatches": b["dispatches"],
                               "busy_span_per_dispatch_us": b["busy_span_per_dispatch_us"],
                               "overlap": b["overlap"],
                               "frac": round(nbytes / (b["busy_span_per_dispatch_us"] * 1e-6) /
                                             HBM_PEAK, 4) if nbytes else None}
        summary[wl] = s
    return lines, summary


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    gap = 50.0
    if "--gap-us" in sys.argv:
        g = sys.argv[sys.argv.index("--gap-us") + 1]
        gap = float(g)
        args = [a for a in args if a != g]
    if "--all" in sys.argv:
        lines, summary = all_workloads(args[0], gap * 1e3)
        for b in lines:
            print(json.dumps(b))
        for s in summary.values():
            print(json.dumps(dict(s, summary=True)))
        return
    needle = args[1] if len(args) > 1 else "csum_kernel<32, 3, true"
    for b in bursts(args[0], needle, gap * 1e3):
        print(json.dumps(b))


if __name__ == "__main__":
    main()
