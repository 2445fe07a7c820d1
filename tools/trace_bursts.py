#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace into launch bursts and summarise each.

usage: trace_bursts.py <run_kernel_trace.csv> [kernel-substring] [--gap-us G]

A burst is a run of dispatches of the selected kernel with less than G us
(default 50) between one dispatch's end and the next one's start. For each
burst: dispatch count, mean per-dispatch duration (what `--stats` averages),
and the busy span (union of dispatch intervals) per dispatch — the effective
time per launch when a graph overlaps launches on several branches, i.e. the
quantity bench.py's HIP events measure over its timed region.
"""
import csv
import json
import sys


def bursts(path, needle, gap_ns):
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if needle in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r["Kernel_Name"]))
    rows.sort()
    out, cur, cur_end = [], [], None
    for s, e, name in rows:
        if cur and s - cur_end > gap_ns:
            out.append(cur)
            cur = []
        cur.append((s, e, name))
        cur_end = e if cur_end is None or len(cur) == 1 else max(cur_end, e)
    if cur:
        out.append(cur)
    res = []
    for b in out:
        busy, last = 0, None
        for s, e, _ in b:                       # union of sorted intervals
            if last is None or s > last:
                busy += e - s
                last = e
            elif e > last:
                busy += e - last
                last = e
        n = len(b)
        res.append({
            "dispatches": n,
            "mean_dispatch_us": round(sum(e - s for s, e, _ in b) / n / 1e3, 3),
            "busy_span_per_dispatch_us": round(busy / n / 1e3, 3),
            "wall_span_per_dispatch_us": round((max(e for _, e, _ in b) - b[0][0]) / n / 1e3, 3),
            "kernel": b[0][2].replace("(anonymous namespace)::", "").split("(")[0],
        })
    return res


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    gap = 50.0
    if "--gap-us" in sys.argv:
        gap = float(sys.argv[sys.argv.index("--gap-us") + 1])
        args = [a for a in args if a != str(sys.argv[sys.argv.index("--gap-us") + 1])]
    needle = args[1] if len(args) > 1 else "csum_kernel<32, 4, true"
    for b in bursts(args[0], needle, gap * 1e3):
        print(json.dumps(b))


if __name__ == "__main__":
    main()
