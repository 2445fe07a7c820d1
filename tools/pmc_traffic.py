#!/usr/bin/env python3
"""Summarise rocprofv3 output into profiles/ (run here, after a GPU session).

  python tools/pmc_traffic.py gpurun_out/prof_<tag> profiles <tag>
(after TAG=<tag> tools/gpu_check.sh on the GPU box)

Reads <prof>/stats/run_kernel_stats.csv, <prof>/bursts_all.jsonl
(tools/trace_bursts.py --all over the same run's kernel trace) and the
separate --pmc passes (<prof>/pmc_fetch, pmc_write, pmc_rdreq), and writes
  profiles/rocprof_<tag>_kernel_stats.csv   (the rocprofv3 --stats summary)
  profiles/rocprof_<tag>_bursts.jsonl       (per-burst means, every workload)
  profiles/pmc_traffic.json                 (HBM bytes per launch, per workload)

HBM accounting per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KB;
on gfx950 FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced
streaming read (16 B/lane global_load), so read bytes = 2 * FETCH_SIZE * 1024.
WRITE_SIZE is exact for 16-B/lane stores and uncalibrated for our 2-byte
result stores (reported as-is, it is <0.2 % of the traffic).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

# (kernel name fragment, grid size or None, workload label): bench.py's
# default geometries. The ZIPF kernels are also what the host path launches
# per staging chunk, so ZIPF is told apart by its grid: the arena span kernel
# has one 256-thread workgroup per 28 KiB of the 43,772,673-byte arena (1,527
# ranges = 390,912 threads), the any-layout packed kernel 8 segments per wave
# (8,192 waves = 524,288 threads).
WORKLOADS = [
    ("csum_kernel<32, 3, true, tulips_amd::(anonymous namespace)::FixedSegs>", None, "F1500"),
    ("csum_kernel<32, 4, true, tulips_amd::(anonymous namespace)::FixedSegs>", None, "F1500"),
    ("csum_kernel<64, 12, true, tulips_amd::(anonymous namespace)::FixedSegs>", None, "F9000"),
    ("csum_span_kernel<7,", 390912, "ZIPF"),
    ("csum_packed_kernel<8, 4, true>", 524288, "ZIPF_any_layout"),
    # 65,536 frames, 16 per 256-thread block (the host path's small bursts
    # launch the same kernels with smaller grids); frame_kernel<OP, ...>:
    # 0 validate, 1 generate in place, 2 compact fields
    # (round 4: a fifth template argument, frames per subgroup, 1 by default)
    ("frame_kernel<0, 16, 6, true, 1>", 1048576, "frames_validate_F1514"),
    ("frame_kernel<1, 16, 6, true, 1>", 1048576, "frames_generate_F1514"),
    ("frame_kernel<2, 16, 6, true, 1>", 1048576, "frames_generate_fields_F1514"),
    ("frame_kernel<0, 16, 6, true>", 1048576, "frames_validate_F1514"),
    ("frame_kernel<1, 16, 6, true>", 1048576, "frames_generate_F1514"),
    ("frame_kernel<2, 16, 6, true>", 1048576, "frames_generate_fields_F1514"),
    # configs[3] as written: one 64-lane wave per segment
    ("csum_kernel<64, 4, true, tulips_amd::(anonymous namespace)::VarSegs>", None,
     "ZIPF_one_wave_per_segment"),
    ("segment_planned_kernel<16, 6>", None, "segment_TSO_64K_mss1460"),
    ("segment_kernel<16, 6>", None, "segment_TSO_64K_mss1460_device_counted"),
    ("seg_prologue_small_kernel", None, "segment_TSO_64K_mss1460_prologue"),
    ("copy_slots_kernel<16, 6>", None, "segment_TSO_64K_mss1460_copy_same_bytes"),
    ("rss_kernel", None, "rss_toeplitz_16M"),
    ("stream_tiles_kernel", None, "F9000_read_same_bytes"),
]
# algorithmic bytes per launch (bench.py): segment bytes; frame bytes; bytes
# read + written by segmentation (super-frames in, segments out); RSS 12 B in
# + 4 B out per tuple
ALGO_BYTES = {"F1500": 65536 * 1500, "F9000": 65536 * 9000, "ZIPF": 43772673,
              "ZIPF_any_layout": 43772673, "ZIPF_one_wave_per_segment": 43772673,
              "frames_validate_F1514": 65536 * 1514, "frames_generate_F1514": 65536 * 1514,
              "frames_generate_fields_F1514": 65536 * 1514 + 65536 * 4,
              "F9000_read_same_bytes": 65536 * 9000,
              "segment_TSO_64K_mss1460": 1024 * 64294 + 45056 * 1514,
              "segment_TSO_64K_mss1460_device_counted": 1024 * 64294 + 45056 * 1514,
              "segment_TSO_64K_mss1460_copy_same_bytes": 1024 * 64294 + 45056 * 1514,
              "rss_toeplitz_16M": (1 << 24) * 16}


def label(name, grid):
    for frag, g, wl in WORKLOADS:
        if frag in name and (g is None or int(grid) == g):
            return wl
    return None


def counters(path):
    per = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return per
    with open(path) as f:
        for r in csv.DictReader(f):
            wl = label(r["Kernel_Name"], r.get("Grid_Size", 0))
            if wl:
                per[wl][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    prof, outdir, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    os.makedirs(outdir, exist_ok=True)
    stats = os.path.join(prof, "stats", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(outdir, f"rocprof_{tag}_kernel_stats.csv"))
    # per-burst serial / overlapped means of every workload (trace_bursts.py --all)
    bursts = os.path.join(prof, "bursts_all.jsonl")
    if os.path.exists(bursts):
        shutil.copy(bursts, os.path.join(outdir, f"rocprof_{tag}_bursts.jsonl"))
    res = {}
    merged = defaultdict(dict)
    for sub in ("pmc_fetch", "pmc_write", "pmc_rdreq"):
        for wl, cs in counters(os.path.join(prof, sub, "run_counter_collection.csv")).items():
            for cn, vals in cs.items():
                merged[wl][cn] = sum(vals) / len(vals)
                merged[wl][cn + "_dispatches"] = len(vals)
    for wl, c in merged.items():
        rd = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024.0
        wr = c.get("WRITE_SIZE", 0.0) * 1024.0
        res[wl] = {
            "hbm_bytes_per_launch": round(rd + wr),
            "read_bytes_per_launch": round(rd),
            "write_bytes_per_launch": round(wr),
            "algorithmic_bytes_per_launch": ALGO_BYTES.get(wl),
            "traffic_over_algorithmic": round((rd + wr) / ALGO_BYTES[wl], 4)
            if wl in ALGO_BYTES else None,
            "raw": {k: round(v, 3) for k, v in c.items()},
            "method": "2*FETCH_SIZE*1024 (gfx950 half-count correction) + WRITE_SIZE*1024; "
                      "separate rocprofv3 --pmc passes, mean over dispatches",
            "source": f"{prof} ({tag})",
        }
    # bench.py reads pmc_traffic.json for every workload's `traffic`: a run
    # that covered fewer workloads than the committed file (e.g. a trace that
    # missed the extras child) goes beside it instead of replacing it
    dst = os.path.join(outdir, "pmc_traffic.json")
    try:
        with open(dst) as f:
            have = set(json.load(f))
    except (OSError, ValueError):
        have = set()
    if not have <= set(res):
        dst = os.path.join(outdir, f"pmc_traffic_{tag}_partial.json")
        print(f"pmc_traffic: {sorted(have - set(res))} missing from this run; wrote {dst}",
              file=sys.stderr)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
