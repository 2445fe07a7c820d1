"""bench.py's multi-rank launch (the driver runs `python bench.py --gpus N`
with no launcher of its own): with WORLD_SIZE unset and --gpus N > 1, the
script starts `torch.distributed.run --nproc-per-node N` itself as a child
process, every rank checks that the process group holds N ranks, and rank 0
prints the one JSON line.

The CPU test drives that launch path with --dry-run (the ranks form the gloo
group and report it, no GPU call); the GPU test runs the whole bench with 4
ranks sharing the one GPU of the test box (--one-device, gloo), every rank's
measured shard checked against the reference's digests.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def _json_lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_self_launch_forms_the_group_without_a_launcher():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--dist-backend", "gloo", "--one-device", "--dry-run"],
                       capture_output=True, text=True, env=_env(), timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 4 and line["dist"]["world_size"] == 4
    assert sorted(line["dist"]["ranks"]) == [0, 1, 2, 3]


def test_single_rank_dry_run_and_world_mismatch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"],
                       capture_output=True, text=True, env=_env(), timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _json_lines(r.stdout)[0]["n_gpus"] == 1
    # a launcher that gives the group a different size than --gpus is refused
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run"], capture_output=True, text=True, env=env, timeout=300,
                       cwd=ROOT)
    assert r.returncode != 0 and "process group has 1 rank" in r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_self_launched_four_ranks_on_one_gpu():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--dist-backend", "gloo", "--one-device", "--steps", "32",
                        "--warmup", "4", "--no-extras"],
                       capture_output=True, text=True, env=_env(), timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout[-2000:]
    line = lines[0]
    assert line["n_gpus"] == 4 and line["dist"]["world_size"] == 4
    assert line["parity"] == "ok", line.get("parity_checked")
    assert line["value"] > 0
    mg = line["multi_gpu"]
    assert mg["library_scatter_from_gpu0"]["parity"] == "ok", mg["library_scatter_from_gpu0"]
    assert mg["library_scatter_from_gpu0"]["kernel_only"]["parity"] == "ok"
    for leg in ("exchange_overlapped", "scatter_from_gpu0", "zipf_byte_balanced"):
        assert mg[leg].get("parity") == "ok", (leg, mg[leg])
    # §8e host-start form: every rank's shard from page-locked host memory
    hs = line["host_start"]
    assert hs["parity"] == "ok", hs
    assert hs["aggregate_GiBps"] > 0 and hs["bytes_per_rank"] == 16 * 65536 * 1500
    # the summary is the line's last key (the driver keeps the output's tail)
    assert list(line)[-1] == "summary"
    assert line["summary"]["host_start_GiBps"] == hs["aggregate_GiBps"]


def test_summary_of_picks_the_judged_figures():
    """bench.summary_of: per config the serial, 4-branch and read-ceiling
    fractions with parity, from the line's roofline and extras."""
    sys.path.insert(0, ROOT)
    import bench
    line = {"value": 6000.0, "parity": "ok", "roofline": {"frac": 0.77},
            "host_start": {"aggregate_GiBps": 380.5},
            "extras": {"F1500": {"frac_of_peak": 0.76, "pipeline": {"frac_of_peak": 0.89},
                                 "read_same_bytes": {"frac_of_peak": 0.79}, "parity": "ok"},
                       "stream_read_F1500_batch": {"frac_of_peak": 0.80},
                       "F9000": {"frac_of_peak": 0.89, "pipeline": {"frac_of_peak": 0.93},
                                 "read_same_bytes": {"frac_of_peak": 0.88}, "parity": "ok"},
                       "ZIPF": {"frac_of_peak": 0.49, "pipeline": {"frac_of_peak": 0.64},
                                "read_same_bytes": {"frac_of_peak": 0.70},
                                "parity": "MISMATCH"},
                       "segment_TSO_64K_mss1460": {"frac_of_peak": 0.69,
                                                   "device_counted": {"frac_of_peak": 0.57},
                                                   "copy_same_bytes": {"frac_of_peak": 0.78}}}}
    s = bench.summary_of(line)
    assert s["F1500"] == {"serial_frac": 0.77, "branches4_frac": 0.89,
                          "read_same_bytes_frac": 0.80, "read_same_pattern_frac": 0.79,
                          "parity": "ok"}
    assert s["F9000"]["serial_frac"] == 0.89 and s["F9000"]["read_same_bytes_frac"] == 0.88
    assert s["ZIPF"]["parity"] == "MISMATCH"
    assert s["segment_serial_frac"] == 0.69 and s["host_start_GiBps"] == 380.5
    assert s["segment_copy_same_bytes_frac"] == 0.78
    assert len(json.dumps(s)) < 900      # fits the driver's stored tail
    # extras missing (N > 1, or the child failed): no crash, configs None
    s = bench.summary_of({"value": 1.0, "parity": "ok", "roofline": {"frac": 0.7},
                          "extras": {"error": "x"}})
    assert s["F9000"] is None and s["F1500"] is None


def test_branch_count_follows_step_count():
    """The timed graph's branches by step count (bench.branches_for): 2 for
    short replays (the driver's 20 steps), 16 for long ones; an explicit
    --streams wins (profiles/probe_graph_k_r04.txt, ab_branches_k_r04.txt)."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.branches_for(20) == 2 and bench.branches_for(127) == 2
    assert bench.branches_for(128) == 16 and bench.branches_for(1024) == 16
    for argv, want in ((["--steps", "20"], 2), (["--steps", "1024"], 16),
                       (["--steps", "20", "--streams", "8"], 8)):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"] + argv,
                           capture_output=True, text=True, env=_env(), timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        assert _json_lines(r.stdout)[0]["config"]["streams"] == want, argv
