"""The hot path on the runtime an integrator gets: tests/native/runtime_check
(a plain C++ process, no torch, the library's NEEDED libamdhip64.so.7
resolved through its RUNPATH to /opt/rocm) drives the C ABI and compares the
SURVEY.md §8c golden digests (tests/golden/digests.json, made by the
reference's own compiled sources) bit-exactly, checks the §8f kernels
(frames, generation, RSS, segmentation) against the golden fixtures and the
oracle, checks the HIP user-object
contract the graph ownership relies on, and runs 500 capture/replay/destroy
cycles with device memory flat. Every pytest GPU run otherwise uses the HIP
runtime torch bundles (tests/test_graph_lifetime.py covers that one).
Semantics: /root/reference/src/stack/Utils.cpp:14-42,
src/stack/tcpv4/Processor.cpp:337-357."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "_build", "runtime_check")
BATCHES = ("F1500", "F1500-tcp", "F9000", "F9000-tcp", "ZIPF", "ZIPF-tcp")


def _threads(pid):
    """Each thread's state and kernel wait channel (/proc), taken from a
    stalled checker before it is killed: a thread parked in the amdgpu
    driver names a GPU wait, one in a futex a host-side lock."""
    out = []
    try:
        for tid in sorted(os.listdir(f"/proc/{pid}/task"), key=int):
            base = f"/proc/{pid}/task/{tid}"
            try:
                with open(f"{base}/comm") as f:
                    comm = f.read().strip()
                with open(f"{base}/stat") as f:
                    state = f.read().rsplit(")", 1)[1].split()[0]
                with open(f"{base}/wchan") as f:
                    wchan = f.read().strip() or "-"
            except OSError:
                continue
            out.append(f"{tid} {comm} {state} {wchan}")
    except OSError as e:
        out.append(f"/proc/{pid}: {e}")
    return "\n".join(out)


def _run(*args, timeout=300):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} is missing: `make native` (or __graft_entry__.build())")
    p = subprocess.Popen([EXE, *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:           # the stall's stderr names its phase
        threads = _threads(p.pid)
        p.kill()
        out, err = p.communicate()
        return -9, None, (f"runtime_check {' '.join(args)}: no exit in {timeout} s\n"
                          f"threads (tid comm state wchan):\n{threads}\n{err}")
    lines = [x for x in out.splitlines() if x.startswith("{")]
    res = json.loads(lines[-1]) if lines else None
    return p.returncode, res, err


def test_zipf_lengths_match_the_spec(golden):
    """CPU: the checker's own §8c Zipf generator reproduces the golden lengths."""
    rc, res, err = _run("zipf-lengths")
    assert rc == 0, err
    z = golden.digests()["zipf_lengths"]
    assert res["total"] == z["total"]
    assert res["fnv1a64"] == z["fnv1a64"]


@pytest.mark.gpu
def test_native_parity_on_integrator_runtime(golden):
    b = golden.digests()["batches"]
    z = golden.digests()["zipf_lengths"]["fnv1a64"]
    want = [f"{k}={b[k]['fnv1a64']}" for k in BATCHES] + [f"ZIPF_LENGTHS={z}"]
    rc, res, err = _run("parity", *want)
    print(json.dumps(res, indent=1))
    assert res is not None, err
    libs = res["runtime"]["hip_runtime_libs"]
    assert libs and all("torch" not in p for p in libs), libs
    bad = {k: v for k, v in res["parity"].items() if not v["ok"]}
    assert rc == 0 and not bad, (bad, err)


@pytest.mark.gpu
def test_native_user_object_contract():
    rc, res, err = _run("user-object")
    print(json.dumps(res, indent=1))
    assert rc == 0, (res, err)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_native_500_graph_cycles():
    rc, res, err = _run("graph-cycles", "500", timeout=540)
    print(json.dumps(res, indent=1))
    assert rc == 0, (res, err)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_native_serial_rate_on_integrator_runtime(golden):
    """The headline kernel through the C ABI on /opt/rocm's runtime, one launch
    at a time over 16 rotated F1500 batches: batch 0 equals the reference
    digest, and the rate is of the order bench.py measures on torch's runtime
    (a loose floor: the figure itself is reported, not asserted)."""
    b = golden.digests()["batches"]["F1500"]
    rc, res, err = _run("serial-rate", "1500", "16", b["fnv1a64"], timeout=240)
    print(json.dumps(res, indent=1))
    assert rc == 0 and res["serial_rate"]["parity"] == "ok", (res, err)
    assert res["serial_rate"]["frac_of_8TBps"] > 0.5, res


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_native_graph_ownership_under_multibranch_churn():
    """Graph ownership (stream_state.h) under churn on /opt/rocm's runtime:
    multi-branch graphs of counting, arena, segmentation and fixed calls
    (each side stream's state attaching its own user object to the graph)
    captured, replayed on other streams (every output checked against the
    direct calls') and destroyed, over 20 s; the second half's graphs leave
    device memory within 4 MiB of where the first half's left it."""
    rc, res, err = _run("graph-churn-stateful", "20", "6", timeout=240)
    print(json.dumps(res, indent=1))
    assert res is not None, err
    assert rc == 0 and res["mismatches"] == 0 and res["destroyed"] > 100, (res, err)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_native_calls_beside_a_global_mode_capture(golden):
    """include/tulips_csum.h, per-stream state, on /opt/rocm's runtime: first
    calls on a fresh stream (verify_arena, batch_arena) and a host and a
    multi-device context made, used and destroyed by one thread while another
    holds a global-mode capture open; the capture survives and replays to
    F1500's digest, and every result equals the reference digests."""
    b = golden.digests()["batches"]
    want = [f"{k}={b[k]['fnv1a64']}" for k in ("F1500", "ZIPF", "ZIPF-tcp")]
    rc, res, err = _run("capture-neutral", *want, timeout=240)
    print(json.dumps(res, indent=1))
    assert res is not None, err
    assert rc == 0 and res["capture_neutral"]["ok"], (res, err)


def write_fixtures(d, oracle):
    """The raw little-endian arrays `runtime_check fixtures` reads from d:
    tests/golden/frames.npz and rss.npz as they are, and super-frames with
    the oracle's segmentation of them."""
    import numpy as np
    from test_segment import pack as seg_pack, super_frame
    d = str(d)
    gdir = os.path.join(ROOT, "tests", "golden")
    fr = np.load(os.path.join(gdir, "frames.npz"))
    for k in ("arena", "offsets", "lengths", "expect"):
        fr[k].tofile(os.path.join(d, f"frames.{k}.bin"))
    rs = np.load(os.path.join(gdir, "rss.npz"))
    for k in ("saddr", "daddr", "sport", "dport"):
        rs[k].tofile(os.path.join(d, f"rss.{k}.bin"))
    for i in range(len(rs["key_names"])):
        rs[f"key_{i}"].tofile(os.path.join(d, f"rss.key_{i}.bin"))
        for tag in ("init0", "initff"):
            rs[f"expect_{i}_{tag}"].tofile(os.path.join(d, f"rss.expect_{i}_{tag}.bin"))
    rng = np.random.default_rng(8)
    payloads = [int(p) for p in rng.integers(1, 64000, 40)] + [1460, 1461, 2920, 0]
    frames = [super_frame(oracle, rng, p) for p in payloads]
    arena, offs, lens = seg_pack(frames, rng)
    mss, stride = 1460, 2048
    first, out, olens = oracle.segment_frames(arena, offs, lens, mss, stride)
    arena.tofile(os.path.join(d, "seg.arena.bin"))
    offs.tofile(os.path.join(d, "seg.offsets.bin"))
    lens.tofile(os.path.join(d, "seg.lengths.bin"))
    np.array([mss, stride], np.uint32).tofile(os.path.join(d, "seg.params.bin"))
    first.tofile(os.path.join(d, "seg.first.bin"))
    out.tofile(os.path.join(d, "seg.out.bin"))
    olens.tofile(os.path.join(d, "seg.out_lengths.bin"))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_native_section8f_kernels_against_fixtures(tmp_path, oracle):
    """The §8f kernels through the C ABI on /opt/rocm's runtime: frame
    validation flags and counters against tests/golden/frames.npz (flags the
    reference's own stack computed), in-place generation restoring the zeroed
    checksum fields of the frames the reference found valid (no other byte
    touched), compact fields equal to those frames' stored fields, Toeplitz RSS
    against tests/golden/rss.npz (the reference's utils::toeplitz, 10 keys x 2
    inits), and segmentation against the oracle (orc_segment_frames; the LSO
    fix-ups are parity-unpinned)."""
    write_fixtures(tmp_path, oracle)
    rc, res, err = _run("fixtures", str(tmp_path), timeout=90)
    print(json.dumps(res, indent=1))
    assert res is not None, err
    bad = {k: v for k, v in res["fixtures"].items() if not v["ok"]}
    assert rc == 0 and not bad and len(res["fixtures"]) == 8, (bad, err)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_native_graph_ownership_across_threads():
    """Graph ownership (stream_state.h) with six host threads on /opt/rocm's
    runtime: each captures (thread-local mode), replays and destroys graphs of
    counting, arena and segmentation calls on its own stream for 15 s, direct
    calls between, so user-object destructors fire and reclaims run on every
    thread at once; every replay exact, device memory back within 32 MiB (a
    leak of the graphs' arrays would be hundreds of MiB)."""
    rc, res, err = _run("thread-churn", "15", "6", timeout=240)
    print(json.dumps(res, indent=1))
    assert res is not None, err
    r = res["thread_churn"]
    assert rc == 0 and r["ok"] and r["mismatches"] == 0 and r["graphs"] > 100, (res, err)
