#!/usr/bin/env python3
"""r06ag diagnostic: `runtime_check fixtures` (the test that stalled once in
r06ae's whole-suite run) repeated in fresh processes, each under its own
60 s limit; stops at the first failure or stall and prints its stderr, whose
phase markers name where it stood. Test infrastructure."""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle import Oracle  # noqa: E402
from test_native_runtime import EXE, write_fixtures  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 20
with tempfile.TemporaryDirectory() as d:
    write_fixtures(d, Oracle())
    for i in range(runs):
        t0 = time.monotonic()
        try:
            p = subprocess.run([EXE, "fixtures", d], capture_output=True, text=True, timeout=60)
        except subprocess.TimeoutExpired as e:
            err = e.stderr.decode() if isinstance(e.stderr, bytes) else (e.stderr or "")
            print(f"run {i}: STALL (60 s)\n{err}", flush=True)
            sys.exit(2)
        dt = time.monotonic() - t0
        print(f"run {i}: rc {p.returncode} {dt:.2f} s", flush=True)
        if p.returncode != 0:
            print(p.stdout[-2000:], p.stderr[-3000:], flush=True)
            sys.exit(1)
print("all runs ok", flush=True)
