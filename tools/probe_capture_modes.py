#!/usr/bin/env python3
"""Which HIP calls made by one thread break another thread's global-mode
stream capture? Thread A begins a capture (hipStreamCaptureModeGlobal, as
torch.cuda.graph does by default) on its stream and records a memset node;
thread B then makes ONE call on its own, non-capturing stream, in global or
relaxed mode; thread A ends the capture. Prints one JSON line per case: B's
return code and whether A's capture survived. Each case runs in a child
process (a broken capture can leave the runtime's state sticky).

  python tools/probe_capture_modes.py [torch|opt]   # the runtime to load

torch = the libamdhip64 torch bundles (ROCm 7.0: what the pytest suite
binds), opt = /opt/rocm/lib (7.2: what a C++ integrator links)."""
import ctypes as C
import json
import os
import subprocess
import sys
import threading

CASES = ["none", "malloc", "malloc_relaxed", "free", "free_relaxed", "sync", "sync_relaxed",
         "memset_async", "is_capturing", "set_device", "lib_verify", "lib_verify_relaxed"]


def runtime(which):
    if which == "opt":
        return C.CDLL("/opt/rocm/lib/libamdhip64.so")
    import torch
    torch.cuda.init()
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                return C.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not loaded")


def child(which, case):
    hip = runtime(which)
    p = C.c_void_p
    ok = lambda rc, what: (rc == 0) or sys.exit(f"{what}: {rc}")  # noqa: E731
    sa, sb = p(), p()
    ok(hip.hipStreamCreateWithFlags(C.byref(sa), 1), "stream a")
    ok(hip.hipStreamCreateWithFlags(C.byref(sb), 1), "stream b")
    a_buf, b_buf, victim = p(), p(), p()
    for q in (a_buf, b_buf, victim):
        ok(hip.hipMalloc(C.byref(q), C.c_size_t(1 << 20)), "malloc")
    n = 4096
    lib = None
    if case.startswith("lib_"):
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        lib = C.CDLL(os.path.join(root, "tulips_amd", "libtulips_csum.so"))
        lib.tulips_csum_verify.argtypes = [p, p, p, p, p, p, p, C.c_uint32, C.c_int, p]
        offs = (C.c_int64 * n)(*[i * 128 for i in range(n)])
        lens = (C.c_uint16 * n)(*([128] * n))
        d_offs, d_lens = p(), p()
        ok(hip.hipMalloc(C.byref(d_offs), C.c_size_t(8 * n)), "malloc")
        ok(hip.hipMalloc(C.byref(d_lens), C.c_size_t(2 * n)), "malloc")
        ok(hip.hipMemcpy(d_offs, offs, C.c_size_t(8 * n), 1), "h2d")
        ok(hip.hipMemcpy(d_lens, lens, C.c_size_t(2 * n), 1), "h2d")
    ok(hip.hipDeviceSynchronize(), "sync")
    go, done = threading.Event(), threading.Event()
    out = {}

    def relaxed(f):
        mode = C.c_int(2)                                    # hipStreamCaptureModeRelaxed
        hip.hipThreadExchangeStreamCaptureMode(C.byref(mode))
        try:
            return f()
        finally:
            hip.hipThreadExchangeStreamCaptureMode(C.byref(mode))

    def b_call():
        q = p()
        if case == "none":
            return 0
        if case == "malloc":
            return hip.hipMalloc(C.byref(q), C.c_size_t(1 << 20))
        if case == "malloc_relaxed":
            return relaxed(lambda: hip.hipMalloc(C.byref(q), C.c_size_t(1 << 20)))
        if case == "free":
            return hip.hipFree(victim)
        if case == "free_relaxed":
            return relaxed(lambda: hip.hipFree(victim))
        if case == "sync":
            return hip.hipStreamSynchronize(sb)
        if case == "sync_relaxed":
            return relaxed(lambda: hip.hipStreamSynchronize(sb))
        if case == "memset_async":
            return hip.hipMemsetAsync(b_buf, 0, C.c_size_t(4096), sb)
        if case == "is_capturing":
            st = C.c_int()
            return hip.hipStreamIsCapturing(sb, C.byref(st))
        if case == "set_device":
            return hip.hipSetDevice(0)
        if case in ("lib_verify", "lib_verify_relaxed"):
            call = lambda: lib.tulips_csum_verify(b_buf, d_offs, d_lens, None, None,  # noqa: E731
                                                  b_buf.value + (512 << 10), victim, n, 1, sb)
            return call() if case == "lib_verify" else relaxed(call)
        raise SystemExit(f"unknown case {case}")

    def thread_b():
        go.wait(30)
        try:
            out["rc_b"] = b_call()
            out["b_last_error"] = hip.hipGetLastError()
        finally:
            done.set()

    tb = threading.Thread(target=thread_b)
    tb.start()
    out["rc_begin"] = hip.hipStreamBeginCapture(sa, 0)         # hipStreamCaptureModeGlobal
    out["rc_node"] = hip.hipMemsetAsync(a_buf, 0, C.c_size_t(4096), sa)
    go.set()
    done.wait(30)
    st = C.c_int(-1)
    out["rc_status"] = hip.hipStreamIsCapturing(sa, C.byref(st))
    out["status_after_b"] = st.value                         # 1 active, 2 invalidated
    g = p()
    out["rc_end"] = hip.hipStreamEndCapture(sa, C.byref(g))
    tb.join(30)
    hip.hipGetLastError()
    out["rc_b_sync"] = hip.hipStreamSynchronize(sb)
    out["capture_ok"] = out["rc_end"] == 0 and bool(g.value)
    print(json.dumps({"runtime": which, "case": case, **out}), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        return
    which = sys.argv[1] if len(sys.argv) > 1 else "torch"
    for case in CASES:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", which, case],
                           capture_output=True, text=True, timeout=120)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
        if r.returncode != 0 or not line:
            print(json.dumps({"runtime": which, "case": case, "child_rc": r.returncode,
                              "stderr": r.stderr.strip()[-300:]}), flush=True)
        else:
            print(line, flush=True)


if __name__ == "__main__":
    main()
