"""Graph-captured calls: the library's arrays live exactly as long as the graph
(tulips_amd/csrc/stream_state.h, include/tulips_csum.h "per-stream state").

The reference's callers own their buffers for the call only
(/root/reference/src/transport/list/Device.cpp:60-62). A captured call needs
arrays that outlive the call (counter shards, the arena calls' span words,
the segmentation workspace), so the library attaches them to the capture's
graph as a HIP user object: destroying the graph and its executables frees
them (at the library's next uncaptured call). Here, on the runtime torch
bundles:

* the runtime honours that contract: a user object moved to a capture's graph
  survives torch's CUDAGraph capture_end (which destroys the template after
  instantiating it) and every replay, and is destroyed with the executable;
* 500 single-stream graphs of counting, arena and segmentation calls are
  captured, replayed (checked against the oracle every time) and destroyed,
  and device memory returns to within 1 MiB of where it started.

tests/test_native_runtime.py runs the same two checks from a plain C++
process on the ROCm runtime an integrator links.
"""
import ctypes as C
import gc
import threading
import time

import numpy as np
import pytest

from test_frames import _dev
from test_segment import pack as seg_pack, super_frame
from test_stream_state import _hip

MODE_INET, MODE_TCP = 1, 2


@pytest.mark.gpu
def test_user_object_lives_with_the_executable():
    import torch
    hip = _hip()
    destroy_fn = C.CFUNCTYPE(None, C.c_void_p)
    fired = []
    cb = destroy_fn(lambda p: fired.append(threading.get_ident()))
    hip.hipStreamGetCaptureInfo_v2.argtypes = [C.c_void_p, C.POINTER(C.c_int),
                                               C.POINTER(C.c_ulonglong), C.POINTER(C.c_void_p),
                                               C.c_void_p, C.c_void_p]
    hip.hipUserObjectCreate.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, destroy_fn,
                                        C.c_uint, C.c_uint]
    hip.hipGraphRetainUserObject.argtypes = [C.c_void_p, C.c_void_p, C.c_uint, C.c_uint]
    x = torch.zeros(1024, device="cuda:0")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        x.add_(1)
        status, cid, graph = C.c_int(), C.c_ulonglong(), C.c_void_p()
        assert hip.hipStreamGetCaptureInfo_v2(s.cuda_stream, C.byref(status), C.byref(cid),
                                              C.byref(graph), None, None) == 0
        assert status.value == 1 and graph.value          # hipStreamCaptureStatusActive
        obj = C.c_void_p()
        assert hip.hipUserObjectCreate(C.byref(obj), None, cb, 1, 1) == 0  # NoDestructorSync
        assert hip.hipGraphRetainUserObject(graph, obj, 1, 1) == 0         # moved to the graph
        x.add_(1)
    time.sleep(0.05)
    assert fired == [], "destroyed with the template: executables do not hold user objects"
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    time.sleep(0.05)
    assert fired == []
    assert float(x[0]) == 6.0                              # 3 replays of 2 adds
    del g
    gc.collect()
    time.sleep(0.05)
    assert len(fired) == 1


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_500_captured_graphs_leave_memory_flat(oracle):
    """500 capture/replay/destroy cycles on one stream, every replay checked
    against the oracle (verify count and results, arena batch, segmentation),
    then one direct call; hipMemGetInfo ends within 1 MiB of its start."""
    import torch
    from tulips_amd import csum
    rng = np.random.default_rng(500)
    n = 4096
    lens = rng.integers(40, 9000, n).astype(np.uint16)
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    total = int(lens.astype(np.int64).sum())
    buf = rng.integers(0, 256, total + 16, dtype=np.uint8)
    src = np.full(n, 0x0100010A, np.uint32)
    dst = np.full(n, 0x0200010A, np.uint32)
    exp_tcp = oracle.batch(buf, offs, lens, src=src, dst=dst, mode=MODE_TCP, nthreads=8)
    exp_inet = oracle.batch(buf, offs, lens, mode=MODE_INET, nthreads=8)
    exp_bad = int(np.count_nonzero(exp_tcp != 0xFFFF))
    a, o, l, ds, dd = _dev(buf, offs.astype(np.int64), lens.view(np.int16), src.view(np.int32),
                           dst.view(np.int32))
    frames = [super_frame(oracle, rng, int(p)) for p in rng.integers(1000, 60000, 24)]
    farena, foffs, flens = seg_pack(frames, rng)
    mss, stride = 1460, 2048
    efirst, eout, elens = oracle.segment_frames(farena, foffs, flens, mss, stride)
    nseg = int(efirst[-1])
    fa, fo, fl = _dev(farena, foffs.astype(np.int64), flens.view(np.int16))
    e_first = torch.from_numpy(efirst.view(np.int32)).to("cuda:0")
    e_out = torch.from_numpy(eout).to("cuda:0")
    e_lens = torch.from_numpy(elens.view(np.int16)).to("cuda:0")
    e_tcp = torch.from_numpy(exp_tcp.view(np.int16)).to("cuda:0")
    e_inet = torch.from_numpy(exp_inet.view(np.int16)).to("cuda:0")
    out_tcp = torch.empty(n, dtype=torch.int16, device="cuda:0")
    bad = torch.empty(1, dtype=torch.int32, device="cuda:0")
    out_inet = torch.empty(n, dtype=torch.int16, device="cuda:0")
    seg_out = torch.empty(nseg * stride, dtype=torch.uint8, device="cuda:0")
    seg_lens = torch.empty(nseg, dtype=torch.int16, device="cuda:0")
    seg_first = torch.empty(len(frames) + 1, dtype=torch.int32, device="cuda:0")
    outs = (out_tcp, bad, out_inet, seg_out, seg_lens, seg_first)
    cap = torch.cuda.Stream()

    def calls(st):
        assert csum.lib.tulips_csum_verify(a.data_ptr(), o.data_ptr(), l.data_ptr(),
                                           ds.data_ptr(), dd.data_ptr(), out_tcp.data_ptr(),
                                           bad.data_ptr(), n, MODE_TCP, st) == 0
        assert csum.lib.tulips_csum_batch_arena(a.data_ptr(), total, o.data_ptr(),
                                                l.data_ptr(), None, None, None,
                                                out_inet.data_ptr(), n, MODE_INET, st) == 0
        assert csum.lib.tulips_csum_segment_frames(fa.data_ptr(), fo.data_ptr(), fl.data_ptr(),
                                                   len(frames), mss, seg_out.data_ptr(), stride,
                                                   nseg, seg_lens.data_ptr(),
                                                   seg_first.data_ptr(), st) == 0

    def poison():
        for t in outs:
            t.fill_(-91)

    def exact():
        # each segment's bytes only (the slot's tail past its length is not written)
        got = seg_out.view(nseg, stride)
        want = e_out.view(nseg, stride)
        keep = (torch.arange(stride, device="cuda:0")[None, :] <
                e_lens.to(torch.int64)[:, None])
        return (torch.equal(out_tcp, e_tcp) and int(bad.item()) == exp_bad and
                torch.equal(out_inet, e_inet) and torch.equal(seg_first, e_first) and
                torch.equal(seg_lens, e_lens) and torch.equal(got[keep], want[keep]))

    calls(cap.cuda_stream)                  # the stream's direct arrays exist before the start
    torch.cuda.synchronize()
    assert exact()
    gc.collect()
    free0, _ = torch.cuda.mem_get_info()
    bad_replays = []
    for cycle in range(500):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            calls(cap.cuda_stream)
        for rep in range(2):
            poison()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            if not exact():
                bad_replays.append((cycle, rep))
        del g
    calls(cap.cuda_stream)                  # reclaims what the destroyed graphs held
    torch.cuda.synchronize()
    gc.collect()
    free1, _ = torch.cuda.mem_get_info()
    assert not bad_replays, bad_replays[:10]
    assert exact()
    # without graph ownership each capture would keep ~1.7 MB (shards, span
    # words, workspace): ~850 MB over 500 graphs
    assert free0 - free1 < (1 << 20), (free0, free1)
    csum.release_stream(cap.cuda_stream)


@pytest.mark.gpu
def test_graph_outlives_release_and_destruction_of_its_capture_stream(oracle):
    """include/tulips_csum.h: tulips_csum_release_stream frees a stream's
    direct arrays; graphs captured on it keep theirs. A counting call and an
    arena call captured on a raw HIP stream, the stream released and
    destroyed, then the graph replayed on other streams: exact every time;
    destroying the graph afterwards returns its arrays."""
    import torch
    from tulips_amd import csum
    hip = _hip()
    rng = np.random.default_rng(77)
    n = 6000
    lens = rng.integers(40, 9000, n).astype(np.uint16)
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    total = int(lens.astype(np.int64).sum())
    buf = rng.integers(0, 256, total + 16, dtype=np.uint8)
    src = np.full(n, 0x0100010A, np.uint32)
    dst = np.full(n, 0x0200010A, np.uint32)
    exp_tcp = oracle.batch(buf, offs, lens, src=src, dst=dst, mode=MODE_TCP, nthreads=8)
    exp_inet = oracle.batch(buf, offs, lens, mode=MODE_INET, nthreads=8)
    a, o, l, ds, dd = _dev(buf, offs.astype(np.int64), lens.view(np.int16), src.view(np.int32),
                           dst.view(np.int32))
    out_tcp = torch.empty(n, dtype=torch.int16, device="cuda:0")
    bad = torch.empty(1, dtype=torch.int32, device="cuda:0")
    out_inet = torch.empty(n, dtype=torch.int16, device="cuda:0")
    s = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0     # hipStreamNonBlocking
    st = s.value
    # the stream's own (direct) arrays exist before the capture
    assert csum.lib.tulips_csum_verify(a.data_ptr(), o.data_ptr(), l.data_ptr(), ds.data_ptr(),
                                       dd.data_ptr(), out_tcp.data_ptr(), bad.data_ptr(), n,
                                       MODE_TCP, st) == 0
    torch.cuda.synchronize()
    ext = torch.cuda.ExternalStream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=ext):
        assert csum.lib.tulips_csum_verify(a.data_ptr(), o.data_ptr(), l.data_ptr(),
                                           ds.data_ptr(), dd.data_ptr(), out_tcp.data_ptr(),
                                           bad.data_ptr(), n, MODE_TCP, st) == 0
        assert csum.lib.tulips_csum_batch_arena(a.data_ptr(), total, o.data_ptr(),
                                                l.data_ptr(), None, None, None,
                                                out_inet.data_ptr(), n, MODE_INET, st) == 0
    torch.cuda.synchronize()
    assert csum.lib.tulips_csum_release_stream(st) == 0
    del ext
    assert hip.hipStreamDestroy(s) == 0
    others = [torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(6):
        for t in (out_tcp, bad, out_inet):
            t.fill_(-91)
        torch.cuda.synchronize()
        with torch.cuda.stream(others[rep % 2]):
            g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out_tcp.cpu().numpy().view(np.uint16), exp_tcp)
        assert int(bad.item()) == int(np.count_nonzero(exp_tcp != 0xFFFF))
        np.testing.assert_array_equal(out_inet.cpu().numpy().view(np.uint16), exp_inet)
    del g
    gc.collect()
    # the next uncaptured call reclaims what the graph held
    assert csum.lib.tulips_csum_batch_arena(a.data_ptr(), total, o.data_ptr(), l.data_ptr(),
                                            None, None, None, out_inet.data_ptr(), n, MODE_INET,
                                            others[0].cuda_stream) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out_inet.cpu().numpy().view(np.uint16), exp_inet)
    for x in others:
        csum.release_stream(x)


@pytest.mark.gpu
def test_first_calls_beside_a_global_mode_capture_in_another_thread(oracle):
    """include/tulips_csum.h, per-stream state: a thread's FIRST calls on a
    fresh stream allocate that stream's arrays (counter shards, span words,
    segmentation workspace), and a pending reclaim frees a destroyed graph's.
    Another thread capturing in torch's default global mode must neither
    refuse those allocations and frees nor be broken by them (they are made
    in relaxed capture mode), and neither may the host-buffer contexts'
    staging, streams and waits. Thread A captures verify + arena + segment on
    its stream; while the capture is open, thread B makes the same calls on a
    new raw stream, with a destroyed graph's arrays pending, then creates,
    uses and destroys a host context and a two-entry multi-device context;
    every result is exact and A's graph replays exactly."""
    import torch
    from tulips_amd import csum
    hip = _hip()
    rng = np.random.default_rng(4242)
    n = 5000
    lens = rng.integers(40, 9000, n).astype(np.uint16)
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    total = int(lens.astype(np.int64).sum())
    buf = rng.integers(0, 256, total + 16, dtype=np.uint8)
    src = np.full(n, 0x0300010A, np.uint32)
    dst = np.full(n, 0x0400010A, np.uint32)
    exp_tcp = oracle.batch(buf, offs, lens, src=src, dst=dst, mode=MODE_TCP, nthreads=8)
    exp_inet = oracle.batch(buf, offs, lens, mode=MODE_INET, nthreads=8)
    exp_bad = int(np.count_nonzero(exp_tcp != 0xFFFF))
    a, o, l, ds, dd = _dev(buf, offs.astype(np.int64), lens.view(np.int16), src.view(np.int32),
                           dst.view(np.int32))
    frames = [super_frame(oracle, rng, int(p)) for p in rng.integers(1000, 60000, 16)]
    farena, foffs, flens = seg_pack(frames, rng)
    mss, stride = 1460, 2048
    efirst, eout, elens = oracle.segment_frames(farena, foffs, flens, mss, stride)
    nseg = int(efirst[-1])
    fa, fo, fl = _dev(farena, foffs.astype(np.int64), flens.view(np.int16))

    def outputs():
        return dict(tcp=torch.full((n,), -91, dtype=torch.int16, device="cuda:0"),
                    bad=torch.full((1,), -91, dtype=torch.int32, device="cuda:0"),
                    inet=torch.full((n,), -91, dtype=torch.int16, device="cuda:0"),
                    seg=torch.full((nseg * stride,), 0x5B, dtype=torch.uint8, device="cuda:0"),
                    seg_lens=torch.full((nseg,), -91, dtype=torch.int16, device="cuda:0"),
                    seg_first=torch.full((len(frames) + 1,), -91, dtype=torch.int32,
                                         device="cuda:0"))

    def calls(st, x):
        return (csum.lib.tulips_csum_verify(a.data_ptr(), o.data_ptr(), l.data_ptr(),
                                            ds.data_ptr(), dd.data_ptr(), x["tcp"].data_ptr(),
                                            x["bad"].data_ptr(), n, MODE_TCP, st),
                csum.lib.tulips_csum_batch_arena(a.data_ptr(), total, o.data_ptr(), l.data_ptr(),
                                                 None, None, None, x["inet"].data_ptr(), n,
                                                 MODE_INET, st),
                csum.lib.tulips_csum_segment_frames(fa.data_ptr(), fo.data_ptr(), fl.data_ptr(),
                                                    len(frames), mss, x["seg"].data_ptr(), stride,
                                                    nseg, x["seg_lens"].data_ptr(),
                                                    x["seg_first"].data_ptr(), st))

    def check(x, who):
        np.testing.assert_array_equal(x["tcp"].cpu().numpy().view(np.uint16), exp_tcp, who)
        assert int(x["bad"].item()) == exp_bad, who
        np.testing.assert_array_equal(x["inet"].cpu().numpy().view(np.uint16), exp_inet, who)
        np.testing.assert_array_equal(x["seg_first"].cpu().numpy().view(np.uint32), efirst, who)
        got_lens = x["seg_lens"].cpu().numpy().view(np.uint16)
        np.testing.assert_array_equal(got_lens, elens, who)
        got = x["seg"].cpu().numpy().reshape(nseg, stride)
        want = eout.reshape(nseg, stride)
        for k in range(nseg):
            assert np.array_equal(got[k, :elens[k]], want[k, :elens[k]]), (who, k)

    # a destroyed graph's arrays pending reclaim when thread B makes its calls
    pend = torch.cuda.Stream()
    x_pend = outputs()
    g0 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g0, stream=pend):
        assert calls(pend.cuda_stream, x_pend) == (0, 0, 0)
    g0.replay()
    torch.cuda.synchronize()
    check(x_pend, "pending graph")
    del g0
    gc.collect()

    cap = torch.cuda.Stream()
    sb = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(sb), 1) == 0       # hipStreamNonBlocking
    x_a, x_b = outputs(), outputs()
    torch.cuda.synchronize()
    go, done = threading.Event(), threading.Event()
    rc_b = []

    host_b = {}

    def thread_b():
        go.wait(60)
        try:
            rc_b.append(calls(sb.value, x_b))
            # the host-buffer contexts (pinned staging, their own streams and,
            # for the multi-device one, worker threads) made, used and freed
            with csum.HostContext(0) as hc:
                host_b["ctx"] = hc.batch(buf, offs, lens, src=src, dst=dst, mode=MODE_TCP)
            with csum.MultiContext([0, 0]) as m:
                host_b["mctx"] = m.batch(buf, offs, lens, src=src, dst=dst, mode=MODE_TCP)
        except Exception as e:                                   # reported below
            host_b["error"] = repr(e)
        finally:
            done.set()

    tb = threading.Thread(target=thread_b)
    tb.start()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=cap):                     # global capture mode
            rc_a = calls(cap.cuda_stream, x_a)
            go.set()
            assert done.wait(60), "thread B did not finish"
    finally:
        go.set()
        tb.join(60)
    assert rc_a == (0, 0, 0)
    assert rc_b == [(0, 0, 0)], f"B's calls beside the capture returned {rc_b}"
    assert "error" not in host_b, host_b.get("error")
    np.testing.assert_array_equal(host_b["ctx"], exp_tcp)
    np.testing.assert_array_equal(host_b["mctx"], exp_tcp)
    torch.cuda.synchronize()
    assert hip.hipStreamSynchronize(sb) == 0
    check(x_b, "thread B (direct, beside the capture)")
    for rep in range(3):
        for t in x_a.values():
            t.fill_(-91 if t.dtype != torch.uint8 else 0x5B)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        check(x_a, f"thread A's graph, replay {rep}")
    del g
    gc.collect()
    assert csum.lib.tulips_csum_release_stream(sb.value) == 0
    assert hip.hipStreamDestroy(sb) == 0
    csum.release_stream(cap.cuda_stream)
    csum.release_stream(pend.cuda_stream)
