"""Per-(device, stream) library state (tulips_amd/csrc/stream_state.h):

* two host threads issuing counting calls on the SAME stream (the legacy NULL
  stream) each get their own totals — the count kernel and its shard
  finalize are queued as one sequence under the stream's lock;
* two host threads segmenting on the same stream each get their own output
  (the prologue and the segment kernel share the stream's workspace);
* a counting call captured in a HIP graph runs on shards of the graph's
  (stream_state.h; their lifetime: tests/test_graph_lifetime.py), so
  replaying the graph on another stream while direct counting calls run on
  the capture stream keeps both totals right;
* tulips_csum_release_stream frees what a stream holds: 100 streams created,
  used (verify, counted validation, segmentation), released and destroyed
  leave device memory flat;
* n == 0 overwrites the counters with zeros (as tulips_csum_verify does).

Counts are checked against the oracle / the reference-pinned frame fixture.
"""
import ctypes as C
import threading

import numpy as np
import pytest

from test_frames import _dev, counters_of, frames_fixture
from test_segment import pack as seg_pack, super_frame

MODE_INET = 1


def _hip():
    """The HIP runtime this process already loaded (torch's copy)."""
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                return C.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not loaded")


def _all_bad(n, L, seed):
    import torch
    rng = np.random.default_rng(seed)
    arena = torch.from_numpy(rng.integers(0, 256, n * L, dtype=np.uint8)).to("cuda:0")
    offs = torch.from_numpy(np.arange(n, dtype=np.int64) * L).to("cuda:0")
    lens = torch.from_numpy(np.full(n, L, np.int16)).to("cuda:0")
    return arena, offs, lens


@pytest.mark.gpu
def test_two_threads_counting_on_one_stream(oracle):
    import torch
    from tulips_amd import csum
    n, L = 8192, 1500
    arena, offs, lens = _all_bad(n, L, 11)
    exp = oracle.batch(arena.cpu().numpy(), np.arange(n, dtype=np.uint64) * L,
                       np.full(n, L, np.uint16), mode=MODE_INET, nthreads=8)
    fx = frames_fixture()
    fa, fo, fl = _dev(fx["arena"], fx["offsets"].astype(np.int64), fx["lengths"].view(np.int16))
    fexp = counters_of(fx["expect"])
    nf = len(fx["offsets"])
    iters = 200
    sizes = [n // 2 + 17 * k for k in range(iters)]
    want = [int(np.count_nonzero(exp[:s] != 0xFFFF)) for s in sizes]
    vcnt = torch.full((iters,), -1, dtype=torch.int32, device="cuda:0")
    fcnt = torch.full((iters, 4), -1, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    errors = []

    def verifier():
        for k in range(iters):
            rc = csum.lib.tulips_csum_verify(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                             None, None, None, vcnt[k].data_ptr(), sizes[k],
                                             MODE_INET, None)
            if rc:
                errors.append(("verify", k, rc))

    def validator():
        for k in range(iters):
            rc = csum.lib.tulips_csum_validate_frames(fa.data_ptr(), fo.data_ptr(),
                                                      fl.data_ptr(), nf, None,
                                                      fcnt[k].data_ptr(), None)
            if rc:
                errors.append(("frames", k, rc))

    ts = [threading.Thread(target=verifier), threading.Thread(target=validator)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errors
    assert vcnt.cpu().numpy().tolist() == want
    np.testing.assert_array_equal(fcnt.cpu().numpy().view(np.uint32),
                                  np.tile(fexp, (iters, 1)))


@pytest.mark.gpu
def test_two_threads_segmenting_on_one_stream(oracle):
    import torch
    from tulips_amd import csum
    rng = np.random.default_rng(3)
    inputs = []
    for k in range(2):
        frames = [super_frame(oracle, rng, int(p)) for p in rng.integers(1000, 20000, 24 + 8 * k)]
        arena, offs, lens = seg_pack(frames, rng)
        inputs.append(_dev(arena, offs.astype(np.int64), lens.view(np.int16)))
    mss, stride = 1460, 2048
    # serial reference outputs (same library, one call each)
    ref = []
    for a, o, l in inputs:
        out, ol, first = csum.segment_frames(a, o, l, mss, stride=stride, stream=0)
        torch.cuda.synchronize()
        ref.append((out.cpu().numpy(), ol.cpu().numpy(), first.cpu().numpy()))
    iters = 60
    bufs = [[(torch.empty(len(ref[i][0]), dtype=torch.uint8, device="cuda:0"),
              torch.zeros(len(ref[i][1]), dtype=torch.int16, device="cuda:0"),
              torch.empty(len(ref[i][2]), dtype=torch.int32, device="cuda:0"))
             for _ in range(iters)] for i in range(2)]
    errors = []

    def worker(i):
        a, o, l = inputs[i]
        cap = int(ref[i][2][-1])
        for k in range(iters):
            out, ol, first = bufs[i][k]
            rc = csum.lib.tulips_csum_segment_frames(a.data_ptr(), o.data_ptr(), l.data_ptr(),
                                                     int(o.numel()), mss, out.data_ptr(),
                                                     stride, cap, ol.data_ptr(),
                                                     first.data_ptr(), None)
            if rc:
                errors.append((i, k, rc))

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errors
    for i in range(2):
        total = int(ref[i][2][-1])
        for k in range(iters):
            out, ol, first = bufs[i][k]
            np.testing.assert_array_equal(first.cpu().numpy(), ref[i][2])
            np.testing.assert_array_equal(ol.cpu().numpy()[:total], ref[i][1][:total])
            got = out.cpu().numpy()
            for j in range(total):
                s = slice(j * stride, j * stride + int(ref[i][1][j]))
                assert np.array_equal(got[s], ref[i][0][s]), (i, k, j)


@pytest.mark.gpu
def test_captured_counting_call_owns_its_shards():
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    fa, fo, fl = _dev(fx["arena"], fx["offsets"].astype(np.int64), fx["lengths"].view(np.int16))
    fexp = counters_of(fx["expect"])
    half = len(fx["offsets"]) // 2
    hexp = counters_of(fx["expect"][:half])
    cap = torch.cuda.Stream()
    g_cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda:0")
    with torch.cuda.stream(cap):  # the stream's direct shards exist before the capture
        csum.validate_frames(fa, fo, fl, counters=g_cnt, want_flags=False)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        csum.validate_frames(fa, fo, fl, counters=g_cnt, want_flags=False)
    other = torch.cuda.Stream()
    d_cnt = torch.full((40, 4), -1, dtype=torch.int32, device="cuda:0")
    g_seen = []
    for k in range(40):
        with torch.cuda.stream(other):
            g.replay()
        # direct counting calls on the capture stream, overlapping the replay
        ho, hl = fo[:half], fl[:half]
        assert csum.lib.tulips_csum_validate_frames(fa.data_ptr(), ho.data_ptr(),
                                                    hl.data_ptr(), half, None,
                                                    d_cnt[k].data_ptr(),
                                                    cap.cuda_stream) == 0
        other.synchronize()
        g_seen.append(g_cnt.cpu().numpy().view(np.uint32).copy())
    torch.cuda.synchronize()
    for s in g_seen:
        np.testing.assert_array_equal(s, fexp)
    np.testing.assert_array_equal(d_cnt.cpu().numpy().view(np.uint32),
                                  np.tile(hexp, (40, 1)))
    del g
    csum.release_stream(cap.cuda_stream)


@pytest.mark.gpu
def test_captured_counting_without_warmup_many_graphs():
    """Counting calls captured on a stream that never counted directly, 20
    graphs on one stream: each capture gets zeroed shards of its own (made in
    relaxed capture mode, zeroed by a kernel node of its graph), and every
    graph's replays count exactly."""
    import torch
    from tulips_amd import csum
    fx = frames_fixture()
    fa, fo, fl = _dev(fx["arena"], fx["offsets"].astype(np.int64), fx["lengths"].view(np.int16))
    fexp = counters_of(fx["expect"])
    cap, other = torch.cuda.Stream(), torch.cuda.Stream()
    graphs = []
    for k in range(20):
        cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda:0")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            csum.validate_frames(fa, fo, fl, counters=cnt, want_flags=False)
        graphs.append((g, cnt))
    for rep in range(2):
        for g, cnt in graphs:
            cnt.fill_(-1)
            torch.cuda.synchronize()
            with torch.cuda.stream(other):
                g.replay()
            torch.cuda.synchronize()
            np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32), fexp)
    del graphs
    torch.cuda.synchronize()
    csum.release_stream(cap.cuda_stream)


@pytest.mark.gpu
def test_release_stream_keeps_memory_flat(oracle):
    import torch
    from tulips_amd import csum
    hip = _hip()
    n, L = 4096, 1500
    arena, offs, lens = _all_bad(n, L, 5)
    fx = frames_fixture()
    fa, fo, fl = _dev(fx["arena"], fx["offsets"].astype(np.int64), fx["lengths"].view(np.int16))
    rng = np.random.default_rng(9)
    frames = [super_frame(oracle, rng, int(p)) for p in rng.integers(3000, 60000, 16)]
    sa, so, sl = _dev(*[(x.astype(np.int64) if x.dtype == np.uint64 else
                         x.view(np.int16) if x.dtype == np.uint16 else x)
                        for x in seg_pack(frames, rng)])
    cnt = torch.zeros(4, dtype=torch.int32, device="cuda:0")
    out = torch.empty(2048 * 1024, dtype=torch.uint8, device="cuda:0")
    olen = torch.zeros(1024, dtype=torch.int16, device="cuda:0")
    first = torch.empty(17, dtype=torch.int32, device="cuda:0")
    aout = torch.empty(n, dtype=torch.int16, device="cuda:0")

    def cycle():
        s = C.c_void_p()
        assert hip.hipStreamCreate(C.byref(s)) == 0
        st = s.value
        assert csum.lib.tulips_csum_verify(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                           None, None, None, cnt.data_ptr(), n, MODE_INET,
                                           st) == 0
        assert csum.lib.tulips_csum_validate_frames(fa.data_ptr(), fo.data_ptr(),
                                                    fl.data_ptr(), int(fo.numel()), None,
                                                    cnt.data_ptr(), st) == 0
        assert csum.lib.tulips_csum_segment_frames(sa.data_ptr(), so.data_ptr(),
                                                   sl.data_ptr(), 16, 1460, out.data_ptr(),
                                                   2048, 1024, olen.data_ptr(),
                                                   first.data_ptr(), st) == 0
        # an arena call (split-form span words: 17 arrays)
        assert csum.lib.tulips_csum_batch_arena(arena.data_ptr(), n * L, offs.data_ptr(),
                                                lens.data_ptr(), None, None, None,
                                                aout.data_ptr(), n, MODE_INET, st) == 0
        assert csum.lib.tulips_csum_release_stream(st) == 0
        assert hip.hipStreamDestroy(s) == 0

    for _ in range(3):
        cycle()
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(100):
        cycle()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    # unreleased, each stream would keep ~1.3 MB (its shards, the scan
    # totals, run map and descriptors, its span words): 130 MB over 100
    # streams
    assert free0 - free1 < 8 << 20, (free0 - free1)
    np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32),
                                  counters_of(fx["expect"]))


@pytest.mark.gpu
def test_captured_arena_calls_own_their_words(oracle):
    """Split-form arena calls captured on a stream with no state yet (the
    words are made in relaxed capture mode), replayed on another stream while
    direct arena calls of another batch run on the capture stream: both
    exact every time."""
    import torch
    from tulips_amd import csum
    rng = np.random.default_rng(77)
    res = []
    for n in (30000, 20000):
        lens = rng.integers(40, 9000, n).astype(np.uint16)
        offs = np.zeros(n, np.uint64)
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
        total = int(lens.astype(np.int64).sum())
        buf = rng.integers(0, 256, total + 16, dtype=np.uint8)
        exp = oracle.batch(buf, offs, lens, mode=MODE_INET, nthreads=8)
        dv = _dev(buf, offs.astype(np.int64), lens.view(np.int16))
        res.append((n, total, dv, exp, torch.empty(n, dtype=torch.int16, device="cuda:0")))
    cap, other = torch.cuda.Stream(), torch.cuda.Stream()

    def call(r, st):
        n, total, (a, o, l), _, out = r
        assert csum.lib.tulips_csum_batch_arena(a.data_ptr(), total, o.data_ptr(), l.data_ptr(),
                                                None, None, None, out.data_ptr(), n,
                                                MODE_INET, st) == 0
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for _ in range(3):
            call(res[0], cap.cuda_stream)
    for _ in range(20):
        res[0][4].fill_(0)
        res[1][4].fill_(0)
        torch.cuda.synchronize()
        with torch.cuda.stream(other):
            g.replay()
        call(res[1], cap.cuda_stream)
        torch.cuda.synchronize()
        for r in res:
            np.testing.assert_array_equal(r[4].cpu().numpy().view(np.uint16), r[3])
    del g
    csum.release_stream(cap.cuda_stream)


@pytest.mark.gpu
def test_captured_contract_breaking_replay_does_not_spoil_the_next(oracle):
    """one captured arena call replayed first over a batch
    that breaks the arena contract (overlapping segments) and then, with the
    same buffers refilled, over valid batches. The split words carry the
    launch's dispatch id, which differs per replay, so the bad replay's
    residue is taken over, never added to: every valid replay is exact."""
    import torch
    from tulips_amd import csum
    rng = np.random.default_rng(4040)
    n = 20000
    lens = rng.integers(1000, 9000, n).astype(np.uint16)
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    total = int(lens.astype(np.int64).sum())
    buf = rng.integers(0, 256, total + 16, dtype=np.uint8)
    exp = oracle.batch(buf, offs, lens, mode=MODE_INET, nthreads=8)
    bad = offs.copy()
    bad[1::3] -= np.minimum(bad[1::3], np.uint64(6000))     # overlaps its predecessors
    bad = np.maximum.accumulate(bad)
    a, o, l = _dev(buf, offs.astype(np.int64), lens.view(np.int16))
    good_o = o.clone()
    bad_o = torch.from_numpy(bad.astype(np.int64)).to("cuda:0")
    out = torch.empty(n, dtype=torch.int16, device="cuda:0")
    cap = torch.cuda.Stream()
    # words made before the capture (direct call on the stream)
    assert csum.lib.tulips_csum_batch_arena(a.data_ptr(), total, o.data_ptr(), l.data_ptr(),
                                            None, None, None, out.data_ptr(), n, MODE_INET,
                                            cap.cuda_stream) == 0
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        assert csum.lib.tulips_csum_batch_arena(a.data_ptr(), total, o.data_ptr(),
                                                l.data_ptr(), None, None, None,
                                                out.data_ptr(), n, MODE_INET,
                                                cap.cuda_stream) == 0
    for rnd in range(3):
        o.copy_(bad_o)
        g.replay()
        torch.cuda.synchronize()
        o.copy_(good_o)
        for _ in range(2):
            out.fill_(0)
            g.replay()
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exp,
                                          err_msg=f"round {rnd}")
    del g
    csum.release_stream(cap.cuda_stream)


@pytest.mark.gpu
def test_captured_arena_call_replayed_on_alternating_streams(oracle):
    """One captured arena call replayed on two streams in turn (two hardware
    queues, whose dispatch ids may run in step), the bytes changed between
    replays: the word array is the graph's, so consecutive launches on it come
    from different queues. The split words' tag offsets the dispatch id by a
    hash of the queue (span_kernel.h launch_tag), so a launch never takes the
    other queue's residue for its partner's part: every replay is exact."""
    import torch
    from tulips_amd import csum
    rng = np.random.default_rng(5151)
    n = 24000
    lens = rng.integers(40, 4000, n).astype(np.uint16)
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    total = int(lens.astype(np.int64).sum())
    bufs = [rng.integers(0, 256, total + 16, dtype=np.uint8) for _ in range(2)]
    exps = [oracle.batch(b, offs, lens, mode=MODE_INET, nthreads=8) for b in bufs]
    a, o, l = _dev(bufs[0], offs.astype(np.int64), lens.view(np.int16))
    srcs = [torch.from_numpy(b).to("cuda:0") for b in bufs]
    out = torch.empty(n, dtype=torch.int16, device="cuda:0")
    cap = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        assert csum.lib.tulips_csum_batch_arena(a.data_ptr(), total, o.data_ptr(),
                                                l.data_ptr(), None, None, None,
                                                out.data_ptr(), n, MODE_INET,
                                                cap.cuda_stream) == 0
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for i in range(32):
        d = (i // 2) % 2
        with torch.cuda.stream(streams[i % 2]):
            a.copy_(srcs[d])
            out.fill_(0)
            g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exps[d],
                                      err_msg=f"replay {i}")
    del g
    csum.release_stream(cap.cuda_stream)


@pytest.mark.gpu
def test_zero_frames_zero_the_counters():
    import torch
    from tulips_amd import csum
    cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    assert csum.lib.tulips_csum_validate_frames(None, None, None, 0, None, cnt.data_ptr(),
                                                st) == 0
    torch.cuda.synchronize()
    assert cnt.cpu().numpy().tolist() == [0, 0, 0, 0]
    cnt.fill_(-1)
    t = csum.Tuning(group=16, unroll=6, nontemporal=1)
    assert csum.lib.tulips_csum_frames_tuned(0, None, None, None, 0, None, cnt.data_ptr(),
                                             t, st) == 0
    torch.cuda.synchronize()
    assert cnt.cpu().numpy().tolist() == [0, 0, 0, 0]


def test_release_stream_without_state_is_ok():
    """Releasing a stream the library never saw is a no-op (CPU: no device
    call is made for an unknown stream)."""
    from tulips_amd import csum
    assert csum.lib.tulips_csum_release_stream(C.c_void_p(0x1234)) == 0
