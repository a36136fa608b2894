"""GPU parity tests of the HIP decoder (XCodecDecoder::decode, xcodec/xcodec_decoder.cc:76-176)
against the oracle: status, decoded bytes, consumed bytes, unknown hash, cache growth."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


def _collision_pair(seed=1):
    rng = np.random.default_rng(seed)
    x = (rng.integers(2, 126, 2048, dtype=np.int64) * 2 + 1).astype(np.uint8)
    y = x.copy()
    y[100] += 2; y[101] -= 2; y[1500] -= 2; y[1501] += 2
    return x, y


def _check(ctx, oracle_mod, streams, warm_streams=None, warm_segments=None):
    import wanproxy_amd as w
    oc = oracle_mod.Cache()
    gc = w.XCodecCache(ctx, 1 << 16)
    dec = w.XCodecDecoder(gc)
    for h, seg in (warm_segments or []):
        import ctypes  # noqa: F401
        gc.enter(h, seg)
    if warm_segments:
        # the oracle cache is warmed through decode of EXTRACTs (same entries)
        oc.decode_batch([b"\xf1\x01" + bytes(seg) for _, seg in warm_segments])
    if warm_streams:
        oc.decode_batch(warm_streams)
        dec.decode_batch(warm_streams)
    want = oc.decode_batch(streams)
    got = dec.decode_batch(streams)
    for i, (g, e) in enumerate(zip(got, want)):
        assert g[0] == e[0], (i, "status", g[0], e[0])
        assert g[2] == e[2], (i, "consumed", g[2], e[2])
        assert g[3] == e[3], (i, "unknown", g[3], e[3])
        assert g[1] == e[1], (i, "bytes", len(g[1]), len(e[1]))
    assert len(gc) == len(oc)
    return got


def test_cfg1_roundtrip(gpu_ctx, oracle_mod):
    d = W.gen(1, 1 << 20)
    enc = oracle_mod.Cache().encode_batch([d])
    got = _check(gpu_ctx, oracle_mod, enc)
    assert got[0][1] == d.tobytes()


def test_charruns_and_escapes(gpu_ctx, oracle_mod):
    bufs = [np.full(512 * 1024, 0xF1, np.uint8), np.full(70000, 7, np.uint8)]
    rng = np.random.default_rng(2)
    e = rng.integers(0, 256, 50000, dtype=np.uint8)
    e[rng.random(50000) < 0.3] = 0xF1
    bufs.append(e)
    enc = oracle_mod.Cache().encode_batch(bufs)
    got = _check(gpu_ctx, oracle_mod, enc)
    assert [g[1] for g in got] == [b.tobytes() for b in bufs]


def test_cfg4_reference_heavy(gpu_ctx, oracle_mod):
    """cfg4 shape: decode cfg3-style encoder output with a decoder cache warmed by the warm-up streams."""
    pool = W.pool(512)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    bufs = W.repeat_buffers(48, 0x88, repeat_pct=90, np_segments=512, pool_bytes=pool)
    ec = oracle_mod.Cache()
    warm_enc = ec.encode_batch(warm)
    enc = ec.encode_batch(bufs)
    got = _check(gpu_ctx, oracle_mod, enc, warm_streams=warm_enc)
    assert [g[1] for g in got] == [b.tobytes() for b in bufs]


def test_error_paths(gpu_ctx, oracle_mod):
    streams = [b"abc\xf1\x07xyz", b"ab\xf1\x02" + bytes(range(8)) + b"tail", b"q\xf1\x01" + b"z" * 100,
               b"q\xf1\x02\x00", b"q\xf1", b"\xf1\x00\xf1\x00x", b"", b"plain", b"\xf1\x00",
               b"x\xf1\x00\xf1", b"\xf1\x03"]
    _check(gpu_ctx, oracle_mod, streams)


def test_output_overflow_leaves_the_cache_unchanged(gpu_ctx, oracle_mod):
    """A batch whose middle stream's output overflows its capacity fails with XC_EINVAL and enters
    nothing: no EXTRACT of any stream of the batch is found afterwards (the slots of the overflowing
    stream's later EXTRACTs were never written), and the same batch with room decodes as the oracle
    does."""
    import wanproxy_amd as w
    segs = [W.gen(0x7700 + i, 2048) for i in range(8)]
    ext = [b"\xf1\x01" + s.tobytes() for s in segs]
    streams = [b"a" + ext[0], b"b" + b"".join(ext[1:6]) + b"c", b"d" + ext[6] + ext[7]]
    gc = w.XCodecCache(gpu_ctx, 1 << 12)
    dec = w.XCodecDecoder(gc)
    seed = [W.gen(0x7800, 2048)]
    assert dec.decode_batch([b"\xf1\x01" + seed[0].tobytes()])[0][0] == 1
    n0 = len(gc)
    with pytest.raises(Exception, match="capacity"):
        dec.decode_batch(streams, out_cap=3 * 2048)
    assert len(gc) == n0
    for s in segs:
        assert gc.lookup(int(oracle_mod.hash_segment(s))) is None
    assert gc.lookup(int(oracle_mod.hash_segment(seed[0]))) is not None
    oc = oracle_mod.Cache()
    oc.decode_batch([b"\xf1\x01" + seed[0].tobytes()])
    assert dec.decode_batch(streams) == oc.decode_batch(streams)
    assert len(gc) == len(oc)


def test_cross_stream_order(gpu_ctx, oracle_mod):
    a, b, c = W.gen(40, 2048), W.gen(41, 2048), W.gen(42, 2048)
    ha, hb, hc = (oracle_mod.hash_segment(s) for s in (a, b, c))
    ref = lambda h: b"\xf1\x02" + int(h).to_bytes(8, "big")  # noqa: E731
    ext = lambda s: b"\xf1\x01" + s.tobytes()  # noqa: E731
    streams = [
        b"hello" + ref(hb) + b"x",                 # REF to a later stream's EXTRACT -> unknown
        ext(a) + b"mid" + ref(ha) + ext(b),        # self reference, then declares b
        ref(hb) + ref(ha) + b"ok",                 # earlier stream's declarations resolve
        ref(hc) + ext(c),                          # unknown first -> its EXTRACT never runs
        ref(hc) + b"z",                            # so c stays unknown here
        ext(c) + ref(hc),                          # now c is declared
    ]
    _check(gpu_ctx, oracle_mod, streams)


def test_extract_collisions(gpu_ctx, oracle_mod):
    x, y = _collision_pair()
    hx = oracle_mod.hash_segment(x)
    ext = lambda s: b"\xf1\x01" + s.tobytes()  # noqa: E731
    streams = [b"pre" + ext(x) + b"post", b"aa" + ext(y) + b"bb", ext(x) + ext(x),
               b"zz" + b"\xf1\x02" + int(hx).to_bytes(8, "big")]
    _check(gpu_ctx, oracle_mod, streams)
    # collision against a cached segment
    _check(gpu_ctx, oracle_mod, [ext(y) + b"q", b"w" + ext(x)], warm_segments=[(hx, x)])


def test_gpu_encode_gpu_decode_roundtrip(gpu_ctx):
    import wanproxy_amd as w
    pool = W.pool(256)
    bufs = W.repeat_buffers(40, 0x99, np_segments=256, pool_bytes=pool) + [W.gen(5, 3000)]
    ec = w.XCodecCache(gpu_ctx, 1 << 14)
    dc = w.XCodecCache(gpu_ctx, 1 << 14)
    enc = w.XCodecEncoder(ec).encode_batch(bufs)
    got = w.XCodecDecoder(dc).decode_batch(enc)
    assert [g[1] for g in got] == [b.tobytes() for b in bufs]
    assert all(g[0] == 1 and g[3] is None for g in got)
    assert len(ec) == len(dc)


@pytest.mark.parametrize("stream_ordered,input_ready", [(False, False), (True, False), (True, True)])
def test_device_resident_decode_plan(gpu_ctx, oracle_mod, stream_ordered, input_ready):
    """xc_decode_plan_create + xc_decode_run on HBM arenas, run three times over a restored cache
    snapshot (the bench's step): same results as the oracle every time.  Stream ordered
    (xc_dplan_set_completion): the runs return once decided, back to back with no host
    synchronisation; input ready (xc_dplan_set_input_ready): each run's parse on the side stream
    beside the previous run's emit, the token arrays alternating; a plan whose capacities are too
    small still fails (k_dres2's bound stops the early return)."""
    import torch
    import wanproxy_amd as w
    pool = W.pool(256)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    bufs = W.repeat_buffers(96, 0x77, 50, np_segments=256, pool_bytes=pool)
    eo = oracle_mod.Cache()
    warm_streams = eo.encode_batch(warm)
    streams = eo.encode_batch(bufs)
    streams.append(streams[3][:1000] + b"\xf1\x02" + bytes(8))  # unknown REF (stops the stream)
    streams.append(b"")
    oc = oracle_mod.Cache()
    oc.decode_batch(warm_streams)
    want = oc.decode_batch(streams)
    gc = w.XCodecCache(gpu_ctx, 1 << 14)
    w.XCodecDecoder(gc).decode_batch(warm_streams)
    gc.snapshot()
    lens = np.array([len(s) for s in streams], np.uint64)
    caps = lens * 205 + 16
    plan = w.DecodePlan(gc, lens, caps)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, s in enumerate(streams):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(s)] = np.frombuffer(s, np.uint8)
    n = len(streams)
    d_in = torch.from_numpy(arena).cuda()
    sets = [(torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda"),
             torch.zeros(3 * n, dtype=torch.int64, device="cuda"),
             torch.zeros(2 * n, dtype=torch.int32, device="cuda")) for _ in range(3)]
    plan.set_completion(stream_ordered)
    plan.set_input_ready(input_ready)
    torch.cuda.synchronize()
    for rep in range(3):
        d_out, u64, i32 = sets[rep]
        if stream_ordered:
            gc.restore_async()
        else:
            gc.restore()
            torch.cuda.synchronize()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), u64.data_ptr(), u64.data_ptr() + 8 * n,
                 i32.data_ptr(), u64.data_ptr() + 16 * n, i32.data_ptr() + 4 * n)
        if not stream_ordered:
            torch.cuda.synchronize()
    gpu_ctx.sync()
    torch.cuda.synchronize()
    for rep in range(3):
        d_out, u64, i32 = sets[rep]
        out = d_out.cpu().numpy()
        r64 = u64.cpu().numpy().astype(np.uint64)
        r32 = i32.cpu().numpy()
        for i, (st, data, cons, unk) in enumerate(want):
            o = int(plan.out_off[i])
            assert int(r32[i]) == st, (rep, i, "status")
            assert int(r64[n + i]) == cons, (rep, i, "consumed")
            assert (int(r64[2 * n + i]) if r32[n + i] else None) == unk, (rep, i, "unknown")
            assert out[o:o + int(r64[i])].tobytes() == data, (rep, i, "bytes")
    assert len(gc) == len(oc)
    st = plan.stats()
    assert st.n_entered > 0 and st.n_ref > 0 and st.rounds >= 1
    small = w.DecodePlan(gc, lens, np.maximum(lens, 1))
    small.set_completion(stream_ordered)
    d_out, u64, i32 = sets[0]
    gc.restore()
    with pytest.raises(w.XCodecError):
        small.run(d_in.data_ptr(), d_out.data_ptr(), u64.data_ptr(), u64.data_ptr() + 8 * n,
                  i32.data_ptr(), u64.data_ptr() + 16 * n, i32.data_ptr() + 4 * n)
    gpu_ctx.sync()


@pytest.mark.parametrize("input_ready", [False, True])
def test_device_resident_resolution_rounds(gpu_ctx, oracle_mod, input_ready):
    """Providers past their own stream's stop (test_cross_stream_order's streams, among ordinary
    ones) through the device-resident plan, four runs back to back over a restored snapshot: the
    round check of k_dfin asks for another resolution round, and with the input ready every run's
    parse enters its EXTRACTs into the batch table of its token set, which alternates between runs
    (xcodec_decoder.cc:101-166)."""
    import torch
    import wanproxy_amd as w
    a, b, c = W.gen(40, 2048), W.gen(41, 2048), W.gen(42, 2048)
    ha, hb, hc = (oracle_mod.hash_segment(s) for s in (a, b, c))
    ref = lambda h: b"\xf1\x02" + int(h).to_bytes(8, "big")  # noqa: E731
    ext = lambda s: b"\xf1\x01" + s.tobytes()  # noqa: E731
    pool = W.pool(64)
    eo = oracle_mod.Cache()
    streams = eo.encode_batch(W.repeat_buffers(12, 0x79, 50, np_segments=64, pool_bytes=pool))
    streams[2:2] = [b"hello" + ref(hb) + b"x", ext(a) + b"mid" + ref(ha) + ext(b), ref(hb) + ref(ha) + b"ok",
                    ref(hc) + ext(c), ref(hc) + b"z", ext(c) + ref(hc)]
    want = oracle_mod.Cache().decode_batch(streams)
    gc = w.XCodecCache(gpu_ctx, 1 << 14)
    gc.snapshot()
    lens = np.array([len(s) for s in streams], np.uint64)
    plan = w.DecodePlan(gc, lens, lens * 205 + 16)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, s in enumerate(streams):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(s)] = np.frombuffer(s, np.uint8)
    n = len(streams)
    d_in = torch.from_numpy(arena).cuda()
    plan.set_completion(True)
    plan.set_input_ready(input_ready)
    sets = [(torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda"),
             torch.zeros(3 * n, dtype=torch.int64, device="cuda"),
             torch.zeros(2 * n, dtype=torch.int32, device="cuda")) for _ in range(4)]
    torch.cuda.synchronize()
    for d_out, u64, i32 in sets:
        gc.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), u64.data_ptr(), u64.data_ptr() + 8 * n,
                 i32.data_ptr(), u64.data_ptr() + 16 * n, i32.data_ptr() + 4 * n)
        assert plan.stats().rounds >= 2
    gpu_ctx.sync()
    torch.cuda.synchronize()
    for rep, (d_out, u64, i32) in enumerate(sets):
        out = d_out.cpu().numpy()
        r64 = u64.cpu().numpy().astype(np.uint64)
        r32 = i32.cpu().numpy()
        for i, (st, data, cons, unk) in enumerate(want):
            o = int(plan.out_off[i])
            assert int(r32[i]) == st, (rep, i, "status")
            assert int(r64[n + i]) == cons, (rep, i, "consumed")
            assert (int(r64[2 * n + i]) if r32[n + i] else None) == unk, (rep, i, "unknown")
            assert out[o:o + int(r64[i])].tobytes() == data, (rep, i, "bytes")


@pytest.mark.parametrize("input_ready", [False, True])
def test_device_resident_cache_hits_and_collisions(gpu_ctx, oracle_mod, input_ready):
    """EXTRACTs whose hash the cache already holds, through the device-resident plan three times
    back to back over a restored snapshot: the same bytes (a cache hit, nothing entered) and other
    bytes under the same hash (a collision: the stream stops there), among ordinary streams and
    EXTRACTs past a stop (xcodec_decoder.cc:101-132).  With the input ready, round 0's cache probes
    run in k_dres2<true> after the side stream's parse; a plan whose output capacities are too
    small still fails there (the output bound goes to k_dfin through s_cnt)."""
    import torch
    import wanproxy_amd as w
    x, y = _collision_pair(3)
    hx = oracle_mod.hash_segment(x)
    segs = [W.gen(0x7900 + i, 2048) for i in range(6)]
    ext = lambda s: b"\xf1\x01" + s.tobytes()  # noqa: E731
    ref = lambda h: b"\xf1\x02" + int(h).to_bytes(8, "big")  # noqa: E731
    pool = W.pool(64)
    eo = oracle_mod.Cache()
    streams = eo.encode_batch(W.repeat_buffers(10, 0x7A, 50, np_segments=64, pool_bytes=pool))
    streams[1:1] = [b"pre" + ext(x) + b"post" + ext(segs[0]), b"aa" + ext(y) + b"bb" + ext(segs[1]),
                    ext(segs[2]) + ext(x) + ref(hx) + ext(segs[3]), ref(hx) + ext(y) + ext(segs[4]),
                    ext(segs[5]) + b"q" * 3000 + ext(x)]
    warm = [ext(x)]
    oc = oracle_mod.Cache()
    oc.decode_batch(warm)
    want = oc.decode_batch(streams)
    assert any(st == 0 for st, _, _, _ in want)  # (the collisions stop their streams)
    gc = w.XCodecCache(gpu_ctx, 1 << 14)
    w.XCodecDecoder(gc).decode_batch(warm)
    gc.snapshot()
    lens = np.array([len(s) for s in streams], np.uint64)
    plan = w.DecodePlan(gc, lens, lens * 205 + 16)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, s in enumerate(streams):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(s)] = np.frombuffer(s, np.uint8)
    n = len(streams)
    d_in = torch.from_numpy(arena).cuda()
    plan.set_completion(True)
    plan.set_input_ready(input_ready)
    sets = [(torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda"),
             torch.zeros(3 * n, dtype=torch.int64, device="cuda"),
             torch.zeros(2 * n, dtype=torch.int32, device="cuda")) for _ in range(3)]
    torch.cuda.synchronize()
    for d_out, u64, i32 in sets:
        gc.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), u64.data_ptr(), u64.data_ptr() + 8 * n,
                 i32.data_ptr(), u64.data_ptr() + 16 * n, i32.data_ptr() + 4 * n)
    gpu_ctx.sync()
    torch.cuda.synchronize()
    for rep, (d_out, u64, i32) in enumerate(sets):
        out = d_out.cpu().numpy()
        r64 = u64.cpu().numpy().astype(np.uint64)
        r32 = i32.cpu().numpy()
        for i, (st, data, cons, unk) in enumerate(want):
            o = int(plan.out_off[i])
            assert int(r32[i]) == st, (rep, i, "status")
            assert int(r64[n + i]) == cons, (rep, i, "consumed")
            assert (int(r64[2 * n + i]) if r32[n + i] else None) == unk, (rep, i, "unknown")
            assert out[o:o + int(r64[i])].tobytes() == data, (rep, i, "bytes")
    assert len(gc) == len(oc)
    # capacities too small for stream 1's output: the run fails, the cache is as restored
    small = w.DecodePlan(gc, lens, np.maximum(lens, 1))
    small.set_completion(True)
    small.set_input_ready(input_ready)
    d_out, u64, i32 = sets[0]
    gc.restore()
    n0 = len(gc)
    with pytest.raises(w.XCodecError):
        small.run(d_in.data_ptr(), d_out.data_ptr(), u64.data_ptr(), u64.data_ptr() + 8 * n,
                  i32.data_ptr(), u64.data_ptr() + 16 * n, i32.data_ptr() + 4 * n)
    gpu_ctx.sync()
    assert len(gc) == n0


@pytest.mark.parametrize("n", [5000, 17000])
def test_device_resident_many_streams(gpu_ctx, oracle_mod, n):
    """Many small streams whose segments repeat across streams (an EXTRACT in one stream, REFs to
    it in later ones; some streams stop on an unknown REF first, so REFs to their EXTRACTs need a
    second resolution round, and some at their end),
    through the device-resident plan with the input ready, twice over a restored snapshot (k_dfin's
    slot prefix over 5000 and 17000 streams: 4 and 17 streams per thread)."""
    import torch
    import wanproxy_amd as w
    pool = W.pool(64)
    eo = oracle_mod.Cache()
    streams = eo.encode_batch(W.repeat_buffers(n, 0x7B + n, 50, slots=2, np_segments=64, pool_bytes=pool))
    for i in range(7, n, 97):  # an unknown REF after the stream's own bytes
        streams[i] = streams[i] + b"\xf1\x02" + int(0x1234567 + i).to_bytes(8, "big")
    for i in range(11, n, 89):  # one before them: the stream's EXTRACTs never run, so later REFs
        streams[i] = b"\xf1\x02" + int(0x7654321 + i).to_bytes(8, "big") + streams[i]  # need a round more
    want = oracle_mod.Cache().decode_batch(streams)
    gc = w.XCodecCache(gpu_ctx, 1 << 16)
    gc.snapshot()
    lens = np.array([len(s) for s in streams], np.uint64)
    plan = w.DecodePlan(gc, lens, lens * 205 + 16)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, s in enumerate(streams):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(s)] = np.frombuffer(s, np.uint8)
    d_in = torch.from_numpy(arena).cuda()
    plan.set_completion(True)
    plan.set_input_ready(True)
    sets = [(torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda"),
             torch.zeros(3 * n, dtype=torch.int64, device="cuda"),
             torch.zeros(2 * n, dtype=torch.int32, device="cuda")) for _ in range(2)]
    torch.cuda.synchronize()
    for d_out, u64, i32 in sets:
        gc.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), u64.data_ptr(), u64.data_ptr() + 8 * n,
                 i32.data_ptr(), u64.data_ptr() + 16 * n, i32.data_ptr() + 4 * n)
    gpu_ctx.sync()
    torch.cuda.synchronize()
    off = np.array([int(plan.out_off[i]) for i in range(n)])
    for rep, (d_out, u64, i32) in enumerate(sets):
        out = d_out.cpu().numpy()
        r64 = u64.cpu().numpy().astype(np.uint64)
        r32 = i32.cpu().numpy()
        for i, (st, data, cons, unk) in enumerate(want):
            assert int(r32[i]) == st, (rep, i, "status")
            assert int(r64[n + i]) == cons, (rep, i, "consumed")
            assert (int(r64[2 * n + i]) if r32[n + i] else None) == unk, (rep, i, "unknown")
            assert out[off[i]:off[i] + int(r64[i])].tobytes() == data, (rep, i, "bytes")
    oc = oracle_mod.Cache()
    oc.decode_batch(streams)
    assert len(gc) == len(oc)
    st = plan.stats()
    assert st.rounds >= 2
    n_ref = sum(s.count(b"\xf1\x02") for s in streams)  # (an upper bound: escapes aside)
    assert 0 < st.n_ref <= n_ref and st.n_extract >= st.n_entered > 0
