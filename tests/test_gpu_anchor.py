"""GPU parity tests of the anchor scan: the first-round scan of a sub-batch takes
its events from the anchor index instead of testing every window end, and the bytes stay those of
the oracle (the reference's encoder, xcodec/xcodec_encoder.cc:60-260).  Forced with XC_SCAN=anchor
(the default picks it for large caches only); the whole GPU suite is also run that way
(tools/gpu_r3m.sh)."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


def _gear(seg):
    """G(p) = sum_{k<32} b[p-k] 2^k mod 2^32 of every position (p < 31: partial)."""
    g = np.zeros(len(seg), np.uint64)
    acc = 0
    for p, b in enumerate(seg.tolist()):
        acc = ((acc << 1) + b) & 0xFFFFFFFF
        g[p] = acc
    return g


def _last_anchor(seg):
    """A segment's anchor offset: its last position j >= 63 with G(j) < 2^26 (None: anchorless)."""
    g = _gear(seg)
    js = [p for p in range(63, len(seg)) if g[p] < (1 << 26)]
    return js[-1] if js else None


def _collision_pair(seed=1, in_anchor=False):
    """x, y with equal 64-bit hashes and different bytes (odd bytes, +-2 at (i, i+1, k, k+1) keep
    both sums); in_anchor: the changes inside the 64-byte context of x's anchor, so the index does
    not propose y's window for x (the collision is invisible to an anchor scan)."""
    rng = np.random.default_rng(seed)
    x = (rng.integers(2, 126, 2048, dtype=np.int64) * 2 + 1).astype(np.uint8)
    i, k = 100, 1500
    if in_anchor:
        j = _last_anchor(x)
        assert j is not None
        i, k = j - 40, j - 10
    y = x.copy()
    y[i] += 2; y[i + 1] -= 2; y[k] -= 2; y[k + 1] += 2
    return x, y


def _plan_run(ctx, cache, bufs, mode="anchor", completion=False):
    """One device-resident run of `bufs` (an EncodePlan in scan mode `mode`); the encoded streams
    and the run's counters."""
    import torch
    import wanproxy_amd as w
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    plan.set_scan(mode)
    if completion:
        plan.set_completion(True)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(max(len(bufs), 1), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    ctx.sync()
    out = d_out.cpu().numpy()
    lens = d_len.cpu().numpy()
    got = [out[int(plan.out_off[i]):int(plan.out_off[i]) + int(lens[i])].tobytes() for i in range(len(bufs))]
    st = plan.stats()
    plan.close()
    return got, st


def _same(got, want):
    assert len(got) == len(want)
    for i, (g, e) in enumerate(zip(got, want)):
        if g != e:
            n = min(len(g), len(e))
            d = next((k for k in range(n) if g[k] != e[k]), n)
            pytest.fail(f"buffer {i}: len gpu {len(g)} oracle {len(e)}, first diff at {d}")


def _pool_cache(ctx, oracle_mod, nseg=512, cap=1 << 15):
    import wanproxy_amd as w
    pool = W.pool(nseg)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    cache = w.XCodecCache(ctx, cap)
    oc = oracle_mod.Cache()
    _same(w.XCodecEncoder(cache).encode_batch(warm), oc.encode_batch(warm))
    return cache, oc, pool


def test_anchor_scan_repeats(gpu_ctx, oracle_mod, monkeypatch):
    """Aligned pool repeats and fresh data (the cfg workloads' shape): every sub-batch is
    anchor-scanned, none falls back, the bytes equal the oracle's."""
    monkeypatch.setenv("XC_SUB_MB", "1")
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod)
    bufs = W.repeat_buffers(64, 0x5151, np_segments=512, pool_bytes=pool)
    got, st = _plan_run(gpu_ctx, cache, bufs)
    _same(got, oc.encode_batch(bufs))
    assert st.anchor_scans == st.sub_batches > 1 and st.anchor_fallbacks == 0, (st.anchor_scans, st.sub_batches)
    assert len(cache) == len(oc)


def test_anchor_scan_shifted_and_cross_buffer(gpu_ctx, oracle_mod, monkeypatch):
    """Repeats at unaligned offsets (proposals the index must find between aligned windows),
    segments declared by earlier buffers of the same batch, a buffer's partial last block."""
    monkeypatch.setenv("XC_SCAN", "anchor")
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod, 256)
    a = W.gen(61, 65536)
    bufs = []
    for k in range(24):
        if k % 4 == 0:
            bufs.append(np.concatenate([W.gen(700 + k, 333 * k + 7), pool[k * 4096 + 99:k * 4096 + 99 + 20000]]))
        elif k % 4 == 1:
            bufs.append(np.concatenate([W.gen(800 + k, 1000 + k), a[k * 50:k * 50 + 30000], W.gen(900 + k, 3333)]))
        elif k % 4 == 2:
            bufs.append(a[k:].copy())
        else:
            bufs.append(np.concatenate([pool[(k % 64) * 2048:(k % 64) * 2048 + 16384], W.gen(950 + k, 5000)]))
    want = oc.encode_batch(bufs)
    got, st = _plan_run(gpu_ctx, cache, bufs, mode="auto")
    _same(got, want)
    assert st.anchor_scans >= 1
    assert len(cache) == len(oc)


def test_anchor_scan_collisions_fall_back(gpu_ctx, oracle_mod):
    """A constructed collision (H equal, bytes different: xcodec_encoder.cc:129-137) at a lookup
    that would set the candidate, invisible to the index (its anchor context differs): the walk
    takes it for a miss, the declaration's hash check finds the cache entry, and the exact scan
    redoes the sub-batch.  A REF at an unaligned position (found through the index) puts the
    lookup there: the hash restarts after it (xcodec_encoder.cc:111-118)."""
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod, 64)
    x, y = _collision_pair(3, in_anchor=True)
    warm = [np.concatenate([x, W.gen(71, 4000)])]
    _same(_plan_run(gpu_ctx, cache, warm)[0], oc.encode_batch(warm))
    seg = pool[5 * 2048:6 * 2048]
    bufs = [np.concatenate([W.gen(72, 100), seg, y, W.gen(73, 5000)]), W.gen(75, 40000),
            np.concatenate([W.gen(76, 300), seg, y])]
    got, st = _plan_run(gpu_ctx, cache, bufs)
    _same(got, oc.encode_batch(bufs))
    assert st.anchor_scans >= 1 and st.anchor_fallbacks >= 1, (st.anchor_scans, st.anchor_fallbacks)


@pytest.mark.parametrize("ch", [0, 0x41, 0xF1, 0x7F])
def test_anchor_scan_char_runs(gpu_ctx, oracle_mod, ch):
    """Constant runs: every position has the same 64-byte context, so a value's runs are either
    all anchors (records run-length coded, dense proposals) or none (an anchorless segment sends
    the run to the exact scan and keeps the cache there)."""
    import wanproxy_amd as w
    cache = w.XCodecCache(gpu_ctx, 1 << 12)
    oc = oracle_mod.Cache()
    bufs = [np.full(512 * 1024, ch, np.uint8), np.concatenate([W.gen(81, 3000), np.full(70000, ch, np.uint8)])]
    got, st = _plan_run(gpu_ctx, cache, bufs)
    _same(got, oc.encode_batch(bufs))
    assert len(got[0]) == 4600
    more = [np.concatenate([np.full(9000, ch, np.uint8), W.gen(82, 20000)]), W.gen(83, 30000)]
    got, st = _plan_run(gpu_ctx, cache, more)
    _same(got, oc.encode_batch(more))


def test_anchor_index_restore_growth_and_backfill(gpu_ctx, oracle_mod):
    """The index across the cache's life: segments entered by exact runs and by the host API are
    backfilled before an anchor run, a restore takes out what was indexed after the snapshot, a
    growth moves the index into the larger tables."""
    import wanproxy_amd as w
    cache = w.XCodecCache(gpu_ctx, 1024)
    oc = oracle_mod.Cache()
    first = W.random_buffers(8, seed0=0xC000)
    _same(_plan_run(gpu_ctx, cache, first, mode="exact")[0], oc.encode_batch(first))
    seg = W.gen(0xC777, 2048)
    h = oracle_mod.hash_segment(seg)
    cache.enter(h, seg)
    oc.enter(h, seg)
    cache.snapshot()
    snap = oc.clone()
    for k in range(3):  # 3 x 1280 segments: the cache grows from 1024
        bufs = W.random_buffers(40, seed0=0xC100 + 100 * k) + [np.concatenate([first[k], seg, first[k + 1]])]
        got, st = _plan_run(gpu_ctx, cache, bufs)
        _same(got, oc.encode_batch(bufs))
        assert st.anchor_scans >= 1
    assert cache.capacity > 1024
    cache.restore()
    again = W.random_buffers(4, seed0=0xC100) + [np.concatenate([first[5], seg, W.gen(0xC999, 9000)])]
    got, st = _plan_run(gpu_ctx, cache, again)
    _same(got, snap.clone().encode_batch(again))
    for k in range(2):  # restore / rerun cycles (the bench's pattern)
        cache.restore()
        got, st = _plan_run(gpu_ctx, cache, again, completion=True)
        _same(got, snap.clone().encode_batch(again))


@pytest.mark.parametrize("wide", [False, True])
def test_anchor_scan_recent_window_after_collisions(gpu_ctx, oracle_mod, monkeypatch, wide):
    """The recent window remembers collision lookups that an anchor scan does not look for (a
    pending candidate makes them irrelevant to the bytes); the tail check finds the run's last ones
    again.  A stateful connection's carried candidate y is declared after x (same hash) was entered
    and y's windows were looked up (collisions, remembering x's entry): the map then answers y and
    the window x (xcodec_cache.h:137-147,182-188), as in the oracle.  wide: run (c) also carries
    20000 small buffers in two sub-batches of > 8192 buffers, so that its cache enters run in
    k_insert and the tail check's probes beside its last emit on the side stream (xc_runtime.hip
    tail_check_side), the compares behind it."""
    import wanproxy_amd as w
    if wide:
        monkeypatch.setenv("XC_SUB_MB", "1")
    x, y = _collision_pair(5, in_anchor=True)
    cache = w.XCodecCache(gpu_ctx, 1 << 12)
    oc = oracle_mod.Cache()
    gs, os_ = w.XCodecStreamEncoder(cache), oracle_mod.Encoder(oc)
    # (a) a candidate y, looked up while absent, carried (encode() only)
    a = np.concatenate([y, W.gen(91, 100)])
    assert gs.encode(a) == os_.encode(a)
    # (b) x entered by an anchor-scanned batch
    b = [np.concatenate([x, W.gen(92, 3000)])]
    _same(_plan_run(gpu_ctx, cache, b)[0], oc.encode_batch(b))
    # (c) y's windows looked up while a candidate is pending: collisions with x (remembered)
    c = [np.concatenate([W.gen(93, 1000), y, W.gen(94, 3000)]), W.gen(95, 9000)]
    if wide:
        c += [W.gen(0x9500 + i, 100) for i in range(20000)]
    got, st = _plan_run(gpu_ctx, cache, c)
    _same(got, oc.encode_batch(c))
    assert st.anchor_scans >= 1
    if wide:
        assert st.sub_batches >= 2 and st.redone == 0, (st.sub_batches, st.redone)
    # (d) y declared: the hash entered twice (map: y, window: x)
    d = W.gen(96, 4096)
    assert gs.encode(d) == os_.encode(d)
    assert gs.flush() == os_.flush()
    # (e) fresh encoders see the window's x
    e = [np.concatenate([W.gen(97, 500), x, W.gen(98, 200)]), np.concatenate([y, x, W.gen(99, 64)])]
    assert w.XCodecEncoder(cache).encode_batch(e) == oc.encode_batch(e)
    assert len(cache) == len(oc)
    # (f) a device-resident run on that cache: replayed by the library into the run's arenas
    f = [np.concatenate([x, W.gen(0x9A, 700)]), np.concatenate([W.gen(0x9B, 90), y]), W.gen(0x9C, 5000)]
    _same(_plan_run(gpu_ctx, cache, f)[0], oc.encode_batch(f))
    assert len(cache) == len(oc)


@pytest.mark.parametrize("ch", [0x41, 0xF1])
def test_anchorless_segment_survives_a_host_enter(gpu_ctx, oracle_mod, ch):
    """An anchor run enters a segment without an anchor (a constant run of a byte whose G never
    falls below 2^26) at an unaligned position (after a REF found through the index): the emit
    records it on the device only.  A host-API enter (xc_cache_enter) in between must not erase that
    record, or the next anchor run would not fall back to the exact scan and would miss the REFs to
    that segment (xcodec_encoder.cc:111-118)."""
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod, 64)
    # (2600 bytes: the declared segment right after the REF is all ch, while every aligned block still
    # has an anchor, so no predicted declaration sends the run to the exact scan)
    run = np.full(2600, ch, np.uint8)
    first = [np.concatenate([W.gen(0xA1, 300), pool[7 * 2048:8 * 2048], run, W.gen(0xA2, 3000)])]
    assert all(_last_anchor(first[0][i:i + 2048]) is not None for i in range(0, len(first[0]) - 2047, 2048))
    got, st = _plan_run(gpu_ctx, cache, first)
    _same(got, oc.encode_batch(first))
    assert st.anchor_scans >= 1 and st.anchor_fallbacks == 0, (st.anchor_scans, st.anchor_fallbacks)
    seg = W.gen(0xA3, 2048)
    h = oracle_mod.hash_segment(seg)
    cache.enter(h, seg)
    oc.enter(h, seg)
    again = [np.concatenate([W.gen(0xA4, 777), np.full(4500, ch, np.uint8), W.gen(0xA5, 2000)]),
             np.concatenate([W.gen(0xA6, 1500), seg, W.gen(0xA7, 100)])]
    want = oc.encode_batch(again)
    assert b"\xf1\x02" in want[0]  # the run is a REF to the anchorless segment in the reference
    got, st = _plan_run(gpu_ctx, cache, again)
    _same(got, want)
    assert len(cache) == len(oc)


def test_anchor_scan_collision_with_a_twin_declared_in_the_same_sub_batch(gpu_ctx, oracle_mod):
    """The invisible collision (y's anchor context differs from x's) at a lookup that would set the
    candidate, where x is not in the cache but declared by an EARLIER buffer of the same anchor-
    scanned sub-batch (the declaration set D, not the cache): the reference sees x in its map at that
    lookup and does not take y as the candidate (xcodec_encoder.cc:129-137).  The REF before y (found
    through the index) puts the lookup exactly at y's window end (xcodec_encoder.cc:111-118)."""
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod, 64)
    x, y = _collision_pair(7, in_anchor=True)
    assert oracle_mod.hash_segment(x) == oracle_mod.hash_segment(y)
    seg = pool[9 * 2048:10 * 2048]
    bufs = [np.concatenate([x, W.gen(0xB1, 4000)]),                       # x: a (predicted) declaration
            W.gen(0xB2, 40000),
            np.concatenate([W.gen(0xB3, 300), seg, y, W.gen(0xB4, 3000)]),  # REF seg, then y's window
            np.concatenate([W.gen(0xB5, 1300), seg, y]),
            np.concatenate([y, W.gen(0xB6, 2500)])]                        # aligned: a cross-buffer D match
    want = oc.encode_batch(bufs)
    got, st = _plan_run(gpu_ctx, cache, bufs)
    _same(got, want)
    assert st.anchor_scans >= 1
    assert len(cache) == len(oc)
    # and once more on the grown cache (x now in the cache, y's windows again at candidate lookups)
    more = [np.concatenate([W.gen(0xB7, 900), seg, y, W.gen(0xB8, 700)]), np.concatenate([x, y])]
    got, st = _plan_run(gpu_ctx, cache, more)
    _same(got, oc.encode_batch(more))


def test_anchor_scan_twin_against_a_carried_candidate(gpu_ctx, oracle_mod):
    """A stateful connection carries a pending candidate whose window is y's; an anchor-scanned batch
    then declares the twin x; the connection's next call completes the lookups after the candidate
    and declares y (a duplicate enter of the hash: the map takes y, the window keeps what it
    remembered), and fresh encoders after it see the reference's answers (xcodec_encoder.cc:77-82,
    203-215; xcodec_cache.h:137-147,182-188)."""
    import wanproxy_amd as w
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod, 64)
    x, y = _collision_pair(9, in_anchor=True)
    seg = pool[3 * 2048:4 * 2048]
    gs, os_ = w.XCodecStreamEncoder(cache), oracle_mod.Encoder(oc)
    a = np.concatenate([W.gen(0xC1, 200), seg, y, W.gen(0xC2, 60)])   # candidate y, carried
    assert gs.encode(a) == os_.encode(a)
    b = [np.concatenate([x, W.gen(0xC3, 4000)]), np.concatenate([W.gen(0xC4, 700), seg, y, W.gen(0xC5, 900)])]
    got, st = _plan_run(gpu_ctx, cache, b)
    _same(got, oc.encode_batch(b))
    assert st.anchor_scans >= 1
    c = W.gen(0xC6, 4200)
    assert gs.encode(c) == os_.encode(c)
    assert gs.flush() == os_.flush()
    e = [np.concatenate([W.gen(0xC7, 300), seg, x, W.gen(0xC8, 90)]), np.concatenate([y, x]),
         np.concatenate([W.gen(0xC9, 300), seg, y])]
    assert w.XCodecEncoder(cache).encode_batch(e) == oc.encode_batch(e)
    assert len(cache) == len(oc)


def _anchorless_random():
    """A 2048-byte segment of random-looking bytes without an anchor (G >= 2^26 at every offset >= 63):
    anchors cluster (G(p) shifts G(p - 1) up), so about one random segment in 10^7 has none; this one
    was declared by the bench's live-cache leg (batch seed 0x555a, tests/golden/anchorless_segment.bin)."""
    import os
    seg = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", "anchorless_segment.bin"), np.uint8)
    assert len(seg) == 2048 and _last_anchor(seg) is None
    return seg


def test_anchor_scan_finds_a_cached_anchorless_segment(gpu_ctx, oracle_mod, monkeypatch):
    """A cached segment without an anchor keeps the cache in anchor mode: windows with no input
    anchor at offsets 63 .. 2047 (gap windows) are proposed beside the index's, so every repeat of
    the segment is found (unaligned, aligned, at a buffer's start and end, across a k_blockhash
    group boundary, twice in a row, right after a REF) with no sub-batch falling back."""
    monkeypatch.setenv("XC_SUB_MB", "1")
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod, 64)
    s = _anchorless_random()
    first = [np.concatenate([s, W.gen(0xB2, 5000)])]  # (declared: the buffer's first segment)
    got, st = _plan_run(gpu_ctx, cache, first)
    _same(got, oc.encode_batch(first))
    g = lambda k, n: W.gen(0xB400 + k, n)
    bufs = [np.concatenate([g(0, 1), s, g(1, 3000)]),
            np.concatenate([g(2, 555), s, g(3, 70)]),
            np.concatenate([g(4, 2047), s, g(5, 2047)]),
            np.concatenate([g(6, 2048), s, g(7, 4096)]),           # aligned
            np.concatenate([s, g(8, 9000)]),                        # at the start
            np.concatenate([g(9, 12000), s]),                       # at the end
            np.concatenate([g(10, 16384 - 700), s, g(11, 9000)]),  # across the first group boundary
            np.concatenate([g(12, 300), s, s, g(13, 1000)]),        # twice
            np.concatenate([g(14, 100), pool[3 * 2048:4 * 2048], s, g(15, 500)])]  # after a REF
    bufs += W.repeat_buffers(40, 0xB5, np_segments=64, pool_bytes=pool)  # (more sub-batches)
    want = oc.encode_batch(bufs)
    assert all(want[i].count(b"\xf1\x02") >= 1 + (i == 7) for i in range(9))
    got, st = _plan_run(gpu_ctx, cache, bufs)
    _same(got, want)
    assert st.anchor_scans == st.sub_batches > 1 and st.anchor_fallbacks == 0, \
        (st.anchor_scans, st.sub_batches, st.anchor_fallbacks)
    assert len(cache) == len(oc)


def test_early_hashing_after_an_async_restore(gpu_ctx, oracle_mod, monkeypatch):
    """The bench's step (xc_cache_restore_async, then the next run of the same plan with its input
    ready, no host synchronisation between): the next run's first sub-batch is hashed on the side
    stream at once, possibly before the restore has removed the previous run's entries.  Run A
    declares blocks X0, X1; after a restore, run B holds [X0][X1][Y] whose window across X1 | Y
    equals a pool segment S, found only through an anchor of S that lies in X1.  The stale tables
    still hold X0 and X1, but a block counts as cached for the anchor records (a cached block after
    a cached block writes none) only through entries that survive the restore: X1's records are
    written and the REF to S is found.  (Which of the two the device runs first is not forced here:
    the test fails only on the interleaving that exposes a stale block, xc_cache.removed_floor.)"""
    import torch
    import wanproxy_amd as w
    monkeypatch.setenv("XC_SUB_MB", "2")
    pool = W.pool(512)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    S = pool[77 * 2048:78 * 2048]
    j = _last_anchor(S)
    assert j is not None and j < 2000
    o = (2048 - j) // 2  # S = X1[o:] + Y[:o], S's anchor in the X1 part
    X0, X1, Y = W.gen(0x7A00, 2048), W.gen(0x7A01, 2048).copy(), W.gen(0x7A02, 2048 * 3).copy()
    X1[o:] = S[:2048 - o]
    Y[:o] = S[2048 - o:]
    fill = W.gen(0x7A03, 65536 - 5 * 2048)
    runs = {"A": W.repeat_buffers(96, 0x7A10, np_segments=512, pool_bytes=pool)}
    runs["B"] = [b.copy() for b in runs["A"]]
    runs["A"][5] = np.concatenate([X0, X1, W.gen(0x7A04, 3 * 2048), fill])
    runs["B"][5] = np.concatenate([X0, X1, Y, fill])
    cache = w.XCodecCache(gpu_ctx, 1 << 14)
    oc = oracle_mod.Cache()
    w.XCodecEncoder(cache).encode_batch(warm)
    oc.encode_batch(warm)
    cache.snapshot()
    want = {k: oc.clone().encode_batch(v) for k, v in runs.items()}
    assert b"\xf1\x02" + int(oracle_mod.hash_segment(S)).to_bytes(8, "big") in want["B"][5]
    plan = w.EncodePlan(cache, [65536] * 96)
    plan.set_completion(True)
    plan.set_input_ready(True)
    plan.set_scan("anchor")
    arenas = {}
    for k, bufs in runs.items():
        arena = np.zeros(plan.in_bytes, np.uint8)
        for i, b in enumerate(bufs):
            arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
        arenas[k] = torch.from_numpy(arena).cuda()
    d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(96, dtype=torch.int64, device="cuda")
    early = []
    for n, k in enumerate("ABABAB"):
        gpu_ctx.sync()
        d_in.copy_(arenas[k])
        torch.cuda.synchronize()  # (the input is complete at the submit)
        if n:
            cache.restore_async()  # (no host synchronisation between it and the next submit)
        plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        plan.wait()
        early.append(int(plan.stats().early_hashed))
        gpu_ctx.sync()
        out, lens = d_out.cpu().numpy(), d_len.cpu().numpy()
        got = [out[int(plan.out_off[i]):int(plan.out_off[i]) + int(lens[i])].tobytes() for i in range(96)]
        _same(got, want[k])
    assert early[1::2] == [1, 1, 1], early  # (every B run hashed ahead: the A run before it ran clean)
    plan.close()


def test_many_anchor_runs_of_one_plan(gpu_ctx, oracle_mod, monkeypatch):
    """Hundreds of anchor-scanned runs of ONE plan (its declaration set reused, cleared as keys and
    values only) over distinct inputs on a live cache: fresh data, aligned pool repeats and repeats of
    earlier runs at unaligned offsets (declarations the predictions miss: another declaration round,
    redone step by step).  Every run finishes and equals the oracle (the set's lo32 keys
    must not fill up across runs)."""
    import torch
    import wanproxy_amd as w
    monkeypatch.setenv("XC_SCAN", "anchor")
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod, 256, cap=1 << 12)
    lens = [65536, 40000, 65536, 12345, 65536, 30001]
    plan = w.EncodePlan(cache, lens)
    plan.set_scan("anchor")
    d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(lens), dtype=torch.int64, device="cuda")
    prev = None
    scans = redone = 0
    for k in range(300):
        rng = np.random.default_rng(0x9000 + k)
        bufs = []
        for i, n in enumerate(lens):
            kind = (k + i) % 3
            if kind == 0 or prev is None:
                b = W.gen(0x9100 + 8 * k + i, n)
            elif kind == 1:  # aligned pool repeats between fresh bytes
                s = int(rng.integers(0, 200)) * 2048
                b = np.concatenate([pool[s:s + 8192], W.gen(0x9200 + 8 * k + i, n)])[:n]
            else:  # an earlier run's bytes at an unaligned offset
                o = int(rng.integers(1, 2047))
                b = np.concatenate([W.gen(0x9300 + 8 * k + i, o), prev[(i + 1) % len(lens)]])[:n]
            if len(b) < n:
                b = np.concatenate([b, W.gen(0x9400 + 8 * k + i, n - len(b))])
            bufs.append(b)
        arena = np.zeros(plan.in_bytes, np.uint8)
        for i, b in enumerate(bufs):
            arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
        d_in.copy_(torch.from_numpy(arena))
        torch.cuda.synchronize()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        gpu_ctx.sync()
        out = d_out.cpu().numpy()
        ln = d_len.cpu().numpy()
        got = [out[int(plan.out_off[i]):int(plan.out_off[i]) + int(ln[i])].tobytes() for i in range(len(bufs))]
        _same(got, oc.encode_batch(bufs))
        st = plan.stats()
        scans += int(st.anchor_scans)
        redone += int(st.redone)
        prev = bufs
    plan.close()
    assert scans >= 250 and redone > 0, (scans, redone)
    assert len(cache) == len(oc)


@pytest.mark.parametrize("min_keys,anchored", [("1", True), ("1000000000", False)])
def test_anchor_min_keys_knob(gpu_ctx, oracle_mod, monkeypatch, min_keys, anchored):
    """XC_ANCHOR_MIN_KEYS (the cached + new keys from which a plan in AUTO mode scans through the
    anchor index, 200 000 by default): a 1-key threshold anchor-scans a small cache's runs, a huge one
    never; both encode the oracle's bytes."""
    monkeypatch.delenv("XC_SCAN", raising=False)
    monkeypatch.setenv("XC_ANCHOR_MIN_KEYS", min_keys)
    monkeypatch.setenv("XC_SUB_MB", "1")
    cache, oc, pool = _pool_cache(gpu_ctx, oracle_mod)
    bufs = W.repeat_buffers(40, 0x5252, np_segments=512, pool_bytes=pool)
    bufs[5] = np.concatenate([W.gen(0x5253, 1111), bufs[3][:50000]])
    got, st = _plan_run(gpu_ctx, cache, bufs, mode="auto")
    _same(got, oc.encode_batch(bufs))
    assert (st.anchor_scans > 0) == anchored, (st.anchor_scans, st.sub_batches)
    assert len(cache) == len(oc)
