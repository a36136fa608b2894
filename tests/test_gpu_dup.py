"""A hash entered twice with different bytes (XCodecMemoryCache::enter, xcodec/xcodec_cache.h:182-188).

The reference asserts that an entered hash is new; a release build overwrites the map value, while
the 64-entry recent window (:94-98,128-147) keeps returning the bytes it remembered for that hash
until 64 later remembers push the entry out.  The only way an encoder reaches it: a stateful
connection's candidate is looked up (a miss) in one call and declared in a later one
(xcodec/xcodec_encoder.cc:77-82,203-215), after another connection entered a different segment with
the same 64-bit hash.  The hash is weak enough to build such a pair: odd bytes with +-2 swaps at
(i, i+1, j, j+1) keep both sums.

Every call's bytes must equal the stateful oracle's (oracle/xc_oracle.c: release semantics with the
recent window), and the cache's entry count the reference map's size."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu

POOL = 96


def _collision_pair(seed=1):
    rng = np.random.default_rng(seed)
    x = (rng.integers(2, 126, 2048, dtype=np.int64) * 2 + 1).astype(np.uint8)
    y = x.copy()
    y[100] += 2; y[101] -= 2; y[1500] -= 2; y[1501] += 2
    return x, y


def _cat(*a):
    return np.concatenate([np.asarray(v, np.uint8) for v in a])


def _run(ctx, oracle_mod, nconn, calls, batch):
    import wanproxy_amd as w
    warm = W.pool_warmup_buffers(POOL)
    oc = oracle_mod.Cache()
    gc = w.XCodecCache(ctx, 1 << 12)
    oc.encode_batch(warm)
    w.XCodecEncoder(gc).encode_batch(warm)
    oenc = [oracle_mod.Encoder(oc) for _ in range(nconn)]
    genc = [w.XCodecStreamEncoder(gc) for _ in range(nconn)]
    want = []
    for k, d, f in calls:
        o = oenc[k].encode(d)
        if f:
            o += oenc[k].flush()[1]
        want.append(o)
    if batch:
        got = w.encode_streams([(genc[k], d, f) for k, d, f in calls])
    else:
        got = []
        for k, d, f in calls:
            o = genc[k].encode(d)
            if f:
                o += genc[k].flush()[1]
            got.append(o)
    bad = [i for i, (g, e) in enumerate(zip(got, want)) if g != e]
    assert not bad, f"calls {bad} differ from the oracle"
    for k in range(nconn):
        assert genc[k].flush() == oenc[k].flush(), k
    assert len(gc) == len(oc)
    return want, gc, oc


def _calls(remembered: bool, evict: int):
    """Connection 0 carries candidate x across calls; connection 1 enters the twin y first.
    remembered: a lookup of y (connection 2) puts y's entry in the recent window before x is
    declared.  evict: REFs of that many distinct pool segments after the declaration (64 push the
    remembered entry out)."""
    x, y = _collision_pair()
    p = W.pool(POOL)
    calls = [
        (0, _cat(x, W.gen(11, 100)), False),      # candidate x, carried (encode() only)
        (1, y, True),                             # y declared by flush(): the hash is in the map
    ]
    if remembered:
        calls.append((2, _cat(y, W.gen(12, 50)), True))  # REF y: remembered in the window
    calls += [
        (0, W.gen(13, 4096), False),              # x declared at cand + 4095: the duplicate enter
        (3, y, True),                             # window: y (REF) / map: x (collision)
        (4, x, True),                             # window: y (collision) / map: x (REF)
    ]
    if evict:
        segs = [p[2048 * i:2048 * (i + 1)] for i in range(evict)]
        calls.append((5, _cat(*segs), True))
    calls += [
        (6, x, True),
        (7, y, True),
        (0, W.gen(14, 300), True),
    ]
    return calls


def _has_ref(stream: bytes) -> bool:
    return b"\xf1\x02" in stream


@pytest.mark.parametrize("batch", [True, False])
@pytest.mark.parametrize("remembered,evict", [(True, 0), (True, 70), (False, 0), (True, 40)])
def test_duplicate_enter_follows_the_release_reference(gpu_ctx, oracle_mod, batch, remembered, evict):
    calls = _calls(remembered, evict)
    want, gc, oc = _run(gpu_ctx, oracle_mod, 8, calls, batch)
    i = 3 if remembered else 2
    # the scenario does reach both answers of the reference (checked on the oracle's own output)
    if remembered:
        assert _has_ref(want[i + 1]) and not _has_ref(want[i + 2]), "window answers y after the overwrite"
    else:
        assert not _has_ref(want[i + 1]) and _has_ref(want[i + 2]), "the map answers x at once"
    last_x, last_y = want[-3], want[-2]
    if remembered and evict < 64:
        assert not _has_ref(last_x) and _has_ref(last_y)
    else:
        assert _has_ref(last_x) and not _has_ref(last_y)


def test_duplicate_enter_then_batches_and_lookups(gpu_ctx, oracle_mod):
    """After the duplicate enter: fresh-encoder batches (xc_encode_batch_host) and direct lookups
    (the <ASK> handler's, xcodec_filter.cc:296) see what the reference's cache returns."""
    import wanproxy_amd as w
    x, y = _collision_pair()
    calls = _calls(True, 0)
    want, gc, oc = _run(gpu_ctx, oracle_mod, 8, calls, True)
    h = int(oracle_mod.hash_segment(x))
    assert h == int(oracle_mod.hash_segment(y))
    p = W.pool(POOL)
    bufs = [_cat(x, W.gen(20, 99)), _cat(y, W.gen(21, 77)),
            _cat(*[p[2048 * i:2048 * (i + 1)] for i in range(70)]), _cat(W.gen(22, 33), x), y]
    o = oc.encode_batch(bufs)
    g = w.XCodecEncoder(gc).encode_batch(bufs)
    assert g == o
    # a direct lookup: the window's bytes or the map's (a remember when the map answers)
    assert gc.lookup(h) == oc.lookup(h)
    assert len(gc) == len(oc)
    # device-resident runs on that cache (xc_encode_run, and submit + poll): the library replays
    # them through the recent window's engine into the run's arenas
    for k, use_poll in enumerate((False, True)):
        more = [_cat(W.gen(30 + k, 64), y, x), _cat(x, W.gen(40 + k, 2100)), W.gen(50 + k, 3000)]
        assert _device_run(gc, more, use_poll) == oc.encode_batch(more), use_poll
        assert len(gc) == len(oc)


def _device_run(cache, bufs, use_poll):
    import torch
    import wanproxy_amd as w
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(bufs), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    if use_poll:
        plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        while not plan.poll():
            pass
    else:
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    cache.ctx.sync()
    out, lens = d_out.cpu().numpy(), d_len.cpu().numpy()
    plan.close()
    return [out[int(plan.out_off[i]):int(plan.out_off[i]) + int(lens[i])].tobytes() for i in range(len(bufs))]


def _device_run_streams(cache, bufs, start, cand, flags):
    """A device-resident run with per-buffer stream states (xc_plan_set_streams): the streams, then
    the stream results (xc_plan_stream_results)."""
    import torch
    import wanproxy_amd as w
    from wanproxy_amd.xcodec import _check, load_library
    lib = load_library()
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    _check(lib.xc_plan_set_streams(plan.h, np.asarray(start, np.uint64), np.asarray(cand, np.int64),
                                   np.asarray(flags, np.uint32)))
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(bufs), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    cache.ctx.sync()
    out, lens = d_out.cpu().numpy(), d_len.cpu().numpy()
    rb, rc = np.zeros(len(bufs), np.uint64), np.zeros(len(bufs), np.int64)
    _check(lib.xc_plan_stream_results(plan.h, rb, rc))
    got = [out[int(plan.out_off[i]):int(plan.out_off[i]) + int(lens[i])].tobytes() for i in range(len(bufs))]
    subs = plan.stats().sub_batches  # (0: no device pass ran, the run was replayed)
    plan.close()
    return got, rb.tolist(), rc.tolist(), subs


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_device_replay_matches_the_device_path_with_stream_state(gpu_ctx, monkeypatch, seed):
    """The replay of a device-resident run (xc_runtime.hip replay_device_run) against the device path
    on the same cache state, with per-buffer stream states (resume offset, carried candidate,
    no-flush: xcodec_encoder.cc:60-82,175-201 between calls): the same streams, stream results and
    cache size.  XC_FORCE_REPLAY=1 (tests only) sends the run to the replay."""
    import wanproxy_amd as w
    rng = np.random.default_rng(seed)
    warm = W.pool_warmup_buffers(POOL)
    p = W.pool(POOL)
    bufs, start, cand, flags = [], [], [], []
    for i in range(16):
        segs = [p[2048 * k:2048 * (k + 1)] for k in rng.integers(0, POOL, int(rng.integers(1, 5)))]
        b = np.concatenate([W.gen(100 * seed + i, int(rng.integers(0, 3000)))] + segs +
                           [W.gen(200 * seed + i, int(rng.integers(0, 500)))])
        a = int(rng.integers(0, min(len(b), 6000) + 1))
        c = int(rng.integers(max(0, a - 4095), a - 2048 + 1)) if a >= 2048 and rng.random() < 0.6 else -1
        bufs.append(b)
        start.append(a)
        cand.append(c)
        flags.append(int(rng.random() < 0.5))
    res = []
    for force in ("0", "1"):
        monkeypatch.setenv("XC_FORCE_REPLAY", force)
        gc = w.XCodecCache(gpu_ctx, 1 << 12)
        w.XCodecEncoder(gc).encode_batch(warm)
        got, rb, rc, subs = _device_run_streams(gc, bufs, start, cand, flags)
        assert (subs == 0) == (force == "1"), (force, subs)
        res.append((got, rb, rc, len(gc)))
        gc.close()
    assert any(c >= 0 for c in cand) and any(f for f in flags)
    for i in range(len(bufs)):
        assert res[0][0][i] == res[1][0][i], f"buffer {i}: stream differs"
    assert res[0][1:] == res[1][1:]
