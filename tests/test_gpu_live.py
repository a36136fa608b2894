"""Back-to-back device-resident runs on a live cache (no restore in between), as a proxy runs.

The reference remembers every map hit in the recent window inside lookup()
(xcodec/xcodec_cache.h:130-147,190-210).  The device cache keeps no window: each run's lookup hits
are packed behind it on the device, copied to pinned memory beside the next run and replayed into
the host window model while the next run works, or before the next operation whose answer depends
on the window.  These tests check that the replayed window is the reference's:
runs back to back through submit / wait (the replay of run k happens inside run k+1's wait), then a
duplicate enter whose answers depend on what the window holds after them, every byte against the
stateful oracle (oracle/xc_oracle.c)."""
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


class Runner:
    """One EncodePlan per batch shape, device arenas kept; run() = submit + wait of one batch."""

    def __init__(self, cache, stream_ordered=True, input_ready=False):
        self.cache = cache
        self.plans = {}
        self.stream_ordered = stream_ordered
        self.input_ready = input_ready

    def run(self, bufs, stats=False):
        import torch
        import wanproxy_amd as w
        key = tuple(len(b) for b in bufs)
        if key not in self.plans:
            plan = w.EncodePlan(self.cache, list(key))
            plan.set_completion(self.stream_ordered)
            plan.set_input_ready(self.input_ready)
            d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
            d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
            d_len = torch.zeros(max(len(bufs), 1), dtype=torch.int64, device="cuda")
            self.plans[key] = (plan, d_in, d_out, d_len)
        plan, d_in, d_out, d_len = self.plans[key]
        arena = np.zeros(plan.in_bytes, np.uint8)
        for i, b in enumerate(bufs):
            arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
        torch.cuda.synchronize()  # (the previous run's device work reads d_in: stream-ordered completion)
        d_in.copy_(torch.from_numpy(arena))
        torch.cuda.synchronize()  # (the input is complete before the submit: input_ready)
        plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        plan.wait()
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        lens = d_len.cpu().numpy()
        got = [out[int(plan.out_off[i]):int(plan.out_off[i]) + int(lens[i])].tobytes() for i in range(len(bufs))]
        return (got, plan.stats()) if stats else got

    def close(self):
        for plan, *_ in self.plans.values():
            plan.close()


def _same(got, want, what):
    bad = [i for i, (g, e) in enumerate(zip(got, want)) if g != e]
    assert len(got) == len(want) and not bad, f"{what}: buffers {bad[:8]} differ from the oracle"


def test_back_to_back_runs_equal_the_oracle(gpu_ctx, oracle_mod, monkeypatch):
    """Six runs on one live cache with fresh seeds (pool repeats, new content, repeats of earlier
    runs' content), two shapes alternating, several sub-batches each: every buffer equals the
    sequential oracle's, and every run's lookup hits were replayed (the window's record)."""
    import wanproxy_amd as w
    monkeypatch.setenv("XC_SUB_MB", "2")
    pool = W.pool(512)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    cache = w.XCodecCache(gpu_ctx, 1 << 14)
    oc = oracle_mod.Cache()
    _same(w.XCodecEncoder(cache).encode_batch(warm), oc.encode_batch(warm), "warm-up")
    r = Runner(cache)
    prev = []
    before = cache.hit_stats()
    for k in range(6):
        bufs = W.repeat_buffers(96 if k % 2 == 0 else 64, 0x6100 + k, np_segments=512, pool_bytes=pool)
        if prev:  # content of the run before, shifted
            bufs[3] = _cat(W.gen(0x6200 + k, 777), prev[5][:40000])
        _same(r.run(bufs), oc.encode_batch(bufs), f"run {k}")
        prev = bufs
    cache.settle()
    st = cache.hit_stats()
    assert st["runs"] - before["runs"] >= 6 and st["hits"] > before["hits"], st
    assert len(cache) == len(oc)
    r.close()


@pytest.mark.parametrize("evict", [0, 40, 70])
def test_window_after_back_to_back_runs(gpu_ctx, oracle_mod, evict):
    """Connection 0 carries candidate x; connection 1 enters the twin y (same hash, other bytes);
    device-resident run A REFs y (the window remembers y), run B REFs `evict` distinct pool segments
    (64 push y out), run C is fresh data; then connection 0 declares x (a duplicate enter: the map
    answers x, the window y while it holds it, xcodec_cache.h:137-147,182-188).  Fresh encoders and
    a direct lookup afterwards see what the reference's cache returns, which depends on the window
    the replayed hits of A, B and C built."""
    import wanproxy_amd as w
    x, y = _collision_pair()
    p = W.pool(POOL)
    warm = W.pool_warmup_buffers(POOL)
    oc = oracle_mod.Cache()
    gc = w.XCodecCache(gpu_ctx, 1 << 12)
    oc.encode_batch(warm)
    w.XCodecEncoder(gc).encode_batch(warm)
    o0, g0 = oracle_mod.Encoder(oc), w.XCodecStreamEncoder(gc)
    o1, g1 = oracle_mod.Encoder(oc), w.XCodecStreamEncoder(gc)
    a = _cat(x, W.gen(11, 100))
    assert g0.encode(a) == o0.encode(a)           # candidate x, looked up (a miss), carried
    assert g1.encode(y) == o1.encode(y)
    assert g1.flush() == o1.flush()               # y declared: the hash is in the map
    r = Runner(gc)
    runs = [[_cat(y, W.gen(12, 50)), W.gen(15, 30000)],                                # A: REF y
            [_cat(*[p[2048 * i:2048 * (i + 1)] for i in range(evict)]) if evict else W.gen(16, 4096),
             W.gen(17, 20000)],                                                        # B
            [W.gen(18, 65536), W.gen(19, 9000)]]                                       # C
    for k, bufs in enumerate(runs):
        _same(r.run(bufs), oc.encode_batch(bufs), f"run {'ABC'[k]}")
    d = W.gen(13, 4096)
    assert g0.encode(d) == o0.encode(d)           # x declared: the duplicate enter
    assert g0.flush() == o0.flush()
    h = int(oracle_mod.hash_segment(x))
    bufs = [_cat(x, W.gen(20, 99)), _cat(y, W.gen(21, 77)), _cat(W.gen(22, 33), x), y]
    want = oc.encode_batch(bufs)
    assert w.XCodecEncoder(gc).encode_batch(bufs) == want
    # the scenario reaches both answers: y from the window while it holds it, x from the map after
    has_ref = [b"\xf1\x02" in s for s in want]
    assert has_ref[1] == (evict < 64) and has_ref[0] == (evict >= 64), has_ref
    assert gc.lookup(h) == oc.lookup(h)
    assert len(gc) == len(oc)
    r.close()


def test_first_sub_batch_hashed_ahead(gpu_ctx, oracle_mod, monkeypatch):
    """xc_plan_set_input_ready: a plan's next run hashes its first sub-batch on the side stream at the
    submit, beside the previous run's last kernels, its compares taking only the entries complete
    then; the later sub-batches' hashing then starts on the side stream right after sub-batch 0's
    set clear, beside sub-batch 0's predictions (xc_runtime.hip launch_first_round: every run here
    has >= 3 sub-batches).  Runs of one plan back to back (some anchor-scanned), a restore in between (the bench's
    step), another plan's run and a host enter in between (which write the cache: no early hashing
    for the next run): every buffer equals the oracle's."""
    import wanproxy_amd as w
    monkeypatch.setenv("XC_SUB_MB", "2")
    pool = W.pool(512)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    cache = w.XCodecCache(gpu_ctx, 1 << 14)
    oc = oracle_mod.Cache()
    _same(w.XCodecEncoder(cache).encode_batch(warm), oc.encode_batch(warm), "warm-up")
    cache.snapshot()
    snap = oc.clone()
    r = Runner(cache, input_ready=True)
    early, redone = [], []
    for k in range(9):
        if k == 3:  # the bench's step: back to the snapshot
            cache.restore()
            oc = snap.clone()
        if k == 5:  # another plan's run writes the cache
            other = [W.gen(0x6400, 70000), np.concatenate([pool[:30000], W.gen(0x6401, 9000)])]
            _same(w.XCodecEncoder(cache).encode_batch(other), oc.encode_batch(other), "other plan")
        if k == 7:  # a host enter
            seg = W.gen(0x6402, 2048)
            cache.enter(oracle_mod.hash_segment(seg), seg)
            oc.enter(oracle_mod.hash_segment(seg), seg)
        bufs = W.repeat_buffers(96, 0x6300 + k, np_segments=512, pool_bytes=pool)
        monkeypatch.setenv("XC_SCAN", "anchor" if k % 2 else "auto")
        if k % 2:  # repeats of the previous run's content at shifted offsets (the same lengths: one plan)
            bufs[7] = _cat(W.gen(0x6310 + k, 1234), prev[11][:65536 - 1234])
            bufs[8] = prev[12].copy()
        got, st = r.run(bufs, stats=True)
        _same(got, oc.encode_batch(bufs), f"run {k}")
        assert st.sub_batches >= 3, st.sub_batches
        early.append(int(st.early_hashed))
        redone.append(int(st.redone))
        prev = bufs
    # every run after one of this plan hashes ahead, except after another plan's run or an enter, or
    # after a run whose asynchronous pass handed a sub-batch back to the host (the shifted repeats can)
    want = [int(k > 0 and k not in (5, 7) and not redone[k - 1]) for k in range(9)]
    assert early == want, (early, redone)
    assert sum(early) >= 4, (early, redone)
    assert len(cache) == len(oc)
    r.close()


def test_two_caches_replay_from_two_threads(gpu_ctx, oracle_mod):
    """Two caches (two contexts) driven from two host threads at once, as two proxies' event threads
    would (include/xcodec_hip.h: one context per thread): both replay their runs' lookup hits into
    their recent windows through the process's one helper pool (runs of >= 1024 buffers use it).  One
    run at a time owns the helpers, the other replays on its own thread; neither waits forever, and
    every buffer of both equals the oracle's."""
    import threading
    import wanproxy_amd as w
    pool = W.pool(256)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    res = {}

    def drive(k):
        try:
            ctx = w.Context(0)
            cache = w.XCodecCache(ctx, 1 << 14)
            oc = oracle_mod.Cache()
            w.XCodecEncoder(cache).encode_batch(warm)
            oc.encode_batch(warm)
            r = Runner(cache)
            before = cache.hit_stats()
            for run in range(3):
                bufs = W.repeat_buffers(1100, 0x6500 + 16 * k + run, slots=4, np_segments=256, pool_bytes=pool)
                _same(r.run(bufs), oc.encode_batch(bufs), f"thread {k} run {run}")
            cache.settle()
            st = cache.hit_stats()
            assert st["runs"] - before["runs"] >= 3 and st["hits"] > before["hits"], st
            assert len(cache) == len(oc)
            r.close()
            res[k] = "ok"
        except BaseException as e:  # noqa: BLE001 (reported below)
            res[k] = repr(e)

    ts = [threading.Thread(target=drive, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(240)
    assert not any(t.is_alive() for t in ts), "a replay did not finish"
    assert res == {0: "ok", 1: "ok"}, res


def test_quiesced_run_status_is_not_dropped(gpu_ctx, oracle_mod):
    """A run finished by another caller (xc_cache_quiesce, the facade's answer to XC_EBUSY) parks its
    status for its submitter: a new submit on that plan fails with XC_EBUSY until the submitter's
    poll / wait took the status; then runs go on, every buffer equal to the oracle's."""
    import torch
    import wanproxy_amd as w
    pool = W.pool(128)
    cache = w.XCodecCache(gpu_ctx, 1 << 12)
    oc = oracle_mod.Cache()
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    w.XCodecEncoder(cache).encode_batch(warm)
    oc.encode_batch(warm)
    bufs = W.repeat_buffers(24, 0x6600, np_segments=128, pool_bytes=pool)
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(bufs), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def outputs():
        torch.cuda.synchronize()
        out, lens = d_out.cpu().numpy(), d_len.cpu().numpy()
        return [out[int(plan.out_off[i]):int(plan.out_off[i]) + int(lens[i])].tobytes() for i in range(len(bufs))]

    plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    cache.quiesce()                                    # another caller finishes the run
    with pytest.raises(w.XCodecError, match="-16"):    # the status is parked: no new run yet
        plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    assert plan.poll()                                 # the submitter takes it
    _same(outputs(), oc.encode_batch(bufs), "quiesced run")
    plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    plan.wait()
    _same(outputs(), oc.encode_batch(bufs), "next run")
    plan.close()


def test_pipelined_stream_ordered_runs_over_distinct_inputs(gpu_ctx, oracle_mod, monkeypatch):
    """The bench's pattern with distinct inputs: one plan, input ready at submit, stream-ordered
    completion, runs submitted back to back with no device synchronisation in between, so that run
    k + 1's early block hashing (every sub-batch, side stream) is enqueued while run k's last
    sub-batch still emits.  Sub-batches >= 1 of run k + 1 wait for run k's last emit (it
    reads the same block arrays).  Every buffer of every run equals the sequential oracle's."""
    import torch
    import wanproxy_amd as w
    monkeypatch.setenv("XC_SUB_MB", "2")
    pool = W.pool(512)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    cache = w.XCodecCache(gpu_ctx, 1 << 15)
    oc = oracle_mod.Cache()
    _same(w.XCodecEncoder(cache).encode_batch(warm), oc.encode_batch(warm), "warm-up")
    n, runs = 96, 8
    plan = w.EncodePlan(cache, [65536] * n)
    plan.set_completion(True)
    plan.set_input_ready(True)
    batches, d_in, d_out, d_len = [], [], [], []
    for k in range(runs):
        bufs = W.repeat_buffers(n, 0x6500 + k, np_segments=512, pool_bytes=pool)
        if k:  # content of the run before at shifted offsets: same shapes, other bytes
            bufs[40] = _cat(W.gen(0x6600 + k, 999), batches[-1][41][:65536 - 999])
        batches.append(bufs)
        arena = np.zeros(plan.in_bytes, np.uint8)
        for i, b in enumerate(bufs):
            arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
        d_in.append(torch.from_numpy(arena).cuda())
        d_out.append(torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda"))
        d_len.append(torch.zeros(n, dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    early = []
    for k in range(runs):
        plan.submit(d_in[k].data_ptr(), d_out[k].data_ptr(), d_len[k].data_ptr())
        plan.wait()
        st = plan.stats()
        early.append(int(st.early_hashed))
        assert st.sub_batches >= 3, st.sub_batches
    gpu_ctx.sync()
    torch.cuda.synchronize()
    for k in range(runs):
        out = d_out[k].cpu().numpy()
        lens = d_len[k].cpu().numpy()
        got = [out[int(plan.out_off[i]):int(plan.out_off[i]) + int(lens[i])].tobytes() for i in range(n)]
        _same(got, oc.encode_batch(batches[k]), f"run {k}")
    assert sum(early) >= runs // 2, early
    assert len(cache) == len(oc)
    plan.close()
