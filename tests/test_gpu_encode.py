"""GPU parity tests: the HIP encode path (through the C ABI) against the oracle.

Bit-exact byte streams are required (integer/byte work)."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


def _esc(n, seed, frac=0.3):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    b[rng.random(n) < frac] = 0xF1
    return b


def _collision_pair(seed=1):
    rng = np.random.default_rng(seed)
    x = (rng.integers(2, 126, 2048, dtype=np.int64) * 2 + 1).astype(np.uint8)
    y = x.copy()
    y[100] += 2; y[101] -= 2; y[1500] -= 2; y[1501] += 2
    return x, y


def _gpu_encode(ctx, bufs, warm=None, cap=1 << 16):
    import wanproxy_amd as w
    cache = w.XCodecCache(ctx, cap)
    enc = w.XCodecEncoder(cache)
    if warm:
        for batch in warm:
            enc.encode_batch(batch)
    return enc.encode_batch(bufs), cache


def _check(ctx, oracle_mod, bufs, warm=None):
    oc = oracle_mod.Cache()
    if warm:
        for batch in warm:
            oc.encode_batch(batch)
    want = oc.encode_batch(bufs)
    got, cache = _gpu_encode(ctx, bufs, warm)
    assert len(got) == len(want)
    for i, (g, e) in enumerate(zip(got, want)):
        if g != e:
            n = min(len(g), len(e))
            d = next((k for k in range(n) if g[k] != e[k]), n)
            pytest.fail(f"buffer {i}: len gpu {len(g)} oracle {len(e)}, first diff at {d}")
    assert len(cache) == len(oc)
    return got


def test_selftest(gpu_ctx):
    gpu_ctx.selftest()


def test_window_hashes(gpu_ctx, oracle_mod):
    import torch
    import wanproxy_amd.xcodec as X
    for d in [W.gen(7, 300_000), _esc(70_000, 3), np.full(10_000, 0xF1, np.uint8)]:
        t = torch.zeros(len(d) + 256, dtype=torch.uint8, device="cuda")
        t[:len(d)] = torch.from_numpy(d)
        out = torch.zeros(len(d), dtype=torch.int64, device="cuda")
        X.window_hashes(gpu_ctx, t.data_ptr(), len(d), out.data_ptr())
        gpu_ctx.sync()
        got = out.cpu().numpy().view(np.uint64)
        assert np.array_equal(got, oracle_mod.window_hashes(d))


def test_segment_hash_kats(gpu_ctx):
    import json
    import os
    import torch
    import wanproxy_amd.xcodec as X
    kats = [int(x, 16) for x in json.load(open(os.path.join(
        os.path.dirname(__file__), "golden", "hash_kats.json")))["kats"]]
    segs = torch.arange(256, dtype=torch.uint8).repeat_interleave(2048).cuda()
    out = torch.zeros(256, dtype=torch.int64, device="cuda")
    X.hash_segments(gpu_ctx, segs.data_ptr(), 256, out.data_ptr())
    gpu_ctx.sync()
    assert out.cpu().numpy().view(np.uint64).tolist() == kats


def test_cache_enter_lookup(gpu_ctx, oracle_mod):
    import wanproxy_amd as w
    c = w.XCodecCache(gpu_ctx, 64)
    seg = W.gen(5, 2048)
    h = oracle_mod.hash_segment(seg)
    assert c.lookup(h) is None
    c.enter(h, seg)
    assert c.lookup(h) == seg.tobytes()
    assert len(c) == 1
    c.snapshot()
    seg2 = W.gen(6, 2048)
    c.enter(oracle_mod.hash_segment(seg2), seg2)
    assert len(c) == 2
    c.restore()
    assert len(c) == 1 and c.lookup(oracle_mod.hash_segment(seg2)) is None
    assert c.lookup(h) == seg.tobytes()


def test_tiny_and_boundaries(gpu_ctx, oracle_mod):
    bufs = [W.gen(5, 0), W.gen(5, 1), W.gen(5, 100), W.gen(6, 2047), W.gen(7, 2048),
            W.gen(8, 2049), W.gen(9, 4095), W.gen(10, 4096), W.gen(11, 4097), W.gen(12, 6143),
            W.gen(13, 8191), W.gen(14, 8192), W.gen(15, 8193), W.gen(16, 12345)]
    _check(gpu_ctx, oracle_mod, bufs)


def test_cfg1_roundtrip_1mib(gpu_ctx, oracle_mod):
    d = W.gen(1, 1 << 20)
    got = _check(gpu_ctx, oracle_mod, [d])
    assert len(got[0]) == 1049600


def test_warm_second_pass_all_refs(gpu_ctx, oracle_mod):
    d = W.gen(1, 1 << 20)
    got = _check(gpu_ctx, oracle_mod, [d], warm=[[d]])
    assert len(got[0]) == 512 * 10


def test_cfg2_random(gpu_ctx, oracle_mod):
    _check(gpu_ctx, oracle_mod, W.random_buffers(64))


def test_cfg3_repeats_warm(gpu_ctx, oracle_mod):
    pool = W.pool(1024)
    warm = [[pool[i:i + 65536] for i in range(0, len(pool), 65536)]]
    bufs = W.repeat_buffers(48, 0x77, np_segments=1024, pool_bytes=pool)
    _check(gpu_ctx, oracle_mod, bufs, warm=warm)


def test_cfg4_variant_90pct(gpu_ctx, oracle_mod):
    pool = W.pool(512)
    warm = [[pool[i:i + 65536] for i in range(0, len(pool), 65536)]]
    bufs = W.repeat_buffers(32, 0x88, repeat_pct=90, np_segments=512, pool_bytes=pool)
    _check(gpu_ctx, oracle_mod, bufs, warm=warm)


@pytest.mark.parametrize("ch", [0, 0xF1, 0x41])
def test_charrun_self_references(gpu_ctx, oracle_mod, ch):
    """Dense self-references (xcodec-encode-decode1 intent): 1 EXTRACT + REFs."""
    bufs = [np.full(512 * 1024, ch, np.uint8), np.full(70000, ch, np.uint8)]
    got = _check(gpu_ctx, oracle_mod, bufs)
    assert len(got[0]) == 4600


def test_escape_heavy(gpu_ctx, oracle_mod):
    _check(gpu_ctx, oracle_mod, [_esc(20000, 5), _esc(70000, 6), _esc(3000, 7, 1.0),
                                 np.full(5000, 0xF1, np.uint8)])


def test_cross_buffer_duplicates(gpu_ctx, oracle_mod):
    """Later buffers reference segments first declared by earlier buffers of the same batch."""
    a = W.gen(21, 65536)
    b = np.concatenate([W.gen(22, 3000), a[:30000], W.gen(23, 5000)])
    c = np.concatenate([a[10000:40000], b[:20000]])
    d = a.copy()
    _check(gpu_ctx, oracle_mod, [a, b, c, d, W.gen(24, 65536), a[::-1].copy()])


def test_shifted_repeats(gpu_ctx, oracle_mod):
    """Repeats at unaligned offsets inside one buffer and across buffers."""
    base = W.gen(31, 20000)
    bufs = []
    for k in range(8):
        parts = [W.gen(100 + k, 777 * k + 5), base[k * 333:k * 333 + 9000], W.gen(200 + k, 1234),
                 base[:7000]]
        bufs.append(np.concatenate(parts))
    _check(gpu_ctx, oracle_mod, bufs)


def test_collisions(gpu_ctx, oracle_mod):
    x, y = _collision_pair()
    bufs = [np.concatenate([W.gen(3, 500), y, W.gen(4, 5000)]),
            np.concatenate([y, x, y, W.gen(5, 3000)])]
    _check(gpu_ctx, oracle_mod, bufs, warm=[[x]])
    _check(gpu_ctx, oracle_mod, [x, np.concatenate([y, W.gen(6, 4000)]), np.concatenate([x, y])])


def test_device_resident_plan_and_restore(gpu_ctx, oracle_mod):
    import torch
    import wanproxy_amd as w
    pool = W.pool(256)
    warm = [pool[i:i + 65536] for i in range(0, len(pool), 65536)]
    bufs = W.repeat_buffers(40, 0x5555, np_segments=256, pool_bytes=pool)
    oc = oracle_mod.Cache()
    oc.encode_batch(warm)
    want = oc.encode_batch(bufs)

    cache = w.XCodecCache(gpu_ctx, 1 << 14)
    w.XCodecEncoder(cache).encode_batch(warm)
    cache.snapshot()
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(bufs), dtype=torch.int64, device="cuda")
    for it in range(3):
        cache.restore()
        d_out.zero_()
        torch.cuda.synchronize()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        gpu_ctx.sync()
        out = d_out.cpu().numpy()
        lens = d_len.cpu().numpy()
        for i in range(len(bufs)):
            o = int(plan.out_off[i])
            assert out[o:o + int(lens[i])].tobytes() == want[i], (it, i)
    st = plan.stats()
    assert st.n_extract + st.n_ref > 0


def test_many_subbatches_async_pipeline(gpu_ctx, oracle_mod, monkeypatch):
    """1 MiB sub-batches: the asynchronous pipeline runs ~10 sub-batches back to back, and the
    gate stops it at every sub-batch that needs the host (a buffer whose lookups hit an earlier
    buffer's new declaration in the same sub-batch, self-referencing char runs, collisions); the
    host then redoes that sub-batch step by step and restarts the pass after it."""
    monkeypatch.setenv("XC_SUB_MB", "1")
    bufs, warm = _mixed_batch()
    _check(gpu_ctx, oracle_mod, bufs, warm=warm)


@pytest.mark.parametrize("blocks", ["1", "3", "8"])
def test_scan_chunk_lengths(gpu_ctx, oracle_mod, monkeypatch, blocks):
    """The scan's chunk length and work unit are chosen per plan from the batch size (2 KiB
    chunks for a few buffers, 16 KiB for big batches); forced here, the bytes do not change."""
    monkeypatch.setenv("XC_CHUNK_BLOCKS", blocks)
    bufs, warm = _mixed_batch()
    _check(gpu_ctx, oracle_mod, bufs, warm=warm)
    _check(gpu_ctx, oracle_mod, W.random_buffers(24) + [W.gen(9, 1 << 20), W.gen(5, 2049)])


def _mixed_batch():
    x, y = _collision_pair(7)
    a = W.gen(51, 65536)
    pool = W.pool(64)
    bufs = []
    for k in range(40):
        kind = k % 8
        if kind == 0:
            bufs.append(W.gen(300 + k, 60000 + 1111 * k))
        elif kind == 1:
            bufs.append(np.concatenate([W.gen(400 + k, 999), a[k * 100:k * 100 + 30000]]))
        elif kind == 2:
            bufs.append(np.full(50000 + k, k & 0xFF, np.uint8))
        elif kind == 3:
            bufs.append(np.concatenate([y, W.gen(500 + k, 3000), x]))
        elif kind == 4:
            bufs.append(pool[(k % 16) * 65536:(k % 16) * 65536 + 65536].copy())
        elif kind == 5:
            bufs.append(bufs[-4][5:].copy())  # shifted copy of a recent buffer
        elif kind == 6:
            bufs.append(_esc(40000, k))
        else:
            bufs.append(a.copy())
    return bufs, [[pool[i:i + 65536] for i in range(0, 8 * 65536, 65536)]]


def test_ref_shadow_misses(gpu_ctx, oracle_mod, monkeypatch):
    """REF shadows: the scan skips the windows after a predicted REF (an aligned block found in
    the cache) and the walk verifies that the REF was emitted.  Here predicted REFs do not
    happen: an unaligned REF just before resets the hash past the aligned position, or the
    cached block is a hash collision, so the gate must stop the asynchronous pass and the
    sub-batch must be redone scanning every position."""
    monkeypatch.setenv("XC_SUB_MB", "1")
    a = W.gen(61, 2048)
    x = np.concatenate([W.gen(62, 100), a, W.gen(63, 65536 - 2148)])      # REF at 2147 hides 4095
    cx, cy = _collision_pair(11)
    y = np.concatenate([W.gen(64, 4096), cy, W.gen(65, 20000)])           # block 2 collides
    z = np.concatenate([W.gen(66, 6144), a, W.gen(67, 9000)])             # a clean aligned REF
    pool = W.pool(16)
    warm = [[a, x[2048:4096].copy(), cx], [pool[i:i + 65536] for i in range(0, 8 * 65536, 65536)]]
    bufs = []
    for k in range(24):
        bufs.append([x, y, z, pool[(k % 8) * 65536:(k % 8) * 65536 + 65536].copy()][k % 4])
    _check(gpu_ctx, oracle_mod, bufs, warm=warm)
    # the same batch as a device-resident plan: every sub-batch with x or y is handed back
    st = _plan_run(gpu_ctx, oracle_mod, bufs, warm)
    assert st.shadow_misses >= 1 and st.redone >= st.shadow_misses, (st.redone, st.shadow_misses)
    st = _plan_run(gpu_ctx, oracle_mod, [z, z[::-1].copy()] * 4, warm)
    assert st.shadow_misses == 0


def _plan_run(ctx, oracle_mod, bufs, warm):
    import torch
    import wanproxy_amd as w
    oc = oracle_mod.Cache()
    for batch in warm:
        oc.encode_batch(batch)
    want = oc.encode_batch(bufs)
    cache = w.XCodecCache(ctx, 1 << 14)
    for batch in warm:
        w.XCodecEncoder(cache).encode_batch(batch)
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(bufs), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    ctx.sync()
    out, lens = d_out.cpu().numpy(), d_len.cpu().numpy()
    for i in range(len(bufs)):
        o = int(plan.out_off[i])
        assert out[o:o + int(lens[i])].tobytes() == want[i], i
    return plan.stats()


def _host_path(ctx, oracle_mod, bufs, warm, cap=None, sub_bytes=0):
    import wanproxy_amd as w
    oc = oracle_mod.Cache()
    for batch in warm:
        oc.encode_batch(batch)
    want = oc.encode_batch(bufs)
    cache = w.XCodecCache(ctx, 1 << 15)
    for batch in warm:
        w.XCodecEncoder(cache).encode_batch(batch)
    plan = w.EncodePlan(cache, [len(b) for b in bufs], sub_bytes=sub_bytes)
    h_in = w.HostBuffer(ctx, plan.in_bytes)
    for i, b in enumerate(bufs):
        h_in.array[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    h_out = w.HostBuffer(ctx, cap if cap is not None else sum(2 * len(b) + 16 for b in bufs))
    lens, pos = plan.run_host(h_in, h_out)
    assert int(pos[0]) == 0
    for i in range(len(bufs)):
        if i:
            assert int(pos[i]) == int(pos[i - 1]) + int(lens[i - 1])
        got = h_out.array[int(pos[i]):int(pos[i]) + int(lens[i])].tobytes()
        assert got == want[i], i
    return plan.stats()


def test_host_path_packed(gpu_ctx, oracle_mod, monkeypatch):
    """xc_encode_run_host: per-sub-batch H2D on a copy stream, encoded streams packed into pinned
    host memory by the packing kernels; with 1 MiB sub-batches, some redone by the host (shadow
    misses, cross-buffer declarations), which must be packed in order too."""
    monkeypatch.setenv("XC_SUB_MB", "1")
    pool = W.pool(16)
    a = W.gen(61, 2048)
    x = np.concatenate([W.gen(62, 100), a, W.gen(63, 65536 - 2148)])
    c = W.gen(70, 40000)
    warm = [[a, x[2048:4096].copy()], [pool[i:i + 65536] for i in range(0, 8 * 65536, 65536)]]
    bufs = []
    for k in range(30):
        bufs.append([x, c, np.concatenate([W.gen(80 + k, 3000), c[:20000]]), _esc(30000, k),
                     pool[(k % 8) * 65536:(k % 8) * 65536 + 65536].copy(), W.gen(90 + k, 777)][k % 6])
    st = _host_path(gpu_ctx, oracle_mod, bufs, warm)
    assert st.redone >= 1
    _host_path(gpu_ctx, oracle_mod, [W.gen(5, 65536) for _ in range(4)], [])


def test_plan_sub_batch_bound(gpu_ctx, oracle_mod):
    """xc_encode_plan_create_sub: a plan's sub-batch bound (the host path's 256 MiB, here 1 and 3 MiB
    over a 6 MiB batch: several sub-batches, their copies and packing pipelined) gives the same
    streams as the oracle; a bound below one buffer's 1 MiB is refused."""
    import wanproxy_amd as w
    pool = W.pool(24 * 32)  # (24 x 64 KiB)
    warm = [[pool[i:i + 65536] for i in range(0, 16 * 65536, 65536)]]
    bufs = [pool[(k % 24) * 65536:(k % 24) * 65536 + 65536].copy() if k % 3 else W.gen(300 + k, 65536)
            for k in range(96)]
    for mb in (1, 3):
        st = _host_path(gpu_ctx, oracle_mod, bufs, warm, sub_bytes=mb << 20)
        assert st.sub_batches >= 6 // mb, (mb, st.sub_batches)
    cache = w.XCodecCache(gpu_ctx, 1 << 12)
    with pytest.raises(w.XCodecError):
        w.EncodePlan(cache, [65536] * 4, sub_bytes=(1 << 20) - 1)


def test_host_path_capacity(gpu_ctx, oracle_mod):
    import wanproxy_amd as w
    with pytest.raises(w.XCodecError):
        _host_path(gpu_ctx, oracle_mod, [W.gen(9, 65536)], [], cap=1000)


def test_input_written_on_context_stream(gpu_ctx, oracle_mod):
    """xc_encode_run is ordered after the context stream (xcodec_hip.h): an input arena filled by
    an asynchronous copy enqueued on xc_ctx_stream just before restore_async + run is the input
    that gets encoded — block hashing on the side stream included."""
    import torch
    import wanproxy_amd as w
    n = 256
    warm = W.pool_warmup_buffers()
    cache = w.XCodecCache(gpu_ctx, W.POOL_SEGMENTS + n * 33 + 1024)
    w.XCodecEncoder(cache).encode_batch(warm)
    cache.snapshot()
    plan = w.EncodePlan(cache, np.full(n, W.BUF, np.uint64))
    d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
    for seed in (0x5555, 0x77):
        bufs = W.repeat_shard(n, seed)
        src = torch.from_numpy(bufs.reshape(-1)).cuda()
        torch.cuda.synchronize()
        with torch.cuda.stream(torch.cuda.ExternalStream(gpu_ctx.stream)):
            d_in.zero_()  # a kernel ahead of the copy: the copy lands late
            d_in[:n * W.BUF].copy_(src, non_blocking=True)
        cache.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        torch.cuda.synchronize()
        ref = oracle_mod.Cache()
        ref.encode_batch(warm)
        want = ref.encode_batch([bufs[i] for i in range(n)])
        lens = d_len.cpu().numpy()
        out = d_out.cpu().numpy()
        for i in range(n):
            o = int(plan.out_off[i])
            assert out[o:o + int(lens[i])].tobytes() == want[i], (seed, i)


@pytest.mark.parametrize("graph", ["1", "0"])
def test_graph_replay_and_recapture(gpu_ctx, oracle_mod, monkeypatch, graph):
    """With XC_GRAPH=1, xc_encode_run replays the asynchronous pass of a single-sub-batch plan as a
    HIP graph captured on the first run with the given arenas; a run with other arenas captures
    again, and a sub-batch the gate hands back to the host (cross-buffer duplicates, self
    references) still takes the step-by-step path after the graph.  Every run equals the oracle;
    the default (direct enqueue) gives the same bytes."""
    import torch
    import wanproxy_amd as w
    monkeypatch.setenv("XC_SUB_MB", "64")  # one sub-batch: the graph path
    monkeypatch.setenv("XC_GRAPH", graph)
    bufs, warm = _mixed_batch()
    oc = oracle_mod.Cache()
    for batch in warm:
        oc.encode_batch(batch)
    want = oc.encode_batch(bufs)
    cache = w.XCodecCache(gpu_ctx, 1 << 14)
    for batch in warm:
        w.XCodecEncoder(cache).encode_batch(batch)
    cache.snapshot()
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    outs = [torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_len = torch.zeros(len(bufs), dtype=torch.int64, device="cuda")
    stats = []
    for it in range(5):
        d_out = outs[it % 2] if it < 4 else outs[0]
        d_out.zero_()
        torch.cuda.synchronize()
        cache.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        torch.cuda.synchronize()
        out, lens = d_out.cpu().numpy(), d_len.cpu().numpy()
        for i in range(len(bufs)):
            o = int(plan.out_off[i])
            assert out[o:o + int(lens[i])].tobytes() == want[i], (it, i)
        st = plan.stats()
        stats.append((st.sub_batches, st.redone, st.n_extract, st.n_ref))
    assert len(set(stats)) == 1 and stats[0][1] > 0, stats  # same pass every run, some redone


@pytest.mark.parametrize("sub_mb", ["64", "1"])
def test_submit_poll_wait(gpu_ctx, oracle_mod, monkeypatch, sub_mb):
    """xc_encode_submit returns before the device has finished; xc_encode_poll reports the run
    unfinished without blocking, then finishes it (including the sub-batches the gate hands back
    to the host: cross-buffer duplicates, self references); xc_encode_wait does the same blocking.
    A second submit while a run is in flight fails with XC_EBUSY, a poll with no run in flight
    fails.  One sub-batch (the graph path) and many.  Every run equals the oracle."""
    import time
    import torch
    import wanproxy_amd as w
    monkeypatch.setenv("XC_SUB_MB", sub_mb)
    bufs, warm = _mixed_batch()
    oc = oracle_mod.Cache()
    for batch in warm:
        oc.encode_batch(batch)
    want = oc.encode_batch(bufs)
    cache = w.XCodecCache(gpu_ctx, 1 << 14)
    for batch in warm:
        w.XCodecEncoder(cache).encode_batch(batch)
    cache.snapshot()
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(bufs), dtype=torch.int64, device="cuda")
    with pytest.raises(w.XCodecError):
        plan.poll()  # nothing in flight
    stats = []
    for it in range(4):
        d_out.zero_()
        torch.cuda.synchronize()
        cache.restore_async()
        plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        if it == 0:
            with pytest.raises(w.XCodecError):
                plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        if it % 2:
            plan.wait()
        else:
            t0 = time.time()
            while not plan.poll():
                assert time.time() - t0 < 60
        torch.cuda.synchronize()
        out, lens = d_out.cpu().numpy(), d_len.cpu().numpy()
        for i in range(len(bufs)):
            o = int(plan.out_off[i])
            assert out[o:o + int(lens[i])].tobytes() == want[i], (it, i)
        st = plan.stats()
        stats.append((st.sub_batches, st.redone, st.n_extract, st.n_ref))
    assert len(set(stats)) == 1 and stats[0][1] > 0, stats


@pytest.mark.parametrize("sub_mb", ["64", "1"])
@pytest.mark.parametrize("mixed", [False, True])
def test_stream_ordered_completion(gpu_ctx, oracle_mod, monkeypatch, mixed, sub_mb):
    """xc_plan_set_completion(XC_COMPLETE_STREAM): runs return once decided (the graph's emit
    has published the control words) and the rest completes in context-stream order, so
    back-to-back restore + run calls with no host synchronisation in between (run, submit + wait,
    submit + poll) each produce the oracle's bytes; a batch whose sub-batch the gate hands back to
    the host (mixed: cross-buffer duplicates, self references) and one that never does; one
    sub-batch (the graph) and many (published by the last k_alloc, aborts by any gate)."""
    import time
    import torch
    import wanproxy_amd as w
    from wanproxy_amd import workloads as W
    monkeypatch.setenv("XC_SUB_MB", sub_mb)  # 64: one sub-batch (the graph path)
    if mixed:
        bufs, warm = _mixed_batch()
    else:
        bufs, warm = list(W.repeat_shard(96, 0x77)), [W.pool_warmup_buffers()]
    oc = oracle_mod.Cache()
    for batch in warm:
        oc.encode_batch(batch)
    want = oc.encode_batch(bufs)
    cache = w.XCodecCache(gpu_ctx, 1 << 15)
    for batch in warm:
        w.XCodecEncoder(cache).encode_batch(batch)
    cache.snapshot()
    plan = w.EncodePlan(cache, [len(b) for b in bufs])
    plan.set_completion(True)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
    d_in = torch.from_numpy(arena).cuda()
    outs = [torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda") for _ in range(3)]
    lens = [torch.zeros(len(bufs), dtype=torch.int64, device="cuda") for _ in range(3)]
    torch.cuda.synchronize()
    stats = []
    for it in range(9):
        d_out, d_len = outs[it % 3], lens[it % 3]
        cache.restore_async()
        if it % 3 == 0:
            plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        else:
            plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
            if it % 3 == 1:
                plan.wait()
            else:
                t0 = time.time()
                while not plan.poll():
                    assert time.time() - t0 < 60
        st = plan.stats()
        stats.append((st.sub_batches, st.redone, st.n_extract, st.n_ref))
    gpu_ctx.sync()
    torch.cuda.synchronize()
    for k in range(3):
        out, ln = outs[k].cpu().numpy(), lens[k].cpu().numpy()
        for i in range(len(bufs)):
            o = int(plan.out_off[i])
            assert out[o:o + int(ln[i])].tobytes() == want[i], (k, i)
    assert len(set(stats)) == 1 and (stats[0][1] > 0) == mixed, stats
    plan.set_completion(False)
    plan.close()
    cache.close()


def test_cache_grows_like_the_reference_map(gpu_ctx, oracle_mod):
    """The reference's memory cache never fills (xcodec/xcodec_cache.h:164,182-188).  A device
    cache created for 1024 segments takes ten times that through several batches, a snapshot taken
    before it grew still restores, and every output equals the oracle's."""
    import wanproxy_amd as w
    cache = w.XCodecCache(gpu_ctx, 1024)
    oc = oracle_mod.Cache()
    enc = w.XCodecEncoder(cache)
    first = W.random_buffers(16, seed0=0x9000)           # 512 segments
    assert enc.encode_batch(first) == oc.encode_batch(first)
    cache.snapshot()
    snap_oracle = oc.clone()
    for k in range(4):                                     # 4 x 2560 = 10240 more segments
        bufs = W.random_buffers(80, seed0=0xA000 + 100 * k)
        assert enc.encode_batch(bufs) == oc.encode_batch(bufs), k
    assert len(cache) == len(oc) == 512 + 10240
    assert cache.capacity >= len(cache) > 1024
    # the pre-growth snapshot: the grown cache returns to it exactly
    cache.restore()
    assert len(cache) == 512
    again = W.random_buffers(8, seed0=0xA000) + first[:4]
    assert enc.encode_batch(again) == snap_oracle.encode_batch(again)
    # enter() and the decoder grow a cache too
    small = w.XCodecCache(gpu_ctx, 4)
    for i in range(12):
        seg = W.gen(700 + i, 2048)
        small.enter(oracle_mod.hash_segment(seg), seg)
    assert len(small) == 12 and small.lookup(oracle_mod.hash_segment(W.gen(705, 2048))) == W.gen(705, 2048).tobytes()
    streams = oracle_mod.Cache().encode_batch(W.random_buffers(40, seed0=0xB000))
    dc = w.XCodecCache(gpu_ctx, 16)
    got = w.XCodecDecoder(dc).decode_batch(streams)
    want = oracle_mod.Cache().decode_batch(streams)
    assert got == want and len(dc) == 40 * 32


@pytest.mark.parametrize("blocks", ["1", "2", "8"])
def test_block_walk_falls_back_on_any_event(gpu_ctx, oracle_mod, monkeypatch, blocks):
    """The block-parallel walk applies only when no event between aligned windows decides
    anything; an unaligned hit behind an aligned REF of the same chunk (a later lane of the chunk's
    event list) must send the buffer to the sequential walk."""
    monkeypatch.setenv("XC_CHUNK_BLOCKS", blocks)
    pool = W.pool(64)
    blk = lambda i: pool[(i % 64) * 2048:(i % 64) * 2048 + 2048]
    bufs = []
    for j in range(32):
        parts = []
        for k in range(6):
            parts.append(blk(j + k))                           # aligned: a cached block (REF)
            parts.append(W.gen(7000 + 16 * j + k, 37 + 211 * ((j + k) % 9)))  # shifts the next copy
        bufs.append(np.concatenate(parts))
    _check(gpu_ctx, oracle_mod, bufs, warm=[[pool[i:i + 65536] for i in range(0, len(pool), 65536)]])


@pytest.mark.parametrize("n,long_buf,scan", [(1024, False, "exact"), (1100, False, "exact"), (1024, False, "anchor"),
                                             (1100, True, "exact"), (1100, True, "anchor")])
def test_emit_forms(gpu_ctx, oracle_mod, monkeypatch, n, long_buf, scan):
    """The emit's forms for sub-batches of >= 1024 buffers (4 waves per buffer): one pass (k_emit1,
    every buffer <= 64 tokens per wave) with the slots inside it (exactly 1024 buffers) or from k_alloc,
    with the cache enters with or without the anchor index; and the two-pass k_emit once one buffer can
    hold more tokens (300 KiB).  Pool repeats, fresh bytes, escape-heavy literals, shifted repeats of
    earlier buffers: every buffer against the oracle."""
    monkeypatch.setenv("XC_SCAN", scan)
    pool = W.pool(512)
    warm = [[pool[i:i + 65536] for i in range(0, len(pool), 65536)]]
    base = W.repeat_buffers(n, 0x7100 + n + long_buf, np_segments=512, pool_bytes=pool)
    bufs = []
    for i in range(n):
        b = base[i][:16384].copy()
        if i % 7 == 3:
            b = _esc(9000 + i, 0x7200 + i)
        elif i % 11 == 5 and i > 20:
            b = np.concatenate([W.gen(0x7300 + i, 1 + i % 2047), bufs[i - 13][:12000]])
        bufs.append(b)
    if long_buf:
        bufs[n // 2] = np.concatenate([pool[:150000], W.gen(0x7400, 150000), _esc(7000, 0x7401)])
    st = _plan_run(gpu_ctx, oracle_mod, bufs, warm)
    assert st.sub_batches == 1, st.sub_batches
    assert (st.anchor_scans > 0) == (scan == "anchor"), st.anchor_scans
