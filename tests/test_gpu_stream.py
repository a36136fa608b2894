"""GPU parity tests of the stateful stream encoder (xc_encoder_* / xc_encode_streams) against
the oracle's stateful XCodecEncoder restatement: every call's output bytes must equal what the
reference's encode(out, in) [+ flush(out)] appends (xcodec/xcodec_encoder.cc:60-201), with
the calls of many connections batched in order over one cache (xcodec/xcodec_filter.cc:122-164).
"""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


def _esc(n, seed, frac=0.2):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    b[rng.random(n) < frac] = 0xF1
    return b


def _run_both(ctx, oracle_mod, nconn, calls, warm=None, batch=True):
    """calls: list of (connection, data, flush).  Returns the per-call outputs (asserted equal)."""
    import wanproxy_amd as w
    oc = oracle_mod.Cache()
    gc = w.XCodecCache(ctx, 1 << 15)
    if warm is not None:
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
    for i, (g, e) in enumerate(zip(got, want)):
        if g != e:
            n = min(len(g), len(e))
            d = next((j for j in range(n) if g[j] != e[j]), n)
            pytest.fail(f"call {i} (conn {calls[i][0]}): len gpu {len(g)} oracle {len(e)}, first diff at {d}")
    # the state left behind: flushing every connection gives the same tails
    for k in range(nconn):
        assert genc[k].flush() == oenc[k].flush(), f"final flush of conn {k}"
    assert len(gc) == len(oc)
    return got


def _split(data, rng, n):
    cuts = sorted(rng.integers(0, len(data), n))
    return np.split(data, cuts)


def test_single_stream_split_calls(gpu_ctx, oracle_mod):
    pool = W.pool(64)
    rng = np.random.default_rng(7)
    data = np.concatenate([W.gen(11, 9000), pool[2048:30000], W.gen(12, 20000), pool[:8192],
                           _esc(7000, 3)])
    parts = _split(data, rng, 12)
    calls = [(0, p, False) for p in parts] + [(0, b"", True)]
    _run_both(gpu_ctx, oracle_mod, 1, calls, warm=[pool[:65536]])


def test_single_stream_call_by_call(gpu_ctx, oracle_mod):
    """xc_encode / xc_flush one call at a time (no batching)."""
    pool = W.pool(32)
    rng = np.random.default_rng(8)
    data = np.concatenate([W.gen(21, 5000), pool[:16384], W.gen(22, 12000)])
    calls = [(0, p, bool(rng.random() < 0.3)) for p in _split(data, rng, 6)]
    _run_both(gpu_ctx, oracle_mod, 1, calls, warm=[pool[:32768]], batch=False)


def test_interleaved_connections(gpu_ctx, oracle_mod):
    """Many connections, calls interleaved in one batch, random TO_BE_CONTINUED (no flush):
    later calls see earlier calls' declarations, across connections."""
    pool = W.pool(128)
    rng = np.random.default_rng(9)
    streams = []
    for c in range(6):
        segs = []
        for j in range(6):
            r = rng.random()
            if r < 0.4:
                a = int(rng.integers(0, 120)) * 2048
                segs.append(pool[a:a + 2048 * int(rng.integers(1, 4))])
            elif r < 0.6 and c > 0:
                segs.append(streams[c - 1][:int(rng.integers(2048, 9000))])  # another connection's data
            else:
                segs.append(W.gen(100 * c + j, int(rng.integers(100, 9000))))
        streams.append(np.concatenate(segs))
    pieces = [list(_split(s, rng, 4)) for s in streams]
    calls = []
    while any(pieces):
        c = int(rng.integers(0, 6))
        if pieces[c]:
            calls.append((c, pieces[c].pop(0), bool(rng.random() < 0.3)))
    _run_both(gpu_ctx, oracle_mod, 6, calls, warm=[pool[:65536], pool[65536:131072]])


def test_repeated_encoder_in_batch(gpu_ctx, oracle_mod):
    """Consecutive calls of one encoder in a batch run in successive rounds."""
    rng = np.random.default_rng(10)
    data = np.concatenate([W.gen(31, 20000), W.gen(31, 20000)])  # repeats its own new data
    calls = [(0, p, False) for p in _split(data, rng, 5)] + [(1, W.gen(32, 5000), True)] + \
            [(0, W.gen(31, 7000), True)]
    _run_both(gpu_ctx, oracle_mod, 2, calls)


def test_carried_candidate_edges(gpu_ctx, oracle_mod):
    """Calls that end just before / at / after a pending declaration point, a carried candidate
    that a REF in the next call discards, and self-references across calls."""
    pool = W.pool(16)
    a = W.gen(41, 6000)
    calls = [
        (0, a[:2047], False), (0, a[2047:2048], False), (0, a[2048:4095], False),
        (0, a[4095:4096], False), (0, a[4096:], False),
        (0, pool[:2048], False),                       # REF: the carried candidate is dropped
        (0, W.gen(42, 3000), False), (0, a[:4096], False), (0, b"", False), (0, b"", True),
        (0, b"", True),                                # flush with nothing pending
        (1, W.gen(43, 2048), False), (1, b"", True),  # exactly one segment: declared by flush
        (2, W.gen(44, 100), False), (2, W.gen(45, 100), True),
    ]
    _run_both(gpu_ctx, oracle_mod, 3, calls, warm=[pool[:32768]])


def test_escapes_and_collisions_across_calls(gpu_ctx, oracle_mod):
    x = (np.random.default_rng(1).integers(2, 126, 2048, dtype=np.int64) * 2 + 1).astype(np.uint8)
    y = x.copy()
    y[100] += 2; y[101] -= 2; y[1500] -= 2; y[1501] += 2  # same hash, different bytes
    e = _esc(5000, 5, 0.5)
    calls = [(0, x, True), (1, e[:3000], False), (1, y[:1000], False), (1, y[1000:], False),
             (1, e[3000:], False), (1, x, False), (1, b"", True)]
    _run_both(gpu_ctx, oracle_mod, 2, calls)


def test_long_call_is_split(gpu_ctx, oracle_mod):
    """One call longer than a device batch item (1 MiB) is run as consecutive pieces."""
    pool = W.pool(64)
    data = np.concatenate([W.gen(51, 700000), pool[:65536], W.gen(52, 500000)])
    calls = [(0, W.gen(53, 3000), False), (0, data, False), (0, W.gen(54, 100), True)]
    _run_both(gpu_ctx, oracle_mod, 1, calls, warm=[pool[:65536]])


@pytest.mark.parametrize("batch", [True, False])
def test_fresh_calls_without_flush(gpu_ctx, oracle_mod, batch):
    """encode() on a clean encoder, flush() after (the reference filter's consume, xcodec_filter.cc:
    146-157), taken by the block-parallel walk: the last block's candidate stays pending (new last
    block), or the tail after a REF of it does; sub-window and exact-multiple lengths; another
    connection repeating a block still pending in the first (not entered yet: declared again)."""
    pool = W.pool(32)
    a, b = W.gen(61, 10240), W.gen(62, 9000)
    calls = [
        (0, a, False), (0, b"", True),                                   # last block new: pending
        (0, np.concatenate([W.gen(63, 4096), pool[:2048]]), False), (0, b"", True),  # last block REF
        (0, np.concatenate([W.gen(64, 3000), pool[2048:4096], W.gen(65, 500)]), False), (0, b"", True),
        (0, W.gen(66, 1500), False), (0, b"", True),                     # no full window
        (0, W.gen(67, 2048), False), (0, b"", True),                     # exactly one block
        (1, b, False), (2, b[-2048 * 3:], False), (1, b"", True), (2, b"", True),  # pending twice
        (3, np.concatenate([pool[4096:8192], a[:6144]]), False), (3, W.gen(68, 700), True),
    ]
    _run_both(gpu_ctx, oracle_mod, 4, calls, warm=[pool[:32768]], batch=batch)
