"""Randomized parity campaign (GPU): batches assembled from the ingredients the encoder's decisions
depend on -- cached pool segments at aligned and shifted offsets, fresh bytes, F1-heavy literals,
char runs, repeats of earlier pieces of the same batch (cross-buffer and self references), the
constructed hash-collision pair, boundary lengths (0, 1, 2047, 2048, 2049) -- under random scan
chunk lengths, sub-batch sizes (many sub-batches) and with or without REF shadows.  Every encoded
buffer equals the oracle's (xcodec/xcodec_encoder.cc:60-201 restated in oracle/xc_oracle.c) and
the device decoder returns every buffer (xcodec/xcodec_decoder.cc:76-176)."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


def _collision_pair(seed):
    rng = np.random.default_rng(seed)
    x = (rng.integers(2, 126, 2048, dtype=np.int64) * 2 + 1).astype(np.uint8)
    y = x.copy()
    y[100] += 2; y[101] -= 2; y[1500] -= 2; y[1501] += 2
    return x, y


def _batch(rng, pool):
    """Buffers of random pieces, both halves of a collision pair among them (with stateful streams
    the pair reaches the duplicate enter of xcodec_cache.h:182-188, tests/test_gpu_dup.py)."""
    x, y = _collision_pair(int(rng.integers(1 << 30)))
    pieces = []
    bufs = []
    for _ in range(int(rng.integers(8, 48))):
        parts = []
        target = int(rng.choice([0, 1, 2047, 2048, 2049, 5000, 30000, 65536, 140000]))
        n = 0
        while n < target:
            r = rng.random()
            if r < 0.3:   # a pool segment, aligned or shifted by the preceding piece
                k = int(rng.integers(len(pool) // 2048))
                p = pool[k * 2048:(k + 1) * 2048]
            elif r < 0.5:
                p = W.gen(int(rng.integers(1 << 40)), int(rng.integers(1, 6000)))
            elif r < 0.58:
                p = np.full(int(rng.integers(1, 9000)), 0xF1 if rng.random() < 0.5 else int(rng.integers(256)), np.uint8)
            elif r < 0.7 and pieces:
                p = pieces[int(rng.integers(len(pieces)))]  # an earlier piece again
            elif r < 0.76:
                p = x if rng.random() < 0.5 else y
            else:
                b = W.gen(int(rng.integers(1 << 40)), int(rng.integers(1, 3000)))
                b[rng.random(b.size) < 0.2] = 0xF1
                p = b
            parts.append(p)
            pieces.append(p)
            n += p.size
        buf = np.concatenate(parts)[:target] if parts else np.zeros(0, np.uint8)
        bufs.append(np.ascontiguousarray(buf))
    return bufs


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_encode_decode(gpu_ctx, oracle_mod, monkeypatch, seed):
    import wanproxy_amd as w
    rng = np.random.default_rng(1000 + seed)
    monkeypatch.setenv("XC_CHUNK_BLOCKS", str(int(rng.choice([1, 2, 3, 5, 8]))))
    monkeypatch.setenv("XC_SUB_MB", str(int(rng.choice([1, 2, 512]))))
    if rng.random() < 0.3:
        monkeypatch.setenv("XC_NO_SHADOW", "1")
    pool = W.pool(64)
    warm = [pool[i:i + 65536] for i in range(0, int(rng.integers(1, 9)) * 65536, 65536)]
    batches = [_batch(rng, pool) for _ in range(2)]
    oc = oracle_mod.Cache()
    gc = w.XCodecCache(gpu_ctx, int(rng.choice([1024, 1 << 16])))  # (small: the cache grows)
    oc.encode_batch(warm)
    w.XCodecEncoder(gc).encode_batch(warm)
    gd = w.XCodecCache(gpu_ctx, 1 << 12)  # the peer's decoder cache (grows)
    for bufs in batches:
        want = oc.encode_batch(bufs)
        got = w.XCodecEncoder(gc).encode_batch(bufs)
        for i, (g, e) in enumerate(zip(got, want)):
            if g != e:
                n = min(len(g), len(e))
                d = next((k for k in range(n) if g[k] != e[k]), n)
                pytest.fail(f"seed {seed} buffer {i} (len {bufs[i].size}): gpu {len(g)} oracle {len(e)}, first diff at {d}")
        assert len(gc) == len(oc)
    # decode every stream in order on a fresh peer cache that first decodes the warm-up streams
    wo = oracle_mod.Cache()
    ws = wo.encode_batch(warm)
    dg = w.XCodecDecoder(gd)
    dg.decode_batch(ws)
    enc_all = []
    oc2 = oracle_mod.Cache()
    oc2.encode_batch(warm)
    for bufs in batches:
        enc_all.append((bufs, oc2.encode_batch(bufs)))
    for bufs, streams in enc_all:
        res = dg.decode_batch(streams)
        for i, (st, out, consumed, unk) in enumerate(res):
            assert st == 1 and unk is None and consumed == len(streams[i]), (seed, i)
            assert out == bufs[i].tobytes(), (seed, i)


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_streams(gpu_ctx, oracle_mod, monkeypatch, seed):
    """Stateful connections (encode() without flush, calls cut at random points and shuffled over
    connections) over one cache against the oracle's stateful encoders, the collision pair included."""
    import wanproxy_amd as w
    rng = np.random.default_rng(2000 + seed)
    monkeypatch.setenv("XC_CHUNK_BLOCKS", str(int(rng.choice([1, 2, 3, 5, 8]))))
    monkeypatch.setenv("XC_SUB_MB", str(int(rng.choice([1, 2, 512]))))
    pool = W.pool(64)
    warm = [pool[i:i + 65536] for i in range(0, int(rng.integers(1, 9)) * 65536, 65536)]
    oc = oracle_mod.Cache()
    gc = w.XCodecCache(gpu_ctx, int(rng.choice([1024, 1 << 16])))
    oc.encode_batch(warm)
    w.XCodecEncoder(gc).encode_batch(warm)
    n = int(rng.integers(2, 12))
    oe = [oracle_mod.Encoder(oc) for _ in range(n)]
    ge = [w.XCodecStreamEncoder(gc) for _ in range(n)]
    for _ in range(3):
        calls = []
        for buf in _batch(rng, pool):
            c = int(rng.integers(n))
            cuts = sorted(rng.integers(0, max(buf.size, 1), int(rng.integers(0, 4))))
            for piece in np.split(buf, cuts):
                calls.append((c, piece, bool(rng.random() < 0.4)))
        want = []
        for c, d, f in calls:
            o = oe[c].encode(d)
            if f:
                o += oe[c].flush()[1]
            want.append(o)
        got = w.encode_streams([(ge[c], d, f) for c, d, f in calls])
        bad = [i for i, (g, e) in enumerate(zip(got, want)) if g != e]
        assert not bad, (seed, bad[:5])
    for c in range(n):
        assert ge[c].flush() == oe[c].flush(), c
    assert len(gc) == len(oc)
