"""The device codec over the persistent COSS cache (wanproxy_amd/csrc/xc_coss.cpp) against the
oracle codec over the oracle's COSS restatement (oracle/xc_coss.c), on cache files small enough
that full stripes are purged inside the batches: every encoded and decoded byte, every decoder
status / consumed count / unknown hash, and the <uuid>.wpc file bytes after close and after a
reopen (XCodecCacheCOSS, xcodec/cache/coss/xcodec_cache_coss.cc:31-377).

Files of 16 stripes or fewer take the reference's degenerate path: with every stripe loaded,
best_erasable_stripe returns stripe 0 (:304-321), whose second copy is then shadowed by the first
(lookup takes the first slot with the range, :200-207), so segments entered there are not found.
The 20 MB file (19 stripes) takes the ordinary path: unloaded stripes are purged and reused."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu

UUID_A = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0"
UUID_B = "12345678-9abc-def0-1234-56789abcdef0"
POOL = 1024


def _batches(n_batches, per_batch, seed):
    """Buffers of 32 segment slots: repeats of a 1024-segment pool (lookup hits), fresh data
    (declarations), and an unaligned repeat of an earlier buffer in every batch."""
    p = W.pool(POOL)
    out = []
    for k in range(n_batches):
        bufs = W.repeat_buffers(per_batch, seed + k, np_segments=POOL, pool_bytes=p)
        bufs[3] = np.concatenate([W.gen(seed + 100 + k, 777), bufs[1][:40000]])
        out.append(bufs)
    return out


def _collision_batch():
    rng = np.random.default_rng(1)
    x = (rng.integers(2, 126, 2048, dtype=np.int64) * 2 + 1).astype(np.uint8)
    y = x.copy()
    y[100] += 2; y[101] -= 2; y[1500] -= 2; y[1501] += 2
    return [x, np.concatenate([W.gen(3, 500), y, W.gen(4, 5000)]), np.concatenate([y, x, y, W.gen(5, 3000)])]


@pytest.mark.parametrize("size_mb,n_batches,per_batch", [(3, 4, 48), (8, 4, 48), (20, 8, 128)])
def test_coss_encode_decode_equal_the_oracle(gpu_ctx, oracle_mod, tmp_path, size_mb, n_batches, per_batch):
    import wanproxy_amd as w
    do, dp = tmp_path / "o", tmp_path / "p"
    do.mkdir()
    dp.mkdir()
    batches = _batches(n_batches, per_batch, 0x501) + [_collision_batch()]
    cut = (2 * n_batches) // 3
    streams = []
    for phase, part in enumerate((batches[:cut], batches[cut:])):  # a reopen between the phases
        oc = oracle_mod.Cache.coss(str(do / ""), UUID_A, size_mb)
        pc = w.CossCache(gpu_ctx, str(dp), UUID_A, size_mb)
        for k, bufs in enumerate(part):
            want = oc.encode_batch(bufs)
            got = w.XCodecEncoder(pc).encode_batch(bufs)
            bad = [i for i, (a, b) in enumerate(zip(want, got)) if a != b]
            assert not bad, (phase, k, bad[:5])
            streams += want
        assert len(oc) == len(pc)
        # COSSStats (xcodec_cache_coss.cc:194-233): every lookup call, misses included
        assert pc.stats() == oc.coss_stats(), phase
        oc.close()
        pc.close()
        assert (do / (UUID_A + ".wpc")).read_bytes() == (dp / (UUID_A + ".wpc")).read_bytes(), phase
    # the peer's decoder over its own COSS cache (REFs to purged segments become unknown hashes)
    oc = oracle_mod.Cache.coss(str(do), UUID_B, size_mb)
    pc = w.CossCache(gpu_ctx, str(dp), UUID_B, size_mb)
    for a in range(0, len(streams), 40):
        chunk = streams[a:a + 40]
        want = oc.decode_batch(chunk)
        got = w.XCodecDecoder(pc).decode_batch(chunk)
        bad = [i for i, (x, y) in enumerate(zip(want, got)) if x != y]
        assert not bad, (a, bad[:5])
    assert pc.stats() == oc.coss_stats()
    oc.close()
    pc.close()
    assert (do / (UUID_B + ".wpc")).read_bytes() == (dp / (UUID_B + ".wpc")).read_bytes()


@pytest.mark.parametrize("size_mb", [3, 20])
def test_coss_stream_encoders_equal_the_oracle(gpu_ctx, oracle_mod, tmp_path, size_mb):
    """Stateful encoders over COSS (the server side's waiting mode: encode() without flush, the
    candidate and pending bytes carried between calls), many connections batched per round
    (xc_coss_encode_streams): every call's bytes, the final flushes and the file equal the oracle's
    stateful encoders over the oracle's COSS cache."""
    import wanproxy_amd as w
    do, dp = tmp_path / "o", tmp_path / "p"
    do.mkdir()
    dp.mkdir()
    oc = oracle_mod.Cache.coss(str(do), UUID_A, size_mb)
    pc = w.CossCache(gpu_ctx, str(dp), UUID_A, size_mb)
    rng = np.random.default_rng(size_mb)
    nconn = 24
    oenc = [oracle_mod.Encoder(oc) for _ in range(nconn)]
    genc = [w.XCodecStreamEncoder(pc) for _ in range(nconn)]
    # each connection's data: pool repeats and fresh data (64 KiB reads), cut at random points
    conns = []
    for k, bufs in enumerate(_batches(4 if size_mb == 3 else 10, nconn, 0x900 + size_mb)):
        for c in range(nconn):
            conns.append((c, bufs[c]))
    for turn in range(0, len(conns), nconn):
        calls = []
        for c, buf in conns[turn:turn + nconn]:
            cuts = sorted(rng.integers(0, len(buf), 2))
            for piece in np.split(buf, cuts):
                calls.append((c, piece, bool(rng.random() < 0.3)))
        rng.shuffle(calls)
        want = []
        for c, d, f in calls:
            o = oenc[c].encode(d)
            if f:
                o += oenc[c].flush()[1]
            want.append(o)
        got = w.encode_streams([(genc[c], d, f) for c, d, f in calls])
        bad = [i for i, (a, b) in enumerate(zip(want, got)) if a != b]
        assert not bad, (turn, bad[:5])
    for c in range(nconn):
        assert genc[c].flush() == oenc[c].flush(), c
    assert len(oc) == len(pc)
    assert pc.stats() == oc.coss_stats()
    oc.close()
    pc.close()
    assert (do / (UUID_A + ".wpc")).read_bytes() == (dp / (UUID_A + ".wpc")).read_bytes()
