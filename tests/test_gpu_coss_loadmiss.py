"""COSS lookups that miss with side effects (xcodec/cache/coss/xcodec_cache_coss.cc:200-220).

A lookup whose index entry points into a stripe no slot holds loads that stripe (detaching the
least fresh slot) and then compares the header's hash at the entry's position: when the header in
the file disagrees with the index, the lookup misses -- after its side effects.  The device mirror
holds no segment for such a hash, so the device encoder treats those windows as the plain misses
they are; the replay finds them from the host's window hashes (xc_replay.h add_load_miss_lookups)
and the decoder's unknown REF is looked up like the reference's, so the Store takes every side
effect in the reference's order.

A header that disagrees with the index: the reference writes one back when a ≤16-stripe file's
stale second copy of a stripe is detached; random enter/lookup and encode sequences on 2–16 stripe
files did not reach the state (every stripe's copies keep one slot), so these tests make it
directly: with both caches open, the same hashes are changed in the file's headers of stripes no
slot holds (after a reopen only the newest stripe is loaded), and the product store reads its
header view again (CossCache._reread_headers, a test hook).  The oracle (oracle/xc_coss.c) reads
the headers from the file at each load; its count of such misses shows the state was reached.
Everything is compared with the oracle: encoded / decoded bytes, decoder status / consumed /
unknown hash, COSSStats and the <uuid>.wpc bytes after close."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu

UUID_A = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0"
UUID_B = "12345678-9abc-def0-1234-56789abcdef0"
STRIPE = 8192 + 512 * 2048
HASH_OFF = 4096  # COSSStripeHeader.hash_array (xcodec_cache_coss.h:162-168)


def _newest_range(path):
    data = open(path, "rb").read()
    n = len(data) // STRIPE
    serial = [int(np.frombuffer(data, np.uint64, 1, r * STRIPE + 8)[0]) for r in range(n)]
    return n, int(np.argmax(serial))


def _tamper(paths, ranges):
    """Change every other nonzero header hash of the given stripes, identically in each file;
    returns the segments whose index entries now disagree with their header (from the first file)."""
    segs = []
    for k, path in enumerate(paths):
        with open(path, "r+b") as f:
            for r in ranges:
                f.seek(r * STRIPE + HASH_OFF)
                h = np.frombuffer(f.read(4096), np.uint64).copy()
                pos = np.flatnonzero(h)[::2]
                if k == 0:
                    for i in pos:
                        f.seek(r * STRIPE + 8192 + int(i) * 2048)
                        segs.append(np.frombuffer(f.read(2048), np.uint8).copy())
                h[pos] ^= np.uint64(1)
                f.seek(r * STRIPE + HASH_OFF)
                f.write(h.tobytes())
    return segs


def _buffers(segs, seed):
    """Buffers that repeat the tampered segments: aligned runs, unaligned runs behind fresh bytes,
    each segment twice in a row (the second lookup finds the first one's declaration)."""
    rng = np.random.default_rng(seed)
    out = []
    for a in range(0, len(segs), 12):
        run = segs[a:a + 12]
        out.append(np.concatenate(run))
        out.append(np.concatenate([W.gen(seed + a, int(rng.integers(1, 3000)))] + run[::-1]))
        out.append(np.concatenate([run[0], run[0], W.gen(seed + a + 1, 5000)]))
    return out


@pytest.mark.parametrize("size_mb", [3, 8])
def test_coss_encode_with_load_misses_equals_the_oracle(gpu_ctx, oracle_mod, tmp_path, size_mb):
    import wanproxy_amd as w
    do, dp = tmp_path / "o", tmp_path / "p"
    do.mkdir()
    dp.mkdir()
    pool = W.pool(1024)
    oc = oracle_mod.Cache.coss(str(do), UUID_A, size_mb)
    pc = w.CossCache(gpu_ctx, str(dp), UUID_A, size_mb)
    for k in range(3 * size_mb):  # fill the file: every stripe written, purges
        bufs = W.repeat_buffers(48, 0x700 + k, np_segments=1024, pool_bytes=pool)
        assert oc.encode_batch(bufs) == w.XCodecEncoder(pc).encode_batch(bufs), k
    oc.close()
    pc.close()
    fo, fp = do / (UUID_A + ".wpc"), dp / (UUID_A + ".wpc")
    assert fo.read_bytes() == fp.read_bytes()
    n, newest = _newest_range(fo)
    assert n == -(-size_mb * 1048576 // STRIPE)
    # reopened: only the newest stripe is loaded; slots 1-15 shadow stripe 0
    oc = oracle_mod.Cache.coss(str(do), UUID_A, size_mb)
    pc = w.CossCache(gpu_ctx, str(dp), UUID_A, size_mb)
    ranges = [r for r in range(1, n) if r != newest]
    segs = _tamper([fo, fp], ranges)
    assert segs
    pc._reread_headers()
    bufs = _buffers(segs, 0x900)
    for a in range(0, len(bufs), 16):
        part = bufs[a:a + 16]
        want = oc.encode_batch(part)
        got = w.XCodecEncoder(pc).encode_batch(part)
        bad = [i for i, (x, y) in enumerate(zip(want, got)) if x != y]
        assert not bad, (a, bad[:5])
    assert oc.coss_load_misses() > 0  # the state was reached
    assert len(oc) == len(pc)
    assert pc.stats() == oc.coss_stats()
    # stateful encoders over the same state: the candidate carried across calls
    more = _buffers(segs[::-1], 0x990)
    oenc = [oracle_mod.Encoder(oc) for _ in range(4)]
    genc = [w.XCodecStreamEncoder(pc) for _ in range(4)]
    for t in range(0, len(more), 4):
        calls = [(c, more[t + c][: len(more[t + c]) // 2 + 777 * c], c == 3) for c in range(min(4, len(more) - t))]
        want = [oenc[c].encode(d) + (oenc[c].flush()[1] if f else b"") for c, d, f in calls]
        got = w.encode_streams([(genc[c], d, f) for c, d, f in calls])
        assert want == got, t
    for c in range(4):
        assert genc[c].flush() == oenc[c].flush(), c
    assert pc.stats() == oc.coss_stats()
    oc.close()
    pc.close()
    assert fo.read_bytes() == fp.read_bytes()


@pytest.mark.parametrize("size_mb", [3, 8])
def test_coss_decode_with_load_misses_equals_the_oracle(gpu_ctx, oracle_mod, tmp_path, size_mb):
    """The peer's decoder: a REF to a hash whose lookup misses after loading its stripe is unknown
    (the decoder stops on it, :144-160) and an EXTRACT of one is looked up, then entered."""
    import wanproxy_amd as w
    do, dp = tmp_path / "o", tmp_path / "p"
    do.mkdir()
    dp.mkdir()
    pool = W.pool(1024)
    enc = oracle_mod.Cache()  # the encoding side: a memory cache that keeps everything
    streams = []
    for k in range(3 * size_mb):
        streams += enc.encode_batch(W.repeat_buffers(48, 0x300 + k, np_segments=1024, pool_bytes=pool))
    oc = oracle_mod.Cache.coss(str(do), UUID_B, size_mb)
    pc = w.CossCache(gpu_ctx, str(dp), UUID_B, size_mb)
    for a in range(0, len(streams), 48):
        assert oc.decode_batch(streams[a:a + 48]) == w.XCodecDecoder(pc).decode_batch(streams[a:a + 48]), a
    oc.close()
    pc.close()
    fo, fp = do / (UUID_B + ".wpc"), dp / (UUID_B + ".wpc")
    assert fo.read_bytes() == fp.read_bytes()
    n, newest = _newest_range(fo)
    oc = oracle_mod.Cache.coss(str(do), UUID_B, size_mb)
    pc = w.CossCache(gpu_ctx, str(dp), UUID_B, size_mb)
    segs = _tamper([fo, fp], [r for r in range(1, n) if r != newest])
    assert segs
    pc._reread_headers()
    bufs = _buffers(segs, 0x500)
    refs = enc.encode_batch(bufs)                     # REFs (the encoder's cache has them all)
    fresh = oracle_mod.Cache().encode_batch(bufs)     # EXTRACTs (a fresh encoder declares them)
    todo = [s for pair in zip(refs, fresh) for s in pair]
    for a in range(0, len(todo), 8):
        want = oc.decode_batch(todo[a:a + 8])
        got = w.XCodecDecoder(pc).decode_batch(todo[a:a + 8])
        bad = [i for i, (x, y) in enumerate(zip(want, got)) if x != y]
        assert not bad, (a, bad[:5])
    assert oc.coss_load_misses() > 0
    assert pc.stats() == oc.coss_stats()
    oc.close()
    pc.close()
    assert fo.read_bytes() == fp.read_bytes()
