"""The persistent COSS cache (XCodecCacheCOSS, xcodec/cache/coss/xcodec_cache_coss.{h,cc}).

CPU: the oracle's restatement (oracle/xc_coss.c) keeps what the reference's own COSS test
(xcodec/cache/coss/test/xcodec-coss1/xcodec-coss1.cc:42-88, stale against the current class) meant
to check: segments entered, the cache closed and reopened, lookups return them.  The product's host
store (wanproxy_amd/csrc/xc_coss.cpp, no device needed) equals the oracle over long random
sequences of enters and lookups on a small cache file (stripe loads, the recent window, use flags,
purges of full stripes, the reopen with its shadowed stripe 0): every lookup result, the statistics
and the <uuid>.wpc file bytes.

GPU (tests/test_gpu_coss.py): the device encoder and decoder over a COSS cache against the oracle
codec over the oracle's COSS cache."""
import os

import numpy as np
import pytest

from wanproxy_amd import workloads as W

UUID = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0"
WPC = UUID + ".wpc"


def _segs(n, seed):
    return W.gen_segments(np.arange(n, dtype=np.uint64) + np.uint64(seed))


def test_oracle_coss_reopen_finds_segments(oracle_mod, tmp_path):
    segs = _segs(3000, 1 << 40)
    hs = [oracle_mod.hash_segment(s) for s in segs]
    c = oracle_mod.Cache.coss(str(tmp_path), UUID, 64)
    for h, s in zip(hs, segs):
        assert c.lookup(h) is None
        c.enter(h, s)
    assert len(c) == 3000
    c.close()
    assert os.path.getsize(tmp_path / WPC) % 1056768 == 0
    c = oracle_mod.Cache.coss(str(tmp_path), UUID, 64)
    assert len(c) == 3000
    # Reopened, the newest stripe (5) is loaded into slot 0 and slots 1-15 are unused with
    # stripe_range 0: lookup takes the first slot whose range matches (xcodec_cache_coss.cc:
    # 200-207), so stripe 0's 512 segments are shadowed by an empty slot until every slot is used;
    # the rest are found (each lookup of another stripe loads it into the next free slot).
    found = [c.lookup(h) for h in hs]
    assert all(f is None for f in found[:512])
    assert all(f == s.tobytes() for f, s in zip(found[512:], segs[512:]))
    c.close()


def _random_ops(rng, n_ops, segs, hs):
    """A mixed sequence: enters of new segments, lookups of entered / absent / recently looked-up
    hashes (recent-window hits), bursts on one stripe's segments."""
    ops, entered = [], []
    nxt = 0
    for _ in range(n_ops):
        r = rng.random()
        if r < 0.45 and nxt < len(segs):
            ops.append(("enter", nxt))
            entered.append(nxt)
            nxt += 1
        elif r < 0.85 and entered:
            ops.append(("lookup", entered[int(rng.integers(0, len(entered)))]))
        elif r < 0.95 and entered:
            k = entered[max(0, len(entered) - 1 - int(rng.integers(0, 64)))]
            ops.append(("lookup", k))
        else:
            ops.append(("miss", int(rng.integers(0, 1 << 62))))
    return ops


def _apply(cache, ops, segs, hs, store_only):
    got = []
    for op, k in ops:
        if op == "enter":
            if store_only is None:
                cache.enter(hs[k], segs[k])
            else:
                cache.enter(hs[k], segs[k], store_only=True)
        else:
            h = hs[k] if op == "lookup" else k
            got.append(cache.lookup(h) if store_only is None else cache.lookup(h, store_only=True))
    return got


@pytest.mark.parametrize("size_mb,nseg,nops", [(3, 9000, 16000), (6, 9000, 16000), (24, 30000, 60000)])
def test_store_equals_oracle(oracle_mod, tmp_path, size_mb, nseg, nops):
    """(24 MB: 23 stripes for 16 slots, so lookups load stripes into slots whose data stays in the
    file until something needs it, and stripes are purged and re-entered)"""
    import wanproxy_amd as w
    segs = _segs(nseg, 7 << 32)
    hs = [oracle_mod.hash_segment(s) for s in segs]
    ops = _random_ops(np.random.default_rng(size_mb), nops, segs, hs)
    da, db = tmp_path / "o", tmp_path / "p"
    da.mkdir()
    db.mkdir()
    for phase in range(3):  # open, work, close; then reopen (the file read back) twice
        o = oracle_mod.Cache.coss(str(da), UUID, size_mb)
        p = w.CossCache(None, str(db), UUID, size_mb)
        part = ops[phase * len(ops) // 3:(phase + 1) * len(ops) // 3]
        a = _apply(o, part, segs, hs, None)
        b = _apply(p, part, segs, hs, True)
        assert len(a) == len(b)
        bad = [i for i, (x, y) in enumerate(zip(a, b)) if x != y]
        assert not bad, (phase, bad[:5])
        assert len(o) == len(p)
        st = p.stats()
        assert st["stripe_limit"] == -(-size_mb * 1048576 // 1056768)
        o.close()
        p.close()
        assert (da / WPC).read_bytes() == (db / WPC).read_bytes(), phase
    # purges happened: fewer segments than entered survive
    assert sum(1 for op, _ in ops if op == "enter") > len(oracle_mod.Cache.coss(str(da), UUID, size_mb))


def test_replay_window_hash_equals_the_oracle(oracle_mod):
    """The replay's host window hash (wanproxy_amd/csrc/xc_replay.h WindowHash, used only for the
    lookups that miss with side effects) gives XCodecHash::mix of every window (xcodec/xcodec_hash.h):
    random bytes with zero bytes (ffs 0) and long 0xFF runs (the 32-bit sums' shifts wrap)."""
    import wanproxy_amd as w
    from wanproxy_amd import xcodec as X
    rng = np.random.default_rng(5)
    d = rng.integers(0, 256, 9000, dtype=np.uint8)
    d[100:400] = 0
    d[3000:6000] = 255
    got = X._window_hashes_host(d)
    assert got.size == d.size - 2047
    for i in list(range(0, 40)) + list(range(900, 1100, 7)) + list(range(2900, 6950, 97)) + [d.size - 2048]:
        assert int(got[i]) == oracle_mod.hash_segment(d[i:i + 2048]), i
