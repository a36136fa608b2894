"""The device cache's spill tier: a cache outgrows the device's share of segment slots and keeps
the rest of its segment bytes in pinned host memory (SegStore, wanproxy_amd/csrc/xc_kernels.h), as
the reference's map grows without bound (xcodec/xcodec_cache.h:164,182-188).  The device's share is
lowered to 1024 slots (a test hook; 2^25 by default), so a few batches spill thousands of segments;
every encoded and decoded byte equals the oracle's, including REFs and unaligned repeats of spilled
segments (their compares read host memory over PCIe), the decoder's copies of spilled segments,
lookups, and a snapshot taken before the spill.  A restore across the cache's growth rebuilds its
tables from the snapshot's entries (a growth re-places every key in parallel, so the undo log alone
could cut an older key's probe chain)."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("spill", [True, False])
def test_encode_and_decode_over_a_spilled_cache(gpu_ctx, oracle_mod, spill):
    """(spill=False: the same sequence with every slot in HBM: the restore across the cache's
    growth -- its tables rebuilt since the snapshot -- keeps every older entry.)"""
    import wanproxy_amd as w
    cache = w.XCodecCache(gpu_ctx, 1024)
    if spill:
        cache._set_device_limit(1024)
    oc = oracle_mod.Cache()
    enc = w.XCodecEncoder(cache)
    first = W.random_buffers(16, seed0=0x9100)  # 512 segments, on the device
    assert enc.encode_batch(first) == oc.encode_batch(first)
    cache.snapshot()
    snap_oracle = oc.clone()
    fresh = []
    for k in range(4):  # 4 x 2560 new segments: most of them spill
        bufs = W.random_buffers(80, seed0=0xA100 + 100 * k)
        fresh += bufs
        assert enc.encode_batch(bufs) == oc.encode_batch(bufs), k
    assert len(cache) == len(oc) == 512 + 10240
    dev, spilled = cache._tiers()
    if spill:
        assert dev == 1024 and spilled >= len(cache) - 1024
    else:
        assert dev >= len(cache) and spilled == 0
    # repeats of spilled segments: aligned (REFs), shifted (the resolve's compares), mixed
    rng = np.random.default_rng(3)
    again = [fresh[-1], fresh[100], np.concatenate([W.gen(5, 777), fresh[200][:30000]]),
             np.concatenate([fresh[150][5000:], first[2][:9000], W.gen(6, 100)])]
    for _ in range(12):
        a, b = rng.integers(0, len(fresh), 2)
        cut = int(rng.integers(1, 60000))
        again.append(np.concatenate([fresh[a][cut:], fresh[b][:cut]]))
    assert enc.encode_batch(again) == oc.encode_batch(again)
    # lookups of spilled and device-resident segments
    for buf in (fresh[-1], first[0]):
        seg = buf[:2048]
        assert cache.lookup(oracle_mod.hash_segment(seg)) == seg.tobytes()
    # the peer: a decoder cache that spills too, decoding the streams (EXTRACTs of every segment,
    # then REFs to spilled ones)
    streams = oracle_mod.Cache().encode_batch(fresh[:120] + fresh[:40])
    dc = w.XCodecCache(gpu_ctx, 512)
    if spill:
        dc._set_device_limit(512)
    got = w.XCodecDecoder(dc).decode_batch(streams)
    want = oracle_mod.Cache().decode_batch(streams)
    assert got == want
    assert (dc._tiers()[1] > 0) == spill
    # the snapshot from before the growth: restored, the cache answers as then (every segment of
    # `first` found, none of the later ones)
    cache.restore()
    assert len(cache) == 512
    for b in first:
        for k in range(0, 32, 3):
            seg = b[2048 * k:2048 * (k + 1)]
            assert cache.lookup(oracle_mod.hash_segment(seg)) == seg.tobytes()
    assert cache.lookup(oracle_mod.hash_segment(fresh[7][:2048])) is None
    back = W.random_buffers(8, seed0=0xA100) + first[:4]
    assert enc.encode_batch(back) == snap_oracle.encode_batch(back)
