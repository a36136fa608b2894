"""Full-size parity at BASELINE.json's configurations, every buffer byte-checked.

The oracle cannot run on the GPU box in test time at 2 GiB, so it ran here: tests/golden/
make_fullsize.py committed, for every buffer of every configuration, the oracle encoder's output
length and a 64-bit sha256 digest of its bytes (tests/golden/fullsize_digests.npz).  The device
outputs are digested the same way and compared buffer by buffer:

* cfg5 (32768 x 64 KiB, 50 % repeats, seed 0x5555, pool-warmed cache) at N = 1, and every shard
  of N = 2, 4, 8 (buffer i -> shard i mod N, each shard against its own cache);
* cfg3 (4096 x 64 KiB, seed 0x77, warm), cfg4's 90 % variant input (seed 0x88), cfg2 (256 x
  64 KiB random, empty cache);
* the device decoder returns every cfg5 buffer from the device encoder's streams (status true,
  every byte consumed, no unknown hash; xcodec/xcodec_decoder.cc:76-176), and cfg4's streams;
* the reference's own round-trip test (xcodec/test/xcodec-encode-decode1/
  xcodec-encode-decode1.cc:41-105) for all 256 byte values: 512 KiB of byte i encodes to one
  EXTRACT + 255 REFs (4600 bytes) and decodes back exactly with the same cache.
"""
import os

import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu

TOTAL = 32768
SEG = 2048
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize_digests.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def _cache_cap(n):
    return W.POOL_SEGMENTS + n * (W.BUF // SEG + 1) + 1024


def _encode(ctx, bufs, warm: bool):
    """Encode an (n, 65536) array on the device as one batch; returns (plan, cache, d_in, d_out,
    lens, warm streams)."""
    import torch
    import wanproxy_amd as w
    n = bufs.shape[0]
    cache = w.XCodecCache(ctx, _cache_cap(n))
    warm_streams = w.XCodecEncoder(cache).encode_batch(W.pool_warmup_buffers()) if warm else []
    plan = w.EncodePlan(cache, np.full(n, W.BUF, np.uint64))
    assert all(int(plan.in_off[i]) == i * W.BUF for i in range(n))
    d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
    d_in[:n * W.BUF] = torch.from_numpy(bufs.reshape(-1)).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # (torch's stream filled the arenas; the library runs on its own)
    plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    torch.cuda.synchronize()
    return plan, cache, d_in, d_out, d_len.cpu().numpy().astype(np.uint64), warm_streams


def _check_digests(gold, case, plan, d_out, lens):
    want_len, want_dig = gold[case + "_len"], gold[case + "_dig"]
    assert lens.size == want_len.size
    bad = np.nonzero(lens != want_len.astype(np.uint64))[0]
    assert bad.size == 0, f"{case}: {bad.size} buffers differ in length from the oracle, first {bad[:8]}"
    dig = W.arena_digests(d_out.cpu().numpy(), plan.out_off, lens)
    bad = np.nonzero(dig != want_dig)[0]
    assert bad.size == 0, f"{case}: {bad.size} buffers differ from the oracle, first {bad[:8]}"


def _decode_round_trip(ctx, plan, d_in, d_out, lens, warm_streams, enc_stats, enc_cache):
    """Device decode of every stream into a fresh decoder cache warmed by decoding the warm-up
    streams: every buffer comes back, status true, all consumed, no unknown REF."""
    import torch
    import wanproxy_amd as w
    n = lens.size
    dc = w.XCodecCache(ctx, _cache_cap(n))
    if warm_streams:
        w.XCodecDecoder(dc).decode_batch(warm_streams)
    dplan = w.DecodePlan(dc, lens, np.full(n, W.BUF, np.uint64))
    d_enc = torch.zeros(dplan.in_bytes, dtype=torch.uint8, device="cuda")
    src = torch.as_tensor(np.asarray(plan.out_off, np.int64), device="cuda")
    dst = torch.as_tensor(np.asarray(dplan.in_off, np.int64), device="cuda")
    ln = torch.as_tensor(lens.astype(np.int64), device="cuda")
    # repack the encoder's arena into the decode plan's layout with one gather on the device
    rel = torch.arange(int(dplan.in_bytes), device="cuda")
    idx = torch.searchsorted(dst, rel, right=True) - 1
    off = rel - dst[idx]
    ok = off < ln[idx]
    d_enc[ok] = d_out[(src[idx] + off)[ok]]
    del rel, idx, off, ok
    d_dec = torch.zeros(dplan.out_bytes, dtype=torch.uint8, device="cuda")
    u64 = torch.zeros(3 * n, dtype=torch.int64, device="cuda")
    i32 = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    p64, p32 = u64.data_ptr(), i32.data_ptr()
    torch.cuda.synchronize()
    dplan.run(d_enc.data_ptr(), d_dec.data_ptr(), p64, p64 + 8 * n, p32, p64 + 16 * n, p32 + 4 * n)
    torch.cuda.synchronize()
    assert all(int(dplan.out_off[i]) == i * W.BUF for i in range(n))
    assert torch.equal(d_dec[:n * W.BUF], d_in[:n * W.BUF])
    r64 = u64.cpu().numpy()
    r32 = i32.cpu().numpy()
    assert (r32[:n] == 1).all()                                  # status true
    assert (r64[:n] == W.BUF).all()                              # decoded length
    assert (r64[n:2 * n] == lens.astype(np.int64)).all()         # consumed everything
    assert (r32[n:2 * n] == 0).all()                             # no unknown REF
    ds = dplan.stats()
    assert int(ds.n_extract) == int(enc_stats.n_extract) and int(ds.n_ref) == int(enc_stats.n_ref)
    assert len(dc) == len(enc_cache)
    dplan.close()
    dc.close()


def test_cfg5_full_size_every_buffer(gpu_ctx, gold):
    shard = W.repeat_shard(TOTAL, 0x5555)
    plan, cache, d_in, d_out, lens, warm_streams = _encode(gpu_ctx, shard, True)
    del shard
    st = plan.stats()
    assert 0.49 < lens.sum() / (TOTAL * W.BUF) < 0.52
    _check_digests(gold, "cfg5_g1_r0", plan, d_out, lens)
    _decode_round_trip(gpu_ctx, plan, d_in, d_out, lens, warm_streams, st, cache)
    plan.close()
    cache.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_cfg5_shards(gpu_ctx, gold, world):
    """Every shard of an N-GPU cfg5 run (one cache per shard) equals the oracle's independent run
    of that shard, every buffer (the per-GPU work of bench.py --gpus N)."""
    for rank in range(world):
        shard = W.repeat_shard(TOTAL, 0x5555, rank, world)
        plan, cache, d_in, d_out, lens, _ = _encode(gpu_ctx, shard, True)
        _check_digests(gold, f"cfg5_g{world}_r{rank}", plan, d_out, lens)
        plan.close()
        cache.close()
        del d_in, d_out


def test_cfg3_and_cfg4_decode(gpu_ctx, gold):
    """cfg3 encode, every buffer; then cfg4: the device decoder over cfg3's streams."""
    bufs = W.repeat_shard(4096, 0x77)
    plan, cache, d_in, d_out, lens, warm_streams = _encode(gpu_ctx, bufs, True)
    assert abs(lens.sum() / (4096 * W.BUF) - 0.5038) < 0.002  # the reference's ratio
    _check_digests(gold, "cfg3", plan, d_out, lens)
    _decode_round_trip(gpu_ctx, plan, d_in, d_out, lens, warm_streams, plan.stats(), cache)


def test_cfg4_variant(gpu_ctx, gold):
    bufs = W.repeat_shard(4096, 0x88, repeat_pct=90)
    plan, cache, d_in, d_out, lens, warm_streams = _encode(gpu_ctx, bufs, True)
    _check_digests(gold, "cfg4v", plan, d_out, lens)
    _decode_round_trip(gpu_ctx, plan, d_in, d_out, lens, warm_streams, plan.stats(), cache)


def test_cfg2_every_buffer(gpu_ctx, gold):
    bufs = np.stack(W.random_buffers(256))
    plan, cache, d_in, d_out, lens, _ = _encode(gpu_ctx, bufs, False)
    assert abs(lens.sum() / (256 * W.BUF) - 1.0010) < 0.0005  # the reference's ratio
    _check_digests(gold, "cfg2", plan, d_out, lens)


def test_reference_char_run_round_trip_256(gpu_ctx):
    """xcodec-encode-decode1.cc:41-105 for every byte value: 2048 bytes of i doubled 8 times
    (512 KiB), one encoder and cache per value; the encoding is smaller (one EXTRACT + 255 REFs =
    4600 bytes) and the decoder with the same cache returns the original exactly."""
    import wanproxy_amd as w
    for i in range(256):
        data = np.full(512 * 1024, i, np.uint8)
        cache = w.XCodecCache(gpu_ctx, 64)
        (enc,) = w.XCodecEncoder(cache).encode_batch([data])
        assert len(enc) == 4600 and len(enc) < data.size, (i, len(enc))
        assert enc[:2] == b"\xf1\x01" and enc[2:2050] == bytes([i]) * 2048
        (res,) = w.XCodecDecoder(cache).decode_batch([enc], out_cap=data.size)
        status, out, consumed, unknown = res
        assert status == 1 and unknown is None and consumed == len(enc), i
        assert out == data.tobytes(), i
        cache.close()
