"""Full-size checks at BASELINE.json's headline configuration (cfg5 on one GPU: 32768 x 64 KiB =
2 GiB, 50% repeats, seed 0x5555, cache warmed with the 8192-segment pool), through properties
that do not need the oracle to run over all 2 GiB:

* round trip: the device encoder's streams, decoded on the device by a second cache warmed from
  the pool's warm-up streams (XCodecDecoder semantics, xcodec/xcodec_decoder.cc:76-176), give
  back every input buffer bit-exactly, with status true, every byte consumed, no unknown hash;
* the decoder executes exactly the encoder's EXTRACT and REF counts, and both caches end with
  the same number of segments;
* the first 64 buffers equal the oracle's encoding byte for byte (the sequential semantics
  beyond them are covered at smaller sizes by tests/test_gpu_encode.py)."""
import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu

TOTAL = 32768
SEG = 2048


def test_cfg5_full_size_round_trip(gpu_ctx, oracle_mod):
    import torch
    import wanproxy_amd as w
    shard = W.repeat_shard(TOTAL, 0x5555)
    n = shard.shape[0]
    warm = W.pool_warmup_buffers()
    cap = W.POOL_SEGMENTS + n * (W.BUF // SEG + 1) + 1024
    ec = w.XCodecCache(gpu_ctx, cap)
    warm_streams = w.XCodecEncoder(ec).encode_batch(warm)
    lens = np.full(n, W.BUF, np.uint64)
    plan = w.EncodePlan(ec, lens)
    assert all(int(plan.in_off[i]) == i * W.BUF for i in range(n))
    d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
    d_in[:n * W.BUF] = torch.from_numpy(shard.reshape(-1)).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # (torch's stream filled the arenas; the library runs on its own)
    plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    torch.cuda.synchronize()
    st = plan.stats()
    slen = d_len.cpu().numpy().astype(np.uint64)
    assert 0.49 < slen.sum() / (n * W.BUF) < 0.52

    # the first buffers against the oracle
    oc = oracle_mod.Cache()
    oc.encode_batch(warm)
    want = oc.encode_batch([shard[i] for i in range(64)])
    for i in range(64):
        o = int(plan.out_off[i])
        assert d_out[o:o + int(slen[i])].cpu().numpy().tobytes() == want[i], i

    # device decode of every stream into a fresh, pool-warmed decoder cache
    dc = w.XCodecCache(gpu_ctx, cap)
    w.XCodecDecoder(dc).decode_batch(warm_streams)
    dplan = w.DecodePlan(dc, slen, np.full(n, W.BUF, np.uint64))
    d_enc = torch.zeros(dplan.in_bytes, dtype=torch.uint8, device="cuda")
    for i in range(n):  # repack the encoder's arena into the decode plan's layout (on the device)
        a, o, m = int(dplan.in_off[i]), int(plan.out_off[i]), int(slen[i])
        d_enc[a:a + m].copy_(d_out[o:o + m])
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
    assert (r64[n:2 * n] == slen.astype(np.int64)).all()         # consumed everything
    assert (r32[n:2 * n] == 0).all()                             # no unknown REF
    ds = dplan.stats()
    assert int(ds.n_extract) == int(st.n_extract) and int(ds.n_ref) == int(st.n_ref)
    assert len(dc) == len(ec)
