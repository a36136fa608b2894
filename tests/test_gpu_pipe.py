"""GPU tests of the XCodec pipe filters over the device codec (wanproxy_amd.pipe.DeviceBackend):
every byte both sides put on the wire (<HELLO>, <FRAME>s, <ASK>s, <LEARN>s, <EOS>/<EOS_ACK>) and
the decoded output must equal the same pipes run over the oracle backend
(xcodec/xcodec_filter.cc:122-526)."""
import numpy as np
import pytest

from wanproxy_amd import pipe as P
from wanproxy_amd import workloads as W

from pipe_harness import UUID_A, UUID_B, OracleBackend, Side, esc_buffer, pump

pytestmark = pytest.mark.gpu

POOL_SEGS = 256


def _warm_oracle(store):
    store.encode_batch(W.pool_warmup_buffers(POOL_SEGS))


def _warm_device(store):
    import wanproxy_amd as w
    w.XCodecEncoder(store).encode_batch(W.pool_warmup_buffers(POOL_SEGS))


def _data():
    p = W.pool(POOL_SEGS)
    bufs = W.repeat_buffers(6, 0x99, np_segments=POOL_SEGS, pool_bytes=p)
    bufs.append(esc_buffer(5000, 3))
    bufs.append(np.concatenate([p[2048:8192], esc_buffer(777, 4), p[:2048]]))
    bufs.append(W.gen(17, 100_000))  # > 32 KiB of output: several frames
    return bufs


def _run(backend, warm, bufs, chunk, waiting=False):
    a = Side(backend, UUID_A, warm=warm, waiting=waiting)
    b = Side(backend, UUID_B)
    for x in bufs:
        assert a.enc.consume(x.tobytes())
        if waiting:
            a.enc.on_read_timeout()
        pump(a, b, chunk)
    a.enc.flush(0)
    pump(a, b, chunk)
    b.enc.flush(0)
    pump(a, b, chunk)
    return a, b


@pytest.mark.parametrize("chunk", [None, 4093])
def test_device_pipes_match_the_oracle_pipes(gpu_ctx, oracle_mod, chunk):
    bufs = _data()
    ga, gb = _run(P.DeviceBackend(gpu_ctx, 1 << 14), _warm_device, bufs, chunk)
    oa, ob = _run(OracleBackend(oracle_mod), _warm_oracle, bufs, chunk)
    assert bytes(gb.sink.data) == b"".join(x.tobytes() for x in bufs)
    assert bytes(ga.wire.log) == bytes(oa.wire.log)  # HELLO, frames, LEARNs, EOS, EOS_ACK
    assert bytes(gb.wire.log) == bytes(ob.wire.log)  # ASKs, EOS_ACK, EOS
    assert b"\xfd" in bytes(gb.wire.log)
    assert ga.enc.eos_ack and gb.enc.eos_ack and gb.dec.upflushed and ga.dec.upflushed


def test_device_pipes_waiting_mode(gpu_ctx, oracle_mod):
    bufs = _data()[-3:]
    ga, gb = _run(P.DeviceBackend(gpu_ctx, 1 << 14), _warm_device, bufs, None, waiting=True)
    oa, ob = _run(OracleBackend(oracle_mod), _warm_oracle, bufs, None, waiting=True)
    assert bytes(gb.sink.data) == b"".join(x.tobytes() for x in bufs)
    assert bytes(ga.wire.log) == bytes(oa.wire.log)


def test_hash_segments_host(gpu_ctx, oracle_mod):
    import wanproxy_amd.xcodec as X
    segs = np.concatenate([W.gen(3, 64 * 2048), esc_buffer(2048, 5, frac=0.9), np.zeros(2048, np.uint8)])
    got = X.hash_segments_host(gpu_ctx, segs)
    want = [oracle_mod.hash_segment(segs[i:i + 2048]) for i in range(0, segs.size, 2048)]
    assert [int(x) for x in got] == [int(x) for x in want]
    assert X.hash_segments_host(gpu_ctx, np.zeros(0, np.uint8)).size == 0


def test_batched_device_pipes_64_connections(gpu_ctx, oracle_mod):
    """64 interleaved connections between two proxies, each proxy's codec calls batched per
    event-loop turn (wanproxy_amd.pipe.Batcher: one xc_encode_streams call for every EncodeFilter
    consume of the turn, one device decode call per peer cache): every wire byte in both
    directions and every decoded byte equal the unbatched filters over the oracle."""
    from pipe_harness import run_connections
    from test_pipe import _conn_inputs
    inputs = _conn_inputs(64, 3, seed=0x2718)
    da, db, dc = run_connections(P.DeviceBackend(gpu_ctx, 1 << 14), _warm_device, inputs, batched=True)
    oa, ob, oc = run_connections(OracleBackend(oracle_mod), _warm_oracle, inputs, batched=False)
    for i, (d, o) in enumerate(zip(dc, oc)):
        assert bytes(d.b_sink.data) == b"".join(x.tobytes() for x in inputs[i]), i
        assert bytes(d.ab.log) == bytes(o.ab.log), i
        assert bytes(d.ba.log) == bytes(o.ba.log), i
    assert da.batcher.device_calls <= 16  # 3 encode turns + a few decode turns, not 192 calls


def test_device_chain_with_deflate_stage(gpu_ctx, oracle_mod):
    """The proxy chain with the zlib stage (EncodeFilter -> DeflateFilter -> wire -> InflateFilter
    -> DecodeFilter, proxy/proxy_connector.cc:146-150,177-189) over the device codec: the compressed
    wire bytes equal the same chain over the oracle, and the peer gets every byte back."""
    from test_zlib import chain_round_trip
    assert chain_round_trip(P.DeviceBackend(gpu_ctx, 1 << 12)) == chain_round_trip(OracleBackend(oracle_mod))
