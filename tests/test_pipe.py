"""CPU tests of the XCodec pipe filters (wanproxy_amd.pipe, mirroring xcodec/xcodec_filter.cc)
over the oracle backend: framing, <HELLO>, <ASK>/<LEARN>, <EOS>/<EOS_ACK>, waiting-mode flush,
partial delivery and the reference's error returns.  The device backend runs the same cases in
tests/test_gpu_pipe.py."""
import struct

import numpy as np
import pytest

from wanproxy_amd import pipe as P
from wanproxy_amd import workloads as W

from pipe_harness import UUID_A, UUID_B, OracleBackend, Side, esc_buffer, parse, pump, run_connections

POOL_SEGS = 256  # a small pool keeps the CPU cases fast


def _pool_warm(oracle_mod):
    warm = W.pool_warmup_buffers(POOL_SEGS)
    return lambda store: store.encode_batch(warm)


def _data(n=6):
    p = W.pool(POOL_SEGS)
    bufs = W.repeat_buffers(n - 2, 0x77, np_segments=POOL_SEGS, pool_bytes=p)
    bufs.append(esc_buffer(5000, 3))          # literals with F1 bytes, short buffer
    bufs.append(np.concatenate([p[:4096], esc_buffer(777, 4)]))
    return bufs


def test_hello_and_frames_match_the_batch_encoder(oracle_mod):
    be = OracleBackend(oracle_mod)
    a = Side(be, UUID_A, warm=_pool_warm(oracle_mod), size=123)
    bufs = _data()
    for b in bufs:
        assert a.enc.consume(b.tobytes())
    msgs = parse(bytes(a.wire.log))
    assert msgs[0] == (P.OP_HELLO, UUID_A.encode() + struct.pack("<Q", 123))
    assert bytes(a.wire.log[:2]) == b"\xff\x2c"
    frames = [m for op, m in msgs[1:] if op == P.OP_FRAME]
    assert all(1 <= len(f) <= P.MAX_FRAME for f in frames)
    # flush after every consume == a fresh encoder per buffer over the same cache
    ref = oracle_mod.Cache()
    _pool_warm(oracle_mod)(ref)
    assert b"".join(frames) == b"".join(ref.encode_batch(bufs))


def test_large_consume_splits_into_32k_frames(oracle_mod):
    be = OracleBackend(oracle_mod)
    a = Side(be, UUID_A)
    data = W.gen(5, 100_000)
    assert a.enc.consume(data.tobytes())
    msgs = parse(bytes(a.wire.log))
    lens = [len(m) for op, m in msgs if op == P.OP_FRAME]
    assert lens[:-1] == [P.MAX_FRAME] * (len(lens) - 1) and 0 < lens[-1] <= P.MAX_FRAME


@pytest.mark.parametrize("chunk", [None, 1, 997])
def test_duplex_ask_learn_round_trip(oracle_mod, chunk):
    """B's cache knows nothing: every REF in A's stream is asked for and learned, and B's
    decoded output is exactly A's input.  Then both sides close with EOS / EOS_ACK."""
    be = OracleBackend(oracle_mod)
    a = Side(be, UUID_A, warm=_pool_warm(oracle_mod))
    b = Side(be, UUID_B)
    bufs = _data()
    for x in bufs:
        assert a.enc.consume(x.tobytes())
        pump(a, b, chunk)
    assert bytes(b.sink.data) == b"".join(x.tobytes() for x in bufs)
    asks = [m for op, m in parse(bytes(b.wire.log)) if op == P.OP_ASK]
    learns = [m for op, m in parse(bytes(a.wire.log)) if op == P.OP_LEARN]
    assert asks and len(asks) == len(learns)
    # every learned segment entered B's copy of A's cache under its hash
    peer = b.registry.find_cache(UUID_A)
    assert peer is not None
    for m in learns:
        assert peer.lookup(be.hash_segment(m)) == m
    # EOS handshake in both directions
    a.enc.flush(0)
    pump(a, b, chunk)
    assert b.dec.received_eos and b.dec.sent_eos_ack and b.sink.flushes == [0]
    b.enc.flush(0)
    pump(a, b, chunk)
    assert a.dec.received_eos and a.dec.received_eos_ack and a.dec.upflushed
    assert b.dec.received_eos_ack and b.dec.upflushed
    assert a.enc.eos_ack and b.enc.eos_ack
    assert a.wire.flushes == [0] and b.wire.flushes == [0]


def test_waiting_mode_defers_the_flush(oracle_mod):
    be = OracleBackend(oracle_mod)
    a = Side(be, UUID_A, waiting=True)
    data = esc_buffer(10_000, 9)
    assert a.enc.consume(data.tobytes())
    assert a.enc.wait_armed
    before = b"".join(m for op, m in parse(bytes(a.wire.log)) if op == P.OP_FRAME)
    a.enc.on_read_timeout()
    assert not a.enc.wait_armed
    frames = b"".join(m for op, m in parse(bytes(a.wire.log)) if op == P.OP_FRAME)
    ref = oracle_mod.Cache()
    assert frames == ref.encode_batch([data])[0]
    assert len(before) < len(frames)
    # TO_BE_CONTINUED: neither flush nor timer
    a2 = Side(be, UUID_A, waiting=True)
    assert a2.enc.consume(data.tobytes(), P.TO_BE_CONTINUED)
    assert not a2.enc.wait_armed


def test_decoder_errors(oracle_mod):
    be = OracleBackend(oracle_mod)

    def fresh():
        s = Side(be, UUID_B)
        return s.dec

    hello = b"\xff\x2c" + UUID_A.encode() + struct.pack("<Q", 1)
    assert not fresh().consume(b"\xfe" + bytes(2048))              # LEARN before HELLO
    assert not fresh().consume(b"\x00\x00\x05abcde")               # FRAME before HELLO
    assert not fresh().consume(hello + b"\x00\x00\x00")            # zero-length frame
    assert not fresh().consume(hello + b"\x00\x80\x01")            # frame > 32768
    assert not fresh().consume(hello + hello)                      # HELLO twice
    assert not fresh().consume(b"\xff\x2b" + bytes(43))            # HELLO length
    assert not fresh().consume(b"\xff\x2c" + b"x" * 36 + bytes(8))  # bad UUID
    assert not fresh().consume(b"\xfc\xfc")                        # duplicate EOS
    assert not fresh().consume(b"\xfb\xfb")                        # duplicate EOS_ACK
    assert not fresh().consume(b"\x42")                            # unknown op
    assert not fresh().consume(b"\xfd" + struct.pack(">Q", 12345))  # ASK for an unknown hash
    # incomplete messages wait for more bytes
    d = fresh()
    assert d.consume(hello[:10]) and d.consume(hello[10:]) and d.consume(b"\x00\x00")
    # collision in LEARN: same hash, different bytes already cached
    d = fresh()
    assert d.consume(hello)
    # odd bytes with +2, -2 at (i, i+1) and -2, +2 at (j, j+1) keep both window sums and every ffs
    seg = esc_buffer(2048, 11)
    i, j = 100, 900
    seg[[i, i + 1, j, j + 1]] = [11, 13, 21, 23]
    seg2 = seg.copy()
    seg2[[i, i + 1, j, j + 1]] = [13, 11, 19, 25]
    assert be.hash_segment(seg.tobytes()) == be.hash_segment(seg2.tobytes())
    assert d.consume(b"\xfe" + seg.tobytes())
    assert not d.consume(b"\xfe" + seg2.tobytes())
    # redundant LEARN is fine
    d = fresh()
    assert d.consume(hello + b"\xfe" + seg.tobytes() + b"\xfe" + seg.tobytes())


def test_encoder_needs_a_valid_uuid(oracle_mod):
    be = OracleBackend(oracle_mod)
    reg = P.CacheRegistry(be)
    bad = P.CodecCache(be.new_store(), "not-a-uuid")
    e = P.EncodeFilter(P.Codec(be, bad, reg))
    e.chain(P.Sink())
    assert not e.consume(b"abc")
    assert not P.DecodeFilter(P.Codec(be, None, reg)).consume(b"\xfc")  # no upstream


def _conn_inputs(n_conn, turns, seed=0x3141):
    """Per connection, per turn: 64 KiB buffers with repeats of a small pool, of other
    connections' earlier buffers (cross-connection duplicates) and F1-heavy literals."""
    p = W.pool(POOL_SEGS)
    rng = np.random.default_rng(seed)
    shared = [W.gen(1000 + k, 8192) for k in range(8)]
    out = []
    for i in range(n_conn):
        row = []
        for t in range(turns):
            kind = (i + t) % 4
            if kind == 0:
                b = W.repeat_buffers(1, 0x500 + 31 * i + t, np_segments=POOL_SEGS, pool_bytes=p)[0]
            elif kind == 1:
                b = np.concatenate([shared[(i * 3 + t) % 8], esc_buffer(3000 + i, i * 7 + t), shared[t % 8]])
            elif kind == 2:
                b = W.gen(2000 + 97 * i + t, 20000 + int(rng.integers(0, 30000)))
            else:
                b = np.concatenate([p[2048 * (i % 50):2048 * (i % 50) + 6000], esc_buffer(900, t)])
            row.append(b)
        out.append(row)
    return out


@pytest.mark.parametrize("chunk", [None, 5000])
def test_batched_turns_equal_sequential_calls(oracle_mod, chunk):
    """The Batcher (one codec call per kind and cache per event-loop turn) gives exactly the wire
    bytes of the unbatched filters called one by one in the same order (oracle backend)."""
    be = OracleBackend(oracle_mod)
    inputs = _conn_inputs(12, 3)
    warm = _pool_warm(oracle_mod)
    sa, sb, sc = run_connections(be, warm, inputs, batched=False, chunk=chunk)
    ba, bb, bc = run_connections(be, warm, inputs, batched=True, chunk=chunk)
    asked = False
    for i, (s, b) in enumerate(zip(sc, bc)):
        assert bytes(b.b_sink.data) == b"".join(x.tobytes() for x in inputs[i])
        assert bytes(b.ab.log) == bytes(s.ab.log), i
        assert bytes(b.ba.log) == bytes(s.ba.log), i
        asked = asked or b"\xfd" in bytes(b.ba.log)
        assert b.a_enc.eos_ack and b.b_enc.eos_ack
    assert asked  # the peer cache started empty: <ASK>/<LEARN> ran, through the sync path
    assert ba.batcher.device_calls < sum(len(r) for r in inputs)


def test_deferred_failure_is_reported_and_tears_the_filter_down(oracle_mod):
    """A deferred decode that fails (a bad opcode inside a frame, xcodec_decoder.cc:169-171) while
    a flush drains the batch: the turn's run() still reports the filter, and its next consume
    returns False, as the reference's consume of that call would have."""
    be = OracleBackend(oracle_mod)
    a = P.Batcher(be)
    reg = P.CacheRegistry(be)
    codec = P.Codec(be, reg.register(P.CodecCache(be.new_store(), UUID_A, 64)), reg, a)
    dec = P.DecodeFilter(codec)
    dec.set_upstream(P.Sink())
    dec.chain(P.Sink())
    hello = bytes([P.OP_HELLO, 44]) + UUID_B.encode() + struct.pack("<Q", 64)
    bad = b"abc\xf1\x07xyz"
    assert dec.consume(hello + bytes([P.OP_FRAME]) + struct.pack(">H", len(bad)) + bad)
    assert a.pending(dec)
    dec.flush(0)                      # drains the batch: the deferred decode fails here
    assert dec.deferred_failed
    assert a.run() == [dec]           # reported by the turn's end
    assert a.run() == []              # once
    assert not dec.consume(bytes([P.OP_FRAME]) + struct.pack(">H", 1) + b"a")
