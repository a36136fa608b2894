"""The zlib stage (wanproxy_amd/zlib_filter.py) against the reference's own DeflateFilter /
InflateFilter (zlib/zlib_filter.cc compiled from /root/reference into oracle/_ref/libzref.so, when
present) and against committed vectors of the reference's deflate bytes; and the proxy chain with
the stage (EncodeFilter -> DeflateFilter -> wire -> InflateFilter -> DecodeFilter,
proxy/proxy_connector.cc:146-150,177-189) round-trips every byte."""
import hashlib
import json
import os

import numpy as np
import pytest

from wanproxy_amd import pipe as P
from wanproxy_amd import workloads as W
from wanproxy_amd.zlib_filter import DeflateFilter, InflateFilter

from pipe_harness import UUID_A, UUID_B, OracleBackend, esc_buffer
from zlib_ref import RefFilter, lib

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "zlib_filter_vectors.json")


def consume_inputs():
    """Consume sizes around the segment and chunk sizes, incompressible and compressible data."""
    rng = np.random.default_rng(7)
    text = (b"GET /index.html HTTP/1.1\r\nHost: example.com\r\n\r\n" * 4000)
    out = [b"", b"a", W.gen(1, 2047).tobytes(), W.gen(2, 2048).tobytes(), W.gen(3, 2049).tobytes(),
           text[:65536], bytes(70000), W.gen(4, 200_000).tobytes(), text[:123457], esc_buffer(9000, 5).tobytes()]
    out += [W.gen(10 + k, int(rng.integers(1, 40000))).tobytes() for k in range(6)]
    return out


class Collect(P.Filter):
    def __init__(self):
        super().__init__()
        self.chunks = []
        self.flushes = 0

    def consume(self, buf, flg=0):
        self.chunks.append(bytes(buf))
        return True

    def flush(self, flg):
        self.flushes += 1


def _ours(deflate, level=0):
    f = DeflateFilter(level) if deflate else InflateFilter()
    c = Collect()
    f.chain(c)
    return f, c


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_deflate_matches_committed_reference_vectors(level):
    want = json.load(open(GOLD))["levels"][str(level)]
    f, c = _ours(True, level)
    got = []
    for data in consume_inputs():
        assert f.consume(data)
        got.append([len(c.chunks[-1]), hashlib.sha256(c.chunks[-1]).hexdigest()])
    n = len(c.chunks)
    f.flush(0)
    fl = b"".join(c.chunks[n:])
    got.append([len(fl), hashlib.sha256(fl).hexdigest()])
    assert got == want
    assert c.flushes == 1


@pytest.mark.parametrize("level", [0, 6, 9])
def test_filters_equal_the_reference_filters(level):
    z = lib()
    if z is None:
        pytest.skip("oracle/_ref/libzref.so not built (reference sources absent)")
    ref_d, ref_i = RefFilter(z, True, level), RefFilter(z, False)
    (d, dc), (i, ic) = _ours(True, level), _ours(False)
    rng = np.random.default_rng(level)
    stream = b""
    for data in consume_inputs():
        ok, want = ref_d.consume(data)
        assert d.consume(data) and ok and dc.chunks[-1] == want
        stream += want
    # the inflaters get the compressed stream cut anywhere (socket reads)
    cuts = np.sort(rng.choice(len(stream), 30, replace=False))
    for a, b in zip(np.r_[0, cuts], np.r_[cuts, len(stream)]):
        ok, want = ref_i.consume(stream[a:b])
        assert i.consume(stream[a:b]) and ok and ic.chunks[-1] == want
    assert b"".join(ic.chunks) == b"".join(consume_inputs())
    n = len(dc.chunks)
    d.flush(0)
    assert b"".join(dc.chunks[n:]) == ref_d.flush()
    n = len(ic.chunks)
    i.flush(0)
    assert b"".join(ic.chunks[n:]) == ref_i.flush()
    # corrupt input: both fail
    ref_bad, (bad, _) = RefFilter(z, False), _ours(False)
    junk = b"\x78\x9c" + bytes([0xFF]) * 64
    assert ref_bad.consume(junk)[0] is False and bad.consume(junk) is False


def test_xcodec_chain_with_deflate_stage(oracle_mod):
    """EncodeFilter -> DeflateFilter(6) -> wire -> InflateFilter -> DecodeFilter, cut into socket
    reads of 5000 bytes: the peer's output is the input, byte for byte."""
    chain_round_trip(OracleBackend(oracle_mod))


def chain_round_trip(be):
    """(also run over the device codec by tests/test_gpu_pipe.py)  Returns the wire bytes."""
    reg_a, reg_b = P.CacheRegistry(be), P.CacheRegistry(be)
    ca = reg_a.register(P.CodecCache(be.new_store(), UUID_A, 1))
    cb = reg_b.register(P.CodecCache(be.new_store(), UUID_B, 1))
    enc = P.EncodeFilter(P.Codec(be, ca, reg_a))
    dfl = DeflateFilter(6)
    wire = Collect()
    enc.chain(dfl)
    dfl.chain(wire)
    inf = InflateFilter()
    dec = P.DecodeFilter(P.Codec(be, cb, reg_b))
    sink = P.Sink()
    inf.chain(dec)
    dec.chain(sink)
    dec.set_upstream(P.Sink())  # (no <ASK>s: every REF is to a segment the stream declared)
    bufs = [W.gen(5, 30000), np.tile(W.gen(6, 4096), 8), esc_buffer(20000, 3), np.tile(W.gen(6, 4096), 3)]
    for b in bufs:
        assert enc.consume(b.tobytes())
    comp = b"".join(wire.chunks)
    for a in range(0, len(comp), 5000):
        assert inf.consume(comp[a:a + 5000])
    assert bytes(sink.data) == b"".join(b.tobytes() for b in bufs)
    return comp
