"""Filter-path throughput: N connections of one proxy, each EncodeFilter
consuming one 64 KiB socket read per event-loop turn (cfg5 data: 50 % repeats of the warm pool),
with and without the cross-connection Batcher; then the peer's DecodeFilters decoding those
pipes per turn.  Prints one JSON line: GiB/s of input through the filters (Python framing
included) and through the codec calls alone (host-to-host device calls).  usage: python tools/pipe_bench.py [N] [TURNS]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import pipe as P  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402
from pipe_harness import UUID_A, UUID_B, Proxy, Conn  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
turns = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ctx = w.Context(0)


class TimedBackend(P.DeviceBackend):
    """The device backend, with the wall time spent inside its codec calls."""
    spent = 0.0

    def _t(self, fn, *a):
        t0 = time.perf_counter()
        r = fn(*a)
        TimedBackend.spent += time.perf_counter() - t0
        return r

    def encode(self, *a):
        return self._t(super().encode, *a)

    def encode_many(self, *a):
        return self._t(super().encode_many, *a)

    def decode(self, *a):
        return self._t(super().decode, *a)

    def decode_many(self, *a):
        return self._t(super().decode_many, *a)


class NullWire(P.Filter):
    """A socket that keeps only the unsent bytes (the harness's Wire also logs everything)."""

    def __init__(self):
        super().__init__()
        self.q = bytearray()

    def consume(self, buf, flg=0):
        self.q += buf
        return True

    def flush(self, flg):
        pass


be = TimedBackend(ctx, 1 << 20)
warm = W.pool_warmup_buffers()
data = W.repeat_shard(n * turns, 0x5555).reshape(turns, n, -1)


def warm_store(store):
    w.XCodecEncoder(store).encode_batch(warm)


res = {"connections": n, "turns": turns, "read_bytes": W.BUF,
       "note": "each mode run twice, the second measured (the first pays one-time pinned/device "
               "allocations of the library's pool and page faults)"}
for batched in (True, True, False, False):
    a = Proxy(be, UUID_A, warm=warm_store, batched=batched)
    b = Proxy(be, UUID_B, batched=batched)
    # the peer's copy of A's cache holds the pool too (steady state: no <ASK>/<LEARN>)
    peer = be.new_store()
    warm_store(peer)
    b.registry.register(P.CodecCache(peer, UUID_A, 64))
    conns = [Conn(a, b) for _ in range(n)]
    for c in conns:
        c.ab = NullWire()
        c.a_enc.chain(c.ab)
    TimedBackend.spent = 0.0
    t0 = time.perf_counter()
    for t in range(turns):
        for i in range(n):
            assert conns[i].a_enc.consume(data[t, i].tobytes())
        a.end_turn()
    enc_s = time.perf_counter() - t0
    enc_dev = TimedBackend.spent
    TimedBackend.spent = 0.0
    # the peer decodes every pipe (frames only: one device decode call per turn)
    t0 = time.perf_counter()
    for c in conns:
        q = bytes(c.ab.q)
        c.ab.q.clear()
        assert c.b_dec.consume(q)
    b.end_turn()
    dec_s = time.perf_counter() - t0
    dec_dev = TimedBackend.spent
    ok = all(bytes(c.b_sink.data) == data[:, i].tobytes() for i, c in enumerate(conns))
    key = "batched" if batched else "unbatched"
    res[key] = {"encode_GiBs": round(n * turns * W.BUF / enc_s / 2**30, 3),
                "encode_ms_per_turn": round(enc_s / turns * 1e3, 3),
                "encode_codec_call_GiBs": round(n * turns * W.BUF / enc_dev / 2**30, 3),
                "decode_GiBs": round(n * turns * W.BUF / dec_s / 2**30, 3),
                "decode_codec_call_GiBs": round(n * turns * W.BUF / dec_dev / 2**30, 3),
                "device_calls": a.batcher.device_calls if batched else n * turns, "round_trip_ok": ok}
    for c in conns:
        c.a_enc.flush(0)
print(json.dumps(res))
