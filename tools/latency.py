"""Host-to-host call latency of the drop-in entry points (one 64 KiB call each): how long one
proxy consume() would wait.  usage (GPU box): python tools/latency.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402


def timeit(f, n=20):
    f()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t0) / n * 1e3


ctx = w.Context(0)
cache = w.XCodecCache(ctx, 1 << 16)
buf = W.gen(9, 65536)
enc = w.XCodecEncoder(cache)
streams = enc.encode_batch([buf])
print("encode_batch 1 x 64 KiB  ms", round(timeit(lambda: enc.encode_batch([buf])), 3))
se = w.XCodecStreamEncoder(cache)
print("stream encode+flush 64 KiB ms", round(timeit(lambda: w.encode_streams([(se, buf, True)])), 3))
dec = w.XCodecDecoder(w.XCodecCache(ctx, 1 << 16))
print("decode_batch 1 stream     ms", round(timeit(lambda: dec.decode_batch(streams)), 3))
bufs = [W.gen(100 + i, 65536) for i in range(256)]
print("encode_batch 256 x 64 KiB ms", round(timeit(lambda: enc.encode_batch(bufs), 5), 3))
