"""Host-path cost of one cross-connection batch: 256 connections x one 64 KiB read (cfg5 data),
through xc_encode_streams (Python wrapper and the C call alone) and xc_encode_batch_host, and the
decode of the result.  usage: python tools/stream_latency.py [N] [REPS]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402
from wanproxy_amd import xcodec as X  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = w.Context(0)
bufs = [np.ascontiguousarray(b) for b in W.repeat_buffers(n, 0x4242)]
res = {}


def best(fn):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3


cache = w.XCodecCache(ctx, 1 << 20)
w.XCodecEncoder(cache).encode_batch(W.pool_warmup_buffers())
encs = [X.XCodecStreamEncoder(cache) for _ in range(n)]
res["batch_host_ms"] = best(lambda: w.XCodecEncoder(cache).encode_batch(bufs))
if encs is not None:
    res["streams_py_ms"] = best(lambda: X.encode_streams([(e, b, True) for e, b in zip(encs, bufs)]))
lib = X.load_library()
lens = np.array([b.size for b in bufs], np.uint64)
flags = np.full(n, X.STREAM_FLUSH, np.uint32)
cap = 2 * lens + 16
off = np.zeros(n, np.uint64)
off[1:] = np.cumsum(cap)[:-1]
out = np.empty(int(cap.sum()), np.uint8)
olen = np.zeros(n, np.uint64)
if encs is not None:
    ea = (X._vp * n)(*[e.h for e in encs])
    pa = (C.c_void_p * n)(*[b.ctypes.data for b in bufs])
    res["streams_c_ms"] = best(lambda: X._check(lib.xc_encode_streams(ea, pa, lens, flags, n, out, off, cap, olen)))
enc = w.XCodecEncoder(cache).encode_batch(bufs)
res["decode_py_ms"] = best(lambda: w.XCodecDecoder(cache).decode_batch(enc))
res["MiB"] = n * 64 / 1024
print(json.dumps({k: round(v, 3) for k, v in res.items()}))
