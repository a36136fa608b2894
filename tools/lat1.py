import os, sys, time
import numpy as np
sys.path.insert(0, os.getcwd())
import wanproxy_amd as w
from wanproxy_amd import workloads as W
ctx = w.Context(0)
cache = w.XCodecCache(ctx, 1 << 16)
buf = W.gen(9, 65536)
enc = w.XCodecEncoder(cache)
for _ in range(5): enc.encode_batch([buf])
t0 = time.perf_counter()
for _ in range(50): enc.encode_batch([buf])
print("encode_batch", (time.perf_counter() - t0) / 50 * 1e3)
