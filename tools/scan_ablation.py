"""Time the encode scan kernel in ablation modes on a cfg3-shaped 4096-buffer batch."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
extra = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # random 64 KiB buffers encoded into the cache first
ctx = w.Context(0)
shard = W.repeat_shard(n, 0x5555)
pool = W.pool()
cache = w.XCodecCache(ctx, W.POOL_SEGMENTS + (n + extra) * 33 + 1024)
w.XCodecEncoder(cache).encode_batch([pool[i:i + W.BUF] for i in range(0, len(pool), W.BUF)])
for s in range(0, extra, 4096):
    k = min(4096, extra - s)
    rnd = W.gen(0xABC0 + s, k * W.BUF).reshape(k, W.BUF)
    w.XCodecEncoder(cache).encode_batch([rnd[i] for i in range(k)])
print(f"cache entries {len(cache)}")
plan = w.EncodePlan(cache, np.full(n, W.BUF, np.uint64))
d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
d_in[:n * W.BUF] = torch.from_numpy(shard.reshape(-1)).cuda()
torch.cuda.synchronize()
lib = w.load_library()
lib.xc__scan_ablation.restype = C.c_double
lib.xc__scan_ablation.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
for mode, name in [(2, "loads+block sums"), (1, "hash, no filter"), (3, "hash+filter, no queue"), (4, "queue appends only"), (5, "L2 filter, no exact"), (0, "full")]:
    us = lib.xc__scan_ablation(plan.h, d_in.data_ptr(), mode, 20)
    print(f"mode {mode} {name:18s} {us:8.1f} us  {n * W.BUF / us / 1e3:7.1f} GB/s")
