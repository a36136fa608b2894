"""Host time of a cfg5 bench step, by phase: restore_async, submit (everything up to the first
asynchronous pass enqueued), wait (the control words and encode_finish), against the device step.
usage (GPU box): python tools/host_overhead.py [steps] [cfg2]  (cfg2: 256 random 64 KiB buffers, empty cache)"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cfg2 = len(sys.argv) > 2 and sys.argv[2] == "cfg2"
    ctx = w.Context(0)
    shard = np.stack(W.random_buffers(256)) if cfg2 else W.repeat_shard(32768, 0x5555, 0, 1)
    n = shard.shape[0]
    cache = w.XCodecCache(ctx, W.POOL_SEGMENTS + n * (W.BUF // 2048 + 1) + 1024)
    if not cfg2:
        w.XCodecEncoder(cache).encode_batch(W.pool_warmup_buffers())
    cache.snapshot()
    plan = w.EncodePlan(cache, np.full(n, W.BUF, dtype=np.uint64))
    plan.set_completion(True)
    d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
    d_in[:n * W.BUF] = torch.from_numpy(shard.reshape(-1)).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ph = {"restore": [], "submit": [], "wait": [], "step": []}
    for i in range(steps + 3):
        t0 = time.perf_counter()
        cache.restore_async()
        t1 = time.perf_counter()
        plan.submit(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
        t2 = time.perf_counter()
        plan.wait()
        t3 = time.perf_counter()
        if i >= 3:
            ph["restore"].append(t1 - t0)
            ph["submit"].append(t2 - t1)
            ph["wait"].append(t3 - t2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        cache.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / steps * 1e3
    print(json.dumps({k: round(float(np.median(v)) * 1e3, 4) for k, v in ph.items() if v} | {"step_ms": round(step_ms, 4)}))


if __name__ == "__main__":
    main()
