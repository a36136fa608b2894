"""cfg3 against caches holding millions of segments (a long-lived proxy's XCodecMemoryCache is
unbounded, xcodec/xcodec_cache.h:164).  For each size: the warm pool, then random segments up to the
size (cold encodes of random 64 KiB buffers generated on the device: every aligned block declared),
a snapshot; then cfg3 (4096 x 64 KiB, 50 % repeats of the pool, seed 0x77) with a restore per step.
The random segments never match cfg3's windows (a 64-bit hash collision aside), so every cfg3 buffer
still equals the oracle's digests for cfg3 on the pool alone: checked.  Prints one JSON line per size:
GiB/s, the scan's time per launch, the kernel breakdown and the filters' false-positive rates.
usage: python tools/bigcache.py [--scan auto|exact|anchor] [SEGMENTS ...] (default 0 2000000 8000000)
(the scan mode of the timed cfg3 plan; the fills run in the default mode)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402

args = sys.argv[1:]
scan = "auto"
if args[:1] == ["--scan"]:
    scan, args = args[1], args[2:]
sizes = [int(x) for x in args] or [0, 2_000_000, 8_000_000]
ctx = w.Context(0)
gold = np.load(os.path.join(ROOT, "tests", "golden", "fullsize_digests.npz"))
bufs = list(W.repeat_shard(4096, 0x77))
lens = np.array([b.size for b in bufs], np.uint64)
for target in sizes:
    cache = w.XCodecCache(ctx, W.POOL_SEGMENTS + target + 4096 * 33 + 65536)
    w.XCodecEncoder(cache).encode_batch(W.pool_warmup_buffers())
    t0 = time.perf_counter()
    fill_buffers = 16384  # 1 GiB of random 64 KiB buffers per run: 524288 segments
    fplan = None
    while len(cache) < W.POOL_SEGMENTS + target:
        left = W.POOL_SEGMENTS + target - len(cache)
        nb = min(fill_buffers, max(1, left // 32))
        if fplan is None or fplan_n != nb:
            if fplan is not None:
                fplan.close()
            fplan = w.EncodePlan(cache, np.full(nb, W.BUF, np.uint64))
            fplan_n = nb
            f_out = torch.empty(fplan.out_bytes, dtype=torch.uint8, device="cuda")
            f_len = torch.empty(nb, dtype=torch.int64, device="cuda")
        f_in = torch.randint(0, 256, (fplan.in_bytes,), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        fplan.run(f_in.data_ptr(), f_out.data_ptr(), f_len.data_ptr())
        del f_in
    if fplan is not None:
        fplan.close()
    fill_s = time.perf_counter() - t0
    keys = len(cache)
    fs = cache.filter_stats()
    cache.snapshot()
    plan = w.EncodePlan(cache, lens)
    plan.set_scan(scan)
    plan.set_completion(True)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + b.size] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(bufs), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step():
        cache.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    steps = 20
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    olen = d_len.cpu().numpy().astype(np.uint64)
    dig = W.arena_digests(d_out.cpu().numpy(), plan.out_off, olen)
    ok = bool(np.array_equal(olen, gold["cfg3_len"].astype(np.uint64)) and np.array_equal(dig, gold["cfg3_dig"]))
    plan.kernel_times(reset=True)
    plan.set_timing(True)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    plan.set_timing(False)
    kt = plan.kernel_times(reset=True)
    st = plan.stats()
    rec = {"cache_segments": keys, "scan": scan, "anchor_scans": int(st.anchor_scans),
           "anchor_fallbacks": int(st.anchor_fallbacks), "fill_s": round(fill_s, 1),
           "cfg3_GiBs": round(int(lens.sum()) / el / 2**30, 2),
           "ms_per_step": round(el * 1e3, 3), "scan_ms_per_launch": round(kt["ms"]["scan"] / max(1, kt["launches"]["scan"]), 4),
           "kernel_ms_per_step": {k: round(v / 3, 4) for k, v in kt["ms"].items()},
           "l1_fp": round(fs["l1_fp"], 4), "l2_fp": round(fs["l2_fp"], 4), "equals_oracle_cfg3": ok}
    print(json.dumps(rec), flush=True)
    plan.close()
    cache.close()
    del d_in, d_out, d_len
    torch.cuda.empty_cache()
