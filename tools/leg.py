"""Run one BASELINE encode leg of bench.py alone (for kernel traces of small configurations).
usage: python tools/leg.py cfg2|cfg3 [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402

case = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ctx = w.Context(0)
if case == "cfg2":
    r = bench.bench_encode_leg(ctx, None, W.random_buffers(256), steps, "cfg2")
else:
    r = bench.bench_encode_leg(ctx, W.pool_warmup_buffers(), list(W.repeat_shard(4096, 0x77)), steps, "cfg3")
print(json.dumps(r))
