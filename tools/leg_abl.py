"""Timing of one encode leg with its output check switched off (diagnostic only: timing ablations,
-DXC_ABLATIONS=1 builds via XC_LIB_PATH, give wrong bytes on purpose; bench.py itself always checks).
usage: python tools/leg_abl.py cfg2|cfg3 [STEPS]   (env: XC_LIB_PATH, XC_ABL_EMIT, XC_ABL_BH, ...)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402

bench.verify_outputs = lambda *a, **k: {"verified_buffers": 0, "verified_against": "none (timing diagnostic)"}
leg = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
ctx = w.Context(0)
if leg == "cfg2":
    r = bench.bench_encode_leg(ctx, None, W.random_buffers(256), steps, None)
else:
    r = bench.bench_encode_leg(ctx, W.pool_warmup_buffers(), list(W.repeat_shard(4096, 0x77)), steps, None)
print(json.dumps({"leg": leg, "value": r["value"], "ms_per_step": r["ms_per_step"],
                  "env": {k: v for k, v in os.environ.items() if k.startswith("XC_")}}))
