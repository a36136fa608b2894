"""Run bench.py's cfg4 decode leg alone (for kernel traces and A/B of the decoder).
usage: python tools/dec_leg.py [steps]"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = w.Context(0)
args = types.SimpleNamespace(decode_streams=4096, steps=steps, warmup=2)
r = bench.bench_decode(args, ctx, W.pool_warmup_buffers())
print(json.dumps(r))
