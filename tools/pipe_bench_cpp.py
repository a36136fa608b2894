"""Filter-path throughput of the C++ filters (include/xcodec_pipe.hpp, tests/cpp/pipe_turns.cpp):
N connections of one proxy, each EncodeFilter consuming one 64 KiB read per event-loop turn (cfg5
data: 50 % repeats of the warm pool), the Batcher running each turn's calls as one device batch,
then the peer's DecodeFilters decoding every pipe; the same with one device call per consume (the
reference's pattern); and the reference's own, unchanged EncodeFilter over the drop-in facade
(oracle/_ref/filter_turns bench, built in the container from the reference's sources: one device call
per consume, xcodec_filter.cc:146-157).  Prints one JSON line.
usage: python tools/pipe_bench_cpp.py [N] [TURNS] [OUT]"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from wanproxy_amd import workloads as W  # noqa: E402
from pipe_harness import write_scenario  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
turns = int(sys.argv[2]) if len(sys.argv) > 2 else 8
data = W.repeat_shard(n * turns, 0x5555).reshape(turns, n, -1)
inputs = [[data[t, i] for t in range(turns)] for i in range(n)]
order = [list(range(n)) for _ in range(turns)]
res = {"connections": n, "turns": turns, "read_bytes": W.BUF, "host": "C++ (include/xcodec_pipe.hpp)"}
with tempfile.TemporaryDirectory() as d:
    for batched in (True, False):
        sc = os.path.join(d, "sc.bin")
        write_scenario(sc, W.pool_warmup_buffers(), order, inputs, batched=batched)
        r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "pipe_turns"), "bench", sc], capture_output=True,
                           text=True, timeout=600)
        if r.returncode:
            raise SystemExit(r.stdout + r.stderr)
        res["batched" if batched else "unbatched"] = json.loads(r.stdout.strip().splitlines()[-1])
    ref = os.path.join(ROOT, "oracle", "_ref", "filter_turns")
    if os.path.exists(ref):
        sc = os.path.join(d, "sc.bin")
        write_scenario(sc, W.pool_warmup_buffers(), order, inputs, batched=False)
        r = subprocess.run([ref, "bench", sc], capture_output=True, text=True, timeout=600)
        if r.returncode:
            raise SystemExit(r.stdout + r.stderr)
        res["reference_filter_unbatched"] = json.loads(r.stdout.strip().splitlines()[-1])
print(json.dumps(res))
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(json.dumps(res) + "\n")
