# Kernel + HIP API trace of the reference's unbatched EncodeFilter over the facade (the
# reference_filter_unbatched leg of tools/pipe_bench_cpp.py, 64 connections x 4 turns).
# usage (GPU box): bash tools/ref_filter_trace.sh TAG   -> gpurun_out/TAG/hip/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1
mkdir -p gpurun_out/$tag
python3 - gpurun_out/$tag/sc.bin <<'PY'
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from wanproxy_amd import workloads as W
from pipe_harness import write_scenario
n, turns = 64, 4
data = W.repeat_shard(n * turns, 0x5555).reshape(turns, n, -1)
write_scenario(sys.argv[1], W.pool_warmup_buffers(), [list(range(n)) for _ in range(turns)],
               [[data[t, i] for t in range(turns)] for i in range(n)], batched=False)
PY
timeout -k 10 120 oracle/_ref/filter_turns bench gpurun_out/$tag/sc.bin > gpurun_out/$tag/plain.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/$tag/hip -o run \
    -- oracle/_ref/filter_turns bench gpurun_out/$tag/sc.bin > gpurun_out/$tag/trace.log 2>&1
