# Quick GPU iteration (on the GPU box): gpu tests, optional scan ablation sweep, a short bench.
# usage: bash tools/gpu_quick.sh TAG [abl]
set -e
tag=${1:-quick}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
if [ "$2" = "abl" ]; then
    for e in 0 4096 12288 24576; do
        timeout -k 10 120 python tools/scan_ablation.py 4096 $e >> $out/abl.log 2>&1
    done
fi
timeout -k 10 300 python bench.py --no-cpu --no-e2e > $out/bench.log 2>&1
python - $out/bench.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "scan avg ms", d["roofline"]["avg_launch_ms"], "frac", d["roofline"]["frac"])
print("kernels", d["kernel_ms_per_step"])
PY
