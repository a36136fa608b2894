# Quick GPU iteration: gpu tests (fail fast), then the bench without the CPU leg.
# usage: bash tools/gpu_quick2.sh TAG [notest]
set -e
tag=${1:-quick}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "$2" != "notest" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
fi
timeout -k 10 400 python bench.py --no-cpu > $out/bench.json 2> $out/bench.err
python - $out/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "frac", d["roofline"]["frac"], "verified", d["verified_buffers"])
print("kernels", d["kernel_ms_per_step"])
print("decode", d["decode"]["value"], d["decode"]["ms_per_step"])
for k, v in d["other_configs"].items(): print(k, v["value"], v["ms_per_step"], v["verified_buffers"])
PY
