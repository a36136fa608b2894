# One GPU check: gpu tests, bench, kernel-trace profile of a short bench, into gpurun_out/$1.
# usage (on the GPU box): bash tools/gpu_check.sh TAG [notest]
set -e
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "$2" != "notest" ]; then
    timeout -k 10 400 python -m pytest tests -m gpu -x -q > $out/tests.log 2>&1
fi
timeout -k 10 300 python bench.py > $out/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 5 --warmup 1 > $out/prof_bench.log 2>&1
echo ok
