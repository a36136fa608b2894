# Round check on the GPU box: gpu tests, the bench line, a kernel-trace profile of the bench
# (cfg5 + cfg4 decode + cfg2/cfg3 legs).  usage: bash tools/gpu_round.sh TAG [notest|nobench]
set -e
tag=${1:-round}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))" > $out/host.txt
cat /sys/fs/cgroup/cpu.max >> $out/host.txt 2>/dev/null || true
if [ "$2" != "notest" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
fi
if [ "$2" != "nobench" ]; then
    timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu --no-e2e --steps 10 > $out/trace.log 2>&1
fi
echo ok
