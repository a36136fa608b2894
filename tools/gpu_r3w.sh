# round-3: the tail check enqueued behind the first pass; host time per step by phase
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3w}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_anchor.py tests/test_gpu_dup.py tests/test_gpu_encode.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 200 python tools/host_overhead.py 20 > $out/host.json 2>&1 || { echo "host rc $?"; tail -20 $out/host.json; exit 1; }
cat $out/host.json
XC_TAIL_LATE=1 timeout -k 10 200 python tools/host_overhead.py 20 > $out/host_late.json 2>&1 || { echo "host rc $?"; tail -20 $out/host_late.json; exit 1; }
cat $out/host_late.json
B_ENV="XC_TAIL_LATE=1" bash tools/ab.sh ${1:-r3w}/ab 3 || { echo "ab failed"; exit 1; }
echo ok
