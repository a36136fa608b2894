# round-3: side-stream block hashing chained back to back (against XC_BH_GATED=1, round 2's
# one-ahead); the whole GPU suite first
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3x}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
B_ENV="XC_BH_GATED=1" bash tools/ab.sh ${1:-r3x}/ab 3 || { echo "ab failed"; exit 1; }
timeout -k 10 200 python tools/host_overhead.py 20 > $out/host.json 2>&1 && cat $out/host.json
echo ok
