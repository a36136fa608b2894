# round-3: cache enters in k_insert (one wave per buffer) before the emit, against XC_EMIT_INSERT=1
# (inside the emit workgroups); the whole GPU suite first
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3af}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
B_ENV="XC_EMIT_INSERT=1" bash tools/ab.sh ${1:-r3af}/ab 3 || { echo "ab failed"; exit 1; }
echo ok
