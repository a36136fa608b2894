# round-3: the duplicate-enter tests, the stream / COSS / fuzz suites, then the whole GPU suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3b}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dup.py tests/test_gpu_stream.py tests/test_gpu_coss.py -x -v --timeout 120 --timeout-method thread > $out/dup.log 2>&1 || { echo "dup rc $?"; tail -30 $out/dup.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/all.log 2>&1; echo "all rc $?"; tail -5 $out/all.log
