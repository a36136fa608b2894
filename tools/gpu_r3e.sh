# round-3: COSS lookups that miss with side effects, replay-engine users, the C++ filter bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3e}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_coss_loadmiss.py tests/test_gpu_coss.py tests/test_gpu_dup.py tests/test_gpu_stream.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 python tools/pipe_bench_cpp.py 256 8 $out/pipe_bench_cpp.json > $out/pipe_bench.log 2>&1; echo "pipe bench rc $?"; tail -2 $out/pipe_bench.log
