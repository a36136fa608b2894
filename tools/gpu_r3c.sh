# round-3: duplicate-enter + C++ pipe tests, the C++ filter-path bench, then the whole GPU suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3c}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dup.py tests/test_gpu_pipe_cpp.py -x -v --timeout 200 --timeout-method thread > $out/new.log 2>&1 || { echo "new rc $?"; tail -40 $out/new.log; exit 1; }
timeout -k 10 300 python tools/pipe_bench_cpp.py 256 8 $out/pipe_bench_cpp.json > $out/pipe_bench.log 2>&1; echo "pipe bench rc $?"; tail -2 $out/pipe_bench.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/all.log 2>&1; echo "all rc $?"; tail -5 $out/all.log
