# round-3: COSS encode throughput, filter-path benches, LOAD_MISS tests at HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3g}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_coss_loadmiss.py tests/test_gpu_pipe_cpp.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python tools/coss_bench.py 1024 6 1024 > $out/coss_bench.json 2> $out/coss_bench.err; echo "coss bench rc $?"; tail -1 $out/coss_bench.json; tail -3 $out/coss_bench.err
timeout -k 10 300 python tools/pipe_bench_cpp.py 256 8 $out/pipe_bench_cpp.json > $out/pipe_bench.log 2>&1; echo "pipe bench rc $?"; tail -2 $out/pipe_bench.log
timeout -k 10 300 python tools/pipe_bench.py 256 8 > $out/pipe_bench_py.log 2>&1; echo "py pipe bench rc $?"; tail -1 $out/pipe_bench_py.log
