# round-3: C++ pipe parity + filter-path bench, dup tests, the bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3d}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dup.py tests/test_gpu_pipe_cpp.py tests/test_gpu_pipe.py tests/test_gpu_cpp.py -x -v --timeout 200 --timeout-method thread > $out/new.log 2>&1 || { echo "new rc $?"; tail -40 $out/new.log; exit 1; }
timeout -k 10 300 python tools/pipe_bench_cpp.py 256 8 $out/pipe_bench_cpp.json > $out/pipe_bench.log 2>&1; echo "pipe bench rc $?"; tail -2 $out/pipe_bench.log
timeout -k 10 300 python tools/pipe_bench.py 256 8 > $out/pipe_bench_py.log 2>&1; echo "py pipe bench rc $?"; tail -1 $out/pipe_bench_py.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err; echo "bench rc $?"; tail -1 $out/bench.json
timeout -k 10 600 python tools/bigcache.py 0 2000000 8000000 > $out/bigcache.log 2>&1; echo "bigcache rc $?"; tail -4 $out/bigcache.log
