# round-3: recent-window model prefilter: dup / stream / pipe tests, the bench's e2e leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3j}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dup.py tests/test_gpu_stream.py tests/test_gpu_pipe.py tests/test_gpu_pipe_cpp.py tests/test_gpu_encode.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python bench.py --no-cpu --no-decode --no-legs > $out/bench.json 2> $out/bench.err; echo "bench rc $?"; tail -1 $out/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('e2e_host_gibs'), d.get('e2e_ms'))"
timeout -k 10 300 python tools/pipe_bench_cpp.py 256 8 $out/pipe_bench_cpp.json > $out/pipe_bench.log 2>&1; echo "pipe bench rc $?"; tail -1 $out/pipe_bench.log
