# round-3: side-stream hashing started beside the first sub-batch's in-line hashing (XC_BH_EARLY=1):
# encode tests with it, cfg5 A/B; the filter-path benches at HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3ai}
mkdir -p $out
XC_BH_EARLY=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_fullsize.py tests/test_gpu_anchor.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
B_ENV="XC_BH_EARLY=1" bash tools/ab.sh ${1:-r3ai}/ab 3 || { echo "ab failed"; exit 1; }
timeout -k 10 300 python tools/pipe_bench_cpp.py 256 8 $out/pipe_bench_cpp.json > $out/pipe_bench.log 2>&1; echo "pipe bench rc $?"; tail -2 $out/pipe_bench.log
timeout -k 10 300 python tools/pipe_bench.py 256 8 > $out/pipe_bench_py.log 2>&1; echo "py pipe bench rc $?"; tail -1 $out/pipe_bench_py.log
echo ok
