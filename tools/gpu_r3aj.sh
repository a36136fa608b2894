# round-3: decoder cache inserts beside the emit (against XC_DCOMMIT_SERIAL=1), decoding tests
# first; cfg3 leg with the cache enters in k_insert against XC_EMIT_INSERT=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3aj}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_pipe.py tests/test_gpu_pipe_cpp.py tests/test_gpu_coss.py tests/test_gpu_dup.py tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
B_ENV="XC_DCOMMIT_SERIAL=1" bash tools/ab_dec.sh ${1:-r3aj}/abdec 3 30 || { echo "abdec failed"; exit 1; }
B_ENV="XC_EMIT_INSERT=1" bash tools/ab_leg.sh ${1:-r3aj}/abcfg3 cfg3 3 || { echo "ab leg failed"; exit 1; }
echo ok
