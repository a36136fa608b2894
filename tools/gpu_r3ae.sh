# round-3: round 0 of the decoder's provider resolution inside the tokenizer (against
# XC_DTOK_NOHASH=1: k_dres1<true> as before); every GPU test that decodes first
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3ae}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_pipe.py tests/test_gpu_pipe_cpp.py tests/test_gpu_coss.py tests/test_gpu_dup.py tests/test_gpu_spill.py tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py tests/test_gpu_coss_loadmiss.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
B_ENV="XC_DTOK_NOHASH=1" bash tools/ab_dec.sh ${1:-r3ae}/abdec 3 30 || { echo "abdec failed"; exit 1; }
echo ok
