# round-3: the streaming tokenizer (decoder tests, then cfg4 A/B against the 1 KiB-window one),
# then the block-hash occupancy variant (cfg5 A/B against libxcodec_hip_b.so)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3t}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_pipe.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $out/dec_tests.log 2>&1 || { echo "dec tests rc $?"; tail -60 $out/dec_tests.log; exit 1; }
tail -1 $out/dec_tests.log
B_ENV="XC_DTOK_WIN=1" bash tools/ab_dec.sh ${1:-r3t}/abdec 3 30 || { echo "abdec failed"; exit 1; }
bash tools/ab.sh ${1:-r3t}/abocc 3 || { echo "ab failed"; exit 1; }
echo ok
