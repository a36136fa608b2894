# round-3: block hashing in passes of 512 anchors at 4 workgroups per CU, tokenizer without
# register copies: anchor / decode GPU tests, then cfg5 A/B against HEAD's library and cfg4 A/B
# against the 1 KiB-window tokenizer
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3u}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_anchor.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_encode.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
XC_SCAN=anchor timeout -k 10 300 python -u -m pytest tests/test_gpu_anchor.py tests/test_gpu_encode.py -x -q --timeout 200 --timeout-method thread > $out/tests_anchor.log 2>&1 || { echo "anchor tests rc $?"; tail -60 $out/tests_anchor.log; exit 1; }
tail -1 $out/tests_anchor.log
B_ENV="XC_DTOK_WIN=1" bash tools/ab_dec.sh ${1:-r3u}/abdec 3 30 || { echo "abdec failed"; exit 1; }
bash tools/ab.sh ${1:-r3u}/ab 3 || { echo "ab failed"; exit 1; }
echo ok
