# round-3: emit payload wire chunks by DPP shift (in-tree) against the baseline (b) and against
# EMIT_PAY=4 (c); encoder GPU tests first
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3v}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_fullsize.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
bash tools/ab.sh ${1:-r3v}/ab_b 3 || { echo "ab failed"; exit 1; }
B_LIB=libxcodec_hip_c.so bash tools/ab.sh ${1:-r3v}/ab_c 2 || { echo "ab c failed"; exit 1; }
echo ok
