# round-3: winnowed anchor lookups (least-ranked key anchor; k_aprop looks up only anchors that can
# be a window's key anchor) against XC_APROP_THIN=0; anchor tests, the suite with every eligible run
# anchor-scanned, the whole suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3ag}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_anchor.py -x -q --timeout 200 --timeout-method thread > $out/anchor.log 2>&1 || { echo "anchor rc $?"; tail -60 $out/anchor.log; exit 1; }
tail -1 $out/anchor.log
XC_SCAN=anchor timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_anchor.log 2>&1 || { echo "tests anchor rc $?"; tail -60 $out/tests_anchor.log; exit 1; }
tail -1 $out/tests_anchor.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
B_ENV="XC_APROP_THIN=0" bash tools/ab.sh ${1:-r3ag}/ab 3 || { echo "ab failed"; exit 1; }
echo ok
