# One pytest selection against the library of HEAD's sources (libxcodec_hip.so) and against an
# alternative build (libxcodec_hip_b.so, e.g. tools/build_commit.sh): does a regression test catch
# what the fix fixes?  usage (GPU box): bash tools/ab_test.sh TAG PYTEST_K_EXPR
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:?tag}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "$2" > $out/a.log 2>&1
echo "a (HEAD) rc $?"; tail -1 $out/a.log
XC_LIB_PATH=$PWD/wanproxy_amd/libxcodec_hip_b.so timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "$2" > $out/b.log 2>&1
echo "b rc $?"; tail -1 $out/b.log
exit 0
