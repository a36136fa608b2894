# COSS: GPU tests of the COSS and replay paths, then tools/coss_bench.py with the replay's phase profile.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5coss}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "coss or dup or live or window" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
XC_REPLAY_PROF=1 timeout -k 10 600 python tools/coss_bench.py > $out/coss_bench.log 2>&1 || { tail -30 $out/coss_bench.log; exit 1; }
grep -v "^replay" $out/coss_bench.log | tail -2
grep "^replay" $out/coss_bench.log | tail -4
