# round-3 check: COSS tests (statistics), the counter list for the scan's TA/TD/TCP analysis
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r3a
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_coss.py -x -v --timeout 200 --timeout-method thread > $out/coss.log 2>&1; echo "coss rc $?"
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1; echo "list rc $?"
grep -E "^\s*(TA_|TD_|TCP_|SQ_INSTS|SQ_INST_CYCLES|SQ_WAIT)" $out/counters.txt | head -100 > $out/ta.txt || true
