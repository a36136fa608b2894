# round-3: split emit A/B (XC_NO_SPLIT), LOAD_MISS tests, the whole GPU suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3f}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_coss_loadmiss.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > $out/tests_a.log 2>&1 || { echo "tests_a rc $?"; tail -60 $out/tests_a.log; exit 1; }
tail -2 $out/tests_a.log
for r in 1 2 3; do
  for mode in 0 1; do
    XC_NO_SPLIT=$mode timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > $out/ab_$mode.$r.log 2>&1 || { echo "bench rc $?"; tail -20 $out/ab_$mode.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/ab_$mode.$r.log').read().strip().splitlines()[-1]); print('no_split=$mode', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_all.log 2>&1; echo "all rc $?"; tail -3 $out/tests_all.log
