# round-3: deferred segment stores: the GPU suite, A/B against XC_NO_DEFER_SEG=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3k}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_all.log 2>&1 || { echo "all rc $?"; tail -40 $out/tests_all.log; exit 1; }
tail -2 $out/tests_all.log
for r in 1 2 3; do
  for mode in 0 1; do
    XC_NO_DEFER_SEG=$mode timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > $out/ab_$mode.$r.log 2>&1 || { echo "bench rc $?"; tail -20 $out/ab_$mode.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/ab_$mode.$r.log').read().strip().splitlines()[-1]); print('no_defer=$mode', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
