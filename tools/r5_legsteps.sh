# Sensitivity of the short legs to the timed step count (20 as in the full bench vs 200), one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r5d; mkdir -p $out
for leg in cfg2 cfg4 cfg3; do
  for st in 20 200 20 200; do
    timeout -k 10 200 python bench.py --only $leg --steps $st --warmup 5 > $out/$leg.$st.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$out/$leg.$st.log').read().strip().splitlines()[-1]); print('$leg', $st, d['value'], d['ms_per_step'])"
  done
done
