# Repeat the N=1 bench (no CPU leg / e2e) R times: bash tools/bench_rep.sh TAG R
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; mkdir -p $out
for i in $(seq 1 ${2:-3}); do
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-live --steps 20 --verify 0 > $out/b$i.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('$out/b$i.log').read().strip().splitlines()[-1]); print(d['value'], d['kernel_ms_per_step'])"
done
