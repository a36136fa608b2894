# A/B of one bench leg (cfg2 / cfg3 / cfg4) under two environments, alternating runs.
# usage (GPU box): bash tools/leg_ab.sh TAG LEG ROUNDS "ENV_A" "ENV_B"   (ENV: VAR=value ..., or "-")
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; leg=$2; mkdir -p $out
for r in $(seq 1 $3); do
  for v in a b; do
    e="$4"; [ $v = b ] && e="$5"; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python bench.py --only $leg --steps 200 > $out/$v$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$out/$v$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
