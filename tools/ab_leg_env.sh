# A/B of one bench leg under an environment setting (on the GPU box).
# usage: B_ENV="VAR=value" bash tools/ab_leg_env.sh cfg2|cfg3 [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in $(seq 1 ${2:-3}); do
  for v in a b; do
    envs=""; [ $v = b ] && envs="$B_ENV"
    r_json=$(env $envs timeout -k 10 120 python tools/leg.py $1 100 2>/dev/null | tail -1) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print('$v', $r, d['value'], d['ms_per_step'])" "$r_json"
  done
done
