# Several environment variants of the cfg5 bench on one box, alternating, ROUNDS rounds.
# usage (GPU box): bash tools/abn_env.sh TAG ROUNDS "name:ENV=v ENV2=v" ...   ("base:" = no env)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 20 ${AB_ARGS:-} > $out/$name.$r.log 2>&1 || { echo "bench $name rc $?"; tail -20 $out/$name.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/$name.$r.log').read().strip().splitlines()[-1]); print('$name', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
