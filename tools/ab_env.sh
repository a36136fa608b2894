# cfg5 bench (or with LEG=cfg2|cfg3|shard8|cfg4 that leg) under several environments of one library
# (XC_LIB_PATH, default the in-tree one), interleaved round by round on one box.
# usage (GPU box): bash tools/ab_env.sh TAG ROUNDS "ENV" ...
# (ENV: VAR=value ... or "-"; ablation switches need a -DXC_ABLATIONS=1 build: tools/build_variant.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  i=0
  for e in "$@"; do
    i=$((i+1)); ee="$e"; [ "$e" = "-" ] && ee=""
    if [ -n "$LEG" ]; then
      env $ee timeout -k 10 200 python bench.py --only $LEG --steps 200 > $out/v$i.$r.log 2>&1 || exit 1
    else
      env $ee timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 20 ${AB_ARGS:-} > $out/v$i.$r.log 2>&1 || exit 1
    fi
    python -c "import json; d=json.loads(open('$out/v$i.$r.log').read().strip().splitlines()[-1]); print('v$i', '$e', $r, d['value'], d['ms_per_step'])"
  done
done
