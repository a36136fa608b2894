# The round-3 final tree (_old/: git archive of 7e4ff8c, built here) against this tree, alternating
# cfg5 bench runs on one box.  usage (GPU box): bash tools/ab_r3.sh TAG [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-ab_r3}
mkdir -p $out
for r in $(seq 1 ${2:-3}); do
  (cd _old && timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > ../$out/r3_$r.log 2>&1) || exit 1
  python -c "import json; d=json.loads(open('$out/r3_$r.log').read().strip().splitlines()[-1]); print('r3', $r, d['value'])"
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 20 > $out/r4_$r.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$out/r4_$r.log').read().strip().splitlines()[-1]); print('r4', $r, d['value'])"
done
