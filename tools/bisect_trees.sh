# cfg5 bench of several source trees (git archives built in-tree: _old = round 3's final, _bis_<commit>)
# and of this tree, one run each per round, on one box.  usage (GPU box): bash tools/bisect_trees.sh TAG ROUNDS DIR...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for r in $(seq 1 $rounds); do
  for d in . "$@"; do
    n=$(basename $d); [ "$d" = . ] && n=head
    extra=""
    grep -q -- "--no-live" $d/bench.py && extra="--no-live"
    (cd $d && timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs $extra --steps 20 > $GRAFT_REPO_ROOT/$out/${n}_$r.log 2>&1) || { echo "$n failed"; tail -5 $out/${n}_$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/${n}_$r.log').read().strip().splitlines()[-1]); print('$n', $r, d['value'])"
  done
done
