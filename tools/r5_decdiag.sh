# Which earlier bench leg slows the cfg4 decode leg (full bench 0.30 ms/step against 0.18 alone), one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5dd}; mkdir -p $out
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $out/$n.log 2>&1 || { tail -5 $out/$n.log; exit 1; }
  python -c "import json; d=json.loads(open('$out/$n.log').read().strip().splitlines()[-1]); x=d.get('decode', d); print('$n', x.get('value'), x.get('ms_per_step'), x.get('steps'))"; }
run only200 --only cfg4 --steps 200 --warmup 5
run cfg5_dec --no-cpu --no-e2e --no-legs --no-live --steps 20 --warmup 5
run cfg5_live_dec --no-cpu --no-e2e --no-legs --steps 20 --warmup 5
run cfg5_e2e_dec --no-cpu --no-legs --no-live --steps 20 --warmup 5
