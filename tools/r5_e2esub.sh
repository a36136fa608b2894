# End-to-end host path (e2e_host_gibs) against the sub-batch byte bound (XC_SUB_MB), one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5e2s}; mkdir -p $out
for r in 1 2; do
  for v in - XC_SUB_MB=512 XC_SUB_MB=256 XC_SUB_MB=128; do
    e="$v"; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py --no-cpu --no-legs --no-live --no-decode --steps 10 > $out/r$r.log 2>&1 || { tail -5 $out/r$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/r$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d.get('e2e_host_gibs'), d.get('e2e_ms'))"
  done
done
