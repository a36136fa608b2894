# Anchor index against the exact scan on 4096-buffer runs (cfg3, and the N=8 per-rank shard of cfg5), one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5cross}; mkdir -p $out
B="--no-cpu --no-e2e --no-decode --no-legs --no-live --steps 50 --total 4096"
for r in 1 2; do
  for v in "-" "XC_SCAN=anchor" "XC_SCAN=anchor XC_SUB_MB=128"; do
    e="$v"; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py $B > $out/s8.$r.log 2>&1 || { tail -5 $out/s8.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/s8.$r.log').read().strip().splitlines()[-1]); print('shard8', '$v', d['value'], d['ms_per_step'], d['stats'].get('sub_batches'), d['stats'].get('anchor_scans'))"
    env $e timeout -k 10 300 python bench.py --only cfg3 --steps 200 --warmup 5 > $out/c3.$r.log 2>&1 || { tail -5 $out/c3.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/c3.$r.log').read().strip().splitlines()[-1]); print('cfg3', '$v', d['value'], d['ms_per_step'])"
  done
done
