# Sub-batch size on 4096-buffer runs (the N=8 per-rank shard of cfg5 and cfg3), exact scan, one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5sub}; mkdir -p $out
B="--no-cpu --no-e2e --no-decode --no-legs --no-live --steps 100 --total 4096"
for r in 1 2; do
  for v in "-" "XC_SUB_MB=128" "XC_SUB_MB=96" "XC_SUB_MB=64"; do
    e="$v"; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py $B > $out/s8.$r.log 2>&1 || { tail -5 $out/s8.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/s8.$r.log').read().strip().splitlines()[-1]); print('shard8', '$v', d['value'], d['ms_per_step'], d['stats'].get('sub_batches'), d['stats'].get('anchor_scans'), d['stats'].get('early_hashed'))"
  done
done
