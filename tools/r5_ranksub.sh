# Per-rank shard sizes of the 1/2/4/8-GPU cfg5 job on one GPU (bench.py --total 16384 / 8192 / 4096 at N=1)
# against the sub-batch bound, one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5rk}; mkdir -p $out
for tot in 16384 8192; do
  for v in - XC_SUB_MB=256 XC_SUB_MB=1024; do
    e="$v"; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-legs --no-live --no-decode --steps 20 --total $tot > $out/t$tot.log 2>&1 || { tail -5 $out/t$tot.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/t$tot.log').read().strip().splitlines()[-1]); s=d['stats']; print('total', $tot, '$v', d['value'], d['ms_per_step'], s.get('sub_batches'), s.get('anchor_scans'), s.get('early_hashed'))"
  done
done
