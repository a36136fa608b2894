# Per-rank shard sizes of the 1/2/4/8-GPU cfg5 job on one GPU (bench.py --total 32768 / 16384 / 8192 / 4096).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5rks}; mkdir -p $out
for r in 1 2; do
  for tot in 32768 16384 8192 4096; do
    timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-legs --no-live --no-decode --steps 20 --total $tot > $out/t$tot.log 2>&1 || { tail -5 $out/t$tot.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/t$tot.log').read().strip().splitlines()[-1]); s=d['stats']; print('total', $tot, d['value'], d['ms_per_step'], s.get('sub_batches'), s.get('anchor_scans'), s.get('early_hashed'), d['verified_buffers'])"
  done
done
