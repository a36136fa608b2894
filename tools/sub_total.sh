# Sub-batch size (XC_SUB_MB) against the per-GPU shard size of an N-GPU cfg5 run (--total 32768/N
# on one GPU), alternating.  usage (GPU box): bash tools/sub_total.sh TOTAL "SIZES" [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/sub_total
mkdir -p $out
t=$1
for r in $(seq 1 ${3:-2}); do
  for s in $2; do
    XC_SUB_MB=$s timeout -k 10 200 python bench.py --total $t --no-cpu --no-e2e --no-decode --verify 4 --steps 20 > $out/t$t.s$s.$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$out/t$t.s$s.$r.log').read().strip().splitlines()[-1]); print('total', $t, 'sub', $s, d['value'], d['ms_per_step'], d['stats']['sub_batches'], d['kernel_ms_per_step'])"
  done
done
