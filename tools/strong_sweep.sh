# Per-GPU work of the N-GPU strong-scaling runs, emulated on one GPU: --total 32768/N buffers.
# usage (GPU box): bash tools/strong_sweep.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-strong}
mkdir -p $out
for t in 32768 16384 8192 4096; do
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --verify 4 --total $t --steps 20 > $out/t$t.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$out/t$t.log').read().strip().splitlines()[-1]); print($t, d['value'], d['ms_per_step'], d['stats']['sub_batches'], d['kernel_ms_per_step'])"
done
