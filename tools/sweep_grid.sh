cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/grid
mkdir -p $out
for g in 0 224 192 160 128; do
  for r in 1 2; do
    XC_SCAN_GRID=$g timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > $out/g${g}_$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$out/g${g}_$r.log').read().strip().splitlines()[-1]); print('$g', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
