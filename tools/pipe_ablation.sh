# Scan ablation modes inside the real pipeline (timing only; XC_SCAN_ABLATION, outputs wrong).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pabl
for m in 0 2 1 3 4 5; do XC_SCAN_ABLATION=$m timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --verify 0 --steps 5 --warmup 1 > gpurun_out/pabl/m$m.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/pabl/m$m.log').read().strip().splitlines()[-1]); print($m, d['value'], d['kernel_ms_per_step'])"; done
