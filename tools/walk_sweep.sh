cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wsw
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wsw/tests.log 2>&1 || exit 1
for b in 4 16 64; do XC_WALK_BPW=$b timeout -k 10 200 python bench.py --no-cpu --no-e2e --verify 4 > gpurun_out/wsw/b$b.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/wsw/b$b.log').read().strip().splitlines()[-1]); print($b, d['value'], d['kernel_ms_per_step'])"; done
