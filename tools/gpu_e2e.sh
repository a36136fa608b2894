cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2e1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e2e1/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/e2e1/bench.log 2>&1
