cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wt
XC_WALK_BPW=4 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wt/trace -o run -- python3 bench.py --no-cpu --no-e2e --steps 2 --warmup 1 --verify 0 > gpurun_out/wt/log 2>&1
