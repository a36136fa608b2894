# Kernel + HIP API trace of one bench leg (host launch timeline beside the device's; no PMC).
# usage (GPU box): bash tools/hiptrace.sh TAG BENCH_ARGS...   -> gpurun_out/TAG/hip/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/$tag/hip -o run \
    -- python3 bench.py "$@" > gpurun_out/$tag/hiptrace.log 2>&1
