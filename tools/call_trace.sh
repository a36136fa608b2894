# HIP API + kernel trace of the single-call latency loop (tools/latency.py): where one 64 KiB
# consume's host time goes.  usage (GPU box): bash tools/call_trace.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$1
timeout -k 10 120 python3 tools/latency.py > gpurun_out/$1/latency.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d gpurun_out/$1/hip -o run \
    -- python3 tools/latency.py > gpurun_out/$1/latency_traced.log 2>&1
