# Host API calls (hip runtime trace) beside the kernel trace of production steps: where the host's turn
# between a run's publication and the next run's first launches goes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5ht}; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $out/tr -o run -- python3 bench.py --no-cpu --no-e2e --no-live --no-legs --no-decode --steps 6 --tail-steps 3 > $out/tr.log 2>&1 || { tail -5 $out/tr.log; exit 1; }
ls $out/tr
