# Kernel timelines of the cfg3 and cfg4 legs (rocprofv3 --kernel-trace), the last steps of each.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5lt}; mkdir -p $out
for leg in cfg3 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$leg -o run -- python3 bench.py --only $leg --steps 40 > $out/$leg.log 2>&1 || exit 1
  python3 tools/timeline.py $out/$leg/run_kernel_trace.csv 40 > $out/timeline_$leg.txt || exit 1
done
echo ok
