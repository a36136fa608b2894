# Host HIP API calls beside the kernel trace of the cfg2 leg (16 MiB one-sub-batch runs): where the
# host's turn between two runs goes (tools/host_gaps.py reads the two CSVs).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5c2}; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $out/tr -o run -- python3 bench.py --only cfg2 --steps 40 > $out/tr.log 2>&1 || { tail -5 $out/tr.log; exit 1; }
find $out/tr -name '*.csv' | head -20
echo ok
