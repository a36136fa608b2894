# Round profile set (on the GPU box): bench line, rocprofv3 kernel-trace stats of the same
# command, PMC passes for HBM traffic.  usage: bash tools/profile_round.sh OUTDIR
set -e
out=${1:-gpurun_out/prof_round}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > $out/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu --no-e2e > $out/trace.log 2>&1
bash tools/pmc_kernels.sh $out/pmc > $out/pmc.log 2>&1
echo done
