# round-3: tokenizer tests + A/B, COSS bench, filter-path benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3gh}
mkdir -p $out
bash tools/gpu_r3h.sh ${1:-r3gh}/h || exit 1
bash tools/gpu_r3g.sh ${1:-r3gh}/g
