cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
for e in 0 4096 12288 24576; do timeout -k 10 120 python tools/scan_ablation.py 4096 $e >> gpurun_out/abl/abl.log 2>&1 || exit 1; done
