# PMC passes over the scan ablation kernels (k_scan<MODE>), one counter group per run.
# usage (on the GPU box): bash tools/pmc_ablation.sh OUTDIR [extra_cache_buffers]
set -e
out=${1:-gpurun_out/pmcabl}
extra=${2:-0}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $out
run() { timeout -k 10 240 rocprofv3 --pmc $1 --kernel-include-regex "k_scan" --output-format csv -d $out/$2 -o run -- python3 tools/scan_ablation.py 4096 $extra > $out/$2.log 2>&1; }
run "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p1
run "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA" p2
run "FETCH_SIZE" p3
echo done
