# PMC passes for the scan's memory-path analysis (TA / TD / TCP / UTCL1), one group per run,
# over a one-step cfg5 bench.  usage (GPU box): bash tools/pmc_scan.sh OUTDIR
set -e
out=${1:-gpurun_out/pmc_scan}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $out
run() { timeout -s KILL 120 rocprofv3 --pmc $1 --output-format csv -d $out/$2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-decode --no-legs > $out/$2.log 2>&1; }
run "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" t1
run "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" t2
run "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum" t3
run "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD" t4
echo done
