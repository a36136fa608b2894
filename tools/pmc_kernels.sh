# PMC passes (one counter group per rocprofv3 run) over a short cfg5 bench run (every kernel).
# usage (on the GPU box): bash tools/pmc_kernels.sh OUTDIR
set -e
out=${1:-gpurun_out/pmc}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $out
run() { timeout -s KILL 240 rocprofv3 --pmc $1 --output-format csv -d $out/$2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-decode --no-legs > $out/$2.log 2>&1; }
run "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p1
run "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA" p2
run "FETCH_SIZE" p3
run "WRITE_SIZE" p4
echo done
