cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/pmcw; mkdir -p $out
run() { XC_WALK_BPW=4 timeout -k 10 240 rocprofv3 --pmc $1 --kernel-include-regex "k_walk" --output-format csv -d $out/$2 -o run -- python3 bench.py --steps 1 --warmup 0 --verify 0 --no-cpu --no-e2e > $out/$2.log 2>&1; }
run "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p1 || exit 1
run "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS" p2 || exit 1
echo done
