# PMC instruction counters (two passes) of one bench leg: bash tools/pmc_leg.sh (on the GPU box; leg shard8) -> gpurun_out/r6sc/pmc_shard8.csv
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r6sc; mkdir -p $out
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/p$i -o run -- python3 bench.py --only shard8 --steps 20 > $out/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_table.py $out $out/pmc_shard8.csv > /dev/null && rm -rf $out/p1 $out/p2 && grep -E "k_scan|k_blockhash|k_emit|k_resolve|k_walk" $out/pmc_shard8.csv
