# round-3: PMC passes of the anchor pipeline (cfg5, 1 step) and the anchor/exact crossover by batch size
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3p}
mkdir -p $out
run() { timeout -s KILL 120 rocprofv3 --pmc $1 --output-format csv -d $out/$2 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-e2e --no-decode --no-legs > $out/$2.log 2>&1 || { echo "pmc $2 rc $?"; tail -5 $out/$2.log; exit 1; }; }
run "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p1
run "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA" p2
run "TCC_HIT_sum TCC_MISS_sum" p3
run "FETCH_SIZE" p4
python3 tools/pmc_table.py $out $out/pmc_table.csv > /dev/null && python3 - $out/pmc_table.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keep = ["k_aprop", "k_blockhash", "k_emit", "k_tailcheck", "k_resolve", "k_blockpredict"]
for r in rows:
    if any(k in r["kernel"] for k in keep):
        print(r["kernel"][:40], {c: r[c] for c in r if c.startswith(("SQ_", "TCC", "FETCH")) and r[c]})
PY
for n in 4096 8192 16384; do
  for m in anchor exact; do
    XC_SCAN=$m timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 --total $n > $out/x_$m.$n.json 2>$out/x_$m.$n.err || { echo "bench $m $n rc $?"; tail -20 $out/x_$m.$n.err; exit 1; }
    python -c "import json; d=json.loads(open('$out/x_$m.$n.json').read().strip().splitlines()[-1]); print('$m', $n, d['value'], d['kernel_ms_per_step'])"
  done
done
