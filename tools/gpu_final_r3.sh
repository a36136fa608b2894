# round-3 final profile set at HEAD: whole GPU suite, FETCH_SIZE / WRITE_SIZE passes -> the stamped
# traffic record (into profiles/r03 so the bench line carries it), the bench line, rocprofv3
# kernel-trace stats of the bench command.  usage (GPU box): bash tools/gpu_final_r3.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3final}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke rc $?"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
run() { timeout -s KILL 240 rocprofv3 --pmc $1 --output-format csv -d $out/pmc/$2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-decode --no-legs > $out/pmc_$2.log 2>&1 || { echo "pmc $2 rc $?"; tail -5 $out/pmc_$2.log; exit 1; }; }
run "FETCH_SIZE" p3
run "WRITE_SIZE" p4
alg=$(python3 -c "import json; print(json.loads(open('profiles/r03/bench_r3s.json').read())['roofline']['alg_bytes_per_step'])")
python3 tools/pmc_traffic.py $out/pmc $out/pmc_traffic_cfg5.json 4 $alg > $out/pmc_traffic.log 2>&1 || { echo "pmc_traffic failed"; cat $out/pmc_traffic.log; exit 1; }
cp $out/pmc_traffic_cfg5.json profiles/r03/pmc_traffic_cfg5.json
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc $?"; tail -30 $out/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('cfg5', d['value'], d['roofline']['frac'], d['roofline']['traffic_over_alg'], 'cfg2', d['other_configs']['cfg2']['value'], 'cfg3', d['other_configs']['cfg3']['value'], 'dec', d['decode']['value'], 'e2e', d['e2e_host_gibs'], 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu --no-e2e --steps 10 > $out/trace.log 2>&1 || { echo "trace rc $?"; tail -20 $out/trace.log; exit 1; }
echo ok
