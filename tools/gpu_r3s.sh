# round-3 profile set at HEAD: GPU tests, the bench line, rocprofv3 kernel-trace stats of the
# bench command, FETCH_SIZE / WRITE_SIZE passes (one counter per run) -> traffic record
# usage (on the GPU box): bash tools/gpu_r3s.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3s}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc $?"; tail -30 $out/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('cfg5', d['value'], d['roofline']['frac'], 'cfg2', d['other_configs']['cfg2']['value'], 'cfg3', d['other_configs']['cfg3']['value'], 'dec', d['decode']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu --no-e2e --steps 10 > $out/trace.log 2>&1 || { echo "trace rc $?"; tail -20 $out/trace.log; exit 1; }
run() { timeout -s KILL 240 rocprofv3 --pmc $1 --output-format csv -d $out/pmc/$2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-decode --no-legs > $out/pmc_$2.log 2>&1 || { echo "pmc $2 rc $?"; tail -5 $out/pmc_$2.log; exit 1; }; }
run "FETCH_SIZE" p3
run "WRITE_SIZE" p4
echo ok
