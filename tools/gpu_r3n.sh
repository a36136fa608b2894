# round-3: anchor scan tests, encode + full-size suites forced into anchor mode, the bench (auto and
# exact), a kernel trace of the auto bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3n}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_anchor.py -x -q --timeout 120 --timeout-method thread > $out/anchor.log 2>&1 || { echo "anchor rc $?"; tail -60 $out/anchor.log; exit 1; }
tail -1 $out/anchor.log
XC_SCAN=anchor timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_fullsize.py tests/test_gpu_dup.py -x -q --timeout 300 --timeout-method thread > $out/tests_anchor.log 2>&1 || { echo "suite(anchor) rc $?"; tail -60 $out/tests_anchor.log; exit 1; }
tail -1 $out/tests_anchor.log
timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 10 > $out/bench.json 2> $out/bench.err || { echo "bench rc $?"; tail -30 $out/bench.err; exit 1; }
tail -1 $out/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('auto', d['value'], d['kernel_ms_per_step'], d['stats']['anchor_scans'], d.get('decode',{}).get('value'), {k: v['value'] for k, v in d.get('other_configs', {}).items()})"
XC_SCAN=anchor timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-decode --steps 10 > $out/bench_anchor.json 2> $out/bench_anchor.err || { echo "bench anchor rc $?"; tail -30 $out/bench_anchor.err; exit 1; }
tail -1 $out/bench_anchor.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('anchor', d['value'], {k: v['value'] for k, v in d.get('other_configs', {}).items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 5 > $out/prof.log 2>&1 || { echo "prof rc $?"; tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1000:9.1f} us')
PY
