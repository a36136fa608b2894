# round-3: the anchor scan: its tests, the whole GPU suite forced into anchor mode,
# the default suite, the bench (auto) and an exact-scan A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3m}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_anchor.py -x -v --timeout 120 --timeout-method thread > $out/anchor.log 2>&1 || { echo "anchor rc $?"; tail -60 $out/anchor.log; exit 1; }
tail -3 $out/anchor.log
XC_SCAN=anchor timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_anchor.log 2>&1 || { echo "suite(anchor) rc $?"; tail -60 $out/tests_anchor.log; exit 1; }
tail -2 $out/tests_anchor.log
timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 10 > $out/bench.json 2> $out/bench.err || { echo "bench rc $?"; tail -30 $out/bench.err; exit 1; }
tail -1 $out/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('auto', d['value'], d['kernel_ms_per_step'], d['stats'], d.get('decode',{}).get('value'), {k: v['value'] for k, v in d.get('other_configs', {}).items()})"
XC_SCAN=exact timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-decode --steps 10 > $out/bench_exact.json 2> $out/bench_exact.err || { echo "bench exact rc $?"; tail -30 $out/bench_exact.err; exit 1; }
tail -1 $out/bench_exact.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['value'], d['kernel_ms_per_step'], {k: v['value'] for k, v in d.get('other_configs', {}).items()})"
