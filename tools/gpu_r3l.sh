# round-3 (re-entry): the GPU suite and the bench line at HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3l}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_all.log 2>&1 || { echo "all rc $?"; tail -40 $out/tests_all.log; exit 1; }
tail -2 $out/tests_all.log
timeout -k 10 300 python bench.py --no-cpu > $out/bench.json 2> $out/bench.err; echo "bench rc $?"; tail -1 $out/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_per_step'], d.get('decode',{}).get('value'), {k: v['value'] for k, v in d.get('other_configs', {}).items()}, d.get('e2e_host_gibs'))"
