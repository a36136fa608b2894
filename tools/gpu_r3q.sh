# round-3: the side stream's block hashing against the main stream's latency-bound kernels (A/B, cfg5)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3q}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_anchor.py -x -q --timeout 120 --timeout-method thread > $out/anchor.log 2>&1 || { echo "anchor rc $?"; tail -60 $out/anchor.log; exit 1; }
tail -1 $out/anchor.log
for r in 1 2 3; do
  for v in "base:" "prio:XC_STREAM_PRIO=1" "lds64:XC_BH_LDS=32" "lds80:XC_BH_LDS=48" "prio_lds64:XC_STREAM_PRIO=1 XC_BH_LDS=32"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > $out/ab_$name.$r.json 2>$out/ab_$name.$r.err || { echo "bench $name rc $?"; tail -20 $out/ab_$name.$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$out/ab_$name.$r.json').read().strip().splitlines()[-1]); print('$name', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
