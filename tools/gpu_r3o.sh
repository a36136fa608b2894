# round-3: anchor-path A/B on one box: block-load modes and a smaller first sub-batch (cfg5, 3 rounds)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3o}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_anchor.py -x -q --timeout 120 --timeout-method thread > $out/anchor.log 2>&1 || { echo "anchor rc $?"; tail -60 $out/anchor.log; exit 1; }
tail -1 $out/anchor.log
for r in 1 2 3; do
  for v in "base:" "nt:XC_BH_NT=1" "first128:XC_FIRST_SUB_MB=128" "first256:XC_FIRST_SUB_MB=256"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > $out/ab_$name.$r.json 2>$out/ab_$name.$r.err || { echo "bench $name rc $?"; tail -20 $out/ab_$name.$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$out/ab_$name.$r.json').read().strip().splitlines()[-1]); print('$name', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
