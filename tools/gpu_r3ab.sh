# round-3: k_emit timing ablations in the diagnostic steps (XC_ABL_EMIT bits: 1 no segment store,
# 2 no wire payload copy, 4 no cache inserts, 8 no payload loads/stores)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3ab}
mkdir -p $out
for r in 1 2; do
for a in 0 1 2 4 8 12; do
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 10 --diag-env XC_ABL_EMIT=$a > $out/abl$a.$r.log 2>&1 || { echo "bench rc $?"; tail -20 $out/abl$a.$r.log; exit 1; }
  python -c "import json; d=json.loads(open('$out/abl$a.$r.log').read().strip().splitlines()[-1]); print('abl', $a, d['value'], d['kernel_ms_per_step'])"
done
done
