# A/B timing of the cfg4 decode leg (bench.py --only cfg4) on one box, alternating A and B as
# tools/ab.sh does.  usage (GPU box): bash tools/ab_dec.sh TAG [ROUNDS] [STEPS]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-abdec}
mkdir -p $out
for r in $(seq 1 ${2:-3}); do
  for v in a b; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so
    envs=""
    if [ $v = b ]; then
      if [ -n "$B_ENV" ]; then envs="$B_ENV"; else lib=$PWD/wanproxy_amd/${B_LIB:-libxcodec_hip_b.so}; fi
    fi
    env $envs XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --only cfg4 --steps ${3:-30} > $out/$v$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$out/$v$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
