# A/B timing on one box: wanproxy_amd/libxcodec_hip.so (A) against B, alternating runs of the cfg5
# bench.  B is wanproxy_amd/libxcodec_hip_b.so (an alternative build), or with B_ENV="VAR=value ..."
# the same library under those environment variables.  usage (GPU box): bash tools/ab.sh TAG [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-ab}
mkdir -p $out
for r in $(seq 1 ${2:-3}); do
  for v in a b; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so
    envs=""
    if [ $v = b ]; then
      if [ -n "$B_ENV" ]; then envs="$B_ENV"; else lib=$PWD/wanproxy_amd/${B_LIB:-libxcodec_hip_b.so}; fi
    fi
    env $envs XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 20 ${AB_ARGS:-} > $out/$v$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$out/$v$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
