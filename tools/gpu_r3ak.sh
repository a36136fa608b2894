# round-3: k_aprop with 1 group per workgroup (library variant) and non-temporal block-hash loads
# (XC_BH_NT=1), against HEAD, alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3ak}
mkdir -p $out
for r in 1 2 3; do
  for v in base ap1 nt; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so; envs=""
    [ $v = ap1 ] && lib=$PWD/wanproxy_amd/libxcodec_hip_ap1.so
    [ $v = nt ] && envs="XC_BH_NT=1"
    env $envs XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > $out/$v.$r.log 2>&1 || { echo "bench $v rc $?"; tail -20 $out/$v.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/$v.$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
