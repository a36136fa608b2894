# round-3: k_aprop groups per workgroup (cfg5) and k_dres1 waves per stream (cfg4), library variants
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3ac}
mkdir -p $out
for r in 1 2; do
  for v in base ap16 ap4; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so; [ $v != base ] && lib=$PWD/wanproxy_amd/libxcodec_hip_$v.so
    XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > $out/$v.$r.log 2>&1 || { echo "bench $v rc $?"; tail -20 $out/$v.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/$v.$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['kernel_ms_per_step'])"
  done
  for v in base dr8 dr16; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so; [ $v != base ] && lib=$PWD/wanproxy_amd/libxcodec_hip_$v.so
    XC_LIB_PATH=$lib timeout -k 10 200 python tools/dec_leg.py 30 > $out/dec_$v.$r.log 2>&1 || { echo "dec $v rc $?"; tail -20 $out/dec_$v.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/dec_$v.$r.log').read().strip().splitlines()[-1]); print('dec_$v', $r, d['value'], d['ms_per_step'])"
  done
done
