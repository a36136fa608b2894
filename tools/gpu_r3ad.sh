# round-3: k_aprop groups per workgroup (cfg5), library variants (grid from the same constant)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3ad}
mkdir -p $out
for r in 1 2; do
  for v in base ap4 ap2; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so; [ $v != base ] && lib=$PWD/wanproxy_amd/libxcodec_hip_$v.so
    XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --steps 20 > $out/$v.$r.log 2>&1 || { echo "bench $v rc $?"; tail -20 $out/$v.$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/$v.$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['kernel_ms_per_step'])"
  done
done
