# A/B of the cfg2 and cfg3 legs: libxcodec_hip.so (a) against libxcodec_hip_b.so (b), alternating, one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5legab}; mkdir -p $out
for r in 1 2 3; do
  for leg in cfg2 cfg3; do
    for v in a b; do
      lib=$PWD/wanproxy_amd/libxcodec_hip.so; [ $v = b ] && lib=$PWD/wanproxy_amd/libxcodec_hip_b.so
      XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --only $leg --steps 200 > $out/$leg.$v$r.log 2>&1 || { tail -5 $out/$leg.$v$r.log; exit 1; }
      python -c "import json; d=json.loads(open('$out/$leg.$v$r.log').read().strip().splitlines()[-1]); print('$leg', '$v', $r, d['value'], d['ms_per_step'])"
    done
  done
done
