# End-to-end host path (bench.py's e2e_host_gibs): HEAD (a) against libxcodec_hip_b.so (b), one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5e2e}; mkdir -p $out
for r in 1 2; do
  for v in a b; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so; [ $v = b ] && lib=$PWD/wanproxy_amd/libxcodec_hip_b.so
    XC_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu --no-legs --no-live --no-decode --steps 10 > $out/$v$r.log 2>&1 || { tail -5 $out/$v$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/$v$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d.get('e2e_host_gibs'), d.get('e2e_ms'))"
  done
done
