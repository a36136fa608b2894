# Three-way cfg5 A/B on one box: libxcodec_hip.so (a), libxcodec_hip_b.so (b), libxcodec_hip_c.so (c),
# ROUNDS rounds, each variant's step times printed (min / median / max over the timed steps).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-ab3}; mkdir -p $out
for r in $(seq 1 ${2:-3}); do
  for v in a b c; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so
    [ $v = b ] && lib=$PWD/wanproxy_amd/libxcodec_hip_b.so
    [ $v = c ] && lib=$PWD/wanproxy_amd/libxcodec_hip_c.so
    XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 20 > $out/$v$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$out/$v$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'])"
  done
done
