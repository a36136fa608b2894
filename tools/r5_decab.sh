# cfg4 decode leg: HEAD (a) against libxcodec_hip_b.so (b) and HEAD with XC_STREAM_PRIO=0 (c), one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5da}; mkdir -p $out
for r in 1 2; do
  for v in a b c; do
    lib=$PWD/wanproxy_amd/libxcodec_hip.so; e=""
    [ $v = b ] && lib=$PWD/wanproxy_amd/libxcodec_hip_b.so
    [ $v = c ] && e="XC_STREAM_PRIO=0"
    env $e XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --only cfg4 --steps 200 --warmup 5 > $out/$v$r.log 2>&1 || { tail -5 $out/$v$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/$v$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
