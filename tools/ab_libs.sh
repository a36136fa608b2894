# A/B/C... on one box: several builds of the library (wanproxy_amd/libxcodec_hip_<name>.so; "main" is
# libxcodec_hip.so), interleaved round by round, on the cfg5 bench or a leg.
# usage (GPU box): bash tools/ab_libs.sh TAG ROUNDS LEG NAME...   (LEG: cfg5, cfg2, cfg3, shard8, cfg4)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; rounds=$2; leg=$3; shift 3
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    lib=$PWD/wanproxy_amd/libxcodec_hip_$v.so
    [ $v = main ] && lib=$PWD/wanproxy_amd/libxcodec_hip.so
    if [ $leg = cfg5 ]; then
      XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 20 > $out/$leg.$v.$r.log 2>&1 || exit 1
    else
      XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --only $leg --steps 200 > $out/$leg.$v.$r.log 2>&1 || exit 1
    fi
    python -c "import json; d=json.loads(open('$out/$leg.$v.$r.log').read().strip().splitlines()[-1]); print('$leg', '$v', $r, d['value'], d['ms_per_step'])"
  done
done
