# A/B on one box of the cfg5 bench (tools/ab.sh) and of the short legs: the library (a) against
# wanproxy_amd/libxcodec_hip_b.so (b), alternating.  usage (GPU box): bash tools/ab_legs.sh TAG ROUNDS LEG...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for leg in "$@"; do
  for r in $(seq 1 $rounds); do
    for v in a b; do
      lib=$PWD/wanproxy_amd/libxcodec_hip.so
      [ $v = b ] && lib=$PWD/wanproxy_amd/${B_LIB:-libxcodec_hip_b.so}
      if [ $leg = cfg5 ]; then
        XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 20 > $out/$leg$v$r.log 2>&1 || exit 1
      else
        XC_LIB_PATH=$lib timeout -k 10 200 python bench.py --only $leg --steps 200 > $out/$leg$v$r.log 2>&1 || exit 1
      fi
      python -c "import json; d=json.loads(open('$out/$leg$v$r.log').read().strip().splitlines()[-1]); print('$leg', '$v', $r, d['value'], d['ms_per_step'])"
    done
  done
done
