# A/B/... timing on one box: alternating runs of the cfg5 bench over several library builds.
# usage (GPU box): bash tools/abn.sh TAG ROUNDS lib_a.so lib_b.so ...   (paths under wanproxy_amd/)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    XC_LIB_PATH=$PWD/wanproxy_amd/$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode ${AB_ARGS:---no-legs} --steps 20 > $out/$lib.$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('$out/$lib.$r.log').read().strip().splitlines()[-1]); print('$lib', $r, d['value'], d['kernel_ms_per_step'], {k: v['value'] for k, v in d.get('other_configs', {}).items()})"
  done
done
