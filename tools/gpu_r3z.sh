# round-3: cfg2 / cfg3 legs exact vs anchor scan; cfg5 sub-batch layouts
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3z}
mkdir -p $out
for r in 1 2; do
  for m in exact anchor; do
    for c in cfg2 cfg3; do
      XC_SCAN=$m timeout -k 10 120 python tools/leg.py $c 200 > $out/$c.$m.$r.json 2>&1 || { echo "leg rc $?"; tail -5 $out/$c.$m.$r.json; exit 1; }
      python -c "import json; d=json.loads(open('$out/$c.$m.$r.json').read().strip().splitlines()[-1]); print('$c', '$m', $r, d['value'], d['ms_per_step'])"
    done
  done
done
bash tools/abn_env.sh ${1:-r3z}/sub 2 "base:" "s1024:XC_SUB_MB=1024" "f256s1024:XC_FIRST_SUB_MB=256 XC_SUB_MB=1024" "f384s1024:XC_FIRST_SUB_MB=384 XC_SUB_MB=1024" "s768:XC_SUB_MB=768"
