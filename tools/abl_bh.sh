cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5n
for m in 0 4 12 2; do
  XC_LIB_PATH=$PWD/wanproxy_amd/libxcodec_hip_b.so timeout -k 10 200 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 10 --diag-env XC_ABL_BH=$m > gpurun_out/r5n/abl$m.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r5n/abl$m.log').read().strip().splitlines()[-1]); print('abl', $m, d['value'], d['kernel_ms_per_step'])"
done
