cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ab
export XC_LIB_PATH=$PWD/wanproxy_amd/libxcodec_hip_b.so
for e in "XC_NONE=0" "XC_ABL_EMIT=4" "XC_ABL_EMIT=8" "XC_ABL_EMIT=12" "XC_ABL_EMIT=1" "XC_SCAN_ABLATION=2" "XC_SCAN_ABLATION=1" "XC_NONE=1"; do
  env $e timeout -k 10 120 python tools/leg_abl.py cfg2 300 > gpurun_out/r5ab/o.log 2>&1 || { cat gpurun_out/r5ab/o.log; exit 1; }
  tail -1 gpurun_out/r5ab/o.log
done
