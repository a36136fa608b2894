cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5w
timeout -k 10 120 python3 tools/lat1.py > gpurun_out/r5w/lat.log 2>&1
XC_LIB_PATH=$PWD/wanproxy_amd/libxcodec_hip_b.so timeout -k 10 120 python3 tools/lat1.py >> gpurun_out/r5w/lat.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d gpurun_out/r5w/hip -o run -- python3 tools/lat1.py > /dev/null 2>&1
cat gpurun_out/r5w/lat.log
