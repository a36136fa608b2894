# rocprofv3 kernel-trace summaries of the cfg5 bench for the library (a) and libxcodec_hip_b.so (b),
# one short run each.  usage (GPU box): bash tools/trace_ab.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-trace_ab}
mkdir -p $out
for v in a b; do
  lib=$PWD/wanproxy_amd/libxcodec_hip.so
  [ $v = b ] && lib=$PWD/wanproxy_amd/libxcodec_hip_b.so
  XC_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o run \
    -- python3 bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 10 > $out/$v.log 2>&1 || exit 1
done
python3 - $out > $out/summary.txt <<'PY'
import csv, sys
out = sys.argv[1]
st = {v: {r["Name"].split("(")[0]: r for r in csv.DictReader(open(f"{out}/{v}/run_kernel_stats.csv"))} for v in "ab"}
for k in sorted(st["a"], key=lambda k: -float(st["a"][k]["TotalDurationNs"]))[:16]:
    b = st["b"].get(k)
    print(f"{k[:48]:48s} a {float(st['a'][k]['AverageNs'])/1e3:9.1f} us x{st['a'][k]['Calls']:>5}   b "
          + (f"{float(b['AverageNs'])/1e3:9.1f} us x{b['Calls']:>5}" if b else "-"))
PY
cat $out/summary.txt
echo "trace ab ok"
