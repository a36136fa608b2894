# VALU / LDS instructions per block of the side-stream block hashing (k_blockhash<false, true>) in
# production steps, for this library and the alternative build (tools/build_commit.sh).
# usage (GPU box): bash tools/pmc_bh.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:?tag}
mkdir -p $out
for v in a b; do
  lib=$PWD/wanproxy_amd/libxcodec_hip.so
  [ $v = b ] && lib=$PWD/wanproxy_amd/libxcodec_hip_b.so
  XC_LIB_PATH=$lib timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv \
      -d $out/$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --no-decode --no-legs --no-live \
      > $out/$v.log 2>&1 || exit 1
  python3 - $out/$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); grid = {}
for r in csv.DictReader(open(f)):
    if "k_blockhash<false, true>" not in r["Kernel_Name"]: continue
    k = (r["Dispatch_Id"]); acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); grid[k] = int(r["Grid_Size"])
blocks = sum(g // 256 * 4 * 8 for g in grid.values())
tot = collections.defaultdict(float)
for k in acc:
    for c, v in acc[k].items(): tot[c] += v
print(sys.argv[1], "dispatches", len(acc), {c: round(v / blocks, 1) for c, v in tot.items() if c != "SQ_WAVES"})
PY
done
