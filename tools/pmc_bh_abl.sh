# VALU / LDS per block of the side-stream block hashing under XC_ABL_BH timing ablations
# (libxcodec_hip_b.so built with -DXC_ABLATIONS=1: wrong results on purpose; the bench's check fails
# after the counters are taken).  usage (GPU box): bash tools/pmc_bh_abl.sh TAG MODE...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:?tag}; shift
mkdir -p $out
for m in "$@"; do
  XC_ABL_BH=$m XC_LIB_PATH=$PWD/wanproxy_amd/libxcodec_hip_b.so timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES \
      --output-format csv -d $out/m$m -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --no-decode \
      --no-legs --no-live > $out/m$m.log 2>&1
  python3 - $out/m$m $m <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); grid = {}
for r in csv.DictReader(open(f)):
    if "k_blockhash<false, true>" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
blocks = sum(g // 256 * 4 * 8 for g in grid.values())
print("XC_ABL_BH", sys.argv[2], "dispatches", len(grid), {c: round(v / max(blocks, 1), 1) for c, v in acc.items() if c != "SQ_WAVES"})
PY
done
