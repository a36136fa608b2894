# HBM traffic of the cfg4 decode leg per kernel (FETCH_SIZE x2 and WRITE_SIZE, separate passes, the calibrated rule of
# tools/pmc_traffic.py): bash tools/pmc_dec.sh TAG (GPU box) -> gpurun_out/TAG/pmc_dec.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-pmcdec}; mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- python3 bench.py --only cfg4 --steps 20 > $out/$c.log 2>&1 || exit 1
done
python3 - "$out" > $out/pmc_dec.txt <<'PY'
import collections, csv, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
for i, c in enumerate(["FETCH_SIZE", "WRITE_SIZE"]):
    for r in csv.DictReader(open(f"{d}/{c}/run_counter_collection.csv")):
        if r["Counter_Name"] != c:
            continue
        k = r["Kernel_Name"].split("(")[0]
        agg[k][i] += float(r["Counter_Value"]) * 1024 * (2 if i == 0 else 1)
        if i == 0:
            agg[k][2] += 1
print("kernel, dispatches, read bytes per dispatch (FETCH_SIZE x2), written bytes per dispatch")
for k, (f, w, n) in sorted(agg.items(), key=lambda x: -(x[1][0] + x[1][1])):
    if n:
        print(f"{k[:60]:60s} {n:5d} {f / n / 1e6:10.1f} MB {w / n / 1e6:10.1f} MB")
# the step record bench.py attaches to its decode object (same library sources only): the kernels of a
# timed step (the restore, round 0 in k_dres2<true>, the parse, k_dfin, k_demit), per dispatch
import json, os
sys.path.insert(0, os.getcwd())
from wanproxy_amd.provenance import source_stamp
step = ("k_demit", "k_dtok<true, false>", "k_dres2<true>", "k_dfin", "k_undo_known")
per = {k: {"read": int(f / n), "write": int(w / n)} for k, (f, w, n) in agg.items() if n and k.split("::")[-1] in step}
line = json.loads([x for x in open(f"{d}/FETCH_SIZE.log").read().splitlines() if x.startswith("{")][-1])
alg = int(line["roofline"]["alg_bytes_per_step"])
tot = sum(v["read"] + v["write"] for v in per.values())
json.dump({"traffic_bytes_per_step": tot, "alg_bytes_per_step": alg, "traffic_over_alg": round(tot / alg, 3),
           "per_kernel_bytes": per, "correction": "FETCH_SIZE x2, WRITE_SIZE x1 (profiles/r06/pmc_calib.json)",
           "src_stamp": source_stamp()}, open(f"{d}/pmc_traffic_cfg4.json", "w"), indent=1)
PY
rm -rf $out/FETCH_SIZE $out/WRITE_SIZE
cat $out/pmc_dec.txt
