"""Per-kernel PMC table (mean per dispatch of the largest grid, i.e. the cfg5 step launches) from
the rocprofv3 passes of tools/gpu.sh pmcinst (PMC_DIR/p1, p2).  usage: pmc_table.py PMC_DIR OUT_CSV"""
import collections
import csv
import glob
import os
import sys

d, out = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
grids = collections.defaultdict(int)
rows = []
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    rows += list(csv.DictReader(open(f)))
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    grids[k] = max(grids[k], int(r["Grid_Size"]))
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    if int(r["Grid_Size"]) == grids[k]:
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
counters = sorted({c for k in vals for c in vals[k]})
with open(out, "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["kernel", "grid", "dispatches"] + counters)
    for k in sorted(vals):
        n = max(len(v) for v in vals[k].values())
        w.writerow([k, grids[k], n] + [round(sum(vals[k][c]) / len(vals[k][c]), 1) if vals[k][c] else ""
                                       for c in counters])
print(open(out).read())
