"""Average duration of each kernel's largest-grid launches (the cfg5 step launches, not the
warm-up encode) from a rocprofv3 kernel trace.  usage: trace_launches.py TRACE.csv OUT_JSON"""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    by[r["Kernel_Name"].split("(")[0]].append((g, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
out = {}
for k, v in by.items():
    g = max(x for x, _ in v)
    d = [t for x, t in v if x == g]
    out[k] = {"grid": g, "launches": len(d), "avg_us": round(sum(d) / len(d), 1)}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out, indent=1))
