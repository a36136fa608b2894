"""Summarise a gpu_check.sh run: test result, bench line, per-kernel time of the last profiled step."""
import collections
import csv
import json
import os
import sys

d = sys.argv[1]
t = os.path.join(d, "tests.log")
if os.path.exists(t):
    print(open(t).read().strip().splitlines()[-1])
b = [x for x in open(os.path.join(d, "bench.log")).read().splitlines() if x.startswith("{")]
if b:
    r = json.loads(b[-1])
    print(r["value"], r["ms_per_step"], r.get("kernel_ms_per_step"), r["roofline"]["frac"])
rows = list(csv.DictReader(open(os.path.join(d, "prof", "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
scans = [i for i, r in enumerate(rows) if "k_scan" in r["Kernel_Name"]]
start, end = scans[-8] - 4, min(scans[-1] + 6, len(rows) - 1)
agg = collections.defaultdict(float)
for r in rows[start:end]:
    agg[r["Kernel_Name"].split("(")[0]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print({k: round(v) for k, v in agg.items()})
print("span", (int(rows[end]["End_Timestamp"]) - int(rows[start]["Start_Timestamp"])) / 1e3)
print("scans", [round((int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3) for i in scans[-8:]])
