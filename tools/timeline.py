"""Print the kernel timeline of the last bench step from a rocprofv3 kernel trace:
start offset, duration and the gap before each launch (us).  usage: timeline.py TRACE.csv [N]
(trace bench.py with --tail-steps 2: its last steps are otherwise the diagnostic ones, whose timing events
add ~6 us before and after every span)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = {}
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get("Queue_Id", "?")
    gap = (s - prev_end[q]) / 1e3 if q in prev_end else 0.0
    prev_end[q] = e
    name = r["Kernel_Name"].split("(")[0].replace("void xc::", "").replace("xc::", "")
    print(f"q{q:>2} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {gap:7.1f}  {name[:60]}")
# step lengths (restore to restore: the k_undo_known launches) and each queue's busy time per step
starts = [int(r["Start_Timestamp"]) for r in rows if "k_undo_known" in r["Kernel_Name"]]
if len(starts) >= 2:
    print("# step lengths (restore to restore), us:", ", ".join(f"{(b - a) / 1e3:.1f}" for a, b in zip(starts, starts[1:])))
    for a, b in zip(starts, starts[1:]):
        busy = {}
        for r in rows:
            s, e = max(int(r["Start_Timestamp"]), a), min(int(r["End_Timestamp"]), b)
            if e > s:
                q = r.get("Queue_Id", "?")
                busy[q] = busy.get(q, 0) + e - s
        print("# busy per queue in the step, us:", ", ".join(f"q{q} {v / 1e3:.1f}" for q, v in sorted(busy.items())))
