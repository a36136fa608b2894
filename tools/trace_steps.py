"""Print the kernel timeline of one step (between two k_undo_dev restores) from a rocprofv3
kernel trace.  usage: python tools/trace_steps.py run_kernel_trace.csv [step_index_from_end]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if "k_undo_" in r["Kernel_Name"]]
i0, i1 = idx[-k - 1], idx[-k]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{r["Kernel_Name"].split("(")[0][:32]:32s} grid {r["Grid_Size_X"]:>8s} wg {r["Workgroup_Size_X"]:>5s} '
          f'start {(s - t0) / 1000:8.2f} us  dur {(e - s) / 1000:8.2f} us')
