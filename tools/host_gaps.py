"""Host HIP API calls merged with the kernels of a rocprofv3 trace (--kernel-trace --hip-runtime-trace,
csv): the last STEPS steps, each starting at a launch of MARK (default k_undo_known, the restore that
opens a bench step), in microseconds from the step's first host call after the previous step's mark.
usage: host_gaps.py TRACE_DIR [STEPS] [MARK]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
mark = sys.argv[3] if len(sys.argv) > 3 else "k_undo_known"


def one(pattern):
    f = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not f:
        sys.exit(f"no {pattern} under {d}")
    return list(csv.DictReader(open(f[0])))


ev = []
launched = {}  # correlation id -> kernel name (a launch call names the kernel it enqueued)
for r in one("*kernel_trace.csv"):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("xc::", "")
    launched[r["Correlation_Id"]] = name
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", name))
for r in one("*hip_api_trace.csv"):
    k = launched.get(r["Correlation_Id"])
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "H", r["Function"] + (" -> " + k if k else "")))
ev.sort()
marks = [i for i, e in enumerate(ev) if e[2] == "K" and e[3].startswith(mark)]
if len(marks) < steps + 1:
    sys.exit(f"{len(marks)} {mark} launches")
# (host calls are ordered by their start; the kernel marks by theirs, so a step opens at the host
# launch of its mark: the hipLaunchKernel just before the mark's kernel is not known, so a step is
# the span between two mark kernels, host calls included)
for k in range(len(marks) - steps - 1, len(marks) - 1):
    a, b = marks[k], marks[k + 1]
    t0 = ev[a][0]
    print(f"--- step from {mark} at {t0}")
    prev_h = None
    for s, e, kind, name in ev[a:b + 1]:
        gap = ""
        if kind == "H":
            if prev_h is not None:
                gap = f"(+{(s - prev_h) / 1e3:.1f})"
            prev_h = e
        print(f"{kind} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {gap:>9} {name[:60]}")
