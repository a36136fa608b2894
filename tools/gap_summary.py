"""Gaps between consecutive kernels of a rocprofv3 kernel trace (tools/gap_bench.hip).
usage: python tools/gap_summary.py KERNEL_TRACE.csv"""
import csv
import statistics
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    prev = None
    pairs = {}
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev is not None:
            pairs.setdefault((prev[0], name), []).append((s - prev[2]) / 1000.0)
        prev = (name, s, e)
    for (a, b), g in sorted(pairs.items()):
        print(f"{a[:24]:24s} -> {b[:24]:24s} n {len(g):4d} gap us median {statistics.median(g):6.2f} "
              f"min {min(g):6.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
