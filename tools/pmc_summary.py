"""Per-kernel PMC counters of one cfg5 encode step (average over the diagnostic steps), from the
rocprofv3 passes of tools/gpu.sh pmcinst (PMC_DIR/p1, p2).  usage: python tools/pmc_summary.py PMC_DIR OUT_CSV"""
import collections
import csv
import os
import sys

from pmc_traffic import steps


def main():
    d, out = sys.argv[1], sys.argv[2]
    table = collections.defaultdict(dict)
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = list(csv.DictReader(open(f)))
        for counter in sorted({r["Counter_Name"] for r in rows}):
            disp = {int(r["Dispatch_Id"]): (r["Kernel_Name"].split("(")[0], float(r["Counter_Value"]))
                    for r in rows if r["Counter_Name"] == counter}
            st = steps(disp)
            acc = collections.defaultdict(float)
            for s in st:
                for i in s:
                    acc[disp[i][0]] += disp[i][1] / len(st)
            for k, v in acc.items():
                table[k][counter] = v
    cols = sorted({c for v in table.values() for c in v})
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel"] + cols)
        for k in sorted(table, key=lambda k: -table[k].get("SQ_WAVE_CYCLES", 0)):
            w.writerow([k] + [f"{table[k].get(c, 0):.0f}" for c in cols])
    print(open(out).read())


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
