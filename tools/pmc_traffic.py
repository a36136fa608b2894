"""HBM traffic per launch of the dominant kernel from rocprofv3 PMC passes (tools/pmc_kernels.sh).

FETCH_SIZE and WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section), on gfx950 FETCH_SIZE
reports half the bytes of wide coalesced streaming reads (16 B per lane), so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  The scan's other reads (8-B gathers into
the L2-resident filter and the lo32 sets) are not calibrated; they are a small share at cfg5.

usage: python tools/pmc_traffic.py PMC_DIR OUT_JSON SUB_BATCHES [kernel_regex]
"""
import csv
import json
import re
import sys


def per_dispatch(path, counter, kernel):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and re.search(kernel, r["Kernel_Name"]):
            out[int(r["Dispatch_Id"])] = (int(r["Grid_Size"]), float(r["Counter_Value"]))
    return out


def main():
    d, out_path = sys.argv[1], sys.argv[2]
    sub_batches = int(sys.argv[3])
    kernel = sys.argv[4] if len(sys.argv) > 4 else r"k_scan<0>"
    fetch = per_dispatch(f"{d}/p3/run_counter_collection.csv", "FETCH_SIZE", kernel)
    write = per_dispatch(f"{d}/p4/run_counter_collection.csv", "WRITE_SIZE", kernel)
    grid = max(g for g, _ in fetch.values())  # the cfg5 step launches (the warm-up encode is smaller)
    f = [v for g, v in fetch.values() if g == grid]
    w = [v for g, v in write.values() if g == grid]
    fetch_kib, write_kib = sum(f) / len(f), sum(w) / len(w)
    rec = {"kernel": kernel, "launches": len(f), "grid": grid, "sub_batches": sub_batches,
           "fetch_size_kib_raw": round(fetch_kib, 1), "write_size_kib": round(write_kib, 1),
           "traffic_bytes_per_launch": int((2 * fetch_kib + write_kib) * 1024),
           "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1; KiB -> bytes"}
    json.dump(rec, open(out_path, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
