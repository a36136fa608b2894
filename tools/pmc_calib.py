"""FETCH_SIZE / WRITE_SIZE (and the TCC request counters) of each tools/fetch_calib.hip dispatch against
the bytes it is known to move: the calibration behind tools/pmc_traffic.py's per-kernel correction.
usage: python tools/pmc_calib.py CALIB_DIR OUT_JSON   (CALIB_DIR: fetch_calib.csv + one rocprofv3 run per pass)"""
import csv
import glob
import json
import os
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    known = {}
    for r in csv.DictReader(open(os.path.join(d, "fetch_calib.csv"))):
        known[r["kernel"]] = (float(r["known_bytes"]), r["what"])
    vals = {}
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals.setdefault(name, {})
            c = r["Counter_Name"]
            vals[name][c] = vals[name].get(c, 0.0) + float(r["Counter_Value"])
    rows = {}
    for k, (b, what) in known.items():
        if k == "gathers":
            continue
        v = vals.get(k, {})
        row = {"known_bytes": int(b), "what": what}
        for c, x in sorted(v.items()):
            row[c] = x
        if "FETCH_SIZE" in v and k.startswith("c_read"):
            row["fetch_bytes_over_known"] = round(v["FETCH_SIZE"] * 1024 / b, 4)
        if "FETCH_SIZE" in v and k.startswith("c_gather"):
            row["fetch_bytes_per_access"] = round(v["FETCH_SIZE"] * 1024 / float(known["gathers"][0]), 2)
        if "WRITE_SIZE" in v and k.startswith("c_write"):
            row["write_bytes_over_known"] = round(v["WRITE_SIZE"] * 1024 / b, 4)
        if "TCC_EA0_RDREQ_sum" in v and k.startswith(("c_read", "c_gather")):
            n = float(known["gathers"][0]) if k.startswith("c_gather") else b
            row["rdreq_per_known_unit"] = round(v["TCC_EA0_RDREQ_sum"] / n * (1 if k.startswith("c_gather") else 128), 4)
        rows[k] = row
    json.dump(rows, open(out, "w"), indent=1)
    for k, r in rows.items():
        print(k, {x: y for x, y in r.items() if x not in ("what",)})


if __name__ == "__main__":
    main()
