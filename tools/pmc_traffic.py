"""HBM traffic of one cfg5 encode step, every kernel, from rocprofv3 PMC passes (tools/gpu.sh pmc).

A step is a cache restore (k_undo_known, or k_undo_dev) followed by the encode's kernels; the PMC runs are
`bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-decode --no-legs --tail-steps 4`, whose last 3
steps are production steps (after the diagnostic ones: the next run's blocks hashed ahead on the side
stream, the records of shadowed blocks dropped, as in the timed steps; round 4's records measured the
diagnostic steps, whose first sub-batch is hashed in line without those drops).  Each of those steps spans the dispatches from its
restore kernel to the next one (the last to the end); only the library's kernels (xc::) count.

FETCH_SIZE and WRITE_SIZE are in KiB.  The correction is calibrated on this GPU by tools/fetch_calib.hip
(tools/gpu.sh calib -> profiles/r06/pmc_calib.json): every read request the L2 sends to memory is one
128-byte line (TCC_EA0_RDREQ x 128 = the known bytes of coalesced reads of 1, 4, 8, 16 and 32 B per
lane, exactly), and FETCH_SIZE tallies each at 64 B (TCC_BUBBLE and TCC_EA0_RDREQ_32B are 0): 0.500 x
the bytes for every streaming width, and 64 B per random 4-, 8- or 16-byte gather (one request, RDREQ
1.00 per access).  So FETCH_SIZE is doubled for every kernel, gathers included: the counters do not
tell a gather's request size apart, so a gather counts as the 128-byte line it lands in (an upper
bound if the fabric fetched 64 B for it); WRITE_SIZE reads 1.000 x the bytes of 1-, 4-, 8- and 16-byte
stores.

usage: python tools/pmc_traffic.py PMC_DIR OUT_JSON SUB_BATCHES|auto [ALG_BYTES_PER_STEP]
(PMC_DIR holds FETCH_SIZE/ and WRITE_SIZE/ runs (tools/gpu.sh pmc), or p3/ and p4/; without
ALG_BYTES_PER_STEP it is the roofline's alg_bytes_per_step of the bench line the FETCH_SIZE pass
printed, PMC_DIR/../pmc_FETCH_SIZE.log)
"""
import collections
import csv
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wanproxy_amd.provenance import source_stamp  # noqa: E402


def dispatches(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out[int(r["Dispatch_Id"])] = (r["Kernel_Name"].split("(")[0], float(r["Counter_Value"]))
    return out


def steps(disp, n=3):
    ids = sorted(disp)
    starts = [i for i in ids if "k_undo_dev" in disp[i][0] or "k_undo_known" in disp[i][0]][-n:]
    bounds = starts + [ids[-1] + 1]
    return [[i for i in ids if bounds[k] <= i < bounds[k + 1] and disp[i][0].startswith(("xc::", "void xc::"))]
            for k in range(len(starts))]


def main():
    d, out_path = sys.argv[1], sys.argv[2]
    # (the FETCH_SIZE pass's bench output: PMC_DIR/../<basename(PMC_DIR)>_FETCH_SIZE.log)
    nd = os.path.normpath(d)
    log = os.path.join(os.path.dirname(nd), os.path.basename(nd) + "_FETCH_SIZE.log")
    line = json.loads([x for x in open(log).read().splitlines() if x.startswith("{")][-1]) \
        if os.path.exists(log) else None
    # (auto: the sub-batches of the bench line the FETCH_SIZE pass printed)
    sub_batches = int(line["stats"]["sub_batches"]) if sys.argv[3] == "auto" else int(sys.argv[3])
    if len(sys.argv) > 4:
        alg = int(sys.argv[4])
    else:
        alg = int(line["roofline"]["alg_bytes_per_step"])
    fd, wd = ("FETCH_SIZE", "WRITE_SIZE") if os.path.isdir(f"{d}/FETCH_SIZE") else ("p3", "p4")
    fetch = dispatches(f"{d}/{fd}/run_counter_collection.csv", "FETCH_SIZE")
    write = dispatches(f"{d}/{wd}/run_counter_collection.csv", "WRITE_SIZE")
    per_kernel = collections.defaultdict(lambda: [0.0, 0.0])
    fs, ws = steps(fetch), steps(write)
    for st in fs:
        for i in st:
            per_kernel[fetch[i][0]][0] += fetch[i][1] / len(fs)
    for st in ws:
        for i in st:
            per_kernel[write[i][0]][1] += write[i][1] / len(ws)
    kib = sum(2 * f + w for f, w in per_kernel.values())
    buffers = int(line["config"]["buffers_per_gpu"]) if line else 32768
    rec = {"steps_averaged": len(fs), "sub_batches": sub_batches, "buffers": buffers,
           "traffic_bytes_per_step": int(kib * 1024), "alg_bytes_per_step": alg,
           "traffic_over_alg": round(kib * 1024 / alg, 3),
           "per_kernel_bytes": {k: {"fetch_x2": int(2 * f * 1024), "write": int(w * 1024)}
                                for k, (f, w) in sorted(per_kernel.items(), key=lambda x: -(2 * x[1][0] + x[1][1]))},
           "correction": "FETCH_SIZE x2 for every kernel (gfx950: each 128-B read request tallied at 64 B, "
                         "calibrated for streaming reads of 1-32 B per lane and 4-16 B gathers, "
                         "profiles/r06/pmc_calib.json), WRITE_SIZE x1 (calibrated); KiB -> bytes",
           # the sources the passes ran (bench.py attaches the record only to the same sources)
           "src_stamp": source_stamp(),
           "commit": subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                                    text=True).stdout.strip() or None}
    json.dump(rec, open(out_path, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
