"""Generate tests/golden/live_digests.npz: per-buffer digests of the ORACLE encoder's output for
the steady-state leg of bench.py (a live cache, no restore between batches), run here on the CPU.

Batches k = 0 .. 7 of cfg5's shape (32768 x 64 KiB, 50 % repeats of the 8192-segment pool) with
seeds 0x5555 + k, encoded one after another against ONE cache warmed with the pool: batch k sees
every segment batches 0 .. k-1 declared (xcodec/xcodec_encoder.cc:60-201, buffers in index order,
each a fresh encoder's encode() + flush(); the oracle is oracle/xc_oracle.c).  Batch 0 is cfg5
(its digests equal fullsize_digests.npz's cfg5_g1_r0).  ``live_b<k>_len`` / ``live_b<k>_dig`` as in
make_fullsize.py.  Test infrastructure (a checker generator), never product code.

    python tests/golden/make_live.py
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

BATCHES = 8
TOTAL = 32768
SEED0 = 0x5555
GROUP = 1024


def main():
    import oracle
    from wanproxy_amd import workloads as W
    oc = oracle.Cache()
    oc.encode_batch(W.pool_warmup_buffers())
    res, meta = {}, {}
    for k in range(BATCHES):
        t0 = time.time()
        bufs = W.repeat_shard(TOTAL, SEED0 + k)
        lens = np.zeros(TOTAL, np.uint32)
        digs = np.zeros(TOTAL, np.uint64)
        for a in range(0, TOTAL, GROUP):
            outs = oc.encode_batch([bufs[i] for i in range(a, min(TOTAL, a + GROUP))])
            for j, o in enumerate(outs):
                lens[a + j] = len(o)
                digs[a + j] = int.from_bytes(hashlib.sha256(o).digest()[:8], "little")
        res[f"live_b{k}_len"] = lens
        res[f"live_b{k}_dig"] = digs
        meta[f"live_b{k}"] = {"seed": hex(SEED0 + k), "buffers": TOTAL,
                              "out_bytes": int(lens.astype(np.uint64).sum()), "cache_segments_after": len(oc),
                              "digest_of_digests": hashlib.sha256(digs.tobytes()).hexdigest()}
        print(f"batch {k}: {meta[f'live_b{k}']}, {time.time() - t0:.1f} s", flush=True)
    np.savez_compressed(os.path.join(HERE, "live_digests.npz"), **res)
    json.dump({"generator": "tests/golden/make_live.py (oracle/xc_oracle.c)",
               "digest": "first 8 bytes of sha256(encoded stream), little-endian uint64",
               "cases": meta}, open(os.path.join(HERE, "live_digests.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
