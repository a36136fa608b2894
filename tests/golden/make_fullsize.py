"""Generate tests/golden/fullsize_digests.npz: per-buffer digests of the ORACLE encoder's output
at BASELINE.json's full sizes (run here, on the CPU; the GPU box only reads the fixture).

For every case, ``<case>_len`` (uint32, encoded length of each buffer) and ``<case>_dig``
(uint64, the first 8 bytes of sha256(encoded stream), little endian):

* ``cfg2``            256 x 64 KiB ``gen(0x1000 + i)``, empty cache (BASELINE configs[1]);
* ``cfg3``            4096 x 64 KiB, 50 % repeats, seed 0x77, pool-warmed cache (configs[2]);
                      these streams are also cfg4's decode input (configs[3]);
* ``cfg4v``           cfg4's variant input: 4096 x 64 KiB, 90 % repeats, seed 0x88, warm pool;
* ``cfg5_g<G>_r<r>``  cfg5 (configs[4]): 32768 x 64 KiB, 50 % repeats, seed 0x5555, buffer i
                      -> GPU i mod G; shard r encoded in index order against its own
                      pool-warmed cache, independently of every other shard,
                      for G = 1, 2, 4, 8.

Every buffer is one fresh encoder's encode() + flush() against the shard's cache, buffers in
index order (xcodec/xcodec_encoder.cc:60-201; the oracle is oracle/xc_oracle.c).
The oracle is test infrastructure: this script is a checker generator, never product code.

    python tests/golden/make_fullsize.py [-j 6]
"""
import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

TOTAL = 32768
GROUP = 1024  # buffers per oracle call (bounds the host arena)


def _digest(b: bytes) -> int:
    return int.from_bytes(hashlib.sha256(b).digest()[:8], "little")


def _buffers(case: str):
    from wanproxy_amd import workloads as W
    if case == "cfg2":
        return np.stack(W.random_buffers(256)), False
    if case == "cfg3":
        return W.repeat_shard(4096, 0x77), True
    if case == "cfg4v":
        return W.repeat_shard(4096, 0x88, repeat_pct=90), True
    g, r = case[len("cfg5_g"):].split("_r")
    return W.repeat_shard(TOTAL, 0x5555, int(r), int(g)), True


def job(case: str):
    import oracle
    from wanproxy_amd import workloads as W
    t0 = time.time()
    bufs, warm = _buffers(case)
    oc = oracle.Cache()
    if warm:
        oc.encode_batch(W.pool_warmup_buffers())
    n = bufs.shape[0]
    lens = np.zeros(n, np.uint32)
    digs = np.zeros(n, np.uint64)
    for a in range(0, n, GROUP):
        outs = oc.encode_batch([bufs[i] for i in range(a, min(n, a + GROUP))])
        for k, o in enumerate(outs):
            lens[a + k] = len(o)
            digs[a + k] = _digest(o)
    return case, lens, digs, len(oc), time.time() - t0


def cases():
    out = ["cfg2", "cfg3", "cfg4v"]
    for g in (1, 2, 4, 8):
        out += [f"cfg5_g{g}_r{r}" for r in range(g)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=6)
    args = ap.parse_args()
    res = {}
    meta = {}
    # the longest job (cfg5_g1_r0, 2 GiB sequential) first
    order = sorted(cases(), key=lambda c: 0 if c == "cfg5_g1_r0" else 1)
    with ProcessPoolExecutor(args.j) as ex:
        for case, lens, digs, ncache, secs in ex.map(job, order):
            res[case + "_len"] = lens
            res[case + "_dig"] = digs
            meta[case] = {"buffers": int(lens.size), "out_bytes": int(lens.astype(np.uint64).sum()),
                          "cache_segments": ncache,
                          "digest_of_digests": hashlib.sha256(digs.tobytes()).hexdigest()}
            print(f"{case}: {lens.size} buffers, {meta[case]['out_bytes']} bytes, {secs:.1f} s", flush=True)
    np.savez_compressed(os.path.join(HERE, "fullsize_digests.npz"), **res)
    json.dump({"generator": "tests/golden/make_fullsize.py (oracle/xc_oracle.c)",
               "digest": "first 8 bytes of sha256(encoded stream), little-endian uint64",
               "cases": meta}, open(os.path.join(HERE, "fullsize_digests.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
