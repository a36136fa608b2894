"""COSS encode throughput beside the memory cache's, same data, host arenas (xc_coss_encode_batch_host
/ xc_encode_batch_host: the COSS path has no device-resident form, every batch is replayed into the
host Store).

A 1024 MB COSS file (the reference's default size, 993 stripes: the ordinary purge path) and a
memory cache, both warmed with the cfg pool (8192 segments); then batches of B x 64 KiB buffers
(50 % pool repeats, fresh splitmix data, BASELINE cfg3's generator with a new seed per batch)
encoded through each.  The first batch of each cache is checked against the oracle encoder over
an oracle cache warmed the same way (COSS: the oracle's own COSS restatement on its own file).

usage: python tools/coss_bench.py [BUFFERS_PER_BATCH] [BATCHES] [SIZE_MB]  -> one JSON line"""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402

import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import xcodec as X  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402

UUID = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0"


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    nbatch = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    size_mb = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    from oracle import oracle as O
    ctx = w.Context(0)
    warm = W.pool_warmup_buffers()
    batches = [list(W.repeat_shard(nb, 0x900 + k)) for k in range(nbatch)]
    gib = nb * W.BUF / 2**30
    res = {"buffers_per_batch": nb, "batches": nbatch, "coss_size_mb": size_mb}
    with tempfile.TemporaryDirectory() as d:
        for kind in ("memory", "coss"):
            if kind == "memory":
                cache, oc = w.XCodecCache(ctx), O.Cache()
            else:
                os.makedirs(os.path.join(d, "p"))
                os.makedirs(os.path.join(d, "o"))
                cache = w.CossCache(ctx, os.path.join(d, "p"), UUID, size_mb)
                oc = O.Cache.coss(os.path.join(d, "o"), UUID, size_mb)
            enc = w.XCodecEncoder(cache)
            enc.encode_batch(warm)
            oc.encode_batch(warm)
            times, api = [], []
            fn = (X.load_library().xc_coss_encode_batch_host if kind == "coss"
                  else X.load_library().xc_encode_batch_host)
            for k, bufs in enumerate(batches):
                t0 = time.perf_counter()
                # XCodecEncoder.encode_batch, with the library call timed on its own (api): the
                # Python packing of the arena and the copies of the outputs into bytes objects are
                # the same for both caches
                arena, offs, lens = X._pack(bufs)
                cap = lens * 2 + 16
                ooff = np.zeros(len(bufs), dtype=np.uint64)
                ooff[1:] = np.cumsum(cap)[:-1]
                out = X._scratch("encode", int(cap.sum()))
                olen = np.zeros(len(bufs), np.uint64)
                t1 = time.perf_counter()
                X._check(fn(cache.h, arena, offs, lens, len(bufs), out, ooff, cap, olen))
                t2 = time.perf_counter()
                got = [out[int(o):int(o) + int(n)].tobytes() for o, n in zip(ooff, olen)]
                times.append(time.perf_counter() - t0)
                api.append(t2 - t1)
                if k == 0:
                    want = oc.encode_batch(bufs)
                    if want != got:
                        raise SystemExit(f"{kind}: batch 0 differs from the oracle")
            steady = times[1:] if len(times) > 1 else times
            steady_api = api[1:] if len(api) > 1 else api
            res[kind] = {"GiBs": round(gib / (sum(steady) / len(steady)), 3),
                         "api_GiBs": round(gib / (sum(steady_api) / len(steady_api)), 3),
                         "ms_per_batch": [round(t * 1e3, 2) for t in times],
                         "api_ms_per_batch": [round(t * 1e3, 2) for t in api],
                         "first_batch_equals_oracle": True}
            if kind == "coss":
                res[kind]["stats"] = cache.stats()
                cache.close()
            else:
                cache.close()
            del oc
    res["note"] = ("host arenas in and out (pinned staging inside the library); steady state = batches "
                   "after the first; every COSS batch is encoded on the device and its cache events "
                   "replayed into the host Store (stripe loads / purges in the reference's order); "
                   "GiBs: the Python encode_batch (arena packing, outputs to bytes); api_GiBs: the "
                   "library call alone (xc_coss_encode_batch_host / xc_encode_batch_host)")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
