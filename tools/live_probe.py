"""Where the live-cache leg's time goes: the same 4-batch sequence as bench.py's live leg, timed
(a) run by run with a device synchronize and the window replay between runs (isolated costs) and
(b) back to back, with a host timestamp after every run.  Diagnostic only (no parity check: the
bench's live leg checks the same sequence)."""
import sys
import os
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import wanproxy_amd as w
    from wanproxy_amd import workloads as W
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    n = 32768
    ctx = w.Context(0)
    warm = W.pool_warmup_buffers()
    cache = w.XCodecCache(ctx, W.POOL_SEGMENTS + nb * n * 33 + 1024)
    w.XCodecEncoder(cache).encode_batch(warm)
    cache.snapshot()
    plan = w.EncodePlan(cache, np.full(n, W.BUF, np.uint64))
    plan.set_completion(True)
    plan.set_input_ready(True)
    d_in = []
    for k in range(nb):
        x = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
        x[:n * W.BUF] = torch.from_numpy(W.repeat_shard(n, 0x5555 + k).reshape(-1)).cuda()
        d_in.append(x)
    d_out = [torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    d_len = [torch.zeros(n, dtype=torch.int64, device="cuda") for _ in range(nb)]
    torch.cuda.synchronize()

    def run(k):
        plan.run(d_in[k].data_ptr(), d_out[k].data_ptr(), d_len[k].data_ptr())

    for rep in range(3):
        cache.restore()
        torch.cuda.synchronize()
        iso = []
        for k in range(nb):
            t0 = time.perf_counter()
            run(k)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            h0 = cache.hit_stats()["host_s"]
            cache.settle()
            t2 = time.perf_counter()
            st = plan.stats()
            iso.append((round((t1 - t0) * 1e3, 3), round((t2 - t1) * 1e3, 3),
                        round((cache.hit_stats()["host_s"] - h0) * 1e3, 3), int(st.anchor_scans),
                        int(st.anchor_fallbacks), len(cache)))
        print("isolated (run ms, settle ms, replay ms, anchor scans, fallbacks, segments):", iso, flush=True)
        cache.restore()
        torch.cuda.synchronize()
        ts = [time.perf_counter()]
        h0 = cache.hit_stats()["host_s"]
        for k in range(nb):
            run(k)
            ts.append(time.perf_counter())
        h1 = cache.hit_stats()["host_s"]
        cache.settle()
        ts.append(time.perf_counter())
        torch.cuda.synchronize()
        ts.append(time.perf_counter())
        d = [round((b - a) * 1e3, 3) for a, b in zip(ts, ts[1:])]
        print(f"back to back (per run ..., settle, sync) ms: {d} total {round((ts[-1] - ts[0]) * 1e3, 2)}"
              f" replay in runs {round((h1 - h0) * 1e3, 3)} ms", flush=True)
        st = plan.stats()
        print("stats", {k: int(getattr(st, k)) for k in ("n_extract", "n_ref", "redone", "early_hashed",
                                                            "anchor_scans", "sub_batches")}, flush=True)
    plan.close()
    cache.close()


if __name__ == "__main__":
    main()
