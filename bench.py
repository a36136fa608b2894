#!/usr/bin/env python3
"""bench.py — XCodec encode GiB/s, device resident, on MI355X.

Workload (BASELINE.json configs[4], the config the metric's 1/2/4/8-GPU figures are quoted
on): 32768 x 64 KiB buffers, 50 % repeated segments (splitmix64 seed 0x5555), buffer i ->
rank i mod N, every rank with its own cache warmed with the 8192-segment pool.  Total work
is fixed as N grows ("scaling": "strong").

One step = restore the warm cache snapshot (enqueued, inside the timed region) + encode the
rank's whole shard, inputs already resident in HBM.  Every buffer is encode()+flush() on a
fresh XCodecEncoder against the rank's cache, buffers in index order
(xcodec/xcodec_encoder.cc:60-201), bit-exact with the reference.

Parity: every rank checks EVERY buffer of its shard against the oracle's per-buffer digests
(tests/golden/fullsize_digests.npz, made by tests/golden/make_fullsize.py: shard r of N encoded
independently with its own cache); jobs without a committed fixture are checked
against the oracle directly.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SEG = 2048
GOLD = os.path.join(ROOT, "tests", "golden", "fullsize_digests.npz")
PROFILE_DIR = os.path.join(ROOT, "profiles", "r06")
# The secondary legs (cfg2, cfg3, cfg4) time at least this many steps: their steps are 0.07-0.36 ms, so
# 20 steps (a few ms) measured the first steps' launch ramp too (cfg4: 1319-1333 GiB/s over 20 steps,
# 1367-1379 over 200, profiles/r05/ab/leg_steps_r5d.txt)
LEG_STEPS = 200
HOST_SUB_MB = 256  # sub-batch bound of the end-to-end (host memory) leg's plan


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--total", type=int, default=32768, help="buffers in the whole job")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every host core this process may use (affinity, capped by the cgroup CPU quota)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--verify", type=int, default=64,
                    help="without a committed digest fixture for the job: buffers checked against the oracle")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--no-legs", action="store_true", help="skip the cfg2 / cfg3 encode lines")
    ap.add_argument("--diag-env", default="",
                    help="KEY=VAL set only for the per-kernel diagnostic steps after the timed region and "
                         "the verification (timing ablations of -DXC_ABLATIONS=1 builds, e.g. XC_ABL_EMIT=4)")
    ap.add_argument("--decode-streams", type=int, default=4096, help="cfg4: streams decoded per step")
    ap.add_argument("--only", choices=["cfg2", "cfg3", "cfg4", "shard8"],
                    help="run just that leg (one GPU) and print its JSON object (kernel traces, A/B)")
    ap.add_argument("--no-live", action="store_true", help="skip the steady-state (live cache) leg")
    ap.add_argument("--tail-steps", type=int, default=0,
                    help="untimed production steps (no timing events) after the diagnostic ones, so that a "
                         "kernel trace's last step is one of the timed kind (tools/timeline.py)")
    ap.add_argument("--live-batches", type=int, default=8)
    ap.add_argument("--live-reps", type=int, default=3)
    return ap.parse_args()


def gold_case(case: str):
    """(lengths, digests) of the oracle's output for a fixture case, or None."""
    if not os.path.exists(GOLD):
        return None
    z = np.load(GOLD)
    if case + "_dig" not in z.files:
        return None
    return z[case + "_len"].astype(np.uint64), z[case + "_dig"]


def verify_outputs(out: np.ndarray, out_off, lens: np.ndarray, case: str, bufs, warm, verify: int) -> dict:
    """Every buffer against the oracle digests of `case` when the fixture holds it; otherwise the
    first `verify` buffers (all of them for small jobs) against an oracle run.  Raises on any
    difference (a bench line is only printed for a verified run)."""
    from wanproxy_amd import workloads as W
    g = gold_case(case) if case else None
    if g is not None:
        want_len, want_dig = g
        if want_len.size != lens.size or not np.array_equal(want_len, lens):
            raise SystemExit(f"bench: encoded lengths differ from the oracle ({case})")
        dig = W.arena_digests(out, out_off, lens)
        bad = np.nonzero(dig != want_dig)[0]
        if bad.size:
            raise SystemExit(f"bench: {bad.size} buffers differ from the oracle ({case}), first {bad[:8]}")
        return {"verified_buffers": int(lens.size), "verified_against": f"oracle digests {case}"}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker only
    oc = oracle.Cache()
    if warm is not None:
        oc.encode_batch(warm)
    n = len(bufs) if len(bufs) <= 4096 else min(verify, len(bufs))
    want = oc.encode_batch([bufs[i] for i in range(n)])
    for i, x in enumerate(want):
        o = int(out_off[i])
        if int(lens[i]) != len(x) or out[o:o + len(x)].tobytes() != x:
            raise SystemExit(f"bench: GPU output of buffer {i} differs from the oracle")
    return {"verified_buffers": n, "verified_against": "oracle run"}


def bench_encode_leg(ctx, warm, bufs, steps, case, input_ready=False):
    """One more encode configuration of BASELINE.json (device resident, one GPU): every step
    restores the cache snapshot (the warm pool, or empty for a cold cache) and encodes bufs."""
    import torch
    import wanproxy_amd as w
    from wanproxy_amd import workloads as W
    n = len(bufs)
    cache = w.XCodecCache(ctx, W.POOL_SEGMENTS + n * (W.BUF // SEG + 1) + 1024)
    if warm is not None:
        w.XCodecEncoder(cache).encode_batch(warm)
    cache.snapshot()
    lens = np.array([b.size for b in bufs], np.uint64)
    plan = w.EncodePlan(cache, lens)
    plan.set_completion(True)  # (stream ordered: every read below follows a device synchronize)
    plan.set_input_ready(input_ready)  # (the shard8 leg: written once before the steps, as in the headline)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, b in enumerate(bufs):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + b.size] = b
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step():
        cache.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    st = plan.stats()
    olen = d_len.cpu().numpy().astype(np.uint64)
    ver = verify_outputs(d_out.cpu().numpy(), plan.out_off, olen, case, bufs, warm, 64)
    alg = int(lens.sum()) + int(olen.sum()) + SEG * (int(st.n_extract) + int(st.n_ref))
    plan.close()
    cache.close()
    return dict({"value": round(int(lens.sum()) / el / 2**30, 3), "unit": "GiB/s", "ms_per_step": round(el * 1e3, 3), "steps": steps,
                 "buffers": n, "out_over_in": round(float(olen.sum()) / float(lens.sum()), 4),
                 "roofline": {"alg_bytes_per_step": alg, "achieved": round(alg / el / 1e9, 1),
                              "frac": round(alg / el / 1e9 / HBM_PEAK_GBS, 4)}}, **ver)


def bench_decode(args, ctx, warm):
    """cfg4 (BASELINE.json configs[3]): decode the cfg3 encoder output (4096 x 64 KiB, 50 %
    repeats, seed 0x77, encoded against the warm pool) on one GPU, device resident.  The decoder
    cache is warmed by decoding the warm-up streams; one step = restore that
    snapshot (enqueued) + xc_decode_run over every stream.  The encoded streams are checked against
    the oracle's digests first; every decoded stream is compared with its original buffer after
    the timed steps (a bit-exact round trip)."""
    import torch
    import wanproxy_amd as w
    from wanproxy_amd import workloads as W

    n = args.decode_streams
    bufs = W.repeat_shard(n, 0x77)
    ec = w.XCodecCache(ctx, W.POOL_SEGMENTS + n * (W.BUF // SEG + 1) + 1024)
    enc = w.XCodecEncoder(ec)
    warm_streams = enc.encode_batch(warm)
    streams = enc.encode_batch([bufs[i] for i in range(n)])
    ec.close()
    lens = np.array([len(x) for x in streams], np.uint64)
    if n == 4096:  # the decoder's input is the oracle's cfg3 output, buffer for buffer
        g = gold_case("cfg3")
        if g is not None and not (np.array_equal(g[0], lens) and
                                  np.array_equal(np.array([W.stream_digest(x) for x in streams], np.uint64), g[1])):
            raise SystemExit("bench: cfg3 streams (cfg4 decode input) differ from the oracle")
    dc = w.XCodecCache(ctx, W.POOL_SEGMENTS + n * (W.BUF // SEG + 1) + 1024)
    w.XCodecDecoder(dc).decode_batch(warm_streams)
    dc.snapshot()
    plan = w.DecodePlan(dc, lens, np.full(n, W.BUF, np.uint64))
    plan.set_completion(True)  # (stream ordered: every read below follows a device synchronize)
    plan.set_input_ready(True)  # (the encoded streams are written once, before the first step)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, x in enumerate(streams):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(x)] = np.frombuffer(x, np.uint8)
    d_in = torch.from_numpy(arena).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    u64 = torch.zeros(3 * n, dtype=torch.int64, device="cuda")
    i32 = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    p64, p32 = u64.data_ptr(), i32.data_ptr()

    def step():
        dc.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), p64, p64 + 8 * n, p32, p64 + 16 * n, p32 + 4 * n)

    steps = max(args.steps, LEG_STEPS)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    st = plan.stats()
    # round trip: decoded stream i == buffer i, status true, everything consumed
    assert all(int(plan.out_off[i]) == i * W.BUF for i in range(n))
    ok = torch.equal(d_out[:n * W.BUF].view(n, W.BUF).cpu(), torch.from_numpy(bufs))
    r64 = u64.cpu().numpy()
    ok = ok and bool((i32[:n].cpu().numpy() == 1).all()) and bool((r64[:n] == W.BUF).all()) \
        and bool((r64[n:2 * n] == lens.astype(np.int64)).all())
    if not ok:
        raise SystemExit("bench: decode round trip differs from the original buffers")
    enc_bytes, dec_bytes = int(lens.sum()), n * W.BUF
    alg = enc_bytes + dec_bytes + SEG * (int(st.n_entered) + int(st.n_ref))
    # the step's HBM traffic from the PMC record of these library sources (tools/pmc_dec.sh), if any
    from wanproxy_amd.provenance import source_stamp
    tr = None
    tp = os.path.join(PROFILE_DIR, "pmc_traffic_cfg4.json")
    if n == 4096 and os.path.exists(tp):
        rec = json.load(open(tp))
        if rec.get("src_stamp") == source_stamp() and rec.get("alg_bytes_per_step") == alg:
            tr = rec
    return {"workload": "cfg4", "streams": n, "value": round(dec_bytes / el / 2**30, 3),
            "unit": "GiB/s decoded (device resident)", "ms_per_step": round(el * 1e3, 3), "steps": steps,
            "enc_GiBs": round(enc_bytes / el / 2**30, 3),
            "roofline": {"bound": "hbm", "alg_bytes_per_step": alg, "achieved": round(alg / el / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / el / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": tr["traffic_bytes_per_step"] if tr else None,
                         "traffic_over_alg": tr["traffic_over_alg"] if tr else None,
                         "traffic_source": os.path.relpath(tp, ROOT) if tr else None},
            "stats": {"n_extract": int(st.n_extract), "n_ref": int(st.n_ref), "n_entered": int(st.n_entered),
                      "rounds": int(st.rounds)},
            "verified_streams": n}


LIVE_GOLD = os.path.join(ROOT, "tests", "golden", "live_digests.npz")


def bench_live(args, ctx, warm, d_in0, step_ms):
    """Steady state: cfg5-shaped batches back to back on ONE live cache, no restore in between (how a
    proxy's cache runs).  Batch k (seed 0x5555 + k; batch 0 is the headline's) sees every segment the
    batches before it declared, and each run's lookup hits reach the recent window model while the
    next run works.  One timed sequence = the batches back to back + the replay of
    the last run's hits (cache.settle()), from the warm snapshot; every buffer of every batch is then
    checked against the oracle's digests of the same sequence (tests/golden/make_live.py)."""
    import torch
    import wanproxy_amd as w
    from wanproxy_amd import workloads as W
    nb = args.live_batches
    n = 32768
    cache = w.XCodecCache(ctx, W.POOL_SEGMENTS + nb * n * (W.BUF // SEG + 1) + 1024)
    w.XCodecEncoder(cache).encode_batch(warm)
    cache.snapshot()
    lens = np.full(n, W.BUF, np.uint64)
    plan = w.EncodePlan(cache, lens)
    plan.set_completion(True)
    plan.set_input_ready(True)  # (every batch's arena is written before the timed sequences)
    d_in = [d_in0]
    for k in range(1, nb):
        x = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
        x[:n * W.BUF] = torch.from_numpy(W.repeat_shard(n, 0x5555 + k).reshape(-1)).cuda()
        d_in.append(x)
    d_out = [torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    d_len = [torch.zeros(n, dtype=torch.int64, device="cuda") for _ in range(nb)]
    torch.cuda.synchronize()

    def sequence():
        for k in range(nb):
            plan.run(d_in[k].data_ptr(), d_out[k].data_ptr(), d_len[k].data_ptr())
        cache.settle()

    times, replay = [], []
    for rep in range(1 + args.live_reps):  # (the first sequence is the warm-up)
        cache.restore()
        torch.cuda.synchronize()
        h0 = cache.hit_stats()
        t0 = time.perf_counter()
        sequence()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        h1 = cache.hit_stats()
        if rep:
            times.append(t1 - t0)
            replay.append((h1["host_s"] - h0["host_s"], h1["runs"] - h0["runs"], h1["hits"] - h0["hits"]))
    # parity: every buffer of every batch (the outputs of the last sequence)
    verified = 0
    z = np.load(LIVE_GOLD) if os.path.exists(LIVE_GOLD) else None
    if z is None or f"live_b{nb - 1}_dig" not in z.files:
        raise SystemExit("bench: live leg without its oracle digests (tests/golden/make_live.py)")
    for k in range(nb):
        olen = d_len[k].cpu().numpy().astype(np.uint64)
        if not np.array_equal(z[f"live_b{k}_len"].astype(np.uint64), olen):
            raise SystemExit(f"bench: live batch {k}: encoded lengths differ from the oracle")
        dig = W.arena_digests(d_out[k].cpu().numpy(), plan.out_off, olen)
        bad = np.nonzero(dig != z[f"live_b{k}_dig"])[0]
        if bad.size:
            raise SystemExit(f"bench: live batch {k}: {bad.size} buffers differ from the oracle, first {bad[:8]}")
        verified += n
    st = plan.stats()
    t = float(np.median(times))
    rs, rr, rh = (float(np.median([r[i] for r in replay])) for i in range(3))
    res = {"value": round(nb * n * W.BUF / t / 2**30, 3), "unit": "GiB/s", "batches": nb,
           "ms_per_batch": round(t / nb * 1e3, 3), "vs_headline": round(step_ms / (t / nb * 1e3), 4),
           "sequence_ms": [round(x * 1e3, 2) for x in times],
           "window_replay": {"host_ms_per_run": round(rs / max(rr, 1) * 1e3, 3), "runs": int(rr),
                             "hits_per_run": int(rh / max(rr, 1)),
                             "note": "host time replaying each run's lookup hits into the recent window "
                                     "model, inside the next run's wait (overlapping it) or in the final "
                                     "settle (inside the timed sequence)"},
           "cache_segments_after": len(cache), "last_batch_stats": {"n_extract": int(st.n_extract),
                                                                    "n_ref": int(st.n_ref),
                                                                    "anchor_scans": int(st.anchor_scans),
                                                                    "anchor_fallbacks": int(st.anchor_fallbacks)},
           "verified_buffers": verified, "verified_against": "oracle digests live_b0..live_b%d" % (nb - 1),
           "workload": f"{nb} cfg5-shaped batches (seeds 0x5555..0x{0x5555 + nb - 1:x}) back to back on one "
                       "live pool-warmed cache, no restore between them; timed from the warm snapshot to the "
                       "last run's window replay"}
    plan.close()
    cache.close()
    return res


def host_cores() -> int:
    """Host cores this process may use: its CPU affinity, capped by a cgroup CPU quota (the GPU
    box grants a quota of cores per GPU while affinity shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(args, shard, warm, world) -> dict:
    """The oracle (the C restatement of xcodec_encoder.cc, kind "port") on the host cores of this
    rank: T threads, each with a private clone of the warm cache, buffers round-robin over the
    threads (sharded like the GPUs), over a bounded sample of the rank's shard; and the same port on
    one thread."""
    from wanproxy_amd import workloads as W
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # CPU baseline: the C restatement (port) of the reference encoder
    nthreads = args.cpu_threads or host_cores()
    n_local = shard.shape[0]
    # the whole shard on T threads (cfg5 at N=1: 2 GiB, about 26 CPU-seconds at 16 threads), and
    # 8192 buffers (512 MiB, about 6 s) on one
    n = n_local
    sample = [shard[i] for i in range(n)]
    oc = oracle.Cache()
    oc.encode_batch(warm)
    secs, _ = oc.encode_sharded_timed(sample, nthreads)
    res = {"value": round(n * W.BUF / secs / 2**30, 4), "unit": "GiB/s", "cores": nthreads,
           "kind": "port",
           "sample": f"first {n} buffers of the rank's cfg5 shard ({n * W.BUF >> 20} MiB), round-robin over "
                     f"{nthreads} threads, each with a private clone of the pool-warmed cache",
           "seconds": round(secs, 3), "host_cpus_visible": os.cpu_count(),
           "cores_allowed": host_cores(), "cores_note": "affinity capped by the cgroup CPU quota (cpu.max)"}
    one = sample[:min(n, 8192)]
    oc1 = oracle.Cache()
    oc1.encode_batch(warm)
    secs1, _ = oc1.encode_sharded_timed(one, 1)
    res["single_thread"] = {"value": round(len(one) * W.BUF / secs1 / 2**30, 4), "unit": "GiB/s", "cores": 1,
                            "sample": f"first {len(one)} buffers ({len(one) * W.BUF >> 20} MiB)",
                            "seconds": round(secs1, 3)}
    if world > 1:
        res["note"] = "measured on rank 0's host cores after the timed region (other ranks idle)"
    return res


def pmc_traffic_path(buffers: int) -> str:
    """The committed PMC record of a cfg5 step over `buffers` buffers per GPU: the whole job at N=1,
    a rank's shard at N>1 (measured on one GPU with bench.py --total <shard>, tools/gpu.sh pmc)."""
    return os.path.join(PROFILE_DIR, "pmc_traffic_cfg5.json" if buffers == 32768 else f"pmc_traffic_cfg5_b{buffers}.json")


def pmc_traffic(sub_batches: int, buffers: int = 32768):
    """HBM bytes per step of the whole encode pipeline from the committed rocprofv3 PMC passes of
    this command (tools/gpu.sh pmc -> tools/pmc_traffic.py -> profiles/r06/), or None when the
    record was taken with other library sources than these (its src_stamp) or another layout."""
    from wanproxy_amd.provenance import source_stamp
    tp = pmc_traffic_path(buffers)
    if not os.path.exists(tp):
        return None
    rec = json.load(open(tp))
    if rec.get("sub_batches") != sub_batches or rec.get("src_stamp") != source_stamp():
        return None
    if rec.get("buffers", 32768) != buffers:
        return None
    return rec


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")

    import torch
    import torch.distributed as dist

    # one process per GPU; on a box with fewer GPUs than ranks (rehearsal only) ranks share them
    ndev = torch.cuda.device_count()
    dev = local_rank if local_rank < ndev else local_rank % max(ndev, 1)
    torch.cuda.set_device(dev)
    if world > 1:
        # barrier and max/sum reductions of timings and counts only: the path shards with no
        # data-path collective
        dist.init_process_group("gloo")

    import wanproxy_amd as w
    from wanproxy_amd import workloads as W

    ctx = w.Context(dev)
    if args.only:
        if args.only == "cfg4":
            print(json.dumps(bench_decode(args, ctx, W.pool_warmup_buffers())))
        elif args.only == "cfg2":
            print(json.dumps(bench_encode_leg(ctx, None, W.random_buffers(256), args.steps, "cfg2")))
        elif args.only == "shard8":
            print(json.dumps(bench_encode_leg(ctx, W.pool_warmup_buffers(), list(W.repeat_shard(32768, 0x5555, 0, 8)),
                                              args.steps, "cfg5_g8_r0", input_ready=True)))
        else:
            print(json.dumps(bench_encode_leg(ctx, W.pool_warmup_buffers(), list(W.repeat_shard(4096, 0x77)),
                                              args.steps, "cfg3")))
        return
    shard = W.repeat_shard(args.total, 0x5555, rank, world)  # (n_local, 65536)
    n_local = shard.shape[0]
    warm = W.pool_warmup_buffers()

    cache = w.XCodecCache(ctx, W.POOL_SEGMENTS + n_local * (W.BUF // SEG + 1) + 1024)
    w.XCodecEncoder(cache).encode_batch(warm)
    cache.snapshot()

    lens = np.full(n_local, W.BUF, dtype=np.uint64)
    plan = w.EncodePlan(cache, lens)
    plan.set_completion(True)  # (stream ordered: every read below follows a device synchronize)
    plan.set_input_ready(True)  # (the input arena is written once, before the first step)
    assert all(int(plan.in_off[i]) == i * W.BUF for i in range(n_local))
    d_in = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
    d_in[:n_local * W.BUF] = torch.from_numpy(shard.reshape(-1)).cuda()
    d_out = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n_local, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step():
        cache.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), d_len.data_ptr())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # the timed steps run as they do in production (the asynchronous pass as one HIP graph launch,
    # no timing events); the per-kernel breakdown comes from extra steps after the timed region
    plan.set_timing(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    st = plan.stats()
    got_len = d_len.cpu().numpy().astype(np.uint64)
    out_bytes = int(got_len.sum())
    in_bytes_rank = n_local * W.BUF
    alg_rank = in_bytes_rank + out_bytes + SEG * (int(st.n_extract) + int(st.n_ref))

    # parity of the timed configuration: every buffer of this rank's shard (after the timed steps,
    # so the output checked is the output of the last timed step)
    case = f"cfg5_g{world}_r{rank}" if args.total == 32768 else None
    ver = verify_outputs(d_out.cpu().numpy(), plan.out_off, got_len, case, shard, warm, args.verify)

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([alg_rank, ver["verified_buffers"], n_local], dtype=torch.float64)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        alg_job, verified_job, n_job = (int(x) for x in s.tolist())
    else:
        alg_job, verified_job, n_job = alg_rank, ver["verified_buffers"], n_local

    diag_steps = 3
    if args.diag_env:  # (after the timed steps and the verification: ablations only change these)
        k, v = args.diag_env.split("=", 1)
        os.environ[k] = v
    plan.kernel_times(reset=True)
    plan.set_timing(True)
    for _ in range(diag_steps):
        step()
    torch.cuda.synchronize()
    plan.set_timing(False)
    kt_all = plan.kernel_times(reset=True)
    for _ in range(args.tail_steps):
        step()
    torch.cuda.synchronize()

    total_in = n_job * W.BUF
    value = total_in * args.steps / elapsed / 2**30
    step_s = elapsed / args.steps

    # roofline: algorithmic bytes of one step = in + out + 2048 * (segments
    # declared + references verified), summed over ranks, against N x 8 TB/s.  The whole encode
    # pipeline is the unit: no single kernel carries the step (kernel_ms_per_step).
    peak = HBM_PEAK_GBS * world
    achieved = alg_job / step_s / 1e9
    # (N>1: every rank's step moves its own shard's bytes on its own GPU; the record is of a rank-sized
    # shard on one GPU, its bytes times N)
    tr = pmc_traffic(int(st.sub_batches), n_local) if args.total == 32768 else None
    tr_job = tr["traffic_bytes_per_step"] * world if tr else None
    anchor = int(st.anchor_scans) > 0
    roofline = {"bound": "hbm", "kernel": "encode step (k_blockhash, k_blockpredict, "
                                          + ("k_aprop, k_aevents" if anchor else "k_scan")
                                          + ", k_resolve, k_walk, k_alloc, k_emit" + (", k_tailcheck)" if anchor else ")"),
                "achieved": round(achieved, 1), "peak": peak, "unit": "GB/s", "frac": round(achieved / peak, 4),
                "traffic": tr_job,
                "traffic_over_alg": round(tr_job / alg_job, 3) if tr else None,
                "traffic_source": (os.path.relpath(pmc_traffic_path(n_local), ROOT)
                                   + ("" if world == 1 else f" (a {n_local}-buffer shard on one GPU, x {world})"))
                if tr else None,
                "alg_bytes_per_step": alg_job,
                "alg_bytes_def": "in + out + 2048 * (n_extract + n_ref) (SURVEY.md §8(d))"}
    # diagnostic: the scan alone, 1 byte per position it covers, HIP events on the library stream
    # around every scan launch of the diagnostic steps
    launches = max(1, kt_all["launches"]["scan"])
    avg_ms = kt_all["ms"]["scan"] / launches
    bytes_per_launch = kt_all["scan_bytes"] / launches
    scan_ach = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0

    # the step's two heaviest kernels by their own algorithmic bytes (HIP events around each launch in
    # the diagnostic steps; the side stream's block hashing shares the GPU with the main stream)
    kernel_rooflines = {}
    for name, bytes_step, what in (
            ("blockhash", in_bytes_rank + SEG * int(st.n_ref),
             "input bytes + the cached segments of predicted REFs compared in registers"),
            ("emit", 2 * SEG * int(st.n_extract) + out_bytes,
             "EXTRACT payload reads + wire bytes + segment-store writes (span: k_insert + k_emit)")):
        n_l = kt_all["launches"].get(name, 0)
        ms = kt_all["ms"].get(name, 0.0)
        if n_l and ms > 0:
            b_l = bytes_step * diag_steps / n_l
            ach = b_l / (ms / n_l * 1e-3) / 1e9
            kernel_rooflines[name] = {"achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                      "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(ms / n_l, 4),
                                      "alg_bytes_per_launch": int(b_l), "alg_bytes_def": what}

    result = {
        "metric": "XCodec encode GiB/s device-resident (cfg5: 32768 x 64 KiB, 50% repeats, warm per-GPU cache)",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64, SURVEY.md §8(d))",
        "config": {"workload": "cfg5", "buffers_total": args.total, "buffer_bytes": W.BUF,
                   "repeat_pct": 50, "seed": "0x5555", "cache": "warm pool, 8192 segments per GPU",
                   "buffers_per_gpu": n_local, "parallelism": f"shard{world}"},
        "roofline": roofline,
        "scan_roofline": {"kernel": "k_aprop + k_aevents (anchor scan)" if anchor else "k_scan",
                          "achieved": round(scan_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(scan_ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(avg_ms, 4),
                          "input_bytes_per_launch": int(bytes_per_launch),
                          "note": "diagnostic: 1 B per scanned position / scan launch time (rank 0, diagnostic steps)"
                          + ("; the anchor scan reads the block hashing's records (8 B per input anchor, 1/64 of "
                             "the positions), not the input: this is its coverage rate, not its traffic" if anchor else "")},
        "kernel_rooflines": kernel_rooflines,
        "kernel_ms_per_step": {k: round(v / diag_steps, 4) for k, v in kt_all["ms"].items()},
        "kernel_ms_note": f"HIP events around every kernel in {diag_steps} steps after the timed region (rank 0)",
        "stats": {"n_extract": int(st.n_extract), "n_ref": int(st.n_ref),
                  "out_over_in": round(out_bytes / in_bytes_rank, 4),
                  "sub_batches": int(st.sub_batches), "outer_rounds": int(st.outer_rounds),
                  "walk_rounds": int(st.walk_rounds), "dense_chunks": int(st.dense_chunks),
                  "redone": int(st.redone), "shadow_misses": int(st.shadow_misses),
                  "anchor_scans": int(st.anchor_scans), "anchor_fallbacks": int(st.anchor_fallbacks),
                  "early_hashed": int(st.early_hashed)},
        "verified_buffers": verified_job,
        "verified_against": ver["verified_against"] if world == 1 else
        f"oracle digests cfg5_g{world}_r* (every rank, every buffer of its shard)" if case else "oracle run",
        "cpu_baseline": None,
    }

    if rank == 0 and world == 1 and not args.no_e2e:
        # end-to-end from host memory (xc_encode_run_host): the input arena in pinned host
        # memory, each sub-batch copied in on a copy stream while earlier ones encode, and every
        # sub-batch's encoded streams packed into pinned host memory by a kernel as it is emitted
        # (a plan of 256 MiB sub-batches: its copies and packing overlap more of the encode than 1 GiB
        # ones, xc_encode_plan_create_sub: 38 -> 43 GiB/s, profiles/r05/ab/e2e_sub_batches_r5x.txt)
        hplan = w.EncodePlan(cache, lens, sub_bytes=HOST_SUB_MB << 20)
        assert hplan.in_bytes == plan.in_bytes and np.array_equal(hplan.in_off, plan.in_off)
        h_in = w.HostBuffer(ctx, hplan.in_bytes)
        h_in.array[:] = d_in.cpu().numpy()
        h_out = w.HostBuffer(ctx, hplan.out_bytes)
        cache.restore_async()
        hplan.run_host(h_in, h_out)  # warm-up (device arenas of the host path)
        reps = 3
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            cache.restore_async()
            hlens, pos = hplan.run_host(h_in, h_out)
        e2e = (time.perf_counter() - t0) / reps
        if not np.array_equal(hlens.astype(np.uint64), got_len):
            raise SystemExit("bench: host path output lengths differ from the device-resident run")
        if case and gold_case(case) is not None:
            if not np.array_equal(W.arena_digests(h_out.array, pos, hlens), gold_case(case)[1]):
                raise SystemExit("bench: host path output differs from the oracle")
        result["e2e_host_gibs"] = round(in_bytes_rank / e2e / 2**30, 3)
        result["e2e_ms"] = round(e2e * 1e3, 2)
        hplan.close()
        result["e2e_note"] = (f"xc_encode_run_host ({HOST_SUB_MB} MiB sub-batches): pinned host input arena -> per-sub-batch H2D "
                              "overlapping the encode -> streams packed into pinned host memory "
                              f"({int(hlens.sum()) >> 20} MiB) by a kernel after each sub-batch; every buffer "
                              "checked against the oracle digests")

    if rank == 0 and world == 1 and not args.no_live and args.total == 32768:
        result["live_cache"] = bench_live(args, ctx, warm, d_in, step_s * 1e3)

    if rank == 0 and world == 1 and not args.no_decode:
        result["decode"] = bench_decode(args, ctx, warm)

    if rank == 0 and world == 1 and not args.no_legs:
        # BASELINE.json configs[1] and [2] (parity-test cases; value stays cfg5)
        result["other_configs"] = {
            "cfg2": dict(bench_encode_leg(ctx, None, W.random_buffers(256), max(args.steps, LEG_STEPS), "cfg2"),
                         workload="256 x 64 KiB, 0% repeats, cold (empty) cache"),
            "cfg3": dict(bench_encode_leg(ctx, warm, list(W.repeat_shard(4096, 0x77)), max(args.steps, LEG_STEPS),
                                          "cfg3"),
                         workload="4096 x 64 KiB, 50% repeats, seed 0x77, warm pool cache"),
            "shard8": dict(bench_encode_leg(ctx, warm, list(W.repeat_shard(32768, 0x5555, 0, 8)),
                                            max(args.steps, LEG_STEPS), "cfg5_g8_r0", input_ready=True),
                           workload="rank 0's shard of cfg5 at N=8 (4096 x 64 KiB, buffers i = 0 mod 8), warm "
                                    "pool cache: the per-GPU unit of the 8-GPU metric, on one GPU"),
        }

    if rank == 0 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args, shard, warm, world)

    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
