"""Long randomized parity campaign on the GPU (beyond tests/test_gpu_fuzz.py's 16 seeds): batch
encodes, stateful stream calls and decodes of truncated / corrupted streams (through XCodecDecoder, and
through a device-resident DecodePlan with the input ready: the early parse and round 0 in k_dres2<true>),
each against the oracle.
Runs seeds until the time budget is spent; prints every failing seed.
usage: python tools/fuzz_campaign.py SECONDS [FIRST_SEED]"""
import os
import sys
import time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402  (the checker)
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402
import tempfile  # noqa: E402

budget = float(sys.argv[1]) if len(sys.argv) > 1 else 200
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
ctx = w.Context(0)
pool = W.pool(64)
t_end = time.time() + budget
fails = 0
runs = {"encode": 0, "streams": 0, "decode": 0, "coss": 0, "plan": 0, "dup": 0, "dplan": 0}


def mangle(rng, streams):
    out = []
    for s in streams:
        s = bytearray(s)
        r = rng.random()
        if r < 0.3 and s:
            s = s[:int(rng.integers(len(s)))]          # truncated (a stream cut mid-token)
        elif r < 0.45 and s:
            s[int(rng.integers(len(s)))] = 0xF1         # a stray magic byte
        elif r < 0.55 and len(s) > 10:
            k = int(rng.integers(len(s) - 1))
            s[k:k + 2] = bytes([0xF1, 0x02])            # a REF to an unknown hash
        out.append(bytes(s))
    return out


def plan_decode(gd, streams, reps):
    """streams through a DecodePlan (stream ordered, input ready), `reps` runs over the cache's
    snapshot; the results of each run as decode_batch's tuples"""
    import torch
    lens = np.array([len(x) for x in streams], np.uint64)
    plan = w.DecodePlan(gd, lens, lens * 205 + 16)
    plan.set_completion(True)
    plan.set_input_ready(True)
    arena = np.zeros(plan.in_bytes, np.uint8)
    for i, x in enumerate(streams):
        arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(x)] = np.frombuffer(x, np.uint8)
    n = len(streams)
    d_in = torch.from_numpy(arena).cuda()
    sets = [(torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda"),
             torch.zeros(3 * n, dtype=torch.int64, device="cuda"),
             torch.zeros(2 * n, dtype=torch.int32, device="cuda")) for _ in range(reps)]
    torch.cuda.synchronize()
    for d_out, u64, i32 in sets:
        gd.restore_async()
        plan.run(d_in.data_ptr(), d_out.data_ptr(), u64.data_ptr(), u64.data_ptr() + 8 * n,
                 i32.data_ptr(), u64.data_ptr() + 16 * n, i32.data_ptr() + 4 * n)
    ctx.sync()
    torch.cuda.synchronize()
    res = []
    for d_out, u64, i32 in sets:
        out, r64, r32 = d_out.cpu().numpy(), u64.cpu().numpy().astype(np.uint64), i32.cpu().numpy()
        res.append([(int(r32[i]), out[int(plan.out_off[i]):int(plan.out_off[i]) + int(r64[i])].tobytes(),
                     int(r64[n + i]), int(r64[2 * n + i]) if r32[n + i] else None) for i in range(n)])
    plan.close()
    return res

while time.time() < t_end:
    if seed % 10 == 0:
        print("progress seed", seed, runs, "fails", fails, flush=True)
    rng = np.random.default_rng(seed)
    os.environ["XC_CHUNK_BLOCKS"] = str(int(rng.choice([1, 2, 3, 5, 8])))
    os.environ["XC_SUB_MB"] = str(int(rng.choice([1, 2, 512])))
    os.environ["XC_NO_SHADOW"] = "1" if rng.random() < 0.3 else "0"
    warm = [pool[i:i + 65536] for i in range(0, int(rng.integers(1, 9)) * 65536, 65536)]
    kinds = os.environ.get("FUZZ_KINDS", "encode,streams,decode").split(",")
    kind = kinds[seed % len(kinds)]
    runs[kind] += 1
    try:
        if kind == "coss":
            size = int(rng.choice([3, 5, 17, 20]))
            d1, d2 = tempfile.mkdtemp(), tempfile.mkdtemp()
            uu = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0"
            oc, gc = oracle.Cache.coss(d1, uu, size), w.CossCache(ctx, d2, uu, size)
            n = int(rng.integers(1, 8))
            oe = [oracle.Encoder(oc) for _ in range(n)]
            ge = [w.XCodecStreamEncoder(gc) for _ in range(n)]
            streams = []
            for _ in range(int(rng.integers(2, 6))):
                bufs = F._batch(rng, pool)
                if rng.random() < 0.5:
                    want = oc.encode_batch(bufs)
                    if w.XCodecEncoder(gc).encode_batch(bufs) != want:
                        raise AssertionError("coss batch encode differs")
                    streams += want
                else:
                    calls = [(int(rng.integers(n)), b, bool(rng.random() < 0.5)) for b in bufs]
                    want = []
                    for c, d, f in calls:
                        o = oe[c].encode(d)
                        if f:
                            o += oe[c].flush()[1]
                        want.append(o)
                    if w.encode_streams([(ge[c], d, f) for c, d, f in calls]) != want:
                        raise AssertionError("coss stream calls differ")
            if len(oc) != len(gc):
                raise AssertionError("coss sizes differ")
            oc.close()
            gc.close()
            if open(os.path.join(d1, uu + ".wpc"), "rb").read() != open(os.path.join(d2, uu + ".wpc"), "rb").read():
                raise AssertionError("coss files differ")
            od, gd = oracle.Cache.coss(d1, uu[::-1], size), w.CossCache(ctx, d2, uu[::-1], size)
            for k in range(0, len(streams), 16):
                if od.decode_batch(streams[k:k + 16]) != w.XCodecDecoder(gd).decode_batch(streams[k:k + 16]):
                    raise AssertionError("coss decode differs")
            od.close()
            gd.close()
            seed += 1
            continue
        if kind == "dup":
            # a hash entered twice (test_gpu_dup's scenario, random order of the later calls), then
            # batches, device-resident runs (replayed by the library) and stream calls mixing x / y
            import test_gpu_dup as D
            want, gc, oc = D._run(ctx, oracle, 8, D._calls(bool(rng.random() < 0.7), int(rng.choice([0, 40, 70]))),
                                  bool(rng.random() < 0.5))
            x, y = D._collision_pair()
            p = W.pool(D.POOL)
            ge, oe = w.XCodecStreamEncoder(gc), oracle.Encoder(oc)
            for _ in range(int(rng.integers(2, 6))):
                parts = [x, y, p[2048 * int(rng.integers(D.POOL)):][:2048], W.gen(int(rng.integers(1 << 30)), 700)]
                bufs = [np.concatenate([parts[int(k)] for k in rng.integers(0, 4, int(rng.integers(1, 5)))])
                        for _ in range(int(rng.integers(1, 5)))]
                r = rng.random()
                if r < 0.4:
                    if D._device_run(gc, bufs, bool(rng.random() < 0.5)) != oc.encode_batch(bufs):
                        raise AssertionError("dup device run differs")
                elif r < 0.7:
                    if w.XCodecEncoder(gc).encode_batch(bufs) != oc.encode_batch(bufs):
                        raise AssertionError("dup batch differs")
                else:
                    for b in bufs:
                        if ge.encode(b) != oe.encode(b):
                            raise AssertionError("dup stream call differs")
                if len(gc) != len(oc):
                    raise AssertionError("dup sizes differ")
            if ge.flush() != oe.flush():
                raise AssertionError("dup final flush differs")
            gc.close()
            seed += 1
            continue
        oc = oracle.Cache()
        gc = w.XCodecCache(ctx, int(rng.choice([1024, 1 << 16])))
        oc.encode_batch(warm)
        w.XCodecEncoder(gc).encode_batch(warm)
        if kind == "plan":
            # device-resident plan: back-to-back restore + run (run / submit+wait / submit+poll) in
            # a random completion mode (stream ordered: no host synchronisation between runs)
            import torch
            gc.snapshot()
            bufs = F._batch(rng, pool)
            want = oc.encode_batch(bufs)
            plan = w.EncodePlan(gc, [len(b) for b in bufs])
            plan.set_completion(bool(rng.random() < 0.7))
            arena = np.zeros(plan.in_bytes, np.uint8)
            for i, b in enumerate(bufs):
                arena[int(plan.in_off[i]):int(plan.in_off[i]) + len(b)] = b
            d_in = torch.from_numpy(arena).cuda()
            reps = int(rng.integers(2, 5))
            outs = [(torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda"),
                     torch.zeros(len(bufs), dtype=torch.int64, device="cuda")) for _ in range(reps)]
            torch.cuda.synchronize()
            for r in range(reps):
                gc.restore_async()
                mode = int(rng.integers(3))
                if mode == 0:
                    plan.run(d_in.data_ptr(), outs[r][0].data_ptr(), outs[r][1].data_ptr())
                else:
                    plan.submit(d_in.data_ptr(), outs[r][0].data_ptr(), outs[r][1].data_ptr())
                    if mode == 1:
                        plan.wait()
                    else:
                        while not plan.poll():
                            pass
            ctx.sync()
            torch.cuda.synchronize()
            for r in range(reps):
                out, ln = outs[r][0].cpu().numpy(), outs[r][1].cpu().numpy()
                for i in range(len(bufs)):
                    o = int(plan.out_off[i])
                    if out[o:o + int(ln[i])].tobytes() != want[i]:
                        raise AssertionError(f"plan run {r} buffer {i} differs")
            plan.close()
        elif kind == "encode":
            for _ in range(int(rng.integers(1, 4))):
                bufs = F._batch(rng, pool)
                if oc.encode_batch(bufs) != w.XCodecEncoder(gc).encode_batch(bufs):
                    raise AssertionError("batch encode differs")
        elif kind == "streams":
            n = int(rng.integers(1, 12))
            oe = [oracle.Encoder(oc) for _ in range(n)]
            ge = [w.XCodecStreamEncoder(gc) for _ in range(n)]
            for _ in range(int(rng.integers(1, 4))):
                calls = []
                for buf in F._batch(rng, pool):
                    c = int(rng.integers(n))
                    cuts = sorted(rng.integers(0, max(buf.size, 1), int(rng.integers(0, 4))))
                    for piece in np.split(buf, cuts):
                        calls.append((c, piece, bool(rng.random() < 0.4)))
                want = []
                for c, d, f in calls:
                    o = oe[c].encode(d)
                    if f:
                        o += oe[c].flush()[1]
                    want.append(o)
                if w.encode_streams([(ge[c], d, f) for c, d, f in calls]) != want:
                    raise AssertionError("stream calls differ")
            for c in range(n):
                if ge[c].flush() != oe[c].flush():
                    raise AssertionError("final flush differs")
        elif kind == "dplan":
            bufs = F._batch(rng, pool)
            mangled = mangle(rng, oc.encode_batch(bufs))
            if rng.random() < 0.5:  # the same segments twice in the batch: EXTRACTs with earlier providers
                mangled = mangled + mangled[:int(rng.integers(1, len(mangled) + 1))]
            od, gd = oracle.Cache(), w.XCodecCache(ctx, 1 << 14)
            od.decode_batch(oracle.Cache().encode_batch(warm))
            w.XCodecDecoder(gd).decode_batch(oracle.Cache().encode_batch(warm))
            gd.snapshot()
            want = od.decode_batch(mangled)
            for got in plan_decode(gd, mangled, 2):
                if got != want:
                    raise AssertionError("plan decode differs")
        else:
            bufs = F._batch(rng, pool)
            streams = oc.encode_batch(bufs)
            mangled = mangle(rng, streams)
            od, gd = oracle.Cache(), w.XCodecCache(ctx, 1 << 12)
            od.decode_batch(oracle.Cache().encode_batch(warm))
            w.XCodecDecoder(gd).decode_batch(oracle.Cache().encode_batch(warm))
            if od.decode_batch(mangled) != w.XCodecDecoder(gd).decode_batch(mangled):
                raise AssertionError("decode differs")
    except Exception as e:  # noqa: BLE001
        fails += 1
        print("FAIL seed", seed, kind, os.environ["XC_CHUNK_BLOCKS"], os.environ["XC_SUB_MB"],
              os.environ["XC_NO_SHADOW"], repr(e)[:200], flush=True)
    seed += 1
print("done seeds", runs, "fails", fails, "next seed", seed, flush=True)
