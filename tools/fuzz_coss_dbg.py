"""Debug one COSS seed of tools/fuzz_campaign.py (same generator), printing the first differing call."""
import os
import sys
import tempfile
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402


def toks(o):
    t, out, lit = 0, [], 0
    while t < len(o):
        if o[t] != 0xF1:
            lit += 1; t += 1; continue
        if o[t + 1] == 0:
            lit += 1; t += 2; continue
        if lit:
            out.append(("L", lit)); lit = 0
        if o[t + 1] == 1:
            out.append(("X", t)); t += 2050
        else:
            out.append(("R", int.from_bytes(bytes(o[t + 2:t + 10]), "big") & 0xFFFF)); t += 10
    if lit:
        out.append(("L", lit))
    return out


seed = int(sys.argv[1])
ctx = w.Context(0)
pool = W.pool(64)
rng = np.random.default_rng(seed)
os.environ["XC_CHUNK_BLOCKS"] = str(int(rng.choice([1, 2, 3, 5, 8])))
os.environ["XC_SUB_MB"] = str(int(rng.choice([1, 2, 512])))
os.environ["XC_NO_SHADOW"] = "1" if rng.random() < 0.3 else "0"
warm = [pool[i:i + 65536] for i in range(0, int(rng.integers(1, 9)) * 65536, 65536)]
size = int(rng.choice([3, 5, 17, 20]))
d1, d2 = tempfile.mkdtemp(), tempfile.mkdtemp()
uu = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0"
oc, gc = oracle.Cache.coss(d1, uu, size), w.CossCache(ctx, d2, uu, size)
n = int(rng.integers(1, 8))
print("size", size, "encoders", n, flush=True)
oe = [oracle.Encoder(oc) for _ in range(n)]
ge = [w.XCodecStreamEncoder(gc) for _ in range(n)]
for rnd in range(int(rng.integers(2, 6))):
    bufs = F._batch(rng, pool)
    if rng.random() < 0.5:
        want = oc.encode_batch(bufs)
        got = w.XCodecEncoder(gc).encode_batch(bufs)
        print("round", rnd, "batch", len(bufs), "equal", want == got, len(oc), len(gc), flush=True)
    else:
        calls = [(int(rng.integers(n)), b, bool(rng.random() < 0.5)) for b in bufs]
        pend = [e.pending for e in ge]
        want = []
        for c, d, f in calls:
            o = oe[c].encode(d)
            if f:
                o += oe[c].flush()[1]
            want.append(o)
        got = w.encode_streams([(ge[c], d, f) for c, d, f in calls])
        bad = [i for i, (a, b) in enumerate(zip(want, got)) if a != b]
        print("round", rnd, "calls", len(calls), "bad", bad[:5], len(oc), len(gc), flush=True)
        for i in range(min(len(calls), (bad[0] + 1) if bad else 0)):
            c, d, f = calls[i]
            xs = []
            o = want[i]
            t = 0
            while t < len(o):
                if o[t] == 0xF1 and o[t + 1] == 1:
                    xs.append(oracle.hash_segment(np.frombuffer(o[t + 2:t + 2050], np.uint8)) & 0xFFFF); t += 2050
                elif o[t] == 0xF1 and o[t + 1] == 2:
                    t += 10
                elif o[t] == 0xF1:
                    t += 2
                else:
                    t += 1
            print("  call", i, "conn", c, "len", d.size, "flush", f, "equal", want[i] == got[i], "declares", xs)
        for i in bad[:1]:
            c, d, f = calls[i]
            prev = [(k, calls[k][1].size, calls[k][2]) for k in range(i) if calls[k][0] == c]
            print(" call", i, "conn", c, "len", d.size, "flush", f, "pending at round start", pend[c], "earlier calls", prev)
            print(" want", toks(want[i])[:30])
            print(" got ", toks(got[i])[:30])
        if bad:
            break
