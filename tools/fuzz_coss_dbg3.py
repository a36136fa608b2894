"""Debug COSS seed 7120: the failing request call by call, checking the device mirror for the
segment call 2 declares."""
import ctypes as C
import os
import sys
import tempfile
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
import wanproxy_amd as w  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402
from wanproxy_amd.xcodec import load_library  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402

seed = int(sys.argv[1])
mode = sys.argv[2] if len(sys.argv) > 2 else "batch"
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
lib = load_library()
mirror = C.c_void_p(lib.xc_coss_cache(gc.h))
n = int(rng.integers(1, 8))
oe = [oracle.Encoder(oc) for _ in range(n)]
ge = [w.XCodecStreamEncoder(gc) for _ in range(n)]


target_bytes = None


def dev_has(h):
    out = np.zeros(2048, np.uint8)
    f = C.c_int()
    lib.xc_cache_lookup(mirror, h, out, C.byref(f))
    if not f.value:
        return 0
    return "same bytes" if target_bytes is not None and out.tobytes() == target_bytes else "OTHER BYTES"


target = None
for rnd in range(int(rng.integers(2, 6))):
    bufs = F._batch(rng, pool)
    if rng.random() < 0.5:
        want = oc.encode_batch(bufs)
        got = w.XCodecEncoder(gc).encode_batch(bufs)
        print("round", rnd, "batch equal", want == got, flush=True)
        continue
    calls = [(int(rng.integers(n)), b, bool(rng.random() < 0.5)) for b in bufs]
    for i, (c, d, f) in enumerate(calls[:7]):
        o = oe[c].encode(d)
        if f:
            o += oe[c].flush()[1]
        if mode == "single":
            g = w.encode_streams([(ge[c], d, f)])[0]
        else:
            g = None
        xs = []
        t = 0
        while t < len(o):
            if o[t] == 0xF1 and o[t + 1] == 1:
                xs.append(oracle.hash_segment(np.frombuffer(o[t + 2:t + 2050], np.uint8)))
                if i == 2 and target_bytes is None:
                    target_bytes = bytes(o[t + 2:t + 2050])
                t += 2050
            elif o[t] == 0xF1 and o[t + 1] == 2:
                t += 10
            elif o[t] == 0xF1:
                t += 2
            else:
                t += 1
        if i == 2 and xs:
            target = xs[0]
            print("  target", hex(target), "store has", gc.lookup(target, store_only=True) == target_bytes if False else "")
        print(" call", i, "conn", c, "len", d.size, "flush", f, "equal" if g is None else g == o,
              "declares", [x & 0xFFFF for x in xs], "device has target", dev_has(target) if target else None,
              "pending", ge[c].pending, flush=True)
    break
