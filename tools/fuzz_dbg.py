"""Debug helper for tests/test_gpu_fuzz.py: one seed under chosen settings, token-level diff of the
first mismatching buffer.  usage: python tools/fuzz_dbg.py SEED [CHUNK_BLOCKS SUB_MB NO_SHADOW]"""
import os
import sys
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
seed = int(sys.argv[1])
rng = np.random.default_rng(1000 + seed)
cb, sm, ns = int(rng.choice([1, 2, 3, 5, 8])), int(rng.choice([1, 2, 512])), rng.random() < 0.3
if len(sys.argv) > 2:
    cb, sm, ns = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "1"
if cb:
    os.environ["XC_CHUNK_BLOCKS"] = str(cb)
os.environ["XC_SUB_MB"] = str(sm)
if ns:
    os.environ["XC_NO_SHADOW"] = "1"
print("settings chunk", cb, "sub_mb", sm, "no_shadow", ns, flush=True)
import oracle, wanproxy_amd as w
from wanproxy_amd import workloads as W
import test_gpu_fuzz as F
pool = W.pool(64)
warm = [pool[i:i + 65536] for i in range(0, int(rng.integers(1, 9)) * 65536, 65536)]
batches = [F._batch(rng, pool) for _ in range(2)]
ctx = w.Context(0) if __name__ == "__main__" else None


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


if __name__ == "__main__":
    oc = oracle.Cache()
    gc = w.XCodecCache(ctx, 1 << 16)
    oc.encode_batch(warm)
    w.XCodecEncoder(gc).encode_batch(warm)
    for bi, bufs in enumerate(batches):
        want = oc.encode_batch(bufs)
        got = w.XCodecEncoder(gc).encode_batch(bufs)
        bad = [i for i, (a, b) in enumerate(zip(want, got)) if a != b]
        print("batch", bi, "bufs", len(bufs), "bad", bad[:8], flush=True)
        for i in bad[:1]:
            print(" buffer", i, "len", bufs[i].size)
            print(" want", toks(want[i])[:40])
            print(" got ", toks(got[i])[:40])
        if bad:
            break

    # split: the batch's buffers before the bad one, then the bad one alone
    if bad:
        i = bad[0]
        oc2, gc2 = oracle.Cache(), w.XCodecCache(ctx, 1 << 16)
        oc2.encode_batch(warm)
        w.XCodecEncoder(gc2).encode_batch(warm)
        for bb in batches[:bi]:
            oc2.encode_batch(bb)
            w.XCodecEncoder(gc2).encode_batch(bb)
        a1 = oc2.encode_batch(bufs[:i]); g1 = w.XCodecEncoder(gc2).encode_batch(bufs[:i])
        print("prefix equal", a1 == g1, flush=True)
        a2 = oc2.encode_batch([bufs[i]]); g2 = w.XCodecEncoder(gc2).encode_batch([bufs[i]])
        print("alone equal", a2 == g2, flush=True)
        # which earlier buffer declares the segment the oracle REFs
        want_t = toks(want[i])
        for j in range(i):
            tj = toks(want[j])
            print("  buf", j, "len", bufs[j].size, "tokens", tj[:12], flush=True)
