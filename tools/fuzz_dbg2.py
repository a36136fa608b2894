"""Debug: the two-buffer batch [3, 4] of fuzz seed 0, device-resident, with plan statistics."""
import os
import sys
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'tools')
import torch
import oracle, wanproxy_amd as w
from wanproxy_amd import workloads as W
import test_gpu_fuzz as F
seed = 0
rng = np.random.default_rng(1000 + seed)
rng.choice([1, 2, 3, 5, 8]); rng.choice([1, 2, 512]); rng.random()
pool = W.pool(64)
warm = [pool[i:i + 65536] for i in range(0, int(rng.integers(1, 9)) * 65536, 65536)]
batches = [F._batch(rng, pool) for _ in range(2)]
bufs = [batches[0][3], batches[0][4]]
ctx = w.Context(0)
oc = oracle.Cache()
oc.encode_batch(warm)
want = oc.encode_batch(bufs)


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


print("want3", toks(want[0]))
print("want4", toks(want[1]))
# which block of buffer 3 has buffer 4's block 1
b4blk1 = bufs[1][2048:4096].tobytes()
b3 = bufs[0].tobytes()
print("buffer 4 block 1 found in buffer 3 at", b3.find(b4blk1))
gc = w.XCodecCache(ctx, 1 << 16)
w.XCodecEncoder(gc).encode_batch(warm)
plan = w.EncodePlan(gc, [b.size for b in bufs])
din = torch.zeros(plan.in_bytes, dtype=torch.uint8, device="cuda")
for i, b in enumerate(bufs):
    din[int(plan.in_off[i]):int(plan.in_off[i]) + b.size] = torch.from_numpy(b).cuda()
dout = torch.zeros(plan.out_bytes, dtype=torch.uint8, device="cuda")
dlen = torch.zeros(2, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
plan.run(din.data_ptr(), dout.data_ptr(), dlen.data_ptr())
torch.cuda.synchronize()
o = dout.cpu().numpy()
L = dlen.cpu().numpy()
got = [o[int(plan.out_off[i]):int(plan.out_off[i]) + int(L[i])].tobytes() for i in range(2)]
st = plan.stats()
print("equal", [g == e for g, e in zip(got, want)])
print("stats", {f: getattr(st, f) for f, _ in st._fields_})
print("got4", toks(got[1]))
