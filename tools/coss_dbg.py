"""Debug helper: COSS stream encoders vs the oracle, turn by turn."""
import sys, tempfile
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import oracle, wanproxy_amd as w
from test_gpu_coss import _batches, UUID_A
size_mb = int(sys.argv[1])
ctx = w.Context(0)
do, dp = tempfile.mkdtemp(), tempfile.mkdtemp()
oc = oracle.Cache.coss(do, UUID_A, size_mb)
pc = w.CossCache(ctx, dp, UUID_A, size_mb)
rng = np.random.default_rng(size_mb)
nconn = 24
oenc = [oracle.Encoder(oc) for _ in range(nconn)]
genc = [w.XCodecStreamEncoder(pc) for _ in range(nconn)]
conns = []
for k, bufs in enumerate(_batches(4 if size_mb == 3 else 10, nconn, 0x900 + size_mb)):
    for c in range(nconn):
        conns.append((c, bufs[c]))
for turn in range(0, len(conns), nconn):
    calls = []
    for c, buf in conns[turn:turn + nconn]:
        cuts = sorted(rng.integers(0, len(buf), 2))
        for piece in np.split(buf, cuts):
            calls.append((c, piece, bool(rng.random() < 0.3)))
    rng.shuffle(calls)
    pend = [genc[c].pending for c in range(nconn)]
    want = []
    for c, d, f in calls:
        o = oenc[c].encode(d)
        if f:
            o += oenc[c].flush()[1]
        want.append(o)
    got = w.encode_streams([(genc[c], d, f) for c, d, f in calls])
    bad = [i for i, (a, b) in enumerate(zip(want, got)) if a != b]
    print("turn", turn, "calls", len(calls), "bad", bad[:5], "len", len(oc), len(pc), oc_stats if (oc_stats:=None) else "", pc.stats(), flush=True)
    for i in bad[:2]:
        c, d, f = calls[i]
        a, b = want[i], got[i]
        n = min(len(a), len(b))
        j = next((x for x in range(n) if a[x] != b[x]), n)
        prev = [k for k in range(i) if calls[k][0] == c]
        print(" call", i, "conn", c, "len", len(d), "flush", f, "pending before turn", pend[c], "earlier calls this turn", prev,
              "out lens", len(a), len(b), "first diff", j, "want", a[max(0,j-4):j+12].hex(), "got", b[max(0,j-4):j+12].hex(), flush=True)
    if bad:
        break
