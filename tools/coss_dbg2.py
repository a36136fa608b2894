"""Debug helper: COSS batch encode vs the oracle (the test's phases), printing mismatches."""
import sys, tempfile
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import oracle, wanproxy_amd as w
from test_gpu_coss import _batches, _collision_batch, UUID_A
ctx = w.Context(0)
for cfg in sys.argv[1:]:
  size_mb, nb, per = (int(x) for x in cfg.split(","))
  print("config", cfg, flush=True)
  batches = _batches(nb, per, 0x501) + [_collision_batch()]
  cut = (2 * nb) // 3
  d1, d2 = tempfile.mkdtemp(), tempfile.mkdtemp()
  for ph, part in enumerate((batches[:cut], batches[cut:])):
      oc = oracle.Cache.coss(d1, UUID_A, size_mb)
      pc = w.CossCache(ctx, d2, UUID_A, size_mb)
      for k, bufs in enumerate(part):
          want = oc.encode_batch(bufs)
          got = w.XCodecEncoder(pc).encode_batch(bufs)
          bad = [i for i, (a, b) in enumerate(zip(want, got)) if a != b]
          print("phase", ph, "batch", k, "bad", bad[:5], len(oc), len(pc), flush=True)
          for i in bad[:2]:
              a, b = want[i], got[i]
              n = min(len(a), len(b))
              j = next((x for x in range(n) if a[x] != b[x]), n)
              print("  item", i, "len", len(bufs[i]), "out", len(a), len(b), "diff at", j, a[max(0, j - 4):j + 12].hex(), b[max(0, j - 4):j + 12].hex(), flush=True)
      oc.close(); pc.close()
