"""Winnowing rule check (round-3 experiment): with segments keyed by their
least-ranked anchor (fingerprint ascending, offset descending, offsets 63..2047), an input anchor a
needs a lookup only if some window start s has a as the least anchor of [s + 63, s + 2047]: with l / r
the nearest better anchors before / after a, s in [l - 62, r - 2048] ∩ [a - 2047, a - 63] ∩
[0, len - 2048].  Brute force over every window on random anchors (and tie-heavy fingerprints):
every window's least anchor is kept; ~6 % of anchors are.  usage: python tools/winnow_check.py"""
import random
def check(seed, L=20000, dens=64, ties=False):
    rnd = random.Random(seed)
    anchors = {}
    for p in range(63, L):
        if rnd.random() < 1/dens:
            anchors[p] = rnd.randrange(4 if ties else 1<<45)
    pos = sorted(anchors)
    rank = lambda p: (anchors[p], -p)   # least wins: fp asc, position desc
    FAR = 2047 - 62
    kept = set()
    for i, a in enumerate(pos):
        fp = anchors[a]
        Lb = None
        for k in range(i-1, -1, -1):
            pk = pos[k]
            if a - pk > FAR: break
            if anchors[pk] < fp: Lb = pk; break
        Rb = None
        for k in range(i+1, len(pos)):
            pk = pos[k]
            if pk - a > FAR: break
            if anchors[pk] <= fp: Rb = pk; break
        lo = max(Lb - 62 if Lb is not None else 0, a - 2047, 0)
        hi = min(Rb - 2048 if Rb is not None else 1<<30, a - 63, L - 2048)
        if lo <= hi: kept.add(a)
    # every window's least-ranked anchor in [s+63, s+2047] must be kept
    for s in range(0, L - 2047):
        inw = [p for p in pos if s + 63 <= p <= s + 2047]
        if not inw: continue
        best = min(inw, key=rank)
        assert best in kept, (seed, s, best)
    return len(kept), len(pos)
tot_k = tot = 0
for sd in range(6):
    k, n = check(sd); tot_k += k; tot += n
print("kept", tot_k, "of", tot, tot_k / tot)
for sd in range(3):
    k, n = check(100 + sd, ties=True)
print("ties ok")
