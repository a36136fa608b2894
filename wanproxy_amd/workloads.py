"""Synthetic workloads of SURVEY.md §8(d) (splitmix64-seeded byte streams).

``gen(seed, n)`` emits the little-endian bytes of successive splitmix64 outputs
of a generator whose state starts at ``seed``.  The configs:

* cfg1: ``gen(1, 1 MiB)`` round trip (CPU plumbing).
* cfg2: 256 buffers ``gen(0x1000 + i, 64 KiB)``, empty cache.
* cfg3: 4096 buffers of 32 segment slots drawn from a splitmix64 state seeded
  0x77: ``r & 1`` -> pool segment ``(r >> 1) % NP`` else ``gen(r, 2048)``;
  cache warmed with the pool (NP = 8192 segments of ``gen(0xABCD, 16 MiB)``,
  encoded as 256 x 64 KiB buffers).
* cfg4: decode of cfg3's encoder output (variant 90 % repeats, seed 0x88).
* cfg5: 32768 buffers, 50 % repeats, seed 0x5555, buffer i -> GPU i mod G.
"""
from __future__ import annotations

import hashlib

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
SEG = 2048
POOL_SEGMENTS = 8192
BUF = 64 * 1024


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * M1
    z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def splitmix64_outputs(seed: int, count: int) -> np.ndarray:
    """The first ``count`` outputs of splitmix64 started at state ``seed``."""
    with np.errstate(over="ignore"):
        k = np.arange(1, count + 1, dtype=np.uint64)
        return _mix(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + k * GAMMA)


def gen(seed: int, n: int) -> np.ndarray:
    words = splitmix64_outputs(seed, (n + 7) // 8)
    return words.astype("<u8").view(np.uint8)[:n].copy()


class SplitMix64:
    """Sequential scalar splitmix64 (for the per-slot draws of cfg3/cfg5)."""

    def __init__(self, seed: int):
        self.state = seed & 0xFFFFFFFFFFFFFFFF

    def next(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def take(self, count: int) -> np.ndarray:
        out = splitmix64_outputs(self.state, count)
        with np.errstate(over="ignore"):
            self.state = int((np.uint64(self.state) + np.uint64(count) * GAMMA))
        return out


def pool(np_segments: int = POOL_SEGMENTS) -> np.ndarray:
    return gen(0xABCD, np_segments * SEG)


def pool_warmup_buffers(np_segments: int = POOL_SEGMENTS) -> list[np.ndarray]:
    p = pool(np_segments)
    return [p[i:i + BUF] for i in range(0, len(p), BUF)]


def random_buffers(count: int, size: int = BUF, seed0: int = 0x1000) -> list[np.ndarray]:
    """cfg2: ``gen(seed0 + i, size)``."""
    return [gen(seed0 + i, size) for i in range(count)]


def repeat_buffers(count: int, seed: int, repeat_pct: int = 50, slots: int = 32,
                   np_segments: int = POOL_SEGMENTS, pool_bytes: np.ndarray | None = None
                   ) -> list[np.ndarray]:
    """cfg3/cfg5 (50 %: ``r & 1``) and cfg4's variant (90 %: ``r % 10 < 9``)."""
    p = pool(np_segments) if pool_bytes is None else pool_bytes
    rng = SplitMix64(seed)
    draws = rng.take(count * slots)
    out = []
    for b in range(count):
        buf = np.empty(slots * SEG, dtype=np.uint8)
        for s in range(slots):
            r = int(draws[b * slots + s])
            rep = (r & 1) if repeat_pct == 50 else (r % 10 < 9)
            if rep:
                k = (r >> 1) % np_segments
                buf[s * SEG:(s + 1) * SEG] = p[k * SEG:(k + 1) * SEG]
            else:
                buf[s * SEG:(s + 1) * SEG] = gen(r, SEG)
        out.append(buf)
    return out


def gen_segments(seeds: np.ndarray, seg: int = SEG) -> np.ndarray:
    """Vectorised ``gen(seed, seg)`` for many seeds -> (len(seeds), seg) uint8."""
    seeds = np.asarray(seeds, dtype=np.uint64)
    words = seg // 8
    out = np.empty((len(seeds), seg), dtype=np.uint8)
    k = np.arange(1, words + 1, dtype=np.uint64) * GAMMA
    with np.errstate(over="ignore"):
        for i in range(0, len(seeds), 8192):
            z = _mix(seeds[i:i + 8192, None] + k[None, :])
            out[i:i + 8192] = z.astype("<u8").view(np.uint8).reshape(-1, seg)
    return out


def repeat_shard(total: int, seed: int, rank: int = 0, world: int = 1, repeat_pct: int = 50,
                 slots: int = 32, np_segments: int = POOL_SEGMENTS,
                 pool_bytes: np.ndarray | None = None) -> np.ndarray:
    """cfg5: buffers i = rank, rank + world, ... of the ``total``-buffer repeat workload
    (same draws as :func:`repeat_buffers`), as an array (n_local, slots * SEG)."""
    p = (pool(np_segments) if pool_bytes is None else pool_bytes).reshape(np_segments, SEG)
    draws = SplitMix64(seed).take(total * slots).reshape(total, slots)[rank::world]
    if repeat_pct == 50:
        rep = (draws & np.uint64(1)).astype(bool)
    else:
        rep = (draws % np.uint64(10)) < np.uint64(9)
    out = np.empty((draws.shape[0], slots, SEG), dtype=np.uint8)
    idx = ((draws >> np.uint64(1)) % np.uint64(np_segments)).astype(np.int64)
    out[rep] = p[idx[rep]]
    fresh = ~rep
    out[fresh] = gen_segments(draws[fresh])
    return out.reshape(draws.shape[0], slots * SEG)


def stream_digest(b) -> int:
    """First 8 bytes of sha256(b) as a little-endian uint64 (the per-buffer digest of
    tests/golden/fullsize_digests.npz)."""
    return int.from_bytes(hashlib.sha256(b).digest()[:8], "little")


def arena_digests(arena: np.ndarray, offs, lens) -> np.ndarray:
    """Per-buffer digests (:func:`stream_digest`) of the streams arena[offs[i]:offs[i]+lens[i]]."""
    mv = memoryview(np.ascontiguousarray(arena))
    return np.array([stream_digest(mv[int(o):int(o) + int(n)]) for o, n in zip(offs, lens)], np.uint64)


def pack(buffers: list[np.ndarray], align: int = 256) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Concatenate buffers into one arena with ``align``-byte aligned starts.

    Returns (arena, offsets, lengths) with uint64 offsets/lengths."""
    lens = np.array([len(b) for b in buffers], dtype=np.uint64)
    offs = np.zeros(len(buffers), dtype=np.uint64)
    pos = 0
    for i, b in enumerate(buffers):
        offs[i] = pos
        pos += (len(b) + align - 1) // align * align
    arena = np.zeros(pos + align, dtype=np.uint8)
    for i, b in enumerate(buffers):
        arena[int(offs[i]):int(offs[i]) + len(b)] = b
    return arena, offs, lens
