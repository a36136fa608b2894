"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline.  The product path
(wanproxy_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_HASH_PATH = os.path.join(HERE, "_ref", "libxcref_hash.so")

_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C")


class XoBytes(C.Structure):
    _fields_ = [("data", C.c_void_p), ("len", C.c_size_t), ("cap", C.c_size_t)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    lib.xo_hash_segment.restype = C.c_uint64
    lib.xo_hash_segment.argtypes = [_u8p]
    lib.xo_window_hashes.argtypes = [_u8p, C.c_size_t, _u64p]
    lib.xo_cache_new.restype = C.c_void_p
    lib.xo_cache_clone.restype = C.c_void_p
    lib.xo_cache_clone.argtypes = [C.c_void_p]
    lib.xo_cache_free.argtypes = [C.c_void_p]
    lib.xo_cache_count.restype = C.c_size_t
    lib.xo_cache_count.argtypes = [C.c_void_p]
    lib.xo_cache_segments.restype = C.c_size_t
    lib.xo_cache_segments.argtypes = [C.c_void_p]
    lib.xo_cache_coss_load_misses.restype = C.c_uint64
    lib.xo_cache_coss_load_misses.argtypes = [C.c_void_p]
    lib.xo_cache_coss_stats.restype = C.c_int
    lib.xo_cache_coss_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    lib.xo_cache_entry.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64), C.c_void_p]
    lib.xo_cache_lookup.restype = C.c_int
    lib.xo_cache_lookup.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]
    lib.xo_cache_enter.argtypes = [C.c_void_p, C.c_uint64, _u8p]
    lib.xo_encode_batch.argtypes = [C.c_void_p, _u8p, _u64p, _u64p, C.c_size_t, _u8p, _u64p,
                                    _u64p, _u64p]
    lib.xo_decode_batch.argtypes = [C.c_void_p, _u8p, _u64p, _u64p, C.c_size_t, _u8p, _u64p,
                                    _u64p, _u64p, _u64p, _i32p, _u64p, _i32p]
    lib.xo_encoder_new.restype = C.c_void_p
    lib.xo_encoder_new.argtypes = [C.c_void_p]
    lib.xo_encoder_free.argtypes = [C.c_void_p]
    lib.xo_encode.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(XoBytes)]
    lib.xo_flush.argtypes = [C.c_void_p, C.POINTER(XoBytes)]
    lib.xo_flush.restype = C.c_int
    lib.xo_bytes_free.argtypes = [C.POINTER(XoBytes)]
    lib.xo_cache_new_coss.restype = C.c_void_p
    lib.xo_cache_new_coss.argtypes = [C.c_char_p, C.c_char_p, C.c_uint64]
    lib.xo_encode_sharded_timed.restype = C.c_double
    lib.xo_encode_sharded_timed.argtypes = [C.c_void_p, _u8p, _u64p, _u64p, C.c_size_t, C.c_int,
                                            C.POINTER(C.c_uint64)]
    return lib


_LIB = None


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = _load()
    return _LIB


def hash_segment(seg: np.ndarray) -> int:
    seg = np.ascontiguousarray(seg, dtype=np.uint8)
    assert seg.size == 2048
    return int(lib().xo_hash_segment(seg))


def window_hashes(data: np.ndarray) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.zeros(len(data), dtype=np.uint64)
    lib().xo_window_hashes(data, len(data), out)
    return out


def _as_u8(b):
    if isinstance(b, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(b), dtype=np.uint8)
    return np.asarray(b, dtype=np.uint8)


def _packed(bufs):
    lens = np.array([len(b) for b in bufs], dtype=np.uint64)
    offs = np.zeros(len(bufs), dtype=np.uint64)
    if len(bufs):
        offs[1:] = np.cumsum(lens)[:-1]
    arena = np.concatenate([_as_u8(b) for b in bufs]) if bufs else np.zeros(0, np.uint8)
    if arena.size == 0:
        arena = np.zeros(1, np.uint8)
    return np.ascontiguousarray(arena), offs, lens


class Cache:
    """XCodecMemoryCache restatement (shared across encode/decode calls)."""

    def __init__(self, handle=None):
        self.h = handle if handle is not None else lib().xo_cache_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().xo_cache_free(self.h)
            self.h = None

    @classmethod
    def coss(cls, directory: str, uuid: str, size_mb: int = 0) -> "Cache":
        """XCodecCacheCOSS (oracle/xc_coss.c) behind the same cache interface; closing it (del)
        runs the destructor's stores."""
        return cls(lib().xo_cache_new_coss(directory.encode(), uuid.encode(), size_mb))

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().xo_cache_free(self.h)
            self.h = None

    def clone(self) -> "Cache":
        return Cache(lib().xo_cache_clone(self.h))

    def __len__(self) -> int:
        return int(lib().xo_cache_count(self.h))

    def coss_stats(self) -> dict:
        """COSSStats of a COSS cache (lookups, window / stripe matches, index, stripe limit, serial)."""
        o = np.zeros(6, np.uint64)
        assert lib().xo_cache_coss_stats(self.h, o.ctypes.data_as(C.POINTER(C.c_uint64)))
        return dict(zip(["lookups", "found_1", "found_2", "index", "stripe_limit", "serial"], (int(x) for x in o)))

    def coss_load_misses(self) -> int:
        """(checks only) lookups that loaded a stripe and then missed (the <=16-stripe second-copy
        state, xcodec_cache_coss.cc:200-220)."""
        return int(lib().xo_cache_coss_load_misses(self.h))

    def entries(self) -> list[tuple[int, bytes]]:
        out = []
        for i in range(int(lib().xo_cache_segments(self.h))):
            h = C.c_uint64()
            seg = np.zeros(2048, np.uint8)
            lib().xo_cache_entry(self.h, i, C.byref(h), seg.ctypes.data_as(C.c_void_p))
            out.append((h.value, seg.tobytes()))
        return out

    def lookup(self, h: int) -> bytes | None:
        """XCodecMemoryCache::lookup (xcodec/xcodec_cache.h:190-210)."""
        p = C.c_void_p()
        if not lib().xo_cache_lookup(self.h, h, C.byref(p)):
            return None
        return C.string_at(p, 2048)

    def enter(self, h: int, seg) -> None:
        """XCodecMemoryCache::enter (xcodec/xcodec_cache.h:182-188)."""
        seg = np.ascontiguousarray(_as_u8(seg))
        assert seg.size == 2048
        lib().xo_cache_enter(self.h, h, seg)

    def encode_batch(self, bufs) -> list[bytes]:
        arena, offs, lens = _packed(bufs)
        cap = lens * 2 + 16
        ooff = np.zeros(len(bufs), dtype=np.uint64)
        if len(bufs):
            ooff[1:] = np.cumsum(cap)[:-1]
        out = np.zeros(max(1, int(cap.sum())), np.uint8)
        olen = np.zeros(len(bufs), np.uint64)
        rc = lib().xo_encode_batch(self.h, arena, offs, lens, len(bufs), out, ooff, cap, olen)
        assert rc == 0
        return [out[int(o):int(o) + int(n)].tobytes() for o, n in zip(ooff, olen)]

    def decode_batch(self, streams, out_cap=None):
        """Returns list of (status, decoded bytes, consumed, unknown-or-None)."""
        arena, offs, lens = _packed(streams)
        # A REF expands 10 -> 2048 bytes: 205x is the worst-case growth.
        cap = (lens * 205 + 16) if out_cap is None else np.full(len(streams), out_cap, np.uint64)
        ooff = np.zeros(len(streams), dtype=np.uint64)
        if len(streams):
            ooff[1:] = np.cumsum(cap)[:-1]
        out = np.zeros(max(1, int(cap.sum())), np.uint8)
        olen = np.zeros(len(streams), np.uint64)
        cons = np.zeros(len(streams), np.uint64)
        st = np.zeros(len(streams), np.int32)
        unk = np.zeros(len(streams), np.uint64)
        hu = np.zeros(len(streams), np.int32)
        rc = lib().xo_decode_batch(self.h, arena, offs, lens, len(streams), out, ooff, cap, olen,
                                   cons, st, unk, hu)
        assert rc == 0
        return [(int(st[i]), out[int(ooff[i]):int(ooff[i]) + int(olen[i])].tobytes(),
                 int(cons[i]), int(unk[i]) if hu[i] else None) for i in range(len(streams))]

    def encode_sharded_timed(self, bufs, nthreads: int) -> tuple[float, int]:
        arena, offs, lens = _packed(bufs)
        tot = C.c_uint64()
        secs = lib().xo_encode_sharded_timed(self.h, arena, offs, lens, len(bufs), nthreads,
                                             C.byref(tot))
        return float(secs), int(tot.value)


# -- the reference's own XCodecHash, compiled from its header (oracle/Makefile `ref`) --
class Encoder:
    """Stateful XCodecEncoder restatement (xcodec/xcodec_encoder.cc:43-201): encode() returns the
    bytes one reference encode(out, in) call appends, flush() -> (bool, bytes)."""

    def __init__(self, cache: Cache):
        self.cache = cache  # keeps the cache alive
        self.h = lib().xo_encoder_new(cache.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().xo_encoder_free(self.h)
            self.h = None

    @staticmethod
    def _take(b: XoBytes) -> bytes:
        out = C.string_at(b.data, b.len) if b.len else b""
        lib().xo_bytes_free(C.byref(b))
        return out

    def encode(self, data) -> bytes:
        d = np.ascontiguousarray(_as_u8(data))
        b = XoBytes()
        lib().xo_encode(self.h, d.ctypes.data if d.size else None, d.size, C.byref(b))
        return self._take(b)

    def flush(self) -> tuple[bool, bytes]:
        b = XoBytes()
        v = lib().xo_flush(self.h, C.byref(b))
        return bool(v), self._take(b)


def ref_hash_lib():
    if not os.path.exists(REF_HASH_PATH):
        return None
    rl = C.CDLL(REF_HASH_PATH)
    rl.xcref_hash_segment.restype = C.c_uint64
    rl.xcref_hash_segment.argtypes = [_u8p]
    rl.xcref_window_hashes.argtypes = [_u8p, C.c_size_t, _u64p]
    return rl
