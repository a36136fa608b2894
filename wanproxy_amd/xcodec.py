"""Python host binding of libxcodec_hip.so (the C ABI in include/xcodec_hip.h).

Mirrors the reference's XCodec objects (bramfeld/wanproxy xcodec/):

* :class:`XCodecCache`  — XCodecMemoryCache (xcodec/xcodec_cache.h:162-211), device resident
* :class:`XCodecEncoder` — XCodecEncoder::encode + flush per buffer (xcodec/xcodec_encoder.cc:60-201)
* :class:`XCodecDecoder` — XCodecDecoder::decode per stream (xcodec/xcodec_decoder.cc:76-176)
* :class:`EncodePlan`   — a device-resident batch (inputs already in HBM) for benchmarks

There is no CPU fallback: if the HIP library or a GPU is missing, construction raises.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import threading
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# XC_LIB_PATH: an alternative build of the same library (A/B timing experiments, tools/ab.sh)
LIB_PATH = os.environ.get("XC_LIB_PATH") or os.path.join(HERE, "libxcodec_hip.so")
SEGMENT_LENGTH = 2048

SYMBOLS = [
    "xc_device_count", "xc_device_place", "xc_ctx_device", "xc_ctx_create", "xc_ctx_destroy", "xc_ctx_stream", "xc_ctx_sync",
    "xc_cache_create", "xc_cache_destroy", "xc_cache_count", "xc_cache_snapshot", "xc_cache_filter_stats",
    "xc_cache_restore", "xc_cache_lookup", "xc_cache_enter", "xc_hash_segments",
    "xc_window_hashes", "xc_encode_plan_create", "xc_encode_plan_create_sub", "xc_plan_destroy", "xc_plan_layout",
    "xc_encode_run", "xc_encode_batch_host", "xc_plan_stats", "xc_decode_batch_host",
    "xc_selftest", "xc_last_error", "xc_cache_restore_async", "xc_plan_set_timing",
    "xc_plan_kernel_times", "xc_host_alloc", "xc_host_free", "xc_encode_run_host",
    "xc_plan_set_streams", "xc_plan_stream_results", "xc_encoder_create", "xc_encoder_destroy",
    "xc_encoder_pending", "xc_encode", "xc_flush", "xc_encode_streams",
    "xc_decode_plan_create", "xc_dplan_destroy", "xc_dplan_layout", "xc_decode_run", "xc_dplan_stats",
    "xc_hash_segments_host", "xc_cache_capacity",
    "xc_coss_open", "xc_coss_close", "xc_coss_cache", "xc_coss_count", "xc_coss_stats", "xc_coss_lookup",
    "xc_coss_enter", "xc_coss_encode_batch_host", "xc_coss_decode_batch_host", "xc_coss_store_lookup",
    "xc_coss_store_enter", "xc_coss_encode_streams", "xc_encode_submit", "xc_encode_poll", "xc_encode_wait",
    "xc_plan_set_completion", "xc_dplan_set_completion", "xc_plan_set_scan", "xc_cache_quiesce",
    "xc_plan_set_input_ready", "xc_dplan_set_input_ready",
]
STREAM_FLUSH = 1  # XC_STREAM_FLUSH

KERNELS = ["scan", "resolve", "walk", "declhash", "emit", "blockhash"]


class XCodecError(RuntimeError):
    pass


class KernelTimes(C.Structure):
    _fields_ = [("ms", C.c_double * len(KERNELS)), ("launches", C.c_uint64 * len(KERNELS)),
                ("scan_bytes", C.c_uint64)]


class RunStats(C.Structure):
    _fields_ = [("n_extract", C.c_uint64), ("n_ref", C.c_uint64), ("in_bytes", C.c_uint64),
                ("out_bytes", C.c_uint64), ("sub_batches", C.c_uint32),
                ("walk_rounds", C.c_uint32), ("outer_rounds", C.c_uint32),
                ("dense_chunks", C.c_uint32), ("redone", C.c_uint32),
                ("shadow_misses", C.c_uint32), ("anchor_scans", C.c_uint32),
                ("anchor_fallbacks", C.c_uint32), ("early_hashed", C.c_uint32), ("reserved", C.c_uint32)]


class DecodeStats(C.Structure):
    _fields_ = [("in_bytes", C.c_uint64), ("n_extract", C.c_uint64), ("n_ref", C.c_uint64),
                ("n_entered", C.c_uint64), ("rounds", C.c_uint32)]


_LIB = None
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
_vp = C.c_void_p


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libxcodec_hip.so (raises if it was not built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # One HIP runtime per process: PyTorch ships its own libamdhip64 (same soname).  Loading
    # torch first makes this library bind to that copy instead of a second /opt/rocm one.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise XCodecError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path)
    for name in SYMBOLS:
        getattr(lib, name)  # every declared entry point must be exported
    lib.xc_last_error.restype = C.c_char_p
    lib.xc_ctx_stream.restype = _vp
    lib.xc_ctx_stream.argtypes = [_vp]
    lib.xc_device_count.argtypes = [C.POINTER(C.c_int)]
    lib.xc_device_place.argtypes = [_u8p, C.c_uint64, C.c_int]
    lib.xc_ctx_device.argtypes = [_vp, C.POINTER(C.c_int)]
    lib.xc_ctx_create.argtypes = [C.c_int, C.POINTER(_vp)]
    lib.xc_ctx_destroy.argtypes = [_vp]
    lib.xc_ctx_sync.argtypes = [_vp]
    lib.xc_cache_create.argtypes = [_vp, C.c_uint64, C.POINTER(_vp)]
    lib.xc_cache_destroy.argtypes = [_vp]
    lib.xc_cache_count.argtypes = [_vp, C.POINTER(C.c_uint64)]
    lib.xc_cache_capacity.argtypes = [_vp, C.POINTER(C.c_uint64)]
    lib.xc_cache_snapshot.argtypes = [_vp]
    lib.xc_cache_filter_stats.argtypes = [_vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.xc_cache_restore.argtypes = [_vp]
    lib.xc_cache_lookup.argtypes = [_vp, C.c_uint64, _u8p, C.POINTER(C.c_int)]
    lib.xc_cache_enter.argtypes = [_vp, C.c_uint64, _u8p]
    lib.xc_hash_segments.argtypes = [_vp, _vp, C.c_uint64, _vp, _vp]
    lib.xc_hash_segments_host.argtypes = [_vp, _u8p, C.c_uint64, _u64p]
    lib.xc_window_hashes.argtypes = [_vp, _vp, C.c_uint64, _vp, _vp]
    lib.xc_encode_plan_create.argtypes = [_vp, _u64p, C.c_uint64, C.POINTER(_vp)]
    lib.xc_encode_plan_create_sub.argtypes = [_vp, _u64p, C.c_uint64, C.c_uint64, C.POINTER(_vp)]
    lib.xc_plan_destroy.argtypes = [_vp]
    lib.xc_plan_layout.argtypes = [_vp, _u64p, _u64p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    lib.xc_encode_run.argtypes = [_vp, _vp, _vp, _vp]
    lib.xc_encode_submit.argtypes = [_vp, _vp, _vp, _vp]
    lib.xc_encode_poll.argtypes = [_vp, C.POINTER(C.c_int)]
    lib.xc_encode_wait.argtypes = [_vp]
    lib.xc_cache_quiesce.argtypes = [_vp]
    lib.xc_plan_set_input_ready.argtypes = [_vp, C.c_int]
    lib.xc_dplan_set_input_ready.argtypes = [_vp, C.c_int]
    lib.xc_plan_set_completion.argtypes = [_vp, C.c_int]
    lib.xc_plan_set_scan.argtypes = [_vp, C.c_int]
    lib.xc_plan_stats.argtypes = [_vp, C.POINTER(RunStats)]
    lib.xc_encode_batch_host.argtypes = [_vp, _u8p, _u64p, _u64p, C.c_uint64, _u8p, _u64p, _u64p,
                                         _u64p]
    lib.xc_decode_batch_host.argtypes = [_vp, _u8p, _u64p, _u64p, C.c_uint64, _u8p, _u64p, _u64p,
                                         _u64p, _u64p, _i32p, _u64p, _i32p]
    lib.xc__decode_bound.argtypes = [_u8p, _u64p, _u64p, C.c_uint64, _u64p]
    lib.xc_selftest.argtypes = [_vp]
    lib.xc_cache_restore_async.argtypes = [_vp]
    lib.xc_plan_set_timing.argtypes = [_vp, C.c_int]
    lib.xc_plan_kernel_times.argtypes = [_vp, C.POINTER(KernelTimes), C.c_int]
    lib.xc_host_alloc.argtypes = [_vp, C.c_uint64, C.POINTER(_vp)]
    lib.xc_host_free.argtypes = [_vp]
    lib.xc_encode_run_host.argtypes = [_vp, _vp, _vp, C.c_uint64, _u64p, _u64p]
    _i64p = np.ctypeslib.ndpointer(np.int64, flags="C")
    _u32p = np.ctypeslib.ndpointer(np.uint32, flags="C")
    lib.xc_plan_set_streams.argtypes = [_vp, _u64p, _i64p, _u32p]
    lib.xc_plan_stream_results.argtypes = [_vp, _u64p, _i64p]
    lib.xc_encoder_create.argtypes = [_vp, C.POINTER(_vp)]
    lib.xc_encoder_destroy.argtypes = [_vp]
    lib.xc_encoder_pending.argtypes = [_vp, C.POINTER(C.c_uint64)]
    lib.xc_encode.argtypes = [_vp, _u8p, C.c_uint64, _u8p, C.c_uint64, C.POINTER(C.c_uint64)]
    lib.xc_flush.argtypes = [_vp, _u8p, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_int)]
    lib.xc_encode_streams.argtypes = [C.POINTER(_vp), C.POINTER(C.c_void_p), _u64p, _u32p, C.c_uint64,
                                      _u8p, _u64p, _u64p, _u64p]
    lib.xc_decode_plan_create.argtypes = [_vp, _u64p, _u64p, C.c_uint64, C.POINTER(_vp)]
    lib.xc_dplan_destroy.argtypes = [_vp]
    lib.xc_dplan_layout.argtypes = [_vp, _u64p, _u64p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    lib.xc_decode_run.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    lib.xc_dplan_stats.argtypes = [_vp, C.POINTER(DecodeStats)]
    lib.xc_dplan_set_completion.argtypes = [_vp, C.c_int]
    lib.xc_coss_open.argtypes = [_vp, C.c_char_p, C.c_char_p, C.c_uint64, C.POINTER(_vp)]
    lib.xc_coss_close.argtypes = [_vp]
    lib.xc_coss_cache.restype = _vp
    lib.xc_coss_cache.argtypes = [_vp]
    lib.xc_coss_count.argtypes = [_vp, C.POINTER(C.c_uint64)]
    lib.xc_coss_stats.argtypes = [_vp, _u64p]
    for name in ("xc_coss_lookup", "xc_coss_store_lookup"):
        getattr(lib, name).argtypes = [_vp, C.c_uint64, _u8p, C.POINTER(C.c_int)]
    for name in ("xc_coss_enter", "xc_coss_store_enter"):
        getattr(lib, name).argtypes = [_vp, C.c_uint64, _u8p]
    lib.xc_coss_encode_batch_host.argtypes = lib.xc_encode_batch_host.argtypes
    lib.xc_coss_encode_streams.argtypes = [_vp] + list(lib.xc_encode_streams.argtypes)
    lib.xc_coss_decode_batch_host.argtypes = lib.xc_decode_batch_host.argtypes
    _LIB = lib
    return lib


# Native objects must be destroyed before the context they live on and before the HIP runtime
# tears itself down at process exit: keep weak references and release them in order at exit.
_LIVE = {"plan": weakref.WeakSet(), "coss": weakref.WeakSet(), "cache": weakref.WeakSet(), "ctx": weakref.WeakSet()}


@atexit.register
def _teardown() -> None:
    for kind in ("plan", "coss", "cache", "ctx"):
        for obj in list(_LIVE[kind]):
            try:
                obj.close()
            except Exception:
                pass


def _check(rc: int) -> None:
    if rc != 0:
        raise XCodecError(f"xcodec_hip error {rc}: {load_library().xc_last_error().decode()}")


def device_count() -> int:
    n = C.c_int(0)
    _check(load_library().xc_device_count(C.byref(n)))
    return n.value


class Context:
    """One GPU (xc_ctx) with its own HIP stream."""

    def __init__(self, device: int = 0):
        lib = load_library()
        self.h = _vp()
        _check(lib.xc_ctx_create(device, C.byref(self.h)))
        self.device = device
        _LIVE["ctx"].add(self)

    @property
    def stream(self) -> int:
        return load_library().xc_ctx_stream(self.h)

    def sync(self) -> None:
        _check(load_library().xc_ctx_sync(self.h))

    def selftest(self) -> None:
        _check(load_library().xc_selftest(self.h))

    def close(self) -> None:
        """Destroy the context; every cache / plan created on it is released first."""
        if getattr(self, "h", None):
            for kind in ("plan", "coss", "cache"):
                for obj in list(_LIVE[kind]):
                    if obj._ctx() is self:
                        obj.close()
            load_library().xc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _as_u8(b) -> np.ndarray:
    if isinstance(b, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(b), dtype=np.uint8)
    return np.ascontiguousarray(b, dtype=np.uint8)


def _pack(bufs):
    """The buffers back to back in a per-thread staging arena (valid until the thread's next
    _pack: the callers hand it to one library call; a fresh 64 MiB array per call paid its page
    faults every batch)."""
    lens = np.array([len(b) for b in bufs], dtype=np.uint64)
    offs = np.zeros(len(bufs), dtype=np.uint64)
    if len(bufs) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    total = int(lens.sum())
    arena = _scratch("pack", total)
    parts = [_as_u8(b) for b in bufs]
    # (a buffer that is itself a view of this thread's staging arena, e.g. from a nested call, would be
    # overwritten while it is copied: such a call packs into a fresh array)
    if any(p.size and np.shares_memory(p, arena) for p in parts):
        arena = np.empty(max(total, 1), np.uint8)
    if total:
        np.concatenate(parts, out=arena[:total])
    return arena, offs, lens


class XCodecCache:
    """XCodecMemoryCache (xcodec/xcodec_cache.h:162-211) held in HBM.

    ``capacity`` is the initial number of 2048-byte segments; like the reference's map, which
    grows without bound, the cache grows before any call that could fill it (xc_cache_create)."""

    def __init__(self, ctx: Context, capacity: int = 1 << 16):
        self.ctx = ctx
        self.h = _vp()
        _check(load_library().xc_cache_create(ctx.h, capacity, C.byref(self.h)))
        _LIVE["cache"].add(self)

    def _ctx(self):
        return self.ctx

    def __len__(self) -> int:
        n = C.c_uint64()
        _check(load_library().xc_cache_count(self.h, C.byref(n)))
        return n.value

    @property
    def capacity(self) -> int:
        """Segments the cache holds before it grows again (it grows on demand)."""
        n = C.c_uint64()
        _check(load_library().xc_cache_capacity(self.h, C.byref(n)))
        return n.value

    def _set_device_limit(self, slots: int) -> None:
        """(tests) The device's share of the segment slots: growth past it spills the segment
        bytes to pinned host memory (xc__cache_set_dev_limit)."""
        lib = load_library()
        lib.xc__cache_set_dev_limit.argtypes = [_vp, C.c_uint64]
        _check(lib.xc__cache_set_dev_limit(self.h, slots))

    def _tiers(self) -> tuple[int, int]:
        """(tests) Segment slots in HBM and in the spill tier."""
        lib = load_library()
        lib.xc__cache_tiers.argtypes = [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        a, b = C.c_uint64(), C.c_uint64()
        _check(lib.xc__cache_tiers(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def lookup(self, h: int) -> bytes | None:
        out = np.zeros(SEGMENT_LENGTH, np.uint8)
        found = C.c_int(0)
        _check(load_library().xc_cache_lookup(self.h, h, out, C.byref(found)))
        return out.tobytes() if found.value else None

    def enter(self, h: int, seg) -> None:
        seg = _as_u8(seg)
        assert seg.size == SEGMENT_LENGTH
        _check(load_library().xc_cache_enter(self.h, h, np.ascontiguousarray(seg)))

    def filter_stats(self) -> dict:
        """Diagnostic: false-positive rates of the level-1 (LDS) and level-2 (L2) filters for a
        random window end (from the filters' word occupancy)."""
        a, b = C.c_double(), C.c_double()
        _check(load_library().xc_cache_filter_stats(self.h, C.byref(a), C.byref(b)))
        return {"l1_fp": a.value, "l2_fp": b.value}

    def snapshot(self) -> None:
        _check(load_library().xc_cache_snapshot(self.h))

    def restore(self) -> None:
        _check(load_library().xc_cache_restore(self.h))

    def restore_async(self) -> None:
        """Enqueue the restore on the context stream (no host synchronisation)."""
        _check(load_library().xc_cache_restore_async(self.h))

    def quiesce(self) -> None:
        """Finish a run submitted on this cache and not yet waited for (xc_cache_quiesce)."""
        _check(load_library().xc_cache_quiesce(self.h))

    def hit_stats(self) -> dict:
        """(bench) The recent window's replay of encoder runs' lookup hits: runs and hits replayed,
        host seconds spent (xc__cache_hit_stats)."""
        lib = load_library()
        lib.xc__cache_hit_stats.argtypes = [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                            C.POINTER(C.c_double)]
        r, h, t = C.c_uint64(), C.c_uint64(), C.c_double()
        _check(lib.xc__cache_hit_stats(self.h, C.byref(r), C.byref(h), C.byref(t)))
        return {"runs": r.value, "hits": h.value, "host_s": t.value}

    def settle(self) -> None:
        """(bench) Replay every finished run's lookup hits into the recent window now (what the next
        window-dependent operation would do first)."""
        lib = load_library()
        lib.xc__cache_settle.argtypes = [_vp]
        _check(lib.xc__cache_settle(self.h))

    def close(self) -> None:
        if getattr(self, "h", None):
            for obj in list(_LIVE["plan"]):
                if obj.cache is self:
                    obj.close()
            load_library().xc_cache_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CossCache:
    """XCodecCacheCOSS (xcodec/cache/coss/xcodec_cache_coss.{h,cc}): the persistent stripe file
    ``<directory>/<uuid>.wpc`` with a device mirror on ``ctx`` (``ctx=None``: the host store alone,
    lookup / enter only).  ``XCodecEncoder`` / ``XCodecDecoder`` take it like an XCodecCache."""

    def __init__(self, ctx: Context | None, directory: str, uuid: str, size_mb: int = 0):
        self.ctx = ctx
        self.h = _vp()
        _check(load_library().xc_coss_open(ctx.h if ctx else None, directory.encode(), uuid.encode(), size_mb,
                                           C.byref(self.h)))
        _LIVE["coss"].add(self)

    def _ctx(self):
        return self.ctx

    def __len__(self) -> int:
        n = C.c_uint64()
        _check(load_library().xc_coss_count(self.h, C.byref(n)))
        return n.value

    def stats(self) -> dict:
        o = np.zeros(6, np.uint64)
        _check(load_library().xc_coss_stats(self.h, o))
        return dict(zip(["lookups", "found_1", "found_2", "index", "stripe_limit", "serial"], (int(x) for x in o)))

    def lookup(self, h: int, store_only: bool = False) -> bytes | None:
        """XCodecCacheCOSS::lookup (side effects included); ``store_only``: the host store alone."""
        out = np.zeros(SEGMENT_LENGTH, np.uint8)
        f = C.c_int()
        fn = load_library().xc_coss_store_lookup if store_only else load_library().xc_coss_lookup
        _check(fn(self.h, h, out, C.byref(f)))
        return out.tobytes() if f.value else None

    def enter(self, h: int, seg, store_only: bool = False) -> None:
        seg = np.ascontiguousarray(_as_u8(seg))
        fn = load_library().xc_coss_store_enter if store_only else load_library().xc_coss_enter
        _check(fn(self.h, h, seg))

    def _reread_headers(self) -> None:
        """(tests) the stripe headers read again from the file, as after another writer changed
        them; the device mirror follows (xc__coss_reread_headers)."""
        lib = load_library()
        lib.xc__coss_reread_headers.argtypes = [_vp]
        _check(lib.xc__coss_reread_headers(self.h))

    def close(self) -> None:
        """~XCodecCacheCOSS: the loaded stripes are written back."""
        if getattr(self, "h", None):
            load_library().xc_coss_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _window_hashes_host(data) -> np.ndarray:
    """(tests) the replay's host window hash (xc_replay.h WindowHash): the hash of every 2048-byte
    window of ``data``, in order."""
    d = np.ascontiguousarray(_as_u8(data))
    out = np.zeros(max(0, d.size - SEGMENT_LENGTH + 1), np.uint64)
    lib = load_library()
    lib.xc__window_hashes_host.argtypes = [_u8p, C.c_uint64, _u64p]
    _check(lib.xc__window_hashes_host(d, d.size, out))
    return out


class XCodecEncoder:
    """Batch form of XCodecEncoder: each buffer is ``encode(out, buf); flush(out)`` on a fresh
    encoder, buffers in index order, one shared cache (xcodec/xcodec_encoder.cc:60-201)."""

    def __init__(self, cache: XCodecCache):
        self.cache = cache

    def encode_batch(self, bufs) -> list[bytes]:
        arena, offs, lens = _pack(bufs)
        cap = lens * 2 + 16
        ooff = np.zeros(len(bufs), dtype=np.uint64)
        if len(bufs) > 1:
            ooff[1:] = np.cumsum(cap)[:-1]
        out = _scratch("encode", int(cap.sum()))
        olen = np.zeros(len(bufs), np.uint64)
        fn = (load_library().xc_coss_encode_batch_host if isinstance(self.cache, CossCache)
              else load_library().xc_encode_batch_host)
        _check(fn(self.cache.h, arena, offs, lens, len(bufs), out, ooff, cap, olen))
        return [out[int(o):int(o) + int(n)].tobytes() for o, n in zip(ooff, olen)]


class XCodecStreamEncoder:
    """XCodecEncoder across calls (xcodec/xcodec_encoder.h:43-63): one per connection, holding
    the reference's state between calls (pending source_ bytes and the candidate).

    ``encode(data)`` returns exactly the bytes the reference's ``encode(out, in)`` appends;
    ``flush()`` returns ``(bool, bytes)`` like ``flush(out)``.  :func:`encode_streams` runs the
    calls of many encoders as one device batch."""

    def __init__(self, cache):
        self.cache = cache
        self.h = _vp()
        # over a COSS cache: the encoder works on its device mirror, encode_streams on the COSS cache
        ch = _vp(load_library().xc_coss_cache(cache.h)) if isinstance(cache, CossCache) else cache.h
        _check(load_library().xc_encoder_create(ch, C.byref(self.h)))
        _LIVE["plan"].add(self)

    def _ctx(self):
        return self.cache.ctx

    @property
    def pending(self) -> int:
        n = C.c_uint64()
        _check(load_library().xc_encoder_pending(self.h, C.byref(n)))
        return n.value

    def encode(self, data) -> bytes:
        return encode_streams([(self, data, False)])[0]

    def flush(self) -> tuple[bool, bytes]:
        if isinstance(self.cache, CossCache):  # (the COSS state follows the flush's events)
            out = encode_streams([(self, b"", True)])[0]
            return len(out) > 0, out
        cap = 2 * self.pending + 16
        out = np.zeros(cap, np.uint8)
        n, em = C.c_uint64(), C.c_int()
        _check(load_library().xc_flush(self.h, out, cap, C.byref(n), C.byref(em)))
        return bool(em.value), out[:n.value].tobytes()

    def close(self) -> None:
        if getattr(self, "h", None):
            load_library().xc_encoder_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_TLS = threading.local()


def _scratch(name: str, n: int) -> np.ndarray:
    """A per-thread output staging array of at least n bytes, kept between calls: a fresh array
    per call pays a page fault per 4 KiB when the library first writes it.  (Results are copied
    out with ``tobytes`` before the next call.)"""
    d = _TLS.__dict__.setdefault("bufs", {})
    a = d.get(name)
    if a is None or a.size < n:
        a = np.empty(max(n, 1), np.uint8)
        d[name] = a
    return a[:max(n, 1)]


def encode_streams(calls) -> list[bytes]:
    """Cross-connection batch (xc_encode_streams): ``calls`` is a sequence of
    ``(encoder, data, flush)``, run in order as ``encoder.encode(data)`` then, when ``flush``,
    ``encoder.flush()`` (EncodeFilter::consume, xcodec/xcodec_filter.cc:122-164).  Returns each
    call's output bytes."""
    calls = list(calls)
    n = len(calls)
    if n == 0:
        return []
    datas = [_as_u8(d) for _, d, _ in calls]
    lens = np.array([d.size for d in datas], np.uint64)
    flags = np.array([STREAM_FLUSH if f else 0 for _, _, f in calls], np.uint32)
    # output bound: pending bytes at the call (at most all earlier input of that encoder)
    pend = {}
    cap = np.zeros(n, np.uint64)
    for k, (e, _, _) in enumerate(calls):
        p = pend.get(id(e), e.pending) + int(lens[k])
        cap[k] = 2 * p + 16
        pend[id(e)] = p
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(cap)[:-1]
    out = _scratch("streams", int(cap.sum()))
    olen = np.zeros(n, np.uint64)
    encs = (_vp * n)(*[e.h for e, _, _ in calls])
    ptrs = (C.c_void_p * n)(*[d.ctypes.data if d.size else None for d in datas])
    c0 = calls[0][0].cache
    if isinstance(c0, CossCache):
        if any(e.cache is not c0 for e, _, _ in calls):
            raise XCodecError("encode_streams: the encoders of one call share one cache")
        _check(load_library().xc_coss_encode_streams(c0.h, encs, ptrs, lens, flags, n, out, off, cap, olen))
    else:
        _check(load_library().xc_encode_streams(encs, ptrs, lens, flags, n, out, off, cap, olen))
    return [out[int(o):int(o) + int(m)].tobytes() for o, m in zip(off, olen)]


class XCodecDecoder:
    """Batch form of XCodecDecoder::decode (xcodec/xcodec_decoder.cc:76-176): one decode call
    per stream, streams in index order, one shared cache.  Returns, per stream,
    ``(status, decoded_bytes, consumed, unknown_hash_or_None)``."""

    def __init__(self, cache: XCodecCache):
        self.cache = cache

    def decode_batch(self, streams, out_cap: int | None = None):
        arena, offs, lens = _pack(streams)
        if out_cap is None:
            # a stream decodes to at most its length plus 2038 bytes per F1 byte in it (only a
            # <F1 02 hash> REF grows, 10 -> 2048 bytes; an EXTRACT keeps 2048 of 2050, an escape
            # shrinks): a tight bound, where 205 x the length would size gigabytes of staging
            cap = np.zeros(len(streams), np.uint64)
            _check(load_library().xc__decode_bound(arena, offs, lens, len(streams), cap))
        else:
            cap = np.full(len(streams), out_cap, np.uint64)
        ooff = np.zeros(len(streams), dtype=np.uint64)
        if len(streams) > 1:
            ooff[1:] = np.cumsum(cap)[:-1]
        out = _scratch("decode", int(cap.sum()))
        olen = np.zeros(len(streams), np.uint64)
        cons = np.zeros(len(streams), np.uint64)
        st = np.zeros(len(streams), np.int32)
        unk = np.zeros(len(streams), np.uint64)
        hu = np.zeros(len(streams), np.int32)
        fn = (load_library().xc_coss_decode_batch_host if isinstance(self.cache, CossCache)
              else load_library().xc_decode_batch_host)
        _check(fn(self.cache.h, arena, offs, lens, len(streams), out, ooff, cap, olen, cons, st, unk, hu))
        return [(int(st[i]), out[int(ooff[i]):int(ooff[i]) + int(olen[i])].tobytes(),
                 int(cons[i]), int(unk[i]) if hu[i] else None) for i in range(len(streams))]


class EncodePlan:
    """A device-resident encode batch: fixed buffer lengths, inputs/outputs in HBM arenas.

    ``run(d_in, d_out, d_len)`` takes raw device pointers (e.g. ``tensor.data_ptr()``)."""

    def __init__(self, cache: XCodecCache, lengths, sub_bytes: int = 0):
        """``sub_bytes``: the sub-batch bound on input bytes (0: the library's default;
        xc_encode_plan_create_sub).  A plan for ``run_host`` pipelines its copies per sub-batch."""
        self.cache = cache
        lens = np.ascontiguousarray(lengths, dtype=np.uint64)
        self.nbuf = len(lens)
        self.lengths = lens
        self.h = _vp()
        _check(load_library().xc_encode_plan_create_sub(cache.h, lens, self.nbuf, int(sub_bytes), C.byref(self.h)))
        self.in_off = np.zeros(self.nbuf, np.uint64)
        self.out_off = np.zeros(self.nbuf, np.uint64)
        ib, ob = C.c_uint64(), C.c_uint64()
        _check(load_library().xc_plan_layout(self.h, self.in_off, self.out_off, C.byref(ib),
                                             C.byref(ob)))
        self.in_bytes, self.out_bytes = ib.value, ob.value
        _LIVE["plan"].add(self)

    def _ctx(self):
        return self.cache.ctx

    def run(self, d_in: int, d_out: int, d_len: int) -> None:
        _check(load_library().xc_encode_run(self.h, d_in, d_out, d_len))

    def set_completion(self, stream_ordered: bool) -> None:
        """xc_plan_set_completion: with ``stream_ordered`` a run returns once it is decided and
        its last device writes complete in the order of the context stream (synchronize with
        ``Context.sync()`` or the device before reading the outputs from another stream)."""
        _check(load_library().xc_plan_set_completion(self.h, 1 if stream_ordered else 0))

    def set_input_ready(self, ready: bool) -> None:
        """xc_plan_set_input_ready: the input arena is complete whenever a run is submitted (not
        written by pending work on any stream), so the first sub-batch is hashed at once beside the
        previous run's last kernels."""
        _check(load_library().xc_plan_set_input_ready(self.h, 1 if ready else 0))

    def set_scan(self, mode: str) -> None:
        """xc_plan_set_scan: "auto" (default), "exact" or "anchor" (DESIGN.md §4.5)."""
        m = {"auto": 0, "exact": 1, "anchor": 2}[mode]
        _check(load_library().xc_plan_set_scan(self.h, m))

    def submit(self, d_in: int, d_out: int, d_len: int) -> None:
        """Enqueue a run and return at once (xc_encode_submit); finish it with poll() / wait()."""
        _check(load_library().xc_encode_submit(self.h, d_in, d_out, d_len))

    def poll(self) -> bool:
        """True once the submitted run has finished (raising if it failed); never blocks while
        the device works (xc_encode_poll)."""
        done = C.c_int(0)
        _check(load_library().xc_encode_poll(self.h, C.byref(done)))
        return bool(done.value)

    def wait(self) -> None:
        """Block until the submitted run has finished (xc_encode_wait)."""
        _check(load_library().xc_encode_wait(self.h))

    def run_host(self, h_in: "HostBuffer", h_out: "HostBuffer"):
        """End-to-end from host memory (xc_encode_run_host): ``h_in`` holds the input arena in
        the plan's layout, the encoded streams come back packed in ``h_out``.  Returns
        ``(lengths, positions)`` of every buffer's stream inside ``h_out``."""
        lens = np.zeros(max(self.nbuf, 1), np.uint64)
        pos = np.zeros(max(self.nbuf, 1), np.uint64)
        _check(load_library().xc_encode_run_host(self.h, h_in.ptr, h_out.ptr, h_out.nbytes, lens, pos))
        return lens[:self.nbuf], pos[:self.nbuf]

    def set_timing(self, mode) -> None:
        """HIP-event kernel timing: False (off), True (every kernel) or "scan" (the scan
        launches only: each event pair adds a few microseconds between dependent launches)."""
        m = 2 if mode == "scan" else (1 if mode else 0)
        _check(load_library().xc_plan_set_timing(self.h, m))

    def kernel_times(self, reset: bool = False) -> dict:
        kt = KernelTimes()
        _check(load_library().xc_plan_kernel_times(self.h, C.byref(kt), 1 if reset else 0))
        return {"ms": {k: kt.ms[i] for i, k in enumerate(KERNELS)},
                "launches": {k: int(kt.launches[i]) for i, k in enumerate(KERNELS)},
                "scan_bytes": int(kt.scan_bytes)}

    def stats(self) -> RunStats:
        st = RunStats()
        _check(load_library().xc_plan_stats(self.h, C.byref(st)))
        return st

    def close(self) -> None:
        if getattr(self, "h", None):
            load_library().xc_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DecodePlan:
    """A device-resident decode batch (xc_decode_plan_create / xc_decode_run): fixed stream
    lengths and output capacities, arenas in HBM.  ``run`` takes raw device pointers: the input
    and output arenas, then nbuf-long arrays out_len, consumed (u64), status (i32), unknown
    (u64), has_unknown (i32)."""

    def __init__(self, cache: XCodecCache, lengths, out_caps):
        self.cache = cache
        lens = np.ascontiguousarray(lengths, dtype=np.uint64)
        caps = np.ascontiguousarray(out_caps, dtype=np.uint64)
        self.nbuf = len(lens)
        self.h = _vp()
        _check(load_library().xc_decode_plan_create(cache.h, lens, caps, self.nbuf, C.byref(self.h)))
        self.in_off = np.zeros(self.nbuf, np.uint64)
        self.out_off = np.zeros(self.nbuf, np.uint64)
        ib, ob = C.c_uint64(), C.c_uint64()
        _check(load_library().xc_dplan_layout(self.h, self.in_off, self.out_off, C.byref(ib), C.byref(ob)))
        self.in_bytes, self.out_bytes = ib.value, ob.value
        _LIVE["plan"].add(self)

    def _ctx(self):
        return self.cache.ctx

    def run(self, d_in: int, d_out: int, d_out_len: int, d_consumed: int, d_status: int,
            d_unknown: int, d_has_unknown: int) -> None:
        _check(load_library().xc_decode_run(self.h, d_in, d_out, d_out_len, d_consumed, d_status,
                                            d_unknown, d_has_unknown))

    def set_completion(self, stream_ordered: bool) -> None:
        """xc_dplan_set_completion (see EncodePlan.set_completion)."""
        _check(load_library().xc_dplan_set_completion(self.h, 1 if stream_ordered else 0))

    def set_input_ready(self, ready: bool) -> None:
        """xc_dplan_set_input_ready (see EncodePlan.set_input_ready): the input is parsed on a side
        stream as soon as a run is submitted."""
        _check(load_library().xc_dplan_set_input_ready(self.h, 1 if ready else 0))

    def stats(self) -> DecodeStats:
        st = DecodeStats()
        _check(load_library().xc_dplan_stats(self.h, C.byref(st)))
        return st

    def close(self) -> None:
        if getattr(self, "h", None):
            load_library().xc_dplan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostBuffer:
    """Pinned, device-mapped host memory (xc_host_alloc) viewed as a numpy uint8 array."""

    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = _vp()
        _check(load_library().xc_host_alloc(ctx.h, self.nbytes, C.byref(p)))
        self.ptr = p.value
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(self.nbytes, 1)).from_address(self.ptr))
        _LIVE["plan"].add(self)  # released with the plans, before the context

    def _ctx(self):
        return self.ctx

    @property
    def cache(self):
        return None

    def close(self) -> None:
        if getattr(self, "ptr", None):
            self.array = None
            load_library().xc_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def hash_segments(ctx: Context, d_segs: int, n: int, d_out: int, stream: int | None = None) -> None:
    _check(load_library().xc_hash_segments(ctx.h, d_segs, n, d_out, stream))


def hash_segments_host(ctx: Context, segs) -> np.ndarray:
    """XCodecHash::hash (xcodec/xcodec_hash.h:166-174) of the consecutive 2048-byte segments in
    host memory ``segs``, computed on the device."""
    segs = np.ascontiguousarray(_as_u8(segs))
    if segs.size % SEGMENT_LENGTH:
        raise ValueError("segments must be whole 2048-byte blocks")
    n = segs.size // SEGMENT_LENGTH
    out = np.zeros(max(n, 1), np.uint64)
    _check(load_library().xc_hash_segments_host(ctx.h, segs, n, out))
    return out[:n]


def window_hashes(ctx: Context, d_in: int, n: int, d_out: int, stream: int | None = None) -> None:
    _check(load_library().xc_window_hashes(ctx.h, d_in, n, d_out, stream))
