"""The proxy's zlib stage: ``DeflateFilter`` / ``InflateFilter`` (``zlib/zlib_filter.{h,cc}``),
chained after the XCodec encoder and before the decoder when a codec sets ``compressor``
(``proxy/proxy_connector.cc:146-150,185-189``).  SURVEY.md §8(f)4.

The reference drives the system libz; so does this stage, through the same entry points with the
same call sequence and buffers (``deflateInit_`` / ``deflate`` / ``inflateInit_`` / ``inflate`` of
``libz.so.1`` over ctypes, a 64 KiB output chunk).  zlib is third-party, byte-serial code whose
output is defined by its own implementation (stored-block boundaries at level 0 even depend on how
the input is handed to it), so the stage stays on the host beside the device codec: a GPU deflate
could not reproduce libz's bytes, and the stage would be a different wire format.

Semantics kept from ``zlib_filter.cc``:

* ``consume``: the received Buffer's segments go through ``deflate`` with ``Z_NO_FLUSH``, the last
  one with ``Z_SYNC_FLUSH``, each call while input remains, appending the output chunk whenever a
  call produced some (``:37-65``); ``InflateFilter`` the same with ``inflate`` (``:117-147``): so
  output zlib still holds when a segment's input is used up comes with the next consume.  A Buffer
  here arrives as one byte string cut into 2048-byte segments (``common/buffer.h:74``: a socket
  read, ``event/io_service.cc:160-180``).  Levels 1-9 do not depend on that cut; level 0's stored
  blocks do, so a level-0 stage fed by a Buffer of another shape (the XCodec encoder's output
  Buffer is assembled from pieces) may cut its stored blocks elsewhere than the reference.
* ``flush``: ``deflate(Z_FINISH)`` is looped only while it returns ``Z_OK`` and produced output,
  so the call that ends the stream (``Z_STREAM_END``) never has its output sent (``:67-86``):
  after the consumes' sync flushes that is the whole tail (final block and Adler-32 trailer), and
  the peer's inflater never sees a stream end.  ``inflate(Z_FINISH)`` on an unfinished stream
  returns ``Z_BUF_ERROR`` (zlib 1.2.11), so the inflater's flush sends nothing (``:149-162``).
  Both then flush the chain.
* ``deflate`` returning ``Z_STREAM_ERROR`` / ``Z_DATA_ERROR`` / ``Z_MEM_ERROR``, or ``inflate``
  returning ``Z_NEED_DICT`` / ``Z_DATA_ERROR`` / ``Z_MEM_ERROR``, makes ``consume`` return
  ``False``.
"""
from __future__ import annotations

import ctypes as C

from .pipe import Filter

SEGMENT = 2048                  # BUFFER_SEGMENT_SIZE (common/buffer.h:74)
DEFLATE_CHUNK_SIZE = 0x10000    # zlib/zlib_filter.h:17
INFLATE_CHUNK_SIZE = 0x10000    # zlib/zlib_filter.h:18

Z_NO_FLUSH, Z_SYNC_FLUSH, Z_FINISH = 0, 2, 4
Z_OK, Z_STREAM_END, Z_NEED_DICT = 0, 1, 2
Z_STREAM_ERROR, Z_DATA_ERROR, Z_MEM_ERROR = -2, -3, -4


class ZStream(C.Structure):
    """``z_stream`` (zlib.h)."""
    _fields_ = [("next_in", C.c_void_p), ("avail_in", C.c_uint), ("total_in", C.c_ulong),
                ("next_out", C.c_void_p), ("avail_out", C.c_uint), ("total_out", C.c_ulong),
                ("msg", C.c_char_p), ("state", C.c_void_p), ("zalloc", C.c_void_p), ("zfree", C.c_void_p),
                ("opaque", C.c_void_p), ("data_type", C.c_int), ("adler", C.c_ulong), ("reserved", C.c_ulong)]


_Z = None


def _libz() -> C.CDLL:
    global _Z
    if _Z is None:
        z = C.CDLL("libz.so.1")
        z.zlibVersion.restype = C.c_char_p
        for name in ("deflateInit_", "inflateInit_"):
            getattr(z, name).argtypes = ([C.POINTER(ZStream), C.c_int, C.c_char_p, C.c_int] if name[0] == "d"
                                         else [C.POINTER(ZStream), C.c_char_p, C.c_int])
        for name in ("deflate", "inflate"):
            getattr(z, name).argtypes = [C.POINTER(ZStream), C.c_int]
        z.deflateEnd.argtypes = z.inflateEnd.argtypes = [C.POINTER(ZStream)]
        _Z = z
    return _Z


class _ZFilter(Filter):
    CHUNK = 0x10000

    def __init__(self):
        super().__init__()
        self.s = ZStream()
        self.out = C.create_string_buffer(self.CHUNK)
        self.s.next_out = C.cast(self.out, C.c_void_p)
        self.s.avail_out = self.CHUNK
        self.pending = b""

    def _take(self, acc: list) -> None:
        # zlib_filter.cc: the chunk is appended whenever the call produced output
        if self.s.avail_out < self.CHUNK:
            acc.append(self.out.raw[:self.CHUNK - self.s.avail_out])
            self.s.next_out = C.cast(self.out, C.c_void_p)
            self.s.avail_out = self.CHUNK

    def _segments(self, buf: bytes, step, bad, inflating: bool = False) -> bytes | None:
        data = bytes(buf)
        keep = C.create_string_buffer(data, len(data)) if data else None
        base = C.addressof(keep) if data else 0
        acc: list = []
        cnt = (len(data) + SEGMENT - 1) // SEGMENT
        for i in range(cnt):
            n = min(SEGMENT, len(data) - i * SEGMENT)
            self.s.next_in = base + i * SEGMENT
            self.s.avail_in = n
            while self.s.avail_in > 0:
                rv = step(C.byref(self.s), Z_NO_FLUSH if i < cnt - 1 else Z_SYNC_FLUSH)
                if rv in bad:
                    return None
                self._take(acc)
                if rv == Z_STREAM_END and self.s.avail_in > 0 and inflating:
                    return None  # (the reference would spin here: input past the stream's end)
        del keep
        return b"".join(acc)


class DeflateFilter(_ZFilter):
    """``zlib/zlib_filter.h:20-32``."""
    CHUNK = DEFLATE_CHUNK_SIZE

    def __init__(self, level: int = 0):
        super().__init__()
        z = _libz()
        if z.deflateInit_(C.byref(self.s), level, z.zlibVersion(), C.sizeof(ZStream)) != Z_OK:
            raise RuntimeError("Could not initialize deflate stream.")

    def consume(self, buf: bytes, flg: int = 0) -> bool:
        out = self._segments(buf, _libz().deflate, (Z_STREAM_ERROR, Z_DATA_ERROR, Z_MEM_ERROR))
        if out is None:
            return False  # "deflate(): ..."
        self.pending = out
        return self.produce(out, flg)

    def flush(self, flg: int) -> None:
        self.s.next_in = None
        self.s.avail_in = 0
        acc: list = []
        while _libz().deflate(C.byref(self.s), Z_FINISH) == Z_OK and self.s.avail_out < self.CHUNK:
            self._take(acc)
        self.pending = b"".join(acc)
        if self.pending:
            self.produce(self.pending)
        Filter.flush(self, flg)

    def __del__(self):
        if getattr(self, "s", None) is not None and _Z is not None:
            _Z.deflateEnd(C.byref(self.s))
            self.s = None


class InflateFilter(_ZFilter):
    """``zlib/zlib_filter.h:34-46``."""
    CHUNK = INFLATE_CHUNK_SIZE

    def __init__(self):
        super().__init__()
        z = _libz()
        if z.inflateInit_(C.byref(self.s), z.zlibVersion(), C.sizeof(ZStream)) != Z_OK:
            raise RuntimeError("Could not initialize inflate stream.")

    def consume(self, buf: bytes, flg: int = 0) -> bool:
        out = self._segments(buf, _libz().inflate, (Z_NEED_DICT, Z_DATA_ERROR, Z_MEM_ERROR), inflating=True)
        if out is None:
            return False  # "inflate(): ..."
        self.pending = out
        return self.produce(out, flg)

    def flush(self, flg: int) -> None:
        self.s.next_in = None
        self.s.avail_in = 0
        acc: list = []
        while _libz().inflate(C.byref(self.s), Z_FINISH) == Z_OK and self.s.avail_out < self.CHUNK:
            self._take(acc)
        self.pending = b"".join(acc)
        if self.pending:
            self.produce(self.pending)
        Filter.flush(self, flg)

    def __del__(self):
        if getattr(self, "s", None) is not None and _Z is not None:
            _Z.inflateEnd(C.byref(self.s))
            self.s = None
