"""ctypes binding of oracle/_ref/libzref.so — the reference's own DeflateFilter / InflateFilter
(zlib/zlib_filter.cc) built from /root/reference by oracle/Makefile (TEST INFRASTRUCTURE ONLY;
absent on the GPU box)."""
import ctypes as C
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(ROOT, "oracle", "_ref", "libzref.so")


def lib():
    if not os.path.exists(PATH):
        return None
    z = C.CDLL(PATH)
    z.zref_new.restype = C.c_void_p
    z.zref_new.argtypes = [C.c_int, C.c_int]
    z.zref_free.argtypes = [C.c_void_p]
    z.zref_consume.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    z.zref_flush.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    return z


class RefFilter:
    def __init__(self, z, deflate: bool, level: int = 0):
        self.z = z
        self.h = z.zref_new(1 if deflate else 0, level)
        self.buf = C.create_string_buffer(1 << 24)

    def consume(self, data: bytes):
        n = C.c_size_t()
        ok = self.z.zref_consume(self.h, data, len(data), self.buf, len(self.buf), C.byref(n))
        assert ok >= 0
        return bool(ok), self.buf.raw[:n.value]

    def flush(self) -> bytes:
        n = C.c_size_t()
        assert self.z.zref_flush(self.h, self.buf, len(self.buf), C.byref(n)) == 0
        return self.buf.raw[:n.value]

    def __del__(self):
        if getattr(self, "h", None):
            self.z.zref_free(self.h)
            self.h = None
