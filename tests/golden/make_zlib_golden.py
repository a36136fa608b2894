"""Generate tests/golden/zlib_filter_vectors.json: the reference DeflateFilter's bytes
(oracle/_ref/libzref.so, built from /root/reference/zlib/zlib_filter.cc) for a fixed sequence of
consumes at several levels, as sha256 + length per consume and flush.  Run here, where the
reference exists; the vectors pin wanproxy_amd/zlib_filter.py without it."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from zlib_ref import RefFilter, lib  # noqa: E402
from test_zlib import consume_inputs  # noqa: E402


def main():
    z = lib()
    assert z is not None, "make -C oracle ref first"
    out = {"source": "zlib/zlib_filter.cc (reference DeflateFilter, system libz)", "levels": {}}
    for level in (0, 1, 6, 9):
        f = RefFilter(z, True, level)
        rec = []
        for data in consume_inputs():
            ok, b = f.consume(data)
            assert ok
            rec.append([len(b), hashlib.sha256(b).hexdigest()])
        fl = f.flush()
        rec.append([len(fl), hashlib.sha256(fl).hexdigest()])
        out["levels"][str(level)] = rec
    json.dump(out, open(os.path.join(HERE, "zlib_filter_vectors.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
