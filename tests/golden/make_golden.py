"""Generate tests/golden/ fixtures (run in the survey/build container, where
/root/reference exists).  Committed outputs are data only:

* hash_kats.json   — the 256 char-run KATs of the reference's own test
                     (xcodec/test/xcodec-hash1/xcodec-hash1.cc:34-291), parsed as numbers.
* window_hashes.npz — H at 4096 positions of gen(7, 256 KiB) and of an escape-heavy
                     buffer, computed by the reference XCodecHash class compiled from
                     its header (oracle/_ref/libxcref_hash.so).
* encode_vectors.json — sha256 + length of oracle encoder outputs for small cases
                     (regression vectors; the oracle itself is pinned by the two above and
                     by the reference's char-run round-trip intent).
"""
import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from wanproxy_amd import workloads as W  # noqa: E402

REF = "/root/reference"


def kats():
    src = open(os.path.join(REF, "xcodec/test/xcodec-hash1/xcodec-hash1.cc")).read()
    body = src[src.index("char_kats[]"):src.index("};", src.index("char_kats[]"))]
    vals = [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]+)ull", body)]
    assert len(vals) == 256, len(vals)
    return vals


def escape_heavy(n, seed):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    b[rng.random(n) < 0.3] = 0xF1
    return b


def main():
    json.dump({"source": "xcodec/test/xcodec-hash1/xcodec-hash1.cc:34-291",
               "kats": [f"0x{v:016x}" for v in kats()]},
              open(os.path.join(HERE, "hash_kats.json"), "w"), indent=1)

    rl = oracle.ref_hash_lib()
    assert rl is not None, "build oracle/_ref first: make -C oracle ref"
    out = {}
    for name, data in [("random", W.gen(7, 256 * 1024)), ("escape", escape_heavy(64 * 1024, 3))]:
        h = np.zeros(len(data), np.uint64)
        rl.xcref_window_hashes(data, len(data), h)
        rng = np.random.default_rng(11)
        pos = np.sort(rng.choice(np.arange(2047, len(data)), 4096, replace=False)).astype(np.uint64)
        out[name + "_seed"] = np.array([7 if name == "random" else 3], np.uint64)
        out[name + "_pos"] = pos
        out[name + "_hash"] = h[pos.astype(np.int64)]
    np.savez_compressed(os.path.join(HERE, "window_hashes.npz"), **out)

    vec = []
    cases = {
        "cfg1_gen1_1MiB": [W.gen(1, 1 << 20)],
        "tiny": [W.gen(5, 100), W.gen(6, 2047), W.gen(7, 2048), W.gen(8, 2049), W.gen(9, 4095),
                 W.gen(10, 4096), W.gen(11, 6143)],
        "charrun_f1_64k": [np.full(65536, 0xF1, np.uint8)],
        "escape_heavy": [escape_heavy(20000, 5), escape_heavy(70000, 6)],
        "cfg2_16": W.random_buffers(16),
    }
    for name, bufs in cases.items():
        c = oracle.Cache()
        outs = c.encode_batch(bufs)
        vec.append({"case": name, "lens": [len(o) for o in outs],
                    "sha256": [hashlib.sha256(o).hexdigest() for o in outs]})
    json.dump(vec, open(os.path.join(HERE, "encode_vectors.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
