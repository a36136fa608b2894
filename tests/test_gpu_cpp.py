"""GPU test of the C++ host layer (include/xcodec_hip.hpp) through its check program
tests/cpp/xchip_roundtrip (built by __graft_entry__.build()): per-connection StreamEncoder calls
(XCodecEncoder::encode [+ flush], xcodec/xcodec_encoder.h:53-57) must append exactly what the
stateful oracle encoder appends, the same calls as one encode_streams batch must give the same
bytes, and Decoder (XCodecDecoder::decode) must give every connection's input back."""
import os
import struct
import subprocess

import numpy as np
import pytest

from wanproxy_amd import workloads as W

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROG = os.path.join(ROOT, "tests", "cpp", "xchip_roundtrip")


def _calls():
    rng = np.random.default_rng(7)
    pool = W.pool(64)
    calls = []
    for k in range(40):
        conn = int(rng.integers(0, 4))
        kind = k % 4
        if kind == 0:
            off = int(rng.integers(0, len(pool) - 9000))
            data = pool[off:off + int(rng.integers(100, 9000))]
        elif kind == 1:
            data = W.gen(100 + k, int(rng.integers(0, 7000)))
        elif kind == 2:
            data = rng.integers(0, 256, int(rng.integers(1, 5000)), dtype=np.uint8)
            data[rng.random(data.size) < 0.3] = 0xF1
        else:
            data = np.concatenate([pool[:4096], W.gen(k, 3000)])
        calls.append((conn, bool(rng.random() < 0.4), data.astype(np.uint8)))
    # every connection ends with a flush, so its stream decodes completely
    for c in range(4):
        calls.append((c, True, W.gen(900 + c, 1234)))
    return calls


def test_cpp_host_layer(tmp_path, oracle_mod):
    assert os.access(PROG, os.X_OK), "tests/cpp/xchip_roundtrip not built (run __graft_entry__.build())"
    calls = _calls()
    cf, of = tmp_path / "calls.bin", tmp_path / "out.bin"
    with open(cf, "wb") as f:
        f.write(struct.pack("<I", len(calls)))
        for conn, fl, data in calls:
            f.write(struct.pack("<IBI", conn, int(fl), data.size))
            f.write(data.tobytes())
    r = subprocess.run([PROG, str(cf), str(of)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "roundtrip ok" in r.stdout, r.stdout + r.stderr
    # every call's bytes against the stateful oracle
    raw = of.read_bytes()
    got, i = [], 0
    while i < len(raw):
        (n,) = struct.unpack_from("<I", raw, i)
        got.append(raw[i + 4:i + 4 + n])
        i += 4 + n
    oc = oracle_mod.Cache()
    enc = {}
    for k, (conn, fl, data) in enumerate(calls):
        e = enc.setdefault(conn, oracle_mod.Encoder(oc))
        want = e.encode(data)
        if fl:
            want += e.flush()[1]
        assert got[k] == want, k
