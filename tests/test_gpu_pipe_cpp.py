"""The C++ pipe filters (include/xcodec_pipe.hpp: EncodeFilter / DecodeFilter of
xcodec/xcodec_filter.cc:122-526 with the cross-connection Batcher) on the GPU, against the oracle
pipes: 64 connections between two proxies, each read consumed in a shuffled order per event-loop
turn, the codec calls of a turn batched (xc_encode_streams, one decode batch per cache), the peer
asking for every segment its empty cache lacks (<ASK>/<LEARN>), <EOS>/<EOS_ACK> both ways.  Every
connection's wire bytes in both directions and both sinks equal the oracle pipes'."""
import os
import subprocess

import numpy as np
import pytest

from wanproxy_amd import workloads as W

from pipe_harness import OracleBackend, esc_buffer, read_outputs, run_scenario, write_scenario

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "pipe_turns")
POOL = 128


def _scenario(seed, nconn=64, turns=3):
    rng = np.random.default_rng(seed)
    p = W.pool(POOL)
    warm = W.pool_warmup_buffers(POOL)
    inputs = []
    for i in range(nconn):
        row = []
        for t in range(turns):
            r = rng.random()
            if r < 0.15:
                row.append(np.zeros(0, np.uint8))                      # no read this turn
            elif r < 0.6:
                row.append(W.repeat_buffers(1, int(rng.integers(1 << 30)), np_segments=POOL, pool_bytes=p)[0])
            elif r < 0.8:
                row.append(esc_buffer(int(rng.integers(1, 70000)), int(rng.integers(1 << 30))))
            else:                                                      # a shifted repeat of a pool run
                k = int(rng.integers(POOL - 8))
                row.append(np.concatenate([W.gen(int(rng.integers(1 << 30)), int(rng.integers(1, 3000))),
                                           p[k * 2048:(k + 6) * 2048]]))
        inputs.append(row)
    order = [list(map(int, rng.permutation(nconn))) for _ in range(turns)]
    return warm, order, inputs


@pytest.mark.parametrize("seed,waiting", [(1, False), (2, True)])
def test_cpp_filters_equal_the_oracle_pipes(oracle_mod, tmp_path, seed, waiting):
    assert os.path.exists(BIN), "build first (make -C wanproxy_amd/csrc)"
    warm, order, inputs = _scenario(seed)
    sc, out = tmp_path / "scenario.bin", tmp_path / "out.bin"
    write_scenario(sc, warm, order, inputs, waiting=waiting)
    r = subprocess.run([BIN, "parity", str(sc), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = read_outputs(out, len(inputs))
    want = run_scenario(OracleBackend(oracle_mod), warm, order, inputs, waiting=waiting)
    for i, (g, e) in enumerate(zip(got, want)):
        assert g[0] == e[0], f"connection {i}: A->B wire bytes differ"
        assert g[1] == e[1], f"connection {i}: B->A wire bytes (ASK / EOS_ACK) differ"
        assert g[2] == e[2] == b"".join(bytes(x) for x in inputs[i]), f"connection {i}: decoded bytes differ"
        assert g[3] == e[3], f"connection {i}: A's sink differs"
