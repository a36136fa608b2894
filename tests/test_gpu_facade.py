"""The drop-in boundary as the proxy uses it, on the GPU: the reference's own, unchanged
EncodeFilter / DecodeFilter (xcodec/xcodec_filter.cc:122-526) compiled against the facade
(facade/xcodec/) and linked with the product library, against the oracle pipes.

oracle/_ref/filter_turns (built in the container by `make -C oracle ref`, from the reference's
sources where they lie, and shipped with the tree; driver tests/facade/filter_turns.cc) runs 64
connections between two proxies turn by turn, one device call per consume (the reference's
unbatched pattern, xcodec_filter.cc:146-157): multi-consume streams, pool repeats that the peer's
empty decoder cache lacks (every one an <ASK> answered by a <LEARN>, xcodec_filter.cc:278-351,
441-455), F1-heavy reads, shifted repeats, <EOS>/<EOS_ACK> both ways.  The peer's decoder cache is
created by the real WanProxyCore::add_cache on <HELLO> with the reference's two arguments
(proxy/wanproxy.h:106-116), i.e. placed by xc_device_place.  Every connection's wire bytes both ways
and both sinks equal the oracle pipes' (tests/pipe_harness.py run_scenario)."""
import json
import os
import subprocess

import pytest

from pipe_harness import OracleBackend, read_outputs, run_scenario, write_scenario
from test_gpu_pipe_cpp import _scenario

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "filter_turns")


def _run(args, env=None):
    assert os.path.exists(BIN), "build first in the container (make -C oracle ref: needs /root/reference)"
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([BIN] + args, capture_output=True, text=True, timeout=600, env=e)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("seed", [3, 4])
def test_reference_filters_over_the_facade_equal_the_oracle_pipes(oracle_mod, tmp_path, seed):
    warm, order, inputs = _scenario(seed)
    sc, out = tmp_path / "scenario.bin", tmp_path / "out.bin"
    write_scenario(sc, warm, order, inputs, waiting=False, batched=False)
    log = _run(["parity", str(sc), str(out)])
    assert "filter_turns parity ok" in log, log
    # both caches made with the reference's arguments land on a device (a 1-GPU box: device 0)
    assert "A's cache on device 0" in log and "decoder cache for A on device 0" in log, log
    got = read_outputs(out, len(inputs))
    want = run_scenario(OracleBackend(oracle_mod), warm, order, inputs, waiting=False, batched=False)
    asks = 0
    for i, (g, e) in enumerate(zip(got, want)):
        assert g[0] == e[0], f"connection {i}: A->B wire bytes differ"
        assert g[1] == e[1], f"connection {i}: B->A wire bytes (ASK / EOS_ACK) differ"
        assert g[2] == e[2] == b"".join(bytes(x) for x in inputs[i]), f"connection {i}: decoded bytes differ"
        assert g[3] == e[3], f"connection {i}: A's sink differs"
        asks += g[1].count(b"\xfd")
    assert asks > 0, "the scenario never asked for a segment"


def test_reference_filter_encode_bench_runs(tmp_path):
    """The unbatched encode path through the reference's EncodeFilter (tools/pipe_bench_cpp.py
    --reference-filter measures it at size): one line, every read consumed."""
    warm, order, inputs = _scenario(5, nconn=16, turns=2)
    sc = tmp_path / "scenario.bin"
    write_scenario(sc, warm, order, inputs, waiting=False, batched=False)
    line = json.loads(_run(["bench", str(sc)]).strip().splitlines()[-1])
    assert line["consume_calls"] == sum(1 for row in inputs for x in row if len(x))
    assert line["bytes"] == sum(len(x) for row in inputs for x in row)
