"""Multi-process GPU rehearsal of bench.py's N-GPU path on one MI355X.

bench.py --gpus N runs one process per GPU (torch.distributed.run), shards buffer i to rank i mod N
with a cache per rank and no data-path collective, and reduces only timings and
counts over gloo.  Here N ranks share the box's one GPU (bench.py maps local rank r to device
r mod device_count): every rank's shard of the full cfg5 job is encoded by the HIP path and checked
buffer by buffer against the oracle's independent run of that shard (the committed digests of
tests/golden/fullsize_digests.npz), and rank 0 prints the job's line."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_sharded_ranks_on_one_gpu(world):
    """world = 8 is the driver's 8-GPU launch shape (8 processes, 8 HIP contexts, gloo, each rank's
    4096-buffer shard as one sub-batch), here with all ranks on the one GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-cpu"]
    env = dict(os.environ, OMP_NUM_THREADS=str(max(1, 16 // world)))
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == world and r["config"]["buffers_per_gpu"] == 32768 // world
    assert r["verified_buffers"] == 32768, r["verified_against"]
    assert "cfg5_g%d" % world in r["verified_against"]
    assert r["roofline"]["peak"] == 8000.0 * world and r["value"] > 0
    # the committed PMC record of a rank-sized shard (profiles/r06/pmc_traffic_cfg5_b*.json), when it
    # was taken with these library sources, gives the line's traffic: a rank's bytes x N
    import bench
    rec = bench.pmc_traffic(int(r["stats"]["sub_batches"]), 32768 // world)
    if rec is not None:
        assert r["roofline"]["traffic"] == rec["traffic_bytes_per_step"] * world, r["roofline"]
        assert "x %d" % world in r["roofline"]["traffic_source"]
