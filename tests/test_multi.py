"""Multi-process CPU tests of the sharded path (gloo, world_size 2).

cfg5 shards buffer i to rank i mod N, each rank with its own cache; there is no data-path
collective.  Here each rank encodes its shard with the oracle (the GPU is not
needed to check the sharding logic) and the checks are:
  * the shards partition the job (gathered buffer ids are 0..total-1 exactly once),
  * each rank's output equals an independent run over the same shard (no cross-rank state),
  * the bench's max-over-ranks timing reduction works over gloo.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import oracle
    from wanproxy_amd import workloads as W
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pool = W.pool(256)
    shard = W.repeat_shard(total, 0x5555, rank, world, np_segments=256, pool_bytes=pool)
    ids = torch.arange(rank, total, world, dtype=torch.int64)
    c = oracle.Cache()
    c.encode_batch([pool[i:i + W.BUF] for i in range(0, len(pool), W.BUF)])
    outs = c.encode_batch([shard[i] for i in range(shard.shape[0])])
    digest = hashlib.sha256(b"".join(outs)).hexdigest()
    gathered = [torch.zeros(total // world, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, ids)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write(f"{digest}\n{','.join(str(int(x)) for g in gathered for x in g)}\n{t.item()}\n")
    dist.destroy_process_group()


def test_sharded_encode_world2(tmp_path, oracle_mod):
    world, total = 2, 16
    mp.spawn(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    from wanproxy_amd import workloads as W
    pool = W.pool(256)
    for r in range(world):
        digest, ids, tmax = open(tmp_path / f"rank{r}.txt").read().split("\n")[:3]
        assert sorted(int(x) for x in ids.split(",")) == list(range(total))
        assert float(tmax) == float(world)
        # independent single-process run of the same shard
        shard = W.repeat_shard(total, 0x5555, r, world, np_segments=256, pool_bytes=pool)
        c = oracle_mod.Cache()
        c.encode_batch([pool[i:i + W.BUF] for i in range(0, len(pool), W.BUF)])
        outs = c.encode_batch([shard[i] for i in range(shard.shape[0])])
        assert hashlib.sha256(b"".join(outs)).hexdigest() == digest
    # the shards together are the job: buffer i of the full batch is shard[i % world][i // world]
    full = W.repeat_shard(total, 0x5555, np_segments=256, pool_bytes=pool)
    for r in range(world):
        sh = W.repeat_shard(total, 0x5555, r, world, np_segments=256, pool_bytes=pool)
        assert np.array_equal(sh, full[r::world])


def test_bench_cli_parses():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--help"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0 and "--gpus" in out.stdout


@pytest.mark.gpu
def test_bench_small_gpu():
    """bench.py end to end on one GPU with a small job (checks the JSON contract)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--total", "256", "--steps", "2",
                          "--warmup", "1", "--cpu-threads", "4"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    r = json.loads(line)
    for k in ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline", "cpu_baseline",
              "config", "dtype", "scaling"]:
        assert k in r
    assert r["value"] > 0 and r["verified_buffers"] > 0
    assert r["roofline"]["frac"] > 0 and r["cpu_baseline"]["cores"] >= 1
