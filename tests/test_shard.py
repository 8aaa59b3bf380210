"""N>1 path on CPU: world_size-2 gloo processes shard a batch by index / by instance and gather
the verdict bytes on rank 0 in the original order (the GPU work is replaced by a deterministic
per-item function so only the sharding and the host gather are under test)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from hbbft_amd.shard import gather_verdicts, shard_by_instance, shard_range


def test_shard_range_covers_batch():
    for n in (0, 1, 7, 65536):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_shard_by_instance_keeps_instances_whole():
    inst = np.repeat(np.arange(10), 64)
    spans = [shard_by_instance(len(inst), inst, r, 4) for r in range(4)]
    assert spans[0][0] == 0 and spans[-1][1] == len(inst)
    for lo, hi in spans:
        assert lo % 64 == 0 and hi % 64 == 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n, rank, world)
    local = bytes((i * 7 + 3) % 2 for i in range(lo, hi))  # stand-in verdicts
    out = gather_verdicts(local, n)
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_verdicts_gloo(world):
    n = 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert out == bytes((i * 7 + 3) % 2 for i in range(n))
