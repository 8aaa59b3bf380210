"""N>1 path on CPU: world_size-2 gloo processes shard the golden ThresholdSign batch
(tests/golden/threshold_sign_n10_t3.json: 2 documents x 10 shares, forged kinds included) by
instance, verify their slice with the C oracle (the GPU engine's role on the box), and gather the
verdict bytes on rank 0 in the original order; the result equals the fixture's verdicts."""
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


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "threshold_sign_n10_t3.json")


def _batch():
    import json
    with open(GOLDEN) as f:
        d = json.load(f)
    items = [(m, s["idx"], bytes.fromhex(s["sig"]), bool(s["valid"])) for m, doc in enumerate(d["docs"])
             for s in doc["shares"]]
    return d, items


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cbls
    from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a
    d, items = _batch()
    inst = np.array([m for m, _, _, _ in items])
    lo, hi = shard_by_instance(len(items), inst, rank, world)
    pks = [g1a(bytes.fromhex(h)) for h in d["pk_shares"]]
    hs = [g2a(bytes.fromhex(doc["hash"])) for doc in d["docs"]]
    local = bytes(int(cbls.verify_g2(pks[i], g2a(sig), hs[m])) for m, i, sig, _ in items[lo:hi])
    out = gather_verdicts(local, len(items))
    if rank == 0:
        q.put((out, [(lo, hi)]))
    else:
        q.put((None, [(lo, hi)]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_shard_by_instance_golden_batch_gloo(world):
    from oracle import cbls
    if not os.path.exists(cbls.LIB_PATH):
        pytest.skip("C oracle not built")
    _, items = _batch()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    out = next(o for o, _ in got if o is not None)
    spans = sorted(sp[0] for _, sp in got)
    assert spans == [(0, 10), (10, 20)]  # one document per rank, never split
    assert out == bytes(int(v) for _, _, _, v in items)


def _max_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["HBH_DIST_BACKEND"] = "gloo"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    got = bench._max_over_ranks(10.0 + rank * 3.5, world, None)
    q.put((rank, got))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_bench_step_time_is_max_over_ranks_gloo(world):
    """bench.py's multi-rank timing: every rank gets the slowest rank's step time (the value the
    JSON line divides the job's units by)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_max_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == {r: 10.0 + (world - 1) * 3.5 for r in range(world)}
