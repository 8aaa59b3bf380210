"""Multi-GPU sharding of independent check batches: one process per GPU, contiguous
ranges of the batch index per rank, no collective on the data path.  A node that receives one
large batch splits it with `shard_range`, each rank verifies its slice on its own GPU, and the
tiny verdict bitmaps are gathered on rank 0 with `gather_verdicts` (torch.distributed; the gloo
backend suffices: the gather is host memory, 1 byte per check).  RCCL/xGMI is deliberately not
used: there is no cross-GPU reduction on this path.
"""
import numpy as np


def shard_range(n, rank, world):
    """[lo, hi) of the batch index owned by `rank` (balanced contiguous split)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def shard_by_instance(n_items, instance_of, rank, world):
    """Contiguous split that never cuts an instance (document / ciphertext) in two, so per-instance
    tables (H, W, H_uv and their Miller-loop lines) are prepared on one GPU only.  `instance_of` is a
    non-decreasing array of instance ids per item."""
    inst = np.asarray(instance_of)
    ninst = int(inst[-1]) + 1 if n_items else 0
    ilo, ihi = shard_range(ninst, rank, world)
    lo = int(np.searchsorted(inst, ilo, side="left"))
    hi = int(np.searchsorted(inst, ihi, side="left"))
    return lo, hi


def gather_verdicts(local, n, group=None):
    """Concatenate every rank's verdict bytes (in rank order) on rank 0; returns None elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = [None] * world if rank == 0 else None
    dist.gather_object(bytes(local), parts, dst=0, group=group)
    if rank != 0:
        return None
    out = b"".join(parts)
    if len(out) != n:
        raise RuntimeError("gathered %d verdicts, expected %d" % (len(out), n))
    return out
