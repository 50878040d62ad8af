"""Multi-GPU sharding of one sketch + dist job.

One process per GPU.  Sequences (and so sketches) are split into contiguous shards;
every rank sketches its shard, the sketch rows are all-gathered (RCCL over xGMI with
the "nccl" backend, gloo on CPU in the tests) so each GPU holds the whole reference set,
and each rank computes its own query rows against all references.  The gather is the
only exchange; the dist rows of different ranks are independent.
"""
from __future__ import annotations


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Rows [lo, hi) of rank `rank` when n rows are split into `world` contiguous shards."""
    return n * rank // world, n * (rank + 1) // world


def all_gather_rows(local, n_total: int, world: int, group=None):
    """Concatenate every rank's `local` rows (a [n_local, w] tensor, any dtype) in rank
    order.  Shards may differ by one row: each is padded to the largest before the
    collective and the padding is dropped afterwards."""
    import torch
    import torch.distributed as dist

    m = max(hi - lo for lo, hi in (shard_range(n_total, world, r) for r in range(world)))
    shape = (m,) + tuple(local.shape[1:])
    buf = torch.zeros(shape, dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = [parts[r][: hi - lo] for r, (lo, hi) in
           enumerate(shard_range(n_total, world, r) for r in range(world))]
    return torch.cat(out, dim=0)
