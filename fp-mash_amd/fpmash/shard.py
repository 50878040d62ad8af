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


def kmer_shard(length: int, k: int, world: int, rank: int) -> tuple[int, int]:
    """Bases [lo, hi) of rank `rank` when one sequence of `length` bases is sketched by
    `world` GPUs: the k-mer starts are split into contiguous ranges and each range keeps the
    k - 1 bases after it (so every k-mer is hashed by exactly one rank)."""
    n_k = max(0, length - k + 1)
    a, b = shard_range(n_k, world, rank)
    return a, (b + k - 1 if b > a else a)


def min_merge(ctx, d_row: int, d_count: int, s: int, world: int, group=None, device=None):
    """The cross-GPU min-merge of one sketch computed in parts: every rank's bottom-s row
    (device pointers: s u64 hashes + a u32 count) is all-gathered (RCCL over xGMI with an
    "nccl" group, or host tensors over gloo when `device` is None) and merged on the device
    with fpm_sketch_merge_dev (MinHashHeap.cpp:68-146: the s smallest distinct of a union are
    the s smallest of the union of the parts' s smallest).  Returns (hashes, count) as host
    arrays."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import fpmash
    L = fpmash.lib()
    dev = device if device is not None else torch.device("cpu")
    row = torch.zeros((1, s + 1), dtype=torch.int64, device=dev)   # hashes, then the count
    if device is not None:
        fpmash._check(L.fpm_memcpy_d2d(ctx.h, row.data_ptr(), d_row, s * 8))
        fpmash._check(L.fpm_memcpy_d2d(ctx.h, row.data_ptr() + s * 8, d_count, 4))
        ctx.synchronize()
    else:
        fpmash._check(L.fpm_memcpy_d2h(ctx.h, row.data_ptr(), d_row, s * 8))
        c = np.zeros(1, np.uint32)
        fpmash._check(L.fpm_memcpy_d2h(ctx.h, c.ctypes.data, d_count, 4))
        row[0, s] = int(c[0])
    parts = [torch.empty_like(row) for _ in range(world)]
    dist.all_gather(parts, row, group=group)
    allr = torch.cat(parts, dim=0)                                   # [world, s + 1]
    if device is None:
        allr_np = allr.numpy()
        rows = fpmash.DeviceBuffer.from_array(ctx, np.ascontiguousarray(allr_np[:, :s]))
        cnts = fpmash.DeviceBuffer.from_array(ctx, allr_np[:, s].astype(np.uint32))
        rp, cp = rows.ptr, cnts.ptr
    else:
        rows_t = allr[:, :s].contiguous()
        cnts_t = allr[:, s].to(torch.int32).contiguous()
        torch.cuda.synchronize(dev)
        rp, cp = rows_t.data_ptr(), cnts_t.data_ptr()
    out = fpmash.DeviceBuffer(ctx, s * 8)
    oc = fpmash.DeviceBuffer(ctx, 4)
    fpmash._check(L.fpm_sketch_merge_dev(ctx.h, rp, cp, world, s, out.ptr, oc.ptr, None))
    ctx.synchronize()
    n = int(oc.to_array(np.uint32, 1)[0])
    h = out.to_array(np.uint64, s)[:n]
    out.free()
    oc.free()
    return h, n
