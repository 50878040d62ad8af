"""Multi-GPU sharding of one sketch + dist job (configs C4 / C5 and a split
genome).  One process per GPU, no exchange in the C4 / C5 data paths:

* C4 (all-vs-all dist): the set is cut into contiguous row blocks and the grid is dealt as
  unordered block pairs (pair_block_jobs); every rank sketches the rows its pairs read from
  the inputs it holds, so no sketch row crosses GPUs.
* C5 (one sketch per genome file): contiguous file ranges per rank; the finished sketches are
  reassembled in file order on rank 0 on the host (all_gather_rows over gloo).
* One sketch split over GPUs (a genome's k-mer ranges, kmer_shard): the bottom-s rows are
  min-merged through RCCL inside libfpmash (min_merge with an fpmash.Comm) -- the one
  collective north_star names ("the final min-merge").
"""
from __future__ import annotations


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Rows [lo, hi) of rank `rank` when n rows are split into `world` contiguous shards."""
    return n * rank // world, n * (rank + 1) // world


def all_gather_rows(local, n_total: int, world: int, group=None, bounds=None, out=None,
                    async_op: bool = False):
    """Concatenate every rank's `local` rows (a [n_local, w] host tensor over gloo, any dtype)
    in rank order (the C5 leg's ordered reassembly of per-file sketches on rank 0).  Shards may differ in size (`bounds`: each rank's [lo, hi), default
    shard_range): each is padded to the largest before the collective and the padding is
    dropped afterwards.  `out`: a preallocated [n_total, w] tensor to write into (its storage
    stays put across calls, so device pointers into it stay valid).  async_op: the
    collective is only launched, and a function is returned that waits for it and returns
    the rows (work on other streams can run meanwhile)."""
    import torch
    import torch.distributed as dist

    if bounds is None:
        bounds = [shard_range(n_total, world, r) for r in range(world)]
    m = max(hi - lo for lo, hi in bounds)
    shape = (m,) + tuple(local.shape[1:])
    buf = torch.zeros(shape, dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    work = dist.all_gather(parts, buf, group=group, async_op=async_op)

    def finish():
        if work is not None:
            work.wait()
        pieces = [parts[r][: hi - lo] for r, (lo, hi) in enumerate(bounds)]
        if out is None:
            return torch.cat(pieces, dim=0)
        torch.cat(pieces, dim=0, out=out)
        return out
    return finish if async_op else finish()


def pair_block_jobs(bounds, rank: int):
    """The all-vs-all dist of one set split into contiguous row blocks (`bounds`: block b =
    rows [lo, hi), block b owned by rank b), dealt so that every UNORDERED pair of rows is
    compared on exactly one rank and every ordered cell (query q, ref r) of the n x n grid is
    written on exactly one rank.  The results of sorted distinct sketches are symmetric
    (compareSketches, CommandDistance.cpp:365-430, is a merge of two sets), so a pair of
    blocks is compared once and written twice (fpm_refset_dist_mirror_dev), and a block
    against itself takes the library's symmetric self path.  Rank i indexes its own block
    and compares, as queries against it:
      * its own block ("self": one grid, the symmetric path);
      * the rows of the (ws - 1) // 2 blocks after it (cyclic), and for even ws the first
        half of block i + ws/2 when i < ws/2 ("mirror": grid qry x ref + its transpose);
      * for even ws and i >= ws/2: the second half of its own block against block i - ws/2
        (a second index), the other half of the pair {i - ws/2, i}.
    Each rank then compares ~n^2 / (2 ws) pairs and writes ~n^2 / ws cells.  Returns a list of
    {"kind": "self" | "mirror", "ref": (lo, hi), "qry": (lo, hi)}; contiguous query blocks are
    merged into one job (a cyclic wrap splits them)."""
    ws = len(bounds)
    lo, hi = bounds[rank]
    jobs = [{"kind": "self", "ref": (lo, hi), "qry": (lo, hi)}]
    if ws == 1:
        return [j for j in jobs if hi > lo]
    h = ws // 2
    segs = []
    for d in range(1, (ws - 1) // 2 + 1):
        segs.append(list(bounds[(rank + d) % ws]))
    if ws % 2 == 0 and rank < h:
        blo, bhi = bounds[rank + h]
        segs.append([blo, blo + (bhi - blo) // 2])
    merged = []
    for a, b in segs:
        if merged and merged[-1][1] == a:
            merged[-1][1] = b
        else:
            merged.append([a, b])
    for a, b in merged:
        jobs.append({"kind": "mirror", "ref": (lo, hi), "qry": (a, b)})
    if ws % 2 == 0 and rank >= h:
        jobs.append({"kind": "mirror", "ref": tuple(bounds[rank - h]),
                     "qry": (lo + (hi - lo) // 2, hi)})
    return [j for j in jobs if j["ref"][1] > j["ref"][0] and j["qry"][1] > j["qry"][0]]


def job_cells(job):
    """The ordered cells (query row, ref row) a pair_block_jobs job writes: the grid rows x
    columns, and for a mirror job its transpose too."""
    (rl, rh), (ql, qh) = job["ref"], job["qry"]
    cells = [(q, r) for q in range(ql, qh) for r in range(rl, rh)]
    if job["kind"] == "mirror":
        cells += [(r, q) for q in range(ql, qh) for r in range(rl, rh)]
    return cells


def kmer_shard(length: int, k: int, world: int, rank: int) -> tuple[int, int]:
    """Bases [lo, hi) of rank `rank` when one sequence of `length` bases is sketched by
    `world` GPUs: the k-mer starts are split into contiguous ranges and each range keeps the
    k - 1 bases after it (so every k-mer is hashed by exactly one rank)."""
    n_k = max(0, length - k + 1)
    a, b = shard_range(n_k, world, rank)
    return a, (b + k - 1 if b > a else a)


def min_merge(ctx, d_row: int, d_count: int, s: int, world: int, comm=None, group=None):
    """The cross-GPU min-merge of one sketch computed in parts (north_star: RCCL "for the final
    min-merge"): every rank's bottom-s row (device pointers: s u64 hashes + a u32 count) is
    merged with every other rank's (MinHashHeap.cpp:68-146: the s smallest distinct of a union
    are the s smallest of the union of the parts' s smallest).  With `comm` (fpmash.Comm) the
    rows are all-gathered by RCCL over xGMI inside libfpmash and merged on the device on the
    context stream (fpm_sketch_min_merge_comm: no host step between them); without it (ranks
    sharing one GPU in the tests and rehearsals, where RCCL refuses two ranks per device) the
    rows go through the gloo `group` as host tensors and are merged by fpm_sketch_merge_dev.
    Returns (hashes, count) as host arrays."""
    import numpy as np

    import fpmash
    L = fpmash.lib()
    out = fpmash.DeviceBuffer(ctx, s * 8)
    oc = fpmash.DeviceBuffer(ctx, 4)
    if comm is not None:
        comm.min_merge(d_row, d_count, s, out.ptr, oc.ptr)
    else:
        import torch
        import torch.distributed as dist
        row = np.zeros((1, s + 1), np.int64)                       # hashes, then the count
        fpmash._check(L.fpm_memcpy_d2h(ctx.h, row.ctypes.data, d_row, s * 8))
        c = np.zeros(1, np.uint32)
        fpmash._check(L.fpm_memcpy_d2h(ctx.h, c.ctypes.data, d_count, 4))
        row[0, s] = int(c[0])
        t = torch.from_numpy(row)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)
        allr = torch.cat(parts, dim=0).numpy()                       # [world, s + 1]
        rows = fpmash.DeviceBuffer.from_array(ctx, np.ascontiguousarray(allr[:, :s]))
        cnts = fpmash.DeviceBuffer.from_array(ctx, allr[:, s].astype(np.uint32))
        fpmash._check(L.fpm_sketch_merge_dev(ctx.h, rows.ptr, cnts.ptr, world, s, out.ptr,
                                             oc.ptr, None))
    n = int(oc.to_array(np.uint32, 1)[0])        # (ordered after the merge on the stream)
    h = out.to_array(np.uint64, s)[:n]
    out.free()
    oc.free()
    return h, n
