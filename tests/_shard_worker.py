"""Worker for test_multirank.test_shard_gather_two_ranks (gloo, CPU): each rank sketches
its shard with the oracle, all-gathers the rows, and checks the gathered reference set and
its own dist rows against a single-process computation."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from fpmash import datagen  # noqa: E402
from fpmash.shard import all_gather_rows, shard_range  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    seqs = datagen.family_dna(3, 4, 600, sub_rate=(0.0, 0.05), seed=1) + [b"ACGT" * 40]
    n, s = len(seqs), 200
    lo, hi = shard_range(n, world, rank)
    P = oracle.params(k=15, s=s)
    mine = oracle.sketch_batch(P, seqs[lo:hi])
    rows = np.zeros((hi - lo, s), np.uint64)
    cnt = np.zeros((hi - lo, 1), np.int64)
    for i, h in enumerate(mine):
        rows[i, :len(h)] = h
        cnt[i, 0] = len(h)
    g_rows = all_gather_rows(torch.from_numpy(rows.view(np.int64)), n, world).numpy().view(np.uint64)
    g_cnt = all_gather_rows(torch.from_numpy(cnt), n, world).numpy()[:, 0]
    # the asynchronous form (bench.c4_leg: the own block's job runs while it is in flight)
    # into a preallocated tensor, uneven bounds
    bnd = [shard_range(n, world, r) for r in range(world)]
    out = torch.empty((n, s), dtype=torch.int64)
    fin = all_gather_rows(torch.from_numpy(rows.view(np.int64)), n, world, bounds=bnd, out=out,
                          async_op=True)
    assert callable(fin)
    assert fin() is out and np.array_equal(out.numpy().view(np.uint64), g_rows)
    full = oracle.sketch_batch(P, seqs)
    for i, h in enumerate(full):
        assert g_cnt[i] == len(h) and np.array_equal(g_rows[i, :len(h)], h), (rank, i)
    refs = [g_rows[i, :g_cnt[i]] for i in range(n)]
    lengths = [len(x) for x in seqs]
    nu, de, _, _ = oracle.dist_grid(refs, lengths, refs[lo:hi], lengths[lo:hi], s, 15, 4.0 ** 15)
    fnu, fde, _, _ = oracle.dist_grid(refs, lengths, refs, lengths, s, 15, 4.0 ** 15)
    assert np.array_equal(nu, fnu[lo * n:hi * n]) and np.array_equal(de, fde[lo * n:hi * n])
    dist.barrier()
    if rank == 0:
        print("shard-ok")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
