"""Worker for test_multirank.test_c4_gathered_path_nccl_one_gpu (-m gpu): the on-device
multi-GPU data path on one GPU.  A one-rank process group with its RCCL ("nccl") group:
  * bench.c4_leg with virtual blocks: the sketch rows and counts all-gathered by RCCL into
    torch tensors (fpmash.shard.all_gather_rows), the block indexes built over those
    torch-allocated pointers (fpm_refset_create_dev) and every virtual rank's self / mirror
    jobs run on them (fpm_refset_dist_list_dev, fpm_refset_dist_mirror_list_dev); sampled
    rows of every grid and transpose checked against the oracle;
  * fpmash.shard.min_merge with device= (the RCCL gather of bottom-s rows into a torch tensor,
    merged by fpm_sketch_merge_dev from its pointers) against the oracle's sketch."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fp-mash_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import fpmash  # noqa: E402


def main():
    ws, rank, local = bench.dist_env()
    assert ws == 1
    # torch (and its RCCL group) before the library's context (two HIP runtimes)
    grp = bench.Group(ws, local, nccl=True, single_rank_nccl=True)
    assert grp.nccl is not None
    ctx = fpmash.Context(local)
    out = {"c4": {}}
    for vb in (2, 3):
        r = bench.c4_leg(ctx, grp, ws, rank, local, n=3000, members=100, s=1000, k=21, steps=1,
                         warmup=1, parity="all", vblocks=vb)
        out["c4"][vb] = {"parity": r["parity"], "pairs": r["pairs"], "jobs": r["jobs_rank0"],
                         "cells": r["cells_rank0"], "collective": r["collective"]}
    # min_merge on device pointers of a torch tensor gathered by RCCL
    import torch
    from fpmash import datagen
    from fpmash.shard import min_merge
    from oracle import oracle as O
    seq = datagen.family_dna(1, 1, 300_000, seed=77)[0]
    P = fpmash.make_params(k=21, s=2000)
    job = ctx.sketch_job(P, [seq], groups=[0], n_groups=1)
    job.run(ctx.stream)
    ctx.synchronize()
    d_rows, d_cnt, _ng, _st = job.device_output()
    h, n = min_merge(ctx, d_rows, d_cnt, 2000, 1, group=grp.nccl,
                     device=torch.device(f"cuda:{local}"))
    exp = O.sketch_batch(O.params(k=21, s=2000), [seq])[0]
    out["min_merge_ok"] = bool(n == len(exp) and np.array_equal(h, exp))
    job.free()
    print("C4NCCL " + json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
