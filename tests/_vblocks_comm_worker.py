"""Worker for test_multirank.test_vblocks_and_comm_one_gpu (-m gpu): the N > 1 paths on one GPU.
  * bench.c4_leg with 2 and 3 virtual blocks: every virtual rank's block-pair jobs
    (fpmash.shard.pair_block_jobs: self jobs on the symmetric path, mirror jobs through
    fpm_refset_dist_mirror_list_dev, the even split's half blocks) on the rows one rank
    sketches locally, no collective; sampled rows of every grid and transpose checked
    against the oracle, and the cells adding up to the whole grid;
  * bench.comm_check: the RCCL min-merge inside libfpmash (fpm_comm_create on a one-rank
    communicator, fpm_sketch_min_merge_comm) against the oracle's sketches;
  * one rank's share of an N = 4 run alone (bench.c4_leg with ws = 4, a one-process group)
    with the oracle check of its grids."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fp-mash_amd")):
    sys.path.insert(0, p)

import bench  # noqa: E402
import fpmash  # noqa: E402


def main():
    grp = bench.Group(1)
    ctx = fpmash.Context(0)
    out = {"c4": {}}
    for vb in (2, 3):
        r = bench.c4_leg(ctx, grp, 1, 0, 0, n=3000, members=100, s=1000, k=21, steps=1,
                         warmup=1, parity="all", vblocks=vb)
        out["c4"][vb] = {"parity": r["parity"], "pairs": r["pairs"], "jobs": r["jobs_rank0"],
                         "cells": r["cells_rank0"], "collective": r["collective"]}
    r = bench.c4_leg(ctx, grp, 4, 3, 0, n=4000, members=100, s=1000, k=21, steps=1, warmup=1,
                     parity="all")
    out["share"] = {"parity": r["parity"], "rows_sketched": r["rows_sketched_rank0"],
                    "rows_owned": r["rows_owned_rank0"], "jobs": r["jobs_rank0"]}
    out["comm"] = bench.comm_check(ctx, grp)
    grp.close()
    print("VBCOMM " + json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
