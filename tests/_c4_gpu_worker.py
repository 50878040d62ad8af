"""Worker for test_multirank.test_c4_leg_ranks_one_gpu (-m gpu): bench.c4_leg, the C4 job
(sketch the rows its block pairs read -> this rank's block pairs of the all-vs-all
grid, fpmash.shard.pair_block_jobs: own block on the symmetric self path, the other block
pairs as a grid + its transpose through fpm_refset_dist_mirror_dev), on WORLD_SIZE ranks that
share the one visible GPU through libfpmash.  Every rank
checks sampled rows of each of its grids and transposes against the oracle."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fp-mash_amd")):
    sys.path.insert(0, p)

# every rank on device 0: no RCCL communicator (it refuses two ranks per device), min-merges
# over gloo (bench.Group.comm)
os.environ["FPMASH_BENCH_ONE_DEVICE"] = "1"

import bench  # noqa: E402
import fpmash  # noqa: E402


def main():
    ws, rank, _local = bench.dist_env()
    grp = bench.Group(ws)                       # gloo only: both ranks use device 0
    ctx = fpmash.Context(0)
    r = bench.c4_leg(ctx, grp, ws, rank, 0, n=3000, members=100, s=1000, k=21, steps=1,
                     warmup=1, parity="all")
    out = {"rank": rank, "parity": r["parity"], "pairs": r["pairs"], "jobs": r["jobs_rank0"],
           "cells": r["cells_rank0"], "candidates_all_ranks": r["candidates_all_ranks"],
           "path": r["path_rank0"]}
    print("C4RANK " + json.dumps(out), flush=True)
    grp.barrier()
    ctx.close()


if __name__ == "__main__":
    main()
