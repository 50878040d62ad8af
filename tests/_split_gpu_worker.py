"""Worker for test_multirank.test_split_leg_two_ranks_one_gpu (-m gpu): bench.split_leg, one
genome sketched in two k-mer ranges by two ranks sharing the one visible GPU, bottom-s rows
all-gathered over gloo and min-merged with fpm_sketch_merge_dev; rank 0 checks the merged
sketch against the whole genome sketched in one piece."""
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
    r = bench.split_leg(ctx, grp, ws, rank, 0, length=6_000_000, s=2000, k=21, steps=1,
                        warmup=1)
    print("SPLITRANK " + json.dumps({"rank": rank, "parity": r.get("parity")}), flush=True)
    grp.barrier()
    ctx.close()


if __name__ == "__main__":
    main()
