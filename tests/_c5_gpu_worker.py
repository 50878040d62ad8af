"""Worker for test_multirank.test_c5_leg_two_ranks_one_gpu (-m gpu): bench.c5_leg, the C5
job (per-file sketches, k=21, s=10,000, files sharded over the ranks as contiguous ranges
balanced by bases, ordered reassembly on rank 0), on two ranks that share the one visible GPU
through libfpmash, with the rows gathered over gloo.  7 genomes of 400 kb split 3 / 4 (or
4 / 3): each genome is ~98 tiles, so the sample pass + group select path of long groups runs.
Rank 0 checks every reassembled genome against the oracle, in file order (Sketch.cpp:346-356:
one sketch per file, emitted in submission order)."""
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
    r = bench.c5_leg(ctx, grp, ws, rank, n_genomes=7, length=400_000, s=10_000, k=21, steps=1,
                     warmup=1, parity="all")
    out = {"rank": rank, "genomes_local": r["rank0"]["genomes"],
           "reassembled": r["reassembled_genomes"], "parity": r.get("parity")}
    print("C5RANK " + json.dumps(out), flush=True)
    grp.barrier()
    ctx.close()


if __name__ == "__main__":
    main()
