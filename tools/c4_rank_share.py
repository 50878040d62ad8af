#!/usr/bin/env python3
"""tools/c4_rank_share.py — one rank's share of bench.py's C4 leg on a single GPU.

    python3 tools/c4_rank_share.py --ws 8 [--rank 0] [--n 50000]

Runs exactly the work rank `rank` of a `ws`-GPU C4 run does (its block of query rows against
all n references, index rebuilt each step) on device 0, so the 8-GPU per-rank step time can be
measured on a one-GPU box.  Prints one JSON line with the per-kernel split.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import fpmash  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    ctx = fpmash.Context(0)
    ctx.set_timing(True)
    r = bench.c4_leg(ctx, bench.Group(1), a.ws, a.rank, n=a.n, steps=a.steps)
    ctx.set_timing(False)
    k = {}
    for kid, name in fpmash.KERNEL_NAMES.items():
        tot, cnt = ctx.kernel_time(kid)
        if cnt:
            k[name] = {"avg_ms": tot / cnt, "launches": cnt}
    r.update({"emulated_rank": a.rank, "emulated_ws": a.ws, "kernels_incl_setup": k,
              "note": "timing events on: includes the sketch launch of the setup"})
    print(json.dumps(r))
    ctx.close()


if __name__ == "__main__":
    main()
