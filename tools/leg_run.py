#!/usr/bin/env python3
"""tools/leg_run.py — one side leg of bench.py alone, for profiling it (tools/pmc_traffic.py
--leg): the C3 -fp leg, the C4 all-vs-all leg (one GPU: the symmetric self path over 50k
sketches), or the C5 RefSeq-scale sketch leg, with few steps and no parity check.  Prints the
leg's JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fp-mash_amd")]

import bench  # noqa: E402
import fpmash  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", choices=["c3", "c4", "c5"], required=True)
    ap.add_argument("--c5-genomes", type=int, default=1000)
    ap.add_argument("--k", type=int, default=21, help="C5's k-mer size (21: the config)")
    ap.add_argument("--no-prefill", action="store_true", help="C4 without the counts prefill")
    a = ap.parse_args()
    grp = bench.Group(1)
    with fpmash.Context(0) as ctx:
        if a.leg == "c3":
            r = bench.c3_leg(ctx, reps=2, parity=False)
        elif a.leg == "c4":
            r = bench.c4_leg(ctx, grp, 1, 0, 0, steps=2, warmup=1, parity=False,
                             prefill=not a.no_prefill)
        else:
            r = bench.c5_leg(ctx, grp, 1, 0, n_genomes=a.c5_genomes, k=a.k, steps=3, warmup=1,
                             parity=False)
    print(json.dumps(r, default=str))


if __name__ == "__main__":
    main()
