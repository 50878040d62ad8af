#!/usr/bin/env python3
"""tools/c5_sketch.py — SURVEY §8(d) C5 on one GPU: its share of 1,000 x 5 Mb genomes
(125 at 8 GPUs), k=21, s=10,000, default (per-file, concatenated) mode: one sketch per
genome.  Sequences are staged in HBM once; the timed region is the sketch kernels
(tile hashing + bottom-s, then the merge rounds of each genome's tile lists).  The first
--check genomes are compared with the CPU oracle (bit-exact sketch sets).

    python3 tools/c5_sketch.py [--genomes 125] [--length 5000000] [--check 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import fpmash  # noqa: E402


def genomes(n, length, seed=5):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    return [acgt[rng.integers(0, 4, size=length)].tobytes() for _ in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=125)
    ap.add_argument("--length", type=int, default=5_000_000)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--s", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", type=int, default=2)
    a = ap.parse_args()
    seqs = genomes(a.genomes, a.length)
    with fpmash.Context(0) as ctx:
        P = fpmash.make_params(k=a.k, s=a.s)
        job = ctx.sketch_job(P, seqs, groups=list(range(len(seqs))), n_groups=len(seqs))
        info = job.info()
        job.run()
        ctx.synchronize()
        ctx.reset_timing()
        ctx.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            job.run()
        ctx.synchronize()
        wall = (time.perf_counter() - t0) / a.reps
        ctx.set_timing(False)
        kt = {}
        for kid in (fpmash.K_SKETCH, fpmash.K_MERGE):
            tot, cnt = ctx.kernel_time(kid)
            kt[fpmash.KERNEL_NAMES[kid]] = {"ms_per_run": tot / a.reps, "launches": cnt // a.reps}
        rows, cnt = job.fetch()
        job.free()
    bases = a.genomes * a.length
    out = {"config": f"C5 share: {a.genomes} x {a.length} bp, k={a.k}, s={a.s}, per-genome sketch",
           "bases": bases, "ms": wall * 1e3, "bases_per_s": bases / wall,
           "tiles": info["n_tiles"], "kmers": info["n_kmers"], "kernels": kt}
    if a.check:
        import oracle
        exp = oracle.sketch_batch(oracle.params(k=a.k, s=a.s), seqs[:a.check])
        out["check"] = [bool(np.array_equal(rows[i, :cnt[i]], e)) for i, e in enumerate(exp)]
    print(json.dumps(out))
    if a.check and not all(out["check"]):
        sys.exit(1)


if __name__ == "__main__":
    main()
