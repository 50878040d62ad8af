#!/usr/bin/env python3
"""tools/c4_rank_share.py — one rank's share of bench.py's C4 leg on a single GPU.

    python3 tools/c4_rank_share.py --ws 8 [--rank 0] [--n 50000]

A rank of a ws-GPU C4 run (bench.c4_leg) sketches its contiguous shard of families, receives
every rank's sketch rows through the all-gather, and runs the dist of its query rows against
all n references (index over the references rebuilt inside the step).  Here the gathered
rows come from one sketch job of all n sequences on device 0, and the rank's own work is
timed: its shard's sketch job and its dist call (fpm_dist_dev16, the same call c4_leg makes).
The all-gather (N x s x 8 B = 400 MB over xGMI) is not in the number.  One JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import fpmash  # noqa: E402
from fpmash import datagen  # noqa: E402
from fpmash.shard import shard_range  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    members, s, k, seq_len = 100, 1000, 21, 2000
    fams = a.n // members
    n = fams * members
    f_lo, f_hi = shard_range(fams, a.ws, a.rank)
    lo, n_loc = f_lo * members, (f_hi - f_lo) * members
    seqs = []
    for f in range(fams):
        seqs += datagen.family_dna(1, members, seq_len, sub_rate=(0.01, 0.10), seed=4000 + f)
    ctx = fpmash.Context(0)
    P = fpmash.make_params(k=k, s=s)
    allj = ctx.sketch_job(P, seqs)                 # the gathered reference set
    own = ctx.sketch_job(P, seqs[lo:lo + n_loc])   # the rank's own shard
    R, C_, _ng, stride = allj.device_output()
    L = fpmash.lib()
    st = ctx.stream
    d_len = fpmash.DeviceBuffer.from_array(ctx, np.full(n, seq_len, np.uint64))
    Ln = d_len.ptr
    outs = [fpmash.DeviceBuffer(ctx, n_loc * n * b) for b in (2, 2, 8, 8, 1)]
    allj.run(st)

    def dist():
        fpmash._check(L.fpm_dist_dev16(ctx.h, R, C_, Ln, stride, n, R + lo * stride * 8,
                                     C_ + lo * 4, Ln + lo * 8, stride, n_loc, 8, s, k, 4.0 ** k,
                                     1.0, 1.0, *[o.ptr for o in outs], st))

    def timed(fn):
        for _ in range(2):
            fn()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        ctx.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    sk_ms = timed(lambda: own.run(st))
    di_ms = timed(dist)
    ctx.set_timing(True)
    dist()
    ctx.synchronize()
    ctx.set_timing(False)
    kern = {}
    for kid, name in fpmash.KERNEL_NAMES.items():
        tot, cnt = ctx.kernel_time(kid)
        if cnt:
            kern[name] = round(tot / cnt, 4)
    print(json.dumps({"emulated_ws": a.ws, "emulated_rank": a.rank, "n": n, "query_rows": n_loc,
                      "pairs": n_loc * n, "sketch_shard_ms": sk_ms, "dist_ms": di_ms,
                      "rank_step_ms_excl_gather": sk_ms + di_ms, "dist_kernels_ms": kern,
                      "note": "all-gather of the 400 MB sketch rows not included"}))
    for b in outs:
        b.free()
    d_len.free()
    own.free()
    allj.free()


if __name__ == "__main__":
    main()
