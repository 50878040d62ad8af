#!/usr/bin/env python3
"""tools/c4_rank_share.py — one rank's share of bench.py's C4 leg on a single GPU.

    python3 tools/c4_rank_share.py --ws 8 [--rank 0] [--n 50000]

A rank of a ws-GPU C4 run (bench.c4_leg) sketches its contiguous block of families, receives
every rank's sketch rows through the all-gather, and runs its block pairs of the all-vs-all
grid (fpmash.shard.pair_block_jobs): the index of its own block (and, for even ws, one more)
rebuilt, its own block on the symmetric self path, and the other block pairs as a grid + its
transpose (fpm_refset_dist_mirror_list_dev: the compact output, u16 counts + the cells with
numer > 0; --full: the five arrays per cell).  Here the gathered rows come from one sketch job of all
n sequences on device 0, and the rank's own work is timed: its block's sketch job and its
dist share (the same calls c4_leg makes).  The all-gather (N x s x 8 B = 400 MB over xGMI) is
not in the number.  One JSON line.
"""
import argparse
import ctypes as C
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
from fpmash.shard import pair_block_jobs, shard_range  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--full", action="store_true", help="the full five-array output")
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    from bench import compact_out
    members, s, k, seq_len = 100, 1000, 21, 2000
    fams = a.n // members
    n = fams * members
    bounds = [tuple(x * members for x in shard_range(fams, a.ws, r)) for r in range(a.ws)]
    lo, hi = bounds[a.rank]
    seqs = []
    for f in range(fams):
        seqs += datagen.family_dna(1, members, seq_len, sub_rate=(0.01, 0.10), seed=4000 + f)
    ctx = fpmash.Context(0)
    P = fpmash.make_params(k=k, s=s)
    allj = ctx.sketch_job(P, seqs)                 # the gathered reference set
    own = ctx.sketch_job(P, seqs[lo:hi])           # the rank's own block
    R, C_, _ng, stride = allj.device_output()
    L = fpmash.lib()
    st = ctx.stream
    d_len = fpmash.DeviceBuffer.from_array(ctx, np.full(n, seq_len, np.uint64))
    Ln = d_len.ptr
    allj.run(st)
    ctx.synchronize()
    jobs = pair_block_jobs(bounds, a.rank) if a.ws > 1 else [
        {"kind": "self", "ref": (0, n), "qry": (0, n)}]
    outs, refsets = [], {}
    for j in jobs:
        (rl, rh), (ql, qh) = j["ref"], j["qry"]
        cells = (rh - rl) * (qh - ql)
        mk = (lambda c: [fpmash.DeviceBuffer(ctx, c * b) for b in (2, 2, 8, 8, 1)]) if a.full \
            else (lambda c: compact_out(ctx, c))
        o = {"p": mk(cells)}
        if j["kind"] == "mirror":
            o["m"] = mk(cells)
        outs.append(o)
        if (rl, rh) not in refsets:
            h = C.c_void_p()
            fpmash._check(L.fpm_refset_create_dev(ctx.h, R + rl * stride * 8, C_ + rl * 4,
                                                  Ln + rl * 8, stride, rh - rl, 8, s, C.byref(h)))
            refsets[(rl, rh)] = h

    def dist():
        if a.ws == 1:
            p_ = outs[0]["p"]
            if a.full:
                fpmash._check(L.fpm_dist_dev16(ctx.h, R, C_, Ln, stride, n, R, C_, Ln, stride, n,
                                               8, s, k, 4.0 ** k, 1.0, 1.0, *[b.ptr for b in p_],
                                               st))
            else:
                fpmash._check(L.fpm_dist_list_dev(ctx.h, R, C_, Ln, stride, n, R, C_, Ln, stride,
                                                  n, 8, s, k, 4.0 ** k, 1.0, 1.0, p_[0].ptr,
                                                  p_[1].ptr, p_[2].ref, st))
            return
        for rs in refsets.values():
            fpmash._check(L.fpm_refset_reindex(rs, st))
        for j, o in zip(jobs, outs):
            (rl, rh), (ql, qh) = j["ref"], j["qry"]
            q = (R + ql * stride * 8, C_ + ql * 4, Ln + ql * 8, stride, qh - ql)
            rs, p_ = refsets[(rl, rh)], o["p"]
            if a.full and j["kind"] == "self":
                fpmash._check(L.fpm_refset_dist_dev(rs, *q, s, 2, k, 4.0 ** k, 1.0, 1.0,
                                                    *[b.ptr for b in p_], st))
            elif a.full:
                fpmash._check(L.fpm_refset_dist_mirror_dev(rs, *q, s, 2, k, 4.0 ** k, 1.0, 1.0,
                                                           *[b.ptr for b in p_],
                                                           *[b.ptr for b in o["m"]], st))
            elif j["kind"] == "self":
                fpmash._check(L.fpm_refset_dist_list_dev(rs, *q, s, k, 4.0 ** k, 1.0, 1.0,
                                                         p_[0].ptr, p_[1].ptr, p_[2].ref, st))
            else:
                m_ = o["m"]
                fpmash._check(L.fpm_refset_dist_mirror_list_dev(
                    rs, *q, s, k, 4.0 ** k, 1.0, 1.0, p_[0].ptr, p_[1].ptr, p_[2].ref,
                    m_[0].ptr, m_[1].ptr, m_[2].ref, st))

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
    ctx.reset_timing()
    ctx.set_timing(True)
    dist()
    ctx.synchronize()
    ctx.set_timing(False)
    last = ctx.last_dist_stats()       # the step's last dist call (its largest job)
    kern = {}
    for kid, name in fpmash.KERNEL_NAMES.items():
        tot, cnt = ctx.kernel_time(kid)
        if cnt:
            kern[name] = {"total_ms": round(tot, 4), "launches": int(cnt)}
    cells = sum((j["ref"][1] - j["ref"][0]) * (j["qry"][1] - j["qry"][0]) *
                (2 if j["kind"] == "mirror" else 1) for j in jobs)
    print(json.dumps({"emulated_ws": a.ws, "emulated_rank": a.rank, "n": n,
                      "output": "full" if a.full else "compact",
                      "jobs": [{"kind": j["kind"], "ref": list(j["ref"]), "qry": list(j["qry"])}
                               for j in jobs],
                      "cells_written": cells, "last_call_stats": last,
                      "sketch_shard_ms": sk_ms, "dist_ms": di_ms,
                      "rank_step_ms_excl_gather": sk_ms + di_ms, "dist_kernels": kern,
                      "note": "all-gather of the 400 MB sketch rows not included"}))
    for rs in refsets.values():
        L.fpm_refset_free(rs)
    for o in outs:
        for bl in o.values():
            for b in bl:
                b.free()
    d_len.free()
    own.free()
    allj.free()


if __name__ == "__main__":
    main()
