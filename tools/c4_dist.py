#!/usr/bin/env python3
"""tools/c4_dist.py — SURVEY §8(d)/(e) C4: one all-vs-all dist of N family-structured
sketches, sharded over the GPUs of one node (strong scaling).

    python3 tools/c4_dist.py [--n 50000]                         # 1 GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port P tools/c4_dist.py --n 50000                # 8 GPUs

Per step, per rank: sketch its shard of the sequences (families are split across ranks,
each family generated from its own seed, so the data does not depend on the GPU count),
all-gather the sketch rows (RCCL over xGMI: N x s x 8 B, 400 MB at C4), then the dist of
its query rows against all N references (counts, distance, FP64 p-value, pass flags, left
in HBM).  The all-gather is the job's only exchange.  With one GPU the query rows are the
reference rows, so the library takes its symmetric self-comparison path.  Rank 0 checks two
query rows against the CPU oracle.
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
from fpmash import datagen  # noqa: E402
from fpmash.shard import all_gather_rows, shard_range  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--seq-len", type=int, default=2000)
    ap.add_argument("--members", type=int, default=100)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--s", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))

    fams = a.n // a.members
    n = fams * a.members
    f_lo, f_hi = shard_range(fams, world, rank)
    lo, hi = f_lo * a.members, f_hi * a.members
    seqs = []
    for f in range(f_lo, f_hi):
        seqs += datagen.family_dna(1, a.members, a.seq_len, sub_rate=(0.01, 0.10), seed=1000 + f)
    s, dev = a.s, torch.device(f"cuda:{local}")
    ctx = fpmash.Context(local)
    L = fpmash.lib()
    P = fpmash.make_params(k=a.k, s=s)
    job = ctx.sketch_job(P, seqs)
    d_rows, d_cnt, _ng, _st = job.device_output()
    n_loc = hi - lo
    loc_rows = torch.empty((n_loc, s), dtype=torch.int64, device=dev)
    loc_cnt = torch.empty((n_loc, 1), dtype=torch.int32, device=dev)
    loc_len = torch.tensor([[len(x)] for x in seqs], dtype=torch.int64, device=dev)
    numer = fpmash.DeviceBuffer(ctx, n_loc * n * 4)
    denom = fpmash.DeviceBuffer(ctx, n_loc * n * 4)
    dval = fpmash.DeviceBuffer(ctx, n_loc * n * 8)
    pval = fpmash.DeviceBuffer(ctx, n_loc * n * 8)
    pss = fpmash.DeviceBuffer(ctx, n_loc * n)
    times = {"sketch": 0.0, "gather": 0.0, "dist": 0.0}
    g = {}

    def step(timed):
        t0 = time.perf_counter()
        job.run()
        fpmash._check(L.fpm_memcpy_d2d(ctx.h, loc_rows.data_ptr(), d_rows, n_loc * s * 8))
        fpmash._check(L.fpm_memcpy_d2d(ctx.h, loc_cnt.data_ptr(), d_cnt, n_loc * 4))
        ctx.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            g["rows"] = all_gather_rows(loc_rows, n, world)
            g["cnt"] = all_gather_rows(loc_cnt, n, world)
            g["len"] = all_gather_rows(loc_len, n, world)
            torch.cuda.synchronize()
        else:
            g["rows"], g["cnt"], g["len"] = loc_rows, loc_cnt, loc_len
        t2 = time.perf_counter()
        R, C_, Ln = g["rows"].data_ptr(), g["cnt"].data_ptr(), g["len"].data_ptr()
        fpmash._check(L.fpm_dist_dev(ctx.h, R, C_, Ln, s, n, R + lo * s * 8, C_ + lo * 4,
                                     Ln + lo * 8, s, n_loc, 8, s, a.k, 4.0 ** a.k, 1.0, 1.0,
                                     numer.ptr, denom.ptr, dval.ptr, pval.ptr, pss.ptr, None))
        ctx.synchronize()
        t3 = time.perf_counter()
        if timed:
            times["sketch"] += t1 - t0
            times["gather"] += t2 - t1
            times["dist"] += t3 - t2

    for _ in range(a.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    st = ctx.last_dist_stats()
    check = None
    if rank == 0 and not a.no_check:
        import oracle
        rows = g["rows"].cpu().numpy().view(np.uint64)
        cnt = g["cnt"].cpu().numpy()[:, 0]
        refs = [rows[i, :cnt[i]] for i in range(n)]
        lens = [a.seq_len] * n
        qs = [0, n_loc - 1]
        def row(buf, qi, dtype):                  # one query row of a device result
            out = np.empty(n, dtype)
            fpmash._check(L.fpm_memcpy_d2h(ctx.h, out.ctypes.data,
                                           buf.ptr + qi * n * out.itemsize, out.nbytes))
            return out
        check = True
        for qi in qs:
            nu, de, _di, pv = oracle.dist_grid(refs, lens, [refs[lo + qi]], [lens[lo + qi]], s,
                                               a.k, 4.0 ** a.k)
            check &= bool(np.array_equal(row(numer, qi, np.uint32), nu) and
                          np.array_equal(row(denom, qi, np.uint32), de))
            check &= bool(np.allclose(row(pval, qi, np.float64), pv, rtol=1e-12, atol=0))
    if rank == 0:
        print(json.dumps({
            "config": f"C4: all-vs-all dist of {n} x {a.seq_len} bp family-structured sketches "
                      f"(k={a.k}, s={s}), sketch + all-gather + dist, {world} GPU(s)",
            "n_gpus": world, "pairs": n * n, "ms_per_step": el / a.steps * 1e3,
            "mpairs_per_s": n * n / (el / a.steps) / 1e6,
            "bases_per_s": n * a.seq_len / (el / a.steps),
            "phase_ms_rank0": {k_: v / a.steps * 1e3 for k_, v in times.items()},
            "dist_path": fpmash.DIST_PATHS[int(st["sparse"])],
            "posting_events_rank0": st["events"], "candidates_rank0": st["candidates"],
            "check_rank0": check}))
    job.free()
    for b in (numer, denom, dval, pval, pss):
        b.free()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    if check is False:
        sys.exit(1)


if __name__ == "__main__":
    main()
