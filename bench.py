#!/usr/bin/env python3
"""bench.py — fp-mash sketch + dist hot path on MI355X (BASELINE.json metric).

One step = the north-star pipeline on one batch of config C2's shape, with the
input already resident in HBM:
  1. sketch -i, k=21, s=1000 of 10,000 x 2,000 bp synthetic sequences
     (lyn2vec-generate shape; family-structured: 100 families x 100 members,
     1-10 % substitutions, so dist has real shared-hash counts);
  2. all-vs-all dist of those 10,000 sketches (1e8 pairs): shared-hash walk +
     distance + FP64 p-value + -d/-v pass flags, results left in HBM.
value = bases pushed through sketch+dist per second, summed over ranks (each rank
owns an independent batch: weak scaling, no data-path collective).

Per-kernel times come from HIP events recorded by libfpmash on the launch stream;
`roofline` is computed for the kernel with the largest share of the step.
`cpu_baseline` times the oracle's CPU port (oracle/liboracle.so, the reference's
algorithm: per-k-mer heap insert, sequential merge per pair, 4096-pair chunks) on
a bounded sample on rank 0, extrapolated to the same step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
sys.path.insert(0, ROOT)

import fpmash  # noqa: E402
from fpmash import datagen  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_ISSUE_PER_S = 1024 * 2.4e9 / 2   # wave64 VALU instructions/s: 1024 SIMDs, 2 cycles each
# per-launch HBM bytes from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.py,
# regenerated on the GPU box whenever the kernels change)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
METRIC = "bases/s sketched + Mpairs/s dist, k=21 s=1000, 1/2/4/8 MI355X; %HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n-seqs", type=int, default=10000)
    ap.add_argument("--seq-len", type=int, default=2000)
    ap.add_argument("--families", type=int, default=100)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--s", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="target CPU seconds per baseline leg")
    return ap.parse_args()


def parse_args_for_test(**kw):
    """Defaults of parse() with overrides (tests)."""
    a = argparse.Namespace(gpus=1, steps=5, warmup=2, n_seqs=10000, seq_len=2000, families=100,
                           k=21, s=1000, no_cpu_baseline=True, cpu_seconds=8.0)
    for k_, v in kw.items():
        setattr(a, k_, v)
    return a


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


class Group:
    """Barrier + max over ranks.  gloo (host-side) keeps the timing collective off
    the device; the data path itself has no collective (independent batches)."""

    def __init__(self, ws):
        self.ws = ws
        self.pg = None
        if ws > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.ws > 1:
            self.dist.barrier()

    def max(self, x):
        if self.ws == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if self.ws == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())


def make_batch(args, rank):
    fam = max(1, args.families)
    members = max(1, args.n_seqs // fam)
    seqs = datagen.family_dna(fam, members, args.seq_len, sub_rate=(0.01, 0.10),
                              seed=1000 + rank)
    return seqs[: args.n_seqs]


def cpu_baseline(args, seqs):
    """Oracle CPU port on a bounded sample (~cpu_seconds per leg), extrapolated to the
    full step.  Same algorithm structure as the reference: per-k-mer heap insert,
    one sequential merge + p-value per pair, 4096-pair chunks over a worker pool."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, 64))
    P = O.params(k=args.k, s=args.s)
    n = len(seqs)
    # sketch leg: calibrate on a small slice, then time a slice sized to the budget
    n_cal = min(n, 20 * threads)
    t0 = time.perf_counter()
    O.sketch_batch(P, seqs[:n_cal], threads=threads)
    rate0 = n_cal / max(time.perf_counter() - t0, 1e-6)
    n_s = int(min(n, max(n_cal, rate0 * args.cpu_seconds)))
    t0 = time.perf_counter()
    sk = O.sketch_batch(P, seqs[:n_s], threads=threads)
    t_s = time.perf_counter() - t0
    sketch_rate = n_s * args.seq_len / t_s
    # dist leg: a ref-block x query-block of the all-vs-all grid (families included)
    lengths = [args.seq_len] * len(sk)
    n_r = min(len(sk), 1000)
    n_cal = max(1, min(len(sk), 2 * threads))
    t0 = time.perf_counter()
    O.dist_grid(sk[:n_r], lengths[:n_r], sk[:n_cal], lengths[:n_cal], args.s, args.k,
                4.0 ** args.k, threads=threads)
    rate0 = n_r * n_cal / max(time.perf_counter() - t0, 1e-6)
    n_q = int(min(len(sk), max(n_cal, rate0 * args.cpu_seconds / n_r)))
    t0 = time.perf_counter()
    O.dist_grid(sk[:n_r], lengths[:n_r], sk[:n_q], lengths[:n_q], args.s, args.k,
                4.0 ** args.k, threads=threads)
    t_d = time.perf_counter() - t0
    dist_rate = n_r * n_q / t_d
    step_s = n * args.seq_len / sketch_rate + n * n / dist_rate
    return {
        "value": n * args.seq_len / step_s,
        "unit": "bases/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"oracle CPU port on {threads} threads: sketch of {n_s} x {args.seq_len} bp "
                   f"in {t_s:.1f} s ({sketch_rate / 1e6:.2f} Mbases/s) + dist of a {n_r} x {n_q} "
                   f"pair block in {t_d:.1f} s ({dist_rate / 1e6:.3f} Mpairs/s, with p-values), "
                   f"extrapolated to {n} seqs + {n * n:.3g} pairs"),
        "sketch_bases_per_s": sketch_rate,
        "dist_pairs_per_s": dist_rate,
        "step_s_extrapolated": step_s,
        "cpu_model": _cpu_model(),
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def fp_text_leg(ctx, reps=3):
    """C3's -fp input step, reported beside the metric (not part of `value`): parse + hash
    the 1,000,000 CFL k-finger lines `sketch -fp` reads (50 lyn2vec-shaped sequences' CFL
    text, tiled to the line cap: ~30 MB).  Device rate = the parse kernels' HIP-event time;
    the wall rate includes the H2D copy of the text and the D2H of the per-line results."""
    base = datagen.cfl_text(datagen.random_dna(50, 2000, seed=3), datagen.lyn2vec_ids(50))
    text = base * 10
    lines = text.count(b"\n")
    ctx.fp_text(text[:100000])                                     # warm
    ctx.reset_timing()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ctx.fp_text(text, max_lines=1_000_000)
    wall = (time.perf_counter() - t0) / reps
    ctx.set_timing(False)
    tot, _cnt = ctx.kernel_time(fpmash.K_FPTEXT)
    ctx.reset_timing()
    dev = tot / reps * 1e-3
    n = len(r["hash"])
    return {"lines": n, "text_bytes": len(text), "device_ms": dev * 1e3,
            "lines_per_s_device": n / dev, "text_GBps_device": len(text) / dev / 1e9,
            "lines_per_s_wall_pcie": n / wall, "wall_ms": wall * 1e3,
            "note": f"{lines} lines in the file, the first 1,000,000 parsed (the -fp line cap)"}


def main():
    args = parse()
    ws, rank, local = dist_env()
    grp = Group(ws)
    ctx = fpmash.Context(local)
    seqs = make_batch(args, rank)
    n = len(seqs)
    P = fpmash.make_params(k=args.k, s=args.s)

    # ---- stage inputs in HBM (outside the timed region)
    job = ctx.sketch_job(P, seqs)
    info = job.info()
    d_rows, d_cnt, ng, stride = job.device_output()
    L = fpmash.lib()
    n_pairs = n * n
    d_numer = fpmash.DeviceBuffer(ctx, n_pairs * 4)
    d_denom = fpmash.DeviceBuffer(ctx, n_pairs * 4)
    d_dist = fpmash.DeviceBuffer(ctx, n_pairs * 8)
    d_pval = fpmash.DeviceBuffer(ctx, n_pairs * 8)
    d_pass = fpmash.DeviceBuffer(ctx, n_pairs)
    lengths = np.full(n, args.seq_len, dtype=np.uint64)
    d_len = fpmash.DeviceBuffer.from_array(ctx, lengths)
    st = ctx.stream

    def step():
        job.run(st)
        # compare + distance + p-value + pass in one call
        fpmash._check(L.fpm_dist_dev(ctx.h, d_rows, d_cnt, d_len.ptr, stride, n, d_rows, d_cnt,
                                     d_len.ptr, stride, n, 8, args.s, args.k, 4.0 ** args.k,
                                     1.0, 1.0, d_numer.ptr, d_denom.ptr, d_dist.ptr, d_pval.ptr,
                                     d_pass.ptr, st))

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    grp.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    t1 = time.perf_counter()
    grp.barrier()
    elapsed = grp.max(t1 - t0)

    # per-kernel times: HIP events around every launch, in separate steps after the timed
    # region (the event records add markers between launches, so they stay out of it)
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(max(3, min(args.steps, 10))):
        step()
    ctx.synchronize()
    ctx.set_timing(False)
    dstats = ctx.last_dist_stats()
    ktimes = {}
    for kid, name in fpmash.KERNEL_NAMES.items():
        tot, cnt = ctx.kernel_time(kid)
        if cnt:
            ktimes[name] = {"total_ms": tot, "launches": cnt, "avg_ms": tot / cnt}
    ctx.reset_timing()

    # sanity: shared-hash counts present (family structure) and no empty sketches
    cnt_host = np.empty(n, dtype=np.uint32)
    fpmash._check(L.fpm_memcpy_d2h(ctx.h, cnt_host.ctypes.data, d_cnt, n * 4))
    numer_sample = d_numer.to_array(np.uint32, min(n_pairs, 1 << 20))

    bases_rank = n * args.seq_len
    total_bases = grp.sum(bases_rank) * args.steps
    total_pairs = grp.sum(n_pairs) * args.steps
    value = total_bases / elapsed

    # roofline of the dominant kernel (algorithmic bytes per launch / avg launch time)
    s = args.s
    N = fpmash.KERNEL_NAMES
    n_hash = int(cnt_host.sum())
    alg = {
        N[fpmash.K_SKETCH]: (info["seq_bytes"] + n_hash * 8,
                             "packed sequence bytes read + 8 B per output hash"),
        N[fpmash.K_INDEX]: (n_hash * 8,
                            "reference sketch hashes read once (8 B each)"),
        N[fpmash.K_COMPARE]: (2 * n_hash * 8,
                              "ref + query sketches read once (8 B per hash)"),
    }
    if dstats["sparse"]:
        # fused sparse dist: the probe writes every cell's final values, the candidate
        # finalize rewrites the candidate cells (and their mirrors on the symmetric path)
        n_cand = dstats["candidates"]
        cells = 2 * n_cand - n if dstats["sparse"] == 2 else n_cand
        alg[N[fpmash.K_FILL]] = (n_pairs * (4 + 4 + 8 + 8 + 1),
                                 "numer/denom/distance/p-value/pass (25 B/pair) written")
        alg[N[fpmash.K_PROBE]] = (n_hash * 8, "query sketch hashes read")
        alg[N[fpmash.K_FINALIZE]] = (n_cand * (8 + 4 + 4) + cells * (8 + 8 + 1),
                                     "candidate + its numer/denom read, distance/p-value/pass "
                                     "written per candidate cell (mirrors included)")
    else:
        alg[N[fpmash.K_PROBE]] = (n_hash * 8 + n_pairs * 8,
                                  "query sketch hashes read + numer/denom (8 B/pair) written")
        alg[N[fpmash.K_FINALIZE]] = (n_pairs * (4 + 4 + 8 + 8 + 1),
                                     "numer+denom read, distance+p-value+pass written per pair")
    traffic = {}
    if os.path.exists(PMC_TRAFFIC):
        traffic = json.load(open(PMC_TRAFFIC)).get("kernels", {})
    dom = max(ktimes, key=lambda k_: ktimes[k_]["total_ms"])
    achieved = alg[dom][0] / (ktimes[dom]["avg_ms"] * 1e-3) / 1e9 if dom in alg else None
    roof = {
        "kernel": dom,
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS if achieved else None,
        "traffic": traffic.get(dom, {}).get("traffic_bytes"),
        # integer kernels: the issue side beside the byte roofline (MI355X: 1024 SIMDs x
        # 2.4 GHz, one wave64 VALU instruction per 2 cycles per SIMD)
        "valu_issue_frac": (traffic[dom]["sq"]["insts_valu"] /
                            (ktimes[dom]["avg_ms"] * 1e-3 * VALU_ISSUE_PER_S)
                            if dom in traffic and "sq" in traffic[dom] else None),
        "wave_state_frac": traffic.get(dom, {}).get("wave_state_frac"),
        "traffic_source": os.path.relpath(PMC_TRAFFIC, ROOT) if dom in traffic else None,
        "alg_bytes_per_launch": alg.get(dom, (None, ""))[0],
        "alg_bytes_formula": alg.get(dom, (None, ""))[1],
        "avg_launch_ms": ktimes[dom]["avg_ms"],
    }
    per_kernel_roof = {}
    for name, (b, _) in alg.items():
        if name in ktimes:
            gbs = b / (ktimes[name]["avg_ms"] * 1e-3) / 1e9
            per_kernel_roof[name] = {"avg_ms": ktimes[name]["avg_ms"], "alg_GBps": gbs,
                                     "frac_hbm": gbs / HBM_PEAK_GBS,
                                     "traffic_bytes": traffic.get(name, {}).get("traffic_bytes")}

    sk_names = [fpmash.KERNEL_NAMES[k_] for k_ in (fpmash.K_SKETCH, fpmash.K_MERGE)]
    di_names = [fpmash.KERNEL_NAMES[k_] for k_ in (fpmash.K_INDEX, fpmash.K_PROBE,
                                                  fpmash.K_COMPARE, fpmash.K_FINALIZE)]
    sk_ms = sum(ktimes.get(x, {}).get("total_ms", 0.0) for x in sk_names) / args.steps
    di_ms = sum(ktimes.get(x, {}).get("total_ms", 0.0) for x in di_names) / args.steps

    fp_leg = fp_text_leg(ctx) if rank == 0 else None

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, seqs)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "bases/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (family-structured lyn2vec-generate-shaped DNA, seeded per rank)",
            "config": {
                "workload": (f"C2 step: sketch -i k={args.k} s={args.s} of {n} x {args.seq_len} bp "
                             f"+ all-vs-all dist of the {n} sketches ({n_pairs:.3g} pairs, "
                             "numer/denom + distance + FP64 p-value), per GPU"),
                "n_seqs_per_gpu": n, "seq_len": args.seq_len, "k": args.k, "s": args.s,
                "pairs_per_gpu": n_pairs, "parallelism": f"independent batch per GPU x{ws}",
            },
            "sketch": {"bases_per_s": total_bases / args.steps / (sk_ms * 1e-3) if sk_ms else None,
                       "device_ms_per_step": sk_ms, "tiles": info["n_tiles"],
                       "kmers": info["n_kmers"]},
            "dist": {"mpairs_per_s": total_pairs / args.steps / (di_ms * 1e-3) / 1e6 if di_ms else None,
                     "device_ms_per_step": di_ms,
                     "pairs_with_shared_hashes_frac_sample": float((numer_sample > 0).mean()),
                     "path": ["dense walk", "bucket index + literal walk",
                              "bucket index + bucketed rank"][int(dstats["sparse"])],
                     "posting_events": dstats["events"], "candidate_pairs": dstats["candidates"]},
            "fp_text": fp_leg,
            "kernels": ktimes,
            "kernel_roofline": per_kernel_roof,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    job.free()
    ctx.close()


if __name__ == "__main__":
    main()
