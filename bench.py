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
    ap.add_argument("--no-fp-text", action="store_true", help="skip the -fp text parse leg")
    ap.add_argument("--no-c3", action="store_true", help="skip the -fp C3 leg")
    ap.add_argument("--no-c4", action="store_true", help="skip the sharded C4 dist leg")
    ap.add_argument("--c4-n", type=int, default=50_000)
    return ap.parse_args()


def parse_args_for_test(**kw):
    """Defaults of parse() with overrides (tests)."""
    a = argparse.Namespace(gpus=1, steps=5, warmup=2, n_seqs=10000, seq_len=2000, families=100,
                           k=21, s=1000, no_cpu_baseline=True, cpu_seconds=8.0,
                           no_fp_text=True, no_c3=True, no_c4=True, c4_n=50_000)
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
    # sketch leg: calibrate on a small slice, then time whole passes over the batch until
    # the leg has run about cpu_seconds / 2
    n_cal = min(n, 20 * threads)
    t0 = time.perf_counter()
    O.sketch_batch(P, seqs[:n_cal], threads=threads)
    rate0 = n_cal / max(time.perf_counter() - t0, 1e-6)
    n_s = int(min(n, max(n_cal, rate0 * args.cpu_seconds / 2)))
    passes = max(1, int(round(rate0 * args.cpu_seconds / 2 / n_s)))
    t0 = time.perf_counter()
    for _ in range(passes):
        sk = O.sketch_batch(P, seqs[:n_s], threads=threads)
    t_s = time.perf_counter() - t0
    sketch_rate = passes * n_s * args.seq_len / t_s
    if n_s < n:
        sk = O.sketch_batch(P, seqs, threads=threads)
    # dist leg: a ref-block x all-queries block of the all-vs-all grid (families included),
    # sized to about cpu_seconds
    lengths = [args.seq_len] * len(sk)
    n_q = len(sk)
    n_cal = max(1, min(len(sk), 2 * threads))
    t0 = time.perf_counter()
    O.dist_grid(sk[:n_cal], lengths[:n_cal], sk, lengths, args.s, args.k,
                4.0 ** args.k, threads=threads)
    rate0 = n_cal * n_q / max(time.perf_counter() - t0, 1e-6)
    n_r = int(min(len(sk), max(n_cal, rate0 * args.cpu_seconds / n_q)))
    t0 = time.perf_counter()
    O.dist_grid(sk[:n_r], lengths[:n_r], sk, lengths, args.s, args.k,
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
                   f"x {passes} pass(es) in {t_s:.1f} s ({sketch_rate / 1e6:.2f} Mbases/s) + dist of a {n_r} x {n_q} "
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


def _group_fp_lines(r, text):
    """initFromFingerprints' grouping (Sketch.cpp:104-134) of one parsed file: a new
    reference wherever the line's ID differs from the previous one; length = the first
    line's value count counted twice + the rest (:117, :134)."""
    n = len(r["hash"])
    new = r["new_id"].astype(bool)
    if n:
        new[0] = True
    starts = np.flatnonzero(new)
    ends = np.append(starts[1:], n)
    nv = r["n_vals"].astype(np.uint64)
    csum = np.concatenate([[0], np.cumsum(nv)])
    lengths = nv[starts] + (csum[ends] - csum[starts])
    return starts, ends, lengths


def c3_leg(ctx, n_seqs=5000, per_file=500, s=1000, reps=3):
    """C3: the -fp path on 5,000 lyn2vec-shaped 2 kb sequences, 1 GPU.
    `sketch -fp` reads at most 1,000,000 lines per call (Sketch.cpp:37, :82), i.e. 500
    sequences of 2,000 CFL k-finger lines, so the 5,000 sequences are 10 files of 500, each
    parsed + hashed on the device (fpm_fp_text_*), grouped into references on the host
    (ID changes), then `dist -fp` of all 5,000 against all 5,000: unsorted u32 lists, the
    reference's literal walk capped at s = 1000 (k = 1, k-mer space 10), on the device.
    Reported beside the metric, not part of `value`."""
    seqs = datagen.random_dna(n_seqs, 2000, seed=33)
    ids = datagen.lyn2vec_ids(n_seqs, seed=33)
    files = [datagen.cfl_text_fast(seqs[i:i + per_file], ids[i:i + per_file])
             for i in range(0, n_seqs, per_file)]
    rows, lens, lengths = [], [], []
    ctx.fp_text(files[0][:100000])                                   # warm
    ctx.reset_timing()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    n_lines = 0
    for f in files:
        r = ctx.fp_text(f, max_lines=1_000_000)
        n_lines += len(r["hash"])
        st, en, ln = _group_fp_lines(r, f)
        h = r["hash"]
        for a, b in zip(st, en):
            rows.append(h[a:b])
        lens.append(en - st)
        lengths.append(ln)
    t_parse_wall = time.perf_counter() - t0
    ctx.set_timing(False)
    parse_ms, _ = ctx.kernel_time(fpmash.K_FPTEXT)
    ctx.reset_timing()
    n = len(rows)
    w = int(max(len(x) for x in rows))
    R = np.zeros((n, w), np.uint32)
    for i, x in enumerate(rows):
        R[i, :len(x)] = x
    rl = np.concatenate(lens).astype(np.uint32)
    rL = np.concatenate(lengths).astype(np.uint64)
    L = fpmash.lib()
    d_R = fpmash.DeviceBuffer.from_array(ctx, R)
    d_rl = fpmash.DeviceBuffer.from_array(ctx, rl)
    d_rL = fpmash.DeviceBuffer.from_array(ctx, rL)
    np_ = n * n
    outs = [fpmash.DeviceBuffer(ctx, np_ * b) for b in (2, 2, 8, 8, 1)]

    def run():
        fpmash._check(L.fpm_dist_dev16(ctx.h, d_R.ptr, d_rl.ptr, d_rL.ptr, w, n, d_R.ptr, d_rl.ptr,
                                     d_rL.ptr, w, n, 4, s, 1, 10.0, 1.0, 1.0,
                                     *[o.ptr for o in outs], ctx.stream))
    run()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    ctx.synchronize()
    dist_ms = (time.perf_counter() - t0) / reps * 1e3
    st = ctx.last_dist_stats()
    numer = outs[0].to_array(np.uint16, np_)
    denom = outs[1].to_array(np.uint16, np_)
    # full-size parity of the index path: the same grid by the dense literal walk of every pair
    same_as_dense = None
    if st["sparse"]:
        ctx.set_dist_mode(fpmash.DIST_DENSE)
        run()
        ctx.synchronize()
        ctx.set_dist_mode(fpmash.DIST_AUTO)
        same_as_dense = bool(np.array_equal(numer, outs[0].to_array(np.uint16, np_)) and
                             np.array_equal(denom, outs[1].to_array(np.uint16, np_)))
    for b in [d_R, d_rl, d_rL] + outs:
        b.free()
    return {"config": f"C3: {n_seqs} x 2000 bp -> CFL k-finger text in {len(files)} files "
                      f"({n_lines} lines, {sum(map(len, files)) / 1e6:.0f} MB), sketch -fp per file "
                      f"+ dist -fp {n} x {n} (s={s}, unsorted u32 walk)",
            "references": n, "lines": n_lines,
            "parse_device_ms": parse_ms, "parse_wall_ms_pcie": t_parse_wall * 1e3,
            "lines_per_s_device": n_lines / (parse_ms * 1e-3),
            "dist_ms": dist_ms, "dist_mpairs_per_s": np_ / (dist_ms * 1e-3) / 1e6,
            "step_device_ms": parse_ms + dist_ms,
            "dist_path": fpmash.DIST_PATHS[int(st["sparse"])],
            "posting_events": st["events"], "candidate_pairs": st["candidates"],
            "pairs_sharing_a_hash": int((numer > 0).sum()),
            "counts_equal_dense_walk": same_as_dense}


def c4_leg(ctx, grp, ws, rank, n=50_000, members=100, s=1000, k=21, steps=3, warmup=1):
    """C4: one all-vs-all dist of n family-structured sketches, the query
    rows sharded over the ranks (strong scaling).  Every GPU holds the whole reference set
    (400 MB at n = 50k: far below one GPU's HBM, so no min-merge / ring exchange is needed,
    as the north star prescribes); each rank sketches it (standing in for loading
    all.msh) outside the timed region, and the timed step is its block of query rows
    against all n references: shared-hash counts, distance, FP64 p-value, pass flags,
    left in HBM.  The index over the references is rebuilt inside every step.  With one
    rank the queries are the references (the library's symmetric self path)."""
    from fpmash.shard import shard_range
    fams = n // members
    n = fams * members
    seqs = datagen.family_dna(fams, members, 2000, sub_rate=(0.01, 0.10), seed=4000)
    P = fpmash.make_params(k=k, s=s)
    job = ctx.sketch_job(P, seqs)
    job.run()
    d_rows, d_cnt, _ng, stride = job.device_output()
    del seqs
    lo, hi = shard_range(n, ws, rank)
    n_loc = hi - lo
    L = fpmash.lib()
    d_len = fpmash.DeviceBuffer.from_array(ctx, np.full(n, 2000, np.uint64))
    outs = [fpmash.DeviceBuffer(ctx, n_loc * n * b) for b in (2, 2, 8, 8, 1)]
    st = ctx.stream

    def run():
        fpmash._check(L.fpm_dist_dev16(ctx.h, d_rows, d_cnt, d_len.ptr, stride, n,
                                     d_rows + lo * stride * 8, d_cnt + lo * 4, d_len.ptr + lo * 8,
                                     stride, n_loc, 8, s, k, 4.0 ** k, 1.0, 1.0,
                                     *[o.ptr for o in outs], st))
    for _ in range(warmup):
        run()
    ctx.synchronize()
    grp.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    ctx.synchronize()
    el = time.perf_counter() - t0
    grp.barrier()
    el = grp.max(el)
    dst = ctx.last_dist_stats()
    cand = grp.sum(dst["candidates"])
    for b in [d_len] + outs:
        b.free()
    job.free()
    return {"config": f"C4: all-vs-all dist of {n} family-structured 2 kb sketches (k={k}, s={s}), "
                      f"query rows sharded over {ws} GPU(s), every GPU holding all references",
            "n_gpus": ws, "pairs": n * n, "steps": steps, "ms_per_step": el / steps * 1e3,
            "mpairs_per_s": n * n / (el / steps) / 1e6, "scaling": "strong",
            "path_rank0": fpmash.DIST_PATHS[int(dst["sparse"])],
            "candidates_all_ranks": cand}


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
    # u16 numer / denom cells (fpm_dist_dev16: counts <= s = 1000)
    d_numer = fpmash.DeviceBuffer(ctx, n_pairs * 2)
    d_denom = fpmash.DeviceBuffer(ctx, n_pairs * 2)
    d_dist = fpmash.DeviceBuffer(ctx, n_pairs * 8)
    d_pval = fpmash.DeviceBuffer(ctx, n_pairs * 8)
    d_pass = fpmash.DeviceBuffer(ctx, n_pairs)
    lengths = np.full(n, args.seq_len, dtype=np.uint64)
    d_len = fpmash.DeviceBuffer.from_array(ctx, lengths)
    st = ctx.stream

    def step():
        job.run(st)
        # compare + distance + p-value + pass in one call
        fpmash._check(L.fpm_dist_dev16(ctx.h, d_rows, d_cnt, d_len.ptr, stride, n, d_rows, d_cnt,
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
    numer_sample = d_numer.to_array(np.uint16, min(n_pairs, 1 << 20))

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
        alg[N[fpmash.K_FILL]] = (n_pairs * (8 + 8 + 1),
                                 "distance/p-value/pass (17 B/pair) written")
        alg[N[fpmash.K_PROBE]] = (n_hash * 8 + n_pairs * (2 + 2),
                                  "query sketch hashes read + u16 numer/denom defaults (4 B/pair) "
                                  "written")
        alg[N[fpmash.K_FINALIZE]] = (n_cand * (8 + 4 + 4) + cells * (2 + 2 + 8 + 8 + 1),
                                     "candidate + its numer/denom read, distance/p-value/pass "
                                     "written per candidate cell (mirrors included)")
    else:
        alg[N[fpmash.K_PROBE]] = (n_hash * 8 + n_pairs * 4,
                                  "query sketch hashes read + u16 numer/denom (4 B/pair) written")
        alg[N[fpmash.K_FINALIZE]] = (n_pairs * (2 + 2 + 8 + 8 + 1),
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

    fp_leg = fp_text_leg(ctx) if rank == 0 and not args.no_fp_text else None
    c3 = c3_leg(ctx, s=args.s) if rank == 0 and not args.no_c3 else None
    c4 = None
    if not args.no_c4:
        job.free()                       # the C2 batch's buffers make room for C4's grid
        for b in (d_numer, d_denom, d_dist, d_pval, d_pass):
            b.free()
        c4 = c4_leg(ctx, grp, ws, rank, n=args.c4_n, s=args.s, k=args.k)

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
                             "u16 numer/denom + distance + FP64 p-value + pass), per GPU"),
                "n_seqs_per_gpu": n, "seq_len": args.seq_len, "k": args.k, "s": args.s,
                "pairs_per_gpu": n_pairs, "parallelism": f"independent batch per GPU x{ws}",
            },
            "sketch": {"bases_per_s": total_bases / args.steps / (sk_ms * 1e-3) if sk_ms else None,
                       "device_ms_per_step": sk_ms, "tiles": info["n_tiles"],
                       "kmers": info["n_kmers"]},
            "dist": {"mpairs_per_s": total_pairs / args.steps / (di_ms * 1e-3) / 1e6 if di_ms else None,
                     "device_ms_per_step": di_ms,
                     "pairs_with_shared_hashes_frac_sample": float((numer_sample > 0).mean()),
                     "path": fpmash.DIST_PATHS[int(dstats["sparse"])],
                     "posting_events": dstats["events"], "candidate_pairs": dstats["candidates"]},
            "fp_text": fp_leg,
            "c3_fp": c3,
            "c4_dist": c4,
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
