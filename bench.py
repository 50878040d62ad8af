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
# per-launch HBM bytes and SQ counters from rocprofv3 PMC passes (tools/pmc_traffic.py, run on
# the GPU box into gpurun_out/TAG/ and copied into profiles/rNN/ here by tools/collect.py).
# Every file carries the build id of the libfpmash.so it measured; counters of another build
# are not attached to this run's kernel times (roofline.traffic etc. null, with a note).
def pmc_dir(arg=None):
    """--pmc-dir, else the newest profiles/rNN that holds a pmc_traffic.json"""
    import glob
    if arg:
        return arg if os.path.isabs(arg) else os.path.join(ROOT, arg)
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "pmc_traffic.json")))
    return os.path.dirname(found[-1]) if found else None


def load_pmc(name, directory):
    """(counters dict, note): the PMC file `name` of `directory` when it measured the build
    loaded now, else (None, why not)."""
    path = os.path.join(directory, name) if directory else None
    if not path or not os.path.exists(path):
        return None, f"no {name}"
    d = json.load(open(path))
    rel = os.path.relpath(path, ROOT)
    have, want = d.get("build_id"), fpmash.build_id()
    if have is None or have != want:
        return None, (f"{rel} measured build {have}, this run loads build {want}: "
                      "counters of another build are not attached")
    d["source"] = rel
    return d, None


def leg_counters(leg, directory=None):
    """A side leg's per-kernel counters (tools/pmc_traffic.py --leg, pmc_<leg>.json of the PMC
    directory, measured on the GPU box on this same build): average launch time, HBM traffic
    rate against the 8 TB/s peak, VALU-issue fraction, wave-state split, L2 hit rate and LDS
    bank-conflict cycles, and the bound those numbers point to (the leg's bound claims are
    read from here, not asserted).  {"note": ...} when there is no profile of this build."""
    d, note = load_pmc(f"pmc_{leg}.json", directory)
    if d is None:
        return {"note": note}
    ks = {}
    for k, v in d.get("kernels", {}).items():
        if not v.get("avg_ns"):
            continue
        hbm = (v.get("traffic_GBps") or 0.0) / HBM_PEAK_GBS
        valu = v.get("valu_issue_frac") or 0.0
        ws_ = v.get("wave_state_frac") or {}
        if max(hbm, valu) >= 0.5:
            bound = "hbm" if hbm >= valu else "valu-issue"
        else:
            bound = "latency (waves waiting %.0f %%, issue-stalled %.0f %%)" % (
                100 * ws_.get("waiting", 0.0), 100 * ws_.get("issue_stall", 0.0))
        ks[k] = {"avg_ms": v["avg_ns"] * 1e-6, "calls": v.get("calls"),
                 "traffic_bytes": v.get("traffic_bytes"), "frac_hbm": hbm,
                 "valu_issue_frac": valu, "wave_state_frac": ws_,
                 "l2_hit_frac": (v.get("l2") or {}).get("hit_frac"),
                 "lds_bank_conflict_cycles": (v.get("l2") or {}).get("lds_bank_conflict_cycles"),
                 "bound_by_counters": bound}
    return {"source": d["source"], "build_id": d.get("build_id"), "command": d.get("command"),
            "kernels": dict(sorted(ks.items(), key=lambda kv: -kv[1]["avg_ms"] *
                                   (kv[1]["calls"] or 1)))}
METRIC = "bases/s sketched + Mpairs/s dist, k=21 s=1000, 1/2/4/8 MI355X; %HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a C2 step is ~1.4 ms: 20 timed steps after 5 warmup steps cost ~35 ms and steady the
    # line (5 steps read 2-5 % high: clocks still ramping)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
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
    ap.add_argument("--no-cli-fp", action="store_true",
                    help="skip the -fp CLI leg (sketch -fp x10, paste -fp, dist -fp)")
    ap.add_argument("--no-gather-check", "--no-vblocks-check", dest="no_gather_check",
                    action="store_true",
                    help="at N = 1: skip the checks of the N > 1 paths on this GPU (C4 with "
                         "three virtual blocks; the RCCL min-merge on a one-rank communicator)")
    ap.add_argument("--no-c4-shares", action="store_true",
                    help="at N = 1: skip timing rank shares of N = 2/4/8 C4 runs on this GPU")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 RefSeq-scale sketch leg")
    ap.add_argument("--no-cli", action="store_true",
                    help="skip the end-to-end CLI leg (fpmash sketch + dist, 1e8 text lines)")
    ap.add_argument("--c5-genomes", type=int, default=1000)
    ap.add_argument("--no-split", action="store_true",
                    help="skip the one-genome-over-all-GPUs sketch leg (RCCL min-merge)")
    ap.add_argument("--split-bases", type=int, default=1_000_000_000)
    ap.add_argument("--no-full-grid", action="store_true",
                    help="skip the comparison run of the C2 step with the full five-array dist "
                         "output (fpm_dist_dev16)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle checks of the C2 / C3 / C4 results")
    ap.add_argument("--pmc-dir", default=None,
                    help="directory of the pmc_*.json counter files to attach (default: the "
                         "newest profiles/rNN holding one); used only when they carry the "
                         "loaded library's build id")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="side file for the full result (per-kernel tables, leg counters, CLI "
                         "phases); '' = none.  The printed line keeps the headline numbers")
    return ap.parse_args()


def parse_args_for_test(**kw):
    """Defaults of parse() with overrides (tests)."""
    a = argparse.Namespace(gpus=1, steps=5, warmup=2, n_seqs=10000, seq_len=2000, families=100,
                           k=21, s=1000, no_cpu_baseline=True, cpu_seconds=8.0,
                           no_fp_text=True, no_c3=True, no_c4=True, c4_n=50_000,
                           no_parity=True, no_c5=True, c5_genomes=1000, no_cli=True,
                           no_split=True, split_bases=1_000_000_000, detail="",
                           no_full_grid=True, pmc_dir=None, no_c4_shares=True)
    for k_, v in kw.items():
        setattr(a, k_, v)
    return a


def timing_steps(steps):
    """Steps run with per-launch HIP events after the timed region (the event records add
    marker packets between launches, so they stay out of the timed steps)."""
    return max(3, min(steps, 10))


def per_step_ms(ktimes, names, n_timed):
    """Device milliseconds per step of the named kernels: their event totals over the
    n_timed event-timed steps (not over --steps: those ran without events)."""
    return sum(ktimes.get(x, {}).get("total_ms", 0.0) for x in names) / n_timed


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("FPMASH_BENCH_ONE_DEVICE"):
        # rehearsal of the N-rank flow on a one-GPU box (tools/rehearse_ranks.sh): every rank
        # on device 0, gathers over gloo (RCCL refuses two ranks on one GPU)
        local = 0
    return ws, rank, local


class Group:
    """Barrier + max / sum over ranks on a host-side gloo group (the timing collectives stay off
    the device; the C2 / C4 / C5 data paths have no collective).  comm(ctx) builds the one
    device communicator the path has: RCCL inside libfpmash (fpmash.Comm) for the split
    genome's min-merge, its unique id broadcast over gloo."""

    def __init__(self, ws):
        self.ws = ws
        self.dist = None
        self._comm = None
        self.comm_error = None     # why the ranks have no communicator (then: gloo)
        if ws > 1:
            import datetime
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
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

    def comm(self, ctx):
        """fpmash.Comm over all ranks on ctx's device (created once; every rank waits for the
        others, up to FPM_COMM_INIT_TIMEOUT_S).  None when the ranks share one GPU
        (FPMASH_BENCH_ONE_DEVICE: RCCL refuses two ranks per device), or when a rank's set-up
        failed (every rank learns it over gloo; `comm_error` says why): min-merges then go
        over gloo, and the leg says so."""
        if (self._comm is None and self.comm_error is None
                and not os.environ.get("FPMASH_BENCH_ONE_DEVICE")):
            rank = 0
            if self.ws > 1:
                import torch
                rank = self.dist.get_rank()
                uid = torch.zeros(fpmash.COMM_ID_BYTES, dtype=torch.uint8)
                if rank == 0:
                    uid[:] = torch.frombuffer(bytearray(fpmash.comm_unique_id()), dtype=torch.uint8)
                self.dist.broadcast(uid, 0)
                uid = bytes(uid.numpy().tobytes())
            else:
                uid = fpmash.comm_unique_id()
            try:
                c, err = fpmash.Comm(ctx, self.ws, rank, uid), None
            except Exception as e:                       # noqa: BLE001 (reported in the leg)
                c, err = None, f"rank {rank}: {e}"
            if self.max(0.0 if c is not None else 1.0) > 0.0:
                # some rank has none: no rank uses its (a set-up whose peers are gone is left
                # to the process exit)
                self.comm_error = err or "a peer rank's RCCL set-up failed"
                print(f"[bench] RCCL communicator unavailable ({self.comm_error}); "
                      "min-merges over gloo", file=sys.stderr, flush=True)
                return None
            self._comm = c
        return self._comm

    def close(self):
        if self._comm is not None:
            self._comm.close()
            self._comm = None


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
    # the reference's own getHash + MinHashHeap (oracle/_ref, compiled from its sources: the
    # k-mer walk re-driven around them) on the same threads, for a sample of records; its
    # rate replaces the port's in the step when it is available
    ref_rate = None
    t0 = time.perf_counter()
    n_ref = min(n, max(4 * threads, int(sketch_rate * args.cpu_seconds / 4 / args.seq_len)))
    rsk = O.ref_sketch_batch(seqs[:n_ref], k=args.k, s=args.s, threads=threads)
    if rsk is not None:
        t_r = time.perf_counter() - t0
        ref_rate = n_ref * args.seq_len / t_r
        ref_same = all(np.array_equal(a, b) for a, b in zip(rsk, sk[:n_ref]))
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
    step_s = n * args.seq_len / (ref_rate or sketch_rate) + n * n / dist_rate
    extra = {}
    if ref_rate:
        extra = {"sketch_kind": "reference: oracle/_ref (hash.cpp, MurmurHash3.cpp, "
                                "MinHashHeap.cpp, HashSet.cpp ... compiled from the reference's "
                                "sources) around a restated addMinHashes walk",
                 "sketch_reference_bases_per_s": ref_rate,
                 "sketch_reference_records": n_ref,
                 "sketch_reference_equals_port": bool(ref_same)}
    return {
        "value": n * args.seq_len / step_s,
        "unit": "bases/s",
        "cores": threads,
        "cores_note": (f"threads used = the CPUs available to this process ({threads}: "
                       f"OMP_NUM_THREADS / sched_getaffinity) of the machine's "
                       f"{os.cpu_count()}"),
        "kind": "port",
        **extra,
        "sample": (f"oracle CPU port on {threads} threads: sketch of {n_s} x {args.seq_len} bp "
                   f"x {passes} pass(es) in {t_s:.1f} s ({sketch_rate / 1e6:.2f} Mbases/s) + dist of a {n_r} x {n_q} "
                   f"pair block in {t_d:.1f} s ({dist_rate / 1e6:.3f} Mpairs/s, with p-values), "
                   f"extrapolated to {n} seqs + {n * n:.3g} pairs"
                   + (f"; the step uses the sketch rate of the reference's own getHash + "
                      f"MinHashHeap (oracle/_ref) on {n_ref} records, {ref_rate / 1e6:.2f} "
                      "Mbases/s" if ref_rate else "")),
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


def fp_text_leg(ctx, reps=5):
    """C3's -fp input step, reported beside the metric (not part of `value`): parse + hash
    the 1,000,000 CFL k-finger lines `sketch -fp` reads (50 lyn2vec-shaped sequences' CFL
    text, tiled to the line cap: ~30 MB).  Device rate = the parse kernels' HIP-event time;
    the wall rate includes the H2D copy of the text and the D2H of the per-line results."""
    base = datagen.cfl_text(datagen.random_dna(50, 2000, seed=3), datagen.lyn2vec_ids(50))
    text = base * 10
    lines = text.count(b"\n")
    for warm in (text[:100000], text):                             # warm (pinned ring too)
        ctx.fp_text(warm, max_lines=1_000_000)
    # per call: the HIP-event total of its launches; the mean over the calls is reported, with
    # the list.  (Round 2 saw one call in five take 21-34 ms: the runtime page-locked the
    # pageable result arrays for the fetch, and releasing them made the driver evict and restore
    # the process's GPU queues -- a GPU-wide 12-30 ms stall, tools/micro/fp_clock.hip,
    # profiles/r03/fp_stall/.  Caller memory now goes through the context's pinned ring.)
    devs, walls = [], []
    for _ in range(reps):
        ctx.reset_timing()
        ctx.set_timing(True)
        t0 = time.perf_counter()
        r = ctx.fp_text(text, max_lines=1_000_000)
        walls.append(time.perf_counter() - t0)
        ctx.set_timing(False)
        tot, _cnt = ctx.kernel_time(fpmash.K_FPTEXT)
        devs.append(tot * 1e-3)
    ctx.reset_timing()
    dev = float(np.mean(devs))
    wall = float(np.mean(walls))
    n = len(r["hash"])
    return {"lines": n, "text_bytes": len(text), "device_ms": dev * 1e3,
            "device_ms_calls": [round(d * 1e3, 4) for d in devs],
            "device_ms_max": max(devs) * 1e3,
            "lines_per_s_device": n / dev, "text_GBps_device": len(text) / dev / 1e9,
            "lines_per_s_wall_pcie": n / wall, "wall_ms": wall * 1e3,
            "note": f"{lines} lines in the file, the first 1,000,000 parsed (the -fp line cap); "
                    f"mean of {reps} calls"}


# ---- parity (the CPU leg's checker: oracle/ restatement, outside every timed region) ----

def _threads():
    t = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    return max(1, min(t, 64))


def fetch_rows(buf, dtype, n_cols, rows):
    """rows [r] of a device matrix [.][n_cols] (query-major dist outputs) -> host [len(rows), n_cols]"""
    isz = np.dtype(dtype).itemsize
    out = np.empty((len(rows), n_cols), dtype=dtype)
    L = fpmash.lib()
    for i, r in enumerate(rows):
        fpmash._check(L.fpm_memcpy_d2h(buf.ctx.h, out[i].ctypes.data,
                                       buf.ptr + int(r) * n_cols * isz, n_cols * isz))
    return out


def sample_rows(n, m, salt=0):
    """m query rows spread over [0, n) (every family of the family-structured batches)"""
    m = min(m, n)
    rng = np.random.default_rng(12345 + salt)
    return np.sort(rng.choice(n, size=m, replace=False)) if m else np.zeros(0, np.int64)


def expanded_rows(outs, n_ref, rows, max_dist=1.0, max_pvalue=1.0):
    """rows [r] of a device dist grid as the five per-cell arrays [len(rows), n_ref]: either
    five device buffers (numer u16, denom u16, distance, p-value, pass: the full output) or
    the compact output (numer u16, denom u16, fpmash.CellList), expanded by
    fpmash.expand_compact's rule for the cells not listed"""
    nu = fetch_rows(outs[0], np.uint16, n_ref, rows)
    de = fetch_rows(outs[1], np.uint16, n_ref, rows)
    if len(outs) == 5:
        return (nu, de, fetch_rows(outs[2], np.float64, n_ref, rows),
                fetch_rows(outs[3], np.float64, n_ref, rows),
                fetch_rows(outs[4], np.uint8, n_ref, rows))
    listed = outs[2].fetch()
    pos = np.full(int(max(rows)) + 1 if len(rows) else 1, -1, np.int64)
    pos[np.asarray(rows, np.int64)] = np.arange(len(rows))
    q = listed["qry"].astype(np.int64)
    keep = q < len(pos)
    keep[keep] = pos[q[keep]] >= 0
    sub = {k: v[keep] for k, v in listed.items()}
    sub["qry"] = pos[q[keep]].astype(np.uint32)
    e = fpmash.expand_compact(nu.reshape(-1), de.reshape(-1), sub, n_ref, max_dist, max_pvalue)
    shp = (len(rows), n_ref)
    return (nu, de, e["distance"].reshape(shp), e["pvalue"].reshape(shp),
            e["pass"].reshape(shp).astype(np.uint8))


def check_grid_rows(outs, n_ref, rows, exp, max_dist=1.0, max_pvalue=1.0):
    """device rows (full or compact output, expanded_rows) vs the oracle's grid of the same
    query rows: counts and pass flags exact, distance and p-value within rtol 1e-12 (the
    north-star tolerance)"""
    nu_o, de_o, di_o, pv_o = (x.reshape(len(rows), n_ref) for x in exp)
    nu, de, di, pv, pa = expanded_rows(outs, n_ref, rows, max_dist, max_pvalue)
    exp_pass = (di_o <= max_dist) & (pv_o <= max_pvalue)
    counts_ok = bool(np.array_equal(nu, nu_o) and np.array_equal(de, de_o))
    dist_ok = bool(np.allclose(di, di_o, rtol=1e-12, atol=0))
    pv_ok = bool(np.allclose(pv, pv_o, rtol=1e-12, atol=0))
    pass_ok = bool(np.array_equal(pa.astype(bool), exp_pass))
    return {"rows": len(rows), "pairs": int(len(rows) * n_ref),
            "pairs_sharing": int((nu_o > 0).sum()),
            "counts_exact": counts_ok, "distance_rtol_1e-12": dist_ok,
            "pvalue_rtol_1e-12": pv_ok, "pass_exact": pass_ok,
            "max_pvalue_rel_err": float(np.max(np.abs(pv - pv_o) / np.maximum(np.abs(pv_o), 1e-300)))
            if pv.size else 0.0,
            "ok": counts_ok and dist_ok and pv_ok and pass_ok}


def parity_summary(c2, c3, c4, c5=None, cli=None, split=None, c4_gather=None, cli_fp=None,
                   comm=None):
    """the line's `parity` object: every oracle check of this run and whether all passed"""
    parts = {"c2": c2, "c3_fp": c3.get("parity") if c3 else None,
             "c4": c4.get("parity") if c4 else None,
             "c4_vblocks": c4_gather.get("parity") if c4_gather else None,
             "comm_min_merge": comm,
             "c5": c5.get("parity") if c5 else None,
             "split": split.get("parity") if split else None,
             "cli": cli.get("parity") if cli else None,
             "cli_fp": cli_fp.get("parity") if cli_fp else None}
    done = [v["ok"] for v in parts.values() if v]
    parts["all_ok"] = all(done) if done else None
    parts["checker"] = ("oracle/ CPU restatement (pinned to the reference's fixtures), "
                        "outside the timed regions")
    return parts


def c2_parity(job, seqs, outs, args, n_rows=200):
    """C2 at full size: all sketches of the batch vs the oracle's CPU port (bit-exact rows
    and counts), and a 200-query-row x all-refs block of the all-vs-all dist."""
    from oracle import oracle as O
    t0 = time.perf_counter()
    th = _threads()
    rows_d, cnt_d = job.fetch()
    exp = O.sketch_batch(O.params(k=args.k, s=args.s), seqs, threads=th)
    sk_ok = all(int(cnt_d[i]) == len(e) and np.array_equal(rows_d[i, :len(e)], e)
                for i, e in enumerate(exp))
    n = len(seqs)
    rows = sample_rows(n, n_rows)
    lengths = [args.seq_len] * n
    g = O.dist_grid(exp, lengths, [exp[int(r)] for r in rows], [lengths[int(r)] for r in rows],
                    args.s, args.k, 4.0 ** args.k, threads=th)
    d = check_grid_rows(outs, n, rows, g)
    return {"sketches": n, "sketch_rows_exact": bool(sk_ok), "dist": d,
            "ok": bool(sk_ok) and d["ok"], "check_s": time.perf_counter() - t0}


def c3_leg(ctx, n_seqs=5000, per_file=500, s=1000, reps=3, parity=True):
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
        # parsed, hashed and grouped into References on the device (fpm_fp_text_refs): the
        # host fetches the line hashes and ~500 reference descriptors per file
        r = ctx.fp_refs(f, max_lines=1_000_000)
        n_lines += r["n_lines"]
        h = r["hash"]
        st = r["first"].astype(np.int64)
        en = np.append(st[1:], r["n_lines"])
        for a, b in zip(st, en):
            rows.append(h[a:b])
        lens.append(en - st)
        lengths.append(r["length"])
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
    # the compact output: u16 counts of every pair + the pairs with numer > 0
    outs = compact_out(ctx, np_)

    def run():
        fpmash._check(L.fpm_dist_list_dev(ctx.h, d_R.ptr, d_rl.ptr, d_rL.ptr, w, n, d_R.ptr,
                                          d_rl.ptr, d_rL.ptr, w, n, 4, s, 1, 10.0, 1.0, 1.0,
                                          outs[0].ptr, outs[1].ptr, outs[2].ref, ctx.stream))
    run()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    ctx.synchronize()
    dist_ms = (time.perf_counter() - t0) / reps * 1e3
    if outs[2].count() > outs[2].cap:
        raise RuntimeError(f"C3 cell list overflow: {outs[2].count()} > {outs[2].cap}")
    st = ctx.last_dist_stats()
    numer = outs[0].to_array(np.uint16, np_)
    denom = outs[1].to_array(np.uint16, np_)
    # full-size parity of the index path: the same grid by the dense literal walk of every pair
    same_as_dense = None
    dense_ms = None
    if st["sparse"]:
        ctx.set_dist_mode(fpmash.DIST_DENSE)
        run()
        ctx.synchronize()
        t0 = time.perf_counter()
        run()           # timed once beside the index path: the dense image walk of every pair
        ctx.synchronize()
        dense_ms = (time.perf_counter() - t0) * 1e3
        ctx.set_dist_mode(fpmash.DIST_AUTO)
        same_as_dense = bool(np.array_equal(numer, outs[0].to_array(np.uint16, np_)) and
                             np.array_equal(denom, outs[1].to_array(np.uint16, np_)))
    par = None
    if parity:
        # the CPU leg's checker: 200 query rows x all 5,000 references by the oracle's
        # literal walk, `.txt` mode (whole lists, walk capped at s) and `.msh` mode (lists
        # truncated to s as loadCapnp does, Sketch.cpp:1117-1120)
        from oracle import oracle as O
        t0 = time.perf_counter()
        th = _threads()
        qrows = sample_rows(n, 200, salt=3)
        par = {}
        for mode, cut in (("txt", None), ("msh", s)):
            lists = [x if cut is None else x[:cut] for x in rows]
            if cut is not None:
                d_rl2 = fpmash.DeviceBuffer.from_array(ctx, np.minimum(rl, cut).astype(np.uint32))
                fpmash._check(L.fpm_dist_list_dev(ctx.h, d_R.ptr, d_rl2.ptr, d_rL.ptr, w, n,
                                                  d_R.ptr, d_rl2.ptr, d_rL.ptr, w, n, 4, s, 1,
                                                  10.0, 1.0, 1.0, outs[0].ptr, outs[1].ptr,
                                                  outs[2].ref, ctx.stream))
                ctx.synchronize()
                d_rl2.free()
            g = O.dist_grid(lists, list(rL), [lists[int(q)] for q in qrows],
                            [rL[int(q)] for q in qrows], s, 1, 10.0, use64=False, threads=th)
            par[mode] = check_grid_rows(outs, n, qrows, g)
        par["ok"] = par["txt"]["ok"] and par["msh"]["ok"]
        par["check_s"] = time.perf_counter() - t0
    for b in [d_R, d_rl, d_rL] + outs:
        b.free()
    return {"output": "u16 numer/denom per pair + listed pairs with numer > 0 (SURVEY 8(d))",
            "config": f"C3: {n_seqs} x 2000 bp -> CFL k-finger text in {len(files)} files "
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
            "counts_equal_dense_walk": same_as_dense, "dense_walk_ms": dense_ms,
            "parity": par}


def compact_out(ctx, cells):
    """device buffers of one grid's compact dist output: u16 numer, u16 denom and the list of
    the cells with numer > 0 (room for 1/16 of the cells, 2^20 to 2^26 entries: the
    family-structured C2 / C4 grids share hashes in 1 % / 0.2 % of their pairs, C3's k-finger
    lists in ~4 %; an overflow is detected and raised after the run)"""
    return [fpmash.DeviceBuffer(ctx, cells * 2), fpmash.DeviceBuffer(ctx, cells * 2),
            fpmash.CellList(ctx, min(cells, max(1 << 20, min(1 << 26, cells // 16))))]


def c4_rows(lo, hi, members=100, seq_len=2000):
    """Rows [lo, hi) of the C4 set: family f (members consecutive rows) generated from its own
    seed, so any rank builds any range of rows without the rest of the set."""
    out = []
    for f in range(lo // members, (hi + members - 1) // members):
        fam = datagen.family_dna(1, members, seq_len, sub_rate=(0.01, 0.10), seed=4000 + f)
        out += fam[max(lo, f * members) - f * members: min(hi, (f + 1) * members) - f * members]
    return out


def merge_spans(ranges):
    """the union of [lo, hi) ranges as sorted disjoint spans"""
    out = []
    for lo, hi in sorted(r for r in ranges if r[1] > r[0]):
        if out and lo <= out[-1][1]:
            out[-1][1] = max(out[-1][1], hi)
        else:
            out.append([lo, hi])
    return [tuple(x) for x in out]


def c4_leg(ctx, grp, ws, rank, local, n=50_000, members=100, s=1000, k=21, seq_len=2000,
           steps=3, warmup=1, parity=True, vblocks=1, cpu=False, prefill=True):
    """C4: one all-vs-all dist of n family-structured sketches, sharded over
    the ranks (strong scaling), with NO data-path collective: north_star keeps RCCL for "the
    final min-merge only where the reference set exceeds one GPU's HBM", and C4's 400 MB set
    fits every GPU many times over.  The reference runs the grid on one pthreads pool
    (CommandDistance.cpp:224-261); here the grid is dealt as unordered block pairs
    (fpmash.shard.pair_block_jobs): every unordered pair of blocks is compared on one rank and
    written twice (grid + transpose: sorted sketches give symmetric results), so a rank
    compares ~n^2 / 2N pairs and writes ~n^2 / N cells.  A timed step on every rank:
      1. sketch the rows its jobs read -- its own block and the (N - 1) / 2 blocks (+ half a
         block for even N) it is paired with, ~(N + 1) / 2N of the set -- from the inputs
         every rank holds (each family generated from its own seed: the same data at any N);
      2. its block pairs on those local rows: the own block on the library's symmetric self
         path, the others through fpm_refset_dist_mirror_list_dev; the indexes are rebuilt
         inside the step; output left in HBM in the compact form of SURVEY §8(b)/(d) (u16
         numer / denom of every cell + distance / FP64 p-value / pass of the cells with
         numer > 0).
    With one rank the whole grid is one fpm_dist_list_dev call on the symmetric self path,
    with the no-shared-hash counts prefilled beside the sketch (fpm_dist_list_prefill).
    One rank's share of an N-rank run is measured alone on one GPU by passing ws = N, rank =
    r with a one-process group (bench `c4_shares`): the rank needs nothing from the others.
    vblocks > 1 (one rank): every virtual rank's jobs of a vblocks-way split run in this
    process (the N > 1 job structure checked on one GPU: every cell written once)."""
    import ctypes as C
    from fpmash.shard import pair_block_jobs, shard_range
    fams = n // members
    n = fams * members
    bounds = [tuple(x * members for x in shard_range(fams, ws, r)) for r in range(ws)]
    if vblocks > 1:
        if ws != 1:
            raise ValueError("vblocks > 1 stands in for more ranks on one rank only")
        vb = [tuple(x * members for x in shard_range(fams, vblocks, r)) for r in range(vblocks)]
        jobs = [j for vr in range(vblocks) for j in pair_block_jobs(vb, vr)]
    else:
        jobs = pair_block_jobs(bounds, rank)
    single = ws == 1 and vblocks == 1          # one self job over the whole set
    # the rows this rank's jobs read, sketched locally in one job (span order)
    spans = merge_spans([j["ref"] for j in jobs] + [j["qry"] for j in jobs])
    base, seqs = [], []
    for lo_, hi_ in spans:
        base.append(len(seqs))
        seqs += c4_rows(lo_, hi_, members, seq_len)
    n_loc = len(seqs)

    def loc(g):
        """local row of global row g"""
        for (lo_, hi_), b_ in zip(spans, base):
            if lo_ <= g < hi_:
                return b_ + g - lo_
        raise KeyError(g)
    P = fpmash.make_params(k=k, s=s)
    job = ctx.sketch_job(P, seqs)
    del seqs
    d_rows, d_cnt, _ng, stride = job.device_output()
    d_len = fpmash.DeviceBuffer.from_array(ctx, np.full(n_loc, seq_len, np.uint64))
    L = fpmash.lib()
    st = ctx.stream

    def rows_at(g):
        """(rows, counts, lengths) device pointers at global row g"""
        r_ = loc(g)
        return d_rows + r_ * stride * 8, d_cnt + r_ * 4, d_len.ptr + r_ * 8
    outs = []
    for j in jobs:
        (rl, rh), (ql, qh) = j["ref"], j["qry"]
        o = {"p": compact_out(ctx, (rh - rl) * (qh - ql))}
        if j["kind"] == "mirror":
            o["m"] = compact_out(ctx, (rh - rl) * (qh - ql))
        outs.append(o)
    refsets = {}
    phase = {"sketch": 0.0, "dist": 0.0}

    def dist_share():
        if single:
            p_ = outs[0]["p"]
            fpmash._check(L.fpm_dist_list_dev(ctx.h, d_rows, d_cnt, d_len.ptr, stride, n, d_rows,
                                              d_cnt, d_len.ptr, stride, n, 8, s, k, 4.0 ** k,
                                              1.0, 1.0, p_[0].ptr, p_[1].ptr, p_[2].ref, st))
            return
        for rs in refsets.values():
            fpmash._check(L.fpm_refset_reindex(rs, st))
        for j, o in zip(jobs, outs):
            (rl, rh), (ql, qh) = j["ref"], j["qry"]
            q = rows_at(ql) + (stride, qh - ql)
            p_ = o["p"]
            if j["kind"] == "self":
                # the query pointers are the refset's own: the library's symmetric self path
                fpmash._check(L.fpm_refset_dist_list_dev(refsets[(rl, rh)], *q, s, k, 4.0 ** k,
                                                         1.0, 1.0, p_[0].ptr, p_[1].ptr,
                                                         p_[2].ref, st))
            else:
                m_ = o["m"]
                fpmash._check(L.fpm_refset_dist_mirror_list_dev(
                    refsets[(rl, rh)], *q, s, k, 4.0 ** k, 1.0, 1.0, p_[0].ptr, p_[1].ptr,
                    p_[2].ref, m_[0].ptr, m_[1].ptr, m_[2].ref, st))

    def run(timed):
        t0 = time.perf_counter()
        if prefill and single:
            # the grid's no-shared-hash counts (10 GB) written beside the sketch kernels on the
            # library's side stream (fpm_dist_list_prefill), instead of beside the rank kernel:
            # 6.34-6.35 -> 5.80 ms, same box, r05n (tools/leg_run.py --no-prefill: the A/B)
            p_ = outs[0]["p"]
            fpmash._check(L.fpm_dist_list_prefill(ctx.h, p_[0].ptr, p_[1].ptr, n, n, s, st))
        job.run(st)
        if timed:
            ctx.synchronize()
        t1 = time.perf_counter()
        dist_share()
        if timed:
            ctx.synchronize()
            phase["sketch"] += t1 - t0
            phase["dist"] += time.perf_counter() - t1
    if not single:
        # the indexes live as long as the leg over the job's output rows (rebuilt in every
        # step by fpm_refset_reindex after the sketch rewrote them)
        job.run(st)
        ctx.synchronize()
        for j in jobs:
            rl, rh = j["ref"]
            if (rl, rh) not in refsets:
                h = C.c_void_p()
                fpmash._check(L.fpm_refset_create_dev(ctx.h, *rows_at(rl), stride, rh - rl, 8,
                                                      s, C.byref(h)))
                refsets[(rl, rh)] = h
    for _ in range(warmup):
        run(False)
    ctx.synchronize()
    grp.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        run(False)
    ctx.synchronize()
    el_own = time.perf_counter() - t0
    grp.barrier()
    el = grp.max(el_own)
    listed = 0
    for o in outs:
        for key in ("p", "m"):
            if key in o:
                c_ = o[key][2].count()
                if c_ > o[key][2].cap:
                    raise RuntimeError(f"C4 cell list overflow: {c_} > {o[key][2].cap}")
                listed += c_
    listed = grp.sum(listed)
    dst = ctx.last_dist_stats()
    cand = grp.sum(dst["candidates"])
    run(True)                                   # one more step, phase-timed (not in el)
    # and one with per-kernel HIP events (the event records add markers between launches)
    ctx.reset_timing()
    ctx.set_timing(True)
    run(False)
    ctx.synchronize()
    ctx.set_timing(False)
    kt = {}
    for kid, name in fpmash.KERNEL_NAMES.items():
        tot, cnt_ = ctx.kernel_time(kid)
        if cnt_:
            kt[name] = {"ms": tot, "launches": cnt_}
    ctx.reset_timing()
    par = None
    rows_h = cnt_h = None
    if (parity and (rank == 0 or parity == "all")) or (cpu and rank == 0 and single):
        rows_h, cnt_h = job.fetch()

    def ref(g):
        r_ = loc(g)
        return rows_h[r_, :cnt_h[r_]]
    if parity and (rank == 0 or parity == "all"):
        # the CPU leg's checker: sampled rows of each of this rank's grids (and their
        # transposes) x all their references
        from oracle import oracle as O
        t_c = time.perf_counter()
        grids = []
        for j, o in zip(jobs, outs):
            (rl, rh), (ql, qh) = j["ref"], j["qry"]
            grids.append((o["p"], (rl, rh), (ql, qh)))
            if j["kind"] == "mirror":
                grids.append((o["m"], (ql, qh), (rl, rh)))
        per = max(4, 50 // len(grids))
        res = []
        for gi, (bufs, (rl, rh), (ql, qh)) in enumerate(grids):
            q = sample_rows(qh - ql, per, salt=4 + gi)
            gr = O.dist_grid([ref(g) for g in range(rl, rh)], [seq_len] * (rh - rl),
                             [ref(ql + int(x)) for x in q], [seq_len] * len(q), s, k, 4.0 ** k,
                             threads=_threads())
            res.append(check_grid_rows(bufs, rh - rl, q, gr))
        par = {"grids": len(grids), "rows": int(sum(r_["rows"] for r_ in res)),
               "pairs": int(sum(r_["pairs"] for r_ in res)),
               "pairs_sharing": int(sum(r_["pairs_sharing"] for r_ in res)),
               "ok": all(r_["ok"] for r_ in res), "check_s": time.perf_counter() - t_c}
    cpu_res = None
    if cpu and rank == 0 and single:
        # the reference's compare (CommandDistance.cpp:365-450: the literal walk + p-value per
        # pair, a worker pool) as the oracle's port on the CPUs available: 100 query rows x all
        # n references, scaled to the n x n grid (no text: the bench's C4 keeps its output in
        # HBM)
        from oracle import oracle as O
        th = _threads()
        qrows = sample_rows(n, 100, salt=9)
        refs = [ref(g) for g in range(n)]
        t_c = time.perf_counter()
        O.dist_grid(refs, [seq_len] * n, [refs[int(q)] for q in qrows], [seq_len] * len(qrows),
                    s, k, 4.0 ** k, threads=th)
        t_s = time.perf_counter() - t_c
        rate = len(qrows) * n / t_s
        cpu_res = {"kind": "port", "cores": th, "pairs_per_s": rate,
                   "grid_s_extrapolated": n * n / rate,
                   "sample": f"oracle literal walk + p-values, {len(qrows)} query rows x {n} "
                             f"references on {th} threads in {t_s:.1f} s, scaled to {n * n:.3g} "
                             "pairs"}
    for rs in refsets.values():
        L.fpm_refset_free(rs)
    for o in outs:
        for bl in o.values():
            for b in bl:
                b.free()
    d_len.free()
    job.free()
    cells = sum((j["ref"][1] - j["ref"][0]) * (j["qry"][1] - j["qry"][0]) *
                (2 if j["kind"] == "mirror" else 1) for j in jobs)
    return {"config": f"C4: all-vs-all dist of {n} family-structured {seq_len} bp sketches "
                      f"(k={k}, s={s}); a step = sketch the rows this rank's block pairs read "
                      f"+ its block pairs (each unordered pair compared once, grid + transpose "
                      f"written), no collective, {ws} GPU(s)",
            "n_gpus": ws, "rank": rank, "pairs": n * n, "steps": steps,
            "ms_per_step": el / steps * 1e3, "ms_per_step_this_rank": el_own / steps * 1e3,
            "output": "u16 numer/denom per pair + listed pairs with numer > 0 (SURVEY 8(d))",
            "listed_pairs_all_ranks": listed,
            "mpairs_per_s": n * n / (el / steps) / 1e6, "scaling": "strong",
            "phase_ms_rank0": {k_: v * 1e3 for k_, v in phase.items()},
            "kernels_rank0": kt,
            "collective": None, "exchange_ms": 0.0,
            "rows_sketched_rank0": n_loc, "rows_owned_rank0": bounds[rank][1] - bounds[rank][0],
            "virtual_blocks": vblocks,
            "jobs_rank0": [{"kind": j["kind"], "ref": list(j["ref"]), "qry": list(j["qry"])}
                           for j in jobs], "cells_rank0": cells,
            "path_rank0": fpmash.DIST_PATHS[int(dst["sparse"])],
            "candidates_all_ranks": cand, "parity": par, "cpu_baseline": cpu_res,
            "speedup_vs_cpu": (cpu_res["grid_s_extrapolated"] / (el / steps)
                               if cpu_res else None)}


def c4_shares(ctx, n=50_000, s=1000, k=21, world_sizes=(2, 4, 8), steps=3, warmup=1):
    """One rank's share of an N-rank C4 run, measured alone on this GPU: C4 has no exchange,
    so rank r of N needs nothing from the other ranks (c4_leg with ws = N, rank = r and a
    one-process group).  Rank 0 and rank N - 1 (for even N the ranks >= N/2 index a second
    block): the slower of the two is the N-GPU step this GPU's numbers predict, with no
    collective time to add."""
    one = Group(1)
    out = {}
    for ws in world_sizes:
        per = {}
        for r in sorted({0, ws - 1}):
            x = c4_leg(ctx, one, ws, r, 0, n=n, s=s, k=k, steps=steps, warmup=warmup,
                       parity=False)
            per[r] = {"ms_per_step": x["ms_per_step"], "phase_ms": x["phase_ms_rank0"],
                      "rows_sketched": x["rows_sketched_rank0"], "cells": x["cells_rank0"]}
        worst = max(v["ms_per_step"] for v in per.values())
        out[ws] = {"ranks": per, "share_ms_max": worst,
                   "projected_mpairs_per_s": n * n / (worst * 1e-3) / 1e6}
    return out


def cli_phases(stderr: bytes, prefix="[fpmash] "):
    """[fpmash] phase: X ms lines (FPMASH_TIMING=1) -> {phase: ms} (repeated phases summed).
    prefix "[fpmash-warm] ": the device warm-up thread's own steps (runtime start, context,
    staging ring), which run beside the main thread's input read; the main thread's wait for
    them is its "device context" phase."""
    out = {}
    for line in stderr.decode(errors="replace").splitlines():
        if line.startswith(prefix) and line.endswith(" ms") and ": " in line:
            name, val = line[len(prefix):-3].rsplit(": ", 1)
            try:
                out[name] = out.get(name, 0.0) + float(val)
            except ValueError:
                pass
    return out


def cli_leg(args, seqs, cpu=None, check=True):
    """The drop-in CLI end to end (CPU wall / GPU wall of the same command), on
    config C2's batch written as one lyn2vec-style FASTA:
      fpmash sketch -i -k 21 -s 1000 c2.fa -o c2     (parse + sketch + .msh write)
      fpmash dist c2.msh c2.msh > out                 (1e8 lines: resident reference set,
                                                       pipelined blocks, ordered text)
    Outside the timed commands: the .msh is byte-compared with the .msh the oracle's
    sketches encode to (tests/mshfmt.write_msh), and the first and last 50 query rows of the
    text (1 M lines, 1 % of the grid) with the oracle's lines; the reference's text step is
    timed on those 1 M lines.  The sketch command runs twice: the first process on a box
    (cold system ROCm libraries) is reported as `cli_sketch_wall_s_first_process`, the
    second is the timed wall."""
    import shutil
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "fp-mash_amd", "bin", "fpmash")
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    tmp = tempfile.mkdtemp(prefix="fpm_cli_", dir=base)
    try:
        ids = datagen.lyn2vec_ids(len(seqs))
        fa = os.path.join(tmp, "c2.fa")
        with open(fa, "wb") as f:
            f.write(datagen.fasta_bytes(seqs, ids))
        # FPMASH_TIMING=1: the host prints each phase's wall time to stderr (no output change)
        env = dict(os.environ, FPMASH_TIMING="1")
        # the first fpmash process on a fresh box pages the system ROCm runtime in from the
        # image (it is not the runtime torch loaded): that call is reported, the next is timed
        sk = [exe, "sketch", "-i", "-k", str(args.k), "-s", str(args.s), "-o", "c2", "c2.fa"]
        t0 = time.perf_counter()
        subprocess.run(sk, cwd=tmp, check=True, capture_output=True, env=env)
        t_first = time.perf_counter() - t0
        t0 = time.perf_counter()
        ps = subprocess.run(sk, cwd=tmp, check=True, capture_output=True, env=env)
        t_sketch = time.perf_counter() - t0
        out_path = os.path.join(tmp, "out.tsv")
        t0 = time.perf_counter()
        with open(out_path, "wb") as f:
            pd = subprocess.run([exe, "dist", "-p", str(_threads()), "c2.msh", "c2.msh"], cwd=tmp,
                                check=True, stdout=f, stderr=subprocess.PIPE, env=env)
        t_dist = time.perf_counter() - t0
        out_bytes = os.path.getsize(out_path)
        n = len(seqs)
        res = {"command_sketch": f"fpmash sketch -i -k {args.k} -s {args.s} -o c2 c2.fa",
               "command_dist": "fpmash dist c2.msh c2.msh > out",
               "fasta_bytes": os.path.getsize(fa), "cli_sketch_wall_s": t_sketch,
               "cli_sketch_wall_s_first_process": t_first,
               "cli_dist_wall_s": t_dist, "dist_lines": n * n, "dist_text_bytes": out_bytes,
               "dist_lines_per_s": n * n / t_dist, "output_dir": base or tempfile.gettempdir(),
               "phases_ms_sketch": cli_phases(ps.stderr), "phases_ms_dist": cli_phases(pd.stderr),
               "warm_thread_ms_sketch": cli_phases(ps.stderr, "[fpmash-warm] ")}
        ph_s, ph_d = res["phases_ms_sketch"], res["phases_ms_dist"]
        if cpu:
            # the same command on the CPU (CPU wall / GPU wall of the same work):
            #   sketch = the reference's kseq_read of the FASTA (oracle/_ref, timed here)
            #          + the sketch at the cpu_baseline leg's rate (reference heap when built)
            #          + the host steps both share (record headers, reference lists, the .msh
            #            write: the same C++ code, phases measured in the GPU command)
            #   dist   = the .msh load (shared host code, measured) + max(compare with
            #            p-values at the cpu_baseline rate, the reference's text step: ostream
            #            lines with `endl` per line, timed below on a 40-row block): the
            #            reference's workers compute while its main thread writes
            from oracle import oracle as O
            t0 = time.perf_counter()
            kscan = O.ref_kseq_scan(fa)
            t_parse = time.perf_counter() - t0 if kscan is not None else None
            rate = cpu.get("sketch_reference_bases_per_s") or cpu["sketch_bases_per_s"]
            host_shared = sum(ph_s.get(x, 0.0) for x in ("record headers", "reference lists",
                                                         "msh write")) * 1e-3
            res["cpu_port_sketch_s"] = n * args.seq_len / rate
            res["cpu_port_dist_s"] = n * n / cpu["dist_pairs_per_s"]
            if t_parse is not None:
                res["cpu_same_work"] = {
                    "sketch_s": t_parse + res["cpu_port_sketch_s"] + host_shared,
                    "sketch_parts_s": {"kseq_read (reference, compiled)": t_parse,
                                       "sketch": res["cpu_port_sketch_s"],
                                       "shared host steps (headers, lists, .msh write)":
                                           host_shared}}
                res["speedup_sketch"] = res["cpu_same_work"]["sketch_s"] / t_sketch
            res["speedup_dist_compute_only"] = res["cpu_port_dist_s"] / t_dist
        if check:
            from oracle import oracle as O
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import mshfmt
            t_c = time.perf_counter()
            exp = O.sketch_batch(O.params(k=args.k, s=args.s), seqs, threads=_threads())
            refs = [dict(name=b"T00000" + i.encode(), comment=b"G00000" + i.encode(),
                         length=len(q), hashes=h) for q, i, h in zip(seqs, ids, exp)]
            hdr = dict(kmer=args.k, windowSize=0, sketchSize=args.s, concatenated=False,
                       noncanonical=False, preserveCase=False, error=0.0, seed=42,
                       alphabet=b"ACGT")
            msh_ok = open(os.path.join(tmp, "c2.msh"), "rb").read() == mshfmt.write_msh(hdr, refs)
            rows = list(range(50)) + list(range(n - 50, n))
            nu, de, di, pv = O.dist_grid(exp, [len(q) for q in seqs], [exp[r] for r in rows],
                                         [len(seqs[r]) for r in rows], args.s, args.k,
                                         4.0 ** args.k, threads=_threads())
            names = [b"T00000" + i.encode() for i in ids]
            want = []
            for x, qr in enumerate(rows):
                for r in range(n):
                    c = x * n + r
                    want.append(b"%s\t%s\t%s\t%s\t%d/%d" % (
                        names[r], names[qr], (b"%g" % di[c]), (b"%g" % pv[c]), nu[c], de[c]))
            h = len(rows) // 2
            with open(out_path, "rb") as f:
                head = [f.readline().rstrip(b"\n") for _ in range(h * n)]
                f.seek(max(0, out_bytes - h * n * 200))
                tail = f.read().split(b"\n")[:-1][-h * n:]
            text_ok = head == want[:h * n] and tail == want[h * n:]
            if cpu and "cpu_same_work" in res:
                # the reference's text step on the 100 checked rows (1 M lines, endl per line)
                tpath = os.path.join(tmp, "ref_text.tsv")
                t0 = time.perf_counter()
                O.write_dist_text(tpath, names, rows, nu, de, di, pv, flush_each=True)
                t_txt = (time.perf_counter() - t0) * n / len(rows)
                load = ph_d.get("reference sketch loaded", 0.0) * 1e-3
                cw = res["cpu_same_work"]
                cw["dist_s"] = load + max(res["cpu_port_dist_s"], t_txt)
                cw["dist_parts_s"] = {"msh load (shared host code)": load,
                                      "compare + p-values": res["cpu_port_dist_s"],
                                      "text, endl per line (timed on 1 M lines = 100 rows, "
                                      "scaled)": t_txt,
                                      "combined as": "load + max(compare, text)"}
                res["speedup_dist"] = cw["dist_s"] / t_dist
                # the north-star figure: sketch + dist of C2, CPU same work / GPU wall
                res["speedup_sketch_plus_dist"] = (cw["sketch_s"] + cw["dist_s"]) / (t_sketch + t_dist)
            res["parity"] = {"msh_byte_identical": bool(msh_ok),
                             "dist_text_rows_checked": len(rows), "dist_text_exact": bool(text_ok),
                             "ok": bool(msh_ok and text_ok), "check_s": time.perf_counter() - t_c}
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def cli_fp_leg(args, cpu=None, check=True, n_seqs=5000, per_file=500):
    """The -fp drop-in end to end (north_star: `mash sketch -fp`, `mash dist -fp`), on C3's
    5,000 lyn2vec-shaped 2 kb sequences as CFL k-finger text in 10 files of 1 M lines
    (`sketch -fp` reads at most 1,000,000 lines per call, Sketch.cpp:37, :82):
      fpmash sketch -fp c3_<i>.txt -o c3_<i>     x 10  (parse + hash + group on the device)
      fpmash paste -fp c3_0.txt ... c3_9.txt -o c3      (host: the .msh inputs joined)
      fpmash dist -fp c3.msh c3.msh > out               (25 M lines: unsorted u32 lists,
                                                          the literal walk, ordered text)
    CPU same work (the reference's per-call structure, timed here):
      sketch = initFromFingerprints' istringstream parse around the reference's compiled
               getHashFingerPrint + HashList::add on one thread (oracle/_ref
               ref_fp_sketch_file; the reference runs it on its main thread) on 2 of the 10
               files, scaled x5, + the .msh write (shared host code, the GPU command's phase);
      paste  = the same host code: its GPU-side wall counts on both sides;
      dist   = the .msh loads (shared host code, measured) + max(compare: the oracle's literal
               walk on all cores over 100 query rows x 5,000, scaled to the grid; text: the
               reference's `endl`-per-line writer on 50 rows x 5,000 = 1 % of the lines,
               scaled), as the reference's workers compute while its main thread writes.
    Outside the timed commands: c3.msh's 5,000 references (names, lengths, hash lists cut to
    paste's default sketch size) against the oracle's initFromFingerprints, and the first and last 20 query rows of the text
    against the oracle's lines."""
    import shutil
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "fp-mash_amd", "bin", "fpmash")
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    tmp = tempfile.mkdtemp(prefix="fpm_clifp_", dir=base)
    try:
        seqs = datagen.random_dna(n_seqs, 2000, seed=33)
        ids = datagen.lyn2vec_ids(n_seqs, seed=33)
        names = [f"c3_{i}" for i in range(0, n_seqs // per_file)]
        sizes = []
        for j, nm in enumerate(names):
            t = datagen.cfl_text_fast(seqs[j * per_file:(j + 1) * per_file],
                                      ids[j * per_file:(j + 1) * per_file])
            with open(os.path.join(tmp, nm + ".txt"), "wb") as f:
                f.write(t)
            sizes.append(len(t))
        del seqs
        env = dict(os.environ, FPMASH_TIMING="1")
        sk_walls, ph_sk = [], []
        for nm in names:
            t0 = time.perf_counter()
            pr = subprocess.run([exe, "sketch", "-fp", nm + ".txt", "-o", nm], cwd=tmp, check=True,
                                capture_output=True, env=env)
            sk_walls.append(time.perf_counter() - t0)
            ph_sk.append(cli_phases(pr.stderr))
        t0 = time.perf_counter()
        subprocess.run([exe, "paste", "-fp"] + [nm + ".txt" for nm in names] + ["-o", "c3"],
                       cwd=tmp, check=True, capture_output=True, env=env)
        t_paste = time.perf_counter() - t0
        out_path = os.path.join(tmp, "out.tsv")
        t0 = time.perf_counter()
        with open(out_path, "wb") as f:
            pd = subprocess.run([exe, "dist", "-fp", "-p", str(_threads()), "c3.msh", "c3.msh"],
                                cwd=tmp, check=True, stdout=f, stderr=subprocess.PIPE, env=env)
        t_dist = time.perf_counter() - t0
        ph_d = cli_phases(pd.stderr)
        t_sk = sum(sk_walls)
        res = {"command_sketch": "fpmash sketch -fp c3_<i>.txt -o c3_<i> (x10, 1 M lines each)",
               "command_paste": "fpmash paste -fp c3_0.txt ... c3_9.txt -o c3",
               "command_dist": "fpmash dist -fp c3.msh c3.msh > out",
               "text_bytes": sum(sizes), "cli_sketch_fp_wall_s": t_sk,
               "cli_sketch_fp_wall_s_per_call": sk_walls, "cli_paste_fp_wall_s": t_paste,
               "cli_dist_fp_wall_s": t_dist, "dist_lines": n_seqs * n_seqs,
               "dist_text_bytes": os.path.getsize(out_path),
               "phases_ms_sketch_first_call": ph_sk[0], "phases_ms_dist": ph_d}
        from oracle import oracle as O
        th = _threads()
        refs = []
        if check or cpu:
            for nm in names:
                r, _u, _l = O.fp_references(open(os.path.join(tmp, nm + ".txt"), "rb").read())
                refs += r
        if cpu:
            t0 = time.perf_counter()
            scan = [O.ref_fp_sketch_files([os.path.join(tmp, nm + ".txt")]) for nm in names[:2]]
            t_scan = time.perf_counter() - t0
            if all(x is not None for x in scan):
                msh_w = sum(p_.get("msh write", 0.0) for p_ in ph_sk) * 1e-3
                cpu_sk = t_scan * len(names) / 2 + msh_w
                # compare: the oracle's literal walk (unsorted u32 lists, S = 1000, k = 1)
                lists = [h for _n, _l, h in refs]
                lens = [l_ for _n, l_, _h in refs]
                n = len(lists)
                qrows = sample_rows(n, 100, salt=5)
                t0 = time.perf_counter()
                nu, de, di, pv = O.dist_grid(lists, lens, [lists[int(q)] for q in qrows],
                                             [lens[int(q)] for q in qrows], 1000, 1, 10.0,
                                             use64=False, threads=th)
                t_cmp = (time.perf_counter() - t0) * n / len(qrows)
                # text: the reference's writer (endl per line) on 50 rows = 1 % of the lines
                nms = [x for x, _l, _h in refs]
                tpath = os.path.join(tmp, "ref_text.tsv")
                t0 = time.perf_counter()
                O.write_dist_text(tpath, nms, qrows[:50], nu[:50 * n], de[:50 * n], di[:50 * n],
                                  pv[:50 * n], flush_each=True)
                t_txt = (time.perf_counter() - t0) * n / 50
                load = (ph_d.get("reference sketch loaded", 0.0) +
                        ph_d.get("query sketch loaded", 0.0)) * 1e-3
                cpu_d = load + max(t_cmp, t_txt)
                res["cpu_same_work"] = {
                    "sketch_fp_s": cpu_sk, "paste_s": t_paste, "dist_fp_s": cpu_d,
                    "sketch_parts_s": {"istringstream parse + getHashFingerPrint (reference, "
                                       "compiled), 1 thread, 2 files x5": t_scan * len(names) / 2,
                                       ".msh writes (shared host code)": msh_w},
                    "dist_parts_s": {".msh loads (shared host code)": load,
                                     f"literal walk + p-values ({th} threads, 100 rows scaled)": t_cmp,
                                     "text, endl per line (50 rows = 1 % of the lines, scaled)":
                                         t_txt, "combined as": "load + max(compare, text)"},
                    "cores": th}
                res["speedup_sketch_fp"] = cpu_sk / t_sk
                res["speedup_dist_fp"] = cpu_d / t_dist
                res["speedup_dist_fp_compute_only"] = t_cmp / t_dist
                res["speedup_fp_sketch_paste_dist"] = (cpu_sk + t_paste + cpu_d) / \
                    (t_sk + t_paste + t_dist)
        if check:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import mshfmt
            t_c = time.perf_counter()
            got = mshfmt.read_msh(os.path.join(tmp, "c3.msh"))["references"]
            # paste loads its inputs with the default sketch size, which cuts every list to
            # its first 1,000 hashes (Sketch.cpp:1117-1122)
            msh_ok = len(got) == len(refs) and all(
                g["name"] == e[0] and int(g["length"]) == int(e[1]) and
                np.array_equal(np.asarray(g["hashes32"], np.uint32), e[2][:1000])
                for g, e in zip(got, refs))
            lists = [h for _n, _l, h in refs]
            lens = [l_ for _n, l_, _h in refs]
            n = len(lists)
            rows = list(range(20)) + list(range(n - 20, n))
            nu, de, di, pv = O.dist_grid(lists, lens, [lists[r] for r in rows],
                                         [lens[r] for r in rows], 1000, 1, 10.0, use64=False,
                                         threads=th)
            nms = [x for x, _l, _h in refs]
            want = [b"%s\t%s\t%s\t%s\t%d/%d" % (nms[r], nms[qr], b"%g" % di[x * n + r],
                                                b"%g" % pv[x * n + r], nu[x * n + r], de[x * n + r])
                    for x, qr in enumerate(rows) for r in range(n)]
            size = os.path.getsize(out_path)
            with open(out_path, "rb") as f:
                head = [f.readline().rstrip(b"\n") for _ in range(20 * n)]
                f.seek(max(0, size - 20 * n * 200))
                tail = f.read().split(b"\n")[:-1][-20 * n:]
            text_ok = head == want[:20 * n] and tail == want[20 * n:]
            res["parity"] = {"msh_references_exact": bool(msh_ok), "references": len(refs),
                             "dist_text_rows_checked": len(rows), "dist_text_exact": bool(text_ok),
                             "ok": bool(msh_ok and text_ok), "check_s": time.perf_counter() - t_c}
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


_ACGT_LUT = None


def c5_genome(g, length):
    """Synthetic C5 genome g: uniform ACGT from its own seed (the data does not depend on the
    GPU count), 2 bits of a random byte per base."""
    global _ACGT_LUT
    if _ACGT_LUT is None:
        acgt = np.frombuffer(b"ACGT", np.uint8)
        b = np.arange(256)
        _ACGT_LUT = np.stack([acgt[(b >> 6) & 3], acgt[(b >> 4) & 3], acgt[(b >> 2) & 3],
                              acgt[b & 3]], axis=1).astype(np.uint8)
    rng = np.random.default_rng(5000 + g)
    r = rng.integers(0, 256, size=(length + 3) // 4, dtype=np.uint8)
    return _ACGT_LUT[r].reshape(-1)[:length].tobytes()


def balanced_file_shards(lengths, ws):
    """Contiguous file ranges per rank balanced by bases: rank r takes the files
    whose base-count prefix midpoint falls in [r, r + 1) / ws of the total."""
    tot = float(sum(lengths)) or 1.0
    bounds = [0] * (ws + 1)
    acc = 0
    r = 1
    for i, L in enumerate(lengths):
        mid = (acc + L / 2.0) / tot
        while r < ws and mid >= r / ws:
            bounds[r] = i
            r += 1
        acc += L
    for rr in range(r, ws + 1):
        bounds[rr] = len(lengths)
    return [(bounds[i], bounds[i + 1]) for i in range(ws)]


def c5_leg(ctx, grp, ws, rank, n_genomes=1000, length=5_000_000, s=10_000, k=21, steps=2,
           warmup=1, parity=True, cpu=False):
    """C5: RefSeq-scale sketch of n_genomes x length bp, k=21, s=10,000, default
    (per-file, concatenated) mode: one sketch per genome.  Files are sharded over the ranks
    as contiguous ranges balanced by bases; each rank stages its genomes in HBM once and the
    timed step is its sketch kernels (tile hashing + bottom-s, then each genome's merge
    rounds).  After the timed steps the per-genome sketches are gathered to rank 0 in file
    order (the ordered reassembly); rank 0 checks the first and the last genome against the
    oracle."""
    from concurrent.futures import ThreadPoolExecutor
    lengths = [length] * n_genomes
    lo, hi = balanced_file_shards(lengths, ws)[rank]
    with ThreadPoolExecutor(max_workers=min(16, _threads())) as ex:
        seqs = list(ex.map(lambda g: c5_genome(g, length), range(lo, hi)))
    n_loc = hi - lo
    P = fpmash.make_params(k=k, s=s)
    job = ctx.sketch_job(P, seqs, groups=list(range(n_loc)), n_groups=n_loc)
    info = job.info()
    del seqs
    st = ctx.stream
    for _ in range(warmup):
        job.run(st)
    ctx.synchronize()
    grp.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        job.run(st)
    ctx.synchronize()
    el = time.perf_counter() - t0
    grp.barrier()
    el_max = grp.max(el)
    # kernel times of this rank (HIP events, extra runs outside the timed ones)
    ctx.reset_timing()
    ctx.set_timing(True)
    ctx.merge_small_spills()                    # reset the counter
    job.run(st)
    ctx.synchronize()
    ctx.set_timing(False)
    spills = ctx.merge_small_spills()           # small-list merges that overflowed their LDS
    kt = {}
    dev_ms = 0.0
    for kid in (fpmash.K_SKETCH, fpmash.K_MERGE):
        tot, cnt = ctx.kernel_time(kid)
        kt[fpmash.KERNEL_NAMES[kid]] = {"ms": tot, "launches": cnt}
        dev_ms += tot
    ctx.reset_timing()
    rows, cnt = job.fetch()
    job.free()
    # ordered reassembly on rank 0 (host rows over gloo: 80 KB per genome)
    if ws > 1:
        import torch
        from fpmash.shard import all_gather_rows
        m = max(h - l for l, h in balanced_file_shards(lengths, ws))
        buf = np.zeros((m, s + 1), np.int64)
        buf[:n_loc, :s] = rows.view(np.int64)
        buf[:n_loc, s] = cnt
        parts = [torch.empty((m, s + 1), dtype=torch.int64) for _ in range(ws)]
        grp.dist.all_gather(parts, torch.from_numpy(buf))
        spans = balanced_file_shards(lengths, ws)
        allr = np.concatenate([parts[r].numpy()[: h - l] for r, (l, h) in enumerate(spans)])
        rows_all, cnt_all = allr[:, :s].view(np.uint64), allr[:, s].astype(np.uint32)
    else:
        rows_all, cnt_all = rows, cnt
    bases_loc = n_loc * length
    alg = info["seq_bytes"] + int(cnt.astype(np.uint64).sum()) * 8
    out = {"config": f"C5: {n_genomes} x {length} bp genomes, k={k}, s={s}, one sketch per "
                     f"genome, files sharded over {ws} GPU(s) (contiguous, balanced by bases)",
           "n_gpus": ws, "genomes": n_genomes, "bases": n_genomes * length, "steps": steps,
           "ms_per_step": el_max / steps * 1e3,
           "bases_per_s": n_genomes * length / (el_max / steps), "scaling": "strong",
           "rank0": {"genomes": n_loc, "bases": bases_loc, "device_ms": dev_ms,
                     "bases_per_s_device": bases_loc / (dev_ms * 1e-3) if dev_ms else None,
                     "alg_bytes": alg,
                     "alg_GBps": alg / (dev_ms * 1e-3) / 1e9 if dev_ms else None,
                     "frac_hbm": alg / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if dev_ms else None,
                     "tiles": info["n_tiles"], "kernels": kt,
                     "merge_small_lds_overflows": spills},
           "reassembled_genomes": int(len(rows_all)) if rank == 0 else None}
    if parity and rank == 0:
        from oracle import oracle as O
        t_c = time.perf_counter()
        # parity="all" (the multi-rank GPU test): every genome, so the reassembled file order
        # is checked across the shard boundaries too
        idx = list(range(n_genomes)) if parity == "all" else sorted({0, n_genomes - 1})
        exp = O.sketch_batch(O.params(k=k, s=s), [c5_genome(g, length) for g in idx],
                             threads=max(2, min(len(idx), _threads())))
        ok = [bool(int(cnt_all[g]) == len(e) and np.array_equal(rows_all[g, :len(e)], e))
              for g, e in zip(idx, exp)]
        out["parity"] = {"genomes_checked": idx, "sketch_exact": ok, "ok": all(ok),
                         "shards": balanced_file_shards(lengths, ws),
                         "check_s": time.perf_counter() - t_c}
    if cpu and rank == 0 and ws == 1:
        # the reference's sketchFile (Sketch.cpp:1299-1488: one MinHashHeap per genome, files
        # dealt to the -p threads) through its own compiled getHash + MinHashHeap (oracle/_ref):
        # one genome per thread on the CPUs available, scaled to the n_genomes files
        from oracle import oracle as O
        th = _threads()
        sample = [c5_genome(g, length) for g in range(min(th, n_genomes))]
        t_c = time.perf_counter()
        rsk = O.ref_sketch_batch(sample, k=k, s=s, threads=th)
        t_s = time.perf_counter() - t_c
        if rsk is not None:
            rate = len(sample) * length / t_s
            out["cpu_baseline"] = {
                "kind": "reference", "cores": th, "bases_per_s": rate,
                "step_s_extrapolated": n_genomes * length / rate,
                "sample": f"{len(sample)} genomes x {length / 1e6:g} Mb, one per thread on {th} "
                          f"threads, the reference's getHash + MinHashHeap (oracle/_ref) in "
                          f"{t_s:.1f} s, scaled to {n_genomes} genomes"}
            out["speedup_vs_cpu"] = out["cpu_baseline"]["step_s_extrapolated"] / (el_max / steps)
    return out


_GENOME_BLOCK = 1 << 22


def split_genome_range(lo, hi):
    """Bases [lo, hi) of the split leg's synthetic genome: uniform ACGT generated in 4 Mb
    blocks from per-block seeds, so any rank builds its own range without the rest."""
    global _ACGT_LUT
    if _ACGT_LUT is None:
        c5_genome(0, 4)                          # builds the byte -> 4 bases table
    out = []
    for b in range(lo // _GENOME_BLOCK, (hi + _GENOME_BLOCK - 1) // _GENOME_BLOCK):
        rng = np.random.default_rng(900_000 + b)
        r = rng.integers(0, 256, size=_GENOME_BLOCK // 4, dtype=np.uint8)
        blk = _ACGT_LUT[r].reshape(-1)
        a, e = max(lo, b * _GENOME_BLOCK) - b * _GENOME_BLOCK, min(hi, (b + 1) * _GENOME_BLOCK) - b * _GENOME_BLOCK
        out.append(blk[a:e])
    return np.concatenate(out).tobytes() if out else b""


def comm_check(ctx, grp, s=2000, k=21):
    """The min-merge's RCCL path (fpm_sketch_min_merge_comm) on a one-rank communicator: one
    300 kb genome sketched in four k-mer ranges, each range's bottom-s row min-merged through
    the communicator (a one-rank gather is a copy, then the device merge) in turn, and the four
    merged rows merged again, against the oracle's sketch of the whole genome."""
    from fpmash.shard import kmer_shard, min_merge
    from oracle import oracle as O
    t0 = time.perf_counter()
    seq = datagen.family_dna(1, 1, 300_000, seed=77)[0]
    P = fpmash.make_params(k=k, s=s)
    comm = grp.comm(ctx)
    parts = [seq[a:b] for a, b in (kmer_shard(len(seq), k, 4, r) for r in range(4))]
    job = ctx.sketch_job(P, parts)
    job.run(ctx.stream)
    d_rows, d_cnt, _ng, stride = job.device_output()
    got = [min_merge(ctx, d_rows + i * stride * 8, d_cnt + i * 4, s, 1, comm=comm)
           for i in range(4)]
    m = np.zeros((4, s), np.uint64)
    for i, (h, n_) in enumerate(got):
        m[i, :n_] = h
    rows_d = fpmash.DeviceBuffer.from_array(ctx, m)
    cnt_d = fpmash.DeviceBuffer.from_array(ctx, np.array([n_ for _, n_ in got], np.uint32))
    o, oc = fpmash.DeviceBuffer(ctx, s * 8), fpmash.DeviceBuffer(ctx, 4)
    fpmash._check(fpmash.lib().fpm_sketch_merge_dev(ctx.h, rows_d.ptr, cnt_d.ptr, 4, s, o.ptr,
                                                    oc.ptr, None))
    n_ = int(oc.to_array(np.uint32, 1)[0])
    merged = o.to_array(np.uint64, s)[:n_]
    job.free()
    exp = O.sketch_batch(O.params(k=k, s=s), [seq])[0]
    exp_parts = O.sketch_batch(O.params(k=k, s=s), parts)
    ok_parts = all(n_i == len(e) and np.array_equal(h, e) for (h, n_i), e in zip(got, exp_parts))
    ok = bool(ok_parts and n_ == len(exp) and np.array_equal(merged, exp))
    res = {"ok": ok and comm is not None, "one_rank_merges_equal_parts": bool(ok_parts),
           "merged_equals_whole": bool(n_ == len(exp) and np.array_equal(merged, exp)),
           "collective": "RCCL in libfpmash (fpm_sketch_min_merge_comm), 1 rank",
           "check_s": time.perf_counter() - t0}
    if comm is None:                 # the RCCL path did not run: not a pass
        res["comm_error"] = grp.comm_error
    return res


def split_leg(ctx, grp, ws, rank, local, length=1_000_000_000, s=10_000, k=21, steps=3,
              warmup=1, parity=True):
    """One sketch split over the GPUs (north_star: "RCCL ... for the final min-merge where a
    single sketch exceeds one GPU"): one genome of `length` bases, its k-mer starts sharded
    into contiguous ranges (fpmash.shard.kmer_shard: k - 1 bases of overlap), each rank
    sketches its range, and the ranks' bottom-s rows are all-gathered (RCCL over xGMI inside
    libfpmash, fpm_sketch_min_merge_comm) and min-merged on the device.  Timed step: sketch +
    gather + merge.  Check (outside the timed steps): the merged sketch equals the sketch of
    the whole genome in one piece, computed on rank 0 (at N = 1: four parts merged in one
    process against the whole); the merge itself is pinned to the oracle in
    tests/test_gpu_parity.py."""
    from fpmash.shard import kmer_shard, min_merge
    lo, hi = kmer_shard(length, k, ws, rank)
    P = fpmash.make_params(k=k, s=s)
    job = ctx.sketch_job(P, [split_genome_range(lo, hi)], groups=[0], n_groups=1)
    d_rows, d_cnt, _ng, _stride = job.device_output()
    st = ctx.stream
    comm = grp.comm(ctx) if ws > 1 else None

    def step():
        job.run(st)
        if ws > 1:
            return min_merge(ctx, d_rows, d_cnt, s, ws, comm=comm, group=None)
        ctx.synchronize()
        return None
    for _ in range(warmup):
        step()
    ctx.synchronize()
    grp.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        merged = step()
    ctx.synchronize()
    el = grp.max(time.perf_counter() - t0)
    rows, cnt = job.fetch()
    job.free()
    if merged is None:
        merged = (rows[0, : cnt[0]], int(cnt[0]))
    out = {"config": f"one {length / 1e9:g} Gb genome, k={k}, s={s}, k-mer starts sharded over "
                     f"{ws} GPU(s), bottom-s rows all-gathered "
                     f"({'RCCL in libfpmash' if comm is not None else 'none' if ws == 1 else 'gloo'})"
                     " and min-merged on the device",
           "n_gpus": ws, "bases": length, "steps": steps, "ms_per_step": el / steps * 1e3,
           "bases_per_s": length / (el / steps), "scaling": "strong"}
    if grp.comm_error:
        out["comm_error"] = grp.comm_error
    if parity and rank == 0:
        t_c = time.perf_counter()
        whole = ctx.sketch(P, [split_genome_range(0, length)])[0]
        ok = bool(len(whole) == merged[1] and np.array_equal(whole, merged[0]))
        res = {"merged_equals_whole": ok}
        if ws == 1:
            # four parts merged in this process (the same merge call the ranks make)
            parts = [split_genome_range(*kmer_shard(length, k, 4, r)) for r in range(4)]
            sk = ctx.sketch(P, parts)
            m = np.zeros((4, s), np.uint64)
            for i, x in enumerate(sk):
                m[i, : len(x)] = x
            rows_d = fpmash.DeviceBuffer.from_array(ctx, m)
            cnt_d = fpmash.DeviceBuffer.from_array(ctx, np.array([len(x) for x in sk], np.uint32))
            o = fpmash.DeviceBuffer(ctx, s * 8)
            oc = fpmash.DeviceBuffer(ctx, 4)
            fpmash._check(fpmash.lib().fpm_sketch_merge_dev(ctx.h, rows_d.ptr, cnt_d.ptr, 4, s,
                                                            o.ptr, oc.ptr, None))
            ctx.synchronize()
            n4 = int(oc.to_array(np.uint32, 1)[0])
            ok4 = bool(n4 == len(whole) and np.array_equal(o.to_array(np.uint64, s)[:n4], whole))
            res["four_parts_merged_equal_whole"] = ok4
            ok = ok and ok4
        res.update({"ok": ok, "check_s": time.perf_counter() - t_c})
        out["parity"] = res
    return out


MAX_LINE_BYTES = 8192     # the driver parses one JSON line of about this size at most


def write_detail(detail, path):
    """The full result (every leg's counters, per-kernel tables, CLI phases) as a side file;
    the printed line keeps only the headline numbers.  Returns the path written, or None."""
    if path == "":
        return None
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(detail, f, indent=1)
        return os.path.relpath(os.path.abspath(path), ROOT)
    except OSError:
        return None


def _r(x, nd=4):
    """a number rounded to nd significant digits (None passes through)"""
    if x is None or isinstance(x, bool):
        return x
    if isinstance(x, int):
        return x
    try:
        return float(f"{float(x):.{nd}g}")
    except (TypeError, ValueError):
        return None


def _ok(part):
    return None if not part else bool(part.get("ok"))


def compact_line(d, detail_path=None):
    """The one JSON line bench.py prints: the contract's fields, `roofline`, `cpu_baseline`,
    parity as booleans and one or two numbers per leg (well under MAX_LINE_BYTES; the
    detail goes to the side file)."""
    g = lambda o, *ks: (o or {}).get(ks[0]) if len(ks) == 1 else g((o or {}).get(ks[0]), *ks[1:])  # noqa: E731
    roof = d.get("roofline") or {}
    cpu = d.get("cpu_baseline")
    par = d.get("parity") or {}
    line = {k: d.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
                                  "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
                                  "dtype", "data")}
    line["config"] = d.get("config")
    line["roofline"] = {k: (_r(roof.get(k)) if isinstance(roof.get(k), float) else roof.get(k))
                        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel",
                                  "avg_launch_ms", "alg_bytes_per_launch", "valu_issue_frac",
                                  "traffic_source", "traffic_note", "build_id")}
    if roof.get("wave_state_frac"):
        line["roofline"]["wave_state_frac"] = {k: _r(v, 3) for k, v in
                                               roof["wave_state_frac"].items()}
    line["cpu_baseline"] = None if not cpu else {
        "value": cpu.get("value"), "unit": cpu.get("unit"), "cores": cpu.get("cores"),
        "cores_note": cpu.get("cores_note"),
        "kind": cpu.get("kind"), "sample": cpu.get("sample"), "cpu_model": cpu.get("cpu_model")}
    line["parity"] = {"c2": _ok(par.get("c2")), "c3_fp": _ok(par.get("c3_fp")),
                      "c4": _ok(par.get("c4")), "c4_vblocks": _ok(par.get("c4_vblocks")),
                      "comm_min_merge": _ok(par.get("comm_min_merge")),
                      "c5": _ok(par.get("c5")),
                      "split": _ok(par.get("split")), "cli": _ok(par.get("cli")),
                      "cli_fp": _ok(par.get("cli_fp")),
                      "all_ok": par.get("all_ok")}
    c3, c4, c5 = d.get("c3_fp"), d.get("c4_dist"), d.get("c5_sketch")
    sp, cli, clf = d.get("split_sketch"), d.get("cli"), d.get("cli_fp")
    legs = {
        "sketch_bases_per_s": _r(g(d, "sketch", "bases_per_s")),
        "sketch_device_ms": _r(g(d, "sketch", "device_ms_per_step")),
        "dist_mpairs_per_s": _r(g(d, "dist", "mpairs_per_s")),
        "dist_device_ms": _r(g(d, "dist", "device_ms_per_step")),
        "dist_path": g(d, "dist", "path"),
        "c2_full_grid_ms": _r(g(d, "config", "full_grid_ms_per_step")),
        "fp_text_lines_per_s": _r(g(d, "fp_text", "lines_per_s_device")),
        "c3_dist_ms": _r(g(c3, "dist_ms")), "c3_dense_walk_ms": _r(g(c3, "dense_walk_ms")),
        "c3_parse_device_ms": _r(g(c3, "parse_device_ms")),
        "c4_ms_per_step": _r(g(c4, "ms_per_step")), "c4_mpairs_per_s": _r(g(c4, "mpairs_per_s")),
        "c4_cpu_mpairs_per_s": _r((g(c4, "cpu_baseline", "pairs_per_s") or 0) / 1e6 or None),
        "c4_speedup_vs_cpu": _r(g(c4, "speedup_vs_cpu"), 3),
        "c4_output": g(c4, "output"),
        "c4_exchange_ms": g(c4, "exchange_ms"),
        "c4_share_ms_n2": _r(g(d, "c4_shares", 2, "share_ms_max")),
        "c4_share_ms_n4": _r(g(d, "c4_shares", 4, "share_ms_max")),
        "c4_share_ms_n8": _r(g(d, "c4_shares", 8, "share_ms_max")),
        "c5_ms_per_step": _r(g(c5, "ms_per_step")), "c5_bases_per_s": _r(g(c5, "bases_per_s")),
        "c5_cpu_bases_per_s": _r(g(c5, "cpu_baseline", "bases_per_s")),
        "c5_speedup_vs_cpu": _r(g(c5, "speedup_vs_cpu"), 3),
        "split_ms_per_step": _r(g(sp, "ms_per_step")),
        "cli_sketch_wall_s": _r(g(cli, "cli_sketch_wall_s")),
        "cli_sketch_wall_s_first_process": _r(g(cli, "cli_sketch_wall_s_first_process")),
        "cli_dist_wall_s": _r(g(cli, "cli_dist_wall_s")),
        "cli_speedup_sketch": _r(g(cli, "speedup_sketch"), 3),
        "cli_speedup_dist": _r(g(cli, "speedup_dist"), 3),
        "cli_speedup_dist_compute_only": _r(g(cli, "speedup_dist_compute_only"), 3),
        "cli_speedup_sketch_plus_dist": _r(g(cli, "speedup_sketch_plus_dist"), 3),
        "cli_fp_sketch_wall_s": _r(g(clf, "cli_sketch_fp_wall_s")),
        "cli_fp_paste_wall_s": _r(g(clf, "cli_paste_fp_wall_s")),
        "cli_fp_dist_wall_s": _r(g(clf, "cli_dist_fp_wall_s")),
        "cli_fp_speedup_sketch": _r(g(clf, "speedup_sketch_fp"), 3),
        "cli_fp_speedup_dist": _r(g(clf, "speedup_dist_fp"), 3),
        "cli_fp_speedup_dist_compute_only": _r(g(clf, "speedup_dist_fp_compute_only"), 3),
        "cli_fp_speedup_all": _r(g(clf, "speedup_fp_sketch_paste_dist"), 3),
        "c3_parse_wall_ms_pcie": _r(g(c3, "parse_wall_ms_pcie")),
    }
    line["legs"] = {k: v for k, v in legs.items() if v is not None}
    line["detail"] = detail_path
    s = json.dumps(line)
    if len(s) > MAX_LINE_BYTES:                 # never let the line outgrow the parser
        line["cpu_baseline"] = line["cpu_baseline"] and {
            k: v for k, v in line["cpu_baseline"].items() if k != "sample"}
        line["legs"] = {k: v for k, v in line["legs"].items() if isinstance(v, (int, float))}
    return line


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
    # The dist output: u16 numer / denom for every cell (4 B per pair) +
    # the list of cells that share hashes (numer > 0) with distance / FP64 p-value / pass
    # (fpm_dist_list_dev).  Every other cell's distance / p-value / pass is closed-form
    # (CommandDistance.cpp:404-408, 435-437 at common = 0); the parity check expands sampled
    # rows to all five values.  Family-structured C2: ~1 % of the pairs share hashes.
    d_numer = fpmash.DeviceBuffer(ctx, n_pairs * 2)
    d_denom = fpmash.DeviceBuffer(ctx, n_pairs * 2)
    cells = fpmash.CellList(ctx, max(1 << 20, n_pairs // 25))
    lengths = np.full(n, args.seq_len, dtype=np.uint64)
    d_len = fpmash.DeviceBuffer.from_array(ctx, lengths)
    st = ctx.stream

    def step():
        # (no counts prefill here: the probe writes the 1e8 cells' defaults as it goes; written
        # beside the sketch kernels instead, fpm_dist_list_prefill, they slowed the sketch and
        # the index build more than the probe gained: 0.996-1.001 -> 1.010-1.016 ms, same box,
        # r05n; on C4's 2.5e9 cells it wins, c4_leg)
        job.run(st)
        fpmash._check(L.fpm_dist_list_dev(ctx.h, d_rows, d_cnt, d_len.ptr, stride, n, d_rows,
                                          d_cnt, d_len.ptr, stride, n, 8, args.s, args.k,
                                          4.0 ** args.k, 1.0, 1.0, d_numer.ptr, d_denom.ptr,
                                          cells.ref, st))

    def run_steps(k):
        for _ in range(k):
            step()

    # (Pipelined steps — the sketch of batch i+1 on a second stream, fpm_stream_create /
    # fpm_event_*, beside the dist of batch i — measured 1.023 vs 0.962 ms per step serial,
    # same box: the tile kernel's workgroups take LDS and CUs from the rank kernel.)
    run_steps(args.warmup)
    ctx.synchronize()
    grp.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps)
    ctx.synchronize()
    t1 = time.perf_counter()
    grp.barrier()
    elapsed = grp.max(t1 - t0)
    n_listed = cells.count()
    if n_listed > cells.cap:
        raise RuntimeError(f"C2 cell list overflow: {n_listed} cells > {cells.cap}")

    # the same step with the full five-array output (fpm_dist_dev16: distance / p-value / pass
    # written for every cell, 21 B per pair), for comparison with rounds 1-3: not `value`
    full_ms = None
    if not args.no_full_grid:
        d_dist = fpmash.DeviceBuffer(ctx, n_pairs * 8)
        d_pval = fpmash.DeviceBuffer(ctx, n_pairs * 8)
        d_pass = fpmash.DeviceBuffer(ctx, n_pairs)

        def full_step():
            job.run(st)
            fpmash._check(L.fpm_dist_dev16(ctx.h, d_rows, d_cnt, d_len.ptr, stride, n, d_rows,
                                           d_cnt, d_len.ptr, stride, n, 8, args.s, args.k,
                                           4.0 ** args.k, 1.0, 1.0, d_numer.ptr, d_denom.ptr,
                                           d_dist.ptr, d_pval.ptr, d_pass.ptr, st))
        for _ in range(args.warmup):
            full_step()
        ctx.synchronize()
        t0f = time.perf_counter()
        for _ in range(args.steps):
            full_step()
        ctx.synchronize()
        full_ms = (time.perf_counter() - t0f) / args.steps * 1e3
        for b in (d_dist, d_pval, d_pass):
            b.free()

    # per-kernel times: HIP events around every launch, in separate steps after the timed
    # region (the event records add markers between launches, so they stay out of it)
    n_timed = timing_steps(args.steps)
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(n_timed):
        step()
    ctx.synchronize()
    ctx.set_timing(False)
    dstats = ctx.last_dist_stats()
    c2_rebuilds = ctx.index_rebuilds()          # one-pass index builds redone so far (C2 only)
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
    c2par = None
    if rank == 0 and not args.no_parity:
        c2par = c2_parity(job, seqs, (d_numer, d_denom, cells), args)

    bases_rank = n * args.seq_len
    total_bases = grp.sum(bases_rank) * args.steps
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
        # sparse dist, compact output: the probe writes every cell's u16 numer / denom
        # defaults; the candidate kernel scatters the candidates' counts (and their mirrors on
        # the symmetric path) and lists the cells with numer > 0
        n_cand = dstats["candidates"]
        ccells = 2 * n_cand - n if dstats["sparse"] == 2 else n_cand
        alg[N[fpmash.K_PROBE]] = (n_hash * 8 + n_pairs * (2 + 2),
                                  "query sketch hashes read + u16 numer/denom defaults (4 B/pair) "
                                  "written")
        alg[N[fpmash.K_FINALIZE]] = (n_cand * (8 + 4 + 4) + ccells * (2 + 2) + n_listed * 25,
                                     "candidate + its counts read, counts scattered per candidate "
                                     "cell (mirrors included), 25 B per listed cell")
    else:
        alg[N[fpmash.K_COMPARE]] = (2 * n_hash * 8 + n_pairs * 4,
                                    "ref + query sketches read + u16 numer/denom (4 B/pair) written")
        alg[N[fpmash.K_FINALIZE]] = (n_pairs * (2 + 2) + n_listed * 25,
                                     "numer/denom read, 25 B per listed cell written")
    pmc_at = pmc_dir(args.pmc_dir)
    pmc, pmc_note = load_pmc("pmc_traffic.json", pmc_at)
    traffic = (pmc or {}).get("kernels", {})
    # the dominant kernel: the longest single launch
    dom = max(ktimes, key=lambda k_: ktimes[k_]["total_ms"] / ktimes[k_]["launches"])
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
        "traffic_source": pmc["source"] if dom in traffic else None,
        "traffic_note": pmc_note if pmc_note else (None if dom in traffic else
                                                   f"no counters for {dom} in {pmc['source']}"),
        "build_id": fpmash.build_id(),
        "alg_bytes_per_launch": alg.get(dom, (None, ""))[0],
        "alg_bytes_formula": alg.get(dom, (None, ""))[1],
        "avg_launch_ms": ktimes[dom]["avg_ms"],
    }
    per_kernel_roof = {}
    for name, (b, _) in alg.items():
        if name in ktimes:
            gbs = b / (ktimes[name]["avg_ms"] * 1e-3) / 1e9
            # (PMC bytes of a kernel group are per step: tools/pmc_traffic.py sums a group's
            # dispatches over the launches of its most frequent kernel, the fill's two
            # variants included)
            per_kernel_roof[name] = {"avg_ms": ktimes[name]["avg_ms"], "alg_GBps": gbs,
                                     "frac_hbm": gbs / HBM_PEAK_GBS,
                                     "traffic_bytes": traffic.get(name, {}).get("traffic_bytes")}

    sk_names = [fpmash.KERNEL_NAMES[k_] for k_ in (fpmash.K_SKETCH, fpmash.K_MERGE)]
    di_names = [fpmash.KERNEL_NAMES[k_] for k_ in (fpmash.K_INDEX, fpmash.K_PROBE,
                                                  fpmash.K_COMPARE, fpmash.K_FINALIZE)]
    sk_ms = per_step_ms(ktimes, sk_names, n_timed)
    di_ms = per_step_ms(ktimes, di_names, n_timed)
    bases_step = grp.sum(bases_rank)
    pairs_step = grp.sum(n_pairs)

    fp_leg = fp_text_leg(ctx) if rank == 0 and not args.no_fp_text else None
    c3 = c3_leg(ctx, s=args.s, parity=not args.no_parity) if rank == 0 and not args.no_c3 else None
    c4 = None
    if not args.no_c4:
        job.free()                       # the C2 batch's buffers make room for C4's grid
        for b in (d_numer, d_denom):
            b.free()
        cells.free()
        c4 = c4_leg(ctx, grp, ws, rank, local, n=args.c4_n, s=args.s, k=args.k,
                    parity=not args.no_parity, cpu=not args.no_cpu_baseline)
    c4g = comm_chk = shares = None
    if ws == 1 and not args.no_gather_check:
        # the N > 1 paths on this GPU, outside every timed number: the C4 job structure of a
        # three-way split (every virtual rank's self / mirror jobs, every grid sampled against
        # the oracle), and the RCCL min-merge inside libfpmash on a one-rank communicator
        if not args.no_c4:
            c4g = c4_leg(ctx, grp, ws, rank, local, n=6000, s=args.s, k=args.k, steps=1,
                         warmup=1, parity="all" if not args.no_parity else False, vblocks=3)
        if not args.no_parity:
            comm_chk = comm_check(ctx, grp)
    if ws == 1 and not args.no_c4 and not args.no_c4_shares:
        shares = c4_shares(ctx, n=args.c4_n, s=args.s, k=args.k)

    c5 = None
    if not args.no_c5:
        c5 = c5_leg(ctx, grp, ws, rank, n_genomes=args.c5_genomes, parity=not args.no_parity,
                    cpu=not args.no_cpu_baseline)

    split = None
    if not args.no_split:
        split = split_leg(ctx, grp, ws, rank, local, length=args.split_bases,
                          parity=not args.no_parity)

    for leg, r_ in (("c3", c3), ("c4", c4), ("c5", c5)):
        if r_ is not None:
            r_["counters"] = leg_counters(leg, pmc_at)

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, seqs)

    cli = None
    if rank == 0 and ws == 1 and not args.no_cli:
        cli = cli_leg(args, seqs, cpu, check=not args.no_parity)
    cli_fp = None
    if rank == 0 and ws == 1 and not args.no_cli_fp:
        cli_fp = cli_fp_leg(args, cpu, check=not args.no_parity)

    if rank == 0:
        detail = {
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
                             f"+ all-vs-all dist of the {n} sketches ({n_pairs:.3g} pairs), per GPU; "
                             "dist output per SURVEY 8(b)/(d): u16 numer/denom of every pair + "
                             "distance/FP64 p-value/pass listed for the pairs with numer > 0 "
                             "(all other pairs: distance 1, p-value 1 by CommandDistance.cpp:"
                             "404-408, 435-437)"),
                "n_seqs_per_gpu": n, "seq_len": args.seq_len, "k": args.k, "s": args.s,
                "pairs_per_gpu": n_pairs, "parallelism": f"independent batch per GPU x{ws}",
                "listed_pairs_per_gpu": n_listed,
                "full_grid_ms_per_step": full_ms,   # distance/p-value/pass written for every pair
            },
            "kernel_timing_steps": n_timed,
            "sketch": {"bases_per_s": bases_step / (sk_ms * 1e-3) if sk_ms else None,
                       "device_ms_per_step": sk_ms, "tiles": info["n_tiles"],
                       "kmers": info["n_kmers"]},
            "dist": {"mpairs_per_s": pairs_step / (di_ms * 1e-3) / 1e6 if di_ms else None,
                     "device_ms_per_step": di_ms,
                     "pairs_with_shared_hashes_frac_sample": float((numer_sample > 0).mean()),
                     "path": fpmash.DIST_PATHS[int(dstats["sparse"])],
                     "posting_events": dstats["events"], "candidate_pairs": dstats["candidates"],
                     "index_one_pass_rebuilds": c2_rebuilds},
            "fp_text": fp_leg,
            "c3_fp": c3,
            "c4_dist": c4,
            "c4_vblocks_check": c4g,
            "c4_shares": shares,
            "comm_check": comm_chk,
            "c5_sketch": c5,
            "split_sketch": split,
            "cli": cli,
            "cli_fp": cli_fp,
            "kernels": ktimes,
            "kernel_roofline": per_kernel_roof,
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity_summary(c2par, c3, c4, c5, cli, split, c4g, cli_fp, comm_chk),
        }
        path = write_detail(detail, args.detail)
        print(json.dumps(compact_line(detail, path)))
    job.free()
    grp.close()
    ctx.close()


if __name__ == "__main__":
    main()
