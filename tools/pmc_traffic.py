#!/usr/bin/env python3
"""tools/pmc_traffic.py — HBM traffic per kernel launch from rocprofv3 PMC counters.

Runs `bench.py` under rocprofv3 three times (FETCH_SIZE and WRITE_SIZE do not fit one pass
on gfx950; a third pass takes SQ instruction counts), then writes per-kernel bytes and
instructions per launch to a JSON file that bench.py reads for `roofline.traffic` and the
VALU-issue utilisation beside it.  Corrections follow MI355X_MICROARCH.md §HBM: FETCH_SIZE on gfx950
tallies 128-B requests at 64 B, so it is doubled; WRITE_SIZE is taken as reported; both
count Infinity-Cache traffic (L2 memory-side requests), so they are an upper bound on
HBM bytes.  rocprofv3 reports both in KiB.

Run it on the GPU box (this process never touches the GPU itself):
    python3 tools/pmc_traffic.py --out gpurun_out/TAG/pmc_traffic.json
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# kernel-name fragments -> bench.py KERNEL_NAMES group (one launch of the group = the sum)
GROUPS = [
    ("sketch_tiles_kernel", "sketch_tiles_kernel"),
    ("merge_kernel", "merge_kernel"),
    ("fp_hash_kernel", "fp_hash_kernel"),
    ("rank_rows_kernel", "candidate compare (rank_rows/walk_cand/compare_grid)"),
    ("walk_cand_kernel", "candidate compare (rank_rows/walk_cand/compare_grid)"),
    ("compare_grid_kernel", "candidate compare (rank_rows/walk_cand/compare_grid)"),
    ("dist_finalize_kernel", "dist finalize (dense / candidate cells)"),
    ("dist_cand_finalize_kernel", "dist finalize (dense / candidate cells)"),
    ("dist_cand_list_kernel", "dist finalize (dense / candidate cells)"),
    ("dist_grid_list_kernel", "dist finalize (dense / candidate cells)"),
    ("qblock_union_kernel", "candidate compare (rank_rows/walk_cand/compare_grid)"),
    ("probe_rows_kernel", "probe_rows_kernel"),
    ("dist_fill_kernel", "dist_fill_kernel"),
    ("dist_fill_flat_kernel", "dist_fill_kernel"),
    ("idx_", "dist index build"),
    ("record_rows_kernel", "dist index build"),
    ("scan_", "dist index build"),
    ("probe_count_kernel", "dist index build"),
    ("sum64_kernel", "dist index build"),
]


def group_of(name: str):
    for frag, g in GROUPS:
        if frag in name:
            return g
    return None


def kernel_key(name: str) -> str:
    """A kernel's short name: 'void fpm::rank_rows_kernel<1024, unsigned short>(...)' ->
    'rank_rows_kernel<1024, unsigned short>'."""
    n = name.split("(")[0].strip()
    for pre in ("void ", "fpm::"):
        n = n.replace(pre, "")
    return n


GROUP_BY = {"fn": group_of}


def run_pass(counter, outdir: str, bench_args: list[str]) -> dict:
    counters = [counter] if isinstance(counter, str) else list(counter)
    cmd = ["rocprofv3", "--pmc"] + counters + ["-d", outdir, "-o", "pmc", "--output-format",
                                               "csv", "--", sys.executable] + bench_args
    env = dict(os.environ, TMPDIR="/tmp")
    with open(os.path.join(outdir + ".log"), "w") as log:
        subprocess.run(cmd, check=True, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT,
                       timeout=600)
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter file under {outdir}")
    per_disp = {c: collections.defaultdict(float) for c in counters}   # (group, dispatch) -> v
    disp = collections.defaultdict(set)                                 # (group, kernel) -> ids
    for row in csv.DictReader(open(files[0])):
        if row["Counter_Name"] not in per_disp:
            continue
        g = GROUP_BY["fn"](row["Kernel_Name"])
        if g is None:
            continue
        per_disp[row["Counter_Name"]][(g, row["Dispatch_Id"])] += float(row["Counter_Value"])
        disp[(g, row["Kernel_Name"])].add(row["Dispatch_Id"])
    # launches of a group = dispatches of its most frequent kernel (each of a group's
    # kernels runs once per bench step: the index build's hist / scans / scatter / buckets)
    launches = collections.defaultdict(int)
    for (g, _k), ids in disp.items():
        launches[g] = max(launches[g], len(ids))
    LAUNCHES.update(launches)
    return per_disp[counter] if isinstance(counter, str) else per_disp


LAUNCHES: dict = {}


def per_launch(per_disp: dict, launches: dict) -> dict:
    tot = collections.defaultdict(float)
    for (g, _), v in per_disp.items():
        tot[g] += v
    return {g: tot[g] * 1024.0 / launches[g] for g in tot if launches.get(g)}


def kernel_times(outdir: str, bench_args: list[str]) -> dict:
    """Average duration (ns) and calls per kernel key from a --kernel-trace --stats pass."""
    cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", outdir, "-o", "kt", "--output-format",
           "csv", "--", sys.executable] + bench_args
    env = dict(os.environ, TMPDIR="/tmp")
    with open(os.path.join(outdir + ".log"), "w") as log:
        subprocess.run(cmd, check=True, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT,
                       timeout=600)
    files = glob.glob(os.path.join(outdir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel trace under {outdir}")
    tot = collections.defaultdict(float)
    calls = collections.defaultdict(int)
    for row in csv.DictReader(open(files[0])):
        k = GROUP_BY["fn"](row["Kernel_Name"])
        if k is None:
            continue
        tot[k] += float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
        calls[k] += 1
    return {k: {"avg_ns": tot[k] / calls[k], "calls": calls[k]} for k in tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc_traffic.json"),
                    help="written under gpurun_out/ on the GPU box; copied into profiles/rNN/ "
                         "in the build container after the pull (tools/collect.py)")
    ap.add_argument("--work", default=os.path.join(ROOT, "gpurun_out", "pmc_traffic"))
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--leg", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2: the bench step, kernels grouped as bench.py reports them; "
                         "c3 / c4 / c5: tools/leg_run.py --leg, per kernel, with durations")
    a = ap.parse_args()
    a.work = a.work + ("" if a.leg == "c2" else "_" + a.leg)
    os.makedirs(a.work, exist_ok=True)
    if a.leg == "c2":
        # the C2 step only: the side legs (-fp text, C3, C4) would add dispatches to the groups
        bench_args = [os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup",
                      str(a.warmup), "--no-cpu-baseline", "--no-fp-text", "--no-c3", "--no-c4",
                      "--no-c5", "--no-cli", "--no-cli-fp", "--no-split", "--no-parity",
                      "--no-full-grid", "--no-gather-check"]
    else:
        bench_args = [os.path.join(ROOT, "tools", "leg_run.py"), "--leg", a.leg]
        if a.leg == "c5":
            # 250 of the 1,000 genomes (per-launch counters of 2.5x fewer tiles; each of the
            # five passes regenerates the genomes on the host)
            bench_args += ["--c5-genomes", "250"]
        GROUP_BY["fn"] = kernel_key
    fetch = run_pass("FETCH_SIZE", os.path.join(a.work, "fetch"), bench_args)
    write = run_pass("WRITE_SIZE", os.path.join(a.work, "write"), bench_args)
    # one "launch" of a group that is several kernels (the index build) is one step's worth
    launches = dict(LAUNCHES)
    sq = run_pass(("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
                   "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"),
                  os.path.join(a.work, "sq"), bench_args)
    sqk = {c: per_launch(v, launches) for c, v in sq.items()}
    # fourth pass: L2 hit / miss requests and LDS bank-conflict cycles
    l2 = run_pass(("SQ_LDS_BANK_CONFLICT", "TCC_HIT_sum", "TCC_MISS_sum"),
                  os.path.join(a.work, "l2"), bench_args)
    l2k = {c: per_launch(v, launches) for c, v in l2.items()}
    f = per_launch(fetch, launches)
    w = per_launch(write, launches)
    res = {}
    for g in sorted(set(f) | set(w)):
        fb = 2.0 * f.get(g, 0.0)          # gfx950: FETCH_SIZE = half the streamed bytes
        wb = w.get(g, 0.0)
        res[g] = {"fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb}
        # SQ counters per launch (per_launch scales by 1024: undo); wave-state split
        sqg = {c.replace("SQ_", "").lower(): v.get(g, 0.0) / 1024.0 for c, v in sqk.items()}
        wc = sqg.get("wave_cycles") or 1.0
        res[g]["sq"] = sqg
        res[g]["wave_state_frac"] = {"active": sqg.get("active_inst_any", 0) / wc,
                                     "issue_stall": sqg.get("wait_inst_any", 0) / wc,
                                     "waiting": sqg.get("wait_any", 0) / wc}
        hit = l2k.get("TCC_HIT_sum", {}).get(g, 0.0) / 1024.0
        miss = l2k.get("TCC_MISS_sum", {}).get(g, 0.0) / 1024.0
        res[g]["l2"] = {"hit_req": hit, "miss_req": miss,
                        "hit_frac": hit / (hit + miss) if hit + miss else None,
                        "lds_bank_conflict_cycles":
                            l2k.get("SQ_LDS_BANK_CONFLICT", {}).get(g, 0.0) / 1024.0}
    if a.leg != "c2":
        kt = kernel_times(os.path.join(a.work, "kt"), bench_args)
        for k, v in res.items():
            t = kt.get(k)
            if not t:
                continue
            v["avg_ns"] = t["avg_ns"]
            v["calls"] = t["calls"]
            secs = t["avg_ns"] * 1e-9
            v["traffic_GBps"] = v["traffic_bytes"] / secs / 1e9 if secs else None
            # wave64 VALU instructions per launch / (launch time x 1024 SIMDs x 2.4 GHz / 2)
            v["valu_issue_frac"] = (v["sq"].get("insts_valu", 0.0) / (secs * 1024 * 2.4e9 / 2)
                                    if secs else None)
    sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
    import fpmash                                   # (reads the .so's build id, no GPU)
    out = {
        "leg": a.leg,
        # the build these counters measured: bench.py drops them from `roofline` when the
        # library it loads carries another id
        "build_id": fpmash.build_id(),
        "command": " ".join(["python3"] + [os.path.relpath(x, ROOT) if x.startswith(ROOT) else x
                                           for x in bench_args]),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                  f"the command above; bytes per launch = "
                  "2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE, KiB x 1024; includes "
                  "Infinity-Cache traffic. A third pass: SQ instruction counts and the "
                  "wave-state split (active / issue-stall / waiting) per launch; a fourth: "
                  "L2 (TCC) hit / miss requests and LDS bank-conflict cycles; side legs add a "
                  "--kernel-trace --stats pass for each kernel's average launch time, the "
                  "achieved traffic rate and the VALU-issue fraction",
        "kernels": res,
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
