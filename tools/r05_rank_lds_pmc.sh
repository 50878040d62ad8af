#!/bin/bash
# tools/r05_rank_lds_pmc.sh — one PMC pass over the C2 step: LDS array cycles, bank conflicts,
# LDS issue stalls and instruction counts of the rank and probe kernels (per launch).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/rank_lds; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS -d $O -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check --steps 3 --warmup 1 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    k = "rank" if "rank_rows" in k else "probe" if "probe_rows" in k else "sketch" if "sketch_tiles" in k else None
    if not k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for k, d in acc.items():
    n = len(disp[k]); print(k, n, {c: round(v / n / 1e6, 2) for c, v in sorted(d.items())}, "(M per launch)")
PY
