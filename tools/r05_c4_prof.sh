#!/bin/bash
# tools/r05_c4_prof.sh — per-kernel stats of the C4 leg alone (with and without the prefill).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o c4 --output-format csv -- python3 tools/leg_run.py --leg c4 --no-prefill > gpurun_out/c4prof.log 2>&1 || { tail -20 gpurun_out/c4prof.log; exit 1; }
f=$(ls gpurun_out/c4prof/*/c4_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/c4prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>4} avg_us {float(r["AverageNs"])/1e3:9.1f}')
PY
