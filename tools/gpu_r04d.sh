#!/bin/bash
# tools/gpu_r04d.sh — after dropping the per-row stretch walk and the rank-layout switch: the
# unsorted / record / refset GPU tests, a kernel trace of the C3 leg (record index + stretch
# walk), and the C4 A/B of the count defaults written by the probe (FPM_FILL_COUNTS=0)
# against the side fill beside the rank kernel.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "unsorted or record or fp or refset or rank or self" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o prof --output-format csv \
  -- python3 tools/leg_run.py --leg c3 > $O/prof_c3.log 2>&1 || { tail -20 $O/prof_c3.log; exit 1; }
f=$(find gpurun_out/prof_c3 -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats_c3.csv && rm -rf gpurun_out/prof_c3
python3 - $O/kernel_stats_c3.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f} total_ms {float(r["TotalDurationNs"])/1e6:8.2f}')
PY
AB_LEG=c4 timeout -k 10 600 bash tools/env_ab.sh FPM_FILL_COUNTS=0 > $O/c4_fillcnt_ab.txt 2>&1 \
  || { tail -20 $O/c4_fillcnt_ab.txt; exit 1; }
cat $O/c4_fillcnt_ab.txt
