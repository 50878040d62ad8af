set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03t
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03t/prof -o ws8 --output-format csv -- python3 tools/c4_rank_share.py --ws 8 --steps 5 > gpurun_out/r03t/ws8.json 2> gpurun_out/r03t/ws8.err || { tail -5 gpurun_out/r03t/ws8.err; exit 1; }
f=$(find gpurun_out/r03t/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.1f} us {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
