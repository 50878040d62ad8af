#!/bin/bash
# tools/gpu_r04b.sh — round-4 measurement pass: CLI write-mode A/B, C3 / C4 legs with kernel
# times, C4 rank shares at N = 2 / 4 / 8 (compact output), new GPU tests, the C3 XCD-tile A/B
# (fp-mash_amd/lib/libfpmash_prexcd.so: dist.hip before the change, tools/build_variant.sh).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "resident_blocks or overflow_rebuilds or list or mirror or unsorted or fp" > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp-text --no-c5 \
  --no-cli --no-split --no-full-grid --detail $O/detail.json > $O/bench.json 2> $O/bench.err \
  || { tail -30 $O/bench.err; exit 1; }
tail -c 700 $O/bench.json
for ws in 2 4 8; do
  timeout -k 10 300 python tools/c4_rank_share.py --ws $ws > $O/share_ws$ws.json 2> $O/share_ws$ws.err \
    || { tail -20 $O/share_ws$ws.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/share_ws$ws.json')); print($ws, round(d['rank_step_ms_excl_gather'],3), round(d['dist_ms'],3))"
done
BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-fp-text --no-c4 --no-c5 --no-cli --no-split --no-full-grid --no-parity" \
  timeout -k 10 600 bash tools/ab_bench.sh fp-mash_amd/lib/libfpmash.so fp-mash_amd/lib/libfpmash_prexcd.so 2 \
  > $O/c3_xcd_ab.txt 2>&1 || { tail -20 $O/c3_xcd_ab.txt; exit 1; }
cat $O/c3_xcd_ab.txt
OUT=$O/cli_ab REPS=3 timeout -k 10 400 bash tools/cli_dist_ab.sh FPMASH_DIST_BLOCK_PAIRS=2000000 > $O/cli_ab.txt 2>&1 \
  || { tail -30 $O/cli_ab.txt; exit 1; }
cat $O/cli_ab.txt
