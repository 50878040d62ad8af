#!/bin/bash
# tools/gpu_r04c.sh — C3 through the record index with the per-query-row stretch walk (A)
# against one candidate per lane (B; the bench also times the dense image walk once), the rank kernel on interleaved lanes (A) against adjacent pairs per lane (B), and the CLI dist with one pwritev() per block (default blocks vs 4 M-pair blocks).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "resident_blocks or fp or dist or refset or c4 or record or unsorted" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-split --no-full-grid --no-parity" \
  timeout -k 10 600 bash tools/ab_bench.sh fp-mash_amd/lib/libfpmash.so fp-mash_amd/lib/libfpmash_pair.so 3 \
  > $O/rank_ab.txt 2>&1 || { tail -20 $O/rank_ab.txt; exit 1; }
cat $O/rank_ab.txt
BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-fp-text --no-c4 --no-c5 --no-cli --no-split --no-full-grid --no-parity" \
  timeout -k 10 600 bash tools/ab_bench.sh fp-mash_amd/lib/libfpmash.so fp-mash_amd/lib/libfpmash_cand.so 2 \
  > $O/c3_xcd_ab.txt 2>&1 || { tail -20 $O/c3_xcd_ab.txt; exit 1; }
cat $O/c3_xcd_ab.txt
OUT=$O/cli_ab REPS=3 timeout -k 10 400 bash tools/cli_dist_ab.sh FPMASH_DIST_BLOCK_PAIRS=4000000 > $O/cli_ab.txt 2>&1 \
  || { tail -30 $O/cli_ab.txt; exit 1; }
cat $O/cli_ab.txt
AB_LEG=c4 timeout -k 10 600 bash tools/env_ab.sh FPM_FILL_COUNTS=0 > $O/c4_fillcnt_ab.txt 2>&1 \
  || { tail -20 $O/c4_fillcnt_ab.txt; exit 1; }
cat $O/c4_fillcnt_ab.txt
