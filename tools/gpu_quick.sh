#!/bin/bash
# tools/gpu_quick.sh TAG "PYTEST_K" "BENCH_ARGS" [CLI_AB_SETTINGS...] — one GPU-box pass for a
# change under work: the GPU tests matching PYTEST_K (skipped if empty), a bench run with
# BENCH_ARGS (skipped if empty), and the CLI dist A/B of the given env settings (skipped if
# none).  Each step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:?tag}; K=${2:-}; BA=${3:-}; shift 3
cd "$(dirname "$0")/.."
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
if [ -n "$BA" ]; then
  timeout -k 10 600 python bench.py $BA --detail $O/detail.json > $O/bench.json 2> $O/bench.err \
    || { tail -30 $O/bench.err; exit 1; }
  tail -c 1200 $O/bench.json
fi
if [ $# -gt 0 ]; then
  OUT=$O/cli_ab REPS=${REPS:-3} timeout -k 10 400 bash tools/cli_dist_ab.sh "$@" > $O/cli_ab.txt 2>&1 \
    || { tail -30 $O/cli_ab.txt; exit 1; }
  cat $O/cli_ab.txt; cat $O/cli_ab/ph.txt
fi
