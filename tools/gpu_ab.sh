#!/bin/bash
# tools/gpu_ab.sh TESTS_K LIB_B [ROUNDS] — one same-box A/B call: the GPU tests selected by
# TESTS_K (pytest -k), then tools/ab_bench.sh of the product library (A) against
# fp-mash_amd/lib/LIB_B.so (B) on the C2 step (BENCH_ARGS overrides the bench flags).
set -o pipefail
cd "$(dirname "$0")/.."
K=${1:?tests -k}; B=${2:?lib}; N=${3:-3}
O=gpurun_out/ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BENCH_ARGS=${BENCH_ARGS:---steps 20 --warmup 3 --no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-full-grid --no-parity} \
  timeout -k 10 900 bash tools/ab_bench.sh fp-mash_amd/lib/libfpmash.so fp-mash_amd/lib/$B.so $N \
  > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
