#!/bin/bash
# tools/r05_rank_ab.sh [ROUNDS] — dist parity tests on the current build, then same-box C2 A/B
# of lib/libfpmash_base.so (A) against lib/libfpmash.so (B).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dist or rank or sorted or refset or index" > gpurun_out/rank_ab_tests.txt 2>&1 || { tail -30 gpurun_out/rank_ab_tests.txt; exit 1; }
tail -3 gpurun_out/rank_ab_tests.txt
bash tools/lib_ab_c2.sh fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so ${1:-3}
