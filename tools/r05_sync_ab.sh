#!/bin/bash
# tools/r05_sync_ab.sh — sketch GPU tests on the current build, then same-box C5 A/B (base = A).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mult.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sketch or split or merge" > gpurun_out/sync_ab_tests.txt 2>&1 || { tail -30 gpurun_out/sync_ab_tests.txt; exit 1; }
tail -2 gpurun_out/sync_ab_tests.txt
bash tools/lib_ab_leg.sh c5 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3
