#!/bin/bash
# tools/r05_idx_ab2.sh — index tests on the current build, then same-box A/B (base = A) on C2
# and C4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "index or dist or rank or refset or prefill or sorted" > gpurun_out/idx_ab2_tests.txt 2>&1 || { tail -30 gpurun_out/idx_ab2_tests.txt; exit 1; }
tail -2 gpurun_out/idx_ab2_tests.txt
bash tools/lib_ab_c2.sh fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 2 && \
bash tools/lib_ab_leg.sh c4 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 2
