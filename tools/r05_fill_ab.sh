#!/bin/bash
# tools/r05_fill_ab.sh — FPM_FILL_EARLY (the counts fill of a large grid from the start of the
# dist call on a CU-masked stream): parity of the compact dist with the switch on (and the
# side fill forced), then the same-box C4 A/B against the default.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
FPM_FILL_EARLY=8 FPM_FILL_COUNTS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dist_list or refset_mirror or dist_self" > $O/pytest_early.log 2>&1 || { tail -20 $O/pytest_early.log; exit 1; }
tail -1 $O/pytest_early.log
AB_LEG=c4 timeout -k 10 700 bash tools/env_ab.sh FPM_FILL_EARLY=8 FPM_FILL_EARLY=4 > $O/c4ab.txt 2>&1; rc=$?
cat $O/c4ab.txt | cut -c1-400
exit $rc
