#!/bin/bash
# tools/r05_idx_wide.sh — FPM_IDX_WIDE=1 (level 2 split in 2 per partition with 32 KB of counters
# and a 127 KB LDS copy, one workgroup per CU) against the default (4 per partition, 16 KB +
# 64 KB, two per CU): index parity with the switch, then the same-box C4 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
FPM_IDX_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "index or sparse_large" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_LEG=c4 timeout -k 10 700 bash tools/env_ab.sh FPM_IDX_WIDE=1 > $O/c4ab.txt 2>&1; rc=$?
cat $O/c4ab.txt | cut -c1-400
exit $rc
