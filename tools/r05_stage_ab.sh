#!/bin/bash
# tools/r05_stage_ab.sh — a sketch staging variant (B, libfpmash.so) against the previous build
# (A, libfpmash_base.so): sketch tests, then same-box A/Bs on the C2 step and on C5.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r05bb}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sketch or fp" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 bash tools/lib_ab_c2.sh fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3 > $O/c2ab.txt 2>&1 || { cat $O/c2ab.txt; exit 1; }
cut -c1-200 $O/c2ab.txt
timeout -k 10 600 bash tools/lib_ab_leg.sh c5 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 2 > $O/c5ab.txt 2>&1 || { cat $O/c5ab.txt; exit 1; }
cut -c1-200 $O/c5ab.txt
