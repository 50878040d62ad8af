#!/bin/bash
# tools/r05_sel_ab.sh — a sketch-kernel variant (B, libfpmash.so) against the previous build
# (A, libfpmash_base.so), both with tight bounds: sketch tests, then the same-box C5 A/B
# (r05w: group_select walking short rows lane-per-row; r05aa: the one-wave path for tiles of
# <= 64 survivors).  AB_OUT names the output directory.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r05w}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sketch" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 bash tools/lib_ab_leg.sh c5 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3 > $O/c5ab.txt 2>&1 || { cat $O/c5ab.txt; exit 1; }
cut -c1-300 $O/c5ab.txt
