#!/bin/bash
# tools/r05_tile_rounds.sh — level-1 index tiles trimmed to whole rounds of 256 (B) against
# fixed 16,384-cell tiles (A, libfpmash_base.so): index / dist tests, then same-box C2 and C4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05ee; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread -k "index or dist or refset or rank or prefill or c4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 bash tools/lib_ab_c2.sh fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3 > $O/c2ab.txt 2>&1 || { cat $O/c2ab.txt; exit 1; }
cut -c1-250 $O/c2ab.txt
timeout -k 10 600 bash tools/lib_ab_leg.sh c4 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 2 > $O/c4ab.txt 2>&1 || { cat $O/c4ab.txt; exit 1; }
cut -c1-250 $O/c4ab.txt
