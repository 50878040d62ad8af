#!/bin/bash
# tools/r05_prefill_nt.sh — the C4 counts prefill with non-temporal stores (B) against plain
# stores (A), same box; prefill parity with the nt build first.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
FPMASH_LIB=fp-mash_amd/lib/libfpmash_nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prefill" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 700 bash tools/lib_ab_leg.sh c4 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash_nt.so 3 > $O/c4ab.txt 2>&1 || { cat $O/c4ab.txt; exit 1; }
cut -c1-400 $O/c4ab.txt
