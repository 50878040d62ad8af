#!/bin/bash
# tools/r05_idx_ab.sh — the split level-2 index pass: index / dist parity on the GPU, then the
# same-box C4 A/B against the previous build (fp-mash_amd/lib/libfpmash_base.so).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "index or dist_list or refset or sparse_large or dist_self" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 700 bash tools/lib_ab_leg.sh c4 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3 > $O/c4ab.txt 2>&1; rc=$?
cat $O/c4ab.txt | cut -c1-400
exit $rc
