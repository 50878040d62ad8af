#!/bin/bash
# tools/r05_tile_ab.sh — level-1 index tiles of 8,192 cells (64 KB staging, 2 workgroups per
# CU) against 16,384 (128 KB, one per CU): index parity, then same-box C4 and C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "index or dist_list or refset or sparse_large or dist_self" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 700 bash tools/lib_ab_leg.sh c4 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash_t8k.so 2 > $O/c4ab.txt 2>&1 || { cat $O/c4ab.txt; exit 1; }
cut -c1-400 $O/c4ab.txt
timeout -k 10 700 bash tools/lib_ab_c2.sh fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash_t8k.so 2 > $O/c2ab.txt 2>&1 || { cat $O/c2ab.txt; exit 1; }
cut -c1-400 $O/c2ab.txt
