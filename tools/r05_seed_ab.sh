#!/bin/bash
# tools/r05_seed_ab.sh — the sketch kernels with the seed pinned once per tile (no per-window
# kernel-argument reload), the redo kernel at 3 waves (no scratch) and the runtime-k
# survivors kernel at 6 waves: sketch parity, then same-box A/B against libfpmash_base.so on
# C5 (k = 21, and k = 17 on 300 genomes: the runtime-k instance) and on the C2 step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sketch" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=fp-mash_amd/lib/libfpmash_base.so; N=fp-mash_amd/lib/libfpmash.so
timeout -k 10 600 bash tools/lib_ab_leg.sh c5 $B $N 3 > $O/c5ab.txt 2>&1 || { cat $O/c5ab.txt; exit 1; }
cut -c1-300 $O/c5ab.txt
LEG_ARGS="--k 17 --c5-genomes 300" timeout -k 10 400 bash tools/lib_ab_leg.sh c5 $B $N 2 > $O/c5k17ab.txt 2>&1 || { cat $O/c5k17ab.txt; exit 1; }
cut -c1-300 $O/c5k17ab.txt
timeout -k 10 500 bash tools/lib_ab_c2.sh $B $N 2 > $O/c2ab.txt 2>&1 || { cat $O/c2ab.txt; exit 1; }
cut -c1-300 $O/c2ab.txt
