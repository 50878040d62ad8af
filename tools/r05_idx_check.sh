#!/bin/bash
# tools/r05_idx_check.sh — the GPU suite on the current build, then the same-box C4 A/B against
# fp-mash_amd/lib/libfpmash_base.so (the round's previous build), then a short C2 bench line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 700 bash tools/lib_ab_leg.sh c4 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 2 > $O/c4ab.txt 2>&1 || { cat $O/c4ab.txt; exit 1; }
cut -c1-400 $O/c4ab.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-gather-check > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print('c2', d['ms_per_step'], d['parity'])"
