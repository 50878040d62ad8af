#!/bin/bash
# tools/r05_every_ab.sh — an adaptive sample rate per long group (every E-th tile, E = k-mers
# / 16 s in [16, 64]; C5: 31) against every 16th (libfpmash_base.so), both with tight bounds:
# sketch tests, the C5 leg with its oracle checks, then the same-box C5 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r05x}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sketch" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-cli --no-cli-fp --no-split --no-gather-check --no-full-grid > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('bench c5', d['legs'].get('c5_ms_per_step'), d['parity'])"
timeout -k 10 600 bash tools/lib_ab_leg.sh c5 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3 > $O/c5ab.txt 2>&1 || { cat $O/c5ab.txt; exit 1; }
cut -c1-300 $O/c5ab.txt
