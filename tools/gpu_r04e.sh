#!/bin/bash
# tools/gpu_r04e.sh — the C3 stretch walk: windowed loads + the diagonal shortcut (A, the
# product) against windowed loads only (libfpmash_win) and neither (libfpmash_w1).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "unsorted or record or fp or refset" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in libfpmash libfpmash_win libfpmash_w1 libfpmash libfpmash_win libfpmash_w1; do
  FPMASH_LIB=fp-mash_amd/lib/$lib.so timeout -k 10 300 python3 tools/leg_run.py --leg c3 > $O/c3_$lib.json 2> $O/c3_$lib.err \
    || { tail -20 $O/c3_$lib.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3_$lib.json').read().strip().splitlines()[-1])
print('$lib', {k: d.get(k) for k in ('dist_ms', 'candidate_pairs', 'counts_equal_dense_walk', 'dense_walk_ms')})"
done
