#!/bin/bash
# tools/gpu_c3ab.sh LIB_B [ROUNDS] — the unsorted / record GPU tests, then the C3 leg
# (tools/leg_run.py --leg c3) alternating the product library (A) and fp-mash_amd/lib/LIB_B.so.
set -o pipefail
cd "$(dirname "$0")/.."
B=${1:?lib}; N=${2:-2}
O=gpurun_out/c3ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "unsorted or record or fp or c3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in $(seq 1 "$N"); do
  for L in A B; do
    lib=fp-mash_amd/lib/libfpmash.so; [ "$L" = B ] && lib=fp-mash_amd/lib/$B.so
    FPMASH_LIB=$lib timeout -k 10 300 python3 tools/leg_run.py --leg c3 > $O/c3_$L$i.json 2> $O/c3_$L$i.err \
      || { tail -20 $O/c3_$L$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c3_$L$i.json').read().strip().splitlines()[-1])
print('$L', {k: d.get(k) for k in ('dist_ms', 'candidate_pairs', 'counts_equal_dense_walk')})"
  done
done
