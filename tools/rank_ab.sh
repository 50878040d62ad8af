#!/bin/bash
# tools/rank_ab.sh NAME... — the C2 step per library build with the sparse dist's fill run
# BEFORE the candidate compare (FPM_FILL_SERIAL=1): per-kernel times without the overlap,
# so the rank kernel is timed alone.  Two rounds; one line per run.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  for n in "$@"; do
    L=$PWD/fp-mash_amd/lib/libfpmash_$n.so; [ "$n" = base ] && L=$PWD/fp-mash_amd/lib/libfpmash.so
    FPM_FILL_SERIAL=1 FPMASH_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-c3 --no-c4 --no-c5 --no-cli --no-fp-text --no-parity > gpurun_out/ra_$n$i.json 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/ra_$n$i.json').read().strip().splitlines()[-1])
print('$n', round(d['ms_per_step'],4), {k[:12]:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
  done
done
