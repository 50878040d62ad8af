#!/bin/bash
# tools/knobs_ab.sh NAME... — same-box A/B of several builds of libfpmash.so (compile-time
# knobs such as -DFPM_RANK_GROUP=8, -DFPM_RANK_WAVES=8, -DFPM_IMG_BLK=3), each built beside the
# product as fp-mash_amd/lib/libfpmash_NAME.so ("base" = the product library).  Two rounds of
# the C2 step (20 timed steps each); one line per run: name, ms/step, per-kernel averages.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  for n in "$@"; do
    L=$PWD/fp-mash_amd/lib/libfpmash_$n.so; [ "$n" = base ] && L=$PWD/fp-mash_amd/lib/libfpmash.so
    FPMASH_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-c3 --no-c4 --no-c5 --no-cli --no-fp-text --no-split --no-parity > gpurun_out/kn_$n$i.json 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/kn_$n$i.json').read().strip().splitlines()[-1])
print('$n', round(d['ms_per_step'],4), {k[:12]:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
  done
done
