#!/bin/bash
# tools/c3_ab.sh NAME... — same-box A/B of library builds (fp-mash_amd/lib/libfpmash_NAME.so,
# "base" = the product) on the C3 leg (dist -fp 5,000 x 5,000): two rounds, one line per run
# with the leg's dist time and the device parse time.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  for n in "$@"; do
    L=$PWD/fp-mash_amd/lib/libfpmash_$n.so; [ "$n" = base ] && L=$PWD/fp-mash_amd/lib/libfpmash.so
    FPMASH_LIB=$L timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      --no-c4 --no-c5 --no-cli --no-cli-fp --no-fp-text --no-split > gpurun_out/c3ab_$n$i.json 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/c3ab_$n$i.json').read().strip().splitlines()[-1])
c=d['c3_fp']; print('$n', round(c['dist_ms'],3), round(c['parse_device_ms'],3), d['parity']['c3_fp']['ok'])"
  done
done
