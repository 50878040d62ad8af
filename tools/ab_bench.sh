#!/bin/bash
# tools/ab_bench.sh LIB_A LIB_B [ROUNDS] — alternate bench.py runs over two builds of
# libfpmash.so on the same GPU (box-to-box spread is ~5 %, larger than most kernel changes).
# Prints one line per run: label, ms/step, the legs' numbers, per-kernel averages (from the
# bench's detail file).  BENCH_ARGS overrides the bench flags.
set -o pipefail
A=$1; B=$2; N=${3:-3}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for L in A B; do
    lib=$A; [ "$L" = B ] && lib=$B
    FPMASH_LIB=$lib timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3 --no-cpu-baseline --no-parity} \
      --detail gpurun_out/ab_$L$i.detail.json > gpurun_out/ab_$L$i.json 2>&1 || exit 1
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$L$i.json').read().strip().splitlines()[-1])
e=json.load(open('gpurun_out/ab_$L$i.detail.json'))
print('$L', round(d['ms_per_step'],4), d.get('legs'), {k[:12]:round(v['avg_ms'],3) for k,v in e['kernels'].items()})"
  done
done
