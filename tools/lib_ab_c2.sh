#!/bin/bash
# tools/lib_ab_c2.sh LIB_A LIB_B [ROUNDS] — same-box A/B of two builds of libfpmash.so on the C2
# step (bench.py, legs off, 20 timed steps), alternating; one line per run: label, ms/step and
# the per-kernel averages.
set -o pipefail
A=${1:?lib A}; B=${2:?lib B}; N=${3:-2}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for L in A B; do
    lib=$A; [ "$L" = B ] && lib=$B
    FPMASH_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check --steps 20 > gpurun_out/c2ab_$L$i.json 2>gpurun_out/c2ab_$L$i.err || { tail -5 gpurun_out/c2ab_$L$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/bench_detail.json'))
print('$L', 'c2', round(d['ms_per_step'], 4), {k[:16]: round(v.get('avg_ms', v.get('ms', 0)) if isinstance(v, dict) else v, 4) for k, v in d.get('kernels', {}).items()})"
  done
done
