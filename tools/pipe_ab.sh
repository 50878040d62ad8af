#!/bin/bash
# tools/pipe_ab.sh [ROUNDS] — same-box A/B of the C2 step with and without --pipeline
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in $(seq 1 "${1:-3}"); do
  for m in base pipe; do
    extra=""; [ $m = pipe ] && extra="--pipeline"
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-c4 --no-c5 \
      --no-cli --no-fp-text --no-split --no-parity $extra > gpurun_out/pipe_$m$i.json 2>&1 || { tail -5 gpurun_out/pipe_$m$i.json; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/pipe_$m$i.json').read().strip().splitlines()[-1])
print('$m', round(d['ms_per_step'],4), round(d['value']/1e9,3), 'Gbases/s')"
  done
done
