#!/bin/bash
# tools/pipe_check.sh [ROUNDS] — the C2 bench line with pipelined steps (default) and the
# serial time it reports beside, ROUNDS runs (the parity checks on).
set -o pipefail
cd "$(dirname "$0")/.."
N=${1:-2}
O=gpurun_out/pipe; mkdir -p $O
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp-text --no-c3 \
    --no-c4 --no-c5 --no-cli --no-split --no-full-grid --detail $O/d$i.json > $O/l$i.json 2> $O/e$i.err \
    || { tail -20 $O/e$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/l$i.json').read().strip().splitlines()[-1])
print(round(d['ms_per_step'],4), round(d['config']['serial_ms_per_step'],4), d['parity']['c2'], '%.4g' % d['value'])"
done
