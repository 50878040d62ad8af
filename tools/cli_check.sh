#!/bin/bash
# tools/cli_check.sh [ROUNDS] — the CLI GPU tests, then the bench's CLI leg ROUNDS times (C2
# FASTA sketch + 1e8-line dist, oracle-checked): walls and the dist command's phase split.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k cli \
  > gpurun_out/t_cli.log 2>&1 || { tail -20 gpurun_out/t_cli.log; exit 1; }
tail -1 gpurun_out/t_cli.log
for i in $(seq 1 "${1:-2}"); do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp-text --no-c3 \
    --no-c4 --no-c5 --no-split > gpurun_out/cli_$i.json 2> gpurun_out/cli_$i.err \
    || { tail -20 gpurun_out/cli_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cli_$i.json').read().strip().splitlines()[-1]); c=d['cli']
print(round(c['cli_sketch_wall_s'], 3), round(c['cli_dist_wall_s'], 3), c['parity']['ok'],
      {k: round(v, 1) for k, v in c['phases_ms_dist'].items()})"
done
