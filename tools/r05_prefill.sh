#!/bin/bash
# tools/r05_prefill.sh — the counts prefill beside the sketch (fpm_dist_list_prefill): dist
# parity on the GPU, then same-box A/Bs with and without it (C2 step, C4 leg), then one bench
# run of C2 + C4 with parity on.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prefill or dist_list or refset or index or dist_self or sparse_large or rank" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
LEGS="--no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check --steps 20"
for i in 1 2; do
  for v in base pre; do
    flag=""; [ $v = base ] && flag="--no-prefill"
    timeout -k 10 300 python bench.py $LEGS $flag > $O/c2_$v$i.json 2> $O/c2_$v$i.err || { tail -20 $O/c2_$v$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/bench_detail.json'))
print('$v', 'c2', round(d['ms_per_step'], 4), {k[:16]: round(v['avg_ms'], 4) for k, v in d['kernels'].items()})" | tee -a $O/ab.txt
  done
done
for i in 1 2; do
  for v in base pre; do
    flag=""; [ $v = base ] && flag="--no-prefill"
    timeout -k 10 300 python tools/leg_run.py --leg c4 $flag > $O/c4_$v$i.json 2>&1 || { tail -20 $O/c4_$v$i.json; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c4_$v$i.json').read().strip().splitlines()[-1])
k=d.get('rank0', {}).get('kernels') or d.get('kernels_rank0') or {}
print('$v', 'c4', round(d['ms_per_step'], 3), {n[:16]: round(v.get('ms', 0), 3) for n, v in k.items()})" | tee -a $O/ab.txt
  done
done
timeout -k 10 600 python bench.py --no-cpu-baseline --no-fp-text --no-c3 --no-c5 --no-cli --no-cli-fp --no-split --no-gather-check > $O/bench_c2c4.json 2> $O/bench_c2c4.err || { tail -20 $O/bench_c2c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c2c4.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['legs'].get('c4_ms_per_step'), d['parity'])"
