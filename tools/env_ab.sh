#!/bin/bash
# tools/env_ab.sh "VAR=VAL[,VAR=VAL]" ... — same-box A/B of runtime switches (FPM_FILL_COUNTS,
# FPM_IDX_ONEPASS, ...) on the C2 step: each setting ("base" = none) runs twice, alternating,
# 20 timed steps each; one line per run: setting, ms/step, per-kernel averages.
# AB_LEG=c4: the C4 leg instead (50k-sketch all-vs-all, 3 timed steps), its ms/step;
# AB_LEG=c5: the C5 leg (tools/leg_run.py --leg c5: 1,000 x 5 Mb, one timed step).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  for s in base "$@"; do
    envs=(); [ "$s" != base ] && IFS=',' read -ra envs <<< "$s"
    tag=$(echo "$s" | tr -c 'A-Za-z0-9' '_')
    if [ "${AB_LEG:-c2}" = c5 ]; then
      env "${envs[@]}" timeout -k 10 300 python tools/leg_run.py --leg c5 > gpurun_out/env_$tag$i.json 2>&1 || exit 1
      python3 -c "
import json; d=json.loads(open('gpurun_out/env_$tag$i.json').read().strip().splitlines()[-1])
print('$s', 'c5', round(d['ms_per_step'],3), {k: round(v['ms'],3) for k, v in d['rank0']['kernels'].items()})"
      continue
    fi
    if [ "${AB_LEG:-c2}" = c4 ]; then
      env "${envs[@]}" timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
        --no-c3 --no-c5 --no-cli --no-cli-fp --no-gather-check --no-fp-text --no-split --no-parity --no-full-grid \
        --detail gpurun_out/env_$tag$i.detail.json > gpurun_out/env_$tag$i.json 2>&1 || exit 1
      python3 -c "
import json; d=json.load(open('gpurun_out/env_$tag$i.detail.json'))['c4_dist']
print('$s', 'c4', round(d['ms_per_step'],3), d['phase_ms_rank0'],
      {k[:14]: round(v['ms'], 3) for k, v in d['kernels_rank0'].items()})"
      continue
    fi
    env "${envs[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-fp-text --no-split --no-parity --no-full-grid \
      --detail gpurun_out/env_$tag$i.detail.json > gpurun_out/env_$tag$i.json 2>&1 || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/env_$tag$i.detail.json'))
print('$s', round(d['ms_per_step'],4), {k[:12]:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
  done
done
