#!/bin/bash
# tools/lib_ab_leg.sh LEG LIB_A LIB_B [ROUNDS] — same-box A/B of two builds of libfpmash.so on
# one side leg (tools/leg_run.py --leg c3|c4|c5 $LEG_ARGS), alternating; one line per run: label,
# ms/step and the leg's per-kernel milliseconds.
set -o pipefail
LEG=${1:?leg}; A=${2:?lib A}; B=${3:?lib B}; N=${4:-2}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for L in A B; do
    lib=$A; [ "$L" = B ] && lib=$B
    FPMASH_LIB=$lib timeout -k 10 300 python tools/leg_run.py --leg "$LEG" $LEG_ARGS > gpurun_out/lab_$L$i.json 2>&1 || { tail -5 gpurun_out/lab_$L$i.json; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/lab_$L$i.json').read().strip().splitlines()[-1])
k=d.get('rank0', {}).get('kernels') or d.get('kernels_rank0') or {}
print('$L', '$LEG', round(d.get('ms_per_step', d.get('dist_ms', 0)), 3), {n[:16]: round(v.get('ms', 0), 3) for n, v in k.items()})"
  done
done
