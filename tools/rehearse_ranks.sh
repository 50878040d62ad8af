#!/bin/bash
# tools/rehearse_ranks.sh [N] — the driver's N-rank bench flow (torch.distributed.run, one
# process per rank) rehearsed on a one-GPU box: every rank on device 0, gathers over gloo
# (FPMASH_BENCH_ONE_DEVICE; RCCL refuses two ranks on one GPU), reduced leg sizes.  Checks
# that main() runs end to end at world size N and prints rank 0's line.
set -o pipefail
cd "$(dirname "$0")/.."
N=${1:-2}
mkdir -p gpurun_out
FPMASH_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$N" \
  --steps 3 --warmup 1 --no-cpu-baseline --no-cli --no-cli-fp --c4-n 6000 --c5-genomes 24 \
  --split-bases 20000000 --detail gpurun_out/rehearse_detail.json \
  > gpurun_out/rehearse.json 2> gpurun_out/rehearse.err || { tail -30 gpurun_out/rehearse.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/rehearse.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['ms_per_step'], d['parity'], d.get('legs'))"
