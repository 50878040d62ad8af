#!/bin/bash
# tools/r05_rehearse.sh — the driver's N > 1 bench flow rehearsed on one GPU (N = 2, then 4).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 650 bash tools/rehearse_ranks.sh 2 && cp gpurun_out/rehearse.json gpurun_out/rehearse_n2.json && \
timeout -k 10 650 bash tools/rehearse_ranks.sh 4 && cp gpurun_out/rehearse.json gpurun_out/rehearse_n4.json
