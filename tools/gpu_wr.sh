#!/bin/bash
# tools/gpu_wr.sh — output-path measurements on the GPU box: the write-rate micro benchmark
# (tools/micro/write_rate, 4 GB into /dev/shm by pwrite / mmap variants), then the CLI dist
# A/B of the write modes (tools/cli_dist_ab.sh), then the compact-list GPU tests and a short
# C2 bench.  Each step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
{ nproc; uname -r; cat /sys/kernel/mm/transparent_hugepage/shmem_enabled; df -h /dev/shm; } > gpurun_out/wr.txt 2>&1
timeout -k 10 120 tools/micro/write_rate /dev/shm/fpm_wr 4096 16 >> gpurun_out/wr.txt 2>&1 &&
timeout -k 10 120 tools/micro/write_rate /dev/shm/fpm_wr 4096 8 >> gpurun_out/wr.txt 2>&1 &&
REPS=3 timeout -k 10 400 bash tools/cli_dist_ab.sh FPMASH_DIST_BLOCK_PAIRS=2000000 > gpurun_out/cli_ab.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "list or mirror" > gpurun_out/t_list.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp-text --no-c3 --no-c5 --no-cli --no-split > gpurun_out/b_c2c4.json 2> gpurun_out/b_c2c4.err
rc=$?
cat gpurun_out/wr.txt gpurun_out/cli_ab.txt; tail -2 gpurun_out/t_list.log; tail -c 1500 gpurun_out/b_c2c4.json
exit $rc
