set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s16
timeout -k 10 900 bash tools/env_ab.sh FPM_FILL_FLAT=1 FPM_FILL_COUNTS=1 FPM_FILL_COUNTS=1,FPM_BENCH_PREFILL=0.7 > gpurun_out/r03s16/env.txt 2>&1 || { tail -5 gpurun_out/r03s16/env.txt; exit 1; }
cat gpurun_out/r03s16/env.txt
