set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s4
timeout -k 10 900 bash tools/env_ab.sh FPM_BENCH_PREFILL=0.55 FPM_BENCH_PREFILL=0.65 FPM_BENCH_PREFILL=0.75 FPM_BENCH_PREFILL=0.85 > gpurun_out/r03s4/env.txt 2>&1 || { tail -5 gpurun_out/r03s4/env.txt; exit 1; }
cat gpurun_out/r03s4/env.txt
