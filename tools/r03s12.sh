set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s12
timeout -k 10 900 bash tools/env_ab.sh FPM_BENCH_PREFILL_PRIO=low FPM_BENCH_PREFILL_PRIO=high FPM_BENCH_PREFILL_PRIO=low,FPM_BENCH_PREFILL=0.8 > gpurun_out/r03s12/env.txt 2>&1 || { tail -5 gpurun_out/r03s12/env.txt; exit 1; }
cat gpurun_out/r03s12/env.txt
