set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s2
# prefill beside the sketch kernels, the fill's side stream masked to n CUs
timeout -k 10 900 bash tools/env_ab.sh FPM_BENCH_PREFILL=1 FPM_BENCH_PREFILL=1,FPM_FILL_CUS=32 \
  FPM_BENCH_PREFILL=1,FPM_FILL_CUS=64 FPM_FILL_CUS=64 > gpurun_out/r03s2/env_prefill.txt 2>&1 \
  || { tail -5 gpurun_out/r03s2/env_prefill.txt; exit 1; }
cat gpurun_out/r03s2/env_prefill.txt
