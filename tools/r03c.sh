set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 400 python -u -m pytest tests/ -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03c/pytest.log 2>&1 || { tail -30 gpurun_out/r03c/pytest.log; exit 1; }
tail -2 gpurun_out/r03c/pytest.log
timeout -k 10 60 ./tools/micro/fp_clock > gpurun_out/r03c/fp_clock.log 2>&1 || { tail -20 gpurun_out/r03c/fp_clock.log; exit 1; }
head -45 gpurun_out/r03c/fp_clock.log
timeout -k 10 400 bash tools/env_ab.sh FPM_IDX_ONEPASS=0 > gpurun_out/r03c/env_ab_c2.txt 2>&1 || { tail -20 gpurun_out/r03c/env_ab_c2.txt; exit 1; }
cat gpurun_out/r03c/env_ab_c2.txt
