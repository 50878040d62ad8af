set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s9
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multirank.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03s9/pytest_base.log 2>&1 || { tail -40 gpurun_out/r03s9/pytest_base.log; exit 1; }
tail -1 gpurun_out/r03s9/pytest_base.log
FPM_RANK_PARTS=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multirank.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03s9/pytest_p4.log 2>&1 || { tail -40 gpurun_out/r03s9/pytest_p4.log; exit 1; }
tail -1 gpurun_out/r03s9/pytest_p4.log
timeout -k 10 900 bash tools/env_ab.sh FPM_RANK_PARTS=2 FPM_RANK_PARTS=4 FPM_RANK_PARTS=8 FPM_RANK_PARTS=4,FPM_BENCH_PREFILL=1 > gpurun_out/r03s9/env.txt 2>&1 || { tail -5 gpurun_out/r03s9/env.txt; exit 1; }
cat gpurun_out/r03s9/env.txt
