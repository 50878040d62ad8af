set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s6
FPM_PREFILL_GRID=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "prefilled" --timeout 120 --timeout-method thread > gpurun_out/r03s6/pytest.log 2>&1 || { tail -40 gpurun_out/r03s6/pytest.log; exit 1; }
tail -1 gpurun_out/r03s6/pytest.log
timeout -k 10 900 bash tools/env_ab.sh FPM_BENCH_PREFILL=0 FPM_PREFILL_GRID=256,FPM_BENCH_PREFILL=0.45 FPM_PREFILL_GRID=512 FPM_PREFILL_GRID=512,FPM_BENCH_PREFILL=0.5 > gpurun_out/r03s6/env.txt 2>&1 || { tail -5 gpurun_out/r03s6/env.txt; exit 1; }
cat gpurun_out/r03s6/env.txt
