set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "prefilled" --timeout 120 --timeout-method thread > gpurun_out/r03s3/pytest.log 2>&1 || { tail -40 gpurun_out/r03s3/pytest.log; exit 1; }
tail -1 gpurun_out/r03s3/pytest.log
timeout -k 10 900 bash tools/env_ab.sh FPM_BENCH_PREFILL=0.3 FPM_BENCH_PREFILL=0.45 FPM_BENCH_PREFILL=0.6 FPM_BENCH_PREFILL=1 > gpurun_out/r03s3/env.txt 2>&1 || { tail -5 gpurun_out/r03s3/env.txt; exit 1; }
cat gpurun_out/r03s3/env.txt
