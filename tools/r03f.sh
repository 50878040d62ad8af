set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
FPM_CHUNK_KMERS=2048 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mult.py -q -k "long or merge or mult or group" --timeout 120 --timeout-method thread > gpurun_out/r03f/pytest_chunk2048.log 2>&1 || { tail -30 gpurun_out/r03f/pytest_chunk2048.log; exit 1; }
tail -1 gpurun_out/r03f/pytest_chunk2048.log
AB_LEG=c5 timeout -k 10 400 bash tools/env_ab.sh FPM_CHUNK_KMERS=2048 > gpurun_out/r03f/env_ab_c5.txt 2>&1 || { tail -20 gpurun_out/r03f/env_ab_c5.txt; exit 1; }
cat gpurun_out/r03f/env_ab_c5.txt
timeout -k 10 900 python3 tools/pmc_traffic.py --leg c5 --out gpurun_out/r03f/pmc_c5.json > gpurun_out/r03f/pmc_c5.log 2>&1 || { tail -20 gpurun_out/r03f/pmc_c5.log; exit 1; }
echo "pmc c5 ok"
