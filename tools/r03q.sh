set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03q
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -k asymptotic -s --timeout 120 --timeout-method thread > gpurun_out/r03q/pytest.log 2>&1
grep PVDIAG gpurun_out/r03q/pytest.log | head -40
