set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03n
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multirank.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03n/pytest.log 2>&1 || { tail -30 gpurun_out/r03n/pytest.log; exit 1; }
tail -1 gpurun_out/r03n/pytest.log
timeout -k 10 700 bash tools/ab_bench.sh fp-mash_amd/lib_ab/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3 > gpurun_out/r03n/ab.txt 2>&1 || { tail -5 gpurun_out/r03n/ab.txt; exit 1; }
cat gpurun_out/r03n/ab.txt
