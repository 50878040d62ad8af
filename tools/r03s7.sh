set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s7
FPMASH_LIB=$PWD/fp-mash_amd/lib/libfpmash_both.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multirank.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03s7/pytest.log 2>&1 || { tail -40 gpurun_out/r03s7/pytest.log; exit 1; }
tail -1 gpurun_out/r03s7/pytest.log
timeout -k 10 900 bash tools/knobs_ab.sh base lo32 self both > gpurun_out/r03s7/knobs.txt 2>&1 || { tail -5 gpurun_out/r03s7/knobs.txt; exit 1; }
cat gpurun_out/r03s7/knobs.txt
