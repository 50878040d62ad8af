set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s13
FPMASH_LIB=$PWD/fp-mash_amd/lib/libfpmash_imgail.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03s13/pytest.log 2>&1 || { tail -40 gpurun_out/r03s13/pytest.log; exit 1; }
tail -1 gpurun_out/r03s13/pytest.log
timeout -k 10 900 bash tools/c3_ab.sh base imgail > gpurun_out/r03s13/c3ab.txt 2>&1 || { tail -5 gpurun_out/r03s13/c3ab.txt; exit 1; }
cat gpurun_out/r03s13/c3ab.txt
