set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03m/pytest.log 2>&1 || { tail -30 gpurun_out/r03m/pytest.log; exit 1; }
tail -1 gpurun_out/r03m/pytest.log
OUT=gpurun_out/r03m/cli REPS=5 timeout -k 10 300 bash tools/cli_ab.sh FPMASH_MSH_WRITE=pwrite || exit 1
