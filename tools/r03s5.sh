set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s5/pytest.log 2>&1 || { tail -40 gpurun_out/r03s5/pytest.log; exit 1; }
tail -1 gpurun_out/r03s5/pytest.log
LEGS=" " bash tools/profile_round.sh r03s5
