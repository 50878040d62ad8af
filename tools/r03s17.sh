set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s17
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s17/pytest.log 2>&1 || { tail -40 gpurun_out/r03s17/pytest.log; exit 1; }
tail -1 gpurun_out/r03s17/pytest.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
