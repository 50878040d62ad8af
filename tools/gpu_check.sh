#!/bin/bash
# tools/gpu_check.sh [TAG] — the round-end sequence on one GPU box: gpu tests, smoke, bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-check}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
tail -1 gpurun_out/${TAG}_bench.json
