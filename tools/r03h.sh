set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03h
timeout -k 10 200 bash tools/cli_trace.sh gpurun_out/r03h/cli || exit 1
find gpurun_out/r03h/cli -name '*.csv' | head -20
