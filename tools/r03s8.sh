set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s8
timeout -k 10 900 bash tools/knobs_ab.sh base ku4 ku12n > gpurun_out/r03s8/knobs.txt 2>&1 || { tail -5 gpurun_out/r03s8/knobs.txt; exit 1; }
cat gpurun_out/r03s8/knobs.txt
