set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r03j REPS=5 timeout -k 10 400 bash tools/cli_ab.sh HSA_ENABLE_SDMA=0 GPU_MAX_HW_QUEUES=1 FPM_NO_WARM=1 || exit 1
