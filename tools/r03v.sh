set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_check.sh r03v && bash tools/profile_round.sh r03v
