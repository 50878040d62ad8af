set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_check.sh r03t && bash tools/profile_round.sh r03t
