set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_check.sh r03u && bash tools/profile_round.sh r03u
