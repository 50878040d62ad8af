set -o pipefail
cd /root/repo
for n in 10000 10240 50000 21876; do echo "n=$n"; timeout -k 5 60 tools/micro/fill_real $n || exit 1; done
