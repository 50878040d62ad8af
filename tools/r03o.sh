set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03o
timeout -k 10 700 bash tools/ab_bench.sh fp-mash_amd/lib_ab/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3 > gpurun_out/r03o/ab.txt 2>&1 || { tail -5 gpurun_out/r03o/ab.txt; exit 1; }
cat gpurun_out/r03o/ab.txt
timeout -k 10 600 bash tools/env_ab.sh FPM_RANK_WGS=8 FPM_RANK_WGS=6 > gpurun_out/r03o/env_c2.txt 2>&1 || { tail -5 gpurun_out/r03o/env_c2.txt; exit 1; }
cat gpurun_out/r03o/env_c2.txt
AB_LEG=c4 timeout -k 10 600 bash tools/env_ab.sh FPM_RANK_WGS=8 > gpurun_out/r03o/env_c4.txt 2>&1 || { tail -5 gpurun_out/r03o/env_c4.txt; exit 1; }
cat gpurun_out/r03o/env_c4.txt
