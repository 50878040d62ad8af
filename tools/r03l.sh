set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r03l
env | grep -i -E "rocr|hip|hsa|gpu|cuda|omp" | grep -v -i "graft" > gpurun_out/r03l/env.txt
ls /sys/class/kfd/kfd/topology/nodes/ > gpurun_out/r03l/nodes.txt 2>&1
ls -la /dev/dri > gpurun_out/r03l/dri.txt 2>&1
nproc >> gpurun_out/r03l/nodes.txt
for i in 1 2 3 4; do
  timeout -k 5 30 tools/micro/init_par nosecond >> gpurun_out/r03l/init.txt || exit 1
  ROCR_VISIBLE_DEVICES=0 timeout -k 5 30 tools/micro/init_par nosecond | sed 's/^/ROCR0 /' >> gpurun_out/r03l/init.txt || exit 1
  HIP_VISIBLE_DEVICES=0 timeout -k 5 30 tools/micro/init_par nosecond | sed 's/^/HIP0 /' >> gpurun_out/r03l/init.txt || exit 1
done
sort gpurun_out/r03l/init.txt; cat gpurun_out/r03l/env.txt gpurun_out/r03l/nodes.txt
