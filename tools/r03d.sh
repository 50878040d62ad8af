set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03d
for i in 1 2 3; do
  for d in 1 0; do
    FPM_PAGEABLE_DIRECT=$d timeout -k 10 60 ./tools/micro/fp_clock > gpurun_out/r03d/fp_clock_d${d}_$i.log 2>&1 || { tail -5 gpurun_out/r03d/fp_clock_d${d}_$i.log; exit 1; }
    grep SUMMARY gpurun_out/r03d/fp_clock_d${d}_$i.log
  done
done
for d in 1 0; do
  FPM_PAGEABLE_DIRECT=$d timeout -k 10 120 python tools/micro/fp_stall.py > gpurun_out/r03d/fp_stall_d$d.log 2>&1 || { tail -5 gpurun_out/r03d/fp_stall_d$d.log; exit 1; }
  echo "fp_stall direct=$d: max events $(awk '{print $5}' gpurun_out/r03d/fp_stall_d$d.log | sort -n | tail -1) ms"
done
