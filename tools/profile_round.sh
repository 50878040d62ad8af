#!/bin/bash
# tools/profile_round.sh TAG [ROUND] — refresh the committed evidence for one round on the GPU box:
#   1. PMC passes (HBM bytes, SQ instruction counts, L2 / LDS) -> profiles/ROUND/pmc_traffic.json,
#      and per side leg (C3 / C4 / C5, LEGS="c3 c4 c5") -> profiles/ROUND/pmc_<leg>.json
#   2. rocprofv3 --kernel-trace --stats of the C2 bench       -> profiles/ROUND/kernel_stats_TAG.csv
#   3. the full default bench line (CPU baseline, C3, C4, C5, CLI) -> profiles/ROUND/bench_TAG.json
# Each GPU step has its own time limit; the first failure ends the script.  On the GPU box
# only gpurun_out/ travels back: outputs go to gpurun_out/profiles_TAG/, copy them into
# profiles/ROUND/ afterwards (the bench reads the newest profiles/rNN/pmc_traffic.json, so the
# fresh PMC file is also put there for step 3).
set -o pipefail
TAG=${1:?tag}
ROUND=${2:-r03}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/profiles_$TAG
mkdir -p $O profiles/$ROUND
timeout -k 10 900 python3 tools/pmc_traffic.py --out $O/pmc_traffic.json \
  > gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
cp $O/pmc_traffic.json profiles/$ROUND/pmc_traffic.json && echo "pmc ok"
rm -rf gpurun_out/pmc_traffic
# the side legs' kernels (C3 -fp walk, C4 fill / rank / index at 2.5e9 pairs, C5 tiles +
# group select): counters + kernel times per kernel
for leg in ${LEGS:-c3 c4 c5}; do
  timeout -k 10 900 python3 tools/pmc_traffic.py --leg $leg --out $O/pmc_$leg.json \
    > gpurun_out/pmc_${leg}_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_${leg}_$TAG.log; exit 1; }
  cp $O/pmc_$leg.json profiles/$ROUND/pmc_$leg.json && echo "pmc $leg ok"
  rm -rf gpurun_out/pmc_traffic_$leg
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o prof --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check \
  --steps 5 --warmup 2 > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats_$TAG.csv && echo "stats ok"
rm -rf gpurun_out/prof_$TAG
timeout -k 10 400 python3 bench.py > $O/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
  || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 600 $O/bench_$TAG.json
