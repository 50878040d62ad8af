#!/bin/bash
# tools/r05_final.sh TAG — round-5 evidence after the last product change, first failure ends
# it: GPU tests, smoke, PMC passes (C2 step + the C3 / C4 / C5 legs), the default bench line
# (reading those fresh counters), rocprofv3 stats of the C2 step.  Outputs under
# gpurun_out/TAG/ (copied into profiles/r05/ after).
set -o pipefail
TAG=${1:-r05s}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
step smoke
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step pmc
timeout -k 10 900 python3 tools/pmc_traffic.py --out $O/pmc_traffic.json --work $O/pmcw > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
rm -rf $O/pmcw
cp $O/pmc_traffic.json profiles/r05/pmc_traffic.json
for leg in c3 c4 c5; do
  step pmc_$leg
  timeout -k 10 900 python3 tools/pmc_traffic.py --leg $leg --out $O/pmc_$leg.json --work $O/pmcw_$leg > $O/pmc_$leg.log 2>&1 || { tail -20 $O/pmc_$leg.log; exit 1; }
  rm -rf $O/pmcw_$leg
  cp $O/pmc_$leg.json profiles/r05/pmc_$leg.json
done
step bench
timeout -k 10 500 python bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check \
  --steps 5 --warmup 2 --detail $O/prof_detail.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; head -12 $O/kernel_stats.csv | cut -c1-160
rm -rf $O/prof
echo "== done $(date +%T)"
