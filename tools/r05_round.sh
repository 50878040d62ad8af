#!/bin/bash
# tools/r05_round.sh — round-5 evidence on one GPU box, first failure ends it:
#   the C5 A/B of the survivors tile kernel at 8 vs 7 waves (libfpmash_base.so = before),
#   the GPU tests, smoke, the default bench line, rocprofv3 stats of the C2 step and the C2
#   step's PMC traffic.  Outputs under gpurun_out/r05r/ (copied into profiles/r05/ after).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step c5ab
timeout -k 10 420 bash tools/lib_ab_leg.sh c5 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 2 > $O/c5ab.txt 2>&1 || { tail -20 $O/c5ab.txt; exit 1; }
cat $O/c5ab.txt
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
step smoke
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench
timeout -k 10 500 python bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check \
  --steps 5 --warmup 2 --detail $O/prof_detail.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; head -12 $O/kernel_stats.csv | cut -c1-160
step pmc
timeout -k 10 900 python3 tools/pmc_traffic.py --out $O/pmc_traffic.json --work $O/pmcw > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
rm -rf $O/pmcw $O/prof
echo "== done $(date +%T)"
