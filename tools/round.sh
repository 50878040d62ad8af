#!/bin/bash
# tools/round.sh TAG [STEP...] — evidence for one build on the GPU box, the first failure ends
# it.  Every output goes under gpurun_out/TAG/ (the only directory that travels back); in the
# build container `python3 tools/collect.py TAG rNN` then copies the files into profiles/rNN/,
# checking that each carries the build id of the local libfpmash.so.
# Steps (default: tests smoke pmc bench rocprof):
#   tests   the -m gpu suite (PYTEST_K selects a subset)
#   smoke   __graft_entry__.smoke()
#   pmc     rocprofv3 PMC passes of the C2 step and the C3 / C4 / C5 legs (LEGS=...):
#           pmc_traffic.json + pmc_<leg>.json, each stamped with the build id
#   bench   the default bench line, reading the counters of this call (--pmc-dir)
#   rocprof rocprofv3 --kernel-trace --stats of the C2 step at the bench's step counts ->
#           kernel_stats.csv, first line "# fpm_build_id=<id>"
#   rehearse N=2 and N=4 ranks of the bench flow on the one GPU (tools/rehearse_ranks.sh)
set -o pipefail
TAG=${1:?tag}; shift
STEPS=${*:-tests smoke pmc bench rocprof}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
C2ONLY="--no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check"
step() { echo "== $1 $(date +%T)"; }
for s in $STEPS; do
  case $s in
  tests)
    step tests
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
    tail -2 $O/pytest.log ;;
  smoke)
    step smoke
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
      || { tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log ;;
  pmc)
    step pmc
    timeout -k 10 900 python3 tools/pmc_traffic.py --out $O/pmc_traffic.json --work $O/pmcw \
      > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
    rm -rf $O/pmcw
    for leg in ${LEGS:-c3 c4 c5}; do
      step pmc_$leg
      timeout -k 10 900 python3 tools/pmc_traffic.py --leg $leg --out $O/pmc_$leg.json \
        --work $O/pmcw > $O/pmc_$leg.log 2>&1 || { tail -20 $O/pmc_$leg.log; exit 1; }
      rm -rf $O/pmcw_$leg
    done ;;
  bench)
    step bench
    pd=""; [ -f $O/pmc_traffic.json ] && pd="--pmc-dir $O"
    timeout -k 10 600 python bench.py $pd ${BENCH_ARGS:-} --detail $O/bench_detail.json \
      > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
    tail -c 3000 $O/bench.json ;;
  rocprof)
    step rocprof
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv \
      -- python3 bench.py $C2ONLY --steps 20 --warmup 5 --detail $O/prof_detail.json \
      > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
    f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
    { echo "# fpm_build_id=$(python3 -c 'import sys; sys.path.insert(0,"fp-mash_amd"); import fpmash; print(fpmash.build_id())') command=bench.py C2 step --steps 20 --warmup 5"; cat "$f"; } > $O/kernel_stats.csv
    head -12 $O/kernel_stats.csv | cut -c1-160
    rm -rf $O/prof ;;
  rehearse)
    for n in 2 4; do
      step rehearse_n$n
      timeout -k 10 700 bash tools/rehearse_ranks.sh $n > $O/rehearse_n$n.txt 2>&1 \
        || { tail -20 $O/rehearse_n$n.txt; exit 1; }
      cp gpurun_out/rehearse.json $O/rehearse_n$n.json; tail -1 $O/rehearse_n$n.txt
    done ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
