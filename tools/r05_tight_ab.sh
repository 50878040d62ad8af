#!/bin/bash
# tools/r05_tight_ab.sh — C5 with tight sample bounds (default) against safe bounds only
# (FPM_TIGHT=0, an A/B build switch), same box.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
AB_LEG=c5 timeout -k 10 700 bash tools/env_ab.sh FPM_TIGHT=0 > $O/c5ab.txt 2>&1; rc=$?
cut -c1-300 $O/c5ab.txt
exit $rc
