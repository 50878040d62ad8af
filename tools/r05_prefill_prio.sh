#!/bin/bash
# tools/r05_prefill_prio.sh — the C4 counts prefill on a low-priority stream (A/B switch
# FPM_PREFILL_LOWPRIO=1) against the default-priority side stream.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
AB_LEG=c4 timeout -k 10 700 bash tools/env_ab.sh FPM_PREFILL_LOWPRIO=1 > $O/c4ab.txt 2>&1; rc=$?
cut -c1-400 $O/c4ab.txt
exit $rc
