#!/bin/bash
# tools/cli_trace.sh OUTDIR — where the CLI sketch's wall goes: writes bench C2's FASTA
# (10,000 x 2 kb) to /dev/shm, runs `fpmash sketch -i` 3 times with FPMASH_TIMING=1 (phase
# lines + wall), then once under rocprofv3 --hip-trace --kernel-trace --memory-copy-trace
# (per-call HIP API durations against the phase marks; FPMASH_CLEAN_EXIT=1 so the runtime's
# teardown runs and the tracer writes its files).  No counters are collected.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/cli_trace}
mkdir -p "$OUT"
T=$(mktemp -d /dev/shm/fpm_cli_XXXX)
python3 - "$T/c2.fa" <<'PY' || exit 1
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "fp-mash_amd")]
from fpmash import datagen
seqs = datagen.family_dna(100, 100, 2000, sub_rate=(0.01, 0.10), seed=1000)
open(sys.argv[1], "wb").write(datagen.fasta_bytes(seqs, datagen.lyn2vec_ids(len(seqs))))
PY
EXE=$PWD/fp-mash_amd/bin/fpmash
# CLI_ENV="VAR=VAL ...": extra environment for the untraced runs (A/B)
for i in 1 2 3; do
  ( cd "$T" && s=$(date +%s.%N) && env $CLI_ENV FPMASH_TIMING=1 timeout -k 10 60 "$EXE" sketch -i -k 21 -s 1000 -o c2 c2.fa 2> "$OLDPWD/$OUT/phases_$i.txt" && e=$(date +%s.%N) && echo "wall $(python3 -c "print(round(($e-$s)*1e3,1))") ms" >> "$OLDPWD/$OUT/phases_$i.txt" ) || exit 1
  rm -f "$T/c2.msh"
done
[ -n "$NO_TRACE" ] || ( cd "$T" && FPMASH_CLEAN_EXIT=1 FPMASH_TIMING=1 timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace \
    -d "$OLDPWD/$OUT/trace" -o cli --output-format csv -- "$EXE" sketch -i -k 21 -s 1000 -o c2 c2.fa \
    2> "$OLDPWD/$OUT/phases_traced.txt" ) || exit 1
rm -rf "$T"
grep -h "wall\|device context\|parse\|sketch (\|lists\|msh" "$OUT"/phases_*.txt
