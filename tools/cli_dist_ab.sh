#!/bin/bash
# tools/cli_dist_ab.sh "VAR=VAL[,VAR=VAL]" ... — same-box A/B of environment settings on the
# CLI `fpmash dist c2.msh c2.msh > out` (1e8 lines) of bench C2's sketches; REPS interleaved
# runs per setting; one line per run: wall, the dist phases and the output's md5.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/cli_dist_ab}
REPS=${REPS:-2}
mkdir -p "$OUT"
T=$(mktemp -d /dev/shm/fpm_cdab_XXXX)
python3 - "$T/c2.fa" <<'PY' || exit 1
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "fp-mash_amd")]
from fpmash import datagen
seqs = datagen.family_dna(100, 100, 2000, sub_rate=(0.01, 0.10), seed=1000)
open(sys.argv[1], "wb").write(datagen.fasta_bytes(seqs, datagen.lyn2vec_ids(len(seqs))))
PY
EXE=$PWD/fp-mash_amd/bin/fpmash
( cd "$T" && timeout -k 10 60 "$EXE" sketch -i -k 21 -s 1000 -o c2 c2.fa 2> /dev/null ) || exit 1
for i in $(seq 1 "$REPS"); do
  for s in base "$@"; do
    envs=(); [ "$s" != base ] && IFS=',' read -ra envs <<< "$s"
    ( cd "$T" && a=$(date +%s%N) && env "${envs[@]}" FPMASH_TIMING=1 timeout -k 10 120 "$EXE" dist -p 16 c2.msh c2.msh > out.tsv \
        2> "$OLDPWD/$OUT/ph.txt" && b=$(date +%s%N) && echo "$s wall_ms $(( (b - a) / 1000000 )) $(grep -oE '(blocks computed|writer [a-z]+|device blocks|reference sketch|rows packed)[^:]*: [0-9.]*' $OLDPWD/$OUT/ph.txt | tr '\n' ' ') md5 $(md5sum < out.tsv | cut -c1-10)" ) || exit 1
    rm -f "$T/out.tsv"
  done
done
rm -rf "$T"
