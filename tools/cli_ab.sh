#!/bin/bash
# tools/cli_ab.sh "VAR=VAL[,VAR=VAL]" ... — same-box A/B of environment settings on the CLI
# sketch of bench C2's FASTA (10,000 x 2 kb): each setting ("base" = none) runs REPS times,
# interleaved; one line per setting: median wall and median of each phase / warm-thread step.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/cli_ab}
REPS=${REPS:-5}
mkdir -p "$OUT"
T=$(mktemp -d /dev/shm/fpm_cliab_XXXX)
python3 - "$T/c2.fa" <<'PY' || exit 1
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "fp-mash_amd")]
from fpmash import datagen
seqs = datagen.family_dna(100, 100, 2000, sub_rate=(0.01, 0.10), seed=1000)
open(sys.argv[1], "wb").write(datagen.fasta_bytes(seqs, datagen.lyn2vec_ids(len(seqs))))
PY
EXE=$PWD/fp-mash_amd/bin/fpmash
for i in $(seq 1 "$REPS"); do
  for s in base "$@"; do
    envs=(); [ "$s" != base ] && IFS=',' read -ra envs <<< "$s"
    tag=$(echo "$s" | tr -c 'A-Za-z0-9' '_')
    ( cd "$T" && a=$(date +%s%N) && env "${envs[@]}" FPMASH_TIMING=1 timeout -k 10 60 "$EXE" sketch -i -k 21 -s 1000 -o c2 c2.fa \
        2> "$OLDPWD/$OUT/$tag.$i.txt" && b=$(date +%s%N) && echo "[wall] $(( (b - a) / 1000 ))" >> "$OLDPWD/$OUT/$tag.$i.txt" ) || exit 1
    rm -f "$T/c2.msh"
  done
done
rm -rf "$T"
python3 - "$OUT" base "$@" <<'PY'
import re, statistics, sys, glob
out = sys.argv[1]
for s in sys.argv[2:]:
    tag = re.sub(r"[^A-Za-z0-9]", "_", s + "\n")
    runs = []
    for f in sorted(glob.glob(f"{out}/{tag}.*.txt")):
        t = open(f).read()
        d = {m.group(1): float(m.group(2)) for m in re.finditer(r"\[fpmash(?:-warm)?\] (.*?): ([\d.]+) ms", t)}
        w = re.search(r"\[wall\] (\d+)", t)
        if w: d["wall"] = int(w.group(1)) / 1e3
        runs.append(d)
    keys = [k for k in runs[0] if k not in ("start",)]
    med = {k[:24]: round(statistics.median(r.get(k, 0) for r in runs), 1) for k in keys}
    print(s, "walls", sorted(round(r.get("wall", 0)) for r in runs), med)
PY
