#!/usr/bin/env python3
"""tools/cli_phases.py — wall-time split of the drop-in CLI on the C2 FASTA (GPU box).

Writes config C2's batch (bench.py's generator) as one FASTA, then runs
  fpmash sketch -i -k 21 -s 1000 -o c2 c2.fa      (FPMASH_TIMING=1: per-phase host times)
  fpmash sketch -i ... tiny.fa                    (fixed cost: process + HIP runtime init)
  fpmash dist c2.msh c2.msh > out
and prints each command's wall clock and phase lines.  Output under /dev/shm, removed after.
"""
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
from fpmash import datagen  # noqa: E402

EXE = os.path.join(ROOT, "fp-mash_amd", "bin", "fpmash")


def run(cmd, cwd, stdout=subprocess.DEVNULL):
    env = dict(os.environ, FPMASH_TIMING="1")
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=cwd, env=env, stdout=stdout, stderr=subprocess.PIPE, check=True)
    wall = time.perf_counter() - t0
    print(f"== {' '.join(cmd)}: {wall * 1e3:.1f} ms")
    for line in r.stderr.decode().splitlines():
        if line.startswith("[fpmash]"):
            print("   " + line)
    return wall


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    seqs = datagen.family_dna(100, n // 100, 2000, sub_rate=(0.01, 0.10), seed=2)
    tmp = tempfile.mkdtemp(prefix="fpm_phase_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        ids = datagen.lyn2vec_ids(len(seqs))
        with open(os.path.join(tmp, "c2.fa"), "wb") as f:
            f.write(datagen.fasta_bytes(seqs, ids))
        with open(os.path.join(tmp, "tiny.fa"), "wb") as f:
            f.write(datagen.fasta_bytes(seqs[:2], ids[:2]))
        for _ in range(2):
            run([EXE, "sketch", "-i", "-k", "21", "-s", "1000", "-o", "tiny", "tiny.fa"], tmp)
            run([EXE, "sketch", "-i", "-k", "21", "-s", "1000", "-o", "c2", "c2.fa"], tmp)
        with open(os.path.join(tmp, "out.tsv"), "wb") as f:
            run([EXE, "dist", "c2.msh", "c2.msh"], tmp, stdout=f)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
