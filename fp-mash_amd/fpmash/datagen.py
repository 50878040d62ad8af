"""Synthetic inputs in the formats the reference's configs use.

- DNA FASTA in lyn2vec's `--type generate` shape (dna_utils.py:7-83,
  lyn2vec.py:196-227): header `>T00000XXXXXXXX G00000XXXXXXXX`, 70-column lines,
  GC-biased uniform bases.  Seeded numpy instead of the reference's unseeded
  random.random() so runs are reproducible.
- Family-structured variants (ancestor + members with a substitution rate) so
  that dist has non-trivial shared-hash counts (unrelated random genomes give
  common = 0 for nearly every pair).
- CFL k-finger text (lyn2vec `--type basic --type_factorization CFL`,
  fingerprint_utils.py:95-110, 443-476; factorizations.py:102-126): one line per
  100-char cyclic window, `<Gid>_0 l1 l2 ...` with the Lyndon factor lengths of
  Duval's algorithm.
"""
from __future__ import annotations

import numpy as np

_B = np.frombuffer(b"ACGT", dtype=np.uint8)
_ID_ALPHA = np.frombuffer(b"0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ", dtype=np.uint8)


def random_dna(n, length, gc=0.5, seed=0):
    """n sequences of `length` bases; P(G)=P(C)=gc/2, P(A)=P(T)=(1-gc)/2."""
    rng = np.random.default_rng(seed)
    p = np.array([(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2])
    codes = rng.choice(4, size=(n, length), p=p).astype(np.uint8)
    arr = _B[codes]
    return [arr[i].tobytes() for i in range(n)]


def family_dna(n_families, members, length, sub_rate=(0.01, 0.10), gc=0.5, seed=0):
    """members per family: an ancestor mutated at a per-member substitution rate."""
    rng = np.random.default_rng(seed)
    anc = random_dna(n_families, length, gc, seed + 7919)
    out = []
    for f in range(n_families):
        a = np.frombuffer(anc[f], dtype=np.uint8)
        for _ in range(members):
            rate = rng.uniform(*sub_rate)
            m = a.copy()
            hit = rng.random(length) < rate
            m[hit] = _B[rng.integers(0, 4, size=int(hit.sum()))]
            out.append(m.tobytes())
    return out


def lyn2vec_ids(n, seed=0):
    rng = np.random.default_rng(seed + 104729)
    tails = _ID_ALPHA[rng.integers(0, len(_ID_ALPHA), size=(n, 8))]
    return [t.tobytes().decode() for t in tails]


def fasta_bytes(seqs, ids=None, width=70):
    """lyn2vec-style FASTA: `>T00000<id> G00000<id>` then `width`-column lines."""
    if ids is None:
        ids = lyn2vec_ids(len(seqs))
    parts = []
    for s, i in zip(seqs, ids):
        parts.append(f">T00000{i} G00000{i}\n".encode())
        for o in range(0, len(s), width):
            parts.append(s[o:o + width] + b"\n")
    return b"".join(parts)


def duval_cfl_lengths(word: bytes):
    """Lyndon factor lengths of `word` (Duval; factorizations.py:102-126)."""
    out = []
    n = len(word)
    k = 0
    while k < n:
        i, j = k, k + 1
        while j < n and word[i] <= word[j]:
            i = k if word[i] < word[j] else i + 1
            j += 1
        while k <= i:
            out.append(j - i)
            k += j - i
    return out


def cfl_lines(seq: bytes, gid: str, window=100):
    """k-finger lines of one sequence (fingerprint_utils.py:95-110, 443-476)."""
    s = seq.upper()
    lines = []
    if len(s) < window:
        shifts = [s]
    else:
        ss = s + s[:window]
        shifts = [ss[i:i + window] for i in range(len(s))]
    for w in shifts:
        lines.append(f"{gid}_0 " + " ".join(str(x) for x in duval_cfl_lengths(w)) + "\n")
    return lines


def cfl_text(seqs, ids, window=100):
    return "".join(l for s, i in zip(seqs, ids) for l in cfl_lines(s, "G00000" + i, window)).encode()


def cfl_text_fast(seqs, ids, window=100, threads=None):
    """cfl_text through the C++ generator (bin/cflgen, same bytes): C3-scale inputs
    (5,000 x 2 kb -> 10 M lines) in seconds instead of minutes."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin", "cflgen")
    inp = b"".join(i.encode() + b"\t" + s + b"\n" for s, i in zip(seqs, ids))
    args = [exe, str(window)] + ([str(threads)] if threads else [])
    return subprocess.run(args, input=inp, stdout=subprocess.PIPE, check=True).stdout
