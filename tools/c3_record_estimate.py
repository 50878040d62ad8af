"""tools/c3_record_estimate.py [N] — the record filter on C3-shaped -fp lists, on the CPU: N
(default 1000) lyn2vec-shaped 2 kb sequences -> CFL k-finger text (fpmash.datagen) -> the
oracle's initFromFingerprints lists; reports records per list, the pairs sharing a record
(the candidates of the device's record index), the fraction with numer > 0 on a sample
(oracle literal walk), and the steps the record-stretch walk takes per candidate, checked
against the literal walk on ~3,000 candidates.  A study tool: oracle/ is the checker here."""
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fp-mash_amd")]
from fpmash import datagen  # noqa: E402
from oracle import oracle as O  # noqa: E402


def records(x, S):
    y = np.asarray(x[:S])
    if len(y) == 0:
        return [], []
    pm = np.maximum.accumulate(y)
    p = np.flatnonzero(np.concatenate([[True], pm[1:] > pm[:-1]]))
    return y[p].tolist(), p.tolist()


def stretch_walk(a, b, S):
    """dist.hip walk_pair_rec restated: (numer, denom, literal steps taken)"""
    RA, PA = records(a, S)
    RB, PB = records(b, S)
    la, lb = len(a), len(b)
    common = x = y = steps = 0
    while x < len(RA) and y < len(RB):
        if RA[x] < RB[y]:
            x += 1
        elif RB[y] < RA[x]:
            y += 1
        else:
            i, j = PA[x], PB[y]
            n = i + j - common
            if n >= S:
                break
            ea = PA[x + 1] if x + 1 < len(RA) else la
            eb = PB[y + 1] if y + 1 < len(RB) else lb
            while i < ea and j < eb and n < S:
                if a[i] < b[j]:
                    i += 1
                elif b[j] < a[i]:
                    j += 1
                else:
                    i += 1
                    j += 1
                    common += 1
                n += 1
                steps += 1
            x += 1
            y += 1
    return common, min(S, la + lb - common), steps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    S = 1000
    seqs = datagen.random_dna(n, 2000, seed=33)
    ids = datagen.lyn2vec_ids(n, seed=33)
    lists = []
    for i in range(0, n, 250):
        refs, _, _ = O.fp_references(datagen.cfl_text_fast(seqs[i:i + 250], ids[i:i + 250]))
        lists += [r[2] for r in refs]
    recs = [set(records(x, S)[0]) for x in lists]
    post = defaultdict(list)
    for i, r in enumerate(recs):
        for v in r:
            post[v].append(i)
    cand = sorted({(a, b) for p in post.values() for a in p for b in p})
    rng = np.random.default_rng(0)
    pos = 0
    for _ in range(3000):
        a, b = rng.integers(0, n, 2)
        pos += O.compare(lists[a], lists[b], S, use64=False)[0] > 0
    steps = 0
    sample = cand[::max(1, len(cand) // 3000)]
    for a, b in sample:
        c, d, st = stretch_walk(lists[a], lists[b], S)
        assert (c, d) == tuple(O.compare(lists[a], lists[b], S, use64=False)), (a, b)
        steps += st
    print(f"lists {n}  records/list {np.mean([len(r) for r in recs]):.2f}  "
          f"record events {sum(len(p) ** 2 for p in post.values())}  "
          f"candidates {len(cand) / n / n:.4f} of the pairs  numer>0 {pos / 3000:.4f} (sample)  "
          f"stretch steps/candidate {steps / len(sample):.1f} (exact on {len(sample)})")


if __name__ == "__main__":
    main()
