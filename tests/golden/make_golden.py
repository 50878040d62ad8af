#!/usr/bin/env python3
"""Generate the small golden vectors in tests/golden/ (build container only).

Sources of truth, in order of strength:
  * the reference's own hot-path sources compiled unmodified into
    oracle/_ref/libfpmref.so (getHash / getHashFingerPrint hash.cpp:12-73,
    MurmurHash3_x64_128 MurmurHash3.cpp:255-331, MinHashHeap MinHashHeap.cpp:68-146,
    HashSet::toHashList HashSet.cpp:78-118) driven by oracle/ref_driver.cpp;
  * 50-digit mpmath for the binomial upper tail that pValue takes from GSL
    (CommandDistance.cpp:433-450; GSL is not in /root/reference).
The reference's data fixtures copied alongside (DNA*-CFL.txt, *.msh, reads*.fastq.gz,
genomes.dist, test_sequence.*) are listed in tests/golden/README.md.

Run:  make -C oracle && python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

R = O.ref()
if R is None:
    sys.exit("oracle/_ref/libfpmref.so missing: run `make -C oracle` with /root/reference present")


def murmur_kats():
    rng = np.random.default_rng(2024)
    cases = []
    dna = b"ACGT"
    for L in list(range(0, 40)) + [47, 64, 100]:
        for seed in (0, 42, 0xFFFFFFFF, int(rng.integers(0, 2 ** 32))):
            data = bytes(rng.integers(0, 256, size=L, dtype=np.uint8)) if L % 3 else \
                bytes(dna[i] for i in rng.integers(0, 4, size=L))
            h64 = R.ref_get_hash(data, L, seed, 1)
            h32 = R.ref_get_hash(data, L, seed, 0)
            cases.append({"data": data.hex(), "seed": seed, "h64": str(h64), "h32": h32})
    cases.append({"data": b"ACGTACGTACGTACGTACGTA".hex(), "seed": 42,
                  "h64": str(R.ref_get_hash(b"ACGTACGTACGTACGTACGTA", 21, 42, 1)),
                  "h32": R.ref_get_hash(b"ACGTACGTACGTACGTACGTA", 21, 42, 0)})
    return cases


def fp_kats():
    rng = np.random.default_rng(77)
    cases = []
    lines = [[8, 34, 57, 1], [5, 2, 34, 59], [], [0], [2 ** 64 - 1, 1]]
    for _ in range(200):
        n = int(rng.integers(0, 20))
        lines.append([int(x) for x in rng.integers(0, 100, size=n)])
    for v in lines:
        a = np.array(v, dtype=np.uint64)
        p = a.ctypes.data_as(O.u64p)
        cases.append({"vals": [str(x) for x in v], "h32": R.ref_get_hash_fp(p, len(v), 42, 0),
                      "h64": str(R.ref_get_hash_fp(p, len(v), 42, 1))})
    return cases


def sketch_kats():
    """Random records through the reference MinHashHeap + getHash (k-mer walk of
    addMinHashes Sketch.cpp:664-735 re-driven in oracle/ref_driver.cpp)."""
    rng = np.random.default_rng(99)
    out = []
    specs = [(21, 1000, 0, "ACGT"), (21, 50, 0, "ACGT"), (16, 300, 0, "ACGT"),
             (32, 200, 0, "ACGT"), (11, 100, 1, "ACGT"), (9, 100, 1, "ACDEFGHIKLMNPQRSTVWY")]
    for k, s, nonc, alpha in specs:
        P = O.params(k=k, s=s, alphabet=alpha, noncanonical=bool(nonc))
        for t in range(4):
            n_rec = int(rng.integers(1, 4))
            recs = []
            for _ in range(n_rec):
                L = int(rng.integers(0, 3000))
                src = np.frombuffer((alpha + "Nacgt-").encode(), dtype=np.uint8)
                pbad = 0.0 if t == 0 else 0.01
                base = np.frombuffer(alpha.encode(), dtype=np.uint8)[
                    rng.integers(0, len(alpha), size=L)].copy()
                m = rng.random(L) < pbad
                base[m] = src[rng.integers(0, len(src), size=int(m.sum()))]
                recs.append(base.tobytes())
            data, off = O.pack_records(recs)
            hs = np.zeros(s + 1, dtype=np.uint64)
            cs = np.zeros(s + 1, dtype=np.uint32)
            n = R.ref_sketch_records(data, off.ctypes.data_as(O.u64p), len(recs), k, s, 42,
                                     int(P.use64), nonc, 0, bytes(P.alphabet),
                                     hs.ctypes.data_as(O.u64p), cs.ctypes.data_as(O.u32p))
            out.append({"k": k, "s": s, "noncanonical": nonc, "alphabet": alpha,
                        "use64": int(P.use64), "records": [r.decode() for r in recs],
                        "hashes": [str(int(x)) for x in hs[:n]],
                        "counts": [int(x) for x in cs[:n]]})
    return out


def pvalue_table():
    import mpmath as mp
    mp.mp.dps = 50
    rows = []
    rng = np.random.default_rng(5)
    xs = [(41, 1000), (35, 1000), (1, 1000), (1000, 1000), (500, 1000), (2, 10), (1, 1),
          (7, 2000), (150, 10000), (9999, 10000), (3, 5)]
    for _ in range(40):
        n = int(rng.integers(1, 5000))
        xs.append((int(rng.integers(1, n + 1)), n))
    for x, n in xs:
        for r in (1e-12, 3.7e-10, 2.2e-6, 1e-3, 0.05, 0.3, 0.7, 0.99):
            k = x - 1
            # Q(k; r, n) = P(X > k) = I_r(k+1, n-k)
            q = mp.betainc(k + 1, n - k, 0, r, regularized=True)
            rows.append({"x": x, "n": n, "r": r, "q": mp.nstr(q, 30)})
    return rows


def pvalue_asymp_table():
    """GSL's asymptotic regimes of gsl_cdf_beta_P (cdf/beta_inc.c, A&S 26.5.17), reached by
    pValue only when the union size n passed as its sketch size exceeds 1e5 (a = x,
    b = n - x + 1; the regime tests are made in double arithmetic, as GSL makes them):
      b > 1e5, a < 10, r < b/(a+b):  P(a, -N log1p(-r)),  N = b + (a-1)/2
      a > 1e5, b < 10, r > a/(a+b):  Q(b, -N log r),      N = a + (b-1)/2
    and the general regime (the incomplete beta) for the neighbours that miss them.  "q" is
    the branch's formula at 50 digits (what the restatement must reproduce), "exact" the
    regularized incomplete beta itself (how far GSL's approximation sits from it)."""
    import mpmath as mp
    mp.mp.dps = 50
    rows = []

    def row(x, n, r):
        a, b = float(x), float(n - x + 1)
        A, B = mp.mpf(x), mp.mpf(n - x + 1)
        ex = mp.betainc(A, B, 0, r, regularized=True)
        if b > 1e5 and a < 10 and r < b / (a + b):
            branch = "small_a"
            q = mp.gammainc(A, 0, -(B + (A - 1) / 2) * mp.log1p(-mp.mpf(r)), regularized=True)
        elif a > 1e5 and b < 10 and r > a / (a + b):
            branch = "large_a"
            q = mp.gammainc(B, -(A + (B - 1) / 2) * mp.log(mp.mpf(r)), mp.inf, regularized=True)
        else:
            branch, q = "general", ex
        rows.append({"x": x, "n": n, "r": r, "branch": branch, "q": mp.nstr(q, 30),
                     "exact": mp.nstr(ex, 30)})

    for n in (100001, 100009, 150000, 400000, 1000000, 4000000):
        for x in range(1, 11):
            for r in (1e-12, 3.7e-10, 2.2e-6, 1e-5, 1e-4):
                row(x, n, r)
    for n in (100001, 200000, 1000000):
        for j in range(0, 10):
            for r in (1.0 - 1e-7, 1.0 - 1e-6, 1.0 - 2e-6):
                row(n - j, n, r)
    # the incomplete gamma's switch at X = shape + 1: below it the upper Q of the
    # large-a branch is 1 - P from the series, the cancellation is largest where P is; rows
    # with X just below, at and just above the switch, for both branches
    for n in (100001, 1000000):
        for j in range(0, 9):
            x = n - j
            a, b = float(x), float(n - x + 1)
            N = a + (b - 1) / 2
            for X in (b + 1 - 1e-6, b + 0.5, b + 1 + 1e-6):
                row(x, n, float(mp.exp(-mp.mpf(X) / N)))
        for x in range(1, 10):
            a, b = float(x), float(n - x + 1)
            N = b + (a - 1) / 2
            for X in (a + 1 - 1e-6, a + 0.5, a + 1 + 1e-6):
                row(x, n, float(-mp.expm1(-mp.mpf(X) / N)))
    return rows


def main():
    if "--pvalue-asymp" in sys.argv:
        rows = pvalue_asymp_table()
        with open(os.path.join(HERE, "pvalue_asymp.json"), "w") as f:
            json.dump(rows, f, indent=0)
        print({"pvalue_asymp": len(rows)})
        return
    gold = {
        "murmur": murmur_kats(),
        "fp": fp_kats(),
        "sketch": sketch_kats(),
        "pvalue": pvalue_table(),
    }
    with open(os.path.join(HERE, "generated.json"), "w") as f:
        json.dump(gold, f, indent=0)
    print({k: len(v) for k, v in gold.items()})


if __name__ == "__main__":
    main()
