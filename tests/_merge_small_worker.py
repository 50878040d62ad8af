"""Run with FPM_MERGE_SMALL=2 (read when libfpmash loads): every merge round on
merge_small_kernel, so lists past its 2,048-entry LDS cap take the global-memory search.
Sketches long multi-tile groups and exits 0 iff they equal the oracle's (test_gpu_parity)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fp-mash_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import fpmash  # noqa: E402
from oracle import oracle as O  # noqa: E402


def rand_seq(rng, n):
    return bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n))


def main():
    assert os.environ.get("FPM_MERGE_SMALL") == "2"
    rng = np.random.default_rng(5)
    recs = [rand_seq(rng, 300_000), rand_seq(rng, 40_000)] + [rand_seq(rng, 30_000) for _ in range(5)]
    groups = [0, 1, 2, 2, 2, 2, 2]
    with fpmash.Context(0) as ctx:
        ctx.merge_small_spills()                     # reset the overflow counter
        for k, s in ((21, 1000), (21, 5000), (16, 3000)):
            got = ctx.sketch(fpmash.make_params(k=k, s=s), recs, groups=groups, n_groups=3)
            exp = O.sketch_batch(O.params(k=k, s=s), recs, groups=groups, n_groups=3)
            for g, e in zip(got, exp):
                if not np.array_equal(np.asarray(g), np.asarray(e)):
                    print("mismatch", k, s, len(g), len(e))
                    return 1
        # s = 5000 lists exceed the 2,048-entry cap: the device counter saw them
        spills = ctx.merge_small_spills()
        if spills == 0:
            print("no LDS overflow counted")
            return 1
    print("ok", spills)
    return 0


if __name__ == "__main__":
    sys.exit(main())
