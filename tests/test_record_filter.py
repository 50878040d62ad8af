"""The record filter behind the sparse path for unsorted (-fp) lists (dist_index.hip,
record_rows_kernel): the literal walk of compareSketches (CommandDistance.cpp:376-415) counts
an equal pair only at a value that is a record (a strict increase of the running maximum) of
both lists among their first min(len, S) entries, so pairs sharing no record get
(0, min(S, la + lb)).  Checked here on the CPU against the oracle's literal walk; the GPU
tests (test_dist_unsorted_record_*) check the device path built on it."""
import numpy as np
import pytest


def records(x, S):
    x = np.asarray(x)[:S]
    if len(x) == 0:
        return set()
    pm = np.maximum.accumulate(x)
    first = np.concatenate([[True], pm[1:] > pm[:-1]])
    return set(x[first].tolist())


@pytest.mark.parametrize("seed", range(4))
def test_pairs_without_a_shared_record_count_nothing(oracle, seed):
    rng = np.random.default_rng(seed)
    n_cand = n_pos = 0
    for _ in range(1500):
        S = int(rng.choice([1, 3, 10, 64, 300]))
        V = int(rng.choice([2, 5, 40, 2 ** 32]))
        a = rng.integers(0, V, int(rng.integers(0, 200)), dtype=np.uint64).astype(np.uint32)
        b = rng.integers(0, V, int(rng.integers(0, 200)), dtype=np.uint64).astype(np.uint32)
        if rng.random() < 0.3 and len(a) and len(b):
            k = int(rng.integers(1, 1 + min(len(a), len(b), 5)))
            a[:k] = b[:k]
        c, d = oracle.compare(a, b, S, use64=False)
        share = bool(records(a, S) & records(b, S))
        n_cand += share
        n_pos += c > 0
        if not share:
            assert (c, d) == (0, min(S, len(a) + len(b)))
    assert n_pos > 0 and n_cand >= n_pos
