"""-M multiplicities on the GPU (fpm_sketch_mult) vs the oracle's heap counts.

MinHashHeap (MinHashHeap.cpp:68-146, multiplicityMinimum 1) counts every occurrence of a kept
hash from its first one on, except that the final maximum of a full sketch stops counting once
the heap holds exactly the final set (ties with the top are rejected, :73).  The oracle runs
that heap literally (oracle/fpm_oracle.c orc_heap_try_insert) and is pinned to the reference's
own counted sketch, new_data/reads/reads.msh (tests/test_oracle_golden.py).  Counts are
integers: bit-exact.
"""
import numpy as np
import pytest

from conftest import GOLDEN
from test_gpu_parity import rand_seq

pytestmark = pytest.mark.gpu


def check(got, exp):
    gh, gc = got
    eh, ec = exp
    assert len(gh) == len(eh)
    for i in range(len(eh)):
        assert np.array_equal(gh[i], eh[i]), f"sketch {i} hashes differ"
        assert np.array_equal(gc[i], ec[i]), \
            f"sketch {i} counts differ at {np.nonzero(gc[i] != ec[i])[0][:10]}"


@pytest.mark.parametrize("k,s", [(21, 1000), (21, 40), (12, 300), (4, 1000), (21, 1)])
def test_mult_individual(ctx, oracle, k, s):
    """-i: one sketch per record; full and partial sketches, repeats (counts > 1, the maximum
    repeated after the heap fills), N windows, lowercase, u32 hashes (k = 12)."""
    import fpmash
    rng = np.random.default_rng(500 + k + s)
    unit = rand_seq(rng, 97)
    seqs = [rand_seq(rng, 2000), unit * 30, rand_seq(rng, 5000, p_bad=0.01, p_lower=0.2),
            b"ACGT" * 500, rand_seq(rng, 30), b"", rand_seq(rng, 300) * 7,
            rand_seq(rng, 20000), b"A" * 100 + rand_seq(rng, 400) + b"A" * 100]
    P = fpmash.make_params(k=k, s=s)
    O = oracle.params(k=k, s=s)
    check(ctx.sketch(P, seqs, counts=True), oracle.sketch_batch(O, seqs, counts=True))


def test_mult_concatenated_and_long_groups(ctx, oracle):
    """Groups of many records (stream order across records and tiles) and long groups that take
    the sample bound and the group selection: positions run over tiles in stream order."""
    import fpmash
    rng = np.random.default_rng(91)
    unit = rand_seq(rng, 3000)
    mosaic = b"".join(rand_seq(rng, 2000) + unit[:2000] for _ in range(40))
    recs = [rand_seq(rng, 300_000), unit * 50, rand_seq(rng, 150_000, p_bad=0.001)] + \
        [rand_seq(rng, 150) for _ in range(200)] + [mosaic, rand_seq(rng, 60_000) + unit * 3]
    groups = [0, 1, 2] + [3] * 200 + [4, 4]
    for s in (1000, 5000):
        P = fpmash.make_params(k=21, s=s)
        got = ctx.sketch(P, recs, groups=groups, n_groups=5, counts=True)
        exp = oracle.sketch_batch(oracle.params(k=21, s=s), recs, groups=groups, n_groups=5,
                                  counts=True)
        check(got, exp)


def test_mult_reads_fixture(ctx):
    """The reference's own counted sketch: reads.msh (`mash sketch -r -I reads reads1.fastq
    reads2.fastq`, minCov 1: the -M heap) = one sketch of both read files' records, streamed
    alternately (sketchFile's round robin over the open files, Sketch.cpp:1411-1419)."""
    import fpmash
    import mshfmt
    import seqio
    a = [r[2] for r in seqio.read_records(f"{GOLDEN}/reads1.fastq.gz")]
    b = [r[2] for r in seqio.read_records(f"{GOLDEN}/reads2.fastq.gz")]
    recs = [x for pair in zip(a, b) for x in pair]
    exp = mshfmt.read_msh(f"{GOLDEN}/reads.msh")["references"][0]
    P = fpmash.make_params(k=21, s=1000)
    h, c = ctx.sketch(P, recs, groups=[0] * len(recs), n_groups=1, counts=True)
    assert np.array_equal(h[0], exp["hashes64"])
    assert np.array_equal(c[0], exp["counts"])
