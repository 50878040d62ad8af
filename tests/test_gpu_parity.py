"""GPU parity: the gfx950 kernels (through the C ABI) vs the CPU oracle.

Integer outputs (hashes, sketch sets, shared-hash counts) must be bit-exact.
Distance and p-value: relative tolerance 1e-12 (BASELINE.json north_star).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

RTOL = 1e-12


def rand_seq(rng, n, p_bad=0.0, p_lower=0.0, alphabet=b"ACGT"):
    a = np.frombuffer(alphabet, dtype=np.uint8)
    s = a[rng.integers(0, len(a), size=n)].copy()
    if p_bad:
        m = rng.random(n) < p_bad
        s[m] = np.frombuffer(b"NRY-*", dtype=np.uint8)[rng.integers(0, 5, size=int(m.sum()))]
    if p_lower:
        m = (rng.random(n) < p_lower) & (s >= 65) & (s <= 90)
        s[m] += 32
    return s.tobytes()


def check_sketches(got, exp):
    assert len(got) == len(exp)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert len(g) == len(e), f"sketch {i}: {len(g)} vs {len(e)} hashes"
        assert np.array_equal(g, e), f"sketch {i} differs"


@pytest.mark.parametrize("k,s,canon", [(21, 1000, True), (21, 1000, False), (16, 200, True),
                                       (32, 500, True), (9, 50, True), (1, 10, False),
                                       (27, 5000, True)])
def test_sketch_individual(ctx, oracle, k, s, canon):
    import fpmash
    rng = np.random.default_rng(1000 + k + s)
    lens = [0, 1, k - 1, k, k + 1, 50, 300, 1000, 1980, 2000, 2100, 4000, 5000, 9000, 20000]
    seqs = [rand_seq(rng, L, p_bad=0.01 if i % 3 == 0 else 0.0, p_lower=0.2 if i % 4 == 1 else 0.0)
            for i, L in enumerate(lens)]
    P = fpmash.make_params(k=k, s=s, noncanonical=not canon)
    O = oracle.params(k=k, s=s, noncanonical=not canon)
    assert P.use64 == O.use64
    got = ctx.sketch(P, seqs)
    exp = oracle.sketch_batch(O, seqs)
    check_sketches(got, exp)


def test_sketch_low_complexity(ctx, oracle):
    """Repeats and palindromes: duplicates and canonical ties."""
    import fpmash
    rng = np.random.default_rng(77)
    seqs = [b"A" * 3000, b"ACGT" * 700, b"AC" * 1500, b"ACGTTGCA" * 300, b"N" * 100,
            b"acgtNNNNacgtacgtacgtacgtacgtacgt" * 40,
            # repeats of a random unit: every hash 4-14 times (crowded, sortable buckets)
            rand_seq(rng, 150) * 14, rand_seq(rng, 600) * 4, rand_seq(rng, 37) * 60]
    for k, s in [(21, 1000), (21, 3), (4, 1000)]:
        P = fpmash.make_params(k=k, s=s)
        got = ctx.sketch(P, seqs)
        exp = oracle.sketch_batch(oracle.params(k=k, s=s), seqs)
        check_sketches(got, exp)


def test_sketch_concatenated_groups(ctx, oracle):
    """Default (non -i) mode: one sketch per group of records, incl. chunked long records
    and many short records packed per tile (sketchFile Sketch.cpp:1354-1422)."""
    import fpmash
    rng = np.random.default_rng(7)
    seqs, groups = [], []
    plan = [(0, [150] * 300), (1, [60000]), (2, [5] * 10), (3, [2000, 30000, 100, 7000]),
            (4, [20] * 40 + [22] * 5), (5, [])]
    for g, lens in plan:
        for L in lens:
            seqs.append(rand_seq(rng, L, p_bad=0.002))
            groups.append(g)
    for k, s in [(21, 1000), (15, 3000)]:
        P = fpmash.make_params(k=k, s=s)
        got = ctx.sketch(P, seqs, groups=groups, n_groups=6)
        exp = oracle.sketch_batch(oracle.params(k=k, s=s), seqs, groups=groups, n_groups=6)
        check_sketches(got, exp)


def test_sketch_seed_and_case(ctx, oracle):
    import fpmash
    rng = np.random.default_rng(3)
    seqs = [rand_seq(rng, 1500, p_lower=0.5) for _ in range(20)]
    for seed in (0, 1, 42, 0xFFFFFFFF):
        for pc in (False, True):
            P = fpmash.make_params(k=21, s=400, seed=seed, preserve_case=pc)
            O = oracle.params(k=21, s=400, seed=seed, preserve_case=pc)
            check_sketches(ctx.sketch(P, seqs), oracle.sketch_batch(O, seqs))


def test_sketch_protein_alphabet(ctx, oracle):
    import fpmash
    rng = np.random.default_rng(11)
    seqs = [rand_seq(rng, 800, alphabet=b"ACDEFGHIKLMNPQRSTVWYBXZ") for _ in range(10)]
    P = fpmash.make_params(k=9, s=300, protein=True)
    O = oracle.params(k=9, s=300, alphabet=fpmash.ALPHABET_PROTEIN, noncanonical=True)
    check_sketches(ctx.sketch(P, seqs), oracle.sketch_batch(O, seqs))


def test_fp_hash_lines(ctx, oracle):
    rng = np.random.default_rng(5)
    lines = [rng.integers(0, 2 ** 63, size=rng.integers(0, 40), dtype=np.uint64)
             for _ in range(5000)]
    lines += [np.array([8, 34, 57, 1], dtype=np.uint64), np.zeros(0, np.uint64)]
    for use64 in (False, True):
        for seed in (42, 7):
            got = ctx.fp_hash_lines(lines, seed=seed, use64=use64)
            exp = np.array([oracle.get_hash_fp(v, seed, use64) for v in lines],
                           dtype=np.uint64 if use64 else np.uint32)
            assert np.array_equal(got, exp)
    assert int(ctx.fp_hash_lines([[8, 34, 57, 1]])[0]) == 819737709


def _family_sketches(oracle, n_fam=6, members=8, L=2000, k=21, s=1000, seed=0):
    import fpmash.datagen as D
    seqs = D.family_dna(n_fam, members, L, sub_rate=(0.0, 0.08), seed=seed)
    sk = oracle.sketch_batch(oracle.params(k=k, s=s), seqs)
    return seqs, sk


@pytest.fixture(params=["auto", "dense", "sparse"])
def dist_mode(request, ctx):
    import fpmash
    ctx.set_dist_mode({"auto": fpmash.DIST_AUTO, "dense": fpmash.DIST_DENSE,
                       "sparse": fpmash.DIST_SPARSE}[request.param])
    yield request.param
    ctx.set_dist_mode(fpmash.DIST_AUTO)


def test_dist_sorted_u64(ctx, oracle, dist_mode):
    seqs, sk = _family_sketches(oracle)
    lengths = [len(x) for x in seqs]
    # uneven sketch sizes, empty lists, truncated sketch size
    sk = sk + [sk[0][:10], np.zeros(0, np.uint64), sk[3][:999]]
    lengths = lengths + [lengths[0], 100, lengths[3]]
    for S in (1000, 500, 37):
        got = ctx.dist(sk, sk[:20], S, use64=True, k=21, ref_lengths=lengths,
                       qry_lengths=lengths[:20])
        nu, de, di, pv = oracle.dist_grid(sk, lengths, sk[:20], lengths[:20], S, 21, 4.0 ** 21)
        assert np.array_equal(got["numer"], nu)
        assert np.array_equal(got["denom"], de)
        np.testing.assert_allclose(got["distance"], di, rtol=RTOL, atol=0)
        np.testing.assert_allclose(got["pvalue"], pv, rtol=RTOL, atol=0)
    assert (got["numer"] > 0).any()


def test_dist_unsorted_u32_fp(ctx, oracle, dist_mode):
    """-fp lists: file-order u32 hashes with duplicates, walked literally."""
    rng = np.random.default_rng(9)
    base = rng.integers(0, 2 ** 32, size=3000, dtype=np.uint64).astype(np.uint32)
    lists = []
    for i in range(40):
        n = int(rng.integers(0, 2100))
        idx = rng.integers(0, 3000 if i % 2 else 200, size=n)
        lists.append(base[idx])
    lengths = [int(rng.integers(1, 20000)) for _ in lists]
    for S in (1000, 2000, 5):
        got = ctx.dist(lists, lists, S, use64=False, k=1, kmer_space=10.0, ref_lengths=lengths,
                       qry_lengths=lengths)
        nu, de, di, pv = oracle.dist_grid(lists, lengths, lists, lengths, S, 1, 10.0, use64=False)
        assert np.array_equal(got["numer"], nu)
        assert np.array_equal(got["denom"], de)
        np.testing.assert_allclose(got["distance"], di, rtol=RTOL, atol=0)
        np.testing.assert_allclose(got["pvalue"], pv, rtol=RTOL, atol=0)


def _skewed_fp_lists(rng, base, n, heavy=4, max_len=2100):
    """CFL-like -fp lists: a few values repeated hundreds of times in most lists (the
    "100" k-finger), the rest drawn from a large vocabulary, in file order."""
    hv = base[:heavy]
    lists = []
    for i in range(n):
        m = int(rng.integers(0, max_len))
        fam = int(rng.integers(0, 40))
        pool = base[heavy + fam * 400: heavy + fam * 400 + 400]
        x = np.where(rng.random(m) < 0.3, hv[rng.integers(0, heavy, size=m)],
                     pool[rng.integers(0, len(pool), size=m)])
        if i % 7 == 0:          # some lists without the heavy values
            x = pool[rng.integers(0, len(pool), size=m)]
        lists.append(x.astype(np.uint32))
    return lists


@pytest.mark.parametrize("mode", ["auto", "sparse"])
def test_dist_unsorted_record_index(ctx, oracle, mode):
    """Unsorted lists with heavily repeated values: the index is rebuilt over each row's
    records (the strict increases of its running maximum among its first min(len, S)
    entries) and the pairs sharing a record are walked on the original lists.  Self set and
    a separate query set, against the literal-walk oracle."""
    import fpmash
    rng = np.random.default_rng(77)
    base = rng.integers(0, 2 ** 32, size=20000, dtype=np.uint64).astype(np.uint32)
    refs = _skewed_fp_lists(rng, base, 90)
    qrys = _skewed_fp_lists(rng, base, 70)
    rl = [int(rng.integers(1, 20000)) for _ in refs]
    ql = [int(rng.integers(1, 20000)) for _ in qrys]
    ctx.set_dist_mode(fpmash.DIST_SPARSE if mode == "sparse" else fpmash.DIST_AUTO)
    try:
        for S in (1000, 2000, 64):
            for (a, al), (b, bl) in (((refs, rl), (refs, rl)), ((refs, rl), (qrys, ql))):
                got = ctx.dist(a, b, S, use64=False, k=1, kmer_space=10.0, ref_lengths=al,
                               qry_lengths=bl)
                st = ctx.last_dist_stats()
                nu, de, di, pv = oracle.dist_grid(a, al, b, bl, S, 1, 10.0, use64=False)
                assert np.array_equal(got["numer"], nu), S
                assert np.array_equal(got["denom"], de), S
                np.testing.assert_allclose(got["pvalue"], pv, rtol=RTOL, atol=0)
                assert (nu > 0).any() and (nu == 0).any()
                if mode == "sparse":
                    assert st["sparse"] == 1, st          # index + literal walk
                    assert st["candidates"] < len(a) * len(b)
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)


def _record_edge_lists(rng):
    """-fp lists at the edges of the record filter: ascending (every entry a record),
    descending (one record), a leading 0, small alphabets (repeated maxima), the shared value
    first in one list and last in the other, long lists whose shared records lie past S
    steps, and empty lists."""
    L = [np.arange(0, 300, dtype=np.uint32), np.arange(0, 300, 2, dtype=np.uint32),
         np.arange(300, 0, -1, dtype=np.uint32), np.array([0, 0, 5, 0, 5, 7], np.uint32),
         np.array([0], np.uint32), np.zeros(0, np.uint32), np.array([9, 1, 2, 3], np.uint32),
         np.array([1, 2, 3, 9], np.uint32),
         np.concatenate([rng.integers(0, 1000, 1500), [4000000000]]).astype(np.uint32),
         np.concatenate([[4000000000], rng.integers(0, 1000, 1500)]).astype(np.uint32)]
    for _ in range(30):
        L.append(rng.integers(0, int(rng.choice([3, 8, 50, 2 ** 32])), int(rng.integers(0, 400)),
                              dtype=np.uint64).astype(np.uint32))
    return L


@pytest.mark.parametrize("mode", ["auto", "sparse"])
def test_dist_unsorted_record_edges(ctx, oracle, mode):
    """The record filter's edge cases (_record_edge_lists) for S = 1, 5, 64, 1000, self set
    and a separate query set, against the literal-walk oracle."""
    import fpmash
    rng = np.random.default_rng(5)
    refs = _record_edge_lists(rng)
    qrys = _record_edge_lists(rng)[::-1]
    rl = [max(1, len(x)) for x in refs]
    ql = [max(1, len(x)) for x in qrys]
    ctx.set_dist_mode(fpmash.DIST_SPARSE if mode == "sparse" else fpmash.DIST_AUTO)
    try:
        for S in (1, 5, 64, 1000):
            for (a, al), (b, bl) in (((refs, rl), (refs, rl)), ((refs, rl), (qrys, ql))):
                got = ctx.dist(a, b, S, use64=False, k=1, kmer_space=10.0, ref_lengths=al,
                               qry_lengths=bl)
                nu, de, di, pv = oracle.dist_grid(a, al, b, bl, S, 1, 10.0, use64=False)
                assert np.array_equal(got["numer"], nu), S
                assert np.array_equal(got["denom"], de), S
                np.testing.assert_allclose(got["pvalue"], pv, rtol=RTOL, atol=0)
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)


@pytest.mark.parametrize("mode", ["auto", "sparse"])
def test_rank_crowded_buckets(ctx, oracle, mode):
    """Sorted u64 lists with a crowded rank bucket: 40-120 values 2^33 apart (distinct 32-bit
    keys, one directory bucket of the rank kernel) beside uniform ones: the rows past the
    unrolled probe widths take the clamped 64-bit loop (NP = 0).  Every grid cell against the
    oracle, self set and a separate query set."""
    import fpmash
    rng = np.random.default_rng(31)
    base = np.uint64(0x9000000000000000)
    pool_c = base + np.arange(400, dtype=np.uint64) * np.uint64(1 << 33)
    pool_u = rng.integers(1, 2 ** 63, size=20000, dtype=np.uint64) * np.uint64(2)
    def lists(n):
        out = []
        for _ in range(n):
            c = rng.choice(pool_c, size=int(rng.integers(40, 120)), replace=False)
            u = rng.choice(pool_u, size=int(rng.integers(200, 900)), replace=False)
            out.append(np.unique(np.concatenate([c, u])))
        return out
    refs, qrys = lists(60), lists(45)
    rl = [len(x) * 5 for x in refs]
    ql = [len(x) * 5 for x in qrys]
    ctx.set_dist_mode(fpmash.DIST_SPARSE if mode == "sparse" else fpmash.DIST_AUTO)
    try:
        for S in (1000, 300):
            for (a, al), (b, bl) in (((refs, rl), (refs, rl)), ((refs, rl), (qrys, ql))):
                got = ctx.dist(a, b, S, ref_lengths=al, qry_lengths=bl)
                nu, de, di, pv = oracle.dist_grid(a, al, b, bl, S, 21, 4.0 ** 21)
                assert np.array_equal(got["numer"], nu), S
                assert np.array_equal(got["denom"], de), S
                assert (nu > 0).any()
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)


def test_streams_events_pipeline(ctx, oracle):
    """fpm_stream_create / fpm_event_*: two sketch jobs of different batches on a second
    stream, each dist on the context stream after its sketch's event (the bench's pipelined
    steps): every grid equals the serial one and the oracle's."""
    import fpmash
    import fpmash.datagen as D
    L = fpmash.lib()
    P = fpmash.make_params(k=21, s=1000)
    batches = [D.family_dna(4, 6, 2000, sub_rate=(0.0, 0.08), seed=sd) for sd in (3, 4, 5)]
    jobs = [ctx.sketch_job(P, b) for b in batches]
    n = len(batches[0])
    lens = fpmash.DeviceBuffer.from_array(ctx, np.full(n, 2000, np.uint64))
    sB = ctx.new_stream()
    ev = [ctx.new_event() for _ in jobs]
    outs = [(fpmash.DeviceBuffer(ctx, n * n * 2), fpmash.DeviceBuffer(ctx, n * n * 2),
             fpmash.CellList(ctx, n * n)) for _ in jobs]
    try:
        for j, e in zip(jobs, ev):          # all sketches on stream B, events after each
            j.run(sB)
            ctx.record(e, sB)
        for j, e, (nu, de, cl) in zip(jobs, ev, outs):
            ctx.wait(ctx.stream, e)
            rows, cnt, _, stride = j.device_output()
            fpmash._check(L.fpm_dist_list_dev(ctx.h, rows, cnt, lens.ptr, stride, n, rows, cnt,
                                              lens.ptr, stride, n, 8, 1000, 21, 4.0 ** 21, 1.0,
                                              1.0, nu.ptr, de.ptr, cl.ref, ctx.stream))
        ctx.synchronize()
        for b, (nu, de, cl) in zip(batches, outs):
            sk = oracle.sketch_batch(oracle.params(k=21, s=1000), b)
            L2 = [2000] * n
            gnu, gde, _, _ = oracle.dist_grid(sk, L2, sk, L2, 1000, 21, 4.0 ** 21)
            assert np.array_equal(nu.to_array(np.uint16, n * n), gnu)
            assert np.array_equal(de.to_array(np.uint16, n * n), gde)
    finally:
        for nu, de, cl in outs:
            nu.free()
            de.free()
            cl.free()
        lens.free()
        for e in ev:
            ctx.free_event(e)
        ctx.free_stream(sB)
        for j in jobs:
            j.free()


def test_pvalue_batch(ctx, oracle):
    """fpm_pvalue_batch_dev: distance and p-value of arbitrary cells (u16 and u32 counts)
    against the oracle's distance / pValue, including x = 0 (p = 1), numer = denom
    (distance 0), tiny and huge genome lengths and the -fp k-mer space."""
    rng = np.random.default_rng(12)
    n = 3000
    denom = rng.integers(1, 2000, size=n).astype(np.uint32)
    numer = np.minimum(rng.integers(0, 2000, size=n), denom).astype(np.uint32)
    numer[:50] = 0
    numer[50:100] = denom[50:100]
    lr = rng.integers(1, 10 ** 9, size=n, dtype=np.uint64)
    lq = rng.integers(1, 10 ** 9, size=n, dtype=np.uint64)
    lr[100:150] = 21
    for dt, k, space in ((np.uint32, 21, 4.0 ** 21), (np.uint16, 21, 4.0 ** 21),
                         (np.uint16, 1, 10.0)):
        d, p = ctx.pvalue_batch(numer.astype(dt), denom.astype(dt), lr, lq, k=k, kmer_space=space)
        for i in range(n):
            assert d[i] == pytest.approx(oracle.distance(int(numer[i]), int(denom[i]), k),
                                         rel=RTOL, abs=0), i
            assert p[i] == pytest.approx(oracle.pvalue(int(numer[i]), int(lr[i]), int(lq[i]),
                                                       space, int(denom[i])), rel=RTOL, abs=0), i


def test_dist_filters(ctx, oracle, dist_mode):
    seqs, sk = _family_sketches(oracle, n_fam=3, members=5)
    # 16 lists (a multiple of 4: the fill kernel's vector path) with an empty one (an empty
    # pair has distance 0)
    sk = sk + [np.zeros(0, np.uint64)]
    lengths = [len(x) for x in seqs] + [100]
    got = ctx.dist(sk, sk, 1000, ref_lengths=lengths, qry_lengths=lengths, max_dist=0.05,
                   max_pvalue=1e-30)
    nu, de, di, pv = oracle.dist_grid(sk, lengths, sk, lengths, 1000, 21, 4.0 ** 21)
    exp = (di <= 0.05) & (pv <= 1e-30)
    assert np.array_equal(got["pass"], exp)
    # a pair dropped by -d keeps p-value 0 (the p-value is not computed for it)
    np.testing.assert_allclose(got["distance"], di, rtol=RTOL, atol=0)
    np.testing.assert_allclose(got["pvalue"], np.where(di <= 0.05, pv, 0.0), rtol=RTOL, atol=0)
    # a -d above 1 keeps every pair; the no-shared-hash cells get p-value 1
    got = ctx.dist(sk, sk, 1000, ref_lengths=lengths, qry_lengths=lengths, max_dist=1.5,
                   max_pvalue=0.5)
    assert np.array_equal(got["pass"], pv <= 0.5)
    np.testing.assert_allclose(got["pvalue"], pv, rtol=RTOL, atol=0)


def test_dist_sparse_large_grid(ctx, oracle):
    """A grid big enough for AUTO to pick the inverted index: counts match a dense run
    and the oracle on a sampled block."""
    import fpmash
    seqs, sk = _family_sketches(oracle, n_fam=20, members=30, seed=3)
    lengths = [len(x) for x in seqs]
    ctx.set_dist_mode(fpmash.DIST_AUTO)
    a = ctx.dist(sk, sk, 1000, ref_lengths=lengths, qry_lengths=lengths)
    st = ctx.last_dist_stats()
    assert st["sparse"] and 0 < st["candidates"] < len(sk) ** 2
    ctx.set_dist_mode(fpmash.DIST_DENSE)
    b = ctx.dist(sk, sk, 1000, ref_lengths=lengths, qry_lengths=lengths)
    ctx.set_dist_mode(fpmash.DIST_AUTO)
    for key in ("numer", "denom", "distance", "pvalue", "pass"):
        assert np.array_equal(a[key], b[key]), key
    nu, de, di, pv = oracle.dist_grid(sk, lengths, sk[:50], lengths[:50], 1000, 21, 4.0 ** 21)
    n = len(sk)
    assert np.array_equal(a["numer"][:50 * n], nu)
    assert np.array_equal(a["denom"][:50 * n], de)


def _sorted_lists(rng):
    """Sorted distinct u64 lists that stress the rank kernel's bucket table: values near
    2**64 (shift 52), tiny values (shift 0), one crowded bucket (long in-bucket search),
    heavy overlap with lists shorter than S (denom < S), long lists (CAP 2048), and the value
    2**64 - 1 (equal to the rank kernel's sentinel) in lists sharing other values."""
    pool = np.unique(rng.integers(0, 2 ** 64, size=6000, dtype=np.uint64))
    lists = []
    for i in range(24):
        n = int(rng.integers(0, 1900))
        lists.append(np.sort(rng.choice(pool[:2500], size=n, replace=False)))
    small = np.arange(0, 6000, 3, dtype=np.uint64)                  # shift 0
    lists += [small[:700], small[::2][:900], small[100:101]]
    top = np.uint64(2 ** 64 - 1) - np.arange(0, 4000, 2, dtype=np.uint64)[::-1]
    lists += [top[-1000:], top[-1500:][::3]]                           # bits = 64
    crowd = np.concatenate([np.arange(1000, 1400, dtype=np.uint64),     # one bucket holds 400
                            np.array([2 ** 62], dtype=np.uint64)])
    lists += [crowd, crowd[::2], np.union1d(crowd[:50], small[:300])]
    core = pool[:300]
    lists += [core, core[:250], core[50:], pool[:2000], pool[1000:3000]]   # near-identical, long
    # the value 2**64 - 1 in A against a B without it (it meets B's sentinels) and with it
    lists += [np.append(core[:280], np.uint64(2 ** 64 - 1)), np.append(core[20:], top[-3:])]
    return lists


def _shared_and_near_lists(rng):
    """Sorted distinct u64 lists for the sparse path's index, probe and rank kernels:
    * 300 values shared by 150 rows (posting buckets of 150 entries, a family of 150),
    * rows built from the same 400 base values offset by 0, 1 or 2 (rows of different offsets
      share no value but every value's bucket and fingerprint: candidates sharing nothing),
    * rows holding v, v + 1 and v ^ 32 together (equal top 32 bits: equal rank keys, so the
      rank kernel's clamped loop; a crowded index bucket), against rows holding only v."""
    top = np.uint64(1) << np.uint64(63)
    common = rng.integers(0, 2 ** 63, size=300, dtype=np.uint64) | top
    lists = []
    for i in range(150):
        own = rng.integers(0, 2 ** 64, size=int(rng.integers(200, 800)), dtype=np.uint64)
        lists.append(np.unique(np.concatenate([common, own])))
    base = (rng.integers(0, 2 ** 62, size=400, dtype=np.uint64) << np.uint64(2)) | top
    for i in range(30):
        pick = np.sort(rng.choice(base, size=int(rng.integers(300, 400)), replace=False))
        lists.append(np.unique(pick + np.uint64(i % 3)))
    v = np.unique(rng.integers(0, 2 ** 62, size=200, dtype=np.uint64) << np.uint64(6)) | top
    for i in range(12):
        vv = rng.choice(v, size=150, replace=False)
        parts = [vv] if i % 2 else [vv, vv + np.uint64(1), vv ^ np.uint64(32)]
        lists.append(np.unique(np.concatenate(parts + [common[: 40 * (i % 3)]])))
    return lists


@pytest.mark.parametrize("compact", [False, True])
def test_dist_shared_rows_and_near_collisions(ctx, oracle, compact):
    """Hashes shared across many rows and same-bucket near-collisions (_shared_and_near_lists)
    through the forced sparse path, as one set against itself (the symmetric probe and rank,
    and the compact list) and against a copy; every cell equals the reference walk's
    (CommandDistance.cpp:376-400) at S = 1000 and S = 300."""
    import fpmash
    rng = np.random.default_rng(77)
    lists = _shared_and_near_lists(rng)
    lengths = [int(x) for x in rng.integers(10 ** 4, 10 ** 6, size=len(lists))]
    ctx.set_dist_mode(fpmash.DIST_SPARSE)
    try:
        for S in (1000, 300):
            nu, de, di, pv = oracle.dist_grid(lists, lengths, lists, lengths, S, 21, 4.0 ** 21)
            for other in (lists, [x.copy() for x in lists]):
                # the compact list is expanded (expand_compact asserts it holds exactly the
                # cells with numer > 0)
                run = ctx.dist_list if compact else ctx.dist
                got = run(lists, other, S, use64=True, k=21, ref_lengths=lengths,
                          qry_lengths=lengths)
                assert np.array_equal(got["numer"].astype(np.uint32), nu), S
                assert np.array_equal(got["denom"].astype(np.uint32), de), S
                np.testing.assert_allclose(got["distance"], di, rtol=RTOL, atol=0)
                assert ctx.last_dist_stats()["sparse"] == 2
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)


@pytest.mark.parametrize("mode", ["sparse", "dense"])
def test_dist_rank_kernel_edges(ctx, oracle, mode):
    import fpmash
    rng = np.random.default_rng(21)
    lists = _sorted_lists(rng)
    lengths = [int(x) for x in rng.integers(1000, 10 ** 6, size=len(lists))]
    ctx.set_dist_mode(fpmash.DIST_SPARSE if mode == "sparse" else fpmash.DIST_DENSE)
    try:
        for S in (1000, 2000, 260, 1):
            got = ctx.dist(lists, lists, S, use64=True, k=21, ref_lengths=lengths,
                           qry_lengths=lengths)
            nu, de, di, pv = oracle.dist_grid(lists, lengths, lists, lengths, S, 21, 4.0 ** 21)
            assert np.array_equal(got["numer"], nu), S
            assert np.array_equal(got["denom"], de), S
            np.testing.assert_allclose(got["distance"], di, rtol=RTOL, atol=0)
            np.testing.assert_allclose(got["pvalue"], pv, rtol=RTOL, atol=0)
            if mode == "sparse":
                assert ctx.last_dist_stats()["sparse"] == 2
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)


def test_dist_self_symmetric_path(ctx, oracle):
    """One sorted set against itself (same buffers) ranks each unordered pair once (in the
    row the probe's pair-parity rule gives it) and mirrors; the result equals the same data
    passed as a separate copy and the oracle."""
    import fpmash
    seqs, sk = _family_sketches(oracle, n_fam=8, members=12, seed=11)
    sk = sk + [sk[0][:10], np.zeros(0, np.uint64), sk[5][:700]]
    lengths = [len(x) for x in seqs] + [50, 100, 3000]
    ctx.set_dist_mode(fpmash.DIST_SPARSE)
    try:
        for S in (1000, 300):
            a = ctx.dist(sk, sk, S, ref_lengths=lengths, qry_lengths=lengths)
            assert ctx.last_dist_stats()["sparse"] == 2
            b = ctx.dist(sk, [x.copy() for x in sk], S, ref_lengths=lengths, qry_lengths=lengths)
            for key in ("numer", "denom", "distance", "pvalue", "pass"):
                assert np.array_equal(a[key], b[key]), key
            nu, de, di, pv = oracle.dist_grid(sk, lengths, sk, lengths, S, 21, 4.0 ** 21)
            assert np.array_equal(a["numer"], nu) and np.array_equal(a["denom"], de)
            np.testing.assert_allclose(a["distance"], di, rtol=RTOL, atol=0)
            np.testing.assert_allclose(a["pvalue"], pv, rtol=RTOL, atol=0)
            # filters on the symmetric path: mirror cells get the same decision
            f = ctx.dist(sk, sk, S, ref_lengths=lengths, qry_lengths=lengths, max_dist=0.1,
                         max_pvalue=1e-10)
            assert np.array_equal(f["pass"], (di <= 0.1) & (pv <= 1e-10))
            np.testing.assert_allclose(f["pvalue"], np.where(di <= 0.1, pv, 0.0), rtol=RTOL,
                                       atol=0)
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)


def test_dist_speculated_probe(ctx, oracle):
    """A dist call of the previous sparse rank-kernel call's shape enqueues its probe before the
    host reads the index build's counters (fpm_ctx_spec_stats).  Kept when the counters confirm
    the path and the capacity; dropped and redone when they do not: more candidates than the
    profile's capacity (sparse random rows, then heavily shared family rows of the same shape),
    an unsorted row (the literal walk), a near-identical set (the dense walk).  Every grid
    equals the oracle's."""
    import fpmash
    import fpmash.datagen as D
    S = 37
    P = oracle.params(k=21, s=S)

    def check(rows, lens):
        got = ctx.dist(rows, rows, S, ref_lengths=lens, qry_lengths=lens)
        nu, de, di, pv = oracle.dist_grid(rows, lens, rows, lens, S, 21, 4.0 ** 21)
        assert np.array_equal(got["numer"], nu) and np.array_equal(got["denom"], de)
        np.testing.assert_allclose(got["pvalue"], pv, rtol=RTOL, atol=0)
        return got

    # 400 rows of 37 hashes: the random rows' posting events (~5 per hash) stay below the
    # 160,000 pairs, the families' (~12 per hash) do not
    rand = oracle.sketch_batch(P, D.family_dna(400, 1, 1500, seed=3))
    fam = oracle.sketch_batch(P, D.family_dna(40, 10, 1500, sub_rate=(0.0, 0.03), seed=4))
    L = [1500] * 400
    assert {len(x) for x in rand} == {len(x) for x in fam} == {S}
    h0, m0 = ctx.spec_stats()
    check(rand, L)                       # sets the profile: capacity min(events, pairs)
    check(rand, L)                       # same shape: the speculated probe is kept
    h1, m1 = ctx.spec_stats()
    assert h1 == h0 + 1 and m1 == m0, (h0, m0, h1, m1)
    g = check(fam, L)                    # more candidates than the capacity: redone
    assert (g["numer"] > 0).sum() >= 4000          # every family pair (40 x 10 x 10)
    h2, m2 = ctx.spec_stats()
    assert m2 == m1 + 1, (m1, m2)
    check(fam, L)                        # the profile grew: kept
    h3, m3 = ctx.spec_stats()
    assert h3 == h2 + 1 and m3 == m2
    uns = [x.copy() for x in fam]
    uns[5] = uns[5][::-1].copy()         # an unsorted row: the literal walk
    check(uns, L)
    assert ctx.last_dist_stats()["sparse"] != 2
    near = [fam[0].copy() for _ in range(400)]
    near[7] = rand[7]                    # near-identical rows: the dense walk
    check(near, L)
    assert ctx.last_dist_stats()["sparse"] == 0
    check(fam, L)
    h4, m4 = ctx.spec_stats()
    assert m4 >= m3 + 1 and h4 >= h3


@pytest.mark.parametrize("layout", ["contiguous", "interleaved"])
def test_dist_family_layouts_and_bridges(ctx, oracle, layout):
    """Families with adjacent ids and with interleaved ids (a family's entries spread over the
    whole id range of every bucket), plus bridge rows that share 1-3 hashes with members of
    several families (pairs whose only shared hashes sit in other families' buckets), and a
    row repeated: every cell equals the oracle, on the symmetric self path and against a copy.
    (Written for the covered-bucket probe skip, measured slower and removed in round 6.)"""
    import fpmash
    seqs, sk = _family_sketches(oracle, n_fam=10, members=12, seed=17)
    lengths = [len(x) for x in seqs]
    if layout == "interleaved":
        order = [f + 10 * m for m in range(12) for f in range(10)]
        sk = [sk[i] for i in order]
        lengths = [lengths[i] for i in order]
    rng = np.random.default_rng(5)
    bridges = []
    for b in range(6):
        picks = [sk[int(i)][rng.integers(0, len(sk[int(i)]), size=1 + b % 3)]
                 for i in rng.choice(len(sk), size=4, replace=False)]
        filler = rng.integers(1, 2 ** 63, size=900, dtype=np.uint64)
        bridges.append(np.unique(np.concatenate(picks + [filler])))
    sk = sk + bridges + [sk[7].copy()]
    lengths = lengths + [2000] * len(bridges) + [lengths[7]]
    ctx.set_dist_mode(fpmash.DIST_SPARSE)
    try:
        a = ctx.dist(sk, sk, 1000, ref_lengths=lengths, qry_lengths=lengths)
        assert ctx.last_dist_stats()["sparse"] == 2
        b = ctx.dist(sk, [x.copy() for x in sk], 1000, ref_lengths=lengths, qry_lengths=lengths)
        nu, de, di, pv = oracle.dist_grid(sk, lengths, sk, lengths, 1000, 21, 4.0 ** 21)
        for got in (a, b):
            assert np.array_equal(got["numer"], nu) and np.array_equal(got["denom"], de)
            np.testing.assert_allclose(got["pvalue"], pv, rtol=RTOL, atol=0)
        n = len(sk)
        nb = len(bridges)
        # the bridges share hashes with family rows: those pairs are counted
        assert (nu.reshape(n, n)[n - 1 - nb:n - 1, :n - 1 - nb] > 0).sum() >= nb
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)


@pytest.mark.parametrize("mode", ["auto", "dense", "sparse"])
def test_dist_dev16_matches_u32(ctx, oracle, mode):
    """fpm_dist_dev16 (u16 numer / denom cells) gives the u32 path's results on the symmetric
    self path, a query subset, unsorted -fp lists (literal walk) and the dense walk; the
    counts equal the oracle's; sketch sizes above 65535 are refused."""
    import fpmash
    seqs, sk = _family_sketches(oracle, n_fam=6, members=8, seed=23)
    sk = sk + [sk[0][:10], np.zeros(0, np.uint64), sk[3][:999]]
    lengths = [len(x) for x in seqs] + [2000, 100, 2000]
    ctx.set_dist_mode({"auto": fpmash.DIST_AUTO, "dense": fpmash.DIST_DENSE,
                       "sparse": fpmash.DIST_SPARSE}[mode])
    try:
        for S in (1000, 300):
            for qry, ql in ((sk, lengths), (sk[5:19], lengths[5:19])):
                a = ctx.dist(sk, qry, S, ref_lengths=lengths, qry_lengths=ql)
                b = ctx.dist16(sk, qry, S, ref_lengths=lengths, qry_lengths=ql)
                for key in ("numer", "denom", "distance", "pvalue", "pass"):
                    assert np.array_equal(a[key].astype(np.float64) if key in ("numer", "denom")
                                          else a[key],
                                          b[key].astype(np.float64) if key in ("numer", "denom")
                                          else b[key]), (S, key)
                nu, de, _di, _pv = oracle.dist_grid(sk, lengths, list(qry), list(ql), S, 21,
                                                    4.0 ** 21)
                assert np.array_equal(b["numer"], nu) and np.array_equal(b["denom"], de)
        rng = np.random.default_rng(4)
        base = rng.integers(0, 2 ** 32, size=800, dtype=np.uint64).astype(np.uint32)
        lists = [base[rng.integers(0, 800, size=int(rng.integers(0, 1500)))] for _ in range(24)]
        fl = [int(rng.integers(1, 9000)) for _ in lists]
        a = ctx.dist(lists, lists, 1000, use64=False, k=1, kmer_space=10.0, ref_lengths=fl,
                     qry_lengths=fl)
        b = ctx.dist16(lists, lists, 1000, use64=False, k=1, kmer_space=10.0, ref_lengths=fl,
                       qry_lengths=fl)
        assert np.array_equal(a["numer"], b["numer"]) and np.array_equal(a["denom"], b["denom"])
        np.testing.assert_array_equal(a["pvalue"], b["pvalue"])
        with pytest.raises(fpmash.FpmError):
            ctx.dist16(sk, sk, 70000, ref_lengths=lengths, qry_lengths=lengths)
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)


def _fp_texts():
    rng = np.random.default_rng(31)
    import fpmash.datagen as D
    texts = [open(os.path.join(GOLDEN, "DNA2-CFL.txt"), "rb").read()[:200000],
             b"", b"\n", b"\n\n\nX 1 2\n", b"ID 1 2 3", b"ID\n", b"   \t \n",
             b"A 1 2\nA 3\nB 4\n\nB 5\nB\t6\r\nC +7 -8 9x 10\nD 18446744073709551615 "
             b"18446744073709551616 3\nE 1\x0b2\x0c3\r\nF abc 1\n  G   5  6  \n",
             b"X " + b" ".join(str(v).encode() for v in rng.integers(0, 2 ** 63, 40)) + b"\n"]
    # random CFL-like lines with mixed separators and ID runs
    lines = []
    for i in range(3000):
        idv = b"T%05d" % (i // int(rng.integers(1, 40)))
        vals = rng.integers(0, 200, size=int(rng.integers(0, 16)))
        sep = [b" ", b"\t", b"  "][int(rng.integers(0, 3))]
        lines.append(idv + sep + sep.join(str(v).encode() for v in vals))
    texts.append(b"\n".join(lines))
    texts.append(D.cfl_text(D.random_dna(30, 300, seed=4), D.lyn2vec_ids(30)))
    # lines of ~1.5 KB: a wave's 64 lines span more than fp_line_kernel's 4 KB LDS window
    # (global-memory path), after and between short lines (staged waves)
    long_lines = [b"L%d " % (i // 3) + b" ".join(str(v).encode() for v in rng.integers(0, 2 ** 40, 120))
                  for i in range(150)]
    texts.append(b"\n".join(lines[:200] + long_lines + lines[200:400]) + b"\n")
    return texts


@pytest.mark.parametrize("use64", [False, True])
def test_fp_text_parse_matches_oracle(ctx, oracle, use64):
    """GPU -fp text parse + line hash == the istream-semantics oracle, incl. blank lines,
    \\t \\r \\v \\f, signs, overflow, non-numeric tokens, no trailing newline, line caps."""
    for t in _fp_texts():
        for cap in (1_000_000, 7, 1, 0):
            got = ctx.fp_text(t, max_lines=cap, seed=42, use64=use64)
            ids, vals, used = oracle.fp_parse(t, limit=cap)
            assert len(got["id_off"]) == len(ids) == used
            prev = None
            for i, (idv, v) in enumerate(zip(ids, vals)):
                o, n = int(got["id_off"][i]), int(got["id_len"][i])
                assert t[o:o + n] == idv
                assert got["n_vals"][i] == len(v)
                assert int(got["hash"][i]) == oracle.get_hash_fp(v, 42, use64)
                if i:
                    assert got["new_id"][i] == (1 if idv != prev else 0)
                else:
                    assert got["new_id"][0] == 2
                prev = idv


@pytest.mark.parametrize("use64", [False, True])
def test_fp_refs_match_oracle(ctx, oracle, use64):
    """fpm_fp_text_refs (the References grouped on the device) == initFromFingerprints'
    grouping of the istream-semantics parse (Sketch.cpp:104-145): a Reference at line 0 and at
    every ID change, its ID, its length (the first line's value count twice, :117 + :134) and
    its line hashes, over the edge-case texts, the three CFL fixtures whole, and line caps."""
    texts = _fp_texts() + [open(os.path.join(GOLDEN, f"DNA{i}-CFL.txt"), "rb").read()
                           for i in (1, 2, 3)]
    for t in texts:
        for cap in (1_000_000, 7, 1, 0):
            got = ctx.fp_refs(t, max_lines=cap, seed=42, use64=use64)
            ids, vals, used = oracle.fp_parse(t, limit=cap)
            assert got["n_lines"] == used
            heads = [i for i in range(used) if i == 0 or ids[i] != ids[i - 1]]
            assert list(got["first"]) == heads
            for r, a in enumerate(heads):
                b = heads[r + 1] if r + 1 < len(heads) else used
                o, n = int(got["id_off"][r]), int(got["id_len"][r])
                assert t[o:o + n] == ids[a]
                assert int(got["length"][r]) == len(vals[a]) + sum(len(v) for v in vals[a:b])
                exp_h = [oracle.get_hash_fp(v, 42, use64) for v in vals[a:b]]
                assert [int(x) for x in got["hash"][a:b]] == exp_h


@pytest.mark.parametrize("k,s", [(21, 1000), (21, 5000), (12, 2000), (21, 10000), (21, 16384),
                                 (21, 16385), (21, 50000)])
def test_sketch_long_groups_sample_bound(ctx, oracle, k, s):
    """Groups of >= 32 tiles take the sample pass (every 16th tile sketched first; its s-th
    smallest hash bounds every tile) and, for s <= ~13.5k, the one-workgroup selection from
    the bounded tile lists (with its merge fallback when the keys below the cut overflow
    LDS: the repeated unit): the sets still equal the reference heap's."""
    import fpmash
    rng = np.random.default_rng(k * 7 + s)
    unit = rand_seq(rng, 3000)
    # random 2 kb stretches alternating with one 2 kb unit (80 copies): the unit's values
    # repeat across the chunks, so the one-workgroup group selection meets duplicates below
    # its first cut and widens it
    mosaic = b"".join(rand_seq(rng, 2000) + unit[:2000] for _ in range(80))
    recs = [rand_seq(rng, 300_000),                        # one long record
            unit * 70,                                     # 210 kb of a repeated unit
            rand_seq(rng, 150_000, p_bad=0.001),           # long, with N windows
            ] + [rand_seq(rng, 60_000) for _ in range(4)] + [mosaic]   # a group of 4 x 60 kb
    groups = [0, 1, 2, 3, 3, 3, 3, 4]
    P = fpmash.make_params(k=k, s=s)
    got = ctx.sketch(P, recs, groups=groups, n_groups=5)
    exp = oracle.sketch_batch(oracle.params(k=k, s=s), recs, groups=groups, n_groups=5)
    check_sketches(got, exp)


@pytest.mark.parametrize("kind", ["random", "repeat"])
def test_sketch_survivors_kernel_redo(ctx, oracle, kind):
    """The survivors-only tile kernel (sketch_tiles_kernel<4096, K, true>: C5's genomes) and
    its redo pass.  A long random group keeps ~130 of a tile's 4,096 windows below its sampled
    bound: no tile overflows (redo_tiles() == 0).  A 2 Mb group of one repeated 3 kb unit has
    ~3,000 distinct k-mers, a third of them below the bound, so every tile's ~1,300 survivors
    (repeats included) overflow its 1,024 slots: each is listed and redone by the plain kernel
    through the device-side count (redo_tiles() > 0).  Both sketches equal the reference
    heap's (MinHashHeap.cpp:68-146)."""
    import fpmash
    rng = np.random.default_rng(11 if kind == "random" else 12)
    seq = rand_seq(rng, 2_000_000) if kind == "random" else rand_seq(rng, 3000) * 667
    P = fpmash.make_params(k=21, s=1000)
    job = ctx.sketch_job(P, [seq], groups=[0], n_groups=1)
    try:
        n_ss = []
        for _ in range(2):                      # the count is reset by every run
            job.run(ctx.stream)
            n_redo = job.redo_tiles()
            n_ss.append(job.sample_short())
            if kind == "random":
                assert n_redo == 0
                assert job.short_groups() == 0  # the tight bound held
            else:
                assert n_redo > 400             # 488 tiles, nearly all of them
                # the sample holds all ~3,000 distinct k-mers: its kt-th smallest leaves the
                # group ~160 of them, so the group is redone under the s-th smallest
                assert job.short_groups() == 1
        # every run starts from the staged a-priori sample bounds (a redo lifts them in the
        # run's bound array only): the same samples are found short on the second run
        assert n_ss[0] == n_ss[1] and n_ss[0] == (0 if kind == "random" else 1), n_ss
        rows, cnt = job.fetch()
    finally:
        job.free()
    exp = oracle.sketch_batch(oracle.params(k=21, s=1000), [seq])
    check_sketches([rows[0, : cnt[0]]], exp)


@pytest.mark.parametrize("s", [2000, 10000])
def test_sketch_tight_bound_short_groups(ctx, oracle, s):
    """Long groups bounded by the sample's kt-th smallest hash (kt ~ f s + 8 sqrt(f s) + 32):
    random genomes keep >= s hashes under it (short_groups() == 0); a genome of one 300 kb unit
    repeated 7 times has ~2.2x as many distinct k-mers as its sample, so the tight bound leaves
    it short and it is redone under the sample's s-th smallest (short_groups() == 1).  Every
    sketch equals the reference heap's, over two runs of the job (bounds recomputed each run)."""
    import fpmash
    rng = np.random.default_rng(s + 3)
    recs = [rand_seq(rng, 2_000_000), rand_seq(rng, 300_000) * 7, rand_seq(rng, 1_500_000)]
    P = fpmash.make_params(k=21, s=s)
    job = ctx.sketch_job(P, recs, groups=[0, 1, 2], n_groups=3)
    try:
        for _ in range(2):
            job.run(ctx.stream)
            assert job.short_groups() == 1
        rows, cnt = job.fetch()
    finally:
        job.free()
    exp = oracle.sketch_batch(oracle.params(k=21, s=s), recs, groups=[0, 1, 2], n_groups=3)
    check_sketches([rows[g, : cnt[g]] for g in range(3)], exp)


def test_sketch_survivors_kernel_off_for_large_s(ctx):
    """s so large that a long group's bound keeps about half a tile's slots (2 x 16 s / tiles
    + 64 > 512): the plain kernel takes the class-4 tiles (redo_tiles() == -1) instead of
    hashing most of them twice."""
    import fpmash
    rng = np.random.default_rng(13)
    job = ctx.sketch_job(fpmash.make_params(k=21, s=20_000), [rand_seq(rng, 2_000_000)],
                         groups=[0], n_groups=1)
    try:
        job.run(ctx.stream)
        assert job.redo_tiles() == -1
    finally:
        job.free()


def test_merge_small_kernel_forced():
    """Every merge round on merge_small_kernel (FPM_MERGE_SMALL=2, in a child process: the
    switch is read when the library loads), including lists longer than its LDS cap that
    it searches in global memory: sketches equal the oracle's."""
    import subprocess
    import sys
    env = dict(os.environ, FPM_MERGE_SMALL="2")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "_merge_small_worker.py")],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("use64,mode", [(True, "sorted"), (False, "fp"), (True, "dense")])
def test_refset_blocks_match_grid(ctx, oracle, use64, mode):
    """fpm_refset_*: references uploaded and indexed once, several query blocks probed
    against the resident index == the one-shot grid (and the oracle), for sorted u64
    sketches (index + rank), unsorted -fp u32 lists (deduplicated index + literal walk) and
    near-identical sets (events past the sparse threshold: dense walk)."""
    import fpmash
    from fpmash import datagen
    rng = np.random.default_rng(11)
    if mode == "fp":
        lists = [rng.integers(0, 40, size=int(rng.integers(1, 300))).astype(np.uint32)
                 for _ in range(60)]
        S, k, space = 200, 1, 10.0
    else:
        seqs = datagen.family_dna(6, 10, 1500, sub_rate=(0.0, 0.02 if mode == "dense" else 0.1),
                                  seed=17)
        lists = oracle.sketch_batch(oracle.params(k=21, s=300), seqs)
        S, k, space = 300, 21, 4.0 ** 21
    lengths = [int(len(x)) * 7 + 1000 for x in lists]
    refs, qrys = lists[:45], lists[15:]
    rl, ql = lengths[:45], lengths[15:]
    rs = ctx.refset(refs, S, use64=use64, ref_lengths=rl,
                    width=max(len(x) for x in lists))
    try:
        # no distance filter: the reference computes the p-value only for pairs that pass
        # it (CommandDistance.cpp:416-423); here every p-value is compared
        got = [rs.dist(qrys[i:i + 13], k=k, kmer_space=space, qry_lengths=ql[i:i + 13],
                       max_dist=-1.0, max_pvalue=0.5) for i in range(0, len(qrys), 13)]
    finally:
        rs.free()
    cat = {key: np.concatenate([g[key] for g in got]) for key in got[0]}
    nu, de, di, pv = oracle.dist_grid(refs, rl, qrys, ql, S, k, space, use64=use64)
    assert np.array_equal(cat["numer"], nu) and np.array_equal(cat["denom"], de)
    assert np.allclose(cat["distance"], di, rtol=1e-12, atol=0)
    assert np.allclose(cat["pvalue"], pv, rtol=1e-12, atol=0)
    assert np.array_equal(cat["pass"], pv <= 0.5)


@pytest.mark.parametrize("s", [50, 1000, 10000])
def test_sketch_merge_dev_matches_whole(ctx, oracle, s):
    """fpm_sketch_merge_dev (the cross-GPU min-merge): one genome sketched in 1-5 k-mer
    ranges (fpmash.shard.kmer_shard), the parts' rows merged on the device, equals the
    oracle's sketch of the whole genome (MinHashHeap semantics), repeats across parts
    included."""
    import fpmash
    from fpmash.shard import kmer_shard
    rng = np.random.default_rng(s)
    unit = rand_seq(rng, 5000)
    genome = rand_seq(rng, 400_000) + unit * 6 + rand_seq(rng, 200_000)
    exp = oracle.sketch_batch(oracle.params(k=21, s=s), [genome])[0]
    P = fpmash.make_params(k=21, s=s)
    for parts in (1, 2, 5):
        segs = [genome[a:b] for a, b in (kmer_shard(len(genome), 21, parts, r)
                                         for r in range(parts))]
        sk = ctx.sketch(P, segs)
        m = np.zeros((parts, s), np.uint64)
        for i, x in enumerate(sk):
            m[i, :len(x)] = x
        rows = fpmash.DeviceBuffer.from_array(ctx, m)
        cnts = fpmash.DeviceBuffer.from_array(ctx, np.array([len(x) for x in sk], np.uint32))
        out = fpmash.DeviceBuffer(ctx, s * 8)
        oc = fpmash.DeviceBuffer(ctx, 4)
        fpmash._check(fpmash.lib().fpm_sketch_merge_dev(ctx.h, rows.ptr, cnts.ptr, parts, s,
                                                        out.ptr, oc.ptr, None))
        ctx.synchronize()
        n = int(oc.to_array(np.uint32, 1)[0])
        assert n == len(exp)
        assert np.array_equal(out.to_array(np.uint64, s)[:n], exp)


@pytest.mark.parametrize("fillcnt", [False, True])
@pytest.mark.parametrize("data", ["self", "other", "fp"])
@pytest.mark.parametrize("maxd,maxp", [(-1.0, -1.0), (0.5, 1.0), (1.0, 1e-10)])
def test_dist_list_equals_dist16(ctx, oracle, data, maxd, maxp, fillcnt, dist_mode):
    """The compact output (fpm_dist_list_dev: u16 counts of every cell + the list of cells
    with numer > 0) expands, by the rule include/fpmash.h states for unlisted cells, to the
    five arrays fpm_dist_dev16 writes; counts and p-values also match the oracle.  Sorted
    sketches against themselves (the symmetric path) and against another set, unsorted -fp
    lists, empty lists, the -d / -v filters, every dist mode, and a context whose side fill
    writes the counts (FPM_FILL_COUNTS=1, the large-grid default)."""
    import fpmash
    from fpmash import datagen
    if fillcnt:
        os.environ["FPM_FILL_COUNTS"] = "1"
        try:
            ctx = fpmash.Context(0)
            ctx.set_dist_mode({"auto": 0, "dense": 1, "sparse": 2}[dist_mode])
        finally:
            del os.environ["FPM_FILL_COUNTS"]
    if data == "fp":
        rng = np.random.default_rng(41)
        sk = [rng.integers(0, 60, size=int(rng.integers(0, 400))).astype(np.uint32)
              for _ in range(90)]
        sk[3] = sk[3][:0]
        qsk = sk[::-1][:50]
        S, k, space, use64 = 300, 1, 10.0, False
        lens = np.array([len(x) * 3 + 7 for x in sk], np.uint64)
        qlens = lens[::-1][:50].copy()
    else:
        P = fpmash.make_params(k=21, s=500)
        seqs = datagen.family_dna(8, 12, 1500, sub_rate=(0.0, 0.08), seed=31)
        seqs += [b"N" * 300, b"", b"ACGT" * 3]          # lists with no k-mer: empty sketches
        sk = ctx.sketch(P, seqs)
        qsk = sk if data == "self" else sk[::-1][:60]
        S, k, space, use64 = 500, 21, 4.0 ** 21, True
        lens = np.array([len(x) for x in seqs], np.uint64)
        qlens = lens if data == "self" else lens[::-1][:60].copy()
    full = ctx.dist16(sk, qsk, S, use64=use64, k=k, kmer_space=space, ref_lengths=lens,
                      qry_lengths=qlens, max_dist=maxd, max_pvalue=maxp)
    comp = ctx.dist_list(sk, qsk, S, use64=use64, k=k, kmer_space=space, ref_lengths=lens,
                         qry_lengths=qlens, max_dist=maxd, max_pvalue=maxp)
    for key in ("numer", "denom", "distance", "pass"):
        assert np.array_equal(comp[key], full[key]), key
    dok = full["distance"] <= maxd if maxd >= 0 else np.ones(len(full["distance"]), bool)
    assert np.array_equal(comp["pvalue"][dok], full["pvalue"][dok])
    nu, de, di, pv = oracle.dist_grid(sk, list(lens), qsk, list(qlens), S, k, space, use64=use64)
    assert np.array_equal(comp["numer"], nu) and np.array_equal(comp["denom"], de)
    assert np.allclose(comp["distance"], di, rtol=1e-12, atol=0)
    assert np.allclose(comp["pvalue"][dok], pv[dok], rtol=1e-12, atol=0)
    assert (comp["numer"] > 0).any() and (comp["numer"] == 0).any()
    if fillcnt:
        ctx.close()


def test_dist_list_capacity(ctx, oracle):
    """A list too small for the cells with numer > 0: the count reports every cell, only
    `cap` entries are written (no write past the buffers), and the binding refuses to fetch;
    a re-run with cap = count lists them all."""
    import fpmash
    from fpmash import datagen
    P = fpmash.make_params(k=21, s=400)
    seqs = datagen.family_dna(4, 10, 1200, sub_rate=(0.0, 0.05), seed=8)
    sk = ctx.sketch(P, seqs)
    lens = [len(x) for x in seqs]
    nu, de, listed = ctx.dist_list(sk, sk, 400, ref_lengths=lens, qry_lengths=lens,
                                   expand=False)
    n = int((nu > 0).sum())
    assert len(listed["qry"]) == n and n > 50
    with pytest.raises(fpmash.FpmError):
        ctx.dist_list(sk, sk, 400, ref_lengths=lens, qry_lengths=lens, cap=17)
    # the count of a short list is still the full count
    lst = fpmash.CellList(ctx, 17)
    R, rl = fpmash._dense(sk, 400, np.uint64)
    bufs = [fpmash.DeviceBuffer.from_array(ctx, a) for a in (R, rl, np.array(lens, np.uint64))]
    out = [fpmash.DeviceBuffer(ctx, len(sk) ** 2 * 2) for _ in range(2)]
    L = fpmash.lib()
    fpmash._check(L.fpm_dist_list_dev(ctx.h, bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, 400, len(sk),
                                      bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, 400, len(sk), 8, 400,
                                      21, 4.0 ** 21, -1.0, -1.0, out[0].ptr, out[1].ptr, lst.ref,
                                      None))
    ctx.synchronize()
    assert lst.count() == n
    for b in bufs + out:
        b.free()
    lst.free()


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("mode", ["sorted", "fp", "dense"])
def test_refset_mirror_matches_oracle(ctx, oracle, mode, compact):
    """fpm_refset_dist_mirror_dev (the block pairs of the sharded C4 all-vs-all): the grid
    (queries x refs) and its transpose (refs as queries x the query rows as refs) both equal
    the oracle's grids of the two orientations; sorted u64 sketches take the sparse path that
    scatters the candidate results to both grids, unsorted -fp u32 lists (not symmetric under
    the literal walk) and a forced dense walk compute the transpose by the swapped call.
    Empty lists and the -d / -v filters included.  compact: fpm_refset_dist_mirror_list_dev
    (u16 counts of both grids + one list of numer > 0 cells per grid), expanded by the rule
    for unlisted cells."""
    import ctypes as C
    import fpmash
    from fpmash import datagen
    rng = np.random.default_rng(23)
    if mode == "fp":
        lists = [rng.integers(0, 40, size=int(rng.integers(1, 300))).astype(np.uint32)
                 for _ in range(70)]
        S, k, space, use64 = 200, 1, 10.0, False
    else:
        seqs = datagen.family_dna(7, 10, 1500, sub_rate=(0.0, 0.1), seed=29)
        lists = oracle.sketch_batch(oracle.params(k=21, s=300), seqs)
        lists[5] = lists[5][:0]                        # an empty sketch on each side
        lists[50] = lists[50][:0]
        S, k, space, use64 = 300, 21, 4.0 ** 21, True
    lengths = [int(len(x)) * 7 + 1000 for x in lists]
    refs, qrys = lists[:33], lists[33:]                 # disjoint row sets (two blocks)
    rl, ql = lengths[:33], lengths[33:]
    w = max(len(x) for x in lists)
    dt = np.uint64 if use64 else np.uint32
    R, rlen = fpmash._dense(refs, w, dt)
    Q, qlen = fpmash._dense(qrys, w, dt)
    L = fpmash.lib()
    keep = []

    def up(a):
        b = fpmash.DeviceBuffer.from_array(ctx, np.ascontiguousarray(a))
        keep.append(b)
        return b.ptr
    dR, drl, dRL = up(R), up(rlen), up(np.array(rl, np.uint64))
    dQ, dql, dQL = up(Q), up(qlen), up(np.array(ql, np.uint64))
    nr, nq = len(refs), len(qrys)
    cb = 2 if compact else 4
    prim = [fpmash.DeviceBuffer(ctx, nr * nq * b) for b in (cb, cb, 8, 8, 1)]
    mirr = [fpmash.DeviceBuffer(ctx, nr * nq * b) for b in (cb, cb, 8, 8, 1)]
    keep += prim + mirr
    lists_ = [fpmash.CellList(ctx, nr * nq), fpmash.CellList(ctx, nr * nq)]
    # the grids are small (AUTO would walk them densely): force the index path for the
    # sorted and -fp cases
    ctx.set_dist_mode(1 if mode == "dense" else 2)
    h = C.c_void_p()
    try:
        fpmash._check(L.fpm_refset_create_dev(ctx.h, dR, drl, dRL, w, nr, 8 if use64 else 4, S,
                                              C.byref(h)))
        for rep in range(2):                            # a second call after a reindex
            if rep:
                fpmash._check(L.fpm_refset_reindex(h, None))
            if compact:
                fpmash._check(L.fpm_refset_dist_mirror_list_dev(
                    h, dQ, dql, dQL, w, nq, S, k, space, 0.9, 0.5, prim[0].ptr, prim[1].ptr,
                    lists_[0].ref, mirr[0].ptr, mirr[1].ptr, lists_[1].ref, None))
                ctx.synchronize()
                got_p, got_m = [
                    [e[x] for x in ("numer", "denom", "distance", "pvalue", "pass")] for e in (
                        fpmash.expand_compact(bb[0].to_array(np.uint16, nr * nq),
                                              bb[1].to_array(np.uint16, nr * nq), lst.fetch(),
                                              n_r, 0.9, 0.5)
                        for bb, lst, n_r in ((prim, lists_[0], nr), (mirr, lists_[1], nq)))]
            else:
                fpmash._check(L.fpm_refset_dist_mirror_dev(h, dQ, dql, dQL, w, nq, S, 4, k, space,
                                                           0.9, 0.5, *[b.ptr for b in prim],
                                                           *[b.ptr for b in mirr], None))
                ctx.synchronize()
                types = (np.uint32, np.uint32, np.float64, np.float64, np.uint8)
                got_p = [b.to_array(t, nr * nq) for b, t in zip(prim, types)]
                got_m = [b.to_array(t, nr * nq) for b, t in zip(mirr, types)]
            for got, (a, al, b, bl) in ((got_p, (refs, rl, qrys, ql)),
                                        (got_m, (qrys, ql, refs, rl))):
                nu, de, di, pv = oracle.dist_grid(a, al, b, bl, S, k, space, use64=use64)
                assert np.array_equal(got[0], nu) and np.array_equal(got[1], de)
                assert np.allclose(got[2], di, rtol=1e-12, atol=0)
                ok = (di <= 0.9)
                assert np.allclose(got[3][ok], pv[ok], rtol=1e-12, atol=0)
                assert np.array_equal(got[4].astype(bool), ok & (pv <= 0.5))
        if mode == "sorted":
            assert ctx.last_dist_stats()["sparse"] == 2
    finally:
        if h:
            L.fpm_refset_free(h)
        ctx.set_dist_mode(0)
        for b in keep:
            b.free()
        for lst in lists_:
            lst.free()


def test_index_one_pass_holds_sketch_partitions(ctx, oracle):
    """The one-pass index build (level-1 slots of 1.5 x mean + 6 sigma) takes bottom-s sketch
    rows without a rebuild (their values taper towards the largest indexed key), and the
    sparse dist over it equals the oracle on sampled rows."""
    import fpmash
    from fpmash import datagen
    seqs = datagen.family_dna(40, 50, 2000, sub_rate=(0.01, 0.1), seed=41)
    sk = ctx.sketch(fpmash.make_params(k=21, s=1000), seqs)
    before = ctx.index_rebuilds()
    lengths = [len(x) for x in seqs]
    rows = list(range(0, len(sk), 97))
    ctx.set_dist_mode(2)
    try:
        d = ctx.dist(sk, sk, 1000, ref_lengths=lengths, qry_lengths=lengths)
    finally:
        ctx.set_dist_mode(0)
    assert ctx.index_rebuilds() == before
    nu, de, di, pv = oracle.dist_grid(sk, lengths, [sk[r] for r in rows], [lengths[r] for r in rows],
                                      1000, 21, 4.0 ** 21)
    n = len(sk)
    got_nu = np.concatenate([d["numer"][r * n:(r + 1) * n] for r in rows])
    got_de = np.concatenate([d["denom"][r * n:(r + 1) * n] for r in rows])
    assert np.array_equal(got_nu, nu) and np.array_equal(got_de, de)


def test_index_one_pass_overflow_rebuilds(ctx, oracle):
    """Skewed keys: 600 sorted sketches that all hold the same 400 values (plus
    their own) put ~2.4e5 entries into the level-1 partition of those values, past its
    one-pass slot; the build flags the overflow and the exact two-pass build replaces it
    (ctx.index_rebuilds() goes up), and the sparse grid still equals the oracle."""
    import fpmash
    rng = np.random.default_rng(77)
    # the shared values span one level-1 partition (keys scale to the largest, ~2^62: a
    # partition is 2^52 wide) but many of its buckets (~1,800 entries each, not one bucket of
    # 240,000: the probe reads every entry of a hash's bucket)
    common = np.unique(rng.integers(1, 1 << 52, size=400, dtype=np.uint64))
    lists = []
    for _ in range(600):
        own = rng.integers(1 << 52, 1 << 62, size=int(rng.integers(50, 200)), dtype=np.uint64)
        lists.append(np.unique(np.concatenate([common, own])))
    L = [len(x) * 3 for x in lists]
    before = ctx.index_rebuilds()
    ctx.set_dist_mode(fpmash.DIST_SPARSE)
    try:
        d = ctx.dist(lists, lists, 500, ref_lengths=L, qry_lengths=L)
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)
    assert ctx.index_rebuilds() > before
    rows = list(range(0, 600, 37))
    nu, de, di, pv = oracle.dist_grid(lists, L, [lists[r] for r in rows], [L[r] for r in rows],
                                      500, 21, 4.0 ** 21)
    n = len(lists)
    got = np.concatenate([d["numer"][r * n:(r + 1) * n] for r in rows])
    gde = np.concatenate([d["denom"][r * n:(r + 1) * n] for r in rows])
    assert np.array_equal(got, nu) and np.array_equal(gde, de)


@pytest.mark.parametrize("n_ref,skew", [(16700, False), (36000, False), (36000, True)])
def test_index_split_level2(ctx, oracle, n_ref, skew):
    """The level-2 index pass beyond one 16k-entry register copy per partition.  E = 1.67e7
    (l2 = 12, partitions of ~16.3k): those over 16,384 entries are read twice and scattered
    through the LDS.  E = 3.6e7 (l2 = 14: C4's geometry): the sub-bucket range split over 2
    workgroups per partition, each scattering its half through the LDS.  skew: every list also
    holds 30 of 4,000 values spread over ~128 buckets of one range, so that range holds
    ~1.1e6 entries: the one-pass slot overflows, the exact build runs, and the range takes
    the global scatter.  Sampled query rows equal the oracle."""
    import fpmash
    rng = np.random.default_rng(n_ref + skew)
    members = 100
    lists = []
    for _ in range(n_ref // members):
        core = rng.integers(1, 2 ** 63, size=1100, dtype=np.uint64)
        pick = np.argpartition(rng.random((members, core.size)), 1000, axis=1)[:, :1000]
        lists += list(np.sort(core[pick], axis=1))
    if skew:
        narrow = np.unique(rng.integers(1 << 40, (1 << 40) + (1 << 46), size=4000, dtype=np.uint64))
        lists = [np.union1d(x, narrow[rng.integers(0, narrow.size, size=30)]) for x in lists]
    L = [len(x) * 5 for x in lists]
    qrows = list(range(0, n_ref, n_ref // 12))[:12]
    qry = [lists[r] for r in qrows]
    S = max(len(x) for x in lists)
    before = ctx.index_rebuilds()
    ctx.set_dist_mode(fpmash.DIST_SPARSE)
    try:
        nu, de, listed = ctx.dist_list(lists, qry, S, ref_lengths=L, qry_lengths=[L[r] for r in qrows],
                                       cap=1 << 20, expand=False)
        st = ctx.last_dist_stats()
    finally:
        ctx.set_dist_mode(fpmash.DIST_AUTO)
    assert st["sparse"]
    assert (ctx.index_rebuilds() > before) == skew
    onu, ode, _, _ = oracle.dist_grid(lists, L, qry, [L[r] for r in qrows], S, 21, 4.0 ** 21,
                                      threads=8, with_pvalue=False)
    assert np.array_equal(nu, onu) and np.array_equal(de, ode)


def test_index_exact_build_forced():
    """FPM_IDX_ONEPASS=0 (read at library load: a child process) forces the exact two-pass
    index build; the sorted and the -fp dist grids still equal the oracle."""
    import subprocess
    import sys
    code = r"""
import os, sys
sys.path[:0] = [%r, %r]
import numpy as np
import fpmash
from fpmash import datagen
from oracle import oracle as O
with fpmash.Context(0) as ctx:
    ctx.set_dist_mode(2)
    seqs = datagen.family_dna(6, 10, 1500, sub_rate=(0.0, 0.1), seed=7)
    sk = O.sketch_batch(O.params(k=21, s=300), seqs)
    L = [len(x) for x in seqs]
    d = ctx.dist(sk, sk, 300, ref_lengths=L, qry_lengths=L)
    nu, de, _, _ = O.dist_grid(sk, L, sk, L, 300, 21, 4.0 ** 21)
    assert np.array_equal(d["numer"], nu) and np.array_equal(d["denom"], de)
    rng = np.random.default_rng(3)
    fl = [rng.integers(0, 40, size=int(rng.integers(1, 300))).astype(np.uint32) for _ in range(50)]
    FL = [len(x) * 7 for x in fl]
    d = ctx.dist(fl, fl, 200, use64=False, k=1, kmer_space=10.0, ref_lengths=FL, qry_lengths=FL)
    nu, de, _, _ = O.dist_grid(fl, FL, fl, FL, 200, 1, 10.0, use64=False)
    assert np.array_equal(d["numer"], nu) and np.array_equal(d["denom"], de)
    assert ctx.index_rebuilds() == 0
print("exact-ok")
""" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
       os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fp-mash_amd"))
    env = dict(os.environ, FPM_IDX_ONEPASS="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "exact-ok" in r.stdout, r.stdout + r.stderr


def test_pvalue_asymptotic_branches_on_device(ctx, oracle):
    """Union sizes above 1e5 (pValue's sketch-size argument is the denominator): the device
    finalize takes GSL's asymptotic regimes of the incomplete beta like the oracle (pinned to
    mpmath by test_pvalue_asymptotic_branches_vs_mpmath), u32 counts through
    fpm_dist_finalize_dev, every cell rtol 1e-12."""
    import ctypes as C
    import fpmash
    L = fpmash.lib()
    rng = np.random.default_rng(11)
    cells = []
    for n in (100001, 100005, 250000, 1000000, 4000000):
        for x in range(0, 12):                  # small a (and its general neighbours)
            cells.append((x, n))
        for j in range(0, 12):                  # large a, small b
            cells.append((n - j, n))
    n_qry = len(cells)
    ref_len = np.array([5e3, 3e5, 5e6, 4.6e9, 1.2e11], dtype=np.uint64)
    qry_len = rng.choice(ref_len, size=n_qry).astype(np.uint64)
    n_ref = len(ref_len)
    numer = np.zeros((n_qry, n_ref), np.uint32)
    denom = np.zeros((n_qry, n_ref), np.uint32)
    for q, (x, n) in enumerate(cells):
        numer[q, :] = x
        denom[q, :] = n
    for k, space in ((21, 4.0 ** 21), (3, 4.0 ** 3), (9, 4.0 ** 9)):
        bufs = [fpmash.DeviceBuffer.from_array(ctx, a) for a in (numer, denom, ref_len, qry_len)]
        outs = [fpmash.DeviceBuffer(ctx, n_qry * n_ref * b) for b in (8, 8, 1)]
        fpmash._check(L.fpm_dist_finalize_dev(ctx.h, *[b.ptr for b in bufs], n_ref, n_qry, k,
                                              space, 1.0, 1.0, *[o.ptr for o in outs], None))
        ctx.synchronize()
        pv = outs[1].to_array(np.float64, n_qry * n_ref).reshape(n_qry, n_ref)
        exp = np.array([[oracle.pvalue(int(numer[q, r]), int(ref_len[r]), int(qry_len[q]), space,
                                       int(denom[q, r])) for r in range(n_ref)]
                        for q in range(n_qry)])
        np.testing.assert_allclose(pv, exp, rtol=RTOL, atol=0)
        for b in bufs + outs:
            b.free()


def test_refset_unsorted_query_block(ctx, oracle):
    """A resident set of sorted sketches against a block of UNSORTED query lists in the
    sparse mode: the probe runs without a count pass, finds the query rows out of order and
    the candidates take the literal walk (the reference's own walk on unsorted lists) instead
    of the rank kernel.  Every cell equals the oracle's grid; the same block with its lists
    sorted takes the rank kernel and matches too."""
    import ctypes as C
    import fpmash
    from fpmash import datagen
    rng = np.random.default_rng(41)
    seqs = datagen.family_dna(6, 10, 1500, sub_rate=(0.0, 0.1), seed=43)
    lists = oracle.sketch_batch(oracle.params(k=21, s=300), seqs)
    refs = lists[:30]
    S, k, space = 300, 21, 4.0 ** 21
    for shuffled in (True, False):
        qrys = []
        for x in lists[30:]:
            y = np.array(x, dtype=np.uint64)
            if shuffled:
                rng.shuffle(y)
            qrys.append(y)
        rl = [int(len(x)) * 5 + 900 for x in refs]
        ql = [int(len(x)) * 5 + 900 for x in qrys]
        w = max(len(x) for x in lists)
        R, rlen = fpmash._dense(refs, w, np.uint64)
        Q, qlen = fpmash._dense(qrys, w, np.uint64)
        L = fpmash.lib()
        bufs = [fpmash.DeviceBuffer.from_array(ctx, np.ascontiguousarray(a))
                for a in (R, rlen, np.array(rl, np.uint64), Q, qlen, np.array(ql, np.uint64))]
        nr, nq = len(refs), len(qrys)
        outs = [fpmash.DeviceBuffer(ctx, nr * nq * b) for b in (4, 4, 8, 8, 1)]
        ctx.set_dist_mode(2)
        h = C.c_void_p()
        try:
            fpmash._check(L.fpm_refset_create_dev(ctx.h, bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, w,
                                                  nr, 8, S, C.byref(h)))
            fpmash._check(L.fpm_refset_dist_dev(h, bufs[3].ptr, bufs[4].ptr, bufs[5].ptr, w, nq,
                                                S, 4, k, space, 1.0, 1.0,
                                                *[b.ptr for b in outs], None))
            ctx.synchronize()
            # 1: the literal walk of the candidates, 2: the rank kernel
            assert ctx.last_dist_stats()["sparse"] == (1 if shuffled else 2)
        finally:
            ctx.set_dist_mode(0)
            if h.value:
                L.fpm_refset_free(h)
        types = (np.uint32, np.uint32, np.float64, np.float64, np.uint8)
        got = [b.to_array(t, nr * nq) for b, t in zip(outs, types)]
        nu, de, di, pv = oracle.dist_grid(refs, rl, qrys, ql, S, k, space, use64=True)
        assert np.array_equal(got[0], nu.ravel()) and np.array_equal(got[1], de.ravel())
        np.testing.assert_allclose(got[2], di.ravel(), rtol=RTOL, atol=0)
        np.testing.assert_allclose(got[3], pv.ravel(), rtol=RTOL, atol=0)
        for b in bufs + outs:
            b.free()


@pytest.mark.parametrize("data", ["self", "other", "fp", "short"])
def test_dist_list_prefill(ctx, oracle, data, dist_mode):
    """fpm_dist_list_prefill before fpm_dist_list_dev (the counts written ahead as (0, S), the
    dist call correcting the pairs with la + lb < S and writing its cells after the prefill):
    the same counts and list as without it, equal to the oracle, in every dist mode; sorted
    sketches against themselves (symmetric path) and another set, unsorted -fp lists (the
    literal walk writes cells in place), short sketches (la + lb < S: the correction), and
    empty lists."""
    import fpmash
    from fpmash import datagen
    if data == "fp":
        rng = np.random.default_rng(43)
        sk = [rng.integers(0, 60, size=int(rng.integers(0, 400))).astype(np.uint32)
              for _ in range(90)]
        sk[5] = sk[5][:0]
        qsk = sk[::-1][:50]
        S, k, space, use64 = 300, 1, 10.0, False
        lens = np.array([len(x) * 3 + 7 for x in sk], np.uint64)
        qlens = lens[::-1][:50].copy()
    else:
        P = fpmash.make_params(k=21, s=500)
        if data == "short":
            rng = np.random.default_rng(5)
            seqs = [bytes(rng.choice(list(b"ACGT"), size=int(rng.integers(15, 700))))
                    for _ in range(70)]
            seqs += datagen.family_dna(2, 10, 900, sub_rate=(0.0, 0.05), seed=6)
        else:
            seqs = datagen.family_dna(8, 12, 1500, sub_rate=(0.0, 0.08), seed=31)
            seqs += [b"N" * 300, b"", b"ACGT" * 3]
        sk = ctx.sketch(P, seqs)
        qsk = sk if data in ("self", "short") else sk[::-1][:60]
        S, k, space, use64 = 500, 21, 4.0 ** 21, True
        lens = np.array([len(x) for x in seqs], np.uint64)
        qlens = lens if qsk is sk else lens[::-1][:60].copy()
    kw = dict(use64=use64, k=k, kmer_space=space, ref_lengths=lens, qry_lengths=qlens)
    a = ctx.dist_list(sk, qsk, S, prefill=True, **kw)
    b = ctx.dist_list(sk, qsk, S, **kw)
    for key in ("numer", "denom", "distance", "pvalue", "pass"):
        assert np.array_equal(a[key], b[key]), key
    nu, de, _, _ = oracle.dist_grid(sk, list(lens), qsk, list(qlens), S, k, space, use64=use64,
                                    with_pvalue=False)
    assert np.array_equal(a["numer"], nu) and np.array_equal(a["denom"], de)
    if data == "short":
        assert (de < S).sum() > 100          # the correction rewrote these


def test_dist_list_prefill_not_taken_over(ctx, oracle):
    """A prefill whose grid the next dist call does not write: that call waits for it, its own
    grid is exact, and the prefilled grid holds (0, S) after the stream work; a second prefill
    while one is pending orders the first before the caller's stream."""
    import fpmash
    from fpmash import datagen
    P = fpmash.make_params(k=21, s=400)
    seqs = datagen.family_dna(5, 10, 1200, sub_rate=(0.0, 0.05), seed=12)
    sk = ctx.sketch(P, seqs)
    n = len(sk)
    lens = [len(x) for x in seqs]
    L = fpmash.lib()
    spare = [fpmash.DeviceBuffer(ctx, 64 * 64 * 2) for _ in range(4)]
    fpmash._check(L.fpm_dist_list_prefill(ctx.h, spare[0].ptr, spare[1].ptr, 64, 64, 300, None))
    fpmash._check(L.fpm_dist_list_prefill(ctx.h, spare[2].ptr, spare[3].ptr, 64, 64, 400, None))
    d = ctx.dist_list(sk, sk, 400, ref_lengths=lens, qry_lengths=lens)
    ctx.synchronize()
    nu, de, _, _ = oracle.dist_grid(sk, lens, sk, lens, 400, 21, 4.0 ** 21, with_pvalue=False)
    assert np.array_equal(d["numer"], nu) and np.array_equal(d["denom"], de)
    for i, S in ((0, 300), (2, 400)):
        assert not spare[i].to_array(np.uint16, 64 * 64).any()
        assert (spare[i + 1].to_array(np.uint16, 64 * 64) == S).all()
    for b in spare:
        b.free()
    assert n > 0
