"""GPU parity of the device FASTA parser (csrc/seqparse.hip, fpm_seq_parse) against the
kseq record rules (kseq.h:170-208) restated in tests/seqio.py, and of sketches of the
parsed records against the oracle.  Records, names, comments and sequence lengths must be
identical; sketches bit-exact."""
import numpy as np
import pytest

import seqio

pytestmark = pytest.mark.gpu


def device_records(ctx, files):
    """[(name, comment, length)] per file from the device parse, dropping a marker that is
    a file's last byte (kseq_read's name read returns -1 there)."""
    job, rec, quality = ctx.seq_parse(files)
    try:
        out = [[] for _ in files]
        for r in range(len(rec["seq_len"])):
            f = int(rec["seg"][r])
            o, hl = int(rec["hdr_off"][r]), int(rec["hdr_len"][r])
            if o + 1 >= len(files[f]):
                continue
            line = files[f][o + 1:o + hl]
            i = 0
            while i < len(line) and line[i] not in b" \t\n\v\f\r":
                i += 1
            name = line[:i]
            comment = line[i + 1:] if i < len(line) else b""
            out[f].append((name, comment, int(rec["seq_len"][r])))
        return out, quality, job
    except Exception:
        ctx.seq_free(job)
        raise


def expected(files):
    return [[(n, c, len(s)) for n, c, s in seqio.parse(f)] for f in files]


def fasta(rng, n_rec, lo, hi, width=70, crlf=False, lower=0.0):
    out = bytearray()
    nl = b"\r\n" if crlf else b"\n"
    for i in range(n_rec):
        L = int(rng.integers(lo, hi + 1))
        seq = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, L)].copy()
        if lower:
            m = rng.random(L) < lower
            seq[m] += 32
        out += b">r%d some comment %d" % (i, i) + nl
        s = seq.tobytes()
        for j in range(0, len(s), width):
            out += s[j:j + width] + nl
    return bytes(out)


EDGE = [
    b"",
    b">",
    b"\n\n>a\nACGT",
    b"preamble text\nmore ACGT\n>x desc\nACGT\nAC GT\n\nTTT>y\nGGG>z inline > marker\nCC",
    b">a\tcomment with tab\nACGT\r\nACGT\r\n>b\r\nAAAA",
    b">a b>c @d\nAC>GT\n@q hdr\nTTTT\n>\n>empty\n>last",
    b">only header",
    b"@r1 x\nACGT\n@r2\nGGGG\n",
    b">n\x00ul\nAC\x00GT\x80\xffAC\n",
    b">a\n" + b"ACGT" * 3000 + b"\n>b\n" + b"T" * 4095 + b"\n",
]


@pytest.mark.parametrize("i", range(len(EDGE)))
def test_seq_parse_edge_cases(ctx, i):
    files = [EDGE[i]]
    got, quality, job = device_records(ctx, files)
    ctx.seq_free(job)
    assert not quality
    assert got == expected(files)


def test_seq_parse_many_files_and_chunk_boundaries(ctx):
    rng = np.random.default_rng(11)
    files = [fasta(rng, 30, 0, 300), fasta(rng, 5, 4000, 9000, width=61, crlf=True),
             b"", b"x" * 4096, fasta(rng, 200, 1, 50, width=7, lower=0.3),
             b">a\n" + b"C" * (4096 - 4), fasta(rng, 3, 100000, 120000, width=80)]
    got, quality, job = device_records(ctx, files)
    ctx.seq_free(job)
    assert not quality
    assert got == expected(files)


def test_seq_parse_flags_fastq(ctx):
    files = [b">a\nACGT\n", b"@r1\nACGT\n+\nIIII\n@r2\nGG\n+\nII\n"]
    _got, quality, job = device_records(ctx, files)
    ctx.seq_free(job)
    assert quality


@pytest.mark.parametrize("per_record", [True, False])
def test_seq_parse_sketch_matches_oracle(ctx, oracle, per_record):
    """Sketches of the device-packed records equal the oracle's sketches of the records
    seqio finds: -i (one per record >= k) and concatenated (one per file)."""
    import fpmash
    rng = np.random.default_rng(5)
    files = [fasta(rng, 40, 0, 3000, lower=0.1), fasta(rng, 2, 30000, 70000, width=60),
             b">short\nACG\n>x\n" + b"ACGTTGCA" * 500 + b"\n", fasta(rng, 300, 10, 400)]
    k, s = 21, 1000
    job, rec, quality = ctx.seq_parse(files)
    assert not quality
    exp_recs = [seqio.parse(f) for f in files]
    groups = np.full(len(rec["seq_len"]), fpmash.NO_GROUP, np.uint32)
    want_groups = []
    g = 0
    r = 0
    for f, recs in enumerate(exp_recs):
        members = []
        for (_n, _c, sq) in recs:
            # device records line up with seqio's (no trailing bare marker in these files)
            assert int(rec["seq_len"][r]) == len(sq)
            if len(sq) >= k:
                if per_record:
                    groups[r] = g
                    want_groups.append([sq])
                    g += 1
                else:
                    members.append(sq)
            r += 1
        if not per_record:
            if members:
                groups[r - len(recs):r] = [g if len(sq) >= k else fpmash.NO_GROUP
                                           for (_n, _c, sq) in recs]
                want_groups.append(members)
                g += 1
    assert r == len(rec["seq_len"])
    P = fpmash.make_params(k=k, s=s)
    try:
        got = ctx.sketch_seq(P, job, groups, g)
    finally:
        ctx.seq_free(job)
    O = oracle.params(k=k, s=s)
    flat, grp = [], []
    for gi, mem in enumerate(want_groups):
        flat += mem
        grp += [gi] * len(mem)
    exp = oracle.sketch_batch(O, flat, groups=grp, n_groups=len(want_groups))
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        assert np.array_equal(a, b)
