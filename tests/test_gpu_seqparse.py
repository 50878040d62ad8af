"""GPU parity of the device FASTA / FASTQ parser (csrc/seqparse.hip, fpm_seq_parse) against
the reference's kseq.h compiled into oracle/_ref (kseq_read over the file, as
Sketch.cpp:478-522 reads it; tests/seqio.py, the Python restatement pinned to it, where
oracle/_ref is absent), and of sketches of the parsed records against the oracle.  Records,
names, comments and sequence lengths must be identical; sketches bit-exact."""
import gzip
import os
import tempfile

import numpy as np
import pytest

import seqio
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def kseq_records(data):
    """[(name, comment, seq)] of kseq_read over `data`: the compiled kseq.h when built, else
    seqio; None where kseq_read returns -2 (truncated quality)."""
    from oracle import oracle as O
    if O.ref() is None:
        try:
            return seqio.parse(data)
        except ValueError:
            return None
    with tempfile.NamedTemporaryFile(suffix=".fq", delete=False) as f:
        f.write(data)
    try:
        recs, st = O.ref_kseq_records(f.name)
    finally:
        os.unlink(f.name)
    return None if st == -2 else [(n, c, s) for n, c, s, _q in recs]


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
    return [[(n, c, len(s)) for n, c, s in kseq_records(f)] for f in files]


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


def fastq(rng, n_rec, lo, hi, crlf=False, at_rate=0.0):
    out = bytearray()
    nl = b"\r\n" if crlf else b"\n"
    for i in range(n_rec):
        L = int(rng.integers(lo, hi + 1))
        seq = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, L)].tobytes()
        q = rng.integers(35, 74, L).astype(np.uint8)
        if at_rate:
            q[rng.random(L) < at_rate] = ord("@")      # Q31 in Phred+33: '@' in quality lines
        out += b"@r%d/1 len=%d" % (i, L) + nl + seq + nl + b"+" + nl + q.tobytes() + nl
    return bytes(out)


FASTQ_OK = [
    b"@r1 x\nACGT\n+\nIIII\n@r2\nGGGG\n+r2\nII@I\n",
    b"@r1\r\nACGT\r\n+\r\nIIII\r\n@r2\r\nGG\r\n+\r\nII\r\n",
    b"@e\n\n+\n\n@f\nA\n+\nI",
    b"@r1\nAC GT\n+\nI I I I\n",
    b"@h\xff1 c\nACGT\n+\nIIII\n\n\n",
]
FASTQ_HOST = [
    b"@r1\nAC\nGT\n+\nII\nII\n@r2\nA\n+\nI\n",        # multi-line: host walk
    b"@r1\nACGT\n+\nIIII@x\n>y\nAC\n",                    # quality longer than the bases
    b"@r1\nAC\xffGT\n+\nIIII\n",                          # 0xff in the sequence line
    b"junk\n@r1\nACGT\n+\nIIII\n",                         # bytes before the first header
]


@pytest.mark.parametrize("i", range(len(FASTQ_OK)))
def test_fastq_device_parse(ctx, i):
    """4-line FASTQ (CRLF, '@' in quality, empty records, spaces, 0xff in a header) parsed on
    the device == kseq_read's records; no host walk needed."""
    files = [FASTQ_OK[i]]
    got, quality, job = device_records(ctx, files)
    ctx.seq_free(job)
    assert not quality
    assert got == expected(files)


@pytest.mark.parametrize("i", range(len(FASTQ_HOST)))
def test_fastq_not_four_line_goes_to_host(ctx, i):
    """FASTQ that kseq_read does not read the 4-line way is handed back to the host walk."""
    _got, quality, job = device_records(ctx, [FASTQ_HOST[i]])
    ctx.seq_free(job)
    assert quality


def test_fastq_fixtures_and_random_device_parse(ctx, oracle):
    """reads1/2.fastq.gz (the fork's fixtures, inflated) and random FASTQ with '@'-rich quality
    and CRLF, several files in one parse: records == kseq_read's, and the -i sketches of the
    device-packed records == the oracle's."""
    import fpmash
    rng = np.random.default_rng(9)
    files = [gzip.open(os.path.join(GOLDEN, "reads1.fastq.gz")).read(),
             fastq(rng, 500, 0, 400, at_rate=0.2),
             gzip.open(os.path.join(GOLDEN, "reads2.fastq.gz")).read(),
             fastq(rng, 50, 2000, 9000, crlf=True)]
    got, quality, job = device_records(ctx, files)
    try:
        assert not quality
        exp = [kseq_records(f) for f in files]
        assert got == [[(n, c, len(s)) for n, c, s in e] for e in exp]
        flat = [s for e in exp for _n, _c, s in e]
        groups = np.array([i if len(s) >= 21 else fpmash.NO_GROUP for i, s in enumerate(flat)],
                          np.uint32)
        keep = [s for s in flat if len(s) >= 21]
        g = np.cumsum(groups != fpmash.NO_GROUP) - 1
        groups = np.where(groups == fpmash.NO_GROUP, groups, g).astype(np.uint32)
        sk = ctx.sketch_seq(fpmash.make_params(k=21, s=1000), job, groups, len(keep))
    finally:
        ctx.seq_free(job)
    want = oracle.sketch_batch(oracle.params(k=21, s=1000), keep)
    assert len(sk) == len(want)
    for a, b in zip(sk, want):
        assert np.array_equal(a, b)
