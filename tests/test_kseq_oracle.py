"""The kseq record rules: tests/seqio.py (the Python restatement the device parser was first
pinned to) against the reference's own kseq.h compiled into oracle/_ref (kseq_read over
gzopen, as Sketch.cpp:478-522 reads a file), on FASTA / FASTQ edge cases, random files and
the fork's FASTQ fixtures.  CPU only; skipped when oracle/_ref is not built."""
import gzip
import os

import numpy as np
import pytest

import seqio
from conftest import GOLDEN

O = pytest.importorskip("oracle.oracle")
pytestmark = pytest.mark.skipif(O.ref() is None, reason="oracle/_ref not built")

FASTA_EDGE = [
    b"",
    b">",
    b"\n\n>a\nACGT",
    b"preamble text\nmore ACGT\n>x desc\nACGT\nAC GT\n\nTTT>y\nGGG>z inline > marker\nCC",
    b">a\tcomment with tab\nACGT\r\nACGT\r\n>b\r\nAAAA",
    b">a b>c @d\nAC>GT\n@q hdr\nTTTT\n>\n>empty\n>last",
    b">only header",
    b">n\x00ul\nAC\x00GT\x80\xffAC\n",
]
FASTQ_EDGE = [
    b"@r1 x\nACGT\n+\nIIII\n@r2\nGGGG\n+r2\nII@I\n",           # '@' inside a quality line
    b"@r1\r\nACGT\r\n+\r\nIIII\r\n@r2\r\nGG\r\n+\r\nII\r\n",  # CRLF
    b"@r1\nAC\nGT\n+\nII\nII\n@r2\nA\n+\nI\n",                 # multi-line records
    b"@r1\nACGT\n+\nII",                                       # truncated quality
    b"@r1\nACGT\n+",                                           # '+' line at EOF
    b"@e\n\n+\n\n@f\nA\n+\nI",                                 # empty sequence, no final '\n'
    b"@r1\nACGT\n+\nIIII@x\n>y\nAC\n",                         # quality longer than the bases
    b"@r1\nAC GT\n+\nI I I I\n",                               # spaces in both lines
]


def _kseq(tmp_path, data):
    p = tmp_path / "x.fq"
    p.write_bytes(data)
    return O.ref_kseq_records(str(p))


def _seqio(data):
    try:
        return [(n, c, s) for n, c, s in seqio.parse(data)], -1
    except ValueError:
        return None, -2


@pytest.mark.parametrize("data", FASTA_EDGE + FASTQ_EDGE)
def test_seqio_equals_compiled_kseq(tmp_path, data):
    recs, st = _kseq(tmp_path, data)
    got, gst = _seqio(data)
    if st == -2:
        # truncated quality: kseq_read returns -2 (the records before it are read)
        assert gst == -2
        return
    assert got == [(n, c, s) for n, c, s, _q in recs]


def test_seqio_equals_compiled_kseq_random(tmp_path):
    rng = np.random.default_rng(3)
    for t in range(30):
        out = bytearray()
        for i in range(int(rng.integers(1, 30))):
            L = int(rng.integers(0, 200))
            seq = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, L)].tobytes()
            if t % 2:
                q = bytes(rng.integers(33, 75, L).astype(np.uint8))
                out += b"@r%d c%d\n%s\n+\n%s\n" % (i, i, seq, q)
            else:
                out += b">r%d c%d\n" % (i, i)
                for j in range(0, len(seq), 60):
                    out += seq[j:j + 60] + b"\n"
        recs, st = _kseq(tmp_path, bytes(out))
        assert st == -1
        assert _seqio(bytes(out))[0] == [(n, c, s) for n, c, s, _q in recs]


@pytest.mark.parametrize("name", ["reads1.fastq.gz", "reads2.fastq.gz"])
def test_fastq_fixtures_compiled_kseq(name):
    path = os.path.join(GOLDEN, name)
    recs, st = O.ref_kseq_records(path)
    assert st == -1 and len(recs) == 1000
    assert seqio.read_records(path) == [(n, c, s) for n, c, s, _q in recs]
    assert all(len(q) == len(s) for _n, _c, s, q in recs)
    assert gzip.open(path).read().count(b"\n+") >= 1000
