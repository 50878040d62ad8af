"""kseq record rules (kseq.h:170-208) in Python — test support for fixture parity, itself
pinned to the reference's kseq.h compiled into oracle/_ref (tests/test_kseq_oracle.py).

Records start at '>' or '@'; name = bytes up to the first isspace; comment = rest
of the header line (a trailing '\r' kept); sequence = isgraph bytes until the next
'>', '+' or '@'; for FASTQ, after the '+' line exactly len(seq) quality bytes in
33..127 are consumed (plus one terminator byte).  A 0xff byte reads as end of file in
kseq's getc (signed char).
"""
import gzip


def _isspace(c):
    return c in b" \t\n\v\f\r"


def read_records(path):
    data = gzip.open(path, "rb").read() if path.endswith(".gz") else open(path, "rb").read()
    return parse(data)


def parse(data: bytes):
    """kseq_read in a loop over `data` (records until it returns -1).  ks_getc returns
    (int)buf[i] of a `char *` buffer: on x86 a 0xff byte reads as -1 (end of file) in the
    skip, sequence, '+' and quality loops; the name / comment reads scan the buffer directly.
    Raises ValueError where kseq_read returns -2 (truncated quality)."""
    n = len(data)
    pos = 0

    def getc():
        nonlocal pos
        if pos >= n:
            return -1
        c = data[pos]
        pos += 1
        return -1 if c == 0xFF else c

    def getuntil(space):
        # ks_getuntil: -1 only when the stream is already at its end; the delimiter consumed
        nonlocal pos
        if pos >= n:
            return None, 0
        j = pos
        if space:
            while j < n and not _isspace(data[j]):
                j += 1
        else:
            while j < n and data[j] != 10:
                j += 1
        s = data[pos:j]
        if j < n:
            d = data[j]
            pos = j + 1
        else:
            d = 0
            pos = n
        return s, d

    recs = []
    last = 0
    while True:
        if last == 0:
            c = getc()
            while c != -1 and c not in (62, 64):
                c = getc()
            if c == -1:
                return recs
            last = c
        name, d = getuntil(True)
        if name is None:
            return recs
        comment = b""
        if d != 10:
            cm, _ = getuntil(False)
            comment = cm if cm is not None else b""
        seq = bytearray()
        c = getc()
        while c != -1 and c not in (62, 43, 64):
            if 33 <= c <= 126:
                seq.append(c)
            c = getc()
        if c in (62, 64):
            last = c
        if c != 43:
            recs.append((bytes(name), bytes(comment), bytes(seq)))
            continue
        c = getc()
        while c != -1 and c != 10:
            c = getc()
        if c == -1:
            raise ValueError("truncated quality")
        q = 0
        c = getc()
        while c != -1 and q < len(seq):
            if 33 <= c <= 127:
                q += 1
            c = getc()
        last = 0
        if q != len(seq):
            raise ValueError("quality shorter than sequence")
        recs.append((bytes(name), bytes(comment), bytes(seq)))
