"""kseq record rules (kseq.h:170-208) in Python — test support for fixture parity.

Records start at '>' or '@'; name = bytes up to the first isspace; comment = rest
of the header line (a trailing '\r' kept); sequence = isgraph bytes until the next
'>', '+' or '@'; for FASTQ, after the '+' line exactly len(seq) quality bytes in
33..127 are consumed (plus one terminator byte).
"""
import gzip


def _isspace(c):
    return c in b" \t\n\v\f\r"


def read_records(path):
    data = gzip.open(path, "rb").read() if path.endswith(".gz") else open(path, "rb").read()
    return parse(data)


def parse(data: bytes):
    recs = []
    n = len(data)
    i = 0
    last = 0
    while True:
        if last == 0:
            while i < n and data[i] not in b">@":
                i += 1
            if i >= n:
                return recs
            i += 1
        if i >= n:
            return recs
        j = i
        while j < n and not _isspace(data[j]):
            j += 1
        name = data[i:j]
        comment = b""
        if j < n:
            c = data[j]
            i = j + 1
            if c != 10:
                k = data.find(b"\n", i)
                k = n if k < 0 else k
                comment = data[i:k]
                i = k + 1
        else:
            i = n
        seq = bytearray()
        c = None
        while i < n:
            c = data[i]
            i += 1
            if c in b">+@":
                break
            if 33 <= c <= 126:
                seq.append(c)
            c = None
        if c is not None and c in b">@":
            last = c
        else:
            last = 0
        if c is not None and c == ord("+"):
            k = data.find(b"\n", i)
            if k < 0:
                raise ValueError("truncated quality")
            i = k + 1
            q = 0
            while i < n and q < len(seq):
                if 33 <= data[i] <= 127:
                    q += 1
                i += 1
            if i < n:
                i += 1   # kseq consumes the byte after the last quality char
            if q != len(seq):
                raise ValueError("quality shorter than sequence")
            last = 0
        recs.append((bytes(name), bytes(comment), bytes(seq)))
        if c is None and i >= n:
            return recs
