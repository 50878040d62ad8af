"""ctypes wrapper of the oracle — TEST INFRASTRUCTURE ONLY.

Loads oracle/liboracle.so (the C restatement, fpm_oracle.c) and, when present,
oracle/_ref/libfpmref.so (the reference's own hashing/MinHashHeap sources built by
oracle/Makefile).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module; the product never does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
f64p = C.POINTER(C.c_double)


class Params(C.Structure):
    _fields_ = [
        ("kmer_size", C.c_int),
        ("sketch_size", C.c_uint64),
        ("seed", C.c_uint32),
        ("use64", C.c_int),
        ("noncanonical", C.c_int),
        ("preserve_case", C.c_int),
        ("alphabet", C.c_ubyte * 256),
    ]


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_get_hash.restype = C.c_uint64
        L.orc_get_hash.argtypes = [C.c_char_p, C.c_int, C.c_uint32, C.c_int]
        L.orc_get_hash_fp.restype = C.c_uint64
        L.orc_get_hash_fp.argtypes = [u64p, C.c_uint64, C.c_uint32, C.c_int]
        L.orc_set_alphabet.argtypes = [C.POINTER(Params), C.c_char_p]
        L.orc_sketch_batch.restype = C.c_int
        L.orc_sketch_batch.argtypes = [C.POINTER(Params), C.c_char_p, u64p, C.c_uint32, u32p,
                                       C.c_uint32, u64p, u32p, u32p, C.c_int]
        L.orc_fp_parse.restype = C.c_uint64
        L.orc_fp_parse.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, u64p, C.c_uint64,
                                   C.c_uint64, u64p, u32p, u64p, u64p]
        L.orc_compare.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int,
                                  C.c_uint64, u64p, u64p]
        L.orc_distance.restype = C.c_double
        L.orc_distance.argtypes = [C.c_uint64, C.c_uint64, C.c_int]
        L.orc_pvalue.restype = C.c_double
        L.orc_pvalue.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_double, C.c_uint64]
        L.orc_binomial_q.restype = C.c_double
        L.orc_binomial_q.argtypes = [C.c_uint64, C.c_double, C.c_uint64]
        L.orc_positional.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int,
                                     u64p, u64p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_write_dist_text.restype = C.c_int
        L.orc_write_dist_text.argtypes = [C.c_char_p, C.c_char_p, u64p, C.c_uint32, u32p,
                                          C.c_uint32, u32p, u32p, f64p, f64p, C.c_void_p,
                                          C.c_int]
        L.orc_dist_grid.restype = C.c_int
        L.orc_dist_grid.argtypes = [C.c_void_p, u32p, u64p, C.c_uint64, C.c_uint32,
                                    C.c_void_p, u32p, u64p, C.c_uint64, C.c_uint32,
                                    C.c_int, C.c_uint64, C.c_int, C.c_double,
                                    u32p, u32p, f64p, f64p, C.c_int]
        _LIB = L
    return _LIB


def ref():
    """The reference's own sources (oracle/_ref); None when not built."""
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "libfpmref.so")
        if not os.path.exists(path):
            return None
        R = C.CDLL(path)
        R.ref_get_hash.restype = C.c_ulonglong
        R.ref_get_hash.argtypes = [C.c_char_p, C.c_int, C.c_uint, C.c_int]
        R.ref_get_hash_fp.restype = C.c_ulonglong
        R.ref_get_hash_fp.argtypes = [u64p, C.c_ulonglong, C.c_uint, C.c_int]
        R.ref_minhash_stream.restype = C.c_ulonglong
        R.ref_minhash_stream.argtypes = [u64p, C.c_ulonglong, C.c_int, C.c_ulonglong, u64p, u32p]
        R.ref_sketch_records.restype = C.c_ulonglong
        R.ref_sketch_records.argtypes = [C.c_char_p, u64p, C.c_uint, C.c_int, C.c_ulonglong,
                                         C.c_uint, C.c_int, C.c_int, C.c_int, C.c_char_p,
                                         u64p, u32p]
        R.ref_sketch_batch_mt.restype = None
        R.ref_sketch_batch_mt.argtypes = [C.c_char_p, u64p, C.c_uint, C.c_int, C.c_ulonglong,
                                          C.c_uint, C.c_int, C.c_int, C.c_int, C.c_char_p,
                                          C.c_int, u64p, u64p]
        R.ref_kseq_records.restype = C.c_void_p
        R.ref_kseq_records.argtypes = [C.c_char_p, u64p, C.POINTER(C.c_int), u64p]
        R.ref_kseq_scan.restype = C.c_int
        R.ref_kseq_scan.argtypes = [C.c_char_p, u64p, u64p]
        R.ref_fp_sketch_file.restype = C.c_longlong
        R.ref_fp_sketch_file.argtypes = [C.c_char_p, C.c_ulonglong, u64p, C.c_uint, C.c_int, u64p]
        R.ref_free.argtypes = [C.c_void_p]
        _REF = R
    return _REF


def _p(a, t):
    return a.ctypes.data_as(t)


def ref_sketch_batch(seqs, k=21, s=1000, seed=42, threads=1):
    """-i sketches of `seqs` through the reference's own getHash + MinHashHeap (oracle/_ref,
    the addMinHashes walk re-driven around them), one heap per record, records taken in turn
    by `threads` C++ threads (ref_sketch_batch_mt: one call for the whole batch, no Python
    dispatch per record).  None when oracle/_ref is not built."""
    R = ref()
    if R is None:
        return None
    alpha = bytearray(256)
    for c in b"ACGT":
        alpha[c] = 1
    alpha = bytes(alpha)
    use64 = int(4.0 ** k > 2.0 ** 32)
    buf, off = pack_records(seqs)
    out = np.zeros((len(seqs), s), np.uint64)
    cnt = np.zeros(len(seqs), np.uint64)
    R.ref_sketch_batch_mt(buf, _p(off, u64p), len(seqs), k, s, seed, use64, 0, 0, alpha,
                          max(1, threads), _p(out, u64p), _p(cnt, u64p))
    return [out[i, :int(cnt[i])] for i in range(len(seqs))]


def ref_kseq_records(path):
    """The reference's kseq.h reader (oracle/_ref: kseq_read over gzopen, as
    Sketch.cpp:478-522 reads a file): ([(name, comment, seq, qual) bytes], last kseq_read
    return: -1 clean end, -2 truncated quality).  None when oracle/_ref is not built."""
    R = ref()
    if R is None:
        return None
    n, st, nb = C.c_uint64(), C.c_int(), C.c_uint64()
    p = R.ref_kseq_records(os.fsencode(path), C.byref(n), C.byref(st), C.byref(nb))
    if not p:
        raise OSError(f"kseq: cannot open {path}")
    try:
        raw = C.string_at(p, nb.value)
    finally:
        R.ref_free(p)
    recs, at = [], 0
    for _ in range(n.value):
        f = []
        for _ in range(4):
            ln = int.from_bytes(raw[at:at + 8], "little")
            f.append(raw[at + 8:at + 8 + ln])
            at += 8 + ln
        recs.append(tuple(f))
    return recs, st.value


def ref_fp_sketch_files(paths, limit=1_000_000, seed=42, use64=False):
    """initFromFingerprints' per-file loop (istringstream parse, the reference's compiled
    getHashFingerPrint, HashList::add) over `paths` on one thread, the line budget shared as
    in one call: (references, lines, hash checksum), or None when oracle/_ref is not built.
    A timing source for the CPU same-work leg of `sketch -fp`, not a parity source."""
    R = ref()
    if R is None:
        return None
    used, hsum, refs = C.c_uint64(0), C.c_uint64(0), 0
    for path in paths:
        n = R.ref_fp_sketch_file(os.fsencode(path), limit, C.byref(used), seed, int(use64),
                                 C.byref(hsum))
        if n < 0:
            raise OSError(f"cannot open {path}")
        refs += n
    return refs, used.value, hsum.value


def ref_kseq_scan(path):
    """kseq_read + the per-record sequence copy over a file (the reference's input step):
    (records, bases), or None when oracle/_ref is not built."""
    R = ref()
    if R is None:
        return None
    n, b = C.c_uint64(), C.c_uint64()
    rc = R.ref_kseq_scan(os.fsencode(path), C.byref(n), C.byref(b))
    if rc == -3:
        raise OSError(f"kseq: cannot open {path}")
    return n.value, b.value


def params(k=21, s=1000, seed=42, alphabet="ACGT", noncanonical=False, preserve_case=False):
    """Sketch::Parameters as sketchParameterSetup (sketchParameterSetup.cpp:9-126) builds them."""
    P = Params()
    P.kmer_size = k
    P.sketch_size = s
    P.seed = seed
    P.noncanonical = int(noncanonical)
    P.preserve_case = int(preserve_case)
    lib().orc_set_alphabet(C.byref(P), alphabet.encode())
    return P


def fp_params(s=1000, seed=42):
    """-fp forces k=1, noncanonical, alphabet 0123456789 (sketchParameterSetup.cpp:78-84)."""
    return params(k=1, s=s, seed=seed, alphabet="0123456789", noncanonical=True)


def get_hash(data: bytes, seed=42, use64=True) -> int:
    return lib().orc_get_hash(data, len(data), seed, int(use64))


def get_hash_fp(vals, seed=42, use64=False) -> int:
    v = np.ascontiguousarray(vals, dtype=np.uint64)
    return lib().orc_get_hash_fp(_p(v, u64p), len(v), seed, int(use64))


def pack_records(seqs):
    """list[bytes] -> (concatenated bytes, offsets u64[n+1])."""
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    return b"".join(seqs), off


def sketch_batch(P, seqs, groups=None, n_groups=None, threads=1, counts=False):
    """Bottom-s sketches of records; returns list of u64 arrays (and counts)."""
    data, off = pack_records(seqs)
    n_rec = len(seqs)
    if groups is not None:
        g = np.ascontiguousarray(groups, dtype=np.uint32)
        ng = int(n_groups if n_groups is not None else (g.max() + 1 if n_rec else 0))
        gp = _p(g, u32p)
    else:
        ng, gp = n_rec, None
    s = int(P.sketch_size)
    out = np.zeros(max(ng, 1) * s, dtype=np.uint64)
    cnt = np.zeros(max(ng, 1), dtype=np.uint32)
    mult = np.zeros(max(ng, 1) * s, dtype=np.uint32) if counts else None
    rc = lib().orc_sketch_batch(C.byref(P), data, _p(off, u64p), n_rec, gp, ng,
                                _p(out, u64p), _p(cnt, u32p),
                                _p(mult, u32p) if counts else None, threads)
    assert rc == 0
    res = [out[i * s:i * s + cnt[i]].copy() for i in range(ng)]
    if counts:
        return res, [mult[i * s:i * s + cnt[i]].copy() for i in range(ng)]
    return res


def fp_parse(text: bytes, limit=1_000_000, lines_used=0):
    """-> (ids list[bytes], values list[np.uint64 array], lines_used)."""
    n_max = text.count(b"\n") + 1
    v_max = len(text) // 2 + 1
    id_off = np.zeros(n_max, dtype=np.uint64)
    id_len = np.zeros(n_max, dtype=np.uint32)
    vals = np.zeros(v_max, dtype=np.uint64)
    lvo = np.zeros(n_max + 1, dtype=np.uint64)
    used = C.c_uint64(lines_used)
    n = lib().orc_fp_parse(text, len(text), limit, C.byref(used), n_max, v_max,
                           _p(id_off, u64p), _p(id_len, u32p), _p(vals, u64p), _p(lvo, u64p))
    ids = [text[int(id_off[i]):int(id_off[i]) + int(id_len[i])] for i in range(n)]
    vl = [vals[int(lvo[i]):int(lvo[i + 1])].copy() for i in range(n)]
    return ids, vl, used.value


def fp_references(text: bytes, seed=42, limit=1_000_000, lines_used=0, last_id=b""):
    """Sketch::initFromFingerprints (Sketch.cpp:56-151) for one file:
    -> list of (name, length, u32 hashes in file order), lines_used, last_id."""
    ids, vals, used = fp_parse(text, limit, lines_used)
    refs = []
    cur = None
    for i, v in zip(ids, vals):
        if i != last_id:
            if cur is not None:
                refs.append(cur)
            cur = [i, len(v), []]
            last_id = i
        if cur is None:
            # the reference dereferences a null Reference here (Sketch.cpp:131)
            raise RuntimeError("fingerprint line continues an ID from a previous file")
        cur[2].append(get_hash_fp(v, seed, use64=False))
        cur[1] += len(v)
    if cur is not None:
        refs.append(cur)
    return [(n, l, np.array(h, dtype=np.uint32)) for n, l, h in refs], used, last_id


def compare(a, b, sketch_size, use64=True):
    a = np.ascontiguousarray(a, dtype=np.uint64 if use64 else np.uint32)
    b = np.ascontiguousarray(b, dtype=np.uint64 if use64 else np.uint32)
    nu, de = C.c_uint64(), C.c_uint64()
    lib().orc_compare(a.ctypes.data, len(a), b.ctypes.data, len(b), int(use64), sketch_size,
                      C.byref(nu), C.byref(de))
    return nu.value, de.value


def positional(a, b, use64=False):
    """triangle -fp compareFingerprints: (matches, min_len, distance, pvalue)."""
    a = np.ascontiguousarray(a, dtype=np.uint64 if use64 else np.uint32)
    b = np.ascontiguousarray(b, dtype=np.uint64 if use64 else np.uint32)
    m, n = C.c_uint64(), C.c_uint64()
    d, p = C.c_double(), C.c_double()
    lib().orc_positional(a.ctypes.data, len(a), b.ctypes.data, len(b), int(use64), C.byref(m),
                         C.byref(n), C.byref(d), C.byref(p))
    return m.value, n.value, d.value, p.value


def distance(common, denom, k):
    return lib().orc_distance(common, denom, k)


def pvalue(x, len_ref, len_qry, kmer_space, sketch_size):
    return lib().orc_pvalue(x, len_ref, len_qry, kmer_space, sketch_size)


def binomial_q(k, p, n):
    return lib().orc_binomial_q(k, p, n)


def dense(lists, width, dtype):
    m = np.zeros((len(lists), max(width, 1)), dtype=dtype)
    lens = np.zeros(len(lists), dtype=np.uint32)
    for i, l in enumerate(lists):
        m[i, :len(l)] = l
        lens[i] = len(l)
    return m, lens


def dist_grid(ref_lists, ref_lengths, qry_lists, qry_lengths, sketch_size, k, kmer_space,
              use64=True, threads=1, with_pvalue=True):
    dt = np.uint64 if use64 else np.uint32
    w = max([len(x) for x in ref_lists + qry_lists] + [1])
    R, rl = dense(ref_lists, w, dt)
    Q, ql = dense(qry_lists, w, dt)
    rL = np.ascontiguousarray(ref_lengths, dtype=np.uint64)
    qL = np.ascontiguousarray(qry_lengths, dtype=np.uint64)
    n = len(ref_lists) * len(qry_lists)
    nu = np.zeros(max(n, 1), np.uint32)
    de = np.zeros(max(n, 1), np.uint32)
    di = np.zeros(max(n, 1), np.float64)
    pv = np.zeros(max(n, 1), np.float64) if with_pvalue else None
    rc = lib().orc_dist_grid(R.ctypes.data, _p(rl, u32p), _p(rL, u64p), w, len(ref_lists),
                             Q.ctypes.data, _p(ql, u32p), _p(qL, u64p), w, len(qry_lists),
                             int(use64), sketch_size, k, kmer_space,
                             _p(nu, u32p), _p(de, u32p), _p(di, f64p),
                             _p(pv, f64p) if with_pvalue else None, threads)
    assert rc == 0
    return nu[:n], de[:n], di[:n], (pv[:n] if with_pvalue else None)


def write_dist_text(path, names, qry_rows, numer, denom, dist, pval, passed=None,
                    flush_each=True):
    """The reference's dist text step (writeOutput, CommandDistance.cpp:276-333: ostream
    formatting, `endl` per line) for the grid block of query rows `qry_rows` x all refs
    (numer ... [len(qry_rows) * len(names)], query-major) into `path`."""
    off = np.zeros(len(names) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in names])
    q = np.ascontiguousarray(qry_rows, np.uint32)
    nu = np.ascontiguousarray(numer, np.uint32)
    de = np.ascontiguousarray(denom, np.uint32)
    di = np.ascontiguousarray(dist, np.float64)
    pv = np.ascontiguousarray(pval, np.float64)
    pa = None if passed is None else np.ascontiguousarray(passed, np.uint8)
    rc = lib().orc_write_dist_text(os.fsencode(path), b"".join(names), _p(off, u64p), len(names),
                                   _p(q, u32p), len(q), _p(nu, u32p), _p(de, u32p), _p(di, f64p),
                                   _p(pv, f64p), None if pa is None else pa.ctypes.data,
                                   int(flush_each))
    if rc:
        raise OSError(f"write_dist_text: {rc}")
