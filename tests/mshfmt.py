"""Minimal Cap'n Proto reader for Mash .msh files (capnp/MinHash.capnp:12-59).

Test support only: decodes the reference's fixture sketches so parity tests can
compare hashes, lengths, names and header fields.  Field offsets follow capnp's
ordinal-order layout for the schema, e.g. the root MinHash
struct has 3 data words [kmerSize@0B, windowSize@4B, minHashesPerWindow@8B,
concatenated bit96, noncanonical bit97, preserveCase bit98, error f32@16B,
hashSeed u32@20B xor 42] and pointers [referenceListOld, locusList, alphabet,
referenceList].
"""
from __future__ import annotations

import struct

import numpy as np


class Msg:
    def __init__(self, data: bytes):
        self.data = data
        n = struct.unpack_from("<I", data, 0)[0] + 1
        sizes = struct.unpack_from(f"<{n}I", data, 4)
        off = 4 + 4 * n
        off += (8 - off % 8) % 8
        self.segs = []
        for s in sizes:
            self.segs.append((off, s))
            off += 8 * s
        self.seg_sizes = sizes

    def word(self, seg, idx):
        base, _ = self.segs[seg]
        return struct.unpack_from("<Q", self.data, base + 8 * idx)[0]

    def byte_off(self, seg, idx):
        return self.segs[seg][0] + 8 * idx

    def follow(self, seg, idx):
        """Resolve the pointer at (seg, idx): returns (seg, ptr_word_idx_for_offset_base, ptr)."""
        p = self.word(seg, idx)
        if p == 0:
            return None
        kind = p & 3
        if kind == 2:   # far pointer
            double = (p >> 2) & 1
            off = (p >> 3) & ((1 << 29) - 1)
            tseg = p >> 32
            if not double:
                return self.follow(tseg, off)
            pad0 = self.word(tseg, off)
            tag = self.word(tseg, off + 1)
            content_seg = pad0 >> 32
            content_off = (pad0 >> 3) & ((1 << 29) - 1)
            return ("far2", content_seg, content_off, tag)
        return ("near", seg, idx, p)

    def _target(self, seg, idx):
        r = self.follow(seg, idx)
        if r is None:
            return None
        if r[0] == "near":
            _, s, i, p = r
            o = (p >> 2) & ((1 << 30) - 1)
            if o & (1 << 29):
                o -= 1 << 30
            return s, i + 1 + o, p
        _, s, start, tag = r
        return s, start, tag

    def struct_at(self, seg, idx):
        t = self._target(seg, idx)
        if t is None:
            return None
        s, start, p = t
        return Struct(self, s, start, (p >> 32) & 0xFFFF, p >> 48)

    def list_at(self, seg, idx):
        t = self._target(seg, idx)
        if t is None:
            return None
        s, start, p = t
        return s, start, (p >> 32) & 7, p >> 35


class Struct:
    def __init__(self, msg, seg, start, dwords, pwords):
        self.m, self.seg, self.start, self.dw, self.pw = msg, seg, start, dwords, pwords

    def u32(self, byte):
        if byte + 4 > 8 * self.dw:
            return 0
        return struct.unpack_from("<I", self.m.data, self.m.byte_off(self.seg, self.start) + byte)[0]

    def u64(self, byte):
        if byte + 8 > 8 * self.dw:
            return 0
        return struct.unpack_from("<Q", self.m.data, self.m.byte_off(self.seg, self.start) + byte)[0]

    def f32(self, byte):
        if byte + 4 > 8 * self.dw:
            return 0.0
        return struct.unpack_from("<f", self.m.data, self.m.byte_off(self.seg, self.start) + byte)[0]

    def bit(self, b):
        if b >= 64 * self.dw:
            return False
        byte = self.m.data[self.m.byte_off(self.seg, self.start) + b // 8]
        return bool((byte >> (b % 8)) & 1)

    def ptr_idx(self, i):
        return self.start + self.dw + i

    def struct(self, i):
        if i >= self.pw:
            return None
        return self.m.struct_at(self.seg, self.ptr_idx(i))

    def text(self, i):
        if i >= self.pw:
            return None
        L = self.m.list_at(self.seg, self.ptr_idx(i))
        if L is None:
            return None
        s, start, esz, n = L
        b = self.m.data[self.m.byte_off(s, start): self.m.byte_off(s, start) + n]
        return b[:-1] if b.endswith(b"\0") else b

    def prim_list(self, i, dtype):
        if i >= self.pw:
            return None
        L = self.m.list_at(self.seg, self.ptr_idx(i))
        if L is None:
            return None
        s, start, esz, n = L
        o = self.m.byte_off(s, start)
        return np.frombuffer(self.m.data, dtype=dtype, count=n, offset=o).copy()

    def struct_list(self, i):
        if i >= self.pw:
            return []
        L = self.m.list_at(self.seg, self.ptr_idx(i))
        if L is None:
            return []
        s, start, esz, nwords = L
        assert esz == 7, "composite list expected"
        tag = self.m.word(s, start)
        n = (tag >> 2) & ((1 << 30) - 1)
        dw, pw = (tag >> 32) & 0xFFFF, tag >> 48
        return [Struct(self.m, s, start + 1 + j * (dw + pw), dw, pw) for j in range(n)]


def read_msh(path_or_bytes):
    data = open(path_or_bytes, "rb").read() if isinstance(path_or_bytes, str) else path_or_bytes
    m = Msg(data)
    root = m.struct_at(0, 0)
    hdr = {
        "kmer": root.u32(0),
        "windowSize": root.u32(4),
        "sketchSize": root.u32(8),
        "concatenated": root.bit(96),
        "noncanonical": root.bit(97),
        "preserveCase": root.bit(98),
        "error": root.f32(16),
        "seed": root.u32(20) ^ 42,
        "alphabet": root.text(2),
        "segments": list(m.seg_sizes),
    }
    rl = root.struct(3)
    refs_new = rl.struct_list(0) if rl is not None else []
    refs = refs_new if refs_new else (root.struct(0).struct_list(0) if root.struct(0) else [])
    hdr["referenceListOld"] = not bool(refs_new)
    out = []
    for r in refs:
        h64 = r.prim_list(5, np.uint64)
        h32 = r.prim_list(4, np.uint32)
        cnt = r.prim_list(6, np.uint32)
        length64 = r.u64(8)
        out.append({
            "name": r.text(2) or b"",
            "comment": r.text(3) or b"",
            "length": length64 if length64 else r.u32(0),
            "hashes64": h64,
            "hashes32": h32,
            "counts": cnt,
            "countsSorted": r.bit(32),
        })
    hdr["references"] = out
    return hdr


# ---------------------------------------------------------------------------
# writer (test support: builds the EXPECTED .msh bytes from oracle sketches, so
# the product's host/Msh.cpp writer is checked against an independent encoder)
# ---------------------------------------------------------------------------

class _Arena:
    """capnp MallocMessageBuilder's allocation model (Sketch.cpp:546 uses the default
    builder): the first segment holds max(need, 1024) words; every later segment holds
    max(need, words allocated so far); an object goes into its pointer's segment when it
    fits there, else into the newest segment with room, behind a far pointer + landing pad."""

    FIRST = 1024

    def __init__(self):
        self.segs = []        # [bytearray of used words, capacity in words]
        self.grow = self.FIRST
        self.newest = None

    def _try(self, s, n):
        seg = self.segs[s]
        used = len(seg[0]) // 8
        if used + n > seg[1]:
            return None
        seg[0].extend(b"\0" * (8 * n))
        return used

    def _arena(self, n):
        if self.newest is not None:
            o = self._try(self.newest, n)
            if o is not None:
                return self.newest, o
        size = max(n, self.grow)
        self.grow = size if not self.segs else self.grow + size
        self.segs.append([bytearray(), size])
        self.newest = len(self.segs) - 1
        return self.newest, self._try(self.newest, n)

    def put(self, s, w, v):
        struct.pack_into("<Q", self.segs[s][0], 8 * w, v & 0xFFFFFFFFFFFFFFFF)

    def get(self, s, w):
        return struct.unpack_from("<Q", self.segs[s][0], 8 * w)[0]

    def obj(self, s, w, n, kind, upper):
        """allocate n words for an object whose pointer lives at (s, w)"""
        o = self._try(s, n)
        if o is not None:
            self.put(s, w, kind | (((o - (w + 1)) & 0x3FFFFFFF) << 2) | (upper << 32))
            return s, o
        ts, to = self._arena(n + 1)
        self.put(s, w, 2 | (to << 3) | (ts << 32))
        self.put(ts, to, kind | (upper << 32))
        return ts, to + 1

    def data(self):
        n = len(self.segs)
        tab = [n - 1] + [len(sg[0]) // 8 for sg in self.segs]
        if len(tab) % 2:
            tab.append(0)
        return struct.pack(f"<{len(tab)}I", *tab) + b"".join(bytes(sg[0]) for sg in self.segs)


def _text(A, s, w, t: bytes):
    n = len(t) + 1
    ts, to = A.obj(s, w, (n + 7) // 8, 1, 2 | (n << 3))
    A.segs[ts][0][8 * to: 8 * to + len(t)] = t


def write_msh(hdr, refs, use64=True, counts=False) -> bytes:
    """Serialize a MinHash message the way Sketch::writeToCapnp (Sketch.cpp:536-642)
    builds it: root, reference list (referenceListOld when the seed is 42, :549), per
    reference name, comment, length64, hashes64/hashes32 (+ counts32), the empty locus
    list, then the scalar fields and the alphabet.  refs: dicts with name, comment,
    length, hashes (ascending), optional counts."""
    A = _Arena()
    A._arena(1)                                   # root pointer
    rs, rw = A.obj(0, 0, 7, 0, 3 | (4 << 16))     # MinHash: 3 data words, 4 pointers
    rp = rw + 3
    seed = hdr.get("seed", 42)
    ls, lw = A.obj(rs, rp + (0 if seed == 42 else 3), 1, 0, 0 | (1 << 16))
    n = len(refs)
    es, ew = A.obj(ls, lw, 1 + 9 * n, 1, 7 | ((9 * n) << 3))
    A.put(es, ew, (n << 2) | ((2 | (7 << 16)) << 32))
    for i, r in enumerate(refs):
        dw = ew + 1 + 9 * i
        pw = dw + 2
        _text(A, es, pw + 2, bytes(r["name"]))
        _text(A, es, pw + 3, bytes(r["comment"]))
        A.put(es, dw + 1, int(r["length"]))
        h = np.asarray(r["hashes"], dtype=np.uint64)
        if len(h):
            m = len(h)
            if use64:
                ts, to = A.obj(es, pw + 5, m, 1, 5 | (m << 3))
                A.segs[ts][0][8 * to: 8 * (to + m)] = h.astype("<u8").tobytes()
            else:
                ts, to = A.obj(es, pw + 4, (m + 1) // 2, 1, 4 | (m << 3))
                A.segs[ts][0][8 * to: 8 * to + 4 * m] = h.astype("<u4").tobytes()
            c = r.get("counts")
            if counts and c is not None and len(c):
                c = np.asarray(c, dtype="<u4")
                ts, to = A.obj(es, pw + 6, (len(c) + 1) // 2, 1, 4 | (len(c) << 3))
                A.segs[ts][0][8 * to: 8 * to + 4 * len(c)] = c.tobytes()
                A.put(es, dw, A.get(es, dw) | (1 << 32))
    # locusList with an empty composite loci list (Sketch.cpp:606-621)
    cs, cw = A.obj(rs, rp + 1, 1, 0, 0 | (1 << 16))
    ts, to = A.obj(cs, cw, 1, 1, 7 | (0 << 3))
    A.put(ts, to, (3 << 32))
    # scalars (Sketch.cpp:623-630): kmer u32@0, windowSize @4, minHashesPerWindow @8,
    # error f32 @16, hashSeed @20 (xor 42), bits 96-98
    w0 = int(hdr["kmer"]) | (int(hdr.get("windowSize", 0)) << 32)
    w1 = int(hdr["sketchSize"]) | (int(hdr.get("concatenated", False)) << 32) | \
        (int(hdr.get("noncanonical", False)) << 33) | (int(hdr.get("preserveCase", False)) << 34)
    err = struct.unpack("<I", struct.pack("<f", float(hdr.get("error", 0.0))))[0]
    w2 = err | ((seed ^ 42) << 32)
    for j, v in enumerate((w0, w1, w2)):
        A.put(rs, rw + j, v)
    _text(A, rs, rp + 2, bytes(hdr["alphabet"]))
    return A.data()
