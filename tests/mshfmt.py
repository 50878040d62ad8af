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
