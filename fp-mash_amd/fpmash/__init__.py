"""fpmash — Python binding of the gfx950 sketch + dist C ABI (include/fpmash.h).

A ctypes mirror of the reference's engine calls for this path:
  Sketch sketching (addMinHashes/MinHashHeap, Sketch.cpp:664-735, 1490-1517) -> Context.sketch
  -fp line hashing (getHashFingerPrint, hash.cpp:45-73)                    -> Context.fp_hash_lines
  compare/compareSketches/pValue (CommandDistance.cpp:335-450)             -> Context.dist
The shared library is built in-tree (fp-mash_amd/lib/libfpmash.so).  There is no
CPU fallback: if the library is missing this import fails, and without a gfx950
device Context() raises FpmError(FPM_ENODEV).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FPMASH_LIB: another build of the same ABI (A/B timing of kernel variants on one box)
LIB_PATH = os.environ.get("FPMASH_LIB") or os.path.join(PKG_ROOT, "lib", "libfpmash.so")
BIN_PATH = os.path.join(PKG_ROOT, "bin", "fpmash")

FPM_OK, FPM_EINVAL, FPM_ENODEV, FPM_EHIP, FPM_ENOMEM = 0, -1, -2, -3, -4
(K_SKETCH, K_MERGE, K_FPHASH, K_COMPARE, K_FINALIZE, K_INDEX, K_PROBE, K_FPTEXT, K_FILL,
 K_SEQPARSE) = range(10)
NO_GROUP = 0xFFFFFFFF
KERNEL_NAMES = {K_SKETCH: "sketch_tiles_kernel", K_MERGE: "merge_kernel",
                K_FPHASH: "fp_hash_kernel", K_COMPARE: "candidate compare (rank_rows/walk_cand/compare_grid)",
                K_FINALIZE: "dist finalize (dense / candidate cells)", K_INDEX: "dist index build",
                K_PROBE: "probe_rows_kernel", K_FPTEXT: "fp text parse (nl index + fp_line)",
                K_FILL: "dist_fill_kernel", K_SEQPARSE: "FASTA parse (seq chunk scan + emit)"}
DIST_AUTO, DIST_DENSE, DIST_SPARSE = 0, 1, 2
# fpm_ctx_last_dist_stats path codes
DIST_PATHS = ["dense walk", "bucket index + literal walk", "bucket index + bucketed rank"]

ALPHABET_NUCLEOTIDE = "ACGT"                     # Sketch.h alphabetNucleotide
ALPHABET_PROTEIN = "ACDEFGHIKLMNPQRSTVWY"         # Sketch.h alphabetProtein

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
f64p = C.POINTER(C.c_double)
u8p = C.POINTER(C.c_uint8)
vp = C.c_void_p

# every symbol include/fpmash.h declares: (name, restype, argtypes)
SYMBOLS = [
    ("fpm_abi_version", C.c_int, []),
    ("fpm_build_id", C.c_char_p, []),
    ("fpm_last_error", C.c_char_p, []),
    ("fpm_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("fpm_ctx_create", C.c_int, [C.c_int, C.POINTER(vp)]),
    ("fpm_ctx_destroy", None, [vp]),
    ("fpm_ctx_stream", vp, [vp]),
    ("fpm_stream_create", C.c_int, [vp, C.POINTER(vp)]),
    ("fpm_stream_destroy", C.c_int, [vp, vp]),
    ("fpm_event_create", C.c_int, [vp, C.POINTER(vp)]),
    ("fpm_event_destroy", C.c_int, [vp, vp]),
    ("fpm_event_record", C.c_int, [vp, vp, vp]),
    ("fpm_stream_wait_event", C.c_int, [vp, vp, vp]),
    ("fpm_ctx_synchronize", C.c_int, [vp]),
    ("fpm_ctx_warm", C.c_int, [vp]),
    ("fpm_malloc", C.c_int, [vp, C.POINTER(vp), C.c_size_t]),
    ("fpm_free", C.c_int, [vp, vp]),
    ("fpm_memcpy_h2d", C.c_int, [vp, vp, vp, C.c_size_t]),
    ("fpm_memcpy_d2h", C.c_int, [vp, vp, vp, C.c_size_t]),
    ("fpm_memcpy_d2d", C.c_int, [vp, vp, vp, C.c_size_t]),
    ("fpm_memset", C.c_int, [vp, vp, C.c_int, C.c_size_t]),
    ("fpm_ctx_set_timing", C.c_int, [vp, C.c_int]),
    ("fpm_ctx_reset_timing", C.c_int, [vp]),
    ("fpm_ctx_kernel_time", C.c_int, [vp, C.c_int, f64p, u64p]),
    ("fpm_ctx_set_dist_mode", C.c_int, [vp, C.c_int]),
    ("fpm_ctx_last_dist_stats", C.c_int, [vp, C.POINTER(C.c_int), u64p, u64p]),
    ("fpm_sketch_batch", C.c_int, [vp, vp, C.c_char_p, u64p, C.c_uint32, u32p, C.c_uint32,
                                   u64p, u32p]),
    ("fpm_sketch_stage", C.c_int, [vp, vp, C.c_char_p, u64p, C.c_uint32, u32p, C.c_uint32,
                                   C.POINTER(vp)]),
    ("fpm_sketch_run", C.c_int, [vp, vp]),
    ("fpm_sketch_device_output", C.c_int, [vp, C.POINTER(vp), C.POINTER(vp), u32p, u32p]),
    ("fpm_sketch_fetch", C.c_int, [vp, u64p, u32p]),
    ("fpm_sketch_mult", C.c_int, [vp, vp, u32p]),
    ("fpm_merge_small_spills", C.c_int, [vp, u64p]),
    ("fpm_sketch_job_info", C.c_int, [vp, u64p, u64p, u64p]),
    ("fpm_sketch_job_redo_tiles", C.c_int, [vp, C.POINTER(C.c_int32)]),
    ("fpm_sketch_job_short_groups", C.c_int, [vp, C.POINTER(C.c_int32)]),
    ("fpm_sketch_job_sample_short", C.c_int, [vp, C.POINTER(C.c_int32)]),
    ("fpm_sketch_job_free", None, [vp]),
    ("fpm_fp_hash_lines", C.c_int, [vp, u64p, u64p, C.c_uint64, C.c_uint32, C.c_uint32, vp]),
    ("fpm_fp_hash_lines_dev", C.c_int, [vp, vp, vp, C.c_uint64, C.c_uint32, C.c_uint32, vp,
                                        vp]),
    ("fpm_fp_text_stage", C.c_int, [vp, C.c_char_p, C.c_uint64, C.c_uint64, C.c_uint32,
                                    C.c_uint32, C.POINTER(vp), u64p]),
    ("fpm_fp_text_fetch", C.c_int, [vp, u64p, u32p, u32p, vp, u8p]),
    ("fpm_fp_text_refs", C.c_int, [vp, C.c_uint64, u64p, u64p, u64p, u32p, u64p]),
    ("fpm_fp_text_free", None, [vp]),
    ("fpm_compare_grid", C.c_int, [vp, vp, u32p, C.c_uint64, C.c_uint32, vp, u32p, C.c_uint64,
                                   C.c_uint32, C.c_uint32, C.c_uint32, u32p, u32p]),
    ("fpm_compare_grid_dev", C.c_int, [vp, vp, vp, C.c_uint64, C.c_uint32, vp, vp, C.c_uint64,
                                       C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp]),
    ("fpm_dist_finalize_dev", C.c_int, [vp, vp, vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.c_double, C.c_double, C.c_double, vp, vp, vp, vp]),
    ("fpm_pvalue_batch_dev", C.c_int, [vp, vp, vp, C.c_uint32, vp, vp, C.c_uint64, C.c_uint32,
                                       C.c_double, vp, vp, vp]),
    ("fpm_dist_dev", C.c_int, [vp, vp, vp, vp, C.c_uint64, C.c_uint32, vp, vp, vp, C.c_uint64,
                               C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_double,
                               C.c_double, C.c_double, vp, vp, vp, vp, vp, vp]),
    ("fpm_dist_dev16", C.c_int, [vp, vp, vp, vp, C.c_uint64, C.c_uint32, vp, vp, vp, C.c_uint64,
                                 C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_double,
                                 C.c_double, C.c_double, vp, vp, vp, vp, vp, vp]),
    ("fpm_dist_list_dev", C.c_int, [vp, vp, vp, vp, C.c_uint64, C.c_uint32, vp, vp, vp,
                                    C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_double, C.c_double, C.c_double, vp, vp, vp, vp]),
    ("fpm_dist_list_prefill", C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp]),
    ("fpm_fp_positional_grid", C.c_int, [vp, vp, u32p, C.c_uint64, C.c_uint32, vp, u32p,
                                         C.c_uint64, C.c_uint32, C.c_uint32, C.c_double,
                                         C.c_double, u32p, u32p, f64p, f64p, u8p]),
    ("fpm_dist", C.c_int, [vp, vp, u32p, u64p, C.c_uint64, C.c_uint32, vp, u32p, u64p,
                           C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                           C.c_double, C.c_double, C.c_double, u32p, u32p, f64p, f64p, u8p]),
    ("fpm_refset_create", C.c_int, [vp, vp, u32p, u64p, C.c_uint64, C.c_uint32, C.c_uint32,
                                    C.c_uint32, C.POINTER(vp)]),
    ("fpm_refset_create_dev", C.c_int, [vp, vp, vp, vp, C.c_uint64, C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.POINTER(vp)]),
    ("fpm_refset_dist_dev", C.c_int, [vp, vp, vp, vp, C.c_uint64, C.c_uint32, C.c_uint32,
                                      C.c_uint32, C.c_uint32, C.c_double, C.c_double, C.c_double,
                                      vp, vp, vp, vp, vp, vp]),
    ("fpm_refset_dist_mirror_dev", C.c_int, [vp, vp, vp, vp, C.c_uint64, C.c_uint32, C.c_uint32,
                                             C.c_uint32, C.c_uint32, C.c_double, C.c_double,
                                             C.c_double, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                             vp]),
    ("fpm_refset_dist_list_dev", C.c_int, [vp, vp, vp, vp, C.c_uint64, C.c_uint32, C.c_uint32,
                                           C.c_uint32, C.c_double, C.c_double, C.c_double, vp,
                                           vp, vp, vp]),
    ("fpm_refset_dist_mirror_list_dev", C.c_int, [vp, vp, vp, vp, C.c_uint64, C.c_uint32,
                                                  C.c_uint32, C.c_uint32, C.c_double, C.c_double,
                                                  C.c_double, vp, vp, vp, vp, vp, vp, vp]),
    ("fpm_refset_reindex", C.c_int, [vp, vp]),
    ("fpm_ctx_index_rebuilds", C.c_int, [vp, u64p]),
    ("fpm_ctx_spec_stats", C.c_int, [vp, u64p, u64p]),
    ("fpm_refset_dist", C.c_int, [vp, vp, u32p, u64p, C.c_uint64, C.c_uint32, C.c_uint32,
                                  C.c_uint32, C.c_double, C.c_double, C.c_double, u32p, u32p,
                                  f64p, f64p, u8p]),
    ("fpm_refset_dist_list", C.c_int, [vp, vp, u32p, u64p, C.c_uint64, C.c_uint32, C.c_uint32,
                                       C.c_uint32, C.c_double, C.c_double, C.c_double,
                                       C.c_uint32, vp, vp, u32p, u32p, f64p, f64p, u8p,
                                       C.c_uint64, u64p]),
    ("fpm_refset_free", None, [vp]),
    ("fpm_sketch_merge_dev", C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, vp, vp, vp]),
    ("fpm_seq_parse", C.c_int, [vp, C.POINTER(C.c_char_p), u64p, C.c_uint32, C.POINTER(vp),
                                u64p, C.POINTER(C.c_int)]),
    ("fpm_seq_records", C.c_int, [vp, u32p, u64p, u64p, u64p]),
    ("fpm_sketch_stage_seq", C.c_int, [vp, vp, vp, u32p, C.c_uint32, C.POINTER(vp)]),
    ("fpm_seq_free", None, [vp]),
    ("fpm_host_alloc", C.c_int, [vp, C.POINTER(vp), C.c_size_t]),
    ("fpm_host_free", C.c_int, [vp, vp]),
    ("fpm_comm_unique_id", C.c_int, [C.c_char_p]),
    ("fpm_comm_create", C.c_int, [vp, C.c_int, C.c_int, C.c_char_p, C.POINTER(vp)]),
    ("fpm_comm_destroy", None, [vp]),
    ("fpm_comm_all_gather", C.c_int, [vp, vp, vp, C.c_size_t, vp]),
    ("fpm_sketch_min_merge_comm", C.c_int, [vp, vp, vp, C.c_uint32, vp, vp, vp]),
]
COMM_ID_BYTES = 128


class CellListStruct(C.Structure):
    """fpm_cell_list (include/fpmash.h): device arrays of the compact dist output's list"""
    _fields_ = [("qry", vp), ("ref", vp), ("dist", vp), ("pvalue", vp), ("pass_", vp),
                ("cap", C.c_uint64), ("count", vp)]


class FpmError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"fpmash error {code}: {msg}")
        self.code = code


class SketchParams(C.Structure):
    """fpm_sketch_params == Sketch::Parameters subset (Sketch.h:40-113)."""
    _fields_ = [
        ("kmer_size", C.c_uint32),
        ("sketch_size", C.c_uint32),
        ("seed", C.c_uint32),
        ("use64", C.c_uint32),
        ("noncanonical", C.c_uint32),
        ("preserve_case", C.c_uint32),
        ("alphabet", C.c_uint8 * 256),
    ]


def make_params(k=21, s=1000, seed=42, alphabet=ALPHABET_NUCLEOTIDE, noncanonical=False,
                preserve_case=False, fingerprint=False, protein=False):
    """sketchParameterSetup (sketchParameterSetup.cpp:9-126) + setAlphabetFromString
    (Sketch.cpp:1260-1289)."""
    if fingerprint:                      # -fp: k=1, noncanonical, "0123456789"
        k, noncanonical, alphabet = 1, True, "0123456789"
    elif protein:
        noncanonical, alphabet = True, ALPHABET_PROTEIN
    P = SketchParams()
    P.kmer_size, P.sketch_size, P.seed = k, s, seed
    P.noncanonical, P.preserve_case = int(noncanonical), int(preserve_case)
    n = 0
    for ch in alphabet.encode():
        if not preserve_case and 96 < ch < 123:
            ch -= 32
        if not P.alphabet[ch]:
            n += 1
        P.alphabet[ch] = 1
    P.use64 = int(float(n) ** k > 2.0 ** 32)
    return P


_LIB = None


def build_id(path=None):
    """The build id a libfpmash.so carries (fpm_build_id: a hash of the sources it was
    compiled from), read from the file's "fpm-build-id:<id>" text without loading it, so a
    process that must not touch the GPU (tools/pmc_traffic.py) can stamp its profiles with it.
    None when the file is absent or carries no id."""
    import mmap
    import re
    path = path or LIB_PATH
    try:
        with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
            hit = re.search(rb"fpm-build-id:([0-9a-f]{16})", m)
            return bytes(hit.group(1)).decode() if hit else None
    except (OSError, ValueError):
        return None


def lib():
    """Load libfpmash.so (raises if the HIP build is absent: no fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built (run `make -C fp-mash_amd`); "
                              "fpmash has no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SYMBOLS:
            # (an older build under FPMASH_LIB, a same-box A/B, may lack the newest entry
            # points; tests/test_abi.py checks the product exports every one)
            f = getattr(L, name, None)
            if f is None:
                continue
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def _check(rc):
    if rc != FPM_OK:
        raise FpmError(rc, lib().fpm_last_error().decode(errors="replace"))


def device_count():
    n = C.c_int(0)
    _check(lib().fpm_device_count(C.byref(n)))
    return n.value


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


def pack_records(seqs):
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    if seqs:
        off[1:] = np.cumsum([len(s) for s in seqs])
    return b"".join(seqs), off


class DeviceBuffer:
    def __init__(self, ctx, nbytes):
        self.ctx, self.nbytes = ctx, int(nbytes)
        p = vp()
        _check(lib().fpm_malloc(ctx.h, C.byref(p), self.nbytes))
        self.ptr = p.value

    @classmethod
    def from_array(cls, ctx, arr):
        arr = np.ascontiguousarray(arr)
        b = cls(ctx, arr.nbytes)
        _check(lib().fpm_memcpy_h2d(ctx.h, b.ptr, arr.ctypes.data, arr.nbytes))
        return b

    def to_array(self, dtype, count):
        out = np.empty(count, dtype=dtype)
        _check(lib().fpm_memcpy_d2h(self.ctx.h, out.ctypes.data, self.ptr, out.nbytes))
        return out

    def free(self):
        if self.ptr:
            lib().fpm_free(self.ctx.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class CellList:
    """Device buffers of a compact dist output's cell list (fpm_cell_list) with room for
    `cap` entries.  .struct is what the *_list_dev calls take (by reference)."""

    def __init__(self, ctx, cap):
        self.ctx, self.cap = ctx, int(max(cap, 1))
        self.bufs = [DeviceBuffer(ctx, self.cap * b) for b in (4, 4, 8, 8, 1)] + \
            [DeviceBuffer(ctx, 8)]
        q, r, d, p, a, c = (b.ptr for b in self.bufs)
        self.struct = CellListStruct(q, r, d, p, a, self.cap, c)

    @property
    def ref(self):
        return C.byref(self.struct)

    def count(self):
        """cells with numer > 0 the last call listed (may exceed cap: then re-run larger)"""
        return int(self.bufs[5].to_array(np.uint64, 1)[0])

    def fetch(self):
        """-> dict of the listed cells' qry, ref, distance, pvalue, pass (host arrays)"""
        n = self.count()
        if n > self.cap:
            raise FpmError(FPM_ENOMEM, f"cell list holds {self.cap} entries, {n} needed")
        m = max(n, 1)
        out = {k: b.to_array(t, m)[:n] for k, b, t in zip(
            ("qry", "ref", "distance", "pvalue", "pass"), self.bufs[:5],
            (np.uint32, np.uint32, np.float64, np.float64, np.uint8))}
        out["pass"] = out["pass"].astype(bool)
        return out

    def free(self):
        for b in self.bufs:
            b.free()


def expand_compact(numer, denom, listed, n_ref, max_dist=-1.0, max_pvalue=-1.0):
    """The five per-cell outputs of a compact result (fpm_dist_list_dev: counts of every
    cell + the list of cells with numer > 0), by the rule include/fpmash.h states: an unlisted
    cell has distance 0 if denom == 0 else 1, p-value 1, and the -d / -v filters at those
    values (CommandDistance.cpp:404-408, 435-437 at common = 0).  numer / denom: flat
    query-major arrays; listed: CellList.fetch()."""
    numer = np.asarray(numer)
    denom = np.asarray(denom)
    dist = np.where(denom == 0, 0.0, 1.0)
    pval = np.ones(len(numer), np.float64)
    ok = np.ones(len(numer), bool)
    if max_dist >= 0:
        ok &= dist <= max_dist
    if max_pvalue >= 0:
        ok &= 1.0 <= max_pvalue
    idx = listed["qry"].astype(np.int64) * n_ref + listed["ref"].astype(np.int64)
    if len(idx) and np.any(numer[idx] == 0):
        raise AssertionError("a listed cell has numer 0")
    if int(np.count_nonzero(numer)) != len(idx) or len(np.unique(idx)) != len(idx):
        raise AssertionError("the list is not exactly the cells with numer > 0")
    dist[idx] = listed["distance"]
    pval[idx] = listed["pvalue"]
    ok[idx] = listed["pass"]
    return {"numer": numer, "denom": denom, "distance": dist, "pvalue": pval, "pass": ok}


class SketchJob:
    """fpm_sketch_stage/run/fetch: inputs staged once in HBM, kernels re-runnable."""

    def __init__(self, ctx, params, seqs, groups=None, n_groups=None):
        self.ctx, self.params = ctx, params
        data, off = pack_records(seqs)
        self._keep = (data, off)
        n_rec = len(seqs)
        if groups is not None:
            g = np.ascontiguousarray(groups, dtype=np.uint32)
            self.n_groups = int(n_groups if n_groups is not None else (int(g.max()) + 1 if n_rec else 0))
            gp = _p(g, u32p)
        else:
            self.n_groups, gp = n_rec, None
        h = vp()
        _check(lib().fpm_sketch_stage(ctx.h, C.byref(params), data, _p(off, u64p), n_rec, gp,
                                      self.n_groups, C.byref(h)))
        self.h = h.value

    def run(self, stream=None):
        _check(lib().fpm_sketch_run(self.h, stream))

    def info(self):
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().fpm_sketch_job_info(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return {"seq_bytes": a.value, "n_tiles": b.value, "n_kmers": c.value}

    def redo_tiles(self):
        """tiles of the last run() the survivors-only kernel handed to the plain one (-1: the
        job does not use that kernel); waits for the device"""
        n = C.c_int32()
        _check(lib().fpm_sketch_job_redo_tiles(self.h, C.byref(n)))
        return n.value

    def short_groups(self):
        """long groups of the last run() redone under the sample's s-th smallest hash after
        the tight bound left them short (-1: no tight bounds in this job)"""
        n = C.c_int32()
        _check(lib().fpm_sketch_job_short_groups(self.h, C.byref(n)))
        return n.value

    def sample_short(self):
        """samples of the last run() the a-priori sample bound left short, redone unbounded
        (-1: the job's samples carry no such bound)"""
        n = C.c_int32()
        _check(lib().fpm_sketch_job_sample_short(self.h, C.byref(n)))
        return n.value

    def device_output(self):
        dh, dc = vp(), vp()
        ng, st = C.c_uint32(), C.c_uint32()
        _check(lib().fpm_sketch_device_output(self.h, C.byref(dh), C.byref(dc), C.byref(ng),
                                              C.byref(st)))
        return dh.value, dc.value, ng.value, st.value

    def fetch(self):
        s = int(self.params.sketch_size)
        out = np.zeros(max(self.n_groups, 1) * s, dtype=np.uint64)
        cnt = np.zeros(max(self.n_groups, 1), dtype=np.uint32)
        _check(lib().fpm_sketch_fetch(self.h, _p(out, u64p), _p(cnt, u32p)))
        return out[: self.n_groups * s].reshape(self.n_groups, s), cnt[: self.n_groups]

    def mult(self, stream=None):
        """-M: fpm_sketch_mult -> [n_groups, s] u32 multiplicities (after run())."""
        s = int(self.params.sketch_size)
        out = np.zeros(max(self.n_groups, 1) * s, dtype=np.uint32)
        _check(lib().fpm_sketch_mult(self.h, stream, _p(out, u32p)))
        return out[: self.n_groups * s].reshape(self.n_groups, s)

    def free(self):
        if self.h:
            lib().fpm_sketch_job_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    """fpm_comm_unique_id: the 128-byte RCCL unique id one rank makes and the others receive
    over a host channel (bench.Group broadcasts it over gloo)."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(lib().fpm_comm_unique_id(buf))
    return buf.raw


class Comm:
    """fpm_comm: an RCCL communicator on the context's device and HIP runtime (the library's
    own), for the cross-GPU min-merge.  Blocks in the constructor until all nranks ranks
    have joined with the same id."""

    def __init__(self, ctx, nranks, rank, uid: bytes):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        h = vp()
        _check(lib().fpm_comm_create(ctx.h, int(nranks), int(rank), uid, C.byref(h)))
        self.h, self.ctx, self.nranks, self.rank = h.value, ctx, int(nranks), int(rank)

    def all_gather(self, d_send, d_recv, nbytes, stream=None):
        _check(lib().fpm_comm_all_gather(self.h, d_send, d_recv, int(nbytes), stream))

    def min_merge(self, d_row, d_count, s, d_out, d_out_count, stream=None):
        """fpm_sketch_min_merge_comm: every rank's bottom-s row gathered and merged on the
        device (enqueued on the stream)"""
        _check(lib().fpm_sketch_min_merge_comm(self.h, d_row, d_count, int(s), d_out,
                                               d_out_count, stream))

    def close(self):
        if self.h:
            lib().fpm_comm_destroy(self.h)
            self.h = None


class Context:
    """One gfx950 device (fpm_ctx)."""

    def __init__(self, device=0):
        h = vp()
        _check(lib().fpm_ctx_create(device, C.byref(h)))
        self.h = h.value
        self.device = device

    def close(self):
        if self.h:
            lib().fpm_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def stream(self):
        return lib().fpm_ctx_stream(self.h)

    def synchronize(self):
        _check(lib().fpm_ctx_synchronize(self.h))

    def new_stream(self):
        """fpm_stream_create: a non-blocking stream of the library's runtime (free with
        free_stream)."""
        s = vp()
        _check(lib().fpm_stream_create(self.h, C.byref(s)))
        return s.value

    def free_stream(self, s):
        _check(lib().fpm_stream_destroy(self.h, s))

    def new_event(self):
        e = vp()
        _check(lib().fpm_event_create(self.h, C.byref(e)))
        return e.value

    def free_event(self, e):
        _check(lib().fpm_event_destroy(self.h, e))

    def record(self, event, stream):
        _check(lib().fpm_event_record(self.h, event, stream))

    def wait(self, stream, event):
        _check(lib().fpm_stream_wait_event(self.h, stream, event))

    def set_timing(self, on=True):
        _check(lib().fpm_ctx_set_timing(self.h, int(on)))

    def reset_timing(self):
        _check(lib().fpm_ctx_reset_timing(self.h))

    def kernel_time(self, kernel):
        t, n = C.c_double(), C.c_uint64()
        _check(lib().fpm_ctx_kernel_time(self.h, kernel, C.byref(t), C.byref(n)))
        return t.value, n.value

    def merge_small_spills(self):
        """fpm_merge_small_spills: small-list merges that overflowed the LDS cap (resets)."""
        v = np.zeros(1, np.uint64)
        _check(lib().fpm_merge_small_spills(self.h, _p(v, u64p)))
        return int(v[0])

    def set_dist_mode(self, mode):
        _check(lib().fpm_ctx_set_dist_mode(self.h, mode))

    def index_rebuilds(self):
        """one-pass index builds redone by the exact build (a level-1 slot overflowed)"""
        v = C.c_uint64()
        _check(lib().fpm_ctx_index_rebuilds(self.h, C.byref(v)))
        return v.value

    def spec_stats(self):
        """(kept, dropped) speculated probes since the context was created (fpm_ctx_spec_stats)"""
        h, m = C.c_uint64(), C.c_uint64()
        _check(lib().fpm_ctx_spec_stats(self.h, C.byref(h), C.byref(m)))
        return h.value, m.value

    def last_dist_stats(self):
        sp, ev, ca = C.c_int(), C.c_uint64(), C.c_uint64()
        _check(lib().fpm_ctx_last_dist_stats(self.h, C.byref(sp), C.byref(ev), C.byref(ca)))
        return {"sparse": sp.value, "events": ev.value, "candidates": ca.value}

    # --- sketch -----------------------------------------------------------
    def sketch(self, params, seqs, groups=None, n_groups=None, counts=False):
        """-> list of ascending u64 arrays (one per sketch); counts=True (-M): also the list
        of their u32 multiplicities."""
        job = SketchJob(self, params, seqs, groups, n_groups)
        try:
            job.run()
            rows, cnt = job.fetch()
            mult = job.mult() if counts else None
        finally:
            job.free()
        hashes = [rows[i, : cnt[i]].copy() for i in range(len(cnt))]
        if counts:
            return hashes, [mult[i, : cnt[i]].copy() for i in range(len(cnt))]
        return hashes

    def sketch_job(self, params, seqs, groups=None, n_groups=None):
        return SketchJob(self, params, seqs, groups, n_groups)

    # --- FASTA text on the device -------------------------------------------------
    def seq_parse(self, files):
        """fpm_seq_parse over file images -> (handle, records dict, quality_lines flag).
        records: seg, hdr_off, hdr_len, seq_len per record (kseq record rules)."""
        n_seg = len(files)
        ptrs = (C.c_char_p * max(n_seg, 1))(*files)
        lens = np.array([len(f) for f in files] + [0], dtype=np.uint64)
        job, n, q = vp(), C.c_uint64(), C.c_int()
        _check(lib().fpm_seq_parse(self.h, ptrs, _p(lens, u64p), n_seg, C.byref(job),
                                   C.byref(n), C.byref(q)))
        n = n.value
        seg = np.zeros(max(n, 1), np.uint32)
        ho, hl, sl = (np.zeros(max(n, 1), np.uint64) for _ in range(3))
        try:
            _check(lib().fpm_seq_records(job, _p(seg, u32p), _p(ho, u64p), _p(hl, u64p),
                                         _p(sl, u64p)))
        except Exception:
            lib().fpm_seq_free(job)
            raise
        return job.value, {"seg": seg[:n], "hdr_off": ho[:n], "hdr_len": hl[:n],
                           "seq_len": sl[:n]}, bool(q.value)

    def sketch_seq(self, params, seq_job, groups, n_groups, counts=False):
        """fpm_sketch_stage_seq + run + fetch over parsed records (the job takes the packed
        records; free the parse handle with seq_free afterwards)."""
        g = np.ascontiguousarray(groups, dtype=np.uint32)
        if g.size == 0:
            g = np.zeros(1, np.uint32)
        h = vp()
        _check(lib().fpm_sketch_stage_seq(self.h, C.byref(params), seq_job, _p(g, u32p),
                                          n_groups, C.byref(h)))
        job = SketchJob.__new__(SketchJob)
        job.ctx, job.params, job.n_groups, job.h, job._keep = self, params, n_groups, h.value, None
        try:
            job.run()
            rows, cnt = job.fetch()
            mult = job.mult() if counts else None
        finally:
            job.free()
        hashes = [rows[i, : cnt[i]].copy() for i in range(len(cnt))]
        if counts:
            return hashes, [mult[i, : cnt[i]].copy() for i in range(len(cnt))]
        return hashes

    @staticmethod
    def seq_free(seq_job):
        lib().fpm_seq_free(seq_job)

    # --- -fp ----------------------------------------------------------------
    def fp_hash_lines(self, values_per_line, seed=42, use64=False):
        off = np.zeros(len(values_per_line) + 1, dtype=np.uint64)
        if values_per_line:
            off[1:] = np.cumsum([len(v) for v in values_per_line])
        vals = (np.concatenate([np.asarray(v, dtype=np.uint64) for v in values_per_line])
                if values_per_line else np.zeros(0, np.uint64))
        return self.fp_hash_flat(vals, off, seed, use64)

    def fp_hash_flat(self, vals, line_off, seed=42, use64=False):
        vals = np.ascontiguousarray(vals, dtype=np.uint64)
        line_off = np.ascontiguousarray(line_off, dtype=np.uint64)
        n = len(line_off) - 1
        out = np.zeros(max(n, 1), dtype=np.uint64 if use64 else np.uint32)
        if vals.size == 0:
            vals = np.zeros(1, np.uint64)
        _check(lib().fpm_fp_hash_lines(self.h, _p(vals, u64p), _p(line_off, u64p), n, seed,
                                       int(use64), out.ctypes.data))
        return out[:n]

    # --- dist ---------------------------------------------------------------
    def dist(self, ref_lists, qry_lists, sketch_size, use64=True, k=21, kmer_space=None,
             ref_lengths=None, qry_lengths=None, max_dist=-1.0, max_pvalue=-1.0,
             finalize=True):
        """All pairs, query-major: returns dict of flat arrays (index q*n_ref + r)."""
        dt = np.uint64 if use64 else np.uint32
        w = max([len(x) for x in list(ref_lists) + list(qry_lists)] + [1])
        R, rl = _dense(ref_lists, w, dt)
        # the same list object on both sides: one upload, and the library may use the
        # pair symmetry of one set against itself
        Q, ql = (R, rl) if qry_lists is ref_lists else _dense(qry_lists, w, dt)
        n = len(ref_lists) * len(qry_lists)
        nu = np.zeros(max(n, 1), np.uint32)
        de = np.zeros(max(n, 1), np.uint32)
        if not finalize:
            _check(lib().fpm_compare_grid(self.h, R.ctypes.data, _p(rl, u32p), w, len(ref_lists),
                                          Q.ctypes.data, _p(ql, u32p), w, len(qry_lists),
                                          8 if use64 else 4, sketch_size, _p(nu, u32p),
                                          _p(de, u32p)))
            return {"numer": nu[:n], "denom": de[:n]}
        if kmer_space is None:
            kmer_space = 4.0 ** k
        rL = np.ascontiguousarray(ref_lengths, dtype=np.uint64)
        qL = np.ascontiguousarray(qry_lengths, dtype=np.uint64)
        di = np.zeros(max(n, 1), np.float64)
        pv = np.zeros(max(n, 1), np.float64)
        pa = np.zeros(max(n, 1), np.uint8)
        _check(lib().fpm_dist(self.h, R.ctypes.data, _p(rl, u32p), _p(rL, u64p), w,
                              len(ref_lists), Q.ctypes.data, _p(ql, u32p), _p(qL, u64p), w,
                              len(qry_lists), 8 if use64 else 4, sketch_size, k, kmer_space,
                              max_dist, max_pvalue, _p(nu, u32p), _p(de, u32p), _p(di, f64p),
                              _p(pv, f64p), _p(pa, u8p)))
        return {"numer": nu[:n], "denom": de[:n], "distance": di[:n], "pvalue": pv[:n],
                "pass": pa[:n].astype(bool)}

    def dist16(self, ref_lists, qry_lists, sketch_size, use64=True, k=21, kmer_space=None,
               ref_lengths=None, qry_lengths=None, max_dist=-1.0, max_pvalue=-1.0):
        """dist() through fpm_dist_dev16 (device buffers, u16 numer / denom cells)."""
        dt = np.uint64 if use64 else np.uint32
        w = max([len(x) for x in list(ref_lists) + list(qry_lists)] + [1])
        R, rl = _dense(ref_lists, w, dt)
        Q, ql = (R, rl) if qry_lists is ref_lists else _dense(qry_lists, w, dt)
        nr, nq = len(ref_lists), len(qry_lists)
        n = nr * nq
        if kmer_space is None:
            kmer_space = 4.0 ** k
        bufs = []

        def up(a):
            b = DeviceBuffer.from_array(self, a)
            bufs.append(b)
            return b.ptr
        try:
            dR, drl = up(R), up(rl)
            dQ, dql = (dR, drl) if qry_lists is ref_lists else (up(Q), up(ql))
            drL = up(np.ascontiguousarray(ref_lengths, dtype=np.uint64))
            dqL = drL if qry_lists is ref_lists and qry_lengths is ref_lengths else \
                up(np.ascontiguousarray(qry_lengths, dtype=np.uint64))
            outs = [DeviceBuffer(self, max(n, 1) * b) for b in (2, 2, 8, 8, 1)]
            bufs += outs
            _check(lib().fpm_dist_dev16(self.h, dR, drl, drL, w, nr, dQ, dql, dqL, w, nq,
                                        8 if use64 else 4, sketch_size, k, kmer_space, max_dist,
                                        max_pvalue, *[o.ptr for o in outs], None))
            self.synchronize()
            res = [o.to_array(t, n) for o, t in zip(outs, (np.uint16, np.uint16, np.float64,
                                                           np.float64, np.uint8))]
        finally:
            for b in bufs:
                b.free()
        return {"numer": res[0], "denom": res[1], "distance": res[2], "pvalue": res[3],
                "pass": res[4].astype(bool)}

    def dist_list(self, ref_lists, qry_lists, sketch_size, use64=True, k=21, kmer_space=None,
                  ref_lengths=None, qry_lengths=None, max_dist=-1.0, max_pvalue=-1.0, cap=None,
                  expand=True, prefill=False):
        """dist() through fpm_dist_list_dev (the compact output: u16 counts + the list of
        cells with numer > 0).  expand=True: the five per-cell arrays (expand_compact), else
        (numer, denom, listed).  prefill=True: the counts prefilled first
        (fpm_dist_list_prefill, taken over by the dist call)."""
        dt = np.uint64 if use64 else np.uint32
        w = max([len(x) for x in list(ref_lists) + list(qry_lists)] + [1])
        R, rl = _dense(ref_lists, w, dt)
        Q, ql = (R, rl) if qry_lists is ref_lists else _dense(qry_lists, w, dt)
        nr, nq = len(ref_lists), len(qry_lists)
        n = nr * nq
        if kmer_space is None:
            kmer_space = 4.0 ** k
        bufs = []

        def up(a):
            b = DeviceBuffer.from_array(self, a)
            bufs.append(b)
            return b.ptr
        lst = None
        try:
            dR, drl = up(R), up(rl)
            dQ, dql = (dR, drl) if qry_lists is ref_lists else (up(Q), up(ql))
            drL = up(np.ascontiguousarray(ref_lengths, dtype=np.uint64))
            dqL = drL if qry_lists is ref_lists and qry_lengths is ref_lengths else \
                up(np.ascontiguousarray(qry_lengths, dtype=np.uint64))
            outs = [DeviceBuffer(self, max(n, 1) * 2) for _ in range(2)]
            bufs += outs
            lst = CellList(self, cap if cap is not None else max(n, 1))
            if prefill:
                _check(lib().fpm_dist_list_prefill(self.h, outs[0].ptr, outs[1].ptr, nr, nq,
                                                   sketch_size, None))
            _check(lib().fpm_dist_list_dev(self.h, dR, drl, drL, w, nr, dQ, dql, dqL, w, nq,
                                           8 if use64 else 4, sketch_size, k, kmer_space,
                                           max_dist, max_pvalue, outs[0].ptr, outs[1].ptr,
                                           lst.ref, None))
            self.synchronize()
            nu, de = (o.to_array(np.uint16, n) for o in outs)
            listed = lst.fetch()
        finally:
            for b in bufs:
                b.free()
            if lst is not None:
                lst.free()
        if not expand:
            return nu, de, listed
        return expand_compact(nu, de, listed, nr, max_dist, max_pvalue)

    def pvalue_batch(self, numer, denom, len_ref, len_qry, k=21, kmer_space=None):
        """fpm_pvalue_batch_dev on host arrays: (distance, p-value) of each cell from its
        counts (u16 or u32) and genome lengths."""
        numer = np.ascontiguousarray(numer)
        denom = np.ascontiguousarray(denom, dtype=numer.dtype)
        if numer.dtype not in (np.uint16, np.uint32):
            raise ValueError("counts must be uint16 or uint32")
        n = len(numer)
        if kmer_space is None:
            kmer_space = 4.0 ** k
        bufs = [DeviceBuffer.from_array(self, a) for a in
                (numer, denom, np.ascontiguousarray(len_ref, dtype=np.uint64),
                 np.ascontiguousarray(len_qry, dtype=np.uint64))]
        outs = [DeviceBuffer(self, max(n, 1) * 8) for _ in range(2)]
        try:
            _check(lib().fpm_pvalue_batch_dev(self.h, bufs[0].ptr, bufs[1].ptr,
                                              numer.dtype.itemsize, bufs[2].ptr, bufs[3].ptr, n,
                                              k, kmer_space, outs[0].ptr, outs[1].ptr, None))
            self.synchronize()
            return outs[0].to_array(np.float64, n), outs[1].to_array(np.float64, n)
        finally:
            for b in bufs + outs:
                b.free()

    def refset(self, ref_lists, sketch_size, use64=True, ref_lengths=None, width=None):
        """A resident reference set (fpm_refset_create): rows uploaded and indexed once."""
        return RefSet(self, ref_lists, sketch_size, use64, ref_lengths, width)

    def fp_text(self, text, max_lines=1_000_000, seed=42, use64=False):
        """-fp file image -> per line: ID (offset, length), value count, hash, new-ID flag."""
        job, n = vp(), C.c_uint64()
        _check(lib().fpm_fp_text_stage(self.h, text, len(text), max_lines, seed, int(use64),
                                       C.byref(job), C.byref(n)))
        n = n.value
        io = np.zeros(max(n, 1), np.uint64)
        il = np.zeros(max(n, 1), np.uint32)
        nv = np.zeros(max(n, 1), np.uint32)
        h = np.zeros(max(n, 1), np.uint64 if use64 else np.uint32)
        ni = np.zeros(max(n, 1), np.uint8)
        try:
            _check(lib().fpm_fp_text_fetch(job, _p(io, u64p), _p(il, u32p), _p(nv, u32p),
                                           h.ctypes.data, _p(ni, u8p)))
        finally:
            lib().fpm_fp_text_free(job)
        return {"id_off": io[:n], "id_len": il[:n], "n_vals": nv[:n], "hash": h[:n],
                "new_id": ni[:n]}

    def fp_refs(self, text, max_lines=1_000_000, seed=42, use64=False):
        """-fp file image -> its References as initFromFingerprints groups them (Sketch.cpp:
        104-145), grouped on the device (fpm_fp_text_refs): first line, ID (offset, length in
        the text), length, and the line hashes (the only per-line fetch)."""
        job, n = vp(), C.c_uint64()
        _check(lib().fpm_fp_text_stage(self.h, text, len(text), max_lines, seed, int(use64),
                                       C.byref(job), C.byref(n)))
        n = n.value
        try:
            nr = C.c_uint64()
            _check(lib().fpm_fp_text_refs(job, 0, C.byref(nr), None, None, None, None))
            m = nr.value
            first = np.zeros(max(m, 1), np.uint64)
            io = np.zeros(max(m, 1), np.uint64)
            il = np.zeros(max(m, 1), np.uint32)
            ln = np.zeros(max(m, 1), np.uint64)
            if m:
                _check(lib().fpm_fp_text_refs(job, m, C.byref(nr), _p(first, u64p), _p(io, u64p),
                                              _p(il, u32p), _p(ln, u64p)))
            h = np.zeros(max(n, 1), np.uint64 if use64 else np.uint32)
            _check(lib().fpm_fp_text_fetch(job, None, None, None, h.ctypes.data, None))
        finally:
            lib().fpm_fp_text_free(job)
        return {"first": first[:m], "id_off": io[:m], "id_len": il[:m], "length": ln[:m],
                "hash": h[:n], "n_lines": n}

    def positional(self, ref_lists, qry_lists, use64=False, max_dist=1.0, max_pvalue=1.0):
        """triangle -fp's positional compare over the grid (query-major)."""
        dt = np.uint64 if use64 else np.uint32
        w = max([len(x) for x in list(ref_lists) + list(qry_lists)] + [1])
        R, rl = _dense(ref_lists, w, dt)
        Q, ql = _dense(qry_lists, w, dt)
        n = len(ref_lists) * len(qry_lists)
        nu = np.zeros(max(n, 1), np.uint32)
        de = np.zeros(max(n, 1), np.uint32)
        di = np.zeros(max(n, 1), np.float64)
        pv = np.zeros(max(n, 1), np.float64)
        pa = np.zeros(max(n, 1), np.uint8)
        _check(lib().fpm_fp_positional_grid(self.h, R.ctypes.data, _p(rl, u32p), w, len(ref_lists),
                                            Q.ctypes.data, _p(ql, u32p), w, len(qry_lists),
                                            8 if use64 else 4, max_dist, max_pvalue, _p(nu, u32p),
                                            _p(de, u32p), _p(di, f64p), _p(pv, f64p), _p(pa, u8p)))
        return {"numer": nu[:n], "denom": de[:n], "distance": di[:n], "pvalue": pv[:n],
                "pass": pa[:n].astype(bool)}


class RefSet:
    """fpm_refset_*: the reference rows stay on the device with their bucket index built
    once; dist() runs one query block against them (results as Context.dist)."""

    def __init__(self, ctx, ref_lists, sketch_size, use64=True, ref_lengths=None, width=None):
        self.ctx, self.use64, self.S = ctx, use64, int(sketch_size)
        self.dt = np.uint64 if use64 else np.uint32
        self.w = int(width or max([len(x) for x in ref_lists] + [1]))
        R, rl = _dense(ref_lists, self.w, self.dt)
        self.n = len(ref_lists)
        rL = np.ascontiguousarray(ref_lengths if ref_lengths is not None else
                                  [0] * self.n, dtype=np.uint64)
        h = vp()
        _check(lib().fpm_refset_create(ctx.h, R.ctypes.data, _p(rl, u32p), _p(rL, u64p), self.w,
                                       self.n, 8 if use64 else 4, self.S, C.byref(h)))
        self.h = h.value

    def dist(self, qry_lists, k=21, kmer_space=None, qry_lengths=None, max_dist=-1.0,
             max_pvalue=-1.0):
        Q, ql = _dense(qry_lists, self.w, self.dt)
        nq = len(qry_lists)
        n = self.n * nq
        qL = np.ascontiguousarray(qry_lengths if qry_lengths is not None else [0] * nq,
                                  dtype=np.uint64)
        if kmer_space is None:
            kmer_space = 4.0 ** k
        nu = np.zeros(max(n, 1), np.uint32)
        de = np.zeros(max(n, 1), np.uint32)
        di = np.zeros(max(n, 1), np.float64)
        pv = np.zeros(max(n, 1), np.float64)
        pa = np.zeros(max(n, 1), np.uint8)
        _check(lib().fpm_refset_dist(self.h, Q.ctypes.data, _p(ql, u32p), _p(qL, u64p), self.w,
                                     nq, self.S, k, kmer_space, max_dist, max_pvalue,
                                     _p(nu, u32p), _p(de, u32p), _p(di, f64p), _p(pv, f64p),
                                     _p(pa, u8p)))
        return {"numer": nu[:n], "denom": de[:n], "distance": di[:n], "pvalue": pv[:n],
                "pass": pa[:n].astype(bool)}

    def free(self):
        if self.h:
            lib().fpm_refset_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _dense(lists, width, dtype):
    m = np.zeros((max(len(lists), 1), max(width, 1)), dtype=dtype)
    lens = np.zeros(max(len(lists), 1), dtype=np.uint32)
    for i, l in enumerate(lists):
        m[i, : len(l)] = l
        lens[i] = len(l)
    return m, lens
