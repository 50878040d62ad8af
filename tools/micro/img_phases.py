"""tools/micro/img_phases.py — phase split of compare_grid_img_kernel (timing experiment).

Needs a build of the library with -DFPM_IMG_PHASES (thread 0 of every workgroup adds
s_memtime deltas per phase): FPMASH_LIB=<that .so> python3 tools/micro/img_phases.py
Phases: U staging, ref mapping (lower bounds), image staging, walk (wave 0).
"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "fp-mash_amd"))
import fpmash  # noqa: E402

rng = np.random.default_rng(1)
n, L, S = 2048, 2000, 1000
base = rng.integers(0, 2 ** 32, size=200000, dtype=np.uint64).astype(np.uint32)
lists = [np.where(rng.random(L) < 0.02, base[0], base[rng.integers(0, len(base), L)]).astype(np.uint32)
         for _ in range(n)]
with fpmash.Context(0) as ctx:
    ctx.set_dist_mode(fpmash.DIST_DENSE)
    ctx.dist(lists, lists, S, use64=False, k=1, kmer_space=10.0, ref_lengths=[L] * n, qry_lengths=[L] * n)
    lib = fpmash.lib()
    f = lib.fpm_debug_img_phases
    f.argtypes = [C.POINTER(C.c_ulonglong)]
    before = (C.c_ulonglong * 8)()
    f(before)
    t0 = time.perf_counter()
    ctx.dist(lists, lists, S, use64=False, k=1, kmer_space=10.0, ref_lengths=[L] * n, qry_lengths=[L] * n)
    wall = time.perf_counter() - t0
    after = (C.c_ulonglong * 8)()
    f(after)
    d = [after[i] - before[i] for i in range(4)]
    tot = sum(d)
    names = ["U staging", "ref mapping", "image staging", "walk (wave 0)"]
    print({k: round(v / tot, 3) for k, v in zip(names, d)}, "wall_ms", round(wall * 1e3, 1))
    tiles = ((n + 31) // 32) ** 2
    print("cycles per tile:", {k: int(v / tiles) for k, v in zip(names, d)})
