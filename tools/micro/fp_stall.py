"""tools/micro/fp_stall.py — where the one-off slow -fp text call comes from.

Runs fpm_fp_text_stage on the bench's 1 M-line CFL text (30 MB) several times per variant and
prints each call's HIP-event kernel total and wall time:
  full     stage + fetch into fresh numpy arrays + free (what Context.fp_text does)
  nofetch  stage + free
  keep     stage + fetch into arrays allocated once + free
  sleep    like full, with a 50 ms host sleep between calls
Run it under `rocprofv3 --kernel-trace` for the per-dispatch durations."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fp-mash_amd")]
import numpy as np  # noqa: E402
import fpmash  # noqa: E402
from fpmash import datagen  # noqa: E402

text = datagen.cfl_text(datagen.random_dna(50, 2000, seed=3), datagen.lyn2vec_ids(50)) * 10
L = fpmash.lib()
reps = int(os.environ.get("REPS", 6))
with fpmash.Context(0) as ctx:
    keep = None

    def call(fetch, arrays=None):
        job, n = C.c_void_p(), C.c_uint64()
        fpmash._check(L.fpm_fp_text_stage(ctx.h, text, len(text), 1_000_000, 42, 0, C.byref(job),
                                          C.byref(n)))
        n = n.value
        if fetch:
            a = arrays or [np.zeros(n, t) for t in (np.uint64, np.uint32, np.uint32, np.uint32,
                                                    np.uint8)]
            P = fpmash._p
            fpmash._check(L.fpm_fp_text_fetch(job, P(a[0], fpmash.u64p), P(a[1], fpmash.u32p),
                                              P(a[2], fpmash.u32p), a[3].ctypes.data,
                                              P(a[4], fpmash.u8p)))
        L.fpm_fp_text_free(job)
        return n

    for variant in os.environ.get("VARIANTS", "full,nofetch,keep,sleep").split(","):
        if variant == "keep" and keep is None:
            keep = [np.zeros(1_000_000, t) for t in (np.uint64, np.uint32, np.uint32, np.uint32,
                                                     np.uint8)]
        for rep in range(reps):
            ctx.synchronize()
            ctx.reset_timing()
            ctx.set_timing(True)
            t0 = time.perf_counter()
            n = call(variant != "nofetch", keep if variant == "keep" else None)
            wall = time.perf_counter() - t0
            ctx.set_timing(False)
            tot, cnt = ctx.kernel_time(fpmash.K_FPTEXT)
            print(f"{variant} rep {rep}: events {tot:.3f} ms over {cnt} launches, "
                  f"wall {wall * 1e3:.2f} ms, lines {n}", flush=True)
            if variant == "sleep":
                time.sleep(0.05)
