#!/usr/bin/env python3
"""tools/micro/fill_rate.py — write rate of the no-shared-hash fill alone (fpm_dist_prefill_dev:
distance + p-value f64 and the pass byte of every cell, 17 B per cell) on an n x n grid."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
import fpmash  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ctx = fpmash.Context(0)
L = fpmash.lib()
cells = n * n
bufs = [fpmash.DeviceBuffer(ctx, cells * b) for b in (8, 8, 1)]
for i in range(reps + 1):
    if i == 1:
        ctx.synchronize()
        t0 = time.perf_counter()
    fpmash._check(L.fpm_dist_prefill_dev(ctx.h, n, n, 1.0, 1.0, bufs[0].ptr, bufs[1].ptr,
                                         bufs[2].ptr, None if os.environ.get("FPM_FILL_CUS") else ctx.stream))
ctx.synchronize()
dt = (time.perf_counter() - t0) / reps
print(f"n={n} cells={cells:.3g} bytes={cells * 17 / 1e9:.2f} GB  {dt * 1e3:.3f} ms  "
      f"{cells * 17 / dt / 1e12:.2f} TB/s  grid_cap={os.environ.get('FPM_FILL_GRID', '-')}")
