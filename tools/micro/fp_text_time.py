"""tools/micro/fp_text_time.py — the bench's -fp text leg alone (1M CFL lines, 30 MB), with the
text staged once before timing, for rocprofv3 --kernel-trace: per-kernel durations of
nl_count / scan / nl_scatter / fp_line against the HIP-event total the bench reports."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fp-mash_amd")]
import fpmash
from fpmash import datagen

text = datagen.cfl_text(datagen.random_dna(50, 2000, seed=3), datagen.lyn2vec_ids(50)) * 10
with fpmash.Context(0) as ctx:
    for warm in (text[:100000], text):
        ctx.fp_text(warm, max_lines=1_000_000)
    for rep in range(int(os.environ.get('REPS', 3))):
        ctx.reset_timing(); ctx.set_timing(True)
        t0 = time.perf_counter()
        r = ctx.fp_text(text, max_lines=1_000_000)
        wall = time.perf_counter() - t0
        ctx.set_timing(False)
        tot, cnt = ctx.kernel_time(fpmash.K_FPTEXT)
        print(f"rep {rep}: events {tot:.3f} ms over {cnt} launches, wall {wall*1e3:.2f} ms, lines {len(r['hash'])}")
