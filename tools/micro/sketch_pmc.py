import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "fp-mash_amd"))
import fpmash
from fpmash import datagen
ctx = fpmash.Context(0)
seqs = datagen.family_dna(100, 100, 2000, sub_rate=(0.01, 0.10), seed=1000)
P = fpmash.make_params(k=21, s=1000)
job = ctx.sketch_job(P, seqs)
for _ in range(5):
    job.run()
ctx.synchronize()
print("ok")
