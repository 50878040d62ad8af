"""Worker for test_multirank: the bench's barrier / max / sum over gloo ranks."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fp-mash_amd"))
import bench  # noqa: E402

ws, rank, local = bench.dist_env()
g = bench.Group(ws)
g.barrier()
mx = g.max(1.0 + rank)
sm = g.sum(10.0 * (rank + 1))
batch = bench.make_batch(bench.parse_args_for_test(n_seqs=40, seq_len=300, families=4), rank)
out = {"rank": rank, "ws": ws, "max": mx, "sum": sm, "batch0": batch[0][:16].decode(),
       "n": len(batch)}
with open(os.environ["FPM_TEST_OUT"] + f".{rank}", "w") as f:
    json.dump(out, f)
