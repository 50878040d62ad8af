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
# the communicator agreement: rank 0's RCCL set-up fails, rank 1's succeeds; neither uses
# one, and both know why (bench.Group.comm; stand-ins for fpmash.Comm / comm_unique_id)


class _Comm:
    def __init__(self, ctx, n, r, uid):
        if r == 0:
            raise RuntimeError("set-up failed")


bench.fpmash.Comm = _Comm
bench.fpmash.comm_unique_id = lambda: bytes(bench.fpmash.COMM_ID_BYTES)
os.environ.pop("FPMASH_BENCH_ONE_DEVICE", None)
c = g.comm(None)
out = {"rank": rank, "ws": ws, "max": mx, "sum": sm, "batch0": batch[0][:16].decode(),
       "n": len(batch), "comm_none": c is None, "comm_error": g.comm_error}
with open(os.environ["FPM_TEST_OUT"] + f".{rank}", "w") as f:
    json.dump(out, f)
