"""N>1 paths on CPU (gloo): the bench's barrier / max / sum helpers and
per-rank batch generation (independent, differently seeded batches per rank)."""
import json
import os
import socket
import subprocess
import sys

from conftest import ROOT


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_group(tmp_path):
    out = str(tmp_path / "res")
    env = dict(os.environ, FPM_TEST_OUT=out)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "_group_worker.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = [json.load(open(out + f".{i}")) for i in range(2)]
    for x in r:
        assert x["ws"] == 2 and x["max"] == 2.0 and x["sum"] == 30.0 and x["n"] == 40
    assert r[0]["batch0"] != r[1]["batch0"]   # each rank owns its own batch


def test_shard_gather_two_ranks():
    """C4 sharding (fpmash.shard): two gloo ranks sketch their shards, all-gather the sketch
    rows (uneven shards), and each rank's dist rows equal the single-process grid's."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "_shard_worker.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "shard-ok" in p.stdout
