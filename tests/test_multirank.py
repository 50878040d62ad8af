"""N>1 paths on CPU (gloo): the bench's barrier / max / sum helpers and
per-rank batch generation (independent, differently seeded batches per rank)."""
import json
import os
import socket
import subprocess
import sys

import pytest

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


@pytest.mark.gpu
def test_c4_leg_two_ranks_one_gpu():
    """bench.c4_leg at world size 2 through libfpmash (both ranks on the one visible GPU,
    rows gathered over gloo): each rank's dist rows of the sharded job match the oracle."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "_c4_gpu_worker.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = [json.loads(l.split(" ", 1)[1]) for l in p.stdout.splitlines() if l.startswith("C4RANK ")]
    assert sorted(r["rank"] for r in res) == [0, 1]
    for r in res:
        assert r["parity"]["ok"], r
        assert r["parity"]["pairs_sharing"] > 0


@pytest.mark.gpu
def test_split_leg_two_ranks_one_gpu():
    """bench.split_leg at world size 2 (both ranks on the one visible GPU, bottom-s rows
    gathered over gloo, merged by fpm_sketch_merge_dev): the merged sketch of the split
    genome equals the whole genome's sketch."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "_split_gpu_worker.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = [json.loads(l.split(" ", 1)[1]) for l in p.stdout.splitlines()
           if l.startswith("SPLITRANK ")]
    assert sorted(r["rank"] for r in res) == [0, 1]
    r0 = [r for r in res if r["rank"] == 0][0]
    assert r0["parity"]["ok"] and r0["parity"]["merged_equals_whole"], r0


def test_kmer_shard_covers_every_kmer_once():
    """fpmash.shard.kmer_shard: the ranks' ranges hold every k-mer start exactly once."""
    from fpmash.shard import kmer_shard
    for L, k, w in [(100, 21, 1), (100, 21, 3), (1_000_003, 21, 8), (30, 21, 8), (5, 21, 2)]:
        starts = []
        for r in range(w):
            lo, hi = kmer_shard(L, k, w, r)
            starts += list(range(lo, max(lo, hi - k + 1)))
        assert starts == list(range(max(0, L - k + 1)))
