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
    """bench.Group over two gloo ranks: barrier / max / sum, one batch per rank, and the
    communicator agreement (one rank's RCCL set-up fails: neither rank uses one)."""
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
        # a failed communicator set-up on one rank: no rank uses one, and each says why
        assert x["comm_none"] and x["comm_error"], x
    assert "set-up failed" in r[0]["comm_error"] and "peer" in r[1]["comm_error"]
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
@pytest.mark.parametrize("ws", [2, 3])
def test_c4_leg_ranks_one_gpu(ws):
    """bench.c4_leg at world size 2 and 3 through libfpmash (all ranks on the one visible GPU,
    each sketching the rows its block pairs read, no collective): every rank's grids and
    transposes (block pairs, including the half-block split of even world sizes) match the
    oracle, and the ranks' cells add up to the whole n x n grid."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ws}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "_c4_gpu_worker.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = [json.loads(l.split(" ", 1)[1]) for l in p.stdout.splitlines() if l.startswith("C4RANK ")]
    assert sorted(r["rank"] for r in res) == list(range(ws))
    assert sum(r["cells"] for r in res) == res[0]["pairs"]
    for r in res:
        assert r["parity"]["ok"], r
        assert r["parity"]["pairs_sharing"] > 0
        assert any(j["kind"] == "mirror" for j in r["jobs"])


@pytest.mark.gpu
def test_vblocks_and_comm_one_gpu():
    """The N > 1 paths on the one GPU (tests/_vblocks_comm_worker.py): C4 with 2 and 3 virtual
    blocks (self / mirror jobs on locally sketched rows, no collective; every grid and transpose
    row sampled against the oracle; the cells add up to the whole grid), rank 3 of an N = 4
    run alone (it sketches its own block and the blocks it is paired with), and the RCCL
    min-merge inside libfpmash on a one-rank communicator against the oracle."""
    cmd = [sys.executable, os.path.join(ROOT, "tests", "_vblocks_comm_worker.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = [json.loads(l.split(" ", 1)[1]) for l in p.stdout.splitlines()
           if l.startswith("VBCOMM ")]
    assert len(res) == 1
    r = res[0]
    for vb, c in r["c4"].items():
        assert c["collective"] is None, c
        assert c["cells"] == c["pairs"], (vb, c)
        assert c["parity"]["ok"] and c["parity"]["pairs_sharing"] > 0, (vb, c)
        assert any(j["kind"] == "mirror" for j in c["jobs"])
    sh = r["share"]
    assert sh["parity"]["ok"] and sh["parity"]["pairs_sharing"] > 0, sh
    # rank 3 of 4: its block, block 0 (the cyclic next, (ws - 1) // 2 = 1 block) and the
    # even split's second index of block 1 against its own second half
    assert sh["rows_owned"] == 1000 and sh["rows_sketched"] == 3000, sh
    assert r["comm"]["ok"], r["comm"]


@pytest.mark.gpu
def test_comm_setup_bounded_without_peers():
    """fpm_comm_create for 2 ranks with only rank 0 present: the set-up gives up after
    FPM_COMM_INIT_TIMEOUT_S with an error naming the limit, instead of blocking for ever (the
    bench then reports the communicator missing and min-merges over gloo).  In a child
    process: an aborted communicator stays out of the test process."""
    code = (
        "import os, sys, time\n"
        f"sys.path[:0] = [{ROOT!r}, {os.path.join(ROOT, 'fp-mash_amd')!r}]\n"
        "os.environ['FPM_COMM_INIT_TIMEOUT_S'] = '4'\n"
        "import fpmash\n"
        "ctx = fpmash.Context(0)\n"
        "t0 = time.time()\n"
        "try:\n"
        "    fpmash.Comm(ctx, 2, 0, fpmash.comm_unique_id())\n"
        "    print('JOINED', flush=True)\n"
        "except Exception as e:\n"
        "    print('ERR', round(time.time() - t0, 1), e, flush=True)\n"
        "ctx.close()\n"
        "print('CLOSED', flush=True)\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith(("ERR", "JOINED"))][-1]
    assert line.startswith("ERR") and "FPM_COMM_INIT_TIMEOUT_S" in line, line
    assert 3.0 <= float(line.split()[1]) < 60.0, line


@pytest.mark.gpu
def test_c5_leg_two_ranks_one_gpu():
    """bench.c5_leg at world size 2 (both ranks on the one visible GPU, sketch rows gathered
    over gloo): uneven file shards (7 genomes over 2 ranks), and every genome of the ordered
    reassembly on rank 0 equals the oracle's sketch of that file (Sketch.cpp:346-356)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "_c5_gpu_worker.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = [json.loads(l.split(" ", 1)[1]) for l in p.stdout.splitlines()
           if l.startswith("C5RANK ")]
    assert sorted(r["rank"] for r in res) == [0, 1]
    assert sorted(r["genomes_local"] for r in res) == [3, 4]
    r0 = [r for r in res if r["rank"] == 0][0]
    assert r0["reassembled"] == 7
    assert r0["parity"]["genomes_checked"] == list(range(7))
    assert r0["parity"]["ok"] and all(r0["parity"]["sketch_exact"]), r0


def test_balanced_file_shards_cover_in_order():
    """bench.balanced_file_shards: contiguous, in file order, every file exactly once."""
    import bench
    for lengths, ws in [([5] * 7, 2), ([1, 100, 1, 1, 1], 2), ([3] * 1000, 8), ([1, 2], 4)]:
        sh = bench.balanced_file_shards(lengths, ws)
        assert len(sh) == ws and sh[0][0] == 0 and sh[-1][1] == len(lengths)
        assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        assert all(lo <= hi for lo, hi in sh)


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


@pytest.mark.parametrize("ws", [1, 2, 3, 4, 5, 6, 7, 8])
def test_pair_block_jobs_cover_every_cell_once(ws):
    """fpmash.shard.pair_block_jobs (the sharded C4 all-vs-all): over all ranks, every ordered
    cell (q, r) of the n x n grid is written exactly once, each unordered pair is compared on
    one rank only, and the ranks' compared pairs are balanced."""
    from fpmash.shard import job_cells, pair_block_jobs, shard_range
    import random
    rng = random.Random(ws)
    for n in (ws, 3 * ws + 1, 40):
        if n < ws:
            continue
        # uneven blocks (contiguous family shards), as bench.c4_leg makes them
        fams = max(ws, n // 3)
        fb = [shard_range(fams, ws, r) for r in range(ws)]
        cuts = sorted(rng.sample(range(1, n), fams - 1)) if fams > 1 else []
        edges = [0] + cuts + [n]
        bounds = [(edges[a], edges[b]) for a, b in fb]
        seen = {}
        work = []
        for r in range(ws):
            w = 0
            for j in pair_block_jobs(bounds, r):
                for c in job_cells(j):
                    seen[c] = seen.get(c, 0) + 1
                (rl, rh), (ql, qh) = j["ref"], j["qry"]
                w += (rh - rl) * (qh - ql) / (2 if j["kind"] == "self" else 1)
            work.append(w)
        assert len(seen) == n * n and set(seen.values()) == {1}, (ws, n)
        assert abs(sum(work) - n * n / 2) <= n, (work, n)


def test_pair_block_jobs_balanced_at_c4_shape():
    """At C4's 500 families x 100 members the per-rank compared pairs stay within 5 % of
    n^2 / (2 ws) at ws = 2, 4, 8 (the cells written within 5 % of n^2 / ws)."""
    from fpmash.shard import pair_block_jobs, shard_range
    n, members = 50_000, 100
    for ws in (2, 4, 8):
        bounds = [tuple(x * members for x in shard_range(n // members, ws, r)) for r in range(ws)]
        for r in range(ws):
            w = cells = 0
            for j in pair_block_jobs(bounds, r):
                (rl, rh), (ql, qh) = j["ref"], j["qry"]
                a = (rh - rl) * (qh - ql)
                w += a / 2 if j["kind"] == "self" else a
                cells += a if j["kind"] == "self" else 2 * a
            assert abs(w / (n * n / (2 * ws)) - 1) < 0.05, (ws, r, w)
            assert abs(cells / (n * n / ws) - 1) < 0.05, (ws, r, cells)
