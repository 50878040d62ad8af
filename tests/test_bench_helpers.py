"""CPU tests of the bench's host-side helpers: the C++ CFL generator (C3 inputs), the -fp
line grouping of the C3 leg, and the C4 leg's query-row sharding."""
import os

import numpy as np

from conftest import GOLDEN
import seqio


def test_cflgen_matches_lyn2vec_fixture():
    """bin/cflgen reproduces lyn2vec's DNA1-CFL.txt from DNA1.fasta byte for byte."""
    from fpmash import datagen
    recs = seqio.read_records(os.path.join(GOLDEN, "DNA1.fasta"))
    ids = [comment.split()[0].decode()[len("G00000"):] for _name, comment, _seq in recs]
    out = datagen.cfl_text_fast([seq for _n, _c, seq in recs], ids, threads=3)
    assert out == open(os.path.join(GOLDEN, "DNA1-CFL.txt"), "rb").read()


def test_cflgen_matches_python_generator():
    """Short records (one window), lowercase, non-ACGT bytes, long records."""
    from fpmash import datagen
    seqs = datagen.random_dna(7, 350, seed=9) + [b"acgtNNacg", b"ACGTACGTAC" * 30, b"A", b"tttt" * 40]
    ids = datagen.lyn2vec_ids(len(seqs), seed=2)
    assert datagen.cfl_text_fast(seqs, ids) == datagen.cfl_text(seqs, ids)
    assert datagen.cfl_text_fast(seqs, ids, window=17) == datagen.cfl_text(seqs, ids, window=17)


def test_c4_row_shards_cover_grid():
    """The C4 leg's query-row blocks partition [0, n) for every GPU count."""
    from fpmash.shard import shard_range
    for n in (1, 7, 50_000):
        for ws in (1, 2, 3, 4, 8):
            spans = [shard_range(n, ws, r) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_sub_rates_divide_by_event_timed_steps():
    """bench's sketch / dist sub-rates: kernel totals come from the event-timed steps run
    after the timed region, so per-step device time divides by their count."""
    import bench
    for steps, n in ((1, 3), (5, 5), (20, 10), (100, 10)):
        assert bench.timing_steps(steps) == n
    kt = {"a": {"total_ms": 1.8, "launches": 10, "avg_ms": 0.18},
          "b": {"total_ms": 0.2, "launches": 10, "avg_ms": 0.02}}
    ms = bench.per_step_ms(kt, ["a", "b", "missing"], bench.timing_steps(20))
    assert abs(ms - 0.2) < 1e-12          # = avg launch time summed over the kernels


def test_parity_summary():
    import bench
    p = bench.parity_summary({"ok": True}, {"parity": {"ok": True}}, None)
    assert p["all_ok"] is True and p["c4"] is None
    p = bench.parity_summary({"ok": True}, {"parity": {"ok": False}}, {"parity": None})
    assert p["all_ok"] is False


def test_c5_file_shards_balanced_by_bases():
    """bench.balanced_file_shards: contiguous file ranges covering every file once, in
    order, each rank's bases within one file of the even share."""
    import bench
    rng = np.random.default_rng(3)
    for ws in (1, 2, 3, 4, 8):
        for lengths in ([5] * 1000, list(rng.integers(1, 100, size=37)), [10, 1, 1, 1, 1, 10]):
            spans = bench.balanced_file_shards(lengths, ws)
            assert spans[0][0] == 0 and spans[-1][1] == len(lengths)
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            share = sum(lengths) / ws
            for lo, hi in spans:
                assert abs(sum(lengths[lo:hi]) - share) <= max(lengths)


def test_c5_genome_deterministic():
    import bench
    a = bench.c5_genome(7, 1001)
    assert a == bench.c5_genome(7, 1001) and a != bench.c5_genome(8, 1001)
    assert len(a) == 1001 and set(a) <= set(b"ACGT")


def test_headline_line_fits_driver_parser():
    """The printed line is built from the full result by compact_line and stays under the
    driver's parse limit (round 3's 26.8 KB line was not parsed).  Canned input: the full
    result of the round-3 bench, which carries every leg."""
    import json
    import bench
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    full = json.load(open(os.path.join(root, "profiles", "r03", "bench_r03_head_final.json")))
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) < bench.MAX_LINE_BYTES
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype",
              "config", "roofline", "cpu_baseline", "parity", "higher_is_better", "scaling",
              "vs_baseline", "data"):
        assert k in line, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert line["parity"]["all_ok"] is True
    assert all(isinstance(v, (bool, type(None))) for v in line["parity"].values())
    assert line["legs"]["c4_ms_per_step"] > 0 and line["legs"]["cli_dist_wall_s"] > 0
    # a pathological detail (huge strings) still yields a parseable line
    full["cpu_baseline"]["sample"] = "x" * 20000
    assert len(json.dumps(bench.compact_line(full))) < bench.MAX_LINE_BYTES
