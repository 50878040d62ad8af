"""The drop-in host CLI (`fp-mash_amd/bin/fpmash`) against the reference's fixtures.

CPU tests: .msh reader/writer round trip on every fixture sketch, `info -d` vs the
fork's own JSON dump, `info -t`, loud failure without a device.
GPU tests: `sketch -fp` byte-identical to DNA{1,2,3}-sketch.msh (plus the stdout
messages), `sketch` of FASTA/FASTQ vs the fixtures, `dist` vs genomes.dist and vs
the oracle for -fp inputs.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
import mshfmt
import seqio

FPMASH = os.path.join(ROOT, "fp-mash_amd", "bin", "fpmash")
ROUNDTRIP = os.path.join(ROOT, "fp-mash_amd", "bin", "msh_roundtrip")
REF_MSH = ["DNA1-sketch.msh", "DNA2-sketch.msh", "DNA3-sketch.msh", "genome1.fna.msh",
           "genome2.fna.msh", "genome3.fna.msh", "read1_2.msh", "reads.msh", "test_sequence.msh"]


def run(args, cwd=None, check=True, env=None):
    p = subprocess.run([FPMASH] + args, cwd=cwd, capture_output=True,
                       env=None if env is None else {**os.environ, **env})
    if check and p.returncode != 0:
        raise AssertionError(f"fpmash {args} failed: {p.stderr.decode()}")
    return p


@pytest.mark.parametrize("name", REF_MSH)
def test_msh_writer_byte_identical_roundtrip(name):
    p = subprocess.run([ROUNDTRIP, os.path.join(GOLDEN, name)], capture_output=True, text=True)
    assert p.returncode == 0 and p.stdout.startswith("same"), p.stdout + p.stderr


@pytest.mark.parametrize("name", REF_MSH)
def test_python_msh_writer_pinned_to_fixtures(name):
    """The test-side encoder (mshfmt.write_msh, independent of host/Msh.cpp) rebuilds
    every fixture .msh byte for byte from its decoded content: it is the expected-bytes
    oracle of the full-size .msh tests below."""
    data = open(os.path.join(GOLDEN, name), "rb").read()
    h = mshfmt.read_msh(data)
    use64 = h["references"][0]["hashes64"] is not None
    refs = [dict(name=r["name"], comment=r["comment"], length=r["length"],
                 hashes=r["hashes64"] if use64 else r["hashes32"], counts=r["counts"])
            for r in h["references"]]
    out = mshfmt.write_msh(h, refs, use64=use64,
                           counts=any(r["countsSorted"] for r in h["references"]))
    assert out == data


def test_info_json_matches_fork_dump():
    out = run(["info", "-d", os.path.join(GOLDEN, "DNA1-sketch.msh")]).stdout
    assert out == open(os.path.join(GOLDEN, "DNA1-sketch.json"), "rb").read()


def test_info_tabular_and_header():
    out = run(["info", "-t", os.path.join(GOLDEN, "read1_2.msh")]).stdout.decode()
    lines = out.splitlines()
    assert lines[0] == "#Hashes\tLength\tID\tComment"
    assert lines[1].startswith("1000\t297777\t./test/reads1.fastq\t[1000 seqs] ")
    hdr = run(["info", "-H", os.path.join(GOLDEN, "DNA1-sketch.msh")]).stdout.decode()
    assert "K-mer size:                    1 (32-bit hashes)" in hdr
    assert "Alphabet:                      0123456789\n" in hdr
    assert "Sketches:                      5" in hdr


def test_info_counts_histogram_and_dump():
    """info -c (printCounts, CommandInfo.cpp:225-262) and the counts block of info -d on the
    reference's counted sketch reads.msh; -c on a sketch without counts fails as the reference's."""
    h = mshfmt.read_msh(os.path.join(GOLDEN, "reads.msh"))["references"][0]
    vals, freq = np.unique(h["counts"], return_counts=True)
    exp = "#Sketch\tBin\tFrequency\n" + "".join(f"reads\t{v}\t{f}\n" for v, f in zip(vals, freq))
    assert run(["info", "-c", os.path.join(GOLDEN, "reads.msh")]).stdout.decode() == exp
    d = run(["info", "-d", os.path.join(GOLDEN, "reads.msh")]).stdout.decode()
    tail = d[d.index('      "counts" :\n'):]
    body = tail[tail.index("[\n") + 2:tail.index("      ]")]
    assert [int(x.strip().rstrip(",")) for x in body.splitlines()] == list(h["counts"])
    assert d.index('      "counts" :') > d.index('      "hashes" :')
    p = run(["info", "-c", os.path.join(GOLDEN, "DNA1-sketch.msh")], check=False)
    assert p.returncode == 1 and b"does not have hash counts" in p.stderr


def test_cli_fails_loudly_without_device():
    import fpmash
    if fpmash.device_count() > 0:
        pytest.skip("device present")
    p = run(["sketch", "-fp", os.path.join(GOLDEN, "DNA1-CFL.txt"), "-o", "/tmp/fpm_nodev"],
            check=False)
    assert p.returncode != 0 and b"no CPU fallback" in p.stderr


def test_dist_failure_leaves_output_file_as_it_was(tmp_path):
    """`dist ... > file` sizes the file ahead of its text (pages allocated while the devices
    come up); an error exit cuts it back to what it held before the command."""
    import fpmash
    if fpmash.device_count() > 0:
        pytest.skip("device present")
    out = tmp_path / "out.tsv"
    out.write_bytes(b"head\n")
    with open(out, "r+b") as f:
        f.seek(0, 2)
        p = subprocess.run([FPMASH, "dist", os.path.join(GOLDEN, "genome1.fna.msh"),
                            os.path.join(GOLDEN, "genome2.fna.msh")], stdout=f,
                           stderr=subprocess.PIPE)
    assert p.returncode == 1 and b"no CPU fallback" in p.stderr
    assert out.read_bytes() == b"head\n"


def test_option_errors():
    p = run(["sketch", "-k", "40", "x.fa"], check=False)
    assert p.returncode != 0 and b"must be an integer between 1 and 32" in p.stderr
    p = run(["dist", "-Q", "a", "b"], check=False)
    assert p.returncode == 1 and b"Unrecognized option: -Q" in p.stderr


# ----------------------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("i", [1, 2, 3])
def test_sketch_fp_byte_identical(tmp_path, i):
    """`fpmash sketch -fp DNA{i}-CFL.txt` == the fork's DNA{i}-sketch.msh, byte for byte."""
    src = os.path.join(GOLDEN, f"DNA{i}-CFL.txt")
    shutil.copy(src, tmp_path / f"DNA{i}-CFL.txt")
    p = run(["sketch", "-fp", f"DNA{i}-CFL.txt", "-o", f"DNA{i}-sketch"], cwd=tmp_path)
    assert p.stdout.decode() == ("Initializing from fingerprints...\n"
                                 f"Processing file: DNA{i}-CFL.txt\nInitialization complete.\n")
    assert p.stderr.decode() == f"Writing to DNA{i}-sketch.msh...\n"
    got = open(tmp_path / f"DNA{i}-sketch.msh", "rb").read()
    assert got == open(os.path.join(GOLDEN, f"DNA{i}-sketch.msh"), "rb").read()


@pytest.mark.gpu
def test_sketch_fasta_byte_identical(tmp_path):
    """`sketch new_data/test_sequence.fasta` (concatenated, 2 records) == test_sequence.msh."""
    os.makedirs(tmp_path / "new_data")
    shutil.copy(os.path.join(GOLDEN, "test_sequence.fasta"), tmp_path / "new_data")
    run(["sketch", "new_data/test_sequence.fasta", "-o", "ts"], cwd=tmp_path)
    assert open(tmp_path / "ts.msh", "rb").read() == \
        open(os.path.join(GOLDEN, "test_sequence.msh"), "rb").read()


@pytest.mark.gpu
def test_sketch_fastq_gz_hashes(tmp_path):
    """Reads with N and quality lines, gzip input: hashes/length == read1_2.msh."""
    exp = mshfmt.read_msh(os.path.join(GOLDEN, "read1_2.msh"))["references"]
    run(["sketch", "-o", str(tmp_path / "r"), os.path.join(GOLDEN, "reads1.fastq.gz"),
         os.path.join(GOLDEN, "reads2.fastq.gz")])
    got = mshfmt.read_msh(str(tmp_path / "r.msh"))["references"]
    for g, e in zip(got, exp):
        assert np.array_equal(g["hashes64"], e["hashes64"])
        assert g["length"] == e["length"]
        assert g["comment"].replace(b"\r", b"") == e["comment"].replace(b"\r", b"")


@pytest.mark.gpu
def test_sketch_individual_matches_oracle(tmp_path, oracle):
    from fpmash import datagen
    seqs = datagen.family_dna(3, 5, 3000, seed=9) + [b"ACGTN" * 10, b"AC"]
    ids = datagen.lyn2vec_ids(len(seqs))
    (tmp_path / "x.fa").write_bytes(datagen.fasta_bytes(seqs, ids))
    run(["sketch", "-i", "-o", "x", "x.fa"], cwd=tmp_path)
    got = mshfmt.read_msh(str(tmp_path / "x.msh"))
    exp = oracle.sketch_batch(oracle.params(), [s for s in seqs if len(s) >= 21])
    assert [r["name"] for r in got["references"]] == \
        [b"T00000" + i.encode() for s, i in zip(seqs, ids) if len(s) >= 21]
    for r, e in zip(got["references"], exp):
        h = r["hashes64"] if r["hashes64"] is not None else np.zeros(0, np.uint64)
        assert np.array_equal(h, e)
    assert not got["concatenated"]


@pytest.mark.gpu
@pytest.mark.parametrize("individual", [False, True])
def test_sketch_files_over_devices(tmp_path, oracle, individual):
    """Several input files spread over the devices (contiguous ranges balanced by bytes; three
    contexts on the one GPU stand in for a node): the .msh is byte-identical to the one-device
    run, and every sketch equals the oracle's."""
    from fpmash import datagen
    names, per_file = [], []
    for f, (n, L) in enumerate([(1, 40000), (7, 900), (3, 5000), (2, 25), (12, 1500)]):
        seqs = datagen.family_dna(1, n, L, seed=50 + f)[:n]
        ids = datagen.lyn2vec_ids(len(seqs))
        (tmp_path / f"f{f}.fa").write_bytes(datagen.fasta_bytes(seqs, ids))
        names.append(f"f{f}.fa")
        per_file.append(seqs)
    flags = ["-i"] if individual else []
    run(["sketch"] + flags + ["-o", "one"] + names, cwd=tmp_path, env={"FPMASH_DEVICE_LIST": "0"})
    run(["sketch"] + flags + ["-o", "many"] + names, cwd=tmp_path,
        env={"FPMASH_DEVICE_LIST": "0,0,0"})
    one = (tmp_path / "one.msh").read_bytes()
    assert (tmp_path / "many.msh").read_bytes() == one
    got = mshfmt.read_msh(one)["references"]
    if individual:
        exp = oracle.sketch_batch(oracle.params(), [s for seqs in per_file for s in seqs
                                                    if len(s) >= 21])
    else:
        flat = [s for seqs in per_file for s in seqs]
        groups = [f for f, seqs in enumerate(per_file) for _ in seqs]
        exp = oracle.sketch_batch(oracle.params(), flat, groups=groups, n_groups=len(per_file))
    assert len(got) == len(exp)
    for r, e in zip(got, exp):
        h = r["hashes64"] if r["hashes64"] is not None else np.zeros(0, np.uint64)
        assert np.array_equal(h, e)


@pytest.mark.gpu
@pytest.mark.parametrize("individual", [False, True])
def test_sketch_counts_M(tmp_path, oracle, individual):
    """`sketch -M`: counts32 of every sketch == the oracle heap's multiplicities, and the file
    is the byte layout of the pinned encoder (mshfmt.write_msh reproduces the counted fixture
    reads.msh); `info -c` prints their histograms."""
    from fpmash import datagen
    rng = np.random.default_rng(5)
    unit = datagen.family_dna(1, 1, 300, seed=4)[0]
    per_file = [datagen.family_dna(1, 3, 4000, seed=7) + [unit * 9],
                [unit * 3 + datagen.family_dna(1, 1, 900, seed=8)[0]],
                datagen.family_dna(2, 4, 1500, seed=9)]
    names = []
    for f, seqs in enumerate(per_file):
        ids = datagen.lyn2vec_ids(len(seqs), seed=f)
        (tmp_path / f"m{f}.fa").write_bytes(datagen.fasta_bytes(seqs, ids))
        names.append(f"m{f}.fa")
    flags = ["-i"] if individual else []
    run(["sketch", "-M", "-s", "500"] + flags + ["-o", "m"] + names, cwd=tmp_path)
    data = (tmp_path / "m.msh").read_bytes()
    h = mshfmt.read_msh(data)
    got = h["references"]
    O = oracle.params(k=21, s=500)
    if individual:
        flat = [s for seqs in per_file for s in seqs]
        eh, ec = oracle.sketch_batch(O, flat, counts=True)
    else:
        flat = [s for seqs in per_file for s in seqs]
        groups = [f for f, seqs in enumerate(per_file) for _ in seqs]
        eh, ec = oracle.sketch_batch(O, flat, groups=groups, n_groups=len(per_file), counts=True)
    assert len(got) == len(eh)
    for r, a, c in zip(got, eh, ec):
        assert np.array_equal(r["hashes64"], a)
        assert np.array_equal(r["counts"], c)
        assert r["countsSorted"]
    assert any(c.max() > 1 for c in ec)
    refs = [dict(name=r["name"], comment=r["comment"], length=r["length"], hashes=r["hashes64"],
                 counts=r["counts"]) for r in got]
    assert mshfmt.write_msh(h, refs, use64=True, counts=True) == data
    out = run(["info", "-c", str(tmp_path / "m.msh")]).stdout.decode().splitlines()
    assert out[0] == "#Sketch\tBin\tFrequency"
    assert len(out) - 1 == sum(len(np.unique(c)) for c in ec)


def c2_fasta(n=10000, seed=1000):
    """Config C2's input: n x 2 kb family-structured lyn2vec-shaped records (the bench batch
    of rank 0) as one FASTA file."""
    from fpmash import datagen
    seqs = datagen.family_dna(100, n // 100, 2000, sub_rate=(0.01, 0.10), seed=seed)[:n]
    ids = datagen.lyn2vec_ids(len(seqs))
    return seqs, ids, datagen.fasta_bytes(seqs, ids)


@pytest.mark.gpu
def test_sketch_c2_10k_msh_byte_identical(tmp_path, oracle):
    """North star "bit-identical .msh" at config C2's full size: `sketch -i -k 21 -s 1000`
    of 10,000 x 2 kb records through the drop-in CLI == the .msh the oracle's sketches
    encode to (mshfmt.write_msh, pinned to every fixture), byte for byte."""
    seqs, ids, fa = c2_fasta()
    (tmp_path / "c2.fa").write_bytes(fa)
    run(["sketch", "-i", "-k", "21", "-s", "1000", "-o", "c2", "c2.fa"], cwd=tmp_path)
    got = (tmp_path / "c2.msh").read_bytes()
    exp_h = oracle.sketch_batch(oracle.params(k=21, s=1000), seqs, threads=8)
    refs = [dict(name=b"T00000" + i.encode(), comment=b"G00000" + i.encode(), length=len(s),
                 hashes=h) for s, i, h in zip(seqs, ids, exp_h)]
    hdr = dict(kmer=21, windowSize=0, sketchSize=1000, concatenated=False, noncanonical=False,
               preserveCase=False, error=0.0, seed=42, alphabet=b"ACGT")
    exp = mshfmt.write_msh(hdr, refs)
    assert len(got) == len(exp)
    assert got == exp


@pytest.mark.gpu
def test_c1_two_files_sketch_then_dist(tmp_path, oracle):
    """Config C1 end to end: two FASTA files of one 2,000 bp record each
    (uniform ACGT, seed 1, lyn2vec headers), `sketch -k 21 -s 1000 a.fa b.fa -o ab` (default
    concatenated mode: one sketch per file, named by the file, commented by its first record)
    then `dist ab.msh ab.msh`: the .msh equals the oracle's sketches encoded by the pinned
    writer, byte for byte, and the four dist lines equal the oracle's (query-major, %g)."""
    from fpmash import datagen
    rng = np.random.default_rng(1)
    seqs = [bytes(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 2000)]) for _ in range(2)]
    ids = datagen.lyn2vec_ids(2)
    for name, s, i in zip(("a.fa", "b.fa"), seqs, ids):
        (tmp_path / name).write_bytes(datagen.fasta_bytes([s], [i]))
    run(["sketch", "-k", "21", "-s", "1000", "a.fa", "b.fa", "-o", "ab"], cwd=tmp_path)
    got = (tmp_path / "ab.msh").read_bytes()
    exp_h = oracle.sketch_batch(oracle.params(k=21, s=1000), seqs)
    refs = [dict(name=f.encode(), comment=b"T00000" + i.encode() + b" G00000" + i.encode(),
                 length=len(s), hashes=h) for f, s, i, h in zip(("a.fa", "b.fa"), seqs, ids, exp_h)]
    hdr = dict(kmer=21, windowSize=0, sketchSize=1000, concatenated=True, noncanonical=False,
               preserveCase=False, error=0.0, seed=42, alphabet=b"ACGT")
    assert got == mshfmt.write_msh(hdr, refs)
    out = run(["dist", "ab.msh", "ab.msh"], cwd=tmp_path).stdout.decode().splitlines()
    exp = []
    for qn, qs, qh in zip(("a.fa", "b.fa"), seqs, exp_h):
        for rn, rs, rh in zip(("a.fa", "b.fa"), seqs, exp_h):
            nu, de = oracle.compare(rh, qh, 1000, use64=True)
            d = oracle.distance(nu, de, 21)
            pv = oracle.pvalue(nu, len(rs), len(qs), 4.0 ** 21, de)
            exp.append(f"{rn}\t{qn}\t{d:g}\t{pv:g}\t{nu}/{de}")
    assert out == exp


@pytest.mark.gpu
def test_dist_genomes_golden():
    """mash/test/ref/genomes.dist: distance, p-value and shared-hash fields."""
    lines = open(os.path.join(GOLDEN, "genomes.dist")).read().splitlines()
    for i, line in enumerate(lines, 1):
        out = run(["dist", os.path.join(GOLDEN, f"genome{i}.fna.msh"),
                   os.path.join(GOLDEN, "reads.msh")]).stdout.decode().splitlines()
        assert len(out) == 1
        g, e = out[0].split("\t"), line.split("\t")
        assert g[0] == f"data/genome{i}.fna" and g[1] == "reads"
        assert g[2:] == e[2:]


@pytest.mark.gpu
def test_dist_fp_txt_matches_oracle(oracle):
    """`dist -fp DNA1-CFL.txt DNA2-CFL.txt DNA1-CFL.txt`: unsorted 2000-entry lists walked
    literally with S=1000, stdout messages interleaved as the reference prints them."""
    a, b = os.path.join(GOLDEN, "DNA1-CFL.txt"), os.path.join(GOLDEN, "DNA2-CFL.txt")
    p = run(["dist", "-fp", a, b, a])
    out = p.stdout.decode().splitlines()
    assert out[:3] == ["Initializing from fingerprints...", f"Processing file: {a}",
                       "Initialization complete."]
    assert out[3:7] == ["Initializing from fingerprints...", f"Processing file: {b}",
                        f"Processing file: {a}", "Initialization complete."]
    refs, _, _ = oracle.fp_references(open(a, "rb").read())
    q1, used, last = oracle.fp_references(open(b, "rb").read())
    q2, _, _ = oracle.fp_references(open(a, "rb").read(), lines_used=used, last_id=last)
    qrys = q1 + q2
    exp = []
    for qn, ql, qh in qrys:
        for rn, rl, rh in refs:
            nu, de = oracle.compare(rh, qh, 1000, use64=False)
            d = oracle.distance(nu, de, 1)
            pv = oracle.pvalue(nu, rl, ql, 10.0, de)
            exp.append(f"{rn.decode()}\t{qn.decode()}\t{d:g}\t{pv:g}\t{nu}/{de}")
    assert out[7:] == exp
    assert b"WARNING: For the k-mer size used (1)" in p.stderr


@pytest.mark.gpu
def test_dist_fp_msh_and_table(tmp_path, oracle):
    for i in (1, 2):
        shutil.copy(os.path.join(GOLDEN, f"DNA{i}-sketch.msh"), tmp_path)
    out = run(["dist", "-fp", "-t", "DNA1-sketch.msh", "DNA2-sketch.msh"],
              cwd=tmp_path).stdout.decode().splitlines()
    r = mshfmt.read_msh(str(tmp_path / "DNA1-sketch.msh"))["references"]
    q = mshfmt.read_msh(str(tmp_path / "DNA2-sketch.msh"))["references"]
    assert out[0] == "#query\t" + "\t".join(x["name"].decode() for x in r)
    for qi, row in enumerate(out[1:]):
        cells = row.split("\t")
        assert cells[0] == q[qi]["name"].decode()
        for ri, c in enumerate(cells[1:]):
            nu, de = oracle.compare(r[ri]["hashes32"][:1000], q[qi]["hashes32"][:1000], 1000,
                                    use64=False)
            assert c == "%g" % oracle.distance(nu, de, 1)


# ----------------------------------------------------------------------------- paste


@pytest.mark.parametrize("name,fp", [("read1_2.msh", False), ("fingerprint_example1_2.msh", True)])
def test_paste_reassembles_fixture(tmp_path, name, fp):
    """Split a two-sketch fixture into one .msh per sketch (the byte-exact writer), paste
    them back: the result is the fixture, byte for byte (read1_2.msh: the fork's
    test/paste_example, fingerprint_example1_2.msh: its `paste -fp` example)."""
    p = subprocess.run([ROUNDTRIP, "--split", os.path.join(GOLDEN, name), str(tmp_path / "part")],
                       capture_output=True, text=True)
    assert p.returncode == 0 and p.stdout.strip() == "2"
    if fp:
        for i in (0, 1):
            (tmp_path / f"part{i}.txt").write_text("")      # -fp wants the .txt siblings
        args = ["paste", "-fp", "part0.txt", "part1.msh", "-o", "joined"]
    else:
        args = ["paste", "joined", "part0.msh", "part1.msh"]
    r = run(args, cwd=tmp_path)
    assert r.stderr.decode() == "Writing joined.msh...\n"
    assert (tmp_path / "joined.msh").read_bytes() == open(os.path.join(GOLDEN, name), "rb").read()


def test_paste_errors(tmp_path):
    shutil.copy(os.path.join(GOLDEN, "read1_2.msh"), tmp_path)
    p = run(["paste", "-l", "-fp", "o", "read1_2.msh"], cwd=tmp_path, check=False)
    assert p.returncode == 1 and b"The options -l and -fp are incompatible." in p.stderr
    p = run(["paste", "o", "x.fa"], cwd=tmp_path, check=False)
    assert p.returncode == 1 and b'"x.fa" does not look like a sketch.' in p.stderr
    p = run(["paste", "-fp", "o", "a.txt"], cwd=tmp_path, check=False)
    assert p.returncode == 1 and b'"a.msh" does not exist but is required.' in p.stderr
    p = run(["paste", "-fp", "o", "read1_2.msh"], cwd=tmp_path, check=False)
    assert p.returncode == 1 and b'"read1_2.txt" does not exist but is required.' in p.stderr
    run(["paste", "o", "read1_2.msh"], cwd=tmp_path)
    p = run(["paste", "o", "read1_2.msh"], cwd=tmp_path, check=False)
    assert p.returncode == 1 and b'"o.msh" exists; remove to write.' in p.stderr


# ----------------------------------------------------------------------------- triangle


def _triangle_rows(text):
    lines = text.splitlines()
    n = int(lines[0].strip())
    names = [lines[1]] + [l.split("\t")[0] for l in lines[2:]]
    vals = [[float(x) for x in l.split("\t")[1:]] for l in lines[2:]]
    return n, names, vals


@pytest.mark.gpu
def test_triangle_msh_matrix_and_edges(oracle):
    files = [os.path.join(GOLDEN, f) for f in
             ("genome1.fna.msh", "genome2.fna.msh", "genome3.fna.msh", "reads.msh")]
    p = run(["triangle"] + files)
    n, names, vals = _triangle_rows(p.stdout.decode())
    refs = [r for f in files for r in mshfmt.read_msh(f)["references"]]
    assert n == 4 and names == [r["name"].decode() for r in refs]
    peak = 0.0
    for i in range(1, n):
        assert len(vals[i - 1]) == i
        for j in range(i):
            nu, de = oracle.compare(refs[i]["hashes64"], refs[j]["hashes64"], 1000)
            d = oracle.distance(nu, de, 21)
            pv = oracle.pvalue(nu, refs[i]["length"], refs[j]["length"], 4.0 ** 21, de)
            assert ("%g" % vals[i - 1][j]) == ("%g" % d)
            peak = max(peak, pv)
    assert p.stderr.decode().startswith("Max p-value: ")
    assert float(p.stderr.decode().split(":")[1]) == pytest.approx(float("%g" % peak), rel=1e-5)
    e = run(["triangle", "-E"] + files).stdout.decode().splitlines()
    assert len(e) == n * (n - 1) // 2
    f1 = e[0].split("\t")
    assert f1[0] == names[1] and f1[1] == names[0] and "/" in f1[4]
    d = run(["triangle", "-d", "0.1"] + files).stdout.decode().splitlines()
    assert all(float(x.split("\t")[2]) <= 0.1 for x in d)


@pytest.mark.gpu
def test_triangle_fp_positional(oracle):
    """triangle -fp: positional compare (matches at equal positions), chi-square p-value."""
    f = os.path.join(GOLDEN, "DNA1-CFL.txt")
    p = run(["triangle", "-fp", "-E", f])
    refs, _, _ = oracle.fp_references(open(f, "rb").read())
    exp = []
    for i in range(1, len(refs)):
        for j in range(i):
            m, mn, dv, pv = oracle.positional(refs[i][2], refs[j][2])
            exp.append((refs[i][0].decode(), refs[j][0].decode(), "%g" % dv, "%g" % pv,
                        f"{m}/{mn}"))
    got = [tuple(l.split("\t")) for l in p.stdout.decode().splitlines()
           if not l.startswith(("Initializing", "Processing", "Initialization"))]
    assert got == exp


@pytest.mark.gpu
def test_positional_grid_abi(ctx, oracle):
    rng = np.random.default_rng(5)
    lists = [rng.integers(0, 20, size=int(rng.integers(0, 60))).astype(np.uint32) for _ in range(9)]
    got = ctx.positional(lists, lists, max_dist=0.9, max_pvalue=0.5)
    for q, b in enumerate(lists):
        for r, a in enumerate(lists):
            m, mn, dv, pv = oracle.positional(a, b)
            k = q * len(lists) + r
            assert got["numer"][k] == m and got["denom"][k] == mn
            if mn:
                assert got["distance"][k] == pytest.approx(dv, rel=1e-12)
            else:
                assert np.isnan(got["distance"][k])
            assert got["pvalue"][k] == pytest.approx(pv, rel=1e-12)
            assert got["pass"][k] == (dv <= 0.9 and pv <= 0.5)


def _oracle_dist_lines(oracle, refs, qrys, S, k, space, comment=False):
    """writeOutput's lines (CommandDistance.cpp:276-333) from the oracle's grid."""
    nu, de, di, pv = oracle.dist_grid([r["hashes64"] for r in refs], [r["length"] for r in refs],
                                      [q["hashes64"] for q in qrys], [q["length"] for q in qrys],
                                      S, k, space)
    out = []
    n = len(refs)
    for qi, q in enumerate(qrys):
        qn = q["name"].decode() + (":" + q["comment"].decode() if comment else "")
        for ri, r in enumerate(refs):
            x = qi * n + ri
            rn = r["name"].decode() + (":" + r["comment"].decode() if comment else "")
            out.append(f"{rn}\t{qn}\t{di[x]:g}\t{pv[x]:g}\t{nu[x]}/{de[x]}")
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("block_pairs,to_file,devices,knobs,extra",
                         [(None, False, None, {}, []), ("50000", False, None, {}, []),
                          (None, True, None, {}, []), ("50000", True, None, {}, []),
                          ("50000", False, "0,0", {}, []), ("50000", True, "0,0,0", {}, []),
                          ("50000", True, None, {"FPMASH_DIST_PREALLOC": "0"}, []),
                          ("50000", True, None, {}, ["-d", "0.2"]),
                          ("50000", True, None, {}, ["-C"])])
def test_dist_resident_blocks_text_exact(tmp_path, oracle, block_pairs, to_file, devices, knobs,
                                         extra):
    """`dist all.msh all.msh` through the resident reference set: one block, and 30+ query
    blocks of 50,000 pairs (FPMASH_DIST_BLOCK_PAIRS) written by the formatter threads in
    order: every line equals the oracle's, in the reference's query-major order.  With
    FPMASH_DEVICE_LIST the blocks go round the contexts (2-3 on the one GPU standing in for
    a node's devices).  A regular file as stdout takes one pwritev() per block at its offset,
    with and without its pages allocated ahead (FPMASH_DIST_PREALLOC=0), with a -d filter (no
    estimate: the file grows as the blocks come) and with -C (name:comment on both sides of
    every line)."""
    from fpmash import datagen
    seqs = datagen.family_dna(12, 100, 2000, sub_rate=(0.01, 0.10), seed=23)
    ids = datagen.lyn2vec_ids(len(seqs), seed=23)
    (tmp_path / "all.fa").write_bytes(datagen.fasta_bytes(seqs, ids))
    run(["sketch", "-i", "-o", "all", "all.fa"], cwd=tmp_path)
    env = dict(os.environ)
    env.update(knobs)
    if block_pairs:
        env["FPMASH_DIST_BLOCK_PAIRS"] = block_pairs
    if devices:
        env["FPMASH_DEVICE_LIST"] = devices
    cmd = [FPMASH, "dist", "-p", "4"] + extra + ["all.msh", "all.msh"]
    if to_file:
        # stdout a regular file; it starts with bytes already written (the offsets start after
        # them, off a page boundary)
        with open(tmp_path / "out.tsv", "wb") as f:
            f.write(b"head\n")
            f.flush()
            p = subprocess.run(cmd, cwd=tmp_path, stdout=f, stderr=subprocess.PIPE, env=env)
        text = (tmp_path / "out.tsv").read_bytes()
        assert text.startswith(b"head\n") and text.endswith(b"\n")
        text = text[5:]
    else:
        p = subprocess.run(cmd, cwd=tmp_path, capture_output=True, env=env)
        text = p.stdout
    assert p.returncode == 0, p.stderr.decode()
    refs = mshfmt.read_msh(str(tmp_path / "all.msh"))["references"]
    exp = _oracle_dist_lines(oracle, refs, refs, 1000, 21, 4.0 ** 21, comment="-C" in extra)
    assert len(exp) == len(refs) ** 2
    if "-d" in extra:
        # compareSketches (CommandDistance.cpp:421-429): a pair past -d is not written
        exp = [x for x in exp if float(x.split("\t")[2]) <= 0.2]
        assert 0 < len(exp) < len(refs) ** 2
    got = text.decode().splitlines()
    assert len(got) == len(exp)
    assert got == exp


def _bgzf(data: bytes, block=65280) -> bytes:
    """BGZF (SAM spec 4.1): raw-deflate blocks of <= 64 KiB, each a gzip member whose extra
    field 'BC' holds the member's size - 1, then the 28-byte empty EOF member."""
    import struct
    import zlib
    out = []
    for i in range(0, len(data), block):
        raw = data[i:i + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        d = c.compress(raw) + c.flush()
        bsize = 18 + len(d) + 8
        out.append(b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" +
                   struct.pack("<H", bsize - 1) + d +
                   struct.pack("<II", zlib.crc32(raw) & 0xffffffff, len(raw)))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def test_seqload_gzip_forms(tmp_path):
    """loadSequenceFile (host/SeqReader.cpp, through bin/seqload) inflates like zlib's gzread,
    which the reference's kseq reads through (Sketch.cpp:38): plain text, one gzip member,
    several members, BGZF (members inflated on several threads), a member followed by
    non-gzip bytes (ignored, as gz_look does), and a truncated member (what inflates)."""
    import gzip
    import random
    seqload = os.path.join(ROOT, "fp-mash_amd", "bin", "seqload")
    rng = random.Random(5)
    text = b"".join(b">r%d c\n" % i + bytes(rng.choice(b"ACGTN") for _ in range(rng.randint(0, 3000)))
                    + b"\n" for i in range(400))
    cases = {
        "plain.fa": text,
        "one.fa.gz": gzip.compress(text),
        "multi.fa.gz": gzip.compress(text[:1000]) + gzip.compress(text[1000:5000]) +
                       gzip.compress(b"") + gzip.compress(text[5000:]),
        "bgzf.fa.gz": _bgzf(text, block=4000),
        "tail.fa.gz": gzip.compress(text) + b"not gzip trailing bytes",
    }
    for name, blob in cases.items():
        (tmp_path / name).write_bytes(blob)
        p = subprocess.run([seqload, str(tmp_path / name)], capture_output=True)
        assert p.returncode == 0, name
        assert p.stdout == text, name
    # a truncated member: gzread returns what inflates and then end of file (no error), so the
    # reference's kseq reads the partial text; libdeflate refuses it and the loader falls back
    import zlib
    cut = gzip.compress(text)[:-100]
    (tmp_path / "cut.fa.gz").write_bytes(cut)
    p = subprocess.run([seqload, str(tmp_path / "cut.fa.gz")], capture_output=True)
    assert p.returncode == 0 and p.stdout == zlib.decompressobj(16 + 15).decompress(cut)
    # a BGZF member whose ISIZE claims ~4 GB: the stream is not taken as BGZF (no output sized
    # from it), libdeflate and then gzread refuse the member, and the load fails cleanly
    import resource
    import struct
    blob = bytearray(_bgzf(text, block=4000))
    at = 0
    for _ in range(3):
        at += struct.unpack("<H", blob[at + 16:at + 18])[0] + 1
    bs = struct.unpack("<H", blob[at + 16:at + 18])[0] + 1
    blob[at + bs - 4:at + bs] = struct.pack("<I", 0xFFFFFFF0)
    (tmp_path / "isize.fa.gz").write_bytes(bytes(blob))
    p = subprocess.run([seqload, str(tmp_path / "isize.fa.gz")], capture_output=True)
    assert p.returncode in (0, 1) and text.startswith(p.stdout)
    assert resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss < 1 << 20    # KiB: < 1 GiB
