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


def run(args, cwd=None, check=True):
    p = subprocess.run([FPMASH] + args, cwd=cwd, capture_output=True)
    if check and p.returncode != 0:
        raise AssertionError(f"fpmash {args} failed: {p.stderr.decode()}")
    return p


@pytest.mark.parametrize("name", REF_MSH)
def test_msh_writer_byte_identical_roundtrip(name):
    p = subprocess.run([ROUNDTRIP, os.path.join(GOLDEN, name)], capture_output=True, text=True)
    assert p.returncode == 0 and p.stdout.startswith("same"), p.stdout + p.stderr


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


def test_cli_fails_loudly_without_device():
    import fpmash
    if fpmash.device_count() > 0:
        pytest.skip("device present")
    p = run(["sketch", "-fp", os.path.join(GOLDEN, "DNA1-CFL.txt"), "-o", "/tmp/fpm_nodev"],
            check=False)
    assert p.returncode != 0 and b"no CPU fallback" in p.stderr


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
