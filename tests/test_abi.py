"""CPU tests of the C ABI boundary: the library loads without a GPU, exports every
symbol include/fpmash.h declares, the binding's signature table matches, and
compute entry points fail loudly (FPM_ENODEV) instead of falling back to the CPU."""
import os
import re

import pytest

from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "fpmash.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fpm_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    import fpmash
    L = fpmash.lib()
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), f"{n} declared in fpmash.h but not exported"


def test_binding_covers_header():
    import fpmash
    bound = {n for n, _, _ in fpmash.SYMBOLS}
    assert bound == set(header_functions())


def test_no_device_fails_loudly():
    import fpmash
    if fpmash.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(fpmash.FpmError) as e:
        fpmash.Context(0)
    assert e.value.code == fpmash.FPM_ENODEV
    assert fpmash.lib().fpm_abi_version() == 1


def test_library_is_gfx950_code_object():
    import subprocess
    import fpmash
    import shutil
    import tempfile
    # --offloading extracts the code objects next to its input: run it on a copy in a
    # scratch directory (not beside the in-tree library, which travels to the GPU box)
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, "libfpmash.so")
        shutil.copy(fpmash.LIB_PATH, lib)
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib],
                             capture_output=True, text=True, cwd=d)
    if out.returncode != 0:
        pytest.skip("llvm-objdump unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_params_match_oracle(oracle):
    import fpmash
    for kw in [dict(k=21), dict(k=16), dict(k=17), dict(k=9, alphabet="ACDEFGHIKLMNPQRSTVWY")]:
        P = fpmash.make_params(**kw)
        O = oracle.params(**kw)
        assert P.use64 == O.use64
        assert bytes(P.alphabet) == bytes(O.alphabet)
    F = fpmash.make_params(fingerprint=True)
    assert (F.kmer_size, F.noncanonical, F.use64) == (1, 1, 0)
