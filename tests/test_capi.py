"""C ABI checks that need no GPU: the library loads, exports every symbol the
header declares, and its host-side parameter logic matches the reference."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, gpu_available

HEADER = os.path.join(ROOT, "include", "mkfhe_amd.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mkacc_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from mkfhe_amd import _lib
    return _lib.load()


def test_library_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lib, n), n


def test_python_binding_covers_header():
    from mkfhe_amd import _lib
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_abi_version(lib):
    assert lib.mkacc_abi_version() == 2


@pytest.mark.parametrize("name,k,n,q,logB,dg", [
    ("STD128_MKNTRU", 2, 765, 45181, 7, 3),
    ("STD128_MKNTRU_3", 8, 765, 45181, 6, 4),
    ("STD128_MKNTRU_4", 16, 765, 45181, 5, 5),
    ("STD100_MKNTRU", 2, 560, 45181, 9, 2),
    ("STD100_MKNTRU_LWE", 2, 500, 32749, 9, 2),
    ("STD100_MKNTRU_LWE_2", 4, 500, 32749, 9, 2),
    ("STD128_MKNTRU_LWE_4", 16, 635, 32749, 7, 3),
])
def test_paramset_table(name, k, n, q, logB, dg, oracle):
    import mkfhe_amd as mk
    p = mk.paramset(name)
    assert (p.k, p.n, p.N, p.q, p.baseG) == (k, n, 2048, q, 1 << logB)
    assert p.Q == 134176769 and p.root == 100530
    assert p.digitsG - 1 == dg == oracle.digits_g(p.Q, p.baseG) - 1
    assert p.method == (mk.MKNTRU_LWE if "_LWE" in name else mk.MKNTRU)


def test_paramset_unknown():
    import mkfhe_amd as mk
    with pytest.raises(mk.MkaccError) as e:
        mk.paramset("STD128")          # single-key set: no MK path
    assert e.value.code == -1


def test_create_rejects_bad_params():
    import mkfhe_amd as mk
    from mkfhe_amd import _lib
    L = _lib.load()
    h = ctypes.c_void_p()
    bad = [
        mk.make_params(mk.MKNTRU, 2, 10, 1024, 134176769, 45181, 1 << 9),   # N != 2048
        mk.make_params(mk.MKNTRU, 2, 10, 2048, 134176769, 45181, 100),      # baseG not a power of 2
        mk.make_params(7, 2, 10, 2048, 134176769, 45181, 1 << 9),           # method invalid
        mk.make_params(mk.MKNTRU, 2, 10, 2048, 134176771, 45181, 1 << 9),   # Q not prime
        mk.make_params(mk.MKNTRU, 2, 10, 2048, (1 << 40) + 1, 45181, 1 << 9),  # Q too wide
    ]
    for p in bad:
        rc = L.mkacc_create(ctypes.byref(p), 0, ctypes.byref(h))
        assert rc in (-1, -2), (p.as_dict(), rc)
        assert _lib.last_error()


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU error path")
def test_create_without_gpu_fails_loudly():
    import mkfhe_amd as mk
    with pytest.raises(mk.MkaccError) as e:
        mk.MKAccumulatorEngine(mk.paramset("STD100_MKNTRU"))
    assert e.value.code == -4
