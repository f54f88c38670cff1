"""The reference-side adapter (integration/mk-acc-amd.h) compiles against the
reference's own headers.

The adapter replaces the reference's accumulator plugin seam
(`UniEncAccumulator`, /root/reference/src/binfhe/include/mk-acc.h:55-80) and is
registered in `BinFHEScheme(BINFHE_METHOD)` (binfhe-base-scheme.h:137-151).  It
must forward both `KeyGenAcc` overloads to a held reference accumulator
(UniEncAccumulatorXZW / _B are `final`, mk-acc-xzw.h:56, mk-acc-xzw_B.h:55), since
`BinFHEScheme::MKKeyGen` calls them through the same pointer
(binfhe-base-scheme.cpp:272, :334).

The reference headers include the generated `config_core.h`; it is produced by
a configure-only CMake run into a scratch directory under /tmp (nothing is
built, nothing lands in the repo).  `g++ -fsyntax-only` then checks
integration/check_adapter.cpp (which reaches every adapter member through the
seam) with -Wall -Wextra -Werror on our code, at NATIVE_SIZE=32 and 64.
Skipped where /root/reference is absent (the GPU box).
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(
    not os.path.isdir(os.path.join(REF, "src/binfhe/include")) or shutil.which("cmake") is None
    or shutil.which("g++") is None,
    reason="reference tree, cmake or g++ not available")


def _config_dir(native_size):
    """Configure-only CMake run of the reference into /tmp; returns the dir holding config_core.h."""
    out = os.path.join(tempfile.gettempdir(), f"mkfhe_refcfg{native_size}")
    hdr = os.path.join(out, "src/core/config_core.h")
    if not os.path.exists(hdr):
        cmd = ["cmake", REF, "-B", out, "-DGIT_SUBMOD_AUTO=OFF", f"-DNATIVE_SIZE={native_size}",
               "-DWITH_OPENMP=OFF", "-DBUILD_UNITTESTS=OFF", "-DBUILD_EXAMPLES=OFF",
               "-DBUILD_BENCHMARKS=OFF", "-DCMAKE_BUILD_TYPE=Release",
               "-DCMAKE_POLICY_VERSION_MINIMUM=3.5"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and os.path.exists(hdr), r.stdout[-2000:] + r.stderr[-2000:]
    with open(hdr) as f:
        assert re.search(rf"#define NATIVEINT {native_size}\b", f.read())
    return os.path.join(out, "src/core")


def _syntax_check(native_size, source):
    cfg = _config_dir(native_size)
    inc = []
    for d in ("src/core/include", "src/core/lib", None, "third-party/cereal/include", "src/binfhe/include"):
        inc += ["-isystem", cfg if d is None else os.path.join(REF, d)]
    cmd = ["g++", "-std=gnu++17", "-fsyntax-only", "-pthread", "-DOPENFHE_VERSION=1.1.1",
           "-Wall", "-Wextra", "-Werror", *inc,
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "integration"), source]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("native_size", [32, 64])
def test_adapter_compiles_against_reference_headers(native_size):
    r = _syntax_check(native_size, os.path.join(ROOT, "integration", "check_adapter.cpp"))
    assert r.returncode == 0, r.stderr[-4000:]


def test_adapter_forwards_both_keygen_overloads():
    """Both KeyGenAcc overloads are overridden in the adapter and forwarded to the held
    reference accumulator (the base-class versions throw not_implemented_error)."""
    with open(os.path.join(ROOT, "integration", "mk-acc-amd.h")) as f:
        src = f.read()
    body = src[src.index("class UniEncAccumulatorAMD"):]
    for key in ("ConstMNTRUPrivateKey", "ConstMKLWEPrivateKey"):
        m = re.search(r"UniEncACCKey KeyGenAcc\([^)]*" + key + r"[^)]*\)\s*const override\s*\{\s*"
                      r"return m_cpu->KeyGenAcc\(", body, re.S)
        assert m, f"KeyGenAcc({key}) is not forwarded to the reference accumulator"
    assert "std::make_shared<UniEncAccumulatorXZW>()" in body
    assert "std::make_shared<UniEncAccumulatorXZW_B>()" in body


def test_a_broken_adapter_fails_the_check(tmp_path):
    """The check has teeth: a signature that drifts from the reference's seam fails to compile."""
    with open(os.path.join(ROOT, "integration", "mk-acc-amd.h")) as f:
        src = f.read()
    # EvalAcc with Pkey by const reference no longer overrides the reference's virtual
    bad = src.replace("std::vector<std::vector<NativePoly>> Pkey, std::vector<NativePoly> /*skf*/",
                      "const std::vector<std::vector<NativePoly>>& Pkey, std::vector<NativePoly> /*skf*/", 1)
    assert bad != src
    (tmp_path / "mk-acc-amd.h").write_text(bad)
    tu = tmp_path / "check.cpp"
    tu.write_text('#include "mk-acc-amd.h"\nint main() { return 0; }\n')
    cfg = _config_dir(32)
    inc = []
    for d in ("src/core/include", "src/core/lib", None, "third-party/cereal/include", "src/binfhe/include"):
        inc += ["-isystem", cfg if d is None else os.path.join(REF, d)]
    r = subprocess.run(["g++", "-std=gnu++17", "-fsyntax-only", "-pthread", "-Wall", "-Werror", *inc,
                        "-I", str(tmp_path), "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "integration"),
                        str(tu)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "override" in r.stderr

