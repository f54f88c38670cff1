"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU suite).

The host C/C++ this repo ships or tests with -- the NTL-free key library
(mkfhe_amd/csrc/mkkeys.cpp: its worker threads, samplers and the key-file
reader that trusts nothing a file says), the CPU oracle (oracle/mkfhe_oracle.c)
and the reference-side adapter's packers (tests/cpp/adapter_pack.cpp, layout
mode) -- is rebuilt with -fsanitize=address,undefined and driven by the same
tests as the normal build.  GPU code is not sanitised here (no GPU ASan on this
pool); the engine library is loaded by the packer binary but not called.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

LIBASAN = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
pytestmark = pytest.mark.skipif(not os.path.isabs(LIBASAN) or not os.path.exists(LIBASAN),
                                reason="gcc has no libasan here")

SAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1:strict_string_checks=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


@pytest.fixture(scope="module")
def sanitized_libs():
    sys.path.insert(0, ROOT)
    from mkfhe_amd import build
    keys = build.build_keys(sanitize=True)
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    return keys, os.path.join(ROOT, "oracle", "build", "libmkfhe_oracle_asan.so")


def test_key_library_and_oracle_under_asan_ubsan(sanitized_libs):
    """Key generation (threads, samplers, Gauss-Jordan), encryption/decryption, the
    key files with every negative case (truncation, sizes past the end, bad
    parameter blocks), and the oracle's KAT, property and gate tests."""
    keys, orc = sanitized_libs
    env = dict(os.environ, LD_PRELOAD=LIBASAN, MKFHE_KEYS_LIB=keys, MKFHE_ORACLE_LIB=orc, MKFHE_ORACLE_THREADS="8",
               **SAN_ENV)
    tests = [os.path.join(ROOT, "tests", t) for t in
             ("test_keys.py", "test_key_defect.py", "test_oracle_kat.py", "test_oracle_props.py", "test_gate.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider", *tests],
                       capture_output=True, text=True, env=env, cwd=ROOT, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail
    assert " passed" in r.stdout, tail


def test_adapter_packers_under_asan_ubsan(sanitized_libs):
    """tests/cpp/adapter_pack.cpp (layout mode: every packed buffer against the
    C-ABI layout, every shape error through its error path) built with the
    sanitizers."""
    sys.path.insert(0, ROOT)
    from mkfhe_amd import _lib
    _, orc = sanitized_libs
    src = os.path.join(ROOT, "tests", "cpp", "adapter_pack.cpp")
    out = os.path.join(ROOT, "tests", "cpp", "build", "adapter_pack_asan")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    lib_dir = os.path.dirname(_lib.LIB_PATH)
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=undefined", "-Wall", "-Wextra", "-Werror", src, "-o", out,
                           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "integration"),
                           "-I", os.path.join(ROOT, "oracle"), "-L", lib_dir, "-lmkfhe_amd", f"-Wl,-rpath,{lib_dir}",
                           orc, f"-Wl,-rpath,{os.path.dirname(orc)}"])
    r = subprocess.run([out, "layout"], capture_output=True, text=True, timeout=300, env=dict(os.environ, **SAN_ENV))
    assert r.returncode == 0 and "layout: ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
    assert "runtime error:" not in r.stderr, r.stderr[-4000:]
