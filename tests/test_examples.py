"""The reference's two example programs, written against the C++ mirror
(examples/boolean-mkntru.cpp, examples/boolean-mklwe.cpp): built here, run on
the MI355X, every NAND of the truth table must decrypt correctly."""
import os
import subprocess

import pytest

from conftest import ROOT

EXAMPLES = ["boolean-mkntru", "boolean-mklwe"]
BUILD = os.path.join(ROOT, "tests", "cpp", "build")


def _build(name):
    from mkfhe_amd import build
    build.build_keys()
    lib_dir = os.path.join(ROOT, "mkfhe_amd", "lib")
    src = os.path.join(ROOT, "examples", name + ".cpp")
    out = os.path.join(BUILD, name)
    deps = [src, os.path.join(ROOT, "include", "mkfhe_amd_binfhe.hpp"), os.path.join(lib_dir, "libmkfhe_amd.so"),
            build.KEYS_OUT]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(BUILD, exist_ok=True)
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
                               src, "-o", out, "-L", lib_dir, "-lmkfhe_amd", "-lmkfhe_keys",
                               f"-Wl,-rpath,{lib_dir}"])
    return out


@pytest.mark.parametrize("name", EXAMPLES)
def test_example_builds(name):
    assert os.path.exists(_build(name))


@pytest.mark.gpu
@pytest.mark.parametrize("name,ps", [("boolean-mkntru", "STD100_MKNTRU"), ("boolean-mkntru", "STD128_MKNTRU"),
                                     ("boolean-mklwe", "STD100_MKNTRU_LWE")])
def test_example_runs(name, ps):
    r = subprocess.run([_build(name), ps], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    if r.returncode != 0 and "drew a nonzero DggR sample" in r.stdout:
        # the reference's key-generation defect (mk-acc-xzw.cpp:160-167), reproduced bit-faithfully
        # and reported by the example: fresh keys of this run are defective (a few per thousand
        # key sets), not the engine.  The truth table is then checked on resampled keys.
        r = subprocess.run([_build(name), ps, "--resample"], capture_output=True, text=True, timeout=300)
        print(r.stdout)
        assert "drew a nonzero DggR sample" not in r.stdout
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Result of encrypted computation") == 4
