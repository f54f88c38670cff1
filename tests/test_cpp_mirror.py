"""Builds and runs the C++ host-mirror tests (tests/cpp/test_binfhe_mirror.cpp)
against libmkfhe_amd.so, linking the CPU oracle as the checker."""
import os
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "cpp", "test_binfhe_mirror.cpp")
OUT = os.path.join(ROOT, "tests", "cpp", "build", "test_binfhe_mirror")


@pytest.fixture(scope="module")
def binary(oracle):
    from mkfhe_amd import _lib
    lib_dir = os.path.dirname(_lib.LIB_PATH)
    orc_dir = os.path.join(ROOT, "oracle", "build")
    from mkfhe_amd import build
    build.build_keys()
    deps = [SRC, os.path.join(ROOT, "include", "mkfhe_amd_binfhe.hpp"), _lib.LIB_PATH, build.KEYS_OUT]
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.check_call([
            "g++", "-std=c++17", "-O2", "-Wall", "-Wextra", SRC, "-o", OUT,
            "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
            "-L", lib_dir, "-lmkfhe_amd", "-lmkfhe_keys", f"-Wl,-rpath,{lib_dir}",
            "-L", orc_dir, "-lmkfhe_oracle", f"-Wl,-rpath,{orc_dir}"])
    return OUT


def test_cpp_mirror_host(binary):
    r = subprocess.run([binary, "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_mirror_gpu_parity(binary):
    r = subprocess.run([binary, "gpu"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
