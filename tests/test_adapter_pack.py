"""The reference-side adapter's conversions, executed.

integration/mk-acc-amd.h (compiled against the reference's headers by
tests/test_integration_adapter.py) converts the reference's key, ciphertext
and accumulator objects to the engine's C-ABI buffers with the templates of
integration/mk-acc-amd-pack.h.  The reference cannot be linked here (NTL is
absent), so tests/cpp/adapter_pack.cpp instantiates the same templates with
stand-in types that offer the reference's accessors and runs them: on the CPU
every packed buffer is compared with the C-ABI layout index by index and every
shape error reaches the error path; on an MI355X reference-shaped keys,
ciphertexts and accumulators go through them into the engine (EvalAcc for XZW
and XZW_B, whole MK-NTRU and MK-LWE NAND gates) and come out equal to the CPU
oracle.  Needs no reference tree, so it also runs on the GPU box.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

PACK_SRC = os.path.join(ROOT, "tests", "cpp", "adapter_pack.cpp")
PACK_OUT = os.path.join(ROOT, "tests", "cpp", "build", "adapter_pack")


def _pack_binary():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from mkfhe_amd import _lib
    pyoracle.build()
    lib_dir = os.path.dirname(_lib.LIB_PATH)
    orc_dir = os.path.join(ROOT, "oracle", "build")
    deps = [PACK_SRC, os.path.join(ROOT, "integration", "mk-acc-amd-pack.h"), os.path.join(ROOT, "include", "mkfhe_amd.h"),
            _lib.LIB_PATH]
    if not os.path.exists(PACK_OUT) or os.path.getmtime(PACK_OUT) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(PACK_OUT), exist_ok=True)
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", PACK_SRC, "-o", PACK_OUT,
                               "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "integration"),
                               "-I", os.path.join(ROOT, "oracle"), "-L", lib_dir, "-lmkfhe_amd",
                               f"-Wl,-rpath,{lib_dir}", "-L", orc_dir, "-lmkfhe_oracle", f"-Wl,-rpath,{orc_dir}"])
    return PACK_OUT


def test_adapter_packers_follow_the_c_abi_layout():
    r = subprocess.run([_pack_binary(), "layout"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "layout: ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_adapter_packers_drive_the_engine_to_the_oracle():
    r = subprocess.run([_pack_binary(), "engine"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0 and "engine: ok" in r.stdout, r.stdout + r.stderr
