"""Host check of the exact FP64 modular product of the 64-bit word path's FP64
kernels (mkfhe_amd/csrc/mkacc_fp64.hpp): tools/fp64_modmul_check.c compares
mm(a, b) = fma(-q, Q, h) + l with the __int128 value a*b - q*Q over random and
corner operands at the operand bounds the kernels rely on (|a b| <= 4 Q^2),
at the config-5 modulus and near 2^50 (CPU, IEEE binary64 as on the GPU)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_fp64_modmul_exact(tmp_path):
    exe = os.path.join(tmp_path, "fp64chk")
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                           os.path.join(ROOT, "tools", "fp64_modmul_check.c"), "-lm"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "FAIL" not in r.stdout and r.stdout.count("exact") == 15
