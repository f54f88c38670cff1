"""Boundary behaviour that needs no GPU: the MKNTRU_B gate is rejected before
any device work (the reference's MKNTRU_B gate is undefined behaviour:
binfhecontext.cpp:174 builds an MNTRU context, binfhe-base-scheme.cpp:1127
passes mod-q words to XZW_B, mk-acc-xzw_B.cpp:120,290 uses them as monomial
exponents up to q - 1 > 2N)."""
import numpy as np
import pytest

from mkfhe_amd.binfhe import MKNTRU, MKNTRU_B, NAND, BinFHEContext, ConfigError


def test_mkntru_b_gate_rejected_in_python_mirror():
    cc = BinFHEContext()
    cc.GenerateBinFHEContext("STD100_MKNTRU", MKNTRU_B)
    ct = np.zeros((2, 560), dtype=np.uint32)
    with pytest.raises(ConfigError, match="MKNTRU_B"):
        cc.EvalBinGate(NAND, ct, ct.copy())


def test_mkntru_gate_without_keys_is_config_error():
    cc = BinFHEContext()
    cc.GenerateBinFHEContext("STD100_MKNTRU", MKNTRU)
    ct = np.zeros((2, 560), dtype=np.uint32)
    with pytest.raises(ConfigError, match="MKBTKeyGen"):
        cc.EvalBinGate(NAND, ct, ct.copy())
