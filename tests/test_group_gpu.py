"""Multi-device groups through the C ABI (mkacc_group_*, include/mkfhe_amd.h):
a group of two contexts on device 0 (this box has one GPU; the code path --
member-0 key conversion, device-to-device key copies, sharded batches on
concurrent host threads -- is the one an 8-GPU node runs with devices 0..7)
must produce output bit-identical to a single context.  Reference entry point:
BinFHEContext::EvalBinGate (binfhecontext.cpp:415-426), SURVEY.md s8e."""
import os

import numpy as np
import pytest

from conftest import Q_MK, make_case

N = 2048


@pytest.mark.gpu
@pytest.mark.parametrize("meth,k,n,q,baseG,B", [("XZW", 2, 6, 45181, 1 << 7, 7), ("XZW_B", 4, 5, 32749, 1 << 9, 5)])
def test_group_evalacc_matches_single_context(oracle, meth, k, n, q, baseG, B):
    import mkfhe_amd as mk
    om = oracle.XZW if meth == "XZW" else oracle.XZW_B
    em = mk.MKNTRU if meth == "XZW" else mk.MKNTRU_LWE
    _, evk, pkey, ct, acc = make_case(oracle, om, k, n, q, baseG, B, seed=31 + k)
    params = mk.make_params(em, k, n, N, Q_MK, q, baseG)
    one = mk.MKAccumulatorEngine(params, 0)
    one.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    want = one.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    grp = mk.MKAccumulatorGroup(params, [0, 0, 0])
    assert grp.size == 3
    grp.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = grp.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert np.array_equal(got, want)
    # and against the oracle on the first gate
    orc = oracle.Oracle(om, k, n, N, Q_MK, q, baseG)
    exp = orc.evalacc_batch(evk, pkey, ct[:1], acc[:1], 1)
    assert np.array_equal(got[:1].astype(np.uint64), exp)


@pytest.mark.gpu
def test_group_wide_path_matches_single_context(oracle):
    """64-bit word path (config 5 stress modulus): keys copied in the wide layout."""
    import mkfhe_amd as mk
    Q = 1125899906826241
    k, n, q, baseG, B = 2, 3, 45181, 1 << 10, 5
    orc = oracle.Oracle(oracle.XZW, k, n, N, Q, q, baseG)
    evk = oracle.fill_uniform(int(np.prod(orc.evk_shape)), Q, 71).reshape(orc.evk_shape)
    pkey = oracle.fill_uniform(int(np.prod(orc.pkey_shape)), Q, 72).reshape(orc.pkey_shape)
    ct = oracle.fill_uniform(B * k * n, q, 73).reshape(B, k, n)
    acc = oracle.fill_uniform(B * k * N, Q, 74).reshape(B, k, N)
    params = mk.make_params(mk.MKNTRU, k, n, N, Q, q, baseG)
    one = mk.MKAccumulatorEngine(params, 0)
    one.upload_keys(evk, pkey)
    want = one.eval_batch(ct, acc)
    grp = mk.MKAccumulatorGroup(params, [0, 0])
    grp.upload_keys(evk, pkey)
    assert np.array_equal(grp.eval_batch(ct, acc), want)


@pytest.mark.gpu
@pytest.mark.parametrize("ps,method", [("STD100_MKNTRU", 0), ("STD100_MKNTRU_LWE", 2)])
def test_group_nand_gates_match_single_context(ps, method):
    """Full NAND gates with real keys: BinFHEContext(devices=[0, 0]) == BinFHEContext(device=0)."""
    from mkfhe_amd.binfhe import NAND, BinFHEContext
    ccs = []
    for dev in (0, [0, 0]):
        cc = BinFHEContext()
        cc.GenerateBinFHEContext(ps, method, dev)
        cc.SetSeed(808)
        sk = cc.MKLWE_KeyGen() if method == 2 else cc.MNTRU_KeyGen()
        cc.MKBTKeyGen(sk)
        if method == 0:
            cc.ctGateGen(sk, NAND)
        ccs.append((cc, sk))
    rng = np.random.default_rng(12)
    m1, m2 = rng.integers(0, 2, 96), rng.integers(0, 2, 96)
    outs = []
    for cc, sk in ccs:
        cc.SetSeed(909)   # identical ciphertexts in both contexts
        c1, c2 = cc.Encrypt(sk, m1), cc.Encrypt(sk, m2)
        out = cc.EvalBinGate(NAND, c1, c2)
        assert np.array_equal(cc.DecryptGate(sk, out), 1 - (m1 & m2)), f"seed 808/909 {ps}"
        outs.append(out)
    if method == 2:
        assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    else:
        assert np.array_equal(outs[0], outs[1])
