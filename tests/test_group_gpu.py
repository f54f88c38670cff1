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


def _device_count():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


@pytest.mark.gpu
@pytest.mark.skipif(_device_count() < 2, reason="needs two GPUs (the peer-copy path between distinct devices)")
def test_group_on_distinct_devices_matches_single_context(oracle):
    """Members on two distinct GPUs take the hipMemcpyPeerAsync path of the key
    sharing (ordered after member 0's stream).  Skipped on a one-GPU box: until an
    8-GPU node runs it, outputs of groups spanning devices are parity unpinned."""
    import mkfhe_amd as mk
    k, n, q, baseG, B = 2, 6, 45181, 1 << 7, 9
    _, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, k, n, q, baseG, B, seed=77)
    params = mk.make_params(mk.MKNTRU, k, n, N, Q_MK, q, baseG)
    one = mk.MKAccumulatorEngine(params, 0)
    one.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    want = one.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    grp = mk.MKAccumulatorGroup(params, [0, 1])
    grp.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    assert np.array_equal(grp.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32)), want)


@pytest.mark.gpu
def test_ksk_reupload_with_another_digit_count_resizes_the_gate_workspace(oracle):
    """a key-switching key re-uploaded with more digits (baseKS 32 -> 8,
    dks 4 -> 6) must reallocate the digit workspace sized for the old key.  The
    gates of the second key must equal those of a fresh context holding only it
    (any key words: both contexts compute the same function of the same key)."""
    import mkfhe_amd as mk
    k, n, q, baseG, B = 2, 8, 45181, 1 << 9, 6
    _, evk, pkey, _, _ = make_case(oracle, oracle.XZW, k, n, q, baseG, B, seed=91)
    params = mk.make_params(mk.MKNTRU, k, n, N, Q_MK, q, baseG)
    rng = np.random.default_rng(5)
    nand = rng.integers(0, q, (k, n), dtype=np.uint32)
    c1 = rng.integers(0, q, (B, k, n), dtype=np.uint32)
    c2 = rng.integers(0, q, (B, k, n), dtype=np.uint32)
    ksk = {}
    for base in (32, 8):
        dks = int(np.ceil(np.log(q) / np.log(base)))
        ksk[base] = rng.integers(0, q, (k, N * dks, n), dtype=np.uint32)
    reused = mk.MKAccumulatorEngine(params, 0)
    reused.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    reused.upload_ksk_mntru(ksk[32], q, 32, n)
    reused.eval_nand_mntru(nand, c1, c2)          # sizes the workspace for dks = 4
    reused.upload_ksk_mntru(ksk[8], q, 8, n)
    got = reused.eval_nand_mntru(nand, c1, c2)
    fresh = mk.MKAccumulatorEngine(params, 0)
    fresh.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    fresh.upload_ksk_mntru(ksk[8], q, 8, n)
    assert np.array_equal(got, fresh.eval_nand_mntru(nand, c1, c2))


@pytest.mark.gpu
def test_failed_ksk_upload_leaves_no_key_of_another_shape(oracle):
    """A key-switching upload that fails its range check must not leave the
    context claiming a key (the shape used to be committed first)."""
    import mkfhe_amd as mk
    k, n, q, baseG, B = 2, 8, 45181, 1 << 9, 3
    _, evk, pkey, _, _ = make_case(oracle, oracle.XZW, k, n, q, baseG, B, seed=92)
    params = mk.make_params(mk.MKNTRU, k, n, N, Q_MK, q, baseG)
    e = mk.MKAccumulatorEngine(params, 0)
    e.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    rng = np.random.default_rng(6)
    good = rng.integers(0, q, (k, N * 4, n), dtype=np.uint32)
    e.upload_ksk_mntru(good, q, 32, n)
    bad = rng.integers(0, q, (k, N * 6, n), dtype=np.uint32)
    bad[1, 7, 3] = q                               # not a canonical residue
    with pytest.raises(mk.MkaccError):
        e.upload_ksk_mntru(bad, q, 8, n)
    nand = rng.integers(0, q, (k, n), dtype=np.uint32)
    c = rng.integers(0, q, (B, k, n), dtype=np.uint32)
    # the old key (dks 4) is still the committed one: gates run with it
    fresh = mk.MKAccumulatorEngine(params, 0)
    fresh.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    fresh.upload_ksk_mntru(good, q, 32, n)
    assert np.array_equal(e.eval_nand_mntru(nand, c, c[::-1].copy()), fresh.eval_nand_mntru(nand, c, c[::-1].copy()))
