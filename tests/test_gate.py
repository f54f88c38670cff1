"""Gate head and tail around EvalAcc: the full
EvalBinGate(NAND) of MK-NTRU (binfhe-base-scheme.cpp:467-515) and MK-LWE
(:380-463) through the HIP engine, bit-exact against the CPU oracle.

CPU tests pin the oracle's new pieces by properties (RoundqQ vs Python's own
IEEE double evaluation, extraction = iNTT then X -> X^-1, KeySwitch2 with the
pre-multiplied table = digit x key contraction); GPU tests compare the engine.
Keys are seed-derived synthetic residues (the reference's key generation needs
NTL, which is absent): KSK2 is built exactly as KeySwitchGen2 stores it,
KSK2[u][j] = j * KSK[u] mod qKS (mntru-pke.cpp:744-755).
"""
import math

import numpy as np
import pytest

from conftest import Q_MK, make_case

N = 2048


def ksk2_from_ksk(ksk, baseKS, qKS):
    """KSK2[u][j][l][i] = j * KSK[u][l][i] mod qKS  ([k][N*dks][n] -> [k][Bks][N*dks][n])."""
    j = np.arange(baseKS, dtype=np.uint64).reshape(1, baseKS, 1, 1)
    return (ksk.astype(np.uint64)[:, None, :, :] * j) % qKS


# ---- CPU: oracle properties -------------------------------------------------------

def test_round_qQ_matches_python_double(oracle):
    rng = np.random.default_rng(1)
    for q, Q in [(45181, Q_MK), (32749, Q_MK), (4096, 32749), (4096, 45181)]:
        vs = list(rng.integers(0, Q, size=2000)) + [0, 1, Q - 1, Q // 2, Q // 2 + 1]
        for v in vs:
            exp = int(math.floor(0.5 + float(v) * float(q) / float(Q))) % q
            assert oracle.round_qQ(int(v), q, Q) == exp


def test_ks_digit_count(oracle):
    # SURVEY.md Appendix A "dks": 4 for MKNTRU (45181), 3 for MKNTRU_LWE (32749)
    assert oracle.ks_digits(45181, 32) == 4
    assert oracle.ks_digits(32749, 32) == 3


def test_extract_is_inverse_ntt_then_automorphism(oracle):
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 1, 45181, 1 << 9, 1, seed=3)
    a = acc[0]
    ext = orc.extract(a)
    psi = oracle.root_of_unity(4096, Q_MK)
    for u in range(2):
        coef = oracle.ntt_inverse(a[u], Q_MK, psi).astype(np.int64)
        expect = np.empty(N, dtype=np.int64)
        expect[0] = coef[0]
        expect[1:] = (-coef[1:][::-1]) % Q_MK        # b[N - j] = -a[j]
        assert np.array_equal(ext[u].astype(np.int64), expect)


def test_keyswitch2_table_equals_contraction(oracle):
    k, n, qKS, baseKS = 2, 7, 45181, 32
    dks = oracle.ks_digits(qKS, baseKS)
    rng = np.random.default_rng(5)
    ksk = rng.integers(0, qKS, size=(k, N * dks, n), dtype=np.uint64)
    ct = rng.integers(0, qKS, size=(k, N), dtype=np.uint64)
    got = oracle.keyswitch2(ksk2_from_ksk(ksk, baseKS, qKS), ct, k, N, n, qKS, baseKS)
    digits = np.stack([(ct // baseKS ** t) % baseKS for t in range(dks)], axis=-1).reshape(k, N * dks)
    exp = np.stack([(digits[u].astype(object) @ ksk[u].astype(object)) % qKS for u in range(k)]).astype(np.uint64)
    assert np.array_equal(got, exp)


# ---- GPU: engine parity --------------------------------------------------------------

def _mntru_setup(mk, oracle, k, n, baseG, B, seed):
    q = qKS = 45181
    baseKS = 32
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, k, n, q, baseG, B, seed=seed)
    dks = oracle.ks_digits(qKS, baseKS)
    ksk = oracle.fill_uniform(k * N * dks * n, qKS, seed * 7 + 1).reshape(k, N * dks, n)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, k, n, N, Q_MK, q, baseG))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    eng.upload_ksk_mntru(ksk.astype(np.uint32), qKS, baseKS, n)
    return orc, eng, evk, pkey, ksk2_from_ksk(ksk, baseKS, qKS), q, qKS, baseKS


@pytest.mark.gpu
def test_gate_tail_mntru(mk_gpu, oracle):
    mk = mk_gpu
    k, n, B = 2, 5, 3
    orc, eng, evk, pkey, ksk2, q, qKS, baseKS = _mntru_setup(mk, oracle, k, n, 1 << 7, B, seed=21)
    acc = oracle.fill_uniform(B * k * N, Q_MK, 99).reshape(B, k, N)
    acc[0, 0, :4] = [0, 1, Q_MK - 1, Q_MK // 2]
    got = eng.gate_tail(acc.astype(np.uint32))
    for b in range(B):
        exp = orc.mntru_tail(acc[b], ksk2, qKS, baseKS, n)
        assert np.array_equal(got[b], exp.astype(np.uint32)), b


# (k, n, log2 B_g, MKACC_LAT): config 4's shape (k = 8, dg = 4) and STD100_MKNTRU_3's
# (k = 8, dg = 2) through both the small-batch and the batch step kernel
@pytest.mark.gpu
@pytest.mark.parametrize("k,n,logB,lat", [(2, 4, 9, ""), (2, 3, 7, ""), (3, 2, 6, ""), (8, 2, 6, "1"), (8, 2, 6, "0"),
                                          (8, 2, 9, "1"), (8, 2, 9, "0"), (2, 3, 7, "q"), (8, 2, 6, "q"),
                                          (16, 2, 5, "q"), (2, 3, 7, "q1"), (8, 2, 6, "q1")])
def test_nand_gate_mntru(mk_gpu, oracle, k, n, logB, lat, monkeypatch):
    mk = mk_gpu
    if lat and lat[0] != "q":
        monkeypatch.setenv("MKACC_LAT", lat)
        monkeypatch.setenv("MKACC_QUAD", "0")   # B = 5 would take the quad kernels
    elif lat == "q1":
        monkeypatch.setenv("MKACC_QUAD", "1")   # one workgroup per gate (no party-parallel form)
    elif lat == "q":
        monkeypatch.delenv("MKACC_LAT", raising=False)   # default: party-parallel, B k <= CUs
    else:
        monkeypatch.setenv("MKACC_QUAD", "0")
    B = 5
    orc, eng, evk, pkey, ksk2, q, qKS, baseKS = _mntru_setup(mk, oracle, k, n, 1 << logB, B, seed=k * 10 + n)
    ct1 = oracle.fill_uniform(B * k * n, q, 31).reshape(B, k, n)
    ct2 = oracle.fill_uniform(B * k * n, q, 32).reshape(B, k, n)
    nand = oracle.fill_uniform(k * n, q, 33).reshape(k, n)
    ct1[0, 0, 0], ct2[0, 0, 0] = q - 1, q - 1                 # wrap in the head's sum
    got = eng.eval_nand_mntru(nand.astype(np.uint32), ct1.astype(np.uint32), ct2.astype(np.uint32))
    tv = orc.mntru_testvector(4)
    for b in range(B):
        ct = oracle.mntru_head(nand, ct1[b], ct2[b], q)
        acc = orc.evalacc(evk, pkey, ct, tv)                   # BootstrapGateCore (:1072-1130)
        exp = orc.mntru_tail(acc, ksk2, qKS, baseKS, n)
        assert np.array_equal(got[b], exp.astype(np.uint32)), b


def _mklwe_setup(mk, oracle, k, n, baseG, seed):
    q = qKS = 32749
    baseKS = 32
    orc, evk, pkey, _, _ = make_case(oracle, oracle.XZW_B, k, n, q, baseG, 1, seed=seed)
    dks = oracle.ks_digits(qKS, baseKS)
    A = oracle.fill_uniform(k * N * baseKS * dks * n, qKS, seed * 7 + 2).reshape(k, N, baseKS, dks, n)
    Bk = oracle.fill_uniform(k * N * baseKS * dks, qKS, seed * 7 + 3).reshape(k, N, baseKS, dks)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU_LWE, k, n, N, Q_MK, q, baseG))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    eng.upload_ksk_mklwe(A.astype(np.uint32), Bk.astype(np.uint32), qKS, baseKS, n)
    return orc, eng, evk, pkey, A, Bk, q, qKS, baseKS


@pytest.mark.gpu
def test_gate_tail_mklwe(mk_gpu, oracle):
    mk = mk_gpu
    k, n, B = 2, 5, 3
    orc, eng, evk, pkey, A, Bk, q, qKS, baseKS = _mklwe_setup(mk, oracle, k, n, 1 << 9, seed=41)
    acc = oracle.fill_uniform(B * k * N, Q_MK, 98).reshape(B, k, N)
    ga, gb = eng.gate_tail(acc.astype(np.uint32))
    for b in range(B):
        ea, eb = orc.mklwe_tail(acc[b], A, Bk, qKS, baseKS, n)
        assert np.array_equal(ga[b], ea.astype(np.uint32)) and int(gb[b]) == eb, b


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,quad", [(2, 4, "0"), (4, 2, "0"), (8, 2, "0"), (2, 4, "1"), (4, 2, "1"), (16, 2, "1"),
                                      (2, 4, "3"), (16, 2, "3")])
def test_nand_gate_mklwe(mk_gpu, oracle, k, n, quad, monkeypatch):
    mk = mk_gpu
    monkeypatch.setenv("MKACC_QUAD", quad)   # "1": mk_quad_kernel (B = 6 gates, one per workgroup); "3": party-parallel
    B = 6
    orc, eng, evk, pkey, A, Bk, q, qKS, baseKS = _mklwe_setup(mk, oracle, k, n, 1 << 9, seed=k * 10 + n + 50)
    a1 = oracle.fill_uniform(B * k * n, q, 61).reshape(B, k, n)
    a2 = oracle.fill_uniform(B * k * n, q, 62).reshape(B, k, n)
    b1 = oracle.fill_uniform(B, q, 63)
    b2 = oracle.fill_uniform(B, q, 64)
    a1[0, 0, :2] = 0
    a2[0, 0, :2] = [0, q - 1]
    got_a, got_b = eng.eval_nand_mklwe(a1, b1, a2, b2)
    for b in range(B):
        c, acc0 = orc.mklwe_head(a1[b], b1[b], a2[b], b2[b], q)
        acc = orc.evalacc(evk, pkey, c, acc0)                  # BootstrapGateCore (:1004-1067)
        ea, eb = orc.mklwe_tail(acc, A, Bk, qKS, baseKS, n)
        assert np.array_equal(got_a[b], ea.astype(np.uint32)) and int(got_b[b]) == eb, b


@pytest.mark.gpu
def test_gate_errors(mk_gpu, oracle):
    mk = mk_gpu
    k, n = 2, 3
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, k, n, 45181, 1 << 9, 1, seed=1)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, k, n, N, Q_MK, 45181, 1 << 9))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    c1 = np.zeros((1, k, n), np.uint32)
    c2 = np.ones((1, k, n), np.uint32)
    with pytest.raises(mk.MkaccError) as e:                 # KSK missing
        eng.gate_tail(np.zeros((1, k, N), np.uint32))
    assert e.value.code == -3
    with pytest.raises(mk.MkaccError):                      # LWE key on an MNTRU context
        eng.upload_ksk_mklwe(np.zeros(1, np.uint32), np.zeros(1, np.uint32), 45181, 32, n)
    ksk = np.zeros((k, N * 4, n), np.uint32)
    eng.upload_ksk_mntru(ksk, 45181, 32, n)
    with pytest.raises(mk.MkaccError) as e:                 # ct word >= q
        eng.eval_nand_mntru(np.zeros((k, n), np.uint32), c1 + 45181, c2)
    assert e.value.code == -5


# Whole gates at the batch size bench.py times: B = 4100 gates run as slices of the
# batch step kernel (units of CUs x 4 = 1024 gates at 256 CUs) on 2 or 4 streams,
# checked on both sides of every unit boundary.  MK-NTRU k = 2 (headline kernel,
# dg = 3), MK-LWE k = 4 (config 3's XZW_B step2 kernel) and MK-NTRU k = 8 at dg = 4
# (config 4's mk_step_kernel with the d_i scratch); short n keeps the oracle fast.
BIG_GATES = [("mntru", 2, 3, 7, "2"), ("mntru", 2, 3, 7, "4"), ("mklwe", 4, 2, 9, "2"), ("mklwe", 4, 2, 9, "3"),
             ("mntru", 8, 2, 6, "2")]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,k,n,logB,streams", BIG_GATES,
                         ids=[f"{c[0]}-k{c[1]}-logB{c[3]}-s{c[4]}" for c in BIG_GATES])
def test_nand_gate_big_batch_slices(mk_gpu, oracle, kind, k, n, logB, streams, monkeypatch):
    mk = mk_gpu
    monkeypatch.setenv("MKACC_STREAMS", streams)
    B, baseKS = 4100, 32
    pick = [0, 1, 1023, 1024, 2047, 2048, 2049, 3071, 3072, 4099]
    seed = 500 + 10 * k + logB
    if kind == "mntru":
        q = qKS = 45181
        orc, evk, pkey, _, _ = make_case(oracle, oracle.XZW, k, n, q, 1 << logB, 1, seed=seed)
        dks = oracle.ks_digits(qKS, baseKS)
        ksk = oracle.fill_uniform(k * N * dks * n, qKS, seed * 7 + 1).reshape(k, N * dks, n)
        eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, k, n, N, Q_MK, q, 1 << logB))
        assert eng.step_kernel_name(B) == ("mk_step2_kernel" if logB > 6 else "mk_step_kernel")
        eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
        eng.upload_ksk_mntru(ksk.astype(np.uint32), qKS, baseKS, n)
        ct1 = oracle.fill_uniform(B * k * n, q, seed + 1).reshape(B, k, n)
        ct2 = oracle.fill_uniform(B * k * n, q, seed + 2).reshape(B, k, n)
        nand = oracle.fill_uniform(k * n, q, seed + 3).reshape(k, n)
        ct1[1024, 0, 0], ct2[1024, 0, 0] = q - 1, q - 1
        got = eng.eval_nand_mntru(nand.astype(np.uint32), ct1.astype(np.uint32), ct2.astype(np.uint32))
        assert got.shape == (B, k, n)
        heads = np.stack([oracle.mntru_head(nand, ct1[b], ct2[b], q) for b in pick])
        acc0 = np.broadcast_to(orc.mntru_testvector(4), (len(pick), k, N)).copy()
        acc = orc.evalacc_batch(evk, pkey, heads, acc0, 8)                 # BootstrapGateCore (:1072-1130)
        for j, b in enumerate(pick):
            exp = orc.mntru_tail_ksk1(acc[j], ksk, qKS, baseKS, n)
            assert np.array_equal(got[b], exp.astype(np.uint32)), b
    else:
        q = qKS = 32749
        orc, evk, pkey, _, _ = make_case(oracle, oracle.XZW_B, k, n, q, 1 << logB, 1, seed=seed)
        dks = oracle.ks_digits(qKS, baseKS)
        A = oracle.fill_uniform(k * N * baseKS * dks * n, qKS, seed * 7 + 2).reshape(k, N, baseKS, dks, n)
        Bk = oracle.fill_uniform(k * N * baseKS * dks, qKS, seed * 7 + 3).reshape(k, N, baseKS, dks)
        eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU_LWE, k, n, N, Q_MK, q, 1 << logB))
        assert eng.step_kernel_name(B) == "mk_step2_kernel"
        eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
        eng.upload_ksk_mklwe(A.astype(np.uint32), Bk.astype(np.uint32), qKS, baseKS, n)
        a1 = oracle.fill_uniform(B * k * n, q, seed + 1).reshape(B, k, n)
        a2 = oracle.fill_uniform(B * k * n, q, seed + 2).reshape(B, k, n)
        b1 = oracle.fill_uniform(B, q, seed + 3)
        b2 = oracle.fill_uniform(B, q, seed + 4)
        a1[2048, 0, :2] = 0
        a2[2048, 0, :2] = [0, q - 1]
        got_a, got_b = eng.eval_nand_mklwe(a1, b1, a2, b2)
        assert got_a.shape == (B, k, n) and got_b.shape == (B,)
        heads = [orc.mklwe_head(a1[b], b1[b], a2[b], b2[b], q) for b in pick]
        acc = orc.evalacc_batch(evk, pkey, np.stack([h[0] for h in heads]), np.stack([h[1] for h in heads]), 8)
        for j, b in enumerate(pick):
            ea, eb = orc.mklwe_tail(acc[j], A, Bk, qKS, baseKS, n)            # (:1004-1067), mklwe-pke.cpp:260-298
            assert np.array_equal(got_a[b], ea.astype(np.uint32)) and int(got_b[b]) == eb, b
