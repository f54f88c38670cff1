"""The 64-bit word path (mkfhe_amd/csrc/mkacc_wide.hpp): EvalAcc for
2^27 <= Q < 2^61, i.e. the reference at NATIVE_SIZE=64 with a wide modulus
(SURVEY.md s8 config 5 stress: Q = 1125899906826241, B_g = 2^10, dg = 4).
Bit-exact against the CPU oracle, whose 64-bit arithmetic is u128-exact.
"""
import os

import numpy as np
import pytest

from conftest import Q_MK, make_case

N = 2048
Q50 = 1125899906826241          # SURVEY.md s0 item 2 / s6 ("cfg5 stress")
PSI50 = 1080667890455           # its minimal primitive 4096-th root, printed by the reference probe


def test_oracle_wide_constants(oracle):
    """Pins the oracle's number theory at 50 bits on the reference's own output."""
    assert oracle.is_prime(Q50) and (Q50 - 1) % (2 * N) == 0 and Q50 < (1 << 50)
    assert oracle.root_of_unity(2 * N, Q50) == PSI50
    assert oracle.digits_g(Q50, 1 << 10) == 5


def test_oracle_wide_ntt_roundtrip(oracle):
    a = oracle.fill_uniform(N, Q50, 9)
    e = oracle.ntt_forward(a, Q50, PSI50)
    assert np.array_equal(oracle.ntt_inverse(e, Q50, PSI50), a)
    # negacyclic product of X and X^(N-1) is -1
    x = np.zeros(N, np.uint64); x[1] = 1
    y = np.zeros(N, np.uint64); y[N - 1] = 1
    prod = (oracle.ntt_forward(x, Q50, PSI50).astype(object) * oracle.ntt_forward(y, Q50, PSI50).astype(object)) % Q50
    z = oracle.ntt_inverse(np.array(prod, dtype=np.uint64), Q50, PSI50)
    assert z[0] == Q50 - 1 and not z[1:].any()


def _eng(mk, method, k, n, Q, q, baseG):
    return mk.MKAccumulatorEngine(mk.make_params(method, k, n, N, Q, q, baseG))


@pytest.mark.gpu
def test_wide_context_and_primitives(mk_gpu, oracle):
    mk = mk_gpu
    eng = _eng(mk, mk.MKNTRU, 2, 4, Q50, 45181, 1 << 10)
    assert eng.wide and eng.dg == 4 and eng.params.root == PSI50
    a = oracle.fill_uniform(3 * N, Q50, 21).reshape(3, N)
    f = eng.ntt_forward(a)
    assert f.dtype == np.uint64
    assert np.array_equal(f, np.stack([oracle.ntt_forward(x, Q50, PSI50) for x in a]))
    assert np.array_equal(eng.ntt_inverse(f), a)
    d = eng.sdd(a)
    assert np.array_equal(d, np.stack([oracle.sdd(x, Q50, 1 << 10, 4) for x in a]))
    # the gate API is the 27-bit kernel's
    with pytest.raises(mk.MkaccError) as e:
        eng.upload_ksk_mntru(np.zeros((2, N * 4, 4), np.uint32), 45181, 32, 4)
    assert e.value.code == -2


@pytest.mark.gpu
@pytest.mark.parametrize("method,k,n,baseG,B", [
    ("XZW", 2, 5, 1 << 10, 3),     # config 5 stress shape (dg = 4)
    ("XZW", 3, 3, 1 << 17, 2),     # dg = 2, three parties
    ("XZW_B", 2, 4, 1 << 10, 3),
    ("XZW_B", 1, 4, 1 << 13, 2),   # dg = 3, one party
])
def test_wide_evalacc_bitexact(mk_gpu, oracle, method, k, n, baseG, B):
    mk = mk_gpu
    m = oracle.XZW if method == "XZW" else oracle.XZW_B
    orc, evk, pkey, ct, acc = make_case(oracle, m, k, n, 45181, baseG, B, seed=k * 7 + n, Q=Q50)
    exp = orc.evalacc(evk, pkey, ct, acc)
    eng = _eng(mk, mk.MKNTRU if method == "XZW" else mk.MKNTRU_LWE, k, n, Q50, 45181, baseG)
    assert eng.wide
    eng.upload_keys(evk.astype(np.uint64), pkey.astype(np.uint64))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint64))
    assert got.dtype == np.uint64
    assert np.array_equal(got, exp), int(np.count_nonzero(got != exp))


# variant -> (MKACC_WIDE_FP, step kernel)
VARIANTS = {"fp64": ("1", "widereg2::step_kernel"), "int": ("0", "wide::step_kernel")}


@pytest.mark.gpu
@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("method", ["XZW", "XZW_B"])
def test_wide_fp64_and_integer_variants(mk_gpu, oracle, monkeypatch, method, variant):
    """Q < 2^50 runs the register-resident FP64 kernel with two waves per gate
    (mkacc_widereg2.hpp) unless MKACC_WIDE_FP=0 selects the integer kernels
    (mkacc_wide.hpp, the path above 2^50): both bit-exact.  The first step's digit
    decomposition sees chosen coefficients (acc = NTT(coefficients)): 0, 1,
    Q-1 and the centring boundary Q>>1, (Q>>1)+1 where the FP64 path picks the
    reference's representative explicitly; keys include all-maximal and
    balanced-boundary words.  (The device-pointer key upload of this path is
    exercised by every bench.py --q-bits 50 run, whose oracle check covers it.)"""
    mk = mk_gpu
    fp, kname = VARIANTS[variant]
    monkeypatch.setenv("MKACC_WIDE_FP", fp)
    m = oracle.XZW if method == "XZW" else oracle.XZW_B
    k, n, B = 2, 3, 3
    orc, evk, pkey, ct, acc = make_case(oracle, m, k, n, 45181, 1 << 10, B, seed=50 + len(method), Q=Q50)
    h = Q50 >> 1
    edge = np.array([0, 1, Q50 - 1, h, h + 1, h - 1, 2, Q50 - 2], dtype=np.uint64)
    coef = oracle.fill_uniform(N, Q50, 77)
    coef[:8] = edge
    coef[-8:] = edge
    acc[0, 0] = oracle.ntt_forward(coef, Q50, PSI50)
    acc[1, 1] = oracle.ntt_forward(np.full(N, h, np.uint64), Q50, PSI50)
    evk.reshape(-1)[:4] = [Q50 - 1, h, h + 1, 0]
    pkey.reshape(-1)[:4] = [Q50 - 1, h, h + 1, 0]
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 4)
    eng = _eng(mk, mk.MKNTRU if method == "XZW" else mk.MKNTRU_LWE, k, n, Q50, 45181, 1 << 10)
    assert eng.wide and eng.step_kernel_name(B) == kname
    eng.upload_keys(evk.astype(np.uint64), pkey.astype(np.uint64))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint64))
    assert np.array_equal(got, exp), int(np.count_nonzero(got != exp))
    # primitives at the same modulus
    a = np.stack([coef, oracle.fill_uniform(N, Q50, 78)])
    f = eng.ntt_forward(a)
    assert np.array_equal(f, np.stack([oracle.ntt_forward(x, Q50, PSI50) for x in a]))
    assert np.array_equal(eng.ntt_inverse(f), a)


@pytest.mark.gpu
@pytest.mark.parametrize("streams", ["2", "3"])
@pytest.mark.parametrize("method", ["XZW", "XZW_B"])
def test_wide_register_kernel_loops_and_slices(mk_gpu, oracle, monkeypatch, method, streams):
    """The FP64 kernel's four 2-wave workgroups per CU loop over their slice of
    the batch, and a batch of two or more units of CUs x 4 gates is cut into
    MKACC_STREAMS slices on streams of their own (wide_launch_batch).  B = 4101
    (not a multiple of four): the sliced run equals the one-stream run word for
    word, a spread sample across the slice boundaries equals the oracle, and the
    last gates equal a separate small batch."""
    mk = mk_gpu
    m = oracle.XZW if method == "XZW" else oracle.XZW_B
    k, n, B = 2, 2, 4101
    orc, evk, pkey, ct, acc = make_case(oracle, m, k, n, 45181, 1 << 10, B, seed=61 + len(method), Q=Q50)
    outs = {}
    for ns in ("1", streams):
        monkeypatch.setenv("MKACC_STREAMS", ns)
        eng = _eng(mk, mk.MKNTRU if method == "XZW" else mk.MKNTRU_LWE, k, n, Q50, 45181, 1 << 10)
        assert eng.step_kernel_name(B) == "widereg2::step_kernel"
        eng.upload_keys(evk.astype(np.uint64), pkey.astype(np.uint64))
        outs[ns] = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint64))
    got = outs[streams]
    assert np.array_equal(outs["1"], got)
    pick = [0, 1, 2, 3, 1023, 1024, 2047, 2048, 3071, 3072, 4100]
    exp = orc.evalacc_batch(evk, pkey, ct[pick], acc[pick], 8)
    assert np.array_equal(got[pick], exp)
    one = eng.eval_batch(ct[-3:].astype(np.uint32), acc[-3:].astype(np.uint64))
    assert np.array_equal(one, got[-3:])


@pytest.mark.gpu
def test_wide_path_matches_fast_path_at_27_bits(mk_gpu, oracle):
    """MKACC_ENGINE=wide forces the 64-bit path on a 27-bit Q: both engines agree bit for bit."""
    mk = mk_gpu
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 6, 45181, 1 << 7, 5, seed=44)
    fast = _eng(mk, mk.MKNTRU, 2, 6, Q_MK, 45181, 1 << 7)
    fast.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    want = fast.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    os.environ["MKACC_ENGINE"] = "wide"
    try:
        wide = _eng(mk, mk.MKNTRU, 2, 6, Q_MK, 45181, 1 << 7)
    finally:
        del os.environ["MKACC_ENGINE"]
    assert wide.wide and not fast.wide
    wide.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = wide.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert np.array_equal(got, want)
    assert np.array_equal(got.astype(np.uint64), orc.evalacc(evk, pkey, ct, acc))


# Top of the supported range (Q < 2^61: the lazy butterflies keep words below
# 6Q < 2^64).  Largest primes = 1 mod 2N below 2^61 and below 2^60 (the
# reference's NATIVE_SIZE=64 MAX_MODULUS_SIZE); digits must satisfy
# log2(B_g) * digitsG <= 63.
Q61 = 2305843009213616129
Q60 = 1152921504606830593


def test_oracle_top_of_range_ntt_roundtrip(oracle):
    for Q in (Q61, Q60):
        assert oracle.is_prime(Q) and (Q - 1) % (2 * N) == 0
        psi = oracle.root_of_unity(2 * N, Q)
        a = oracle.fill_uniform(N, Q, 5)
        a[:8] = Q - 1
        assert np.array_equal(oracle.ntt_inverse(oracle.ntt_forward(a, Q, psi), Q, psi), a)


@pytest.mark.gpu
def test_wide_primitives_top_of_range(mk_gpu, oracle):
    """NTT / iNTT / SDD at a 61-bit Q: the lazy ranges' worst case (words up to 6Q)."""
    mk = mk_gpu
    eng = _eng(mk, mk.MKNTRU, 2, 3, Q61, 45181, 1 << 21)
    assert eng.wide and eng.dg == 2
    psi = oracle.root_of_unity(2 * N, Q61)
    assert eng.params.root == psi
    a = oracle.fill_uniform(4 * N, Q61, 31).reshape(4, N)
    a[0] = Q61 - 1                      # all-maximal residues
    a[1, ::2] = 0
    f = eng.ntt_forward(a)
    assert np.array_equal(f, np.stack([oracle.ntt_forward(x, Q61, psi) for x in a]))
    assert np.array_equal(eng.ntt_inverse(f), a)
    assert np.array_equal(eng.sdd(a), np.stack([oracle.sdd(x, Q61, 1 << 21, 2) for x in a]))


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["XZW", "XZW_B"])
def test_wide_evalacc_60bit(mk_gpu, oracle, method):
    """EvalAcc at the reference's largest NATIVE_SIZE=64 modulus size (60 bits)."""
    mk = mk_gpu
    m = oracle.XZW if method == "XZW" else oracle.XZW_B
    orc, evk, pkey, ct, acc = make_case(oracle, m, 2, 3, 45181, 1 << 20, 2, seed=60, Q=Q60)
    exp = orc.evalacc(evk, pkey, ct, acc)
    eng = _eng(mk, mk.MKNTRU if method == "XZW" else mk.MKNTRU_LWE, 2, 3, Q60, 45181, 1 << 20)
    assert eng.wide
    eng.upload_keys(evk.astype(np.uint64), pkey.astype(np.uint64))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint64))
    assert np.array_equal(got, exp), int(np.count_nonzero(got != exp))


@pytest.mark.gpu
def test_wide_rejects_q_at_2_61(mk_gpu):
    mk = mk_gpu
    # the range check comes before the primality check
    with pytest.raises(mk.MkaccError) as e:
        _eng(mk, mk.MKNTRU, 2, 3, (1 << 61) + 1, 45181, 1 << 21)
    assert e.value.code == -2
