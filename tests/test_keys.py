"""Host key material (include/mkfhe_keys.h): NTL-free key
generation, encryption and decryption, on the CPU.

Key generation is randomized in the reference (clock-seeded), so there is no
bit-exact target; these tests pin each function by the algebraic relation the
reference's construction guarantees (F * F^-1 = I, s * s^-1 = 1,
Pkey + CRS * s small, evk slots encrypting the right secret bits, key-switching
rows decrypting to s_i * B^t, fresh round trips), and the whole chain by the
NAND truth table through the CPU oracle: decrypt(oracle gate(real keys)) =
NAND.  That last test also pins the oracle's EvalAcc composition semantically
(DESIGN.md s3).
"""
import os

import numpy as np
import pytest

from conftest import Q_MK

K = pytest.importorskip("mkfhe_amd.keys")

N = 2048


@pytest.fixture(scope="module")
def lib():
    from mkfhe_amd import build
    build.build_keys()
    return K.load()


def centred(x, m):
    x = np.asarray(x, dtype=np.int64) % m
    return np.where(x > m // 2, x - m, x)


def test_paramset_matches_reference_table(lib):
    # binfhecontext.cpp:85-87, 129-144; mk-cryptoparameters.h:143-144
    p = K.paramset("STD128_MKNTRU", 0)
    assert (p.acc.k, p.acc.n, p.acc.N, p.acc.Q, p.acc.q, p.acc.baseG, p.acc.digitsG) == (2, 765, N, Q_MK, 45181, 128, 4)
    assert (p.ks.qKS, p.ks.baseKS, p.ks.n_out) == (45181, 32, 765)
    assert (p.sigma, p.sigma_unienc, p.sigma_r) == (0.5, 0.25, 0.15)
    assert (p.lwe_keydist, p.ring_keydist) == (K.DIST_TERNARY, K.DIST_GAUSSIAN)
    p = K.paramset("STD100_MKNTRU", 0)
    assert (p.acc.n, p.acc.baseG, p.sigma) == (560, 512, 0.75)
    p = K.paramset("STD100_MKNTRU_LWE_2", 2)
    assert (p.acc.k, p.acc.n, p.acc.q, p.ks.qKS, p.sigma) == (4, 500, 32749, 32749, 1.9)
    assert (p.lwe_keydist, p.ring_keydist) == (K.DIST_BINARY, K.DIST_TERNARY)
    with pytest.raises(Exception):
        K.paramset("STD128", 0)


def test_host_ntt_matches_oracle(lib, oracle):
    p = K.paramset("STD128_MKNTRU", 0)
    a = oracle.fill_uniform(3 * N, Q_MK, 17).reshape(3, N)
    got = K.ntt_forward(p, a)
    psi = oracle.root_of_unity(2 * N, Q_MK)
    exp = np.stack([oracle.ntt_forward(x, Q_MK, psi) for x in a])
    assert np.array_equal(got.astype(np.uint64), exp)
    assert np.array_equal(K.ntt_inverse(p, got).astype(np.uint64), a)


@pytest.mark.parametrize("ps", ["STD100_MKNTRU", "STD128_MKNTRU"])
def test_mntru_keygen_inverse(lib, ps):
    p = K.paramset(ps, 0)
    sk = K.mntru_keygen(p, 3)
    q = p.ks.qKS
    assert set(np.unique(sk.F).tolist()) <= {0, 1, q - 1}           # UNIFORM_TERNARY (mntru-pke.cpp:124-139)
    for u in range(p.acc.k):
        prod = (sk.F[u].astype(np.int64) @ sk.Finv[u].astype(np.int64)) % q
        assert np.array_equal(prod, np.eye(p.acc.n, dtype=np.int64))
    assert np.array_equal(sk.F_col0, sk.F[:, :, 0])


def test_keygen_is_deterministic_and_thread_independent(lib):
    p = K.paramset("STD100_MKNTRU", 0)
    a = K.mntru_keygen(p, 11)
    old = os.environ.get("OMP_NUM_THREADS")
    try:
        os.environ["OMP_NUM_THREADS"] = "1"
        b = K.mntru_keygen(p, 11)
        bk1 = K.bt_keygen(p, a, seed=5)
        os.environ["OMP_NUM_THREADS"] = "7"
        bk2 = K.bt_keygen(p, a, seed=5)
    finally:
        if old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = old
    assert np.array_equal(a.F, b.F) and np.array_equal(a.Finv, b.Finv)
    for f in ("crs", "skN", "pkey", "evk", "ksk"):
        assert np.array_equal(getattr(bk1, f), getattr(bk2, f)), f
    c = K.mntru_keygen(p, 12)
    assert not np.array_equal(a.F, c.F)


def test_seed_zero_draws_fresh_csprng_keys(lib):
    """seed 0 (the reference's behaviour): each call keys ChaCha20 with 256 fresh bits
    (mkkeys.cpp), so two key sets differ everywhere, the CRS included, and they are
    valid keys (s s^-1 = 1, Pkey + CRS s small, encryptions round trip)."""
    p = K.paramset("STD100_MKNTRU", 0)
    a, b = K.mntru_keygen(p, 0), K.mntru_keygen(p, 0)
    assert not np.array_equal(a.F, b.F)
    bk1, bk2 = K.bt_keygen(p, a), K.bt_keygen(p, a)
    for f in ("crs", "skN", "pkey", "evk", "ksk"):
        assert not np.array_equal(getattr(bk1, f), getattr(bk2, f)), f
    Q = p.acc.Q
    assert np.all((bk1.skN_eval.astype(np.uint64) * bk1.skNinv_eval) % Q == 1)
    for u in range(p.acc.k):
        e_eval = (bk1.pkey[u, 0].astype(np.uint64) + bk1.crs[0].astype(np.uint64) * bk1.skN_eval[u] % Q) % Q
        assert np.abs(centred(K.ntt_inverse(p, e_eval.astype(np.uint32)), Q)).max() <= 3
    m = np.random.default_rng(3).integers(0, 2, 64)
    assert np.array_equal(K.mntru_decrypt(p, a, K.mntru_encrypt(p, a, m), variant=K.DECRYPT2), m)


@pytest.fixture(scope="module")
def mntru_keys(lib):
    p = K.paramset("STD100_MKNTRU", 0)
    sk = K.mntru_keygen(p, 21)
    bk = K.bt_keygen(p, sk, seed=22)
    return p, sk, bk


def test_ring_secret_and_pkey_relations(mntru_keys):
    p, sk, bk = mntru_keys
    Q = p.acc.Q
    # s_u: Gaussian(0.5) truncated -> almost all in {-1, 0, 1}; EVAL form and inverse
    s = centred(bk.skN, Q)
    assert np.abs(s).max() <= 2 and 0 < np.count_nonzero(s)
    assert np.array_equal(K.ntt_forward(p, bk.skN), bk.skN_eval)
    assert np.all((bk.skN_eval.astype(np.uint64) * bk.skNinv_eval) % Q == 1)
    # Pkey[u][i] = e - CRS_i * s_u with e <- DGG(0.25): Pkey + CRS_i s_u is small
    for u in range(p.acc.k):
        for i in range(bk.crs.shape[0]):
            e_eval = (bk.pkey[u, i].astype(np.uint64) + bk.crs[i].astype(np.uint64) * bk.skN_eval[u] % Q) % Q
            e = centred(K.ntt_inverse(p, e_eval.astype(np.uint32)), Q)
            assert np.abs(e).max() <= 3


def test_acc_key_slots_encrypt_the_secret_bits(mntru_keys):
    """KeyGenAcc (mk-acc-xzw.cpp:38-87): ek[u][0][i] encrypts [s==1], ek[u][1][i] encrypts [s==-1];
    slot (0,0) and ek[0][0][n] are KDM keys.  With m_dggR = 0.15 the mask r is zero except with
    probability ~1e-6 per key, so d_t = e0 + m g_t (+ r_t CRS_t) reads off m directly."""
    p, sk, bk = mntru_keys
    Q, q, n, dg = p.acc.Q, p.ks.qKS, p.acc.n, bk.crs.shape[0]
    col0 = sk.F_col0
    rng = np.random.default_rng(0)
    for u in range(p.acc.k):
        for i in [1, 2] + list(rng.integers(3, n, 4)):
            for sgn in (0, 1):
                want = int(col0[u, i] == (1 if sgn == 0 else q - 1))
                for t in range(dg):
                    d = centred(K.ntt_inverse(p, bk.evk[u, sgn, i, t, 0]), Q)
                    g = pow(p.acc.baseG, t + 1, Q)
                    d[0] -= want * g
                    assert np.abs(d).max() <= 3, (u, i, sgn, t)
    # KDM slot: d_t * s = e0 s + m g_t
    s_eval = bk.skN_eval[0].astype(np.uint64)
    for t in range(dg):
        g = pow(p.acc.baseG, t + 1, Q)
        ds = centred(K.ntt_inverse(p, ((bk.evk[0, 0, n, t, 0] * s_eval) % Q).astype(np.uint32)), Q)
        ds[0] -= g
        assert np.abs(ds).max() <= 40
    # unused KDM slots of the other parties are zero (nullptr in the reference)
    assert not bk.evk[1, :, n].any() and not bk.evk[0, 1, n].any()


def test_mntru_ksk_rows_decrypt_to_scaled_secret(mntru_keys):
    """KeySwitchGen2 (mntru-pke.cpp:624-760): <KSK[u][i*dks+t], F_u[:,0]> = s_u[i] B^t + e."""
    p, sk, bk = mntru_keys
    q, B = p.ks.qKS, p.ks.baseKS
    k, n, N_, dg, nk, dks = K.dims(p)
    s = centred(bk.skN, p.acc.Q)
    rows = np.arange(0, N * dks, 97)
    for u in range(k):
        dec = (bk.ksk[u, rows].astype(np.int64) @ sk.F[u, :, 0].astype(np.int64)) % q
        i, t = rows // dks, rows % dks
        want = (s[u, i] * (B ** t)) % q
        assert np.abs(centred(dec - want, q)).max() <= 12


def test_mntru_encrypt_decrypt_roundtrip(mntru_keys):
    p, sk, _ = mntru_keys
    m = np.random.default_rng(2).integers(0, 2, 300)
    ct = K.mntru_encrypt(p, sk, m, seed=9)
    assert np.array_equal(K.mntru_decrypt(p, sk, ct, variant=K.DECRYPT2), m)   # Decrypt2: + q/8
    ctn = K.mntru_ctgate(p, sk, seed=10)
    inner = sum(int(ctn[u].astype(np.int64) @ sk.F[u, :, 0].astype(np.int64)) for u in range(p.acc.k)) % p.acc.q
    assert abs(int(centred(inner - 5 * p.acc.q // 8, p.acc.q))) <= 12          # ctGateGen: 5q/8 + e


def test_mklwe_keys_and_roundtrip(lib):
    p = K.paramset("STD100_MKNTRU_LWE", 2)
    sk = K.mklwe_keygen(p, 4)
    assert set(np.unique(sk.s).tolist()) <= {0, 1}
    m = np.random.default_rng(3).integers(0, 2, 300)
    a, b = K.mklwe_encrypt(p, sk, m, seed=5)
    assert np.array_equal(K.mklwe_decrypt(p, sk, a, b), m)


def test_mklwe_ksk_rows(lib):
    """KeySwitchGen (mklwe-pke.cpp:176-258): B - <A, s> = svN[i] * j * B^t + e."""
    p = K.paramset("STD100_MKNTRU_LWE", 2)
    sk = K.mklwe_keygen(p, 4)
    bk = K.bt_keygen(p, sk, seed=6)
    q, Bk = p.ks.qKS, p.ks.baseKS
    k, n, N_, dg, nk, dks = K.dims(p)
    assert bk.ksk_A.shape == (k, N, Bk, dks, n) and bk.ksk_B.shape == (k, N, Bk, dks)
    s = centred(bk.skN, p.acc.Q)
    for u in range(k):
        for i in (0, 5, 2047):
            A = bk.ksk_A[u, i].astype(np.int64)
            dec = (bk.ksk_B[u, i].astype(np.int64) - A @ sk.s[u].astype(np.int64)) % q
            j = np.arange(Bk)[:, None]
            t = np.arange(dks)[None, :]
            want = (s[u, i] * j * Bk ** t) % q
            assert np.abs(centred(dec - want, q)).max() <= 20


def _mntru_gates_oracle(oracle, ps, m1, m2, seed):
    p = K.paramset(ps, 0)
    k, n, N_, dg, nk, dks = K.dims(p)
    sk = K.mntru_keygen(p, seed)
    bk = K.bt_keygen(p, sk, seed=seed + 1)
    ctn = K.mntru_ctgate(p, sk, seed + 2)
    c1 = K.mntru_encrypt(p, sk, m1, seed=seed + 3)
    c2 = K.mntru_encrypt(p, sk, m2, seed=seed + 4)
    orc = oracle.Oracle(oracle.XZW, k, n, N, p.acc.Q, p.acc.q, p.acc.baseG)
    heads = np.stack([oracle.mntru_head(ctn, c1[i], c2[i], p.acc.q) for i in range(len(m1))])
    acc0 = np.broadcast_to(orc.mntru_testvector(4), (len(m1), k, N)).copy()
    acc = orc.evalacc_batch(bk.evk, bk.pkey, heads, acc0, os.cpu_count() or 1)
    out = np.stack([orc.mntru_tail_ksk1(acc[i], bk.ksk, p.ks.qKS, p.ks.baseKS, n) for i in range(len(m1))])
    return K.mntru_decrypt(p, sk, out.astype(np.uint32), mod=p.ks.qKS)


def test_nand_truth_table_mkntru_through_oracle(lib, oracle):
    """boolean-mkntru with real keys: decrypt(EvalBinGate(NAND)) on the CPU oracle."""
    m1 = np.array([0, 0, 1, 1, 1, 0, 1, 0])
    m2 = np.array([0, 1, 0, 1, 1, 1, 0, 0])
    got = _mntru_gates_oracle(oracle, "STD100_MKNTRU", m1, m2, 31)
    assert np.array_equal(got, 1 - (m1 & m2))


def test_nand_truth_table_mklwe_through_oracle(lib, oracle):
    """boolean-mklwe with real keys through the CPU oracle."""
    p = K.paramset("STD100_MKNTRU_LWE", 2)
    k, n, N_, dg, nk, dks = K.dims(p)
    sk = K.mklwe_keygen(p, 41)
    bk = K.bt_keygen(p, sk, seed=42)
    m1 = np.array([0, 0, 1, 1, 1, 0])
    m2 = np.array([0, 1, 0, 1, 1, 1])
    a1, b1 = K.mklwe_encrypt(p, sk, m1, seed=43)
    a2, b2 = K.mklwe_encrypt(p, sk, m2, seed=44)
    orc = oracle.Oracle(oracle.XZW_B, k, n, N, p.acc.Q, 2 * N, p.acc.baseG)
    cs, accs = zip(*[orc.mklwe_head(a1[i], b1[i], a2[i], b2[i], p.acc.q) for i in range(len(m1))])
    acc = orc.evalacc_batch(bk.evk, bk.pkey, np.stack(cs), np.stack(accs), os.cpu_count() or 1)
    A, Bk = bk.ksk_A.astype(np.uint64), bk.ksk_B.astype(np.uint64)
    outs = [orc.mklwe_tail(acc[i], A, Bk, p.ks.qKS, p.ks.baseKS, n) for i in range(len(m1))]
    oa = np.stack([o[0] for o in outs]).astype(np.uint32)
    ob = np.array([o[1] for o in outs], dtype=np.uint32)
    assert np.array_equal(K.mklwe_decrypt(p, sk, oa, ob, mod=p.ks.qKS), 1 - (m1 & m2))


def test_error_behaviour(lib):
    from mkfhe_amd.binfhe import BinFHEContext, ConfigError
    cc = BinFHEContext()
    cc.GenerateBinFHEContext("STD100_MKNTRU", 0)
    with pytest.raises(ConfigError):
        cc.MKLWE_KeyGen()                   # binfhecontext.cpp:244-249
    sk = cc.MNTRU_KeyGen()
    with pytest.raises(ConfigError):
        cc.ctGateGen(sk, 1)                 # binfhe-base-scheme.cpp:341-342
    with pytest.raises(ConfigError):
        cc.EvalBinGate(3, cc.Encrypt(sk, 0), cc.Encrypt(sk, 1))   # no MKBTKeyGen yet
    with pytest.raises(ConfigError):
        cc.GenerateBinFHEContext("STD100_MKNTRU", 1 + 5)


def test_keys_header_symbols_bound_and_exported(lib):
    """Every function include/mkfhe_keys.h declares is exported and bound in mkfhe_amd/keys.py."""
    import re
    from conftest import ROOT
    txt = open(os.path.join(ROOT, "include", "mkfhe_keys.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"\b(mkkg_[a-z0-9_]+)\s*\(", txt))
    assert len(names) >= 26
    assert names == set(K.SIGNATURES)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.mkkg_abi_version() == 3


def test_key_files_roundtrip(mntru_keys, tmp_path):
    """Key wire format: save -> load is the identity, params travel along."""
    p, sk, bk = mntru_keys
    f_sk, f_bk = str(tmp_path / "sk.mkfk"), str(tmp_path / "bt.mkfk")
    K.save_secret_key(f_sk, p, sk)
    K.save_btkey(f_bk, p, bk)
    p2, sk2 = K.load_secret_key(f_sk)
    assert np.array_equal(sk2.F, sk.F) and np.array_equal(sk2.Finv, sk.Finv)
    assert (p2.acc.k, p2.acc.n, p2.acc.Q, p2.acc.root, p2.ks.qKS, p2.sigma) == \
        (p.acc.k, p.acc.n, p.acc.Q, p.acc.root, p.ks.qKS, p.sigma)
    p3, bk2 = K.load_btkey(f_bk)
    for f in ("crs", "skN", "skN_eval", "skNinv_eval", "pkey", "evk", "ksk"):
        assert np.array_equal(getattr(bk2, f), getattr(bk, f)), f
    assert bk2.ksk_A is None
    kind, _, count = K.file_info(f_bk)
    assert kind == K.FILE_BTKEY and count == 7


def test_key_file_rejects_corruption(lib, tmp_path):
    p = K.paramset("STD100_MKNTRU_LWE", 2)
    sk = K.mklwe_keygen(p, 77)
    f = str(tmp_path / "s.mkfk")
    K.save_secret_key(f, p, sk)
    assert np.array_equal(K.load_secret_key(f)[1].s, sk.s)
    raw = bytearray(open(f, "rb").read())
    raw[-20] ^= 1                                  # a data byte of the last section
    open(f, "wb").write(bytes(raw))
    with pytest.raises(Exception, match="checksum"):
        K.load_secret_key(f)
    open(f, "wb").write(b"NOTAKEY!" + bytes(raw[8:]))
    with pytest.raises(Exception, match="MKFHEKEY"):
        K.load_secret_key(f)
    with pytest.raises(Exception):
        K.load_btkey(str(tmp_path / "missing.mkfk"))


def test_key_file_rejects_bad_sizes_and_params(lib, tmp_path):
    """The reader bounds every file-supplied size by the bytes the file holds and
    refuses a parameter block that is not a valid MK parameter set, before any
    buffer is sized from it (the format is ours: the reference serialises no MK
    key, binfhecontext-ser.h:10-24)."""
    import struct
    p = K.paramset("STD100_MKNTRU_LWE", 2)
    sk = K.mklwe_keygen(p, 78)
    f = str(tmp_path / "s.mkfk")
    K.save_secret_key(f, p, sk)
    good = bytes(open(f, "rb").read())
    head = 8 + 4 + 4 + 18 * 8 + 4                        # magic, version, kind, params, count
    assert good[head:head + 1] == b"s"                    # the first section: name, words, data

    def bad(raw, match):
        open(f, "wb").write(bytes(raw))
        with pytest.raises(Exception, match=match):
            K.load_secret_key(f)

    bad(good[:len(good) // 2], "truncated")               # cut inside the data
    bad(good[:head + 10], "truncated")                    # cut inside a section header
    raw = bytearray(good)
    raw[head + 16:head + 24] = struct.pack("<Q", 1 << 62)  # section words far past the end
    bad(raw, "larger than the file")
    raw = bytearray(good)
    raw[head + 16:head + 24] = struct.pack("<Q", (len(good) - head) // 4)   # one word too many
    bad(raw, "larger than the file")
    raw = bytearray(good)
    raw[head - 4:head] = struct.pack("<I", 0xFFFFFFFF)    # section count
    bad(raw, "section count")
    raw = bytearray(good)
    raw[12:16] = struct.pack("<I", 77)                    # kind
    bad(raw, "kind")
    for word, value in ((3, 3), (4, 4), (1, 1 << 20), (6, 3), (12, 0x7FF8000000000000)):   # N, Q, k, baseG, sigma NaN
        raw = bytearray(good)
        raw[16 + 8 * word:24 + 8 * word] = struct.pack("<Q", value)
        bad(raw, "parameter block")
    open(f, "wb").write(good)
    assert np.array_equal(K.load_secret_key(f)[1].s, sk.s)
