"""The device-pointer entry points bench.py times, the device key upload, the
input-range reporting of the device path, the key caches of the accumulator
seam, and the bench's own B = 4096 full-n shape -- all against the oracle."""
import json
import os

import numpy as np
import pytest

from conftest import Q_MK, ROOT, make_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mk():
    import mkfhe_amd
    return mkfhe_amd


def _t(a, dev="cuda:0"):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        return torch.from_numpy(a.view(np.int64)).to(dev)
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)


def _engine(mk, method, k, n, q, baseG, Q=Q_MK):
    return mk.MKAccumulatorEngine(mk.make_params(method, k, n, 2048, Q, q, baseG))


@pytest.mark.parametrize("meth,word", [("XZW", 4), ("XZW", 8), ("XZW_B", 4)])
def test_upload_keys_device_and_device_batch(mk, oracle, meth, word):
    """keys uploaded from device memory (u32 / u64 words) + separate in/out device buffers."""
    import torch
    om, em, q = (oracle.XZW, mk.MKNTRU, 45181) if meth == "XZW" else (oracle.XZW_B, mk.MKNTRU_LWE, 32749)
    orc, evk, pkey, ct, acc = make_case(oracle, om, 2, 5, q, 1 << 7, 5, seed=31 + word)
    exp = orc.evalacc(evk, pkey, ct, acc)
    eng = _engine(mk, em, 2, 5, q, 1 << 7)
    wd = np.uint64 if word == 8 else np.uint32
    eng.upload_keys_device(_t(evk.astype(wd)), _t(pkey.astype(wd)))
    d_ct, d_in = _t(ct.astype(np.uint32)), _t(acc.astype(np.uint32))
    d_out = torch.empty_like(d_in)
    eng.eval_batch_device(d_ct, d_in, d_out, 5)
    eng.sync()
    assert np.array_equal(d_out.cpu().numpy().view(np.uint32), exp.astype(np.uint32))
    assert np.array_equal(d_in.cpu().numpy().view(np.uint32), acc.astype(np.uint32))   # input untouched
    # in place (d_in aliased to d_out)
    eng.eval_batch_device(d_ct, d_in, d_in, 5)
    eng.sync()
    assert np.array_equal(d_in.cpu().numpy().view(np.uint32), exp.astype(np.uint32))


def test_upload_keys_device_wide(mk, oracle):
    """64-bit word path (config 5 stress modulus): Montgomery-form keys built on the device."""
    Q50 = 1125899906826241
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 3, 45181, 1 << 10, 2, seed=55, Q=Q50)
    exp = orc.evalacc(evk, pkey, ct, acc)
    eng = _engine(mk, mk.MKNTRU, 2, 3, 45181, 1 << 10, Q=Q50)
    assert eng.wide
    eng.upload_keys_device(_t(evk.astype(np.uint64)), _t(pkey.astype(np.uint64)))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint64))
    assert np.array_equal(got, exp.astype(np.uint64))


def test_upload_keys_device_rejects_noncanonical(mk, oracle):
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 3, 45181, 1 << 7, 1, seed=9)
    eng = _engine(mk, mk.MKNTRU, 2, 3, 45181, 1 << 7)
    bad = evk.astype(np.uint32).copy()
    bad.reshape(-1)[12345] = Q_MK
    with pytest.raises(mk.MkaccError) as e:
        eng.upload_keys_device(_t(bad), _t(pkey.astype(np.uint32)))
    assert e.value.code == -5                       # MKACC_E_RANGE
    with pytest.raises(mk.MkaccError) as e:         # and no keys are left behind
        eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert e.value.code == -3                       # MKACC_E_NOKEYS


def test_device_entry_reports_out_of_range_inputs(mk, oracle):
    import torch
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 3, 45181, 1 << 7, 4, seed=10)
    eng = _engine(mk, mk.MKNTRU, 2, 3, 45181, 1 << 7)
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    d_in, d_out = _t(acc.astype(np.uint32)), None
    d_out = torch.empty_like(d_in)
    ct_bad = ct.astype(np.uint32).copy()
    ct_bad[2, 1, 0] = 45181                       # a ciphertext word not mod q
    eng.eval_batch_device(_t(ct_bad), d_in, d_out, 4)
    with pytest.raises(mk.MkaccError) as e:
        eng.sync()
    assert e.value.code == -5
    eng.sync()                                    # reported once, then cleared
    acc_bad = acc.astype(np.uint32).copy()
    acc_bad[3, 0, 7] = Q_MK                        # an accumulator word not canonical
    eng.eval_batch_device(_t(ct.astype(np.uint32)), _t(acc_bad), d_out, 4)
    with pytest.raises(mk.MkaccError):
        eng.sync()
    # a clean batch afterwards is exact
    eng.eval_batch_device(_t(ct.astype(np.uint32)), d_in, d_out, 4)
    eng.sync()
    assert np.array_equal(d_out.cpu().numpy().view(np.uint32), orc.evalacc(evk, pkey, ct, acc).astype(np.uint32))


def test_gate_device_entry_reports_out_of_range_inputs(mk):
    import torch
    from mkfhe_amd import keys as K
    p = K.paramset("STD100_MKNTRU", 0)
    eng = mk.MKAccumulatorEngine(p.acc)
    k, n = p.acc.k, p.acc.n
    rng = np.random.default_rng(3)
    evk = rng.integers(0, Q_MK, size=eng.evk_shape, dtype=np.uint32)
    pkey = rng.integers(0, Q_MK, size=eng.pkey_shape, dtype=np.uint32)
    eng.upload_keys(evk, pkey)
    dks = 4
    ksk = rng.integers(0, p.ks.qKS, size=(k, 2048 * dks, n), dtype=np.uint32)
    eng.upload_ksk_mntru(ksk, p.ks.qKS, p.ks.baseKS, n)
    a1 = rng.integers(0, p.acc.q, size=(2, k, n), dtype=np.uint32)
    a2 = rng.integers(0, p.acc.q, size=(2, k, n), dtype=np.uint32)
    nand = rng.integers(0, p.acc.q, size=(k, n), dtype=np.uint32)
    a2[1, 1, 3] = p.acc.q
    out = torch.empty((2, k, n), dtype=torch.int32, device="cuda:0")
    eng.eval_nand_device(_t(nand), _t(a1), None, _t(a2), None, out, None, 2)
    with pytest.raises(mk.MkaccError) as e:
        eng.sync()
    assert e.value.code == -5


def test_accumulator_key_cache_survives_recycled_arrays(mk, oracle):
    """EvalAcc with key set A, drop A, EvalAcc with key set B (which may
    reuse A's memory / id), and an in-place edit of B -- every result must follow
    the keys actually passed."""
    acc_obj = mk.accumulator_for(mk.make_params(mk.MKNTRU, 2, 3, 2048, Q_MK, 45181, 1 << 7))
    for seed in (1, 2):
        orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 3, 45181, 1 << 7, 1, seed=seed)
        e32, p32 = evk.astype(np.uint32), pkey.astype(np.uint32)
        a = acc[0].astype(np.uint32).copy()
        acc_obj.EvalAcc(e32, p32, None, a, ct[0].astype(np.uint32))
        assert np.array_equal(a, orc.evalacc(evk, pkey, ct[0], acc[0]).astype(np.uint32)), seed
        # same array objects, edited in place: must be re-uploaded
        e32.reshape(-1)[::97] = (e32.reshape(-1)[::97] + 1) % Q_MK
        evk2 = e32.astype(np.uint64)
        a = acc[0].astype(np.uint32).copy()
        acc_obj.EvalAcc(e32, p32, None, a, ct[0].astype(np.uint32))
        assert np.array_equal(a, orc.evalacc(evk2, pkey, ct[0], acc[0]).astype(np.uint32)), seed
        del e32, p32, evk, evk2


def test_mkntru_b_gate_is_rejected(mk):
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU_B, 2, 4, 2048, Q_MK, 32749, 1 << 9))
    A = np.zeros((2, 2048, 32, 3, 4), dtype=np.uint32)
    with pytest.raises(mk.MkaccError, match="MKNTRU_B"):
        eng.upload_ksk_mklwe(A, np.zeros((2, 2048, 32, 3), dtype=np.uint32), 32749, 32, 4)
    z = np.zeros((1, 2, 4), dtype=np.uint32)
    eng.ks = mk._lib.MkaccKsParams(32749, 32, 4)   # past the Python-side "no ksk" check, into the C ABI
    with pytest.raises(mk.MkaccError, match="MKNTRU_B"):
        eng.eval_nand_mklwe(z, np.zeros(1, np.uint32), z + 1, np.zeros(1, np.uint32))


def _big(fname):
    f = os.path.join(ROOT, "tests", "golden", fname)
    return json.load(open(f)) if os.path.exists(f) else None


@pytest.mark.parametrize("which", ["mkntru", "mklwe"])
def test_bench_shape_b4096_full_n(mk, oracle, which):
    """The benched shapes at full n, B = 4096 in one batch (every wave slot of every
    workgroup, two rounds of the chip's 2048 slots, cut into two slices on two
    streams -- the launches bench.py times): STD128_MKNTRU (headline, XZW, k = 2)
    and STD100_MKNTRU_LWE_2 (config 3, XZW_B, k = 4).  The whole output against
    the committed oracle digest, per gate, and two runs identical."""
    import hashlib
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden
    name, method, k, n, q, baseG, Q, B, seed, fname = make_golden.BIG_BATCHES[which]
    g = _big(fname)
    assert g is not None, f"tests/golden/{fname} missing (make_golden.py --big-batch {which})"
    orc, evk, pkey, ct, acc = make_golden.big_batch_inputs(which=which)
    eng = _engine(mk, mk.MKNTRU if method == oracle.XZW else mk.MKNTRU_LWE, k, n, q, baseG)
    assert eng.step_kernel_name(B) == "mk_step2_kernel"
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    r1 = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    r2 = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    bad = [b for b in range(g["B"]) if hashlib.sha256(np.ascontiguousarray(r1[b], dtype="<u8").tobytes()
                                                      ).hexdigest()[:16] != g["gate_sha256_16"][b]]
    assert not bad, f"{len(bad)} gates differ from the oracle, first {bad[:16]}"
    assert make_golden.digest(r1) == g["sha256"]
    assert np.array_equal(r1, r2)


@pytest.mark.parametrize("ps,method", [("STD100_MKNTRU", 0), ("STD100_MKNTRU_LWE", 2)])
def test_upload_ksk_device_matches_host_upload(mk, ps, method):
    """mkacc_upload_ksk_*_device (bench.py's broadcast buffer) == the host upload, and a
    word >= qKS is refused without leaving a key behind."""
    import torch
    from mkfhe_amd import keys as K
    p = K.paramset(ps, method)
    k, n = p.acc.k, p.acc.n
    rng = np.random.default_rng(17)
    dks = 4 if method == 0 else 3
    outs = []
    for dev_upload in (False, True):
        eng = mk.MKAccumulatorEngine(p.acc)
        eng.upload_keys(rng.integers(0, Q_MK, size=eng.evk_shape, dtype=np.uint32) * 0 + 5,
                        rng.integers(0, Q_MK, size=eng.pkey_shape, dtype=np.uint32) * 0 + 7)
        r2 = np.random.default_rng(18)
        if method == 0:
            ksk = r2.integers(0, p.ks.qKS, size=(k, 2048 * dks, n), dtype=np.uint32)
            if dev_upload:
                eng.upload_ksk_device(p.ks.qKS, p.ks.baseKS, n, d_ksk=_t(ksk))
            else:
                eng.upload_ksk_mntru(ksk, p.ks.qKS, p.ks.baseKS, n)
            a1 = r2.integers(0, p.acc.q, size=(3, k, n), dtype=np.uint32)
            a2 = r2.integers(0, p.acc.q, size=(3, k, n), dtype=np.uint32)
            outs.append(eng.eval_nand_mntru(r2.integers(0, p.acc.q, size=(k, n), dtype=np.uint32), a1, a2))
        else:
            A = r2.integers(0, p.ks.qKS, size=(k, 2048, 32, dks, n), dtype=np.uint32)
            Bk = r2.integers(0, p.ks.qKS, size=(k, 2048, 32, dks), dtype=np.uint32)
            if dev_upload:
                eng.upload_ksk_device(p.ks.qKS, p.ks.baseKS, n, d_A=_t(A), d_B=_t(Bk))
            else:
                eng.upload_ksk_mklwe(A, Bk, p.ks.qKS, p.ks.baseKS, n)
            a1 = r2.integers(0, p.acc.q, size=(3, k, n), dtype=np.uint32)
            a2 = r2.integers(0, p.acc.q, size=(3, k, n), dtype=np.uint32)
            b = r2.integers(0, p.acc.q, size=3, dtype=np.uint32)
            outs.append(np.concatenate([x.reshape(-1) for x in eng.eval_nand_mklwe(a1, b, a2, b)]))
    assert np.array_equal(outs[0], outs[1])
    eng = mk.MKAccumulatorEngine(p.acc)
    if method == 0:
        bad = torch.full((k * 2048 * dks * n,), int(p.ks.qKS), dtype=torch.int32, device="cuda:0")
        with pytest.raises(mk.MkaccError) as e:
            eng.upload_ksk_device(p.ks.qKS, p.ks.baseKS, n, d_ksk=bad)
        assert e.value.code == -5


def test_key_upload_keeps_a_pending_batch_error(mk, oracle):
    """a device key upload must not clear an input-range error of an
    earlier device batch that mkacc_sync has not reported yet."""
    import torch
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 3, 45181, 1 << 7, 2, seed=12)
    eng = _engine(mk, mk.MKNTRU, 2, 3, 45181, 1 << 7)
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    ct_bad = ct.astype(np.uint32).copy()
    ct_bad[0, 0, 0] = 45181
    d_in = _t(acc.astype(np.uint32))
    eng.eval_batch_device(_t(ct_bad), d_in, torch.empty_like(d_in), 2)
    eng.upload_keys_device(_t(evk.astype(np.uint32)), _t(pkey.astype(np.uint32)))
    with pytest.raises(mk.MkaccError) as e:
        eng.sync()
    assert e.value.code == -5


def test_wide_device_entry_reports_out_of_range_inputs(mk, oracle):
    """the 64-bit word path range-checks device accumulator words too
    (FP64 kernels for Q < 2^50, integer kernels above)."""
    import torch
    for Q, fp in ((1125899906826241, True), (1152921504606830593, False)):
        if not oracle.is_prime(Q):
            continue
        orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 2, 45181, 1 << 10, 2, seed=13, Q=Q)
        eng = _engine(mk, mk.MKNTRU, 2, 2, 45181, 1 << 10, Q=Q)
        assert eng.wide and eng.wide_fp == fp
        eng.upload_keys(evk.astype(np.uint64), pkey.astype(np.uint64))
        acc_bad = acc.astype(np.uint64).copy()
        acc_bad[1, 1, 5] = Q
        d_in = _t(acc_bad)
        eng.eval_batch_device(_t(ct.astype(np.uint32)), d_in, torch.empty_like(d_in), 2)
        with pytest.raises(mk.MkaccError) as e:
            eng.sync()
        assert e.value.code == -5
