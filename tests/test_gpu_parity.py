"""Bit-exact parity of the HIP engine (through the C ABI) against the CPU oracle.

Small-n cases run every code path (first KDM step, later steps, both methods,
every supported digit count) at the real ring size N = 2048; the full-size
cases run the reference parameter sets end to end on a few gates.
"""
import numpy as np
import pytest

from conftest import Q_MK, make_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mk():
    import mkfhe_amd
    return mkfhe_amd


def _engine(mk, method, k, n, q, baseG):
    p = mk.make_params(method, k, n, 2048, Q_MK, q, baseG)
    return mk.MKAccumulatorEngine(p)


def test_native_library_loaded(mk):
    import mkfhe_amd._lib as L
    lib = L.load()
    assert lib.mkacc_abi_version() == 2


def test_ntt_forward_inverse_parity(mk, oracle):
    eng = _engine(mk, mk.MKNTRU, 2, 4, 45181, 1 << 9)
    psi = oracle.root_of_unity(4096, Q_MK)
    a = oracle.fill_uniform(7 * 2048, Q_MK, 77).reshape(7, 2048)
    fw = eng.ntt_forward(a.astype(np.uint32))
    for i in range(7):
        assert np.array_equal(fw[i], oracle.ntt_forward(a[i], Q_MK, psi).astype(np.uint32)), i
    inv = eng.ntt_inverse(fw)
    assert np.array_equal(inv, a.astype(np.uint32))
    for i in range(7):
        assert np.array_equal(eng.ntt_inverse(a[i:i + 1].astype(np.uint32))[0],
                              oracle.ntt_inverse(a[i], Q_MK, psi).astype(np.uint32))


def test_ntt_edge_values(mk, oracle):
    eng = _engine(mk, mk.MKNTRU, 2, 4, 45181, 1 << 9)
    psi = oracle.root_of_unity(4096, Q_MK)
    cases = np.stack([np.zeros(2048), np.full(2048, Q_MK - 1), np.eye(1, 2048, 0)[0],
                      np.eye(1, 2048, 2047)[0]]).astype(np.uint64)
    fw = eng.ntt_forward(cases.astype(np.uint32))
    for i in range(len(cases)):
        assert np.array_equal(fw[i], oracle.ntt_forward(cases[i], Q_MK, psi).astype(np.uint32))


@pytest.mark.parametrize("logB", [9, 7, 6, 5])
def test_sdd_parity(mk, oracle, logB):
    eng = _engine(mk, mk.MKNTRU, 2, 4, 45181, 1 << logB)
    x = oracle.fill_uniform(3 * 2048, Q_MK, 5 + logB).reshape(3, 2048)
    x[0, :8] = [0, 1, Q_MK // 2 - 1, Q_MK // 2, Q_MK // 2 + 1, Q_MK - 1, (1 << logB) // 2, (1 << logB)]
    got = eng.sdd(x.astype(np.uint32))
    for i in range(3):
        exp = oracle.sdd(x[i], Q_MK, 1 << logB, eng.dg)
        assert np.array_equal(got[i], exp.astype(np.uint32))


CASES = [
    # method, k, n, q, baseG, B
    ("XZW", 2, 4, 45181, 1 << 9, 3),      # STD100_MKNTRU shape, dg=2
    ("XZW", 2, 5, 45181, 1 << 7, 2),      # STD128_MKNTRU shape, dg=3
    ("XZW", 3, 3, 45181, 1 << 6, 2),      # dg=4
    ("XZW", 2, 3, 45181, 1 << 5, 2),      # dg=5 (STD128_MKNTRU_4 base)
    ("XZW_B", 2, 4, 32749, 1 << 9, 3),    # STD100_MKNTRU_LWE shape
    ("XZW_B", 4, 3, 32749, 1 << 9, 2),    # 4 parties
    ("XZW_B", 2, 3, 32749, 1 << 7, 2),    # dg=3
    ("XZW", 1, 6, 45181, 1 << 9, 2),      # single party
    ("XZW", 5, 2, 45181, 1 << 9, 5),      # odd party count, odd batch
    ("XZW", 16, 2, 45181, 1 << 5, 2),     # STD128_MKNTRU_4 shape: 16 parties, dg=5
    ("XZW_B", 16, 2, 32749, 1 << 7, 3),   # STD128_MKNTRU_LWE_4 shape: 16 parties, dg=3
    ("XZW", 8, 3, 45181, 1 << 6, 2),      # STD128_MKNTRU_3 shape (config 4): 8 parties, dg=4
    ("XZW_B", 3, 3, 32749, 1 << 6, 3),    # dg=4, binary keys
    ("XZW", 8, 2, 45181, 1 << 9, 2),      # STD100_MKNTRU_3 shape: 8 parties, dg=2
    ("XZW_B", 6, 2, 32749, 1 << 9, 3),    # 6 parties, dg=2 (one-launch step loop at k = 5..8)
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-k{c[1]}-n{c[2]}-logB{c[4].bit_length() - 1}-B{c[5]}" for c in CASES])
def test_evalacc_small_parity(mk, oracle, case):
    meth, k, n, q, baseG, B = case
    om = oracle.XZW if meth == "XZW" else oracle.XZW_B
    em = mk.MKNTRU if meth == "XZW" else mk.MKNTRU_LWE
    orc, evk, pkey, ct, acc = make_case(oracle, om, k, n, q, baseG, B, seed=k * 100 + n)
    # exercise the monomial edge cases c = 0 and c = 2N-1 (and 2N for XZW_B)
    ct[0, 0, 0] = 0
    if om == oracle.XZW:
        ct[0, k - 1, n - 1] = q - 1
    else:
        ct[0, k - 1, n - 1] = 4096
        ct[-1, 0, n - 1] = 4095
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8)
    eng = mk.MKAccumulatorEngine(mk.make_params(em, k, n, 2048, Q_MK, q, baseG))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert np.array_equal(got, exp.astype(np.uint32))
    # u64 upload path gives the same
    eng.upload_keys(evk, pkey)
    assert np.array_equal(eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32)), got)


DSCR_CASES = [c for c in CASES if c[0] == "XZW" and c[1] >= 2]


@pytest.mark.parametrize("dscr", ["0", "1"])
@pytest.mark.parametrize("case", DSCR_CASES, ids=[f"k{c[1]}-logB{c[4].bit_length() - 1}" for c in DSCR_CASES])
def test_evalacc_dscr_modes(mk, oracle, case, dscr, monkeypatch):
    """Both d_i modes of the XZW step kernel (recomputed per party pass, or
    computed by the first pass and reloaded from the HBM scratch; the engine
    picks by k, MKACC_DSCR forces one) give the oracle's accumulators."""
    meth, k, n, q, baseG, B = case
    monkeypatch.setenv("MKACC_DSCR", dscr)   # read when the context sizes its workspace
    monkeypatch.setenv("MKACC_LAT", "0")     # the batch step kernel (small B would take mk_lat_kernel
    monkeypatch.setenv("MKACC_QUAD", "0")    # or mk_quad_kernel)
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, k, n, q, baseG, B + 2, seed=k * 31 + n)
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, k, n, 2048, Q_MK, q, baseG))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert np.array_equal(got, exp.astype(np.uint32))


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-k{c[1]}-logB{c[4].bit_length() - 1}" for c in CASES])
def test_evalacc_step_kernels(mk, oracle, case, monkeypatch):
    """The batch step kernel the engine selects -- mk_step2_kernel (digit NTTs
    first, one key stream per pass) at dg <= 3, mk_step_kernel at dg >= 4 --
    gives the oracle's accumulators for every case shape, with the monomial edge
    cases in the first and last gate; MKACC_LAT=0 and MKACC_QUAD=0 keep small batches
    off the small-batch kernels."""
    meth, k, n, q, baseG, B = case
    monkeypatch.setenv("MKACC_LAT", "0")
    monkeypatch.setenv("MKACC_QUAD", "0")
    om = oracle.XZW if meth == "XZW" else oracle.XZW_B
    em = mk.MKNTRU if meth == "XZW" else mk.MKNTRU_LWE
    orc, evk, pkey, ct, acc = make_case(oracle, om, k, n, q, baseG, B + 3, seed=k * 17 + n + 2)
    ct[0, 0, 0] = 0
    ct[-1, k - 1, n - 1] = q - 1 if om == oracle.XZW else 4096
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8)
    eng = mk.MKAccumulatorEngine(mk.make_params(em, k, n, 2048, Q_MK, q, baseG))
    assert eng.step_kernel_name(B + 3) == ("mk_step2_kernel" if eng.dg <= 3 else "mk_step_kernel")
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert np.array_equal(got, exp.astype(np.uint32))


LAT_CASES = [c for c in CASES if 2 <= c[1] <= 8 and c[4] != 1 << 5]


@pytest.mark.parametrize("lat", ["1", "0"])
@pytest.mark.parametrize("case", LAT_CASES,
                         ids=[f"{c[0]}-k{c[1]}-logB{c[4].bit_length() - 1}" for c in LAT_CASES])
def test_evalacc_small_batch_kernel(mk, oracle, case, lat, monkeypatch):
    """The one-wave-per-party step kernel (mk_lat_kernel, chosen for small
    batches; MKACC_LAT forces it on or off) gives the oracle's accumulators for
    both methods, k = 2..8 parties and dg = 2..4."""
    meth, k, n, q, baseG, B = case
    monkeypatch.setenv("MKACC_LAT", lat)   # read at context creation
    monkeypatch.setenv("MKACC_QUAD", "0")  # small batches would take mk_quad_kernel
    om = oracle.XZW if meth == "XZW" else oracle.XZW_B
    em = mk.MKNTRU if meth == "XZW" else mk.MKNTRU_LWE
    orc, evk, pkey, ct, acc = make_case(oracle, om, k, n, q, baseG, B + 1, seed=k * 13 + n)
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8)
    eng = mk.MKAccumulatorEngine(mk.make_params(em, k, n, 2048, Q_MK, q, baseG))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert np.array_equal(got, exp.astype(np.uint32))


@pytest.mark.parametrize("meth", ["XZW", "XZW_B"])
@pytest.mark.parametrize("logB", [9, 7, 6])   # dg = 2, 3, 4
def test_evalacc_two_party_split_digit_kernel(mk, oracle, meth, logB, monkeypatch):
    """Two parties, batches of at most one gate per CU: mk_latd_kernel (each party's
    digits over two waves, the f-part's over dg waves) equals the oracle and the
    one-wave-per-party kernel word for word, first step and later steps."""
    monkeypatch.setenv("MKACC_LAT", "1")
    monkeypatch.setenv("MKACC_QUAD", "0")
    om = oracle.XZW if meth == "XZW" else oracle.XZW_B
    em = mk.MKNTRU if meth == "XZW" else mk.MKNTRU_LWE
    q = 45181 if meth == "XZW" else 32749
    B = 5
    orc, evk, pkey, ct, acc = make_case(oracle, om, 2, 4, q, 1 << logB, B, seed=71 + logB)
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8).astype(np.uint32)
    outs = {}
    for split, name in (("1", "mk_latd_run_kernel"), ("0", "mk_lat_run_kernel")):
        monkeypatch.setenv("MKACC_LATD", split)
        eng = mk.MKAccumulatorEngine(mk.make_params(em, 2, 4, 2048, Q_MK, q, 1 << logB))
        monkeypatch.delenv("MKACC_LATD")            # read once, at context creation
        assert eng.step_kernel_name(B) == name       # steps 1..kn-1 in one launch (step 0: its own)
        eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
        outs[split] = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
        assert np.array_equal(outs[split], exp), name
    assert np.array_equal(outs["1"], outs["0"])


def test_interface_mirror_evalacc(mk, oracle):
    """UniEncAccumulatorXZW.EvalAcc updates acc in place like the reference."""
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 3, 45181, 1 << 9, 1, seed=9)
    exp = orc.evalacc(evk, pkey, ct[0], acc[0]).astype(np.uint32)
    accm = mk.accumulator_for(mk.make_params(mk.MKNTRU, 2, 3, 2048, Q_MK, 45181, 1 << 9))
    assert isinstance(accm, mk.UniEncAccumulatorXZW)
    a = acc[0].astype(np.uint32).copy()
    accm.EvalAcc(evk.astype(np.uint32), pkey.astype(np.uint32), None, a, ct[0].astype(np.uint32))
    assert np.array_equal(a, exp)


@pytest.mark.parametrize("name,B", [("STD100_MKNTRU", 2), ("STD128_MKNTRU", 2), ("STD100_MKNTRU_LWE", 2)])
def test_evalacc_full_paramset_parity(mk, oracle, name, B):
    p = mk.paramset(name)
    om = oracle.XZW if p.method == mk.MKNTRU else oracle.XZW_B
    orc, evk, pkey, ct, acc = make_case(oracle, om, p.k, p.n, p.q, p.baseG, B, seed=p.n)
    # start from the BootstrapGateCore test vector (binfhe-base-scheme.cpp:1093-1115)
    acc[:] = orc.mntru_testvector(4)
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8)
    eng = mk.MKAccumulatorEngine(p)
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert np.array_equal(got, exp.astype(np.uint32))


def test_batch_invariance(mk, oracle):
    """Gates are independent: permuting / duplicating the batch permutes the output."""
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 4, 45181, 1 << 7, 9, seed=3)
    eng = _engine(mk, mk.MKNTRU, 2, 4, 45181, 1 << 7)
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    out = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    perm = np.array([8, 3, 3, 0, 7, 1, 1, 2, 5])
    out2 = eng.eval_batch(ct[perm].astype(np.uint32), acc[perm].astype(np.uint32))
    assert np.array_equal(out2, out[perm])
    single = eng.eval_batch(ct[4:5].astype(np.uint32), acc[4:5].astype(np.uint32))
    assert np.array_equal(single[0], out[4])


def test_errors(mk, oracle):
    eng = _engine(mk, mk.MKNTRU, 2, 3, 45181, 1 << 9)
    ct = np.zeros((1, 2, 3), np.uint32)
    acc = np.zeros((1, 2, 2048), np.uint32)
    with pytest.raises(mk.MkaccError) as e:
        eng.eval_batch(ct, acc)                          # keys not uploaded
    assert e.value.code == -3
    evk = np.zeros(eng.evk_shape, np.uint32)
    pkey = np.zeros(eng.pkey_shape, np.uint32)
    eng.upload_keys(evk, pkey)
    with pytest.raises(mk.MkaccError) as e:
        eng.eval_batch(np.full((1, 2, 3), 45181, np.uint32), acc)   # ct >= q
    assert e.value.code == -5
    with pytest.raises(mk.MkaccError) as e:
        eng.eval_batch(ct, np.full((1, 2, 2048), Q_MK, np.uint32))  # non-canonical acc
    assert e.value.code == -5
    bad = evk.copy()
    bad.flat[123] = Q_MK
    with pytest.raises(mk.MkaccError):
        eng.upload_keys(bad, pkey)
    assert eng.eval_batch(ct[:0], acc[:0]).shape == (0, 2, 2048)


@pytest.mark.parametrize("lat", ["0", "1"])
def test_evalacc_many_gates_every_wave_slot(mk, oracle, lat, monkeypatch):
    """512 gates (every wave slot of every workgroup, all CUs partly busy),
    three repeated runs: bit-exact and run-to-run identical, with the batch
    step kernel and with the one-wave-per-party kernel.  Guards against the
    co-resident-workgroup corruption of round 1."""
    monkeypatch.setenv("MKACC_LAT", lat)
    monkeypatch.setenv("MKACC_QUAD", "0")
    B = 512
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 2, 45181, 1 << 7, B, seed=77)
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 16).astype(np.uint32)
    eng = _engine(mk, mk.MKNTRU, 2, 2, 45181, 1 << 7)
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    for _ in range(3):
        got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
        bad = [g for g in range(B) if not np.array_equal(got[g], exp[g])]
        assert not bad, f"gates differing from the oracle: {bad[:16]}"


# (method, k, n, log2 B_g): the headline kernel's shape (mk_step2_kernel, dg = 3),
# config 3's (the MK-LWE step2 kernel, XZW_B, k = 4, dg = 2) and the config-4
# kernel's (mk_step_kernel with its d_i scratch, k >= 4, dg = 4)
SPLIT_SHAPES = {"step2-k2-dg3": ("XZW", 2, 3, 7), "step2-mklwe-k4-dg2": ("XZW_B", 4, 2, 9),
                "dscr-k4-dg4": ("XZW", 4, 2, 6)}


@pytest.mark.parametrize("streams", ["2", "3", "4"])
@pytest.mark.parametrize("shape", list(SPLIT_SHAPES))
def test_two_stream_batch_split(mk, oracle, shape, streams, monkeypatch):
    """MKACC_STREAMS=2..4 cuts a batch of two or more units of resident gates into
    slices whose step launches run on streams of their own: the output equals the
    one-stream run word for word, and a spread sample across the slice boundaries
    equals the oracle.  B = 4100 (units of 1024 gates at 256 CUs): 2048 + 2052,
    1024 + 1024 + 2052, 1024 x 3 + 1028.  Every default batch kernel: MK-NTRU and
    MK-LWE step2 kernels, and the config-4 one, which reads its per-gate d_i scratch
    at the slice's gate offset."""
    meth, k, n, logb = SPLIT_SHAPES[shape]
    monkeypatch.setenv("MKACC_LAT", "0")
    om = oracle.XZW if meth == "XZW" else oracle.XZW_B
    q, baseG, B = (45181 if meth == "XZW" else 32749), 1 << logb, 4100
    orc, evk, pkey, ct, acc = make_case(oracle, om, k, n, q, baseG, B, seed=91 + k + (meth == "XZW_B"))
    # monomial edge exponents on both sides of every slice boundary
    for g in (1023, 1024, 2047, 2048, 3071, 3072):
        ct[g, 0, 0] = 0 if g % 2 else (q - 1 if om == oracle.XZW else 2 * 2048)
    params = mk.make_params(mk.MKNTRU if meth == "XZW" else mk.MKNTRU_LWE, k, n, 2048, Q_MK, q, baseG)
    outs = {}
    for ns in ("1", streams):
        monkeypatch.setenv("MKACC_STREAMS", ns)
        eng = mk.MKAccumulatorEngine(params)
        assert eng.step_kernel_name(B) == ("mk_step_kernel" if logb == 6 else "mk_step2_kernel")
        eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
        outs[ns] = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
        del eng
    assert np.array_equal(outs["1"], outs[streams])
    pick = [0, 1, 1023, 1024, 2047, 2048, 3071, 3072, 4099]
    exp = orc.evalacc_batch(evk, pkey, ct[pick], acc[pick], 8)
    assert np.array_equal(outs[streams][pick], exp.astype(np.uint32))


@pytest.mark.parametrize("k,B", [(5, 256), (6, 256), (3, 512)])
def test_small_batch_run_kernel_at_its_residency_limit(mk, oracle, k, B, monkeypatch):
    """mk_lat_run_kernel (the steps after the first in one launch) is taken only while
    every gate's workgroup is resident at once: floor(4 occ / k) workgroups per CU,
    capped by LDS -- at k = 5, 6 one per CU, so B = 256 on 256 CUs is the limit.  The
    whole batch equals the oracle on a spread sample, the first and last gate
    included."""
    monkeypatch.delenv("MKACC_LAT", raising=False)
    monkeypatch.setenv("MKACC_QUAD", "0")
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, k, 2, 45181, 1 << 9, B, seed=300 + k)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, k, 2, 2048, Q_MK, 45181, 1 << 9))
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if cus != 256:
        pytest.skip(f"sized for 256 CUs, device has {cus}")
    assert eng.step_kernel_name(B) == "mk_lat_run_kernel"
    assert eng.step_kernel_name(B + 1) != "mk_lat_run_kernel"
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    pick = [0, 1, B // 2, B - 2, B - 1]
    exp = orc.evalacc_batch(evk, pkey, ct[pick], acc[pick], 8)
    assert np.array_equal(got[pick], exp.astype(np.uint32))


QUAD_CASES = [c for c in CASES]


@pytest.mark.parametrize("occ", ["1", "2", "3"])
@pytest.mark.parametrize("case", QUAD_CASES,
                         ids=[f"{c[0]}-k{c[1]}-n{c[2]}-logB{c[4].bit_length() - 1}" for c in QUAD_CASES])
def test_evalacc_quad_kernel(mk, oracle, case, occ, monkeypatch):
    """mk_quad_kernel (one gate per workgroup, every polynomial spread over its four
    waves, mkacc_quad.hpp; MKACC_QUAD=1) equals the oracle for both methods, k = 1..16,
    dg = 2..5, with the monomial edge cases c = 0, 2N - 1 (and 2N for XZW_B): the first
    step in its own launch, the others in one mk_quad_run_kernel launch.  occ "2": the
    two-workgroups-per-CU form; "3": the party-parallel form (a workgroup per party,
    mk_quadp_run_kernel; k = 1 keeps mk_quad_run_kernel), whose small n switches the
    index party every few steps and wraps the sv slot ring."""
    meth, k, n, q, baseG, B = case
    if occ == "2" and baseG == 1 << 5:
        pytest.skip("the two-workgroups-per-CU form is built for dg <= 4")
    monkeypatch.setenv("MKACC_QUAD", occ)   # "2": mk_quad2_kernel, tables in HBM, two workgroups per CU
    om = oracle.XZW if meth == "XZW" else oracle.XZW_B
    em = mk.MKNTRU if meth == "XZW" else mk.MKNTRU_LWE
    orc, evk, pkey, ct, acc = make_case(oracle, om, k, n, q, baseG, B + 2, seed=k * 41 + n)
    ct[0, 0, 0] = 0
    if om == oracle.XZW:
        ct[-1, k - 1, n - 1] = q - 1
    else:
        ct[-1, k - 1, n - 1] = 4096
        ct[0, 0, n - 1] = 4095
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8)
    eng = mk.MKAccumulatorEngine(mk.make_params(em, k, n, 2048, Q_MK, q, baseG))
    pre = {"2": "mk_quad2", "3": "mk_quadp" if k > 1 else "mk_quad"}.get(occ, "mk_quad")
    assert eng.step_kernel_name(B + 2) == (pre + "_run_kernel" if k * n > 1 else pre + "_kernel")
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    assert np.array_equal(got, exp.astype(np.uint32))


# the party-parallel form with several parties per workgroup (B > CUs / k): G = ceil(k /
# ceil(k / min(k, CUs / B))) workgroups per gate on a 256-CU MI355X
QUADP_GROUPED = [
    # method, k, n, q, baseG, B
    ("XZW", 8, 3, 45181, 1 << 6, 64),      # G = 4, two parties each (config 4 shape, dg = 4)
    ("XZW_B", 16, 2, 32749, 1 << 7, 40),   # G = 6: five workgroups of 3 parties, one of 1
    ("XZW", 5, 3, 45181, 1 << 9, 100),     # G = 2: 3 + 2 parties
    ("XZW_B", 4, 4, 32749, 1 << 9, 128),   # G = 2 (STD100_MKNTRU_LWE_2 shape)
    ("XZW", 2, 5, 45181, 1 << 7, 128),     # G = k = 2 at B = CUs / 2
    # two workgroups per CU (mk_quadp2_run_kernel, MKACC_QUAD=4, CUs / 2 < B <= CUs, dg <= 4)
    ("XZW", 8, 3, 45181, 1 << 6, 200),     # G = 2, four parties each, dg = 4 (one share per load)
    ("XZW_B", 4, 4, 32749, 1 << 9, 256),   # G = 2 at B = CUs
    ("XZW", 2, 5, 45181, 1 << 7, 256),     # G = 2 = k
    ("XZW", 3, 3, 45181, 1 << 5, 200),     # dg = 5: no two-per-CU form, one workgroup per gate
]


@pytest.mark.parametrize("case", QUADP_GROUPED, ids=[f"{c[0]}-k{c[1]}-n{c[2]}-B{c[5]}" for c in QUADP_GROUPED])
def test_evalacc_quadp_grouped(mk, oracle, case, monkeypatch):
    """mk_quadp_run_kernel (and above CUs / 2 gates mk_quadp2_run_kernel) where a workgroup owns several parties (its passes run one
    after the other, the index party's last, and it publishes one summed share): every
    gate of the batch equals the oracle; small n turns the index workgroup over every
    few steps, including turns shorter than the four-slot ring."""
    meth, k, n, q, baseG, B = case
    if B > 128:
        monkeypatch.setenv("MKACC_QUAD", "4")   # the two-per-CU form (opt-in)
    om = oracle.XZW if meth == "XZW" else oracle.XZW_B
    em = mk.MKNTRU if meth == "XZW" else mk.MKNTRU_LWE
    orc, evk, pkey, ct, acc = make_case(oracle, om, k, n, q, baseG, B, seed=k * 7 + n + B)
    ct[0, 0, 0] = 0
    ct[-1, k - 1, n - 1] = q - 1 if om == oracle.XZW else 4096
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8)
    eng = mk.MKAccumulatorEngine(mk.make_params(em, k, n, 2048, Q_MK, q, baseG))
    want = "mk_quadp_run_kernel" if B <= 128 else "mk_quadp2_run_kernel" if baseG > 1 << 5 else "mk_quad_run_kernel"
    assert eng.step_kernel_name(B) == want
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    bad = [b for b in range(B) if not np.array_equal(got[b], exp[b].astype(np.uint32))]
    assert not bad, bad[:8]


@pytest.mark.parametrize("name,B,occ", [("STD128_MKNTRU", 3, "1"), ("STD100_MKNTRU_LWE", 2, "1"),
                                        ("STD100_MKNTRU_LWE_2", 256, "1"), ("STD128_MKNTRU", 3, "3"),
                                        ("STD100_MKNTRU_LWE_2", 64, "3"), ("STD128_MKNTRU_3", 1, "3")])
def test_evalacc_quad_kernel_full_paramsets(mk, oracle, name, B, occ, monkeypatch):
    """The quad kernel at full n (1530 / 1000 / 2000 / 6120 steps in one launch), up to
    one gate per CU, against the oracle on a spread sample; occ "3" is the party-parallel
    form (B = 64 at k = 4: 256 workgroups, one on every CU)."""
    monkeypatch.setenv("MKACC_QUAD", occ)
    p = mk.paramset(name)
    om = oracle.XZW if p.method == mk.MKNTRU else oracle.XZW_B
    orc, evk, pkey, ct, acc = make_case(oracle, om, p.k, p.n, p.q, p.baseG, B, seed=p.n + B)
    acc[:] = orc.mntru_testvector(4)
    eng = mk.MKAccumulatorEngine(p)
    assert eng.step_kernel_name(B) == ("mk_quadp_run_kernel" if occ == "3" else "mk_quad_run_kernel")
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    pick = sorted({0, B // 2, B - 1})
    exp = orc.evalacc_batch(evk, pkey, ct[pick], acc[pick], 8)
    assert np.array_equal(got[pick], exp.astype(np.uint32))
