"""Property tests of the oracle restatement (no reference vector covers these;
they mirror the reference's own property-style tests, UnitTestNTT.cpp:84,131)."""
import numpy as np
import pytest

Q = 134176769


def schoolbook_negacyclic(a, b, q):
    n = len(a)
    out = [0] * n
    for i in range(n):
        for j in range(n):
            k = i + j
            if k < n:
                out[k] = (out[k] + a[i] * b[j]) % q
            else:
                out[k - n] = (out[k - n] - a[i] * b[j]) % q
    return out


def test_ntt_roundtrip_2048(oracle):
    psi = oracle.root_of_unity(4096, Q)
    a = oracle.fill_uniform(2048, Q, 11)
    assert np.array_equal(oracle.ntt_inverse(oracle.ntt_forward(a, Q, psi), Q, psi), a)


def test_ntt_is_negacyclic_convolution(oracle):
    N = 64
    psi = oracle.root_of_unity(2 * N, Q)
    a = oracle.fill_uniform(N, Q, 5)
    b = oracle.fill_uniform(N, Q, 6)
    A = oracle.ntt_forward(a, Q, psi)
    B = oracle.ntt_forward(b, Q, psi)
    prod = np.array([(int(x) * int(y)) % Q for x, y in zip(A, B)], dtype=np.uint64)
    got = oracle.ntt_inverse(prod, Q, psi)
    assert list(got) == schoolbook_negacyclic([int(x) for x in a], [int(x) for x in b], Q)


def test_ntt_eval_points(oracle):
    # EVAL slot j holds a(psi^(2*brv(j)+1)) (transformnat-impl.h:705-760)
    N = 16
    psi = oracle.root_of_unity(2 * N, Q)
    a = [int(x) for x in oracle.fill_uniform(N, Q, 9)]
    A = oracle.ntt_forward(a, Q, psi)
    for j in range(N):
        rj = int(format(j, "04b")[::-1], 2)
        x = pow(psi, 2 * rj + 1, Q)
        assert int(A[j]) == sum(c * pow(x, i, Q) for i, c in enumerate(a)) % Q


@pytest.mark.parametrize("logB,dg", [(9, 2), (7, 3), (6, 4), (5, 5)])
def test_sdd_reconstruction(oracle, logB, dg):
    """c = r0 + sum_i digit_i * B^(i+1) + B^(dg+1) * carry, with r0 the dropped
    low digit (mk-acc.cpp:63-66) and |digit| <= B/2 (approximate gadget)."""
    B = 1 << logB
    x = oracle.fill_uniform(2048, Q, 21 + logB)
    dig = oracle.sdd(x, Q, B, dg)
    for t in range(2048):
        v = int(x[t])
        c = v if v < Q // 2 else v - Q
        low = c & (B - 1)
        r0 = low - B if low >= B // 2 else low
        s = 0
        for i in range(dg):
            d = int(dig[i, t])
            d = d if d < Q // 2 else d - Q
            assert -B // 2 <= d < B // 2
            s += d * B ** (i + 1)
        assert (c - r0 - s) % (B ** (dg + 1)) == 0


def test_evalacc_deterministic_and_input_sensitive(oracle):
    from conftest import make_case
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW, 2, 3, 45181, 1 << 9, 2, seed=1)
    a0 = orc.evalacc(evk, pkey, ct[0], acc[0])
    a1 = orc.evalacc(evk, pkey, ct[0], acc[0])
    assert np.array_equal(a0, a1)
    ct2 = ct[0].copy()
    ct2[1, 2] = (ct2[1, 2] + 1000) % 45181
    assert not np.array_equal(a0, orc.evalacc(evk, pkey, ct2, acc[0]))
    # batch entry point == per-gate calls
    ab = orc.evalacc_batch(evk, pkey, ct, acc, 2)
    assert np.array_equal(ab[0], a0)
    assert np.array_equal(ab[1], orc.evalacc(evk, pkey, ct[1], acc[1]))


def test_evalacc_zero_keys_zero_output(oracle):
    # HbProd with all-zero keys and P gives acc <- 0 at the first (KDM) step and
    # acc + 0 afterwards, so the result is 0
    from conftest import make_case
    orc, evk, pkey, ct, acc = make_case(oracle, oracle.XZW_B, 2, 2, 32749, 1 << 9, 1, seed=2)
    out = orc.evalacc(np.zeros_like(evk), np.zeros_like(pkey), ct[0], acc[0])
    assert not out.any()
