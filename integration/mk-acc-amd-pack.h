// mk-acc-amd-pack.h -- the conversions of the reference-side adapter
// (mk-acc-amd.h) between the reference's key / ciphertext objects and the
// engine's C-ABI buffers (include/mkfhe_amd.h), written once as templates over
// the access pattern the reference's types offer, so that:
//   * mk-acc-amd.h instantiates them with the reference's own types
//     (UniEncACCKeyImpl, NativePoly, NativeVector, ...; compiled against the
//     reference headers by tests/test_integration_adapter.py), and
//   * tests/cpp/adapter_pack.cpp instantiates them with stand-in types of the
//     same shape and EXECUTES them: every buffer is compared with the C-ABI
//     layout, and on an MI355X the packed buffers run through the engine and
//     are compared with the CPU oracle (tests/test_integration_adapter.py).
//
// No reference header is included here.  Accessors used (the reference's):
//   key table   K[u][j][i]  (UniEncACCKeyImpl::GetElements(), mk-acckey.h:44-51), an
//               UniEncEvalKey = shared_ptr<UniEncEvalKeyImpl> or null (mk-acc-xzw.cpp:66-80)
//   eval key    e->GetElements()[d][t]  ([dg][2] NativePoly, mk-evalkey.h:33-35)
//   polynomial  p[s].ConvertToInt<W>()  (PolyImpl::operator[], NativeInteger)
//   vector      v.GetLength(), v[i].ConvertToInt<W>()  (NativeVector)
// Errors go to `fail(message)`, which must not return (the adapter throws
// OPENFHE_THROW(config_error, ...), the test a std::runtime_error).
#ifndef MK_ACC_AMD_PACK_H
#define MK_ACC_AMD_PACK_H

#include <cstddef>
#include <cstdint>

namespace mkacc_pack {

// (*ek)[u][j][i] -> GetElements()[d][t][s]  into  evk [k][nk][n1][dg][2][N]
// (mkacc_upload_keys).  Entries the reference leaves empty ((*ek)[u][1][n], and
// (*ek)[u][0][n] for u > 0, mk-acc-xzw.cpp:66-80) are unused by EvalAcc: zeros.
template <class W, class KeyTable, class Fail>
void pack_evk(const KeyTable& K, uint32_t k, uint32_t nk, uint32_t n1, uint32_t dg, uint32_t N, W* evk,
              const Fail& fail) {
    if (K.size() != k) fail("bootstrapping key has the wrong number of parties");
    size_t o = 0;
    for (uint32_t u = 0; u < k; ++u) {
        if (K[u].size() < nk) fail("bootstrapping key has the wrong shape");
        for (uint32_t j = 0; j < nk; ++j) {
            if (K[u][j].size() != n1) fail("bootstrapping key has the wrong dimension");
            for (uint32_t i = 0; i < n1; ++i) {
                const auto& e = K[u][j][i];
                if (e == nullptr) {
                    for (size_t s = 0; s < size_t(dg) * 2 * N; ++s) evk[o + s] = W(0);
                    o += size_t(dg) * 2 * N;
                    continue;
                }
                const auto& el = e->GetElements();
                if (el.size() != dg) fail("bootstrapping key has the wrong number of digits");
                for (uint32_t d = 0; d < dg; ++d) {
                    if (el[d].size() != 2) fail("bootstrapping key digit is not a (d, f) pair");
                    for (uint32_t t = 0; t < 2; ++t, o += N) {
                        if (el[d][t].GetLength() != N) fail("bootstrapping key polynomial has the wrong length");
                        for (uint32_t s = 0; s < N; ++s) evk[o + s] = el[d][t][s].template ConvertToInt<W>();
                    }
                }
            }
        }
    }
}

// Pkey[u][d][s]  into  pkey [k][dg][N]
template <class W, class PkeyT, class Fail>
void pack_pkey(const PkeyT& Pkey, uint32_t k, uint32_t dg, uint32_t N, W* pk, const Fail& fail) {
    if (Pkey.size() != k) fail("Pkey has the wrong number of parties");
    for (uint32_t u = 0; u < k; ++u) {
        if (Pkey[u].size() < dg) fail("Pkey has the wrong number of digits");
        for (uint32_t d = 0; d < dg; ++d) {
            if (Pkey[u][d].GetLength() != N) fail("Pkey polynomial has the wrong length");
            for (uint32_t s = 0; s < N; ++s) pk[(size_t(u) * dg + d) * N + s] = Pkey[u][d][s].template ConvertToInt<W>();
        }
    }
}

// MK-NTRU KeySwitch2 key: the engine takes KSK2[u][1] ([k][N dks][n], mkacc_upload_ksk_mntru);
// KeySwitchGen2 stores KSK2[u][j] = j KSK2[u][1] mod qKS, [k][baseKS][N dks][n] (mntru-pke.cpp:740-755).
template <class KSK2Elems, class Fail>
void pack_ksk2(const KSK2Elems& E, uint32_t k, uint32_t N, uint32_t dks, uint32_t n, uint32_t* w, const Fail& fail) {
    if (E.size() != k) fail("KeySwitch2 key has the wrong number of parties");
    for (uint32_t u = 0; u < k; ++u) {
        if (E[u].size() < 2 || E[u][1].size() != size_t(N) * dks) fail("KeySwitch2 key has the wrong shape");
        for (size_t l = 0; l < size_t(N) * dks; ++l) {
            if (E[u][1][l].GetLength() != n) fail("KeySwitch2 key row has the wrong length");
            for (uint32_t i = 0; i < n; ++i)
                w[(u * size_t(N) * dks + l) * n + i] = E[u][1][l][i].template ConvertToInt<uint32_t>();
        }
    }
}

// MK-LWE KeySwitch key (mklwe-pke.cpp:176-258): A [k][N][baseKS][dks] vectors of n, B [k][N][baseKS][dks]
// into wa [k][N][baseKS][dks][n], wb [k][N][baseKS][dks] (mkacc_upload_ksk_mklwe)
template <class AT, class BT, class Fail>
void pack_lwe_ksk(const AT& A, const BT& Bk, uint32_t k, uint32_t N, uint32_t base, uint32_t dks, uint32_t n,
                  uint32_t* wa, uint32_t* wb, const Fail& fail) {
    if (A.size() != k || Bk.size() != k) fail("key-switching key has the wrong number of parties");
    for (uint32_t u = 0; u < k; ++u) {
        if (A[u].size() != N || Bk[u].size() != N) fail("key-switching key has the wrong dimension");
        for (uint32_t i = 0; i < N; ++i) {
            if (A[u][i].size() != base || Bk[u][i].size() != base) fail("key-switching key has the wrong base");
            for (uint32_t a = 0; a < base; ++a) {
                if (A[u][i][a].size() != dks || Bk[u][i][a].size() != dks)
                    fail("key-switching key has the wrong number of digits");
                for (uint32_t j = 0; j < dks; ++j) {
                    const size_t r = ((size_t(u) * N + i) * base + a) * dks + j;
                    wb[r] = Bk[u][i][a][j].template ConvertToInt<uint32_t>();
                    if (A[u][i][a][j].GetLength() != n) fail("key-switching key row has the wrong length");
                    for (uint32_t l = 0; l < n; ++l) wa[r * n + l] = A[u][i][a][j][l].template ConvertToInt<uint32_t>();
                }
            }
        }
    }
}

// k vectors of n words (an MNTRU ciphertext's GetElements(), an MK-LWE ciphertext's GetA(),
// an EvalAcc input ct) into dst [k][n]
template <class Vecs, class Fail>
void pack_vectors(const Vecs& v, uint32_t k, uint32_t n, uint32_t* dst, const Fail& fail) {
    if (v.size() != k) fail("ciphertext has the wrong number of parties");
    for (uint32_t u = 0; u < k; ++u) {
        if (v[u].GetLength() != n) fail("ciphertext has the wrong dimension");
        for (uint32_t i = 0; i < n; ++i) dst[size_t(u) * n + i] = v[u][i].template ConvertToInt<uint32_t>();
    }
}

// one polynomial of N words (an accumulator row, EVALUATION order) into dst [N]
template <class W, class Poly, class Fail>
void pack_poly(const Poly& p, uint32_t N, W* dst, const Fail& fail) {
    if (p.GetLength() != N) fail("polynomial has the wrong length");
    for (uint32_t j = 0; j < N; ++j) dst[j] = p[j].template ConvertToInt<W>();
}

}  // namespace mkacc_pack

#endif  // MK_ACC_AMD_PACK_H
