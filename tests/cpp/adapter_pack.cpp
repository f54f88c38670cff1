// Executes the reference-side adapter's conversions (integration/mk-acc-amd-pack.h,
// instantiated by integration/mk-acc-amd.h with the reference's own types) on
// stand-in types that offer the same accessors as the reference's
// UniEncACCKeyImpl / UniEncEvalKeyImpl / NativePoly / NativeVector /
// NativeInteger (mk-acckey.h:44-90, mk-evalkey.h:33-60, lat-backend.h:51) and
// the key-switching keys (mntru-keyswitchkey2.h:26, mklwe-keyswitchkey.h:28-29).
//
//   adapter_pack layout   (CPU) every packed buffer equals the C-ABI layout of
//                         include/mkfhe_amd.h, written out index by index here, and
//                         every shape error reaches the adapter's error path
//   adapter_pack engine   (MI355X) keys, ciphertexts and accumulators held in
//                         reference-shaped objects go through the packers into the
//                         engine (EvalAcc for XZW and XZW_B, whole MK-NTRU and MK-LWE
//                         NAND gates) and come out equal to the CPU oracle (oracle/,
//                         the checker) run on buffers this file lays out itself.
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mk-acc-amd-pack.h"
#include "mkfhe_amd.h"
#include "mkfhe_oracle.h"

namespace {

// ---- stand-ins: the reference's accessors, nothing else ---------------------------
struct Int {   // NativeInteger
    uint64_t v = 0;
    template <class T>
    T ConvertToInt() const {
        return static_cast<T>(v);
    }
};
struct Vec {   // NativeVector / NativePoly: GetLength(), operator[] -> Int
    std::vector<Int> w;
    uint32_t GetLength() const { return static_cast<uint32_t>(w.size()); }
    const Int& operator[](size_t i) const { return w[i]; }
};
struct EvalKey {   // UniEncEvalKeyImpl: [dg][2] polynomials
    std::vector<std::vector<Vec>> el;
    const std::vector<std::vector<Vec>>& GetElements() const { return el; }
};
using KeyTable = std::vector<std::vector<std::vector<std::shared_ptr<EvalKey>>>>;   // [k][nk][n+1]

int g_fail = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);        \
            ++g_fail;                                                       \
        }                                                                   \
    } while (0)

struct PackError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
const auto fail = [](const char* m) { throw PackError(m); };

Vec vec_from(const uint64_t* p, size_t n) {
    Vec v;
    v.w.resize(n);
    for (size_t i = 0; i < n; ++i) v.w[i].v = p[i];
    return v;
}

// A bootstrapping key in the reference's object form whose words are `flat`, the
// C-ABI layout [k][nk][n+1][dg][2][N] -- built from the reference's semantics
// ((*ek)[u][j][i] -> digit d -> (d_i, f_i) t); entries the reference leaves empty are
// null (and zeroed in `flat`).
KeyTable key_table(std::vector<uint64_t>& flat, uint32_t k, uint32_t nk, uint32_t n, uint32_t dg, uint32_t N) {
    KeyTable K(k, std::vector<std::vector<std::shared_ptr<EvalKey>>>(nk, std::vector<std::shared_ptr<EvalKey>>(n + 1)));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < nk; ++j)
            for (uint32_t i = 0; i <= n; ++i) {
                const size_t base = ((size_t(u) * nk + j) * (n + 1) + i) * dg * 2 * N;
                if (i == n && (j == 1 || u > 0)) {   // mk-acc-xzw.cpp:66-80: only (*ek)[0][0][n] is the KDM key
                    std::memset(flat.data() + base, 0, size_t(dg) * 2 * N * 8);
                    continue;
                }
                auto e = std::make_shared<EvalKey>();
                e->el.assign(dg, std::vector<Vec>(2));
                for (uint32_t d = 0; d < dg; ++d)
                    for (uint32_t t = 0; t < 2; ++t) e->el[d][t] = vec_from(flat.data() + base + (size_t(d) * 2 + t) * N, N);
                K[u][j][i] = e;
            }
    return K;
}

template <class F>
bool throws(F f) {
    try {
        f();
    } catch (const PackError&) {
        return true;
    }
    return false;
}

// ---- layout (CPU) -----------------------------------------------------------------
void layout() {
    const uint32_t k = 3, nk = 2, n = 4, dg = 3, N = 16;
    // every word encodes its own reference indices, so a permuted pack shows up
    auto word = [](uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e, uint64_t f) {
        return ((((a * 8 + b) * 64 + c) * 8 + d) * 4 + e) * 4096 + f + 1;
    };
    KeyTable K(k, std::vector<std::vector<std::shared_ptr<EvalKey>>>(nk, std::vector<std::shared_ptr<EvalKey>>(n + 1)));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < nk; ++j)
            for (uint32_t i = 0; i <= n; ++i) {
                if (i == n && (j == 1 || u > 0)) continue;
                auto e = std::make_shared<EvalKey>();
                e->el.assign(dg, std::vector<Vec>(2));
                for (uint32_t d = 0; d < dg; ++d)
                    for (uint32_t t = 0; t < 2; ++t) {
                        e->el[d][t].w.resize(N);
                        for (uint32_t s = 0; s < N; ++s) e->el[d][t].w[s].v = word(u, j, i, d, t, s);
                    }
                K[u][j][i] = e;
            }
    std::vector<uint64_t> evk(size_t(k) * nk * (n + 1) * dg * 2 * N, 7);
    mkacc_pack::pack_evk(K, k, nk, n + 1, dg, N, evk.data(), fail);
    size_t bad = 0;
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < nk; ++j)
            for (uint32_t i = 0; i <= n; ++i)
                for (uint32_t d = 0; d < dg; ++d)
                    for (uint32_t t = 0; t < 2; ++t)
                        for (uint32_t s = 0; s < N; ++s) {
                            const uint64_t want = (i == n && (j == 1 || u > 0)) ? 0 : word(u, j, i, d, t, s);
                            bad += evk[(((((size_t(u) * nk + j) * (n + 1) + i) * dg + d) * 2 + t) * N) + s] != want;
                        }
    CHECK(bad == 0);

    // P [k][dg][N]
    std::vector<std::vector<Vec>> P(k, std::vector<Vec>(dg));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t d = 0; d < dg; ++d) {
            P[u][d].w.resize(N);
            for (uint32_t s = 0; s < N; ++s) P[u][d].w[s].v = word(u, 0, 0, d, 0, s);
        }
    std::vector<uint32_t> pk(size_t(k) * dg * N);
    mkacc_pack::pack_pkey(P, k, dg, N, pk.data(), fail);
    bad = 0;
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t d = 0; d < dg; ++d)
            for (uint32_t s = 0; s < N; ++s) bad += pk[(size_t(u) * dg + d) * N + s] != uint32_t(word(u, 0, 0, d, 0, s));
    CHECK(bad == 0);

    // KSK2 [k][baseKS][N dks][n] -> its j = 1 rows
    const uint32_t base = 4, dks = 2;
    std::vector<std::vector<std::vector<Vec>>> E(k, std::vector<std::vector<Vec>>(base, std::vector<Vec>(N * dks)));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < base; ++j)
            for (uint32_t l = 0; l < N * dks; ++l) {
                E[u][j][l].w.resize(n);
                for (uint32_t i = 0; i < n; ++i) E[u][j][l].w[i].v = word(u, j, l, i, 0, 0) & 0xFFFFFFFFu;
            }
    std::vector<uint32_t> w(size_t(k) * N * dks * n);
    mkacc_pack::pack_ksk2(E, k, N, dks, n, w.data(), fail);
    bad = 0;
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t l = 0; l < N * dks; ++l)
            for (uint32_t i = 0; i < n; ++i) bad += w[(size_t(u) * N * dks + l) * n + i] != uint32_t(word(u, 1, l, i, 0, 0));
    CHECK(bad == 0);

    // MK-LWE KSK: A [k][N][base][dks](n), B [k][N][base][dks]
    std::vector<std::vector<std::vector<std::vector<Vec>>>> A(
        k, std::vector<std::vector<std::vector<Vec>>>(N, std::vector<std::vector<Vec>>(base, std::vector<Vec>(dks))));
    std::vector<std::vector<std::vector<std::vector<Int>>>> Bk(
        k, std::vector<std::vector<std::vector<Int>>>(N, std::vector<std::vector<Int>>(base, std::vector<Int>(dks))));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t i = 0; i < N; ++i)
            for (uint32_t a = 0; a < base; ++a)
                for (uint32_t j = 0; j < dks; ++j) {
                    Bk[u][i][a][j].v = word(u, i, a, j, 3, 0) & 0xFFFFFFFFu;
                    A[u][i][a][j].w.resize(n);
                    for (uint32_t l = 0; l < n; ++l) A[u][i][a][j].w[l].v = word(u, i, a, j, 2, l) & 0xFFFFFFFFu;
                }
    std::vector<uint32_t> wa(size_t(k) * N * base * dks * n), wb(size_t(k) * N * base * dks);
    mkacc_pack::pack_lwe_ksk(A, Bk, k, N, base, dks, n, wa.data(), wb.data(), fail);
    bad = 0;
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t i = 0; i < N; ++i)
            for (uint32_t a = 0; a < base; ++a)
                for (uint32_t j = 0; j < dks; ++j) {
                    const size_t r = ((size_t(u) * N + i) * base + a) * dks + j;
                    bad += wb[r] != uint32_t(word(u, i, a, j, 3, 0));
                    for (uint32_t l = 0; l < n; ++l) bad += wa[r * n + l] != uint32_t(word(u, i, a, j, 2, l));
                }
    CHECK(bad == 0);

    // ciphertexts [k][n], polynomials [N]
    std::vector<Vec> ct(k);
    for (uint32_t u = 0; u < k; ++u) {
        ct[u].w.resize(n);
        for (uint32_t i = 0; i < n; ++i) ct[u].w[i].v = 100 * u + i;
    }
    std::vector<uint32_t> c(size_t(k) * n);
    mkacc_pack::pack_vectors(ct, k, n, c.data(), fail);
    bad = 0;
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t i = 0; i < n; ++i) bad += c[size_t(u) * n + i] != 100 * u + i;
    CHECK(bad == 0);
    std::vector<uint64_t> row(N);
    mkacc_pack::pack_poly(P[1][2], N, row.data(), fail);
    CHECK(row[5] == word(1, 0, 0, 2, 0, 5));

    // every shape error takes the error path (the adapter's OPENFHE_THROW(config_error))
    std::vector<uint64_t> sink(evk.size());
    KeyTable K2 = K;
    K2.pop_back();
    CHECK(throws([&] { mkacc_pack::pack_evk(K2, k, nk, n + 1, dg, N, sink.data(), fail); }));
    K2 = K;
    K2[1][0].pop_back();
    CHECK(throws([&] { mkacc_pack::pack_evk(K2, k, nk, n + 1, dg, N, sink.data(), fail); }));
    K2 = K;
    {
        auto e = std::make_shared<EvalKey>(*K2[2][1][3]);
        e->el.pop_back();
        K2[2][1][3] = e;
    }
    CHECK(throws([&] { mkacc_pack::pack_evk(K2, k, nk, n + 1, dg, N, sink.data(), fail); }));
    K2 = K;
    {
        auto e = std::make_shared<EvalKey>(*K2[0][0][0]);
        e->el[1][1].w.pop_back();
        K2[0][0][0] = e;
    }
    CHECK(throws([&] { mkacc_pack::pack_evk(K2, k, nk, n + 1, dg, N, sink.data(), fail); }));
    auto P2 = P;
    P2[2].pop_back();
    CHECK(throws([&] { mkacc_pack::pack_pkey(P2, k, dg, N, pk.data(), fail); }));
    auto E2 = E;
    E2[1][1].pop_back();
    CHECK(throws([&] { mkacc_pack::pack_ksk2(E2, k, N, dks, n, w.data(), fail); }));
    auto A2 = A;
    A2[0][3][1][0].w.pop_back();
    CHECK(throws([&] { mkacc_pack::pack_lwe_ksk(A2, Bk, k, N, base, dks, n, wa.data(), wb.data(), fail); }));
    auto ct2 = ct;
    ct2[1].w.pop_back();
    CHECK(throws([&] { mkacc_pack::pack_vectors(ct2, k, n, c.data(), fail); }));
    CHECK(throws([&] { mkacc_pack::pack_vectors(ct, k + 1, n, c.data(), fail); }));
}

// ---- engine vs oracle (MI355X) -----------------------------------------------------
constexpr uint64_t kQ = 134176769;
constexpr uint32_t kN = 2048;

bool engine_ok(int rc, const char* what) {
    if (rc == MKACC_OK) return true;
    std::printf("FAIL %s: %d %s\n", what, rc, mkacc_last_error());
    ++g_fail;
    return false;
}

// EvalAcc of B gates through the packers, against the oracle on the flat layout
void engine_evalacc(uint32_t method, uint32_t k, uint32_t n, uint64_t q, uint32_t logB, uint64_t seed) {
    const uint32_t nk = method == MKACC_METHOD_MKNTRU ? 2 : 1;
    orc_params op{method == MKACC_METHOD_MKNTRU ? (uint32_t)ORC_XZW : (uint32_t)ORC_XZW_B, k, n, kN, kQ,
                  method == MKACC_METHOD_MKNTRU ? q : 2 * kN, 1u << logB, orc_digits_g(kQ, 1u << logB),
                  orc_root_of_unity(2 * kN, kQ)};
    const uint32_t dg = op.digitsG - 1;
    orc_ctx* oc = orc_ctx_create(&op);
    std::vector<uint64_t> evk(orc_evk_words(&op)), pkey(size_t(k) * dg * kN);
    orc_fill_uniform(evk.data(), evk.size(), kQ, seed);
    orc_fill_uniform(pkey.data(), pkey.size(), kQ, seed + 1);
    const KeyTable K = key_table(evk, k, nk, n, dg, kN);   // zeroes the unused entries in evk
    std::vector<std::vector<Vec>> P(k, std::vector<Vec>(dg));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t d = 0; d < dg; ++d) P[u][d] = vec_from(pkey.data() + (size_t(u) * dg + d) * kN, kN);
    const size_t B = 3;
    std::vector<uint64_t> ct(B * k * n), acc(B * k * kN);
    orc_fill_uniform(ct.data(), ct.size(), method == MKACC_METHOD_MKNTRU ? q : 2 * kN, seed + 2);
    orc_fill_uniform(acc.data(), acc.size(), kQ, seed + 3);

    // the adapter's side: reference-shaped objects -> packers -> engine
    std::vector<uint32_t> evk_p(evk.size()), pkey_p(pkey.size()), ct_p(ct.size()), acc_p(acc.size());
    mkacc_pack::pack_evk(K, k, nk, n + 1, dg, kN, evk_p.data(), fail);
    mkacc_pack::pack_pkey(P, k, dg, kN, pkey_p.data(), fail);
    for (size_t b = 0; b < B; ++b) {
        std::vector<Vec> cv(k);
        for (uint32_t u = 0; u < k; ++u) {
            cv[u] = vec_from(ct.data() + (b * k + u) * n, n);
            mkacc_pack::pack_poly(vec_from(acc.data() + (b * k + u) * kN, kN), kN, acc_p.data() + (b * k + u) * kN, fail);
        }
        mkacc_pack::pack_vectors(cv, k, n, ct_p.data() + b * k * n, fail);
    }
    mkacc_params p{method, k, n, kN, kQ, q, 1u << logB, op.digitsG, op.psi};
    mkacc_ctx* c = nullptr;
    if (engine_ok(mkacc_create(&p, 0, &c), "mkacc_create") && engine_ok(mkacc_upload_keys(c, evk_p.data(), pkey_p.data()), "upload") &&
        engine_ok(mkacc_eval_batch(c, ct_p.data(), acc_p.data(), acc_p.data(), B), "eval")) {
        orc_evalacc_batch(oc, evk.data(), pkey.data(), ct.data(), acc.data(), B, 4);
        size_t bad = 0;
        for (size_t s = 0; s < acc.size(); ++s) bad += acc_p[s] != acc[s];
        std::printf("evalacc method %u k %u: %zu of %zu words differ\n", method, k, bad, acc.size());
        CHECK(bad == 0);
    }
    mkacc_destroy(c);
    orc_ctx_destroy(oc);
}

// whole MK-NTRU NAND gates: KSK2 in its reference form [k][baseKS][N dks][n], KSK2[u][j] = j KSK2[u][1]
void engine_nand_mntru(uint32_t k, uint32_t n, uint64_t seed) {
    const uint64_t q = 45181, qKS = 45181;
    const uint32_t baseKS = 32, logB = 7;
    orc_params op{ORC_XZW, k, n, kN, kQ, q, 1u << logB, orc_digits_g(kQ, 1u << logB), orc_root_of_unity(2 * kN, kQ)};
    const uint32_t dg = op.digitsG - 1, dks = orc_ks_digits(qKS, baseKS);
    orc_ctx* oc = orc_ctx_create(&op);
    std::vector<uint64_t> evk(orc_evk_words(&op)), pkey(size_t(k) * dg * kN);
    orc_fill_uniform(evk.data(), evk.size(), kQ, seed);
    orc_fill_uniform(pkey.data(), pkey.size(), kQ, seed + 1);
    const KeyTable K = key_table(evk, k, 2, n, dg, kN);
    std::vector<std::vector<Vec>> P(k, std::vector<Vec>(dg));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t d = 0; d < dg; ++d) P[u][d] = vec_from(pkey.data() + (size_t(u) * dg + d) * kN, kN);
    std::vector<uint32_t> ksk1(size_t(k) * kN * dks * n);
    orc_fill_uniform_u32(ksk1.data(), ksk1.size(), qKS, seed + 2);
    std::vector<std::vector<std::vector<Vec>>> E(k, std::vector<std::vector<Vec>>(baseKS, std::vector<Vec>(kN * dks)));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < baseKS; ++j)
            for (uint32_t l = 0; l < kN * dks; ++l) {
                E[u][j][l].w.resize(n);
                for (uint32_t i = 0; i < n; ++i)
                    E[u][j][l].w[i].v = j * uint64_t(ksk1[(size_t(u) * kN * dks + l) * n + i]) % qKS;
            }
    const size_t B = 2;
    std::vector<uint64_t> nand(size_t(k) * n), c1(B * k * n), c2(B * k * n);
    orc_fill_uniform(nand.data(), nand.size(), q, seed + 3);
    orc_fill_uniform(c1.data(), c1.size(), q, seed + 4);
    orc_fill_uniform(c2.data(), c2.size(), q, seed + 5);

    std::vector<uint32_t> evk_p(evk.size()), pkey_p(pkey.size()), w(ksk1.size()), nand_p(nand.size()),
        a1(c1.size()), a2(c2.size()), out(B * k * n);
    mkacc_pack::pack_evk(K, k, 2, n + 1, dg, kN, evk_p.data(), fail);
    mkacc_pack::pack_pkey(P, k, dg, kN, pkey_p.data(), fail);
    mkacc_pack::pack_ksk2(E, k, kN, dks, n, w.data(), fail);
    auto as_vecs = [&](const uint64_t* src) {
        std::vector<Vec> v(k);
        for (uint32_t u = 0; u < k; ++u) v[u] = vec_from(src + size_t(u) * n, n);
        return v;
    };
    mkacc_pack::pack_vectors(as_vecs(nand.data()), k, n, nand_p.data(), fail);
    for (size_t b = 0; b < B; ++b) {
        mkacc_pack::pack_vectors(as_vecs(c1.data() + b * k * n), k, n, a1.data() + b * k * n, fail);
        mkacc_pack::pack_vectors(as_vecs(c2.data() + b * k * n), k, n, a2.data() + b * k * n, fail);
    }
    mkacc_params p{MKACC_METHOD_MKNTRU, k, n, kN, kQ, q, 1u << logB, op.digitsG, op.psi};
    const mkacc_ks_params ks{qKS, baseKS, n};
    mkacc_ctx* c = nullptr;
    if (engine_ok(mkacc_create(&p, 0, &c), "mkacc_create") && engine_ok(mkacc_upload_keys(c, evk_p.data(), pkey_p.data()), "upload") &&
        engine_ok(mkacc_upload_ksk_mntru(c, &ks, w.data()), "ksk") &&
        engine_ok(mkacc_eval_nand_mntru(c, nand_p.data(), a1.data(), a2.data(), out.data(), B), "nand")) {
        size_t bad = 0;
        std::vector<uint64_t> head(size_t(k) * n), acc(size_t(k) * kN), res(size_t(k) * n);
        for (size_t b = 0; b < B; ++b) {
            orc_mntru_head(nand.data(), c1.data() + b * k * n, c2.data() + b * k * n, head.data(), k, n, q);
            orc_mntru_testvector(oc, 4, acc.data());
            orc_evalacc(oc, evk.data(), pkey.data(), head.data(), acc.data());
            orc_mntru_tail_ksk1(oc, acc.data(), ksk1.data(), qKS, baseKS, n, res.data());
            for (size_t s = 0; s < res.size(); ++s) bad += out[b * k * n + s] != res[s];
        }
        std::printf("nand mntru k %u: %zu of %zu words differ\n", k, bad, out.size());
        CHECK(bad == 0);
    }
    mkacc_destroy(c);
    orc_ctx_destroy(oc);
}

// whole MK-LWE NAND gates: KSK in its reference form A [k][N][baseKS][dks](n), B [k][N][baseKS][dks]
void engine_nand_mklwe(uint32_t k, uint32_t n, uint64_t seed) {
    const uint64_t q = 32749, qKS = 32749;
    const uint32_t baseKS = 32, logB = 9;
    orc_params op{ORC_XZW_B, k, n, kN, kQ, 2 * kN, 1u << logB, orc_digits_g(kQ, 1u << logB), orc_root_of_unity(2 * kN, kQ)};
    const uint32_t dg = op.digitsG - 1, dks = orc_ks_digits(qKS, baseKS);
    orc_ctx* oc = orc_ctx_create(&op);
    std::vector<uint64_t> evk(orc_evk_words(&op)), pkey(size_t(k) * dg * kN);
    orc_fill_uniform(evk.data(), evk.size(), kQ, seed);
    orc_fill_uniform(pkey.data(), pkey.size(), kQ, seed + 1);
    const KeyTable K = key_table(evk, k, 1, n, dg, kN);
    std::vector<std::vector<Vec>> P(k, std::vector<Vec>(dg));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t d = 0; d < dg; ++d) P[u][d] = vec_from(pkey.data() + (size_t(u) * dg + d) * kN, kN);
    const size_t rows = size_t(k) * kN * baseKS * dks;
    std::vector<uint64_t> A(rows * n), Bf(rows);
    orc_fill_uniform(A.data(), A.size(), qKS, seed + 2);
    orc_fill_uniform(Bf.data(), Bf.size(), qKS, seed + 3);
    std::vector<std::vector<std::vector<std::vector<Vec>>>> Ao(
        k, std::vector<std::vector<std::vector<Vec>>>(kN, std::vector<std::vector<Vec>>(baseKS, std::vector<Vec>(dks))));
    std::vector<std::vector<std::vector<std::vector<Int>>>> Bo(
        k, std::vector<std::vector<std::vector<Int>>>(kN, std::vector<std::vector<Int>>(baseKS, std::vector<Int>(dks))));
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t i = 0; i < kN; ++i)
            for (uint32_t a = 0; a < baseKS; ++a)
                for (uint32_t j = 0; j < dks; ++j) {
                    const size_t r = ((size_t(u) * kN + i) * baseKS + a) * dks + j;
                    Ao[u][i][a][j] = vec_from(A.data() + r * n, n);
                    Bo[u][i][a][j].v = Bf[r];
                }
    const size_t B = 2;
    std::vector<uint64_t> a1(B * k * n), a2(B * k * n), b1(B), b2(B);
    orc_fill_uniform(a1.data(), a1.size(), q, seed + 4);
    orc_fill_uniform(a2.data(), a2.size(), q, seed + 5);
    orc_fill_uniform(b1.data(), B, q, seed + 6);
    orc_fill_uniform(b2.data(), B, q, seed + 7);

    std::vector<uint32_t> evk_p(evk.size()), pkey_p(pkey.size()), wa(A.size()), wb(Bf.size()), a1p(a1.size()),
        a2p(a2.size()), b1p(B), b2p(B), oa(B * k * n), ob(B);
    mkacc_pack::pack_evk(K, k, 1, n + 1, dg, kN, evk_p.data(), fail);
    mkacc_pack::pack_pkey(P, k, dg, kN, pkey_p.data(), fail);
    mkacc_pack::pack_lwe_ksk(Ao, Bo, k, kN, baseKS, dks, n, wa.data(), wb.data(), fail);
    for (size_t b = 0; b < B; ++b) {
        std::vector<Vec> v1(k), v2(k);
        for (uint32_t u = 0; u < k; ++u) {
            v1[u] = vec_from(a1.data() + (b * k + u) * n, n);
            v2[u] = vec_from(a2.data() + (b * k + u) * n, n);
        }
        mkacc_pack::pack_vectors(v1, k, n, a1p.data() + b * k * n, fail);
        mkacc_pack::pack_vectors(v2, k, n, a2p.data() + b * k * n, fail);
        b1p[b] = uint32_t(b1[b]);
        b2p[b] = uint32_t(b2[b]);
    }
    mkacc_params p{MKACC_METHOD_MKNTRU_LWE, k, n, kN, kQ, q, 1u << logB, op.digitsG, op.psi};
    const mkacc_ks_params ks{qKS, baseKS, n};
    mkacc_ctx* c = nullptr;
    if (engine_ok(mkacc_create(&p, 0, &c), "mkacc_create") && engine_ok(mkacc_upload_keys(c, evk_p.data(), pkey_p.data()), "upload") &&
        engine_ok(mkacc_upload_ksk_mklwe(c, &ks, wa.data(), wb.data()), "ksk") &&
        engine_ok(mkacc_eval_nand_mklwe(c, a1p.data(), b1p.data(), a2p.data(), b2p.data(), oa.data(), ob.data(), B), "nand")) {
        size_t bad = 0;
        std::vector<uint64_t> cc(size_t(k) * n), acc(size_t(k) * kN), ra(size_t(k) * n);
        for (size_t b = 0; b < B; ++b) {
            orc_mklwe_head(oc, a1.data() + b * k * n, b1[b], a2.data() + b * k * n, b2[b], q, n, 4, cc.data(), acc.data());
            orc_evalacc(oc, evk.data(), pkey.data(), cc.data(), acc.data());
            uint64_t rb = 0;
            orc_mklwe_tail(oc, acc.data(), A.data(), Bf.data(), qKS, baseKS, n, ra.data(), &rb);
            for (size_t s = 0; s < ra.size(); ++s) bad += oa[b * k * n + s] != ra[s];
            bad += ob[b] != rb;
        }
        std::printf("nand mklwe k %u: %zu words differ\n", k, bad);
        CHECK(bad == 0);
    }
    mkacc_destroy(c);
    orc_ctx_destroy(oc);
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "layout";
    if (mode == "layout") {
        layout();
    } else if (mode == "engine") {
        engine_evalacc(MKACC_METHOD_MKNTRU, 2, 3, 45181, 7, 901);
        engine_evalacc(MKACC_METHOD_MKNTRU_LWE, 3, 2, 32749, 9, 902);
        engine_nand_mntru(2, 3, 903);
        engine_nand_mklwe(2, 3, 904);
    } else {
        std::printf("usage: adapter_pack layout|engine\n");
        return 2;
    }
    std::printf("%s: %s\n", mode.c_str(), g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}
