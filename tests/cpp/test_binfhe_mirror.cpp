// C++ tests of the host mirror (include/mkfhe_amd_binfhe.hpp) written the way
// the reference's own binfhe unit tests read: build params, keys and an
// accumulator, call EvalAcc, compare.  The expected values come from the CPU
// oracle (oracle/mkfhe_oracle.c), which only tests may link.
//
//   ./test_binfhe_mirror cpu   -- host logic only (no GPU calls)
//   ./test_binfhe_mirror gpu   -- bit-exact parity through the HIP engine
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mkfhe_amd_binfhe.hpp"
#include "mkfhe_oracle.h"

using namespace mkfhe_amd;

static int g_fail = 0;
#define EXPECT(cond)                                                               \
    do {                                                                           \
        if (!(cond)) {                                                             \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);   \
            ++g_fail;                                                              \
        }                                                                          \
    } while (0)
template <class E, class F>
static bool throws(F f) {
    try {
        f();
    } catch (const E&) {
        return true;
    } catch (...) {
        return false;
    }
    return false;
}

static const uint64_t kQ = 134176769;

// ---- host-only checks ---------------------------------------------------------
static void test_cpu() {
    auto p = UniEncCryptoParams::FromParamSet("STD128_MKNTRU", MKNTRU);
    EXPECT(p->Getk() == 2 && p->GetLatticeParam() == 765 && p->GetN() == 2048);
    EXPECT(p->GetQ() == kQ && p->Getq() == 45181 && p->GetBaseG() == 128 && p->GetDigitsG() == 4);
    auto pl = UniEncCryptoParams::FromParamSet("STD100_MKNTRU_LWE_2", MKNTRU_LWE);
    EXPECT(pl->Getk() == 4 && pl->GetLatticeParam() == 500 && pl->Getq() == 32749 && pl->GetDigitsG() == 3);
    // reference error behaviour: config_error on a non-power-of-two gadget base
    // (mk-cryptoparameters.h:146-147) and on an invalid method
    EXPECT(throws<config_error>([] { UniEncCryptoParams(2, 2048, kQ, 45181, 100, MKNTRU, 10); }));
    EXPECT(throws<config_error>([] { UniEncCryptoParams(2, 2048, kQ, 45181, 512, GINX, 10); }));
    EXPECT(throws<config_error>([] { UniEncCryptoParams::FromParamSet("STD128", MKNTRU); }));
    EXPECT(throws<config_error>([] { MakeUniEncAccumulator(LMKCDEY); }));
    EXPECT(dynamic_cast<UniEncAccumulatorXZW*>(MakeUniEncAccumulator(MKNTRU).get()) != nullptr);
    EXPECT(dynamic_cast<UniEncAccumulatorXZW_B*>(MakeUniEncAccumulator(MKNTRU_LWE).get()) != nullptr);
    // EvalAcc without keys: config_error before any device work (binfhe-base-scheme.cpp:1075-1080)
    auto acc = MakeUniEncAccumulator(MKNTRU);
    ConstUniEncACCKey none;
    MKACCCiphertext a = std::make_shared<MKACCCiphertextImpl>();
    EXPECT(throws<config_error>([&] { acc->EvalAcc(p, none, {}, {}, a, {}); }));
    // the method check is per accumulator class
    auto accB = MakeUniEncAccumulator(MKNTRU_B);
    ConstUniEncACCKey some = std::make_shared<const UniEncACCKeyImpl>();
    EXPECT(throws<config_error>([&] { accB->EvalAcc(p, some, {}, {}, a, {}); }));

    // BinFHEContext key generation / encryption / decryption run on the host
    // (libmkfhe_keys.so); the device context is only created by MKBTKeyGen / EvalBinGate.
    BinFHEContext cc;
    cc.GenerateBinFHEContext(STD100_MKNTRU, MKNTRU);
    cc.SetSeed(7);
    auto sk = cc.MNTRU_KeyGen();
    EXPECT(sk->Getk() == 2 && sk->GetLength() == 560 && sk->GetModulus() == 45181);
    EXPECT(throws<config_error>([&] { cc.MKLWE_KeyGen(); }));          // binfhecontext.cpp:244-249
    EXPECT(throws<config_error>([&] { cc.ctGateGen(sk, AND); }));      // binfhe-base-scheme.cpp:341-342
    for (int m = 0; m < 2; ++m) {
        auto ct = cc.Encrypt(sk, m);
        EXPECT(ct->GetModulus() == 45181 && ct->GetptModulus() == 4);
        MNTRUPlaintext r = -1;
        cc.Decrypt2(sk, ct, &r);
        EXPECT(r == m);
    }
    auto c0 = cc.Encrypt(sk, 0), c1 = cc.Encrypt(sk, 1);
    EXPECT(throws<config_error>([&] { cc.EvalBinGate(NAND, c0, c1); }));  // keys not generated
    {   // MKNTRU_B gates are undefined in the reference (binfhe-base-scheme.cpp:1127, mk-acc-xzw_B.cpp:120)
        BinFHEContext cb;
        cb.GenerateBinFHEContext(STD100_MKNTRU, MKNTRU_B);
        bool named = false;
        try {
            cb.EvalBinGate(NAND, c0, c1);
        } catch (const config_error& e) {
            named = std::strstr(e.what(), "MKNTRU_B") != nullptr;
        }
        EXPECT(named);
    }
    // secret-key file round trip (mkfhe_keys.h wire format)
    const std::string f = std::string(std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp") + "/mkfhe_sk_test.mkfk";
    cc.SaveSecretKey(f, sk);
    auto sk2 = cc.LoadMNTRUSecretKey(f);
    EXPECT(sk2->F() == sk->F() && sk2->Finv() == sk->Finv());
    MNTRUPlaintext r1 = -1;
    cc.Decrypt2(sk2, c1, &r1);
    EXPECT(r1 == 1);
    std::remove(f.c_str());
    EXPECT(throws<config_error>([&] { cc.LoadMNTRUSecretKey(f); }));
    BinFHEContext cl;
    cl.GenerateBinFHEContext(STD100_MKNTRU_LWE, MKNTRU_LWE);
    auto skl = cl.MKLWE_KeyGen();
    for (int m = 0; m < 2; ++m) {
        auto ct = cl.Encrypt(skl, m);
        MKLWEPlaintext r = -1;
        cl.Decrypt(skl, ct, &r);
        EXPECT(r == m);
    }
}

// ---- GPU parity ------------------------------------------------------------------
struct Case {
    BINFHE_METHOD method;
    uint32_t k, n;
    uint64_t q;
    uint32_t baseG;
    uint32_t B;
};

static std::vector<uint64_t> uniform(size_t n, uint64_t bound, uint64_t seed) {
    std::vector<uint64_t> v(n);
    orc_fill_uniform(v.data(), n, bound, seed);
    return v;
}

static void run_case(const Case& cs, uint64_t seed) {
    const uint32_t N = 2048;
    auto params = std::make_shared<UniEncCryptoParams>(cs.k, N, kQ, cs.q, cs.baseG, cs.method, cs.n);
    auto acc = MakeUniEncAccumulator(cs.method);
    const mkacc_params eff = acc->Params(*params);
    const uint32_t dg = eff.digitsG - 1, nk = cs.method == MKNTRU ? 2 : 1;

    orc_params op{};
    op.method = cs.method == MKNTRU ? ORC_XZW : ORC_XZW_B;
    op.k = cs.k; op.n = cs.n; op.N = N; op.Q = kQ; op.q = cs.q; op.baseG = cs.baseG;
    op.digitsG = eff.digitsG; op.psi = eff.root;
    orc_ctx* oc = orc_ctx_create(&op);
    EXPECT(oc != nullptr);

    // keys: the reference containers, filled with seed-derived residues
    auto evk = uniform(orc_evk_words(&op), kQ, seed * 10 + 1);
    auto pk = uniform((size_t)cs.k * dg * N, kQ, seed * 10 + 2);
    auto ek = std::make_shared<UniEncACCKeyImpl>(cs.k, nk, cs.n + 1);
    size_t o = 0;
    for (uint32_t u = 0; u < cs.k; ++u)
        for (uint32_t j = 0; j < nk; ++j)
            for (uint32_t i = 0; i <= cs.n; ++i) {
                auto key = std::make_shared<UniEncEvalKeyImpl>(dg, 2);
                for (uint32_t d = 0; d < dg; ++d)
                    for (uint32_t c = 0; c < 2; ++c, o += N)
                        key->GetElements()[d][c] =
                            NativePoly(NativeVector(evk.begin() + o, evk.begin() + o + N), EVALUATION);
                (*ek)[u][j][i] = key;
            }
    std::vector<std::vector<NativePoly>> Pkey(cs.k);
    for (uint32_t u = 0; u < cs.k; ++u)
        for (uint32_t d = 0; d < dg; ++d) {
            const size_t b = ((size_t)u * dg + d) * N;
            Pkey[u].emplace_back(NativeVector(pk.begin() + b, pk.begin() + b + N), EVALUATION);
        }
    ConstUniEncACCKey cek = ek;

    const uint64_t bound = cs.method == MKNTRU ? cs.q : 2 * N;
    auto ct = uniform((size_t)cs.B * cs.k * cs.n, bound, seed * 10 + 3);
    auto acc0 = uniform((size_t)cs.B * cs.k * N, kQ, seed * 10 + 4);
    ct[0] = 0;                                            // monomial edge c = 0
    ct[(size_t)cs.k * cs.n - 1] = bound - 1;              // and c = 2N - 1
    auto expect = acc0;
    EXPECT(orc_evalacc_batch(oc, evk.data(), pk.data(), ct.data(), expect.data(), cs.B, 8) == 0);

    std::vector<MKACCCiphertext> accs;
    std::vector<std::vector<NativeVector>> cts;
    for (uint32_t b = 0; b < cs.B; ++b) {
        std::vector<NativePoly> el;
        std::vector<NativeVector> c;
        for (uint32_t u = 0; u < cs.k; ++u) {
            const size_t ao = ((size_t)b * cs.k + u) * N, co = ((size_t)b * cs.k + u) * cs.n;
            el.emplace_back(NativeVector(acc0.begin() + ao, acc0.begin() + ao + N), EVALUATION);
            c.emplace_back(ct.begin() + co, ct.begin() + co + cs.n);
        }
        accs.push_back(std::make_shared<MKACCCiphertextImpl>(el));
        cts.push_back(c);
    }
    // gate 0 through the reference-shaped EvalAcc, the rest as a batch
    MKACCCiphertext a0 = accs[0];
    acc->EvalAcc(params, cek, Pkey, {}, a0, cts[0]);
    std::vector<MKACCCiphertext> rest(accs.begin() + 1, accs.end());
    std::vector<std::vector<NativeVector>> rcts(cts.begin() + 1, cts.end());
    acc->EvalAccBatch(params, cek, Pkey, rest, rcts);
    size_t bad = 0;
    for (uint32_t b = 0; b < cs.B; ++b)
        for (uint32_t u = 0; u < cs.k; ++u)
            for (uint32_t j = 0; j < N; ++j)
                bad += accs[b]->GetElements()[u][j] != expect[((size_t)b * cs.k + u) * N + j];
    if (bad) std::fprintf(stderr, "case method=%d k=%u n=%u: %zu coefficients differ\n", cs.method, cs.k, cs.n, bad);
    EXPECT(bad == 0);

    // primitives: SetFormat (NTT) and SignedDigitDecompose against the oracle
    NativePoly x(uniform(N, kQ, seed * 10 + 5), COEFFICIENT);
    NativePoly y = x;
    acc->SetFormat(params, y, EVALUATION);
    std::vector<uint64_t> ref = x.values;
    orc_ntt_forward(ref.data(), N, kQ, eff.root);
    EXPECT(y.values == ref && y.format == EVALUATION);
    acc->SetFormat(params, y, COEFFICIENT);
    EXPECT(y == x);
    std::vector<NativePoly> digits;
    acc->SignedDigitDecompose(params, x, digits);
    std::vector<uint64_t> rd((size_t)dg * N);
    orc_sdd(x.values.data(), rd.data(), N, kQ, cs.baseG, dg);
    EXPECT(digits.size() == dg);
    for (uint32_t d = 0; d < dg && d < digits.size(); ++d)
        EXPECT(std::memcmp(digits[d].values.data(), rd.data() + (size_t)d * N, N * 8) == 0);

    // range errors keep the reference's exception class (math_error)
    auto badacc = std::make_shared<MKACCCiphertextImpl>(accs[0]->GetElements());
    badacc->GetElements()[0][5] = kQ;
    EXPECT(throws<math_error>([&] { acc->EvalAcc(params, cek, Pkey, {}, badacc, cts[0]); }));
    orc_ctx_destroy(oc);
}

// ---- full NAND gates through BinFHEContext ----------------------------------------------
static void test_gpu_gates(BINFHE_METHOD method, uint32_t k, uint32_t n, uint32_t baseG, uint64_t seed) {
    const uint32_t N = 2048, B = 3, baseKS = 32;
    const bool lwe = method != MKNTRU;
    const uint64_t q = lwe ? 32749 : 45181, qKS = q;
    BinFHEContext cc;
    cc.GenerateBinFHEContext(UniEncCryptoParams(k, N, kQ, q, baseG, method, n));
    // reference error behaviour before keys exist
    auto c0 = std::make_shared<MNTRUCiphertextImpl>(std::vector<NativeVector>(k, NativeVector(n, 0)), q);
    auto c1 = std::make_shared<MNTRUCiphertextImpl>(*c0);
    if (!lwe) EXPECT(throws<config_error>([&] { cc.EvalBinGate(NAND, c0, c1); }));
    EXPECT(throws<config_error>([&] { cc.EvalBinGate(NAND, c0, c0); }));
    const mkacc_params eff = cc.GetParams()->abi();
    const uint32_t dg = eff.digitsG - 1, nk = lwe ? 1 : 2;
    mkacc_ks_params ks{qKS, baseKS, n};
    const uint32_t dks = mkacc_ks_digits(&ks);

    orc_params op{};
    op.method = lwe ? ORC_XZW_B : ORC_XZW;
    op.k = k; op.n = n; op.N = N; op.Q = kQ; op.q = q; op.baseG = baseG; op.digitsG = eff.digitsG; op.psi = eff.root;
    orc_ctx* oc = orc_ctx_create(&op);

    UniEncBTKey ek;
    auto evk = uniform(orc_evk_words(&op), kQ, seed * 10 + 1);
    auto pk = uniform((size_t)k * dg * N, kQ, seed * 10 + 2);
    auto acck = std::make_shared<UniEncACCKeyImpl>(k, nk, n + 1);
    size_t o = 0;
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < nk; ++j)
            for (uint32_t i = 0; i <= n; ++i) {
                auto key = std::make_shared<UniEncEvalKeyImpl>(dg, 2);
                for (uint32_t d = 0; d < dg; ++d)
                    for (uint32_t c = 0; c < 2; ++c, o += N)
                        key->GetElements()[d][c] = NativePoly(NativeVector(evk.begin() + o, evk.begin() + o + N), EVALUATION);
                (*acck)[u][j][i] = key;
            }
    ek.BSkey = acck;
    ek.Pkey.resize(k);
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t d = 0; d < dg; ++d) {
            const size_t b = ((size_t)u * dg + d) * N;
            ek.Pkey[u].emplace_back(NativeVector(pk.begin() + b, pk.begin() + b + N), EVALUATION);
        }
    // key-switching keys, shaped as KeySwitchGen2 / KeySwitchGen produce them
    std::vector<uint64_t> ksk2, A, Bk;
    if (!lwe) {
        auto ksk = uniform((size_t)k * N * dks * n, qKS, seed * 10 + 3);
        ksk2.resize((size_t)k * baseKS * N * dks * n);
        std::vector<std::vector<std::vector<NativeVector>>> K2(k, std::vector<std::vector<NativeVector>>(baseKS));
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t jj = 0; jj < baseKS; ++jj) {
                K2[u][jj].resize((size_t)N * dks);
                for (size_t l = 0; l < (size_t)N * dks; ++l) {
                    NativeVector row(n);
                    for (uint32_t i = 0; i < n; ++i) {
                        row[i] = (jj * ksk[((size_t)u * N * dks + l) * n + i]) % qKS;
                        ksk2[(((size_t)u * baseKS + jj) * N * dks + l) * n + i] = row[i];
                    }
                    K2[u][jj][l] = std::move(row);
                }
            }
        ek.KSkey2 = std::make_shared<MNTRUSwitchingKey2Impl>(std::move(K2));
    } else {
        A = uniform((size_t)k * N * baseKS * dks * n, qKS, seed * 10 + 4);
        Bk = uniform((size_t)k * N * baseKS * dks, qKS, seed * 10 + 5);
        MKLWESwitchingKeyImpl::A4 a4(k, std::vector<std::vector<std::vector<NativeVector>>>(
                                            N, std::vector<std::vector<NativeVector>>(baseKS, std::vector<NativeVector>(dks))));
        MKLWESwitchingKeyImpl::B4 b4(k, std::vector<std::vector<std::vector<uint64_t>>>(
                                            N, std::vector<std::vector<uint64_t>>(baseKS, std::vector<uint64_t>(dks))));
        size_t r = 0;
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t j = 0; j < N; ++j)
                for (uint32_t d = 0; d < baseKS; ++d)
                    for (uint32_t t = 0; t < dks; ++t, ++r) {
                        a4[u][j][d][t] = NativeVector(A.begin() + r * n, A.begin() + (r + 1) * n);
                        b4[u][j][d][t] = Bk[r];
                    }
        ek.LKSkey = std::make_shared<MKLWESwitchingKeyImpl>(std::move(a4), std::move(b4));
    }
    cc.BTKeyLoad(ek);

    auto w1 = uniform((size_t)B * k * n, q, seed * 10 + 6), w2 = uniform((size_t)B * k * n, q, seed * 10 + 7);
    auto wb = uniform(2 * B, q, seed * 10 + 8), wn = uniform((size_t)k * n, q, seed * 10 + 9);
    auto vecs = [&](const std::vector<uint64_t>& w, uint32_t b) {
        std::vector<NativeVector> e(k);
        for (uint32_t u = 0; u < k; ++u) e[u] = NativeVector(w.begin() + ((size_t)b * k + u) * n, w.begin() + ((size_t)b * k + u + 1) * n);
        return e;
    };
    size_t bad = 0;
    std::vector<uint64_t> acc((size_t)k * N), out((size_t)k * n);
    if (!lwe) {
        std::vector<NativeVector> nv(k);
        for (uint32_t u = 0; u < k; ++u) nv[u] = NativeVector(wn.begin() + (size_t)u * n, wn.begin() + (size_t)(u + 1) * n);
        cc.SetctNAND(std::make_shared<MNTRUCiphertextImpl>(nv, q));
        std::vector<MNTRUCiphertext> x1, x2;
        for (uint32_t b = 0; b < B; ++b) {
            x1.push_back(std::make_shared<MNTRUCiphertextImpl>(vecs(w1, b), q));
            x2.push_back(std::make_shared<MNTRUCiphertextImpl>(vecs(w2, b), q));
        }
        auto res = cc.EvalBinGate(NAND, x1, x2);
        auto single = cc.EvalBinGate(NAND, ConstMNTRUCiphertext(x1[1]), ConstMNTRUCiphertext(x2[1]));
        EXPECT(single->GetElements() == res[1]->GetElements());
        for (uint32_t b = 0; b < B; ++b) {
            std::vector<uint64_t> ct((size_t)k * n);
            orc_mntru_head(wn.data(), w1.data() + (size_t)b * k * n, w2.data() + (size_t)b * k * n, ct.data(), k, n, q);
            orc_mntru_testvector(oc, 4, acc.data());
            EXPECT(orc_evalacc(oc, evk.data(), pk.data(), ct.data(), acc.data()) == 0);
            orc_mntru_tail(oc, acc.data(), ksk2.data(), qKS, baseKS, n, out.data());
            for (uint32_t u = 0; u < k; ++u)
                for (uint32_t i = 0; i < n; ++i) bad += res[b]->GetElements()[u][i] != out[(size_t)u * n + i];
        }
    } else {
        std::vector<MKLWECiphertext> x1, x2;
        for (uint32_t b = 0; b < B; ++b) {
            x1.push_back(std::make_shared<MKLWECiphertextImpl>(vecs(w1, b), wb[b], q));
            x2.push_back(std::make_shared<MKLWECiphertextImpl>(vecs(w2, b), wb[B + b], q));
        }
        auto res = cc.EvalBinGate(NAND, x1, x2);
        for (uint32_t b = 0; b < B; ++b) {
            std::vector<uint64_t> c((size_t)k * n);
            orc_mklwe_head(oc, w1.data() + (size_t)b * k * n, wb[b], w2.data() + (size_t)b * k * n, wb[B + b], q, n, 4,
                           c.data(), acc.data());
            EXPECT(orc_evalacc(oc, evk.data(), pk.data(), c.data(), acc.data()) == 0);
            uint64_t ob = 0;
            orc_mklwe_tail(oc, acc.data(), A.data(), Bk.data(), qKS, baseKS, n, out.data(), &ob);
            bad += res[b]->GetB() != ob;
            for (uint32_t u = 0; u < k; ++u)
                for (uint32_t i = 0; i < n; ++i) bad += res[b]->GetA()[u][i] != out[(size_t)u * n + i];
        }
    }
    if (bad) std::fprintf(stderr, "gate method=%d k=%u n=%u: %zu words differ\n", method, k, n, bad);
    EXPECT(bad == 0);
    EXPECT(throws<not_implemented_error>([&] {
        if (lwe) {
            auto a = std::make_shared<MKLWECiphertextImpl>(vecs(w1, 0), 0, q);
            auto b = std::make_shared<MKLWECiphertextImpl>(vecs(w2, 0), 0, q);
            cc.EvalBinGate(AND, ConstMKLWECiphertext(a), ConstMKLWECiphertext(b));
        } else {
            auto a = std::make_shared<MNTRUCiphertextImpl>(vecs(w1, 0), q);
            auto b = std::make_shared<MNTRUCiphertextImpl>(vecs(w2, 0), q);
            cc.EvalBinGate(AND, ConstMNTRUCiphertext(a), ConstMNTRUCiphertext(b));
        }
    }));
    orc_ctx_destroy(oc);
}

static void test_gpu() {
    const Case cases[] = {
        {MKNTRU, 2, 4, 45181, 1 << 9, 3},      // STD100_MKNTRU shape
        {MKNTRU, 2, 3, 45181, 1 << 7, 2},      // STD128_MKNTRU shape (dg = 3)
        {MKNTRU_LWE, 4, 3, 32749, 1 << 9, 2},  // STD100_MKNTRU_LWE_2 shape
        {MKNTRU, 3, 2, 45181, 1 << 6, 2},      // dg = 4
    };
    uint64_t seed = 1;
    for (const Case& c : cases) run_case(c, seed++);
    test_gpu_gates(MKNTRU, 2, 3, 1 << 7, 11);
    test_gpu_gates(MKNTRU_LWE, 2, 3, 1 << 9, 12);
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    try {
        if (mode == "cpu") test_cpu();
        else test_gpu();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "unexpected exception: %s\n", e.what());
        return 2;
    }
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("ok (%s)\n", mode.c_str());
    return 0;
}
