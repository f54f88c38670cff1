// mk-acc-amd.h -- reference-side adapter: the MI355X engine behind the
// reference's accumulator plugin seam.
//
// Goes into the reference tree next to mk-acc-xzw.h (src/binfhe/include) and
// compiles against the reference's own headers plus include/mkfhe_amd.h of this
// repo (tests/test_integration_adapter.py checks exactly that on every CPU run).
//
// Seam replaced: class UniEncAccumulator (reference src/binfhe/include/mk-acc.h:55-80),
// chosen in BinFHEScheme(BINFHE_METHOD) (binfhe-base-scheme.h:137-151):
//   * EvalAcc      -> the engine (mkacc_eval_batch, one gate)        mk-acc-xzw.cpp:89-130 / mk-acc-xzw_B.cpp:103-132
//   * KeyGenAcc x2 -> forwarded to the reference's own CPU accumulator  mk-acc.h:59-67, mk-acc-xzw.h:56-61,
//                    (UniEncAccumulatorXZW / _B are `final`, so it is   mk-acc-xzw_B.h:55-62
//                    held, not inherited).  BinFHEScheme::MKKeyGen calls KeyGenAcc through the same
//                    UniEncACCscheme pointer (binfhe-base-scheme.cpp:272, :334), so key generation
//                    keeps working and stays bit-identical to the reference's.
//   * EvalAccBatch -> B independent EvalAcc calls in one engine pass (extension)
//   * EvalNANDBatch-> B whole NAND gates (head, BootstrapGateCore, extraction, ModSwitch, KeySwitch2 /
//                    KeySwitch) on the GPU: BinFHEScheme::EvalBinGate binfhe-base-scheme.cpp:380-515 (extension)
//
// Errors follow the reference's convention (exception.h:162): an engine status
// becomes OPENFHE_THROW(config_error / math_error, text).
#ifndef MK_ACC_AMD_H
#define MK_ACC_AMD_H

#include "mk-acc.h"
#include "mk-acc-xzw.h"
#include "mk-acc-xzw_B.h"
#include "binfhe-base-params.h"
#include "mklwe-cryptoparameters.h"
#include "mklwe-keyswitchkey.h"
#include "mntru-cryptoparameters.h"
#include "mntru-keyswitchkey2.h"
#include "mkfhe_amd.h"

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace lbcrypto {

class UniEncAccumulatorAMD final : public UniEncAccumulator {
    // NATIVE_SIZE=32 -> uint32_t words, NATIVE_SIZE=64 -> uint64_t (mkacc_*_u64 entry points)
    using Word = NativeInteger::Integer;
    static int EngineEval(mkacc_ctx* c, const uint32_t* ct, uint32_t* acc, size_t B) {
        return mkacc_eval_batch(c, ct, acc, acc, B);
    }
    static int EngineEval(mkacc_ctx* c, const uint32_t* ct, uint64_t* acc, size_t B) {
        return mkacc_eval_batch_u64(c, ct, acc, acc, B);
    }
    static int EngineUpload(mkacc_ctx* c, const uint32_t* evk, const uint32_t* pkey) {
        return mkacc_upload_keys(c, evk, pkey);
    }
    static int EngineUpload(mkacc_ctx* c, const uint64_t* evk, const uint64_t* pkey) {
        return mkacc_upload_keys_u64(c, evk, pkey);
    }

public:
    explicit UniEncAccumulatorAMD(BINFHE_METHOD method, int device = 0) : m_method(method), m_device(device) {
        if (method == MKNTRU)
            m_cpu = std::make_shared<UniEncAccumulatorXZW>();
        else if (method == MKNTRU_B || method == MKNTRU_LWE)
            m_cpu = std::make_shared<UniEncAccumulatorXZW_B>();
        else
            OPENFHE_THROW(config_error, "method is invalid");
    }
    UniEncAccumulatorAMD(const UniEncAccumulatorAMD&)            = delete;
    UniEncAccumulatorAMD& operator=(const UniEncAccumulatorAMD&) = delete;
    ~UniEncAccumulatorAMD() {
        if (m_ctx)
            mkacc_destroy(m_ctx);
    }

    // ---- key generation: the reference's own code, unchanged ----------------
    UniEncACCKey KeyGenAcc(const std::shared_ptr<UniEncCryptoParams>& params, const std::vector<NativePoly>& invskNTT,
                           const ConstMNTRUPrivateKey& MNTRUsk, const std::vector<NativePoly>& CRS) const override {
        return m_cpu->KeyGenAcc(params, invskNTT, MNTRUsk, CRS);
    }
    UniEncACCKey KeyGenAcc(const std::shared_ptr<UniEncCryptoParams>& params, const std::vector<NativePoly>& invskNTT,
                           const ConstMKLWEPrivateKey& MKLWEsk, const std::vector<NativePoly>& CRS) const override {
        return m_cpu->KeyGenAcc(params, invskNTT, MKLWEsk, CRS);
    }

    // ---- the hot path --------------------------------------------------------
    // Same contract as UniEncAccumulatorXZW{,_B}::EvalAcc: acc (EVALUATION) is
    // replaced by the accumulator after the k*n blind-rotation steps; skf is
    // unused, as in the reference.
    void EvalAcc(const std::shared_ptr<UniEncCryptoParams>& params, ConstUniEncACCKey& ek,
                 std::vector<std::vector<NativePoly>> Pkey, std::vector<NativePoly> /*skf*/, MKACCCiphertext& acc,
                 const std::vector<NativeVector>& ct) const override {
        std::vector<MKACCCiphertext> accs{acc};
        std::vector<std::vector<NativeVector>> cts{ct};
        EvalAccBatch(params, ek, Pkey, accs, cts);
    }

    // B independent EvalAcc calls (acc[b], ct[b]) in one engine pass.
    void EvalAccBatch(const std::shared_ptr<UniEncCryptoParams>& params, ConstUniEncACCKey& ek,
                      const std::vector<std::vector<NativePoly>>& Pkey, std::vector<MKACCCiphertext>& acc,
                      const std::vector<std::vector<NativeVector>>& ct) const {
        std::lock_guard<std::mutex> g(m_mu);
        const size_t B = acc.size();
        if (ct.size() != B)
            OPENFHE_THROW(config_error, "EvalAccBatch: acc and ct must have the same length");
        if (B == 0)
            return;
        const uint32_t k = params->Getk(), N = params->GetN();
        if (ct[0].size() != k)
            OPENFHE_THROW(config_error, "EvalAccBatch: ciphertext has the wrong number of parties");
        const uint32_t n = ct[0][0].GetLength();
        // XZW scales c = ct*2N/q with the ciphertext's own modulus (mk-acc-xzw.cpp:96,110); XZW_B takes
        // ct mod 2N as is (mk-acc-xzw_B.cpp:103-132), so there q only matters to the gate head.
        const uint64_t q = ct[0][0].GetModulus().ConvertToInt<uint64_t>();
        Prepare(params, ek, n, (m_method == MKNTRU || !m_ctx) ? q : m_p.q);
        UploadKeys(ek, Pkey);
        std::vector<uint32_t> c(B * k * n);
        std::vector<Word> a(B * k * N);
        for (size_t b = 0; b < B; ++b) {
            if (ct[b].size() != k || acc[b] == nullptr || acc[b]->GetElements().size() != k)
                OPENFHE_THROW(config_error, "EvalAccBatch: ciphertext/accumulator has the wrong number of parties");
            for (uint32_t u = 0; u < k; ++u) {
                const NativeVector& cu = ct[b][u];
                if (cu.GetLength() != n)
                    OPENFHE_THROW(config_error, "EvalAccBatch: ragged ciphertext");
                for (uint32_t i = 0; i < n; ++i)
                    c[(b * k + u) * n + i] = cu[i].ConvertToInt<uint32_t>();
                const NativePoly& p = acc[b]->GetElements()[u];
                if (p.GetFormat() != Format::EVALUATION)
                    OPENFHE_THROW(config_error, "EvalAccBatch: accumulator must be in EVALUATION format");
                for (uint32_t j = 0; j < N; ++j)
                    a[(b * k + u) * N + j] = p[j].ConvertToInt<Word>();
            }
        }
        Check(EngineEval(m_ctx, c.data(), a.data(), B));
        for (size_t b = 0; b < B; ++b) {
            auto& polys = acc[b]->GetElements();
            for (uint32_t u = 0; u < k; ++u) {
                NativeVector v(N, params->GetQ());
                for (uint32_t j = 0; j < N; ++j)
                    v[j] = NativeInteger(a[(b * k + u) * N + j]);
                polys[u].SetValues(std::move(v), Format::EVALUATION);
            }
        }
    }

    // ---- whole NAND gates on the GPU (BinFHEScheme::EvalBinGate, batch form) --
    // MK-NTRU: out[b] = KeySwitch2(ModSwitch(extract(BootstrapGateCore(ctNAND - (ct1[b] + ct2[b])))))
    // (binfhe-base-scheme.cpp:467-515, 1072-1130).  Bit-identical to B reference calls.
    std::vector<MNTRUCiphertext> EvalNANDBatch(const std::shared_ptr<UniEncCryptoParams>& params,
                                               const std::shared_ptr<MNTRUCryptoParams>& ntru,
                                               ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey,
                                               ConstMNTRUSwitchingKey2& ksk2, ConstMNTRUCiphertext& ctNAND,
                                               const std::vector<MNTRUCiphertext>& ct1,
                                               const std::vector<MNTRUCiphertext>& ct2) const {
        std::lock_guard<std::mutex> g(m_mu);
        if (m_method != MKNTRU)
            OPENFHE_THROW(config_error, "EvalNANDBatch(MNTRU) needs the MKNTRU accumulator");
        if (ek == nullptr)
            OPENFHE_THROW(config_error,
                          "Bootstrapping keys have not been generated. Please call MKBTKeyGen "
                          "before calling bootstrapping.");
        const size_t B = ct1.size();
        if (ct2.size() != B)
            OPENFHE_THROW(config_error, "ct1 and ct2 must have the same length");
        const uint32_t k = ntru->Getk(), n = ntru->Getn();
        Prepare(params, ek, n, ntru->Getq().ConvertToInt<uint64_t>());
        UploadKeys(ek, Pkey);
        const mkacc_ks_params ks{ntru->GetqKS().ConvertToInt<uint64_t>(), ntru->GetBaseKS(), n};
        UploadKSK2(ks, ksk2);
        std::vector<uint32_t> nand(k * n), a1(B * k * n), a2(B * k * n), out(B * k * n);
        PackMNTRU(*ctNAND, nand.data(), k, n);
        for (size_t b = 0; b < B; ++b) {
            if (ct1[b] == ct2[b])
                OPENFHE_THROW(config_error, "Input ciphertexts should be independant");
            PackMNTRU(*ct1[b], a1.data() + b * k * n, k, n);
            PackMNTRU(*ct2[b], a2.data() + b * k * n, k, n);
        }
        Check(mkacc_eval_nand_mntru(m_ctx, nand.data(), a1.data(), a2.data(), out.data(), B));
        std::vector<MNTRUCiphertext> res(B);
        for (size_t b = 0; b < B; ++b) {
            std::vector<NativeVector> c(k, NativeVector(n, ntru->GetqKS()));
            for (uint32_t u = 0; u < k; ++u)
                for (uint32_t i = 0; i < n; ++i)
                    c[u][i] = NativeInteger(out[(b * k + u) * n + i]);
            res[b] = std::make_shared<MNTRUCiphertextImpl>(std::move(c));
        }
        return res;
    }

    // MK-LWE: out[b] = KeySwitch(ModSwitch(extract(BootstrapGateCore(ModSwitch_2N((0, 5q/8) - (ct1[b] + ct2[b]))))))
    // (binfhe-base-scheme.cpp:380-463, 1004-1067).
    std::vector<MKLWECiphertext> EvalNANDBatch(const std::shared_ptr<UniEncCryptoParams>& params,
                                               const std::shared_ptr<MKLWECryptoParams>& lwe,
                                               ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey,
                                               ConstMKLWESwitchingKey& ksk, const std::vector<MKLWECiphertext>& ct1,
                                               const std::vector<MKLWECiphertext>& ct2) const {
        std::lock_guard<std::mutex> g(m_mu);
        if (m_method != MKNTRU_LWE && m_method != MKNTRU_B)
            OPENFHE_THROW(config_error, "EvalNANDBatch(MKLWE) needs the MKNTRU_LWE accumulator");
        if (ek == nullptr)
            OPENFHE_THROW(config_error,
                          "Bootstrapping keys have not been generated. Please call MKBTKeyGen "
                          "before calling bootstrapping.");
        const size_t B = ct1.size();
        if (ct2.size() != B)
            OPENFHE_THROW(config_error, "ct1 and ct2 must have the same length");
        const uint32_t k = lwe->Getk(), n = lwe->Getn();
        Prepare(params, ek, n, lwe->Getq().ConvertToInt<uint64_t>());
        UploadKeys(ek, Pkey);
        const mkacc_ks_params ks{lwe->GetqKS().ConvertToInt<uint64_t>(), lwe->GetBaseKS(), n};
        UploadKSK(ks, ksk);
        std::vector<uint32_t> a1(B * k * n), a2(B * k * n), b1(B), b2(B), oa(B * k * n), ob(B);
        for (size_t b = 0; b < B; ++b) {
            if (ct1[b] == ct2[b])
                OPENFHE_THROW(config_error, "Input ciphertexts should be independant");
            PackMKLWE(*ct1[b], a1.data() + b * k * n, k, n);
            PackMKLWE(*ct2[b], a2.data() + b * k * n, k, n);
            b1[b] = ct1[b]->GetB().ConvertToInt<uint32_t>();
            b2[b] = ct2[b]->GetB().ConvertToInt<uint32_t>();
        }
        Check(mkacc_eval_nand_mklwe(m_ctx, a1.data(), b1.data(), a2.data(), b2.data(), oa.data(), ob.data(), B));
        std::vector<MKLWECiphertext> res(B);
        for (size_t b = 0; b < B; ++b) {
            std::vector<NativeVector> a(k, NativeVector(n, lwe->GetqKS()));
            for (uint32_t u = 0; u < k; ++u)
                for (uint32_t i = 0; i < n; ++i)
                    a[u][i] = NativeInteger(oa[(b * k + u) * n + i]);
            res[b] = std::make_shared<MKLWECiphertextImpl>(std::move(a), NativeInteger(ob[b]));
        }
        return res;
    }

    // The two gate batches with the BinFHECryptoParams that BinFHEScheme holds
    // (binfhe-base-params.h:106-140), so the scheme-side patch is one call
    // (INTEGRATION.md §3).
    std::vector<MNTRUCiphertext> EvalNANDBatch(const std::shared_ptr<BinFHECryptoParams>& params,
                                               ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey,
                                               ConstMNTRUSwitchingKey2& ksk2, ConstMNTRUCiphertext& ctNAND,
                                               const std::vector<MNTRUCiphertext>& ct1,
                                               const std::vector<MNTRUCiphertext>& ct2) const {
        return EvalNANDBatch(params->GetUniEncParams(), params->GetMatrixNTRUParams(), ek, Pkey, ksk2, ctNAND, ct1,
                             ct2);
    }
    std::vector<MKLWECiphertext> EvalNANDBatch(const std::shared_ptr<BinFHECryptoParams>& params,
                                               ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey,
                                               ConstMKLWESwitchingKey& ksk, const std::vector<MKLWECiphertext>& ct1,
                                               const std::vector<MKLWECiphertext>& ct2) const {
        return EvalNANDBatch(params->GetUniEncParams(), params->GetMKLWEParams(), ek, Pkey, ksk, ct1, ct2);
    }

private:
    static void Check(int rc) {
        if (rc == MKACC_OK)
            return;
        if (rc == MKACC_E_RANGE)
            OPENFHE_THROW(math_error, mkacc_last_error());
        OPENFHE_THROW(config_error, mkacc_last_error());
    }

    uint32_t EngineMethod() const {
        return m_method == MKNTRU ? MKACC_METHOD_MKNTRU
                                  : (m_method == MKNTRU_B ? MKACC_METHOD_MKNTRU_B : MKACC_METHOD_MKNTRU_LWE);
    }

    // One engine context per adapter; (re)created when the shape changes.
    void Prepare(const std::shared_ptr<UniEncCryptoParams>& P, ConstUniEncACCKey& ek, uint32_t n, uint64_t q) const {
        if (ek == nullptr)
            OPENFHE_THROW(config_error,
                          "Bootstrapping keys have not been generated. Please call MKBTKeyGen "
                          "before calling bootstrapping.");
        mkacc_params p{};
        p.method  = EngineMethod();
        p.k       = P->Getk();
        p.n       = n;
        p.N       = P->GetN();
        p.Q       = P->GetQ().ConvertToInt<uint64_t>();
        p.q       = q;
        p.baseG   = P->GetBaseG();
        p.digitsG = P->GetDigitsG();
        p.root    = P->GetPolyParams()->GetRootOfUnity().ConvertToInt<uint64_t>();
        if (m_ctx && p.k == m_p.k && p.n == m_p.n && p.N == m_p.N && p.Q == m_p.Q && p.q == m_p.q &&
            p.baseG == m_p.baseG && p.digitsG == m_p.digitsG && p.root == m_p.root)
            return;
        if (m_ctx)
            mkacc_destroy(m_ctx);
        m_ctx = nullptr;
        m_key.reset();
        m_ksk2.reset();
        m_ksk.reset();
        Check(mkacc_create(&p, m_device, &m_ctx));
        m_p = p;
    }

    // Flatten (*ek)[u][j][i] -> GetElements()[digit][0|1] into [k][nk][n+1][dg][2][N] once per key object.
    // Entries the reference leaves empty ((*ek)[u][1][n], and (*ek)[u][0][n] for u > 0,
    // mk-acc-xzw.cpp:66-80) are unused by EvalAcc and sent as zeros.
    void UploadKeys(ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey) const {
        const uint32_t k = m_p.k, N = m_p.N, dg = m_p.digitsG - 1, n1 = m_p.n + 1;
        const uint32_t nk = m_method == MKNTRU ? 2 : 1;
        if (Pkey.size() != k)
            OPENFHE_THROW(config_error, "Pkey has the wrong number of parties");
        std::vector<Word> pk(mkacc_pkey_words(m_ctx));  // [k][dg][N]
        for (uint32_t u = 0; u < k; ++u) {
            if (Pkey[u].size() < dg)
                OPENFHE_THROW(config_error, "Pkey has the wrong number of digits");
            for (uint32_t d = 0; d < dg; ++d)
                for (uint32_t s = 0; s < N; ++s)
                    pk[(size_t(u) * dg + d) * N + s] = Pkey[u][d][s].ConvertToInt<Word>();
        }
        // Pkey arrives by value on every call, so it is compared by content; the
        // key object is held, so its address cannot be recycled while cached.
        if (m_key == ek && m_pkey == pk)
            return;
        const auto& K = ek->GetElements();
        if (K.size() != k)
            OPENFHE_THROW(config_error, "bootstrapping key has the wrong number of parties");
        std::vector<Word> evk(mkacc_evk_words(m_ctx), Word(0));
        size_t o = 0;
        for (uint32_t u = 0; u < k; ++u) {
            if (K[u].size() < nk)
                OPENFHE_THROW(config_error, "bootstrapping key has the wrong shape");
            for (uint32_t j = 0; j < nk; ++j) {
                if (K[u][j].size() != n1)
                    OPENFHE_THROW(config_error, "bootstrapping key has the wrong dimension");
                for (uint32_t i = 0; i < n1; ++i) {
                    const auto& e = K[u][j][i];
                    if (e == nullptr) {
                        o += size_t(dg) * 2 * N;
                        continue;
                    }
                    const auto& el = e->GetElements();
                    if (el.size() != dg)
                        OPENFHE_THROW(config_error, "bootstrapping key has the wrong number of digits");
                    for (uint32_t d = 0; d < dg; ++d)
                        for (uint32_t t = 0; t < 2; ++t, o += N)
                            for (uint32_t s = 0; s < N; ++s)
                                evk[o + s] = el[d][t][s].ConvertToInt<Word>();
                }
            }
        }
        m_key.reset();
        Check(EngineUpload(m_ctx, evk.data(), pk.data()));
        m_key  = ek;
        m_pkey = std::move(pk);
    }

    // KeySwitch2 key: the engine takes KSK2[u][1] ([k][N*dks][n]); KeySwitchGen2
    // stores KSK2[u][j] = j * KSK2[u][1] mod qKS (mntru-pke.cpp:740-755).
    void UploadKSK2(const mkacc_ks_params& ks, ConstMNTRUSwitchingKey2& K) const {
        if (K == nullptr)
            OPENFHE_THROW(config_error, "key-switching key has not been generated (MKBTKeyGen)");
        if (m_ksk2 == K)
            return;
        const uint32_t k = m_p.k, N = m_p.N, n = ks.n_out, dks = mkacc_ks_digits(&ks);
        const auto& E = K->GetElements();  // [k][baseKS][N*dks][n]
        std::vector<uint32_t> w(size_t(k) * N * dks * n);
        for (uint32_t u = 0; u < k; ++u) {
            if (E.size() != k || E[u].size() < 2 || E[u][1].size() != size_t(N) * dks)
                OPENFHE_THROW(config_error, "KeySwitch2 key has the wrong shape");
            for (size_t l = 0; l < size_t(N) * dks; ++l)
                for (uint32_t i = 0; i < n; ++i)
                    w[(u * size_t(N) * dks + l) * n + i] = E[u][1][l][i].ConvertToInt<uint32_t>();
        }
        m_ksk2.reset();
        Check(mkacc_upload_ksk_mntru(m_ctx, &ks, w.data()));
        m_ksk2 = K;
    }

    // MK-LWE KeySwitch key (mklwe-pke.cpp:176-258): A [k][N][baseKS][dks][n], B [k][N][baseKS][dks].
    void UploadKSK(const mkacc_ks_params& ks, ConstMKLWESwitchingKey& K) const {
        if (K == nullptr)
            OPENFHE_THROW(config_error, "key-switching key has not been generated (MKBTKeyGen)");
        if (m_ksk == K)
            return;
        const uint32_t k = m_p.k, N = m_p.N, n = ks.n_out, base = ks.baseKS, dks = mkacc_ks_digits(&ks);
        const auto& A = K->GetElementsA();
        const auto& Bk = K->GetElementsB();
        std::vector<uint32_t> wa(size_t(k) * N * base * dks * n), wb(size_t(k) * N * base * dks);
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t i = 0; i < N; ++i)
                for (uint32_t a = 0; a < base; ++a)
                    for (uint32_t j = 0; j < dks; ++j) {
                        const size_t r = ((size_t(u) * N + i) * base + a) * dks + j;
                        wb[r] = Bk[u][i][a][j].ConvertToInt<uint32_t>();
                        for (uint32_t l = 0; l < n; ++l)
                            wa[r * n + l] = A[u][i][a][j][l].ConvertToInt<uint32_t>();
                    }
        m_ksk.reset();
        Check(mkacc_upload_ksk_mklwe(m_ctx, &ks, wa.data(), wb.data()));
        m_ksk = K;
    }

    static void PackMNTRU(const MNTRUCiphertextImpl& ct, uint32_t* dst, uint32_t k, uint32_t n) {
        const auto& e = ct.GetElements();
        if (e.size() != k)
            OPENFHE_THROW(config_error, "ciphertext has the wrong number of parties");
        for (uint32_t u = 0; u < k; ++u) {
            if (e[u].GetLength() != n)
                OPENFHE_THROW(config_error, "ciphertext has the wrong dimension");
            for (uint32_t i = 0; i < n; ++i)
                dst[u * n + i] = e[u][i].ConvertToInt<uint32_t>();
        }
    }
    static void PackMKLWE(const MKLWECiphertextImpl& ct, uint32_t* dst, uint32_t k, uint32_t n) {
        const auto& a = ct.GetA();
        if (a.size() != k)
            OPENFHE_THROW(config_error, "ciphertext has the wrong number of parties");
        for (uint32_t u = 0; u < k; ++u) {
            if (a[u].GetLength() != n)
                OPENFHE_THROW(config_error, "ciphertext has the wrong dimension");
            for (uint32_t i = 0; i < n; ++i)
                dst[u * n + i] = a[u][i].ConvertToInt<uint32_t>();
        }
    }

    BINFHE_METHOD m_method;
    int m_device;
    std::shared_ptr<UniEncAccumulator> m_cpu;  // reference XZW / XZW_B: KeyGenAcc
    mutable std::mutex m_mu;
    mutable mkacc_ctx* m_ctx = nullptr;
    mutable mkacc_params m_p{};
    mutable std::shared_ptr<const UniEncACCKeyImpl> m_key;
    mutable std::vector<Word> m_pkey;
    mutable std::shared_ptr<const MNTRUSwitchingKey2Impl> m_ksk2;
    mutable std::shared_ptr<const MKLWESwitchingKeyImpl> m_ksk;
};

}  // namespace lbcrypto

#endif  // MK_ACC_AMD_H
