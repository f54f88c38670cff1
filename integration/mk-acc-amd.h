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
//   * a device list -> the batches shard over the GPUs of the node (mkacc_group_*: keys converted once and
//                    copied device to device over xGMI, contiguous gate shards, bit-identical outputs)
//
// Errors follow the reference's convention (exception.h:162): an engine status
// becomes OPENFHE_THROW(config_error / math_error, text).
//
// The conversions between the reference's objects and the C-ABI buffers are the
// templates of mk-acc-amd-pack.h, instantiated here with the reference's types and
// executed on stand-in types by tests/cpp/adapter_pack.cpp (layout checks on the
// CPU; engine-vs-oracle on an MI355X).
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
#include "mk-acc-amd-pack.h"

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace lbcrypto {

class UniEncAccumulatorAMD final : public UniEncAccumulator {
    // NATIVE_SIZE=32 -> uint32_t words, NATIVE_SIZE=64 -> uint64_t (mkacc_*_u64 entry points)
    using Word = NativeInteger::Integer;
    // one engine context, or (device list of two or more) a group of them
    int EngineEval(const uint32_t* ct, uint32_t* acc, size_t B) const {
        return m_group ? mkacc_group_eval_batch(m_group, ct, acc, acc, B) : mkacc_eval_batch(m_ctx, ct, acc, acc, B);
    }
    int EngineEval(const uint32_t* ct, uint64_t* acc, size_t B) const {
        return m_group ? mkacc_group_eval_batch_u64(m_group, ct, acc, acc, B)
                       : mkacc_eval_batch_u64(m_ctx, ct, acc, acc, B);
    }
    int EngineUpload(const uint32_t* evk, const uint32_t* pkey) const {
        return m_group ? mkacc_group_upload_keys(m_group, evk, pkey) : mkacc_upload_keys(m_ctx, evk, pkey);
    }
    int EngineUpload(const uint64_t* evk, const uint64_t* pkey) const {
        return m_group ? mkacc_group_upload_keys_u64(m_group, evk, pkey) : mkacc_upload_keys_u64(m_ctx, evk, pkey);
    }
    int EngineUploadKSK2(const mkacc_ks_params& ks, const uint32_t* w) const {
        return m_group ? mkacc_group_upload_ksk_mntru(m_group, &ks, w) : mkacc_upload_ksk_mntru(m_ctx, &ks, w);
    }
    int EngineUploadKSK(const mkacc_ks_params& ks, const uint32_t* wa, const uint32_t* wb) const {
        return m_group ? mkacc_group_upload_ksk_mklwe(m_group, &ks, wa, wb) : mkacc_upload_ksk_mklwe(m_ctx, &ks, wa, wb);
    }
    // member 0 answers the shape queries (every member has the same parameters)
    mkacc_ctx* Ctx0() const { return m_group ? mkacc_group_member(m_group, 0) : m_ctx; }

public:
    explicit UniEncAccumulatorAMD(BINFHE_METHOD method, int device = 0)
        : UniEncAccumulatorAMD(method, std::vector<int>{device}) {}
    // Two or more devices: every batch (EvalAccBatch, EvalNANDBatch) shards over them.
    UniEncAccumulatorAMD(BINFHE_METHOD method, std::vector<int> devices)
        : m_method(method), m_devices(std::move(devices)) {
        if (m_devices.empty())
            OPENFHE_THROW(config_error, "UniEncAccumulatorAMD: empty device list");
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
        if (m_group)
            mkacc_group_destroy(m_group);
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
        Prepare(params, ek, n, (m_method == MKNTRU || !Ctx0()) ? q : m_p.q);
        UploadKeys(ek, Pkey);
        std::vector<uint32_t> c(B * k * n);
        std::vector<Word> a(B * k * N);
        for (size_t b = 0; b < B; ++b) {
            if (acc[b] == nullptr || acc[b]->GetElements().size() != k)
                OPENFHE_THROW(config_error, "EvalAccBatch: accumulator has the wrong number of parties");
            mkacc_pack::pack_vectors(ct[b], k, n, c.data() + b * k * n, Fail);
            for (uint32_t u = 0; u < k; ++u) {
                const NativePoly& p = acc[b]->GetElements()[u];
                if (p.GetFormat() != Format::EVALUATION)
                    OPENFHE_THROW(config_error, "EvalAccBatch: accumulator must be in EVALUATION format");
                mkacc_pack::pack_poly(p, N, a.data() + (b * k + u) * N, Fail);
            }
        }
        Check(EngineEval(c.data(), a.data(), B));
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
        Check(m_group ? mkacc_group_eval_nand_mntru(m_group, nand.data(), a1.data(), a2.data(), out.data(), B)
                      : mkacc_eval_nand_mntru(m_ctx, nand.data(), a1.data(), a2.data(), out.data(), B));
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
        Check(m_group ? mkacc_group_eval_nand_mklwe(m_group, a1.data(), b1.data(), a2.data(), b2.data(), oa.data(),
                                                    ob.data(), B)
                      : mkacc_eval_nand_mklwe(m_ctx, a1.data(), b1.data(), a2.data(), b2.data(), oa.data(), ob.data(), B));
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
    static void Fail(const char* what) { OPENFHE_THROW(config_error, what); }

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
        if (Ctx0() && p.k == m_p.k && p.n == m_p.n && p.N == m_p.N && p.Q == m_p.Q && p.q == m_p.q &&
            p.baseG == m_p.baseG && p.digitsG == m_p.digitsG && p.root == m_p.root)
            return;
        if (m_ctx)
            mkacc_destroy(m_ctx);
        if (m_group)
            mkacc_group_destroy(m_group);
        m_ctx   = nullptr;
        m_group = nullptr;
        m_key.reset();
        m_ksk2.reset();
        m_ksk.reset();
        if (m_devices.size() > 1)
            Check(mkacc_group_create(&p, m_devices.data(), static_cast<uint32_t>(m_devices.size()), &m_group));
        else
            Check(mkacc_create(&p, m_devices[0], &m_ctx));
        m_p = p;
    }

    // Flatten (*ek)[u][j][i] -> GetElements()[digit][0|1] into [k][nk][n+1][dg][2][N] once per key object.
    // Entries the reference leaves empty ((*ek)[u][1][n], and (*ek)[u][0][n] for u > 0,
    // mk-acc-xzw.cpp:66-80) are unused by EvalAcc and sent as zeros.
    void UploadKeys(ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey) const {
        const uint32_t k = m_p.k, N = m_p.N, dg = m_p.digitsG - 1, n1 = m_p.n + 1;
        const uint32_t nk = m_method == MKNTRU ? 2 : 1;
        std::vector<Word> pk(mkacc_pkey_words(Ctx0()));  // [k][dg][N]
        mkacc_pack::pack_pkey(Pkey, k, dg, N, pk.data(), Fail);
        // Pkey arrives by value on every call, so it is compared by content; the
        // key object is held, so its address cannot be recycled while cached.
        if (m_key == ek && m_pkey == pk)
            return;
        std::vector<Word> evk(mkacc_evk_words(Ctx0()));
        mkacc_pack::pack_evk(ek->GetElements(), k, nk, n1, dg, N, evk.data(), Fail);
        m_key.reset();
        Check(EngineUpload(evk.data(), pk.data()));
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
        std::vector<uint32_t> w(size_t(k) * N * dks * n);
        mkacc_pack::pack_ksk2(K->GetElements(), k, N, dks, n, w.data(), Fail);   // [k][baseKS][N*dks][n]
        m_ksk2.reset();
        Check(EngineUploadKSK2(ks, w.data()));
        m_ksk2 = K;
    }

    // MK-LWE KeySwitch key (mklwe-pke.cpp:176-258): A [k][N][baseKS][dks][n], B [k][N][baseKS][dks].
    void UploadKSK(const mkacc_ks_params& ks, ConstMKLWESwitchingKey& K) const {
        if (K == nullptr)
            OPENFHE_THROW(config_error, "key-switching key has not been generated (MKBTKeyGen)");
        if (m_ksk == K)
            return;
        const uint32_t k = m_p.k, N = m_p.N, n = ks.n_out, base = ks.baseKS, dks = mkacc_ks_digits(&ks);
        std::vector<uint32_t> wa(size_t(k) * N * base * dks * n), wb(size_t(k) * N * base * dks);
        mkacc_pack::pack_lwe_ksk(K->GetElementsA(), K->GetElementsB(), k, N, base, dks, n, wa.data(), wb.data(), Fail);
        m_ksk.reset();
        Check(EngineUploadKSK(ks, wa.data(), wb.data()));
        m_ksk = K;
    }

    static void PackMNTRU(const MNTRUCiphertextImpl& ct, uint32_t* dst, uint32_t k, uint32_t n) {
        mkacc_pack::pack_vectors(ct.GetElements(), k, n, dst, Fail);
    }
    static void PackMKLWE(const MKLWECiphertextImpl& ct, uint32_t* dst, uint32_t k, uint32_t n) {
        mkacc_pack::pack_vectors(ct.GetA(), k, n, dst, Fail);
    }

    BINFHE_METHOD m_method;
    std::vector<int> m_devices;
    std::shared_ptr<UniEncAccumulator> m_cpu;  // reference XZW / XZW_B: KeyGenAcc
    mutable std::mutex m_mu;
    mutable mkacc_ctx* m_ctx     = nullptr;   // one device
    mutable mkacc_group* m_group = nullptr;   // two or more
    mutable mkacc_params m_p{};
    mutable std::shared_ptr<const UniEncACCKeyImpl> m_key;
    mutable std::vector<Word> m_pkey;
    mutable std::shared_ptr<const MNTRUSwitchingKey2Impl> m_ksk2;
    mutable std::shared_ptr<const MKLWESwitchingKeyImpl> m_ksk;
};

}  // namespace lbcrypto

#endif  // MK_ACC_AMD_H
