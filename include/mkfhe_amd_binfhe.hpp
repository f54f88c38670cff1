// mkfhe_amd_binfhe.hpp -- C++ host mirror of the reference's multi-key
// accumulator plugin interface, over the C ABI in mkfhe_amd.h.
//
// Mirrors (names, argument meaning, error behaviour) of the reference:
//   class UniEncAccumulator            src/binfhe/include/mk-acc.h:55-80
//   UniEncAccumulatorXZW::EvalAcc      src/binfhe/lib/mk-acc-xzw.cpp:89-130   (MKNTRU)
//   UniEncAccumulatorXZW_B::EvalAcc    src/binfhe/lib/mk-acc-xzw_B.cpp:103-132 (MKNTRU_B, MKNTRU_LWE)
//   SignedDigitDecompose(poly)         src/binfhe/lib/mk-acc.cpp:54-80
//   UniEncCryptoParams                 src/binfhe/include/mk-cryptoparameters.h:124-181
//   UniEncEvalKeyImpl [dg][2]          src/binfhe/include/mk-evalkey.h:33-35
//   UniEncACCKeyImpl [k][nk][n+1]      src/binfhe/include/mk-acckey.h:44-51
//   MKACCCiphertextImpl (k polys)      src/binfhe/include/mk-ciphertext.h:68-71
//   BINFHE_METHOD values               src/binfhe/include/binfhe-constants.h:129-137
//   accumulator choice by method       src/binfhe/include/binfhe-base-scheme.h:137-151
//   OPENFHE_THROW(config_error, ...)   src/core/include/utils/exception.h:162
//
// Every evaluation runs on the HIP engine (libmkfhe_amd.so); there is no CPU
// path.  Link with -lmkfhe_amd.  Header-only.
#ifndef MKFHE_AMD_BINFHE_HPP
#define MKFHE_AMD_BINFHE_HPP

#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "mkfhe_amd.h"

namespace mkfhe_amd {

// ---- exceptions (reference exception.h: openfhe_error and subclasses) -------
class openfhe_error : public std::runtime_error {
public:
    explicit openfhe_error(const std::string& m) : std::runtime_error(m) {}
};
class config_error : public openfhe_error {
public:
    using openfhe_error::openfhe_error;
};
class math_error : public openfhe_error {
public:
    using openfhe_error::openfhe_error;
};
class not_implemented_error : public openfhe_error {
public:
    using openfhe_error::openfhe_error;
};
// device / runtime failure (no reference counterpart: the reference has no device)
class device_error : public openfhe_error {
public:
    using openfhe_error::openfhe_error;
};

// Translate an MKACC status into the reference's exception types.
inline void check(int rc) {
    if (rc == MKACC_OK) return;
    const std::string msg = mkacc_last_error();
    switch (rc) {
        case MKACC_E_ARG:
        case MKACC_E_NOKEYS:
        case MKACC_E_UNSUPPORTED: throw config_error(msg);
        case MKACC_E_RANGE: throw math_error(msg);
        default: throw device_error(msg);
    }
}

// ---- enums (binfhe-constants.h:129-137) ---------------------------------------
enum BINFHE_METHOD { INVALID_METHOD = 0, AP, GINX, LMKCDEY, MKNTRU, MKNTRU_B, MKNTRU_LWE };
enum Format { EVALUATION = 0, COEFFICIENT = 1 };

inline uint32_t to_abi_method(BINFHE_METHOD m) {
    switch (m) {
        case MKNTRU: return MKACC_METHOD_MKNTRU;
        case MKNTRU_B: return MKACC_METHOD_MKNTRU_B;
        case MKNTRU_LWE: return MKACC_METHOD_MKNTRU_LWE;
        default: throw config_error("method is invalid");
    }
}

// ---- ring elements ------------------------------------------------------------
// NativePoly over Z_Q[X]/(X^N + 1): N canonical residues in the reference's
// EVALUATION (bit-reversed NTT) or COEFFICIENT order.
using NativeVector = std::vector<uint64_t>;
struct NativePoly {
    NativeVector values;
    Format format = EVALUATION;
    NativePoly() = default;
    NativePoly(uint32_t N, Format f) : values(N, 0), format(f) {}
    NativePoly(NativeVector v, Format f) : values(std::move(v)), format(f) {}
    uint32_t GetLength() const { return (uint32_t)values.size(); }
    Format GetFormat() const { return format; }
    uint64_t& operator[](size_t i) { return values[i]; }
    const uint64_t& operator[](size_t i) const { return values[i]; }
    bool operator==(const NativePoly& o) const { return format == o.format && values == o.values; }
};

// ---- parameters ----------------------------------------------------------------
// The UniEncCryptoParams fields EvalAcc reads.  digitsG is derived as the
// reference does (ceil(log Q / log B_g), mk-cryptoparameters.h:141-142).
class UniEncCryptoParams {
public:
    UniEncCryptoParams(uint32_t k, uint32_t N, uint64_t Q, uint64_t q, uint32_t baseG, BINFHE_METHOD method,
                       uint32_t n)
        : m_method(method) {
        if (baseG < 2 || (baseG & (baseG - 1))) throw config_error("Gadget base should be a power of two.");
        mkacc_params p{};
        p.method = to_abi_method(method);
        p.k = k;
        p.n = n;
        p.N = N;
        p.Q = Q;
        p.q = q;
        p.baseG = baseG;
        m_p = p;
    }
    // BINFHE_PARAMSET by name (binfhecontext.cpp:129-144), e.g. "STD128_MKNTRU"
    static std::shared_ptr<UniEncCryptoParams> FromParamSet(const std::string& name, BINFHE_METHOD method) {
        mkacc_params p{};
        check(mkacc_paramset(name.c_str(), to_abi_method(method), &p));
        auto r = std::make_shared<UniEncCryptoParams>(p.k, p.N, p.Q, p.q, p.baseG, method, p.n);
        r->m_p = p;
        return r;
    }
    uint32_t Getk() const { return m_p.k; }
    uint32_t GetN() const { return m_p.N; }
    uint32_t GetLatticeParam() const { return m_p.n; }
    uint64_t GetQ() const { return m_p.Q; }
    uint64_t Getq() const { return m_p.q; }
    uint32_t GetBaseG() const { return m_p.baseG; }
    // 0 until a context has derived it (see UniEncAccumulator::Params)
    uint32_t GetDigitsG() const { return m_p.digitsG; }
    BINFHE_METHOD GetMethod() const { return m_method; }
    const mkacc_params& abi() const { return m_p; }
    void set_abi(const mkacc_params& p) { m_p = p; }

private:
    mkacc_params m_p{};
    BINFHE_METHOD m_method;
};

// ---- keys and accumulator ciphertexts -----------------------------------------------
class UniEncEvalKeyImpl {
public:
    UniEncEvalKeyImpl() = default;
    UniEncEvalKeyImpl(uint32_t rows, uint32_t cols) : m_elements(rows, std::vector<NativePoly>(cols)) {}
    explicit UniEncEvalKeyImpl(std::vector<std::vector<NativePoly>> e) : m_elements(std::move(e)) {}
    const std::vector<std::vector<NativePoly>>& GetElements() const { return m_elements; }
    std::vector<std::vector<NativePoly>>& GetElements() { return m_elements; }

private:
    std::vector<std::vector<NativePoly>> m_elements;   // [digitsG-1][2]
};
using UniEncEvalKey = std::shared_ptr<UniEncEvalKeyImpl>;

class UniEncACCKeyImpl {
public:
    UniEncACCKeyImpl() = default;
    UniEncACCKeyImpl(uint32_t d1, uint32_t d2, uint32_t d3)
        : m_key(d1, std::vector<std::vector<UniEncEvalKey>>(d2, std::vector<UniEncEvalKey>(d3))) {}
    const std::vector<std::vector<std::vector<UniEncEvalKey>>>& GetElements() const { return m_key; }
    std::vector<std::vector<std::vector<UniEncEvalKey>>>& GetElements() { return m_key; }
    // [u][j][i]
    std::vector<std::vector<UniEncEvalKey>>& operator[](uint32_t i) { return m_key[i]; }
    const std::vector<std::vector<UniEncEvalKey>>& operator[](uint32_t i) const { return m_key[i]; }

private:
    std::vector<std::vector<std::vector<UniEncEvalKey>>> m_key;   // [k][2 (XZW) | 1 (XZW_B)][n+1]
};
using UniEncACCKey = std::shared_ptr<UniEncACCKeyImpl>;
using ConstUniEncACCKey = const std::shared_ptr<const UniEncACCKeyImpl>;

class MKACCCiphertextImpl {
public:
    MKACCCiphertextImpl() = default;
    explicit MKACCCiphertextImpl(std::vector<NativePoly> e) : m_elements(std::move(e)) {}
    const std::vector<NativePoly>& GetElements() const { return m_elements; }
    std::vector<NativePoly>& GetElements() { return m_elements; }

private:
    std::vector<NativePoly> m_elements;   // (c_1, ..., c_k), EVALUATION
};
using MKACCCiphertext = std::shared_ptr<MKACCCiphertextImpl>;

// ---- device context ----------------------------------------------------------------
// One mkacc_ctx per accumulator object (one HIP stream); keys are flattened
// into the C-ABI layout and uploaded once per distinct key object.
class DeviceContext {
public:
    DeviceContext(const mkacc_params& p, int device) {
        check(mkacc_create(&p, device, &m_ctx));
        check(mkacc_get_params(m_ctx, &m_p));
    }
    ~DeviceContext() { mkacc_destroy(m_ctx); }
    DeviceContext(const DeviceContext&) = delete;
    DeviceContext& operator=(const DeviceContext&) = delete;
    mkacc_ctx* get() const { return m_ctx; }
    const mkacc_params& params() const { return m_p; }
    const void* key_token = nullptr;
    const void* pkey_token = nullptr;

private:
    mkacc_ctx* m_ctx = nullptr;
    mkacc_params m_p{};
};

// ---- the accumulator plugin seam (mk-acc.h:55-80) -----------------------------------
class UniEncAccumulator {
public:
    explicit UniEncAccumulator(int device = 0) : m_device(device) {}
    virtual ~UniEncAccumulator() = default;

    // acc (EVALUATION) <- EvalAcc(acc); ct[u] holds the n words of party u
    // (XZW: mod q, scaled internally by floor(.*2N/q); XZW_B: already mod 2N).
    // Pkey and skf are taken by value as in the reference; skf is unused.
    virtual void EvalAcc(const std::shared_ptr<UniEncCryptoParams>& params, ConstUniEncACCKey& ek,
                         std::vector<std::vector<NativePoly>> Pkey, std::vector<NativePoly> skf,
                         MKACCCiphertext& acc, const std::vector<NativeVector>& ct) const {
        (void)skf;
        std::vector<MKACCCiphertext> accs{acc};
        std::vector<std::vector<NativeVector>> cts{ct};
        EvalAccBatch(params, ek, Pkey, accs, cts);
    }

    // Batch extension: B independent gates in one pass of the engine.
    void EvalAccBatch(const std::shared_ptr<UniEncCryptoParams>& params, ConstUniEncACCKey& ek,
                      const std::vector<std::vector<NativePoly>>& Pkey, std::vector<MKACCCiphertext>& accs,
                      const std::vector<std::vector<NativeVector>>& cts) const {
        if (!ek)
            throw config_error(
                "Bootstrapping keys have not been generated. Please call MKBTKeyGen before calling bootstrapping.");
        check_method(params->GetMethod());
        DeviceContext& dc = context(*params);
        upload(dc, ek, Pkey);
        const mkacc_params& p = dc.params();
        const size_t B = accs.size();
        if (cts.size() != B) throw config_error("one ciphertext per accumulator is required");
        std::vector<uint32_t> hct(B * p.k * p.n), hacc(B * p.k * p.N);
        for (size_t b = 0; b < B; ++b) {
            if (cts[b].size() != p.k) throw config_error("ciphertext must hold k vectors");
            for (uint32_t u = 0; u < p.k; ++u) {
                if (cts[b][u].size() != p.n) throw config_error("ciphertext vector length must be n");
                for (uint32_t i = 0; i < p.n; ++i) hct[(b * p.k + u) * p.n + i] = (uint32_t)cts[b][u][i];
            }
            const auto& el = accs[b]->GetElements();
            if (el.size() != p.k) throw config_error("accumulator must hold k polynomials");
            for (uint32_t u = 0; u < p.k; ++u) {
                if (el[u].GetLength() != p.N || el[u].format != EVALUATION)
                    throw config_error("accumulator polynomials must be length-N EVALUATION");
                for (uint32_t j = 0; j < p.N; ++j) {
                    if (el[u][j] >= p.Q) throw math_error("accumulator word not a canonical residue mod Q");
                    hacc[(b * p.k + u) * p.N + j] = (uint32_t)el[u][j];
                }
            }
        }
        check(mkacc_eval_batch(dc.get(), hct.data(), hacc.data(), hacc.data(), B));
        for (size_t b = 0; b < B; ++b) {
            auto& el = accs[b]->GetElements();
            for (uint32_t u = 0; u < p.k; ++u)
                for (uint32_t j = 0; j < p.N; ++j) el[u][j] = hacc[(b * p.k + u) * p.N + j];
        }
    }

    // SignedDigitDecompose(params, input, output) (mk-acc.cpp:54-80): output
    // receives digitsG - 1 COEFFICIENT polys (the first digit is dropped).
    void SignedDigitDecompose(const std::shared_ptr<UniEncCryptoParams>& params, const NativePoly& input,
                              std::vector<NativePoly>& output) const {
        DeviceContext& dc = context(*params);
        const mkacc_params& p = dc.params();
        const uint32_t dg = p.digitsG - 1;
        std::vector<uint32_t> in(p.N), out((size_t)dg * p.N);
        for (uint32_t j = 0; j < p.N; ++j) in[j] = (uint32_t)input[j];
        check(mkacc_sdd(dc.get(), in.data(), out.data(), 1));
        output.assign(dg, NativePoly(p.N, COEFFICIENT));
        for (uint32_t d = 0; d < dg; ++d)
            for (uint32_t j = 0; j < p.N; ++j) output[d][j] = out[(size_t)d * p.N + j];
    }

    // NativePoly::SetFormat through the engine's NTT (poly-impl.h:412-432)
    void SetFormat(const std::shared_ptr<UniEncCryptoParams>& params, NativePoly& poly, Format f) const {
        if (poly.format == f) return;
        DeviceContext& dc = context(*params);
        std::vector<uint32_t> a(poly.values.begin(), poly.values.end()), o(a.size());
        check(f == EVALUATION ? mkacc_ntt_forward(dc.get(), a.data(), o.data(), 1)
                              : mkacc_ntt_inverse(dc.get(), a.data(), o.data(), 1));
        poly.values.assign(o.begin(), o.end());
        poly.format = f;
    }

    // Effective parameters (digitsG, root derived) of the device context.
    mkacc_params Params(const UniEncCryptoParams& params) const { return context(params).params(); }

protected:
    virtual void check_method(BINFHE_METHOD m) const = 0;

private:
    DeviceContext& context(const UniEncCryptoParams& params) const {
        std::lock_guard<std::mutex> g(m_mu);
        if (!m_ctx || std::memcmp(&m_key, &params.abi(), sizeof(mkacc_params)) != 0) {
            m_ctx.reset();
            m_ctx = std::make_unique<DeviceContext>(params.abi(), m_device);
            m_key = params.abi();
        }
        return *m_ctx;
    }

public:
    // Flatten ek [k][nk][n+1] x [dg][2] x N and Pkey [k][dg] x N into the C-ABI
    // layout and upload them once per key object.
    static void upload(DeviceContext& dc, ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey) {
        if (dc.key_token == ek.get() && dc.pkey_token == (const void*)Pkey.data()) return;
        const mkacc_params& p = dc.params();
        const uint32_t dg = p.digitsG - 1, nk = p.method == MKACC_METHOD_MKNTRU ? 2 : 1, N = p.N;
        const auto& K = ek->GetElements();
        if (K.size() != p.k) throw config_error("accumulator key must have k parties");
        std::vector<uint32_t> evk(mkacc_evk_words(dc.get())), pk(mkacc_pkey_words(dc.get()));
        size_t o = 0;
        for (uint32_t u = 0; u < p.k; ++u) {
            if (K[u].size() < nk) throw config_error("accumulator key has too few key sets");
            for (uint32_t j = 0; j < nk; ++j) {
                if (K[u][j].size() != p.n + 1) throw config_error("accumulator key must have n+1 entries");
                for (uint32_t i = 0; i <= p.n; ++i) {
                    const auto& E = K[u][j][i]->GetElements();
                    if (E.size() != dg) throw config_error("eval key must have digitsG-1 rows");
                    for (uint32_t d = 0; d < dg; ++d)
                        for (uint32_t c = 0; c < 2; ++c, o += N)
                            for (uint32_t s = 0; s < N; ++s) evk[o + s] = (uint32_t)E[d][c][s];
                }
            }
        }
        if (Pkey.size() != p.k) throw config_error("Pkey must have k parties");
        for (uint32_t u = 0; u < p.k; ++u) {
            if (Pkey[u].size() != dg) throw config_error("Pkey must have digitsG-1 polys per party");
            for (uint32_t d = 0; d < dg; ++d)
                for (uint32_t s = 0; s < N; ++s) pk[((size_t)u * dg + d) * N + s] = (uint32_t)Pkey[u][d][s];
        }
        check(mkacc_upload_keys(dc.get(), evk.data(), pk.data()));
        dc.key_token = ek.get();
        dc.pkey_token = Pkey.data();
    }

private:
    int m_device;
    mutable std::mutex m_mu;
    mutable std::unique_ptr<DeviceContext> m_ctx;
    mutable mkacc_params m_key{};
};

// MKNTRU accumulator, ternary secret (mk-acc-xzw.cpp)
class UniEncAccumulatorXZW : public UniEncAccumulator {
public:
    using UniEncAccumulator::UniEncAccumulator;

protected:
    void check_method(BINFHE_METHOD m) const override {
        if (m != MKNTRU) throw config_error("method is invalid for UniEncAccumulatorXZW");
    }
};

// MKNTRU_B / MKNTRU_LWE accumulator, binary secret (mk-acc-xzw_B.cpp)
class UniEncAccumulatorXZW_B : public UniEncAccumulator {
public:
    using UniEncAccumulator::UniEncAccumulator;

protected:
    void check_method(BINFHE_METHOD m) const override {
        if (m != MKNTRU_B && m != MKNTRU_LWE) throw config_error("method is invalid for UniEncAccumulatorXZW_B");
    }
};

// BinFHEScheme(method)'s accumulator choice (binfhe-base-scheme.h:137-151)
inline std::shared_ptr<UniEncAccumulator> MakeUniEncAccumulator(BINFHE_METHOD method, int device = 0) {
    if (method == MKNTRU) return std::make_shared<UniEncAccumulatorXZW>(device);
    if (method == MKNTRU_B || method == MKNTRU_LWE) return std::make_shared<UniEncAccumulatorXZW_B>(device);
    throw config_error("method is invalid");
}


// =====================================================================================
// Gate level: BinFHEContext::EvalBinGate for MK-NTRU and MK-LWE
// (binfhecontext.h:336-338, binfhe-base-scheme.cpp:380-515).
// =====================================================================================

// binfhe-constants.h:143
enum BINGATE { OR, AND, NOR, NAND, XOR_FAST, XNOR_FAST, MAJORITY, AND3, OR3, AND4, OR4, CMUX, XOR, XNOR };

// The multi-key parameter sets of binfhe-constants.h:95-110 (binfhecontext.cpp:129-144)
enum BINFHE_PARAMSET {
    STD128_MKNTRU, STD128_MKNTRU_2, STD128_MKNTRU_3, STD128_MKNTRU_4,
    STD128_MKNTRU_LWE, STD128_MKNTRU_LWE_2, STD128_MKNTRU_LWE_3, STD128_MKNTRU_LWE_4,
    STD100_MKNTRU, STD100_MKNTRU_2, STD100_MKNTRU_3, STD100_MKNTRU_4,
    STD100_MKNTRU_LWE, STD100_MKNTRU_LWE_2, STD100_MKNTRU_LWE_3, STD100_MKNTRU_LWE_4,
};
inline const char* ParamSetName(BINFHE_PARAMSET s) {
    static const char* names[] = {
        "STD128_MKNTRU", "STD128_MKNTRU_2", "STD128_MKNTRU_3", "STD128_MKNTRU_4",
        "STD128_MKNTRU_LWE", "STD128_MKNTRU_LWE_2", "STD128_MKNTRU_LWE_3", "STD128_MKNTRU_LWE_4",
        "STD100_MKNTRU", "STD100_MKNTRU_2", "STD100_MKNTRU_3", "STD100_MKNTRU_4",
        "STD100_MKNTRU_LWE", "STD100_MKNTRU_LWE_2", "STD100_MKNTRU_LWE_3", "STD100_MKNTRU_LWE_4"};
    return names[s];
}

// MNTRU ciphertext: k vectors of n words mod q (mntru-ciphertext.h:28-31, p = 4)
class MNTRUCiphertextImpl {
public:
    MNTRUCiphertextImpl() = default;
    MNTRUCiphertextImpl(std::vector<NativeVector> e, uint64_t q) : m_elements(std::move(e)), m_q(q) {}
    const std::vector<NativeVector>& GetElements() const { return m_elements; }
    std::vector<NativeVector>& GetElements() { return m_elements; }
    uint64_t GetModulus() const { return m_q; }
    uint64_t GetptModulus() const { return m_p; }
    uint32_t Getk() const { return (uint32_t)m_elements.size(); }
    uint32_t GetLength() const { return m_elements.empty() ? 0 : (uint32_t)m_elements[0].size(); }

private:
    std::vector<NativeVector> m_elements;
    uint64_t m_q = 0, m_p = 4;
};
using MNTRUCiphertext = std::shared_ptr<MNTRUCiphertextImpl>;
using ConstMNTRUCiphertext = const std::shared_ptr<const MNTRUCiphertextImpl>;

// MK-LWE ciphertext: (a_1..a_k, b) mod q (mklwe-ciphertext.h:55-58)
class MKLWECiphertextImpl {
public:
    MKLWECiphertextImpl() = default;
    MKLWECiphertextImpl(std::vector<NativeVector> a, uint64_t b, uint64_t q) : m_a(std::move(a)), m_b(b), m_q(q) {}
    const std::vector<NativeVector>& GetA() const { return m_a; }
    std::vector<NativeVector>& GetA() { return m_a; }
    uint64_t GetB() const { return m_b; }
    uint64_t GetModulus() const { return m_q; }
    uint64_t GetptModulus() const { return m_p; }
    uint32_t Getk() const { return (uint32_t)m_a.size(); }
    uint32_t GetLength() const { return m_a.empty() ? 0 : (uint32_t)m_a[0].size(); }

private:
    std::vector<NativeVector> m_a;
    uint64_t m_b = 0, m_q = 0, m_p = 4;
};
using MKLWECiphertext = std::shared_ptr<MKLWECiphertextImpl>;
using ConstMKLWECiphertext = const std::shared_ptr<const MKLWECiphertextImpl>;

// KeySwitchGen2's table KSK2[u][j][l] = j * KSK[u][l] mod qKS, [k][baseKS][N*dks]
// of n-vectors (mntru-pke.cpp:624-760).  The engine reads KSK2[u][1].
class MNTRUSwitchingKey2Impl {
public:
    explicit MNTRUSwitchingKey2Impl(std::vector<std::vector<std::vector<NativeVector>>> k) : m_key(std::move(k)) {}
    const std::vector<std::vector<std::vector<NativeVector>>>& GetElements() const { return m_key; }

private:
    std::vector<std::vector<std::vector<NativeVector>>> m_key;
};
using MNTRUSwitchingKey2 = std::shared_ptr<const MNTRUSwitchingKey2Impl>;

// MK-LWE KeySwitchGen (mklwe-pke.cpp:176-258): A[u][j][d][t] n-vectors, B[u][j][d][t]
class MKLWESwitchingKeyImpl {
public:
    using A4 = std::vector<std::vector<std::vector<std::vector<NativeVector>>>>;
    using B4 = std::vector<std::vector<std::vector<std::vector<uint64_t>>>>;
    MKLWESwitchingKeyImpl(A4 a, B4 b) : m_a(std::move(a)), m_b(std::move(b)) {}
    const A4& GetElementsA() const { return m_a; }
    const B4& GetElementsB() const { return m_b; }

private:
    A4 m_a;
    B4 m_b;
};
using MKLWESwitchingKey = std::shared_ptr<const MKLWESwitchingKeyImpl>;

// The fields of the reference UniEncBTKey (binfhe-base-scheme.h:65-83) the
// gate path reads.
struct UniEncBTKey {
    UniEncACCKey BSkey;
    MNTRUSwitchingKey2 KSkey2;
    MKLWESwitchingKey LKSkey;
    std::vector<std::vector<NativePoly>> Pkey;
    std::vector<NativePoly> f;
};

// BinFHEContext subset for multi-key NAND gates on one MI355X.  Key generation
// (MNTRU_KeyGen / MKBTKeyGen / ctGateGen) needs NTL in the reference and is
// not part of this engine: keys are loaded with BTKeyLoad / SetctNAND.
class BinFHEContext {
public:
    void GenerateBinFHEContext(BINFHE_PARAMSET set, BINFHE_METHOD method, int device = 0) {
        if (method != MKNTRU && method != MKNTRU_B && method != MKNTRU_LWE)
            throw config_error("method is invalid");
        m_method = method;
        m_params = UniEncCryptoParams::FromParamSet(ParamSetName(set), method);
        m_dc = std::make_unique<DeviceContext>(m_params->abi(), device);
        m_params->set_abi(m_dc->params());
        m_keys = false;
        m_ctNAND.reset();
    }
    // custom parameters (the reference's explicit-parameter overload, binfhecontext.h:94)
    void GenerateBinFHEContext(const UniEncCryptoParams& params, int device = 0) {
        m_method = params.GetMethod();
        m_params = std::make_shared<UniEncCryptoParams>(params);
        m_dc = std::make_unique<DeviceContext>(m_params->abi(), device);
        m_params->set_abi(m_dc->params());
        m_keys = false;
        m_ctNAND.reset();
    }
    const std::shared_ptr<UniEncCryptoParams>& GetParams() const { return m_params; }
    // modKS = mod and baseKS = 32 in every MK set (binfhecontext.cpp:129-144)
    mkacc_ks_params GetKSParams() const { return mkacc_ks_params{m_params->Getq(), 32, m_params->GetLatticeParam()}; }

    void BTKeyLoad(const UniEncBTKey& ek) {
        need_context();
        if (!ek.BSkey) throw config_error("BSkey is empty");
        UniEncAccumulator::upload(*m_dc, ek.BSkey, ek.Pkey);
        const mkacc_ks_params ks = GetKSParams();
        const uint32_t k = m_params->Getk(), N = m_params->GetN(), n = ks.n_out;
        const uint32_t dks = mkacc_ks_digits(&ks);
        if (m_method == MKNTRU) {
            if (!ek.KSkey2) throw config_error("KSkey2 is empty");
            const auto& K2 = ek.KSkey2->GetElements();
            if (K2.size() != k) throw config_error("KSkey2 must have k parties");
            std::vector<uint32_t> h((size_t)k * N * dks * n);
            for (uint32_t u = 0; u < k; ++u) {
                if (K2[u].size() < 2 || K2[u][1].size() != (size_t)N * dks)
                    throw config_error("KSkey2[u] must be [baseKS][N*dks]");
                for (size_t l = 0; l < (size_t)N * dks; ++l) {
                    const NativeVector& row = K2[u][1][l];
                    if (row.size() != n) throw config_error("KSkey2 rows must have n words");
                    for (uint32_t i = 0; i < n; ++i) h[((size_t)u * N * dks + l) * n + i] = (uint32_t)row[i];
                }
            }
            check(mkacc_upload_ksk_mntru(m_dc->get(), &ks, h.data()));
        } else {
            if (!ek.LKSkey) throw config_error("LKSkey is empty");
            const auto& A = ek.LKSkey->GetElementsA();
            const auto& Bk = ek.LKSkey->GetElementsB();
            const size_t rows = (size_t)k * N * ks.baseKS * dks;
            std::vector<uint32_t> ha(rows * n), hb(rows);
            size_t r = 0;
            for (uint32_t u = 0; u < k; ++u)
                for (uint32_t j = 0; j < N; ++j)
                    for (uint32_t d = 0; d < ks.baseKS; ++d)
                        for (uint32_t t = 0; t < dks; ++t, ++r) {
                            const NativeVector& row = A.at(u).at(j).at(d).at(t);
                            if (row.size() != n) throw config_error("LKSkey rows must have n words");
                            for (uint32_t i = 0; i < n; ++i) ha[r * n + i] = (uint32_t)row[i];
                            hb[r] = (uint32_t)Bk.at(u).at(j).at(d).at(t);
                        }
            check(mkacc_upload_ksk_mklwe(m_dc->get(), &ks, ha.data(), hb.data()));
        }
        m_keys = true;
    }
    // the NAND constant ciphertext that ctGateGen produces (binfhe-base-scheme.cpp:340-376)
    void SetctNAND(MNTRUCiphertext ct) { m_ctNAND = std::move(ct); }

    MNTRUCiphertext EvalBinGate(BINGATE gate, ConstMNTRUCiphertext& ct1, ConstMNTRUCiphertext& ct2) const {
        if (ct1 == ct2) throw config_error("Input ciphertexts should be independant");
        return EvalBinGate(gate, std::vector<MNTRUCiphertext>{std::const_pointer_cast<MNTRUCiphertextImpl>(ct1)},
                           std::vector<MNTRUCiphertext>{std::const_pointer_cast<MNTRUCiphertextImpl>(ct2)})[0];
    }
    MKLWECiphertext EvalBinGate(BINGATE gate, ConstMKLWECiphertext& ct1, ConstMKLWECiphertext& ct2) const {
        if (ct1 == ct2) throw config_error("Input ciphertexts should be independant");
        return EvalBinGate(gate, std::vector<MKLWECiphertext>{std::const_pointer_cast<MKLWECiphertextImpl>(ct1)},
                           std::vector<MKLWECiphertext>{std::const_pointer_cast<MKLWECiphertextImpl>(ct2)})[0];
    }

    // Batch extension: B independent NAND gates in one engine pass.
    std::vector<MNTRUCiphertext> EvalBinGate(BINGATE gate, const std::vector<MNTRUCiphertext>& ct1,
                                             const std::vector<MNTRUCiphertext>& ct2) const {
        need_gate(gate, MKNTRU);
        if (!m_ctNAND) throw config_error("ctNAND has not been generated (ctGateGen)");
        const uint32_t k = m_params->Getk(), n = m_params->GetLatticeParam();
        const size_t B = ct1.size();
        if (ct2.size() != B) throw config_error("ct1 and ct2 must have the same length");
        std::vector<uint32_t> a1(B * k * n), a2(B * k * n), nand(k * n), out(B * k * n);
        pack(*m_ctNAND, nand.data(), k, n);
        for (size_t b = 0; b < B; ++b) {
            if (ct1[b] == ct2[b]) throw config_error("Input ciphertexts should be independant");
            pack(*ct1[b], a1.data() + b * k * n, k, n);
            pack(*ct2[b], a2.data() + b * k * n, k, n);
        }
        check(mkacc_eval_nand_mntru(m_dc->get(), nand.data(), a1.data(), a2.data(), out.data(), B));
        std::vector<MNTRUCiphertext> res(B);
        for (size_t b = 0; b < B; ++b) {
            std::vector<NativeVector> e(k, NativeVector(n));
            for (uint32_t u = 0; u < k; ++u)
                for (uint32_t i = 0; i < n; ++i) e[u][i] = out[(b * k + u) * n + i];
            res[b] = std::make_shared<MNTRUCiphertextImpl>(std::move(e), GetKSParams().qKS);
        }
        return res;
    }
    std::vector<MKLWECiphertext> EvalBinGate(BINGATE gate, const std::vector<MKLWECiphertext>& ct1,
                                             const std::vector<MKLWECiphertext>& ct2) const {
        need_gate(gate, MKNTRU_LWE);
        const uint32_t k = m_params->Getk(), n = m_params->GetLatticeParam();
        const size_t B = ct1.size();
        if (ct2.size() != B) throw config_error("ct1 and ct2 must have the same length");
        std::vector<uint32_t> a1(B * k * n), a2(B * k * n), b1(B), b2(B), oa(B * k * n), ob(B);
        for (size_t b = 0; b < B; ++b) {
            if (ct1[b] == ct2[b]) throw config_error("Input ciphertexts should be independant");
            packA(*ct1[b], a1.data() + b * k * n, k, n);
            packA(*ct2[b], a2.data() + b * k * n, k, n);
            b1[b] = (uint32_t)ct1[b]->GetB();
            b2[b] = (uint32_t)ct2[b]->GetB();
        }
        check(mkacc_eval_nand_mklwe(m_dc->get(), a1.data(), b1.data(), a2.data(), b2.data(), oa.data(), ob.data(),
                                    B));
        std::vector<MKLWECiphertext> res(B);
        for (size_t b = 0; b < B; ++b) {
            std::vector<NativeVector> a(k, NativeVector(n));
            for (uint32_t u = 0; u < k; ++u)
                for (uint32_t i = 0; i < n; ++i) a[u][i] = oa[(b * k + u) * n + i];
            res[b] = std::make_shared<MKLWECiphertextImpl>(std::move(a), ob[b], GetKSParams().qKS);
        }
        return res;
    }

private:
    void need_context() const {
        if (!m_dc) throw config_error("call GenerateBinFHEContext first");
    }
    void need_gate(BINGATE gate, BINFHE_METHOD family) const {
        need_context();
        if (gate != NAND) throw not_implemented_error("only NAND is supported (ctGateGen, binfhe-base-scheme.cpp:341-342)");
        const bool lwe = m_method != MKNTRU;
        if (lwe != (family != MKNTRU)) throw config_error("ciphertext type does not match the context method");
        if (!m_keys)
            throw config_error(
                "Bootstrapping keys have not been generated. Please call MKBTKeyGen before calling bootstrapping.");
    }
    static void pack(const MNTRUCiphertextImpl& c, uint32_t* dst, uint32_t k, uint32_t n) {
        if (c.Getk() != k || c.GetLength() != n) throw config_error("ciphertext must be k x n");
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t i = 0; i < n; ++i) dst[u * n + i] = (uint32_t)c.GetElements()[u][i];
    }
    static void packA(const MKLWECiphertextImpl& c, uint32_t* dst, uint32_t k, uint32_t n) {
        if (c.Getk() != k || c.GetLength() != n) throw config_error("ciphertext must be k x n");
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t i = 0; i < n; ++i) dst[u * n + i] = (uint32_t)c.GetA()[u][i];
    }

    BINFHE_METHOD m_method = MKNTRU;
    std::shared_ptr<UniEncCryptoParams> m_params;
    std::unique_ptr<DeviceContext> m_dc;
    bool m_keys = false;
    MNTRUCiphertext m_ctNAND;
};

}  // namespace mkfhe_amd

#endif  // MKFHE_AMD_BINFHE_HPP
