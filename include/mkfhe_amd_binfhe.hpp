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

}  // namespace mkfhe_amd

#endif  // MKFHE_AMD_BINFHE_HPP
