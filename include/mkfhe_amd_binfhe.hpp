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
//   BinFHEContext MK subset            src/binfhe/include/binfhecontext.h:98-338
//     (GenerateBinFHEContext, MNTRU_KeyGen, MKLWE_KeyGen, MKBTKeyGen, ctGateGen,
//      Encrypt, EvalBinGate(NAND), Decrypt / Decrypt2 / DecryptNAND)
//
// Every evaluation runs on the HIP engine (libmkfhe_amd.so); there is no CPU
// path.  Key material comes from libmkfhe_keys.so (host C++, include/mkfhe_keys.h).
// Link with -lmkfhe_amd -lmkfhe_keys.  Header-only.
#ifndef MKFHE_AMD_BINFHE_HPP
#define MKFHE_AMD_BINFHE_HPP

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "mkfhe_amd.h"
#include "mkfhe_keys.h"

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

// MKBTKeyGen under RDefectPolicy::REJECT drew a bootstrapping key whose DggR
// sample r is nonzero (the reference's KeyGenXZW defect, mk-acc-xzw.cpp:160-167;
// include/mkfhe_keys.h)
class key_defect_error : public config_error {
public:
    using config_error::config_error;
};

// Translate a status of the key library (libmkfhe_keys, same codes) with its own error text.
inline void checkk(int rc) {
    if (rc == MKACC_OK) return;
    const std::string msg = mkkg_last_error();
    switch (rc) {
        case MKKG_E_RDEFECT: throw key_defect_error(msg);
        case MKACC_E_ARG:
        case MKACC_E_NOKEYS:
        case MKACC_E_UNSUPPORTED: throw config_error(msg);
        case MKACC_E_RANGE: throw math_error(msg);
        default: throw device_error(msg);
    }
}

// What MKBTKeyGen does about a bootstrapping key with DggR sample r != 0
// (mkkg_acc_keygen_ex): KEEP = the reference's keys (counted, GetRDefects()),
// REJECT = key_defect_error, RESAMPLE = redraw r in the affected slots.
enum class RDefectPolicy : uint32_t { KEEP = MKKG_RDEFECT_KEEP, REJECT = MKKG_RDEFECT_REJECT,
                                      RESAMPLE = MKKG_RDEFECT_RESAMPLE };

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
    // What is on the device: the key OBJECT itself is held (so its address
    // cannot be recycled for another key while it is cached) and Pkey by value
    // (it is passed by value, and is only k*dg*N words).
    std::shared_ptr<const UniEncACCKeyImpl> key_ref;
    std::vector<uint32_t> pkey_words;

private:
    mkacc_ctx* m_ctx = nullptr;
    mkacc_params m_p{};
};

// A multi-device group (mkacc_group_*): one context per device, keys converted
// once and copied device to device, batches sharded across the members.
class GroupContext {
public:
    GroupContext(const mkacc_params& p, const std::vector<int>& devices) {
        check(mkacc_group_create(&p, devices.data(), (uint32_t)devices.size(), &m_g));
        check(mkacc_get_params(mkacc_group_member(m_g, 0), &m_p));
    }
    ~GroupContext() { mkacc_group_destroy(m_g); }
    GroupContext(const GroupContext&) = delete;
    GroupContext& operator=(const GroupContext&) = delete;
    mkacc_group* get() const { return m_g; }
    const mkacc_params& params() const { return m_p; }

private:
    mkacc_group* m_g = nullptr;
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
    // layout and upload them once per key object and Pkey content.
    static void upload(DeviceContext& dc, ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey) {
        std::vector<uint32_t> pk = flatten_pkey(dc.params(), Pkey);
        if (dc.key_ref == ek && dc.pkey_words == pk) return;   // keys already on the device
        std::vector<uint32_t> evk = flatten_evk(dc.params(), ek);
        dc.key_ref.reset();
        check(mkacc_upload_keys(dc.get(), evk.data(), pk.data()));
        dc.key_ref = ek;
        dc.pkey_words = std::move(pk);
    }
    static std::vector<uint32_t> flatten_pkey(const mkacc_params& p, const std::vector<std::vector<NativePoly>>& Pkey) {
        const uint32_t dg = p.digitsG - 1, N = p.N;
        if (Pkey.size() != p.k) throw config_error("Pkey must have k parties");
        std::vector<uint32_t> pk((size_t)p.k * dg * N);
        for (uint32_t u = 0; u < p.k; ++u) {
            if (Pkey[u].size() != dg) throw config_error("Pkey must have digitsG-1 polys per party");
            for (uint32_t d = 0; d < dg; ++d)
                for (uint32_t s = 0; s < N; ++s) pk[((size_t)u * dg + d) * N + s] = (uint32_t)Pkey[u][d][s];
        }
        return pk;
    }
    static std::vector<uint32_t> flatten_evk(const mkacc_params& p, ConstUniEncACCKey& ek) {
        const uint32_t dg = p.digitsG - 1, nk = p.method == MKACC_METHOD_MKNTRU ? 2 : 1, N = p.N;
        const auto& K = ek->GetElements();
        if (K.size() != p.k) throw config_error("accumulator key must have k parties");
        std::vector<uint32_t> evk((size_t)p.k * nk * (p.n + 1) * dg * 2 * N);
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
        return evk;
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
enum BINFHE_OUTPUT { INVALID_OUTPUT = 0, FRESH, BOOTSTRAPPED, LARGE_DIM, SMALL_DIM };  // binfhe-constants.h:117-123
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
    void SetptModulus(uint64_t p) { m_p = p; }
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
    void SetptModulus(uint64_t p) { m_p = p; }
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

// ---- secret keys (NTL-free generation: include/mkfhe_keys.h) --------------------------
using MNTRUPlaintext = int64_t;
using MKLWEPlaintext = int64_t;

// MNTRUPrivateKeyImpl (mntru-privatekey.h:23-110): per party an n x n matrix F
// and its inverse mod qKS, stored flat [k][n][n] (row l, column j).
class MNTRUPrivateKeyImpl {
public:
    MNTRUPrivateKeyImpl(uint32_t k, uint32_t n, uint64_t mod, std::vector<uint32_t> F, std::vector<uint32_t> Finv)
        : m_k(k), m_n(n), m_mod(mod), m_F(std::move(F)), m_Finv(std::move(Finv)) {}
    uint32_t Getk() const { return m_k; }
    uint32_t GetLength() const { return m_n; }
    uint64_t GetModulus() const { return m_mod; }
    const std::vector<uint32_t>& F() const { return m_F; }
    const std::vector<uint32_t>& Finv() const { return m_Finv; }
    // GetF_col0 (mntru-privatekey.h:56-70): the LWE-style secret, [k][n]
    std::vector<NativeVector> GetF_col0() const {
        std::vector<NativeVector> r(m_k, NativeVector(m_n));
        for (uint32_t u = 0; u < m_k; ++u)
            for (uint32_t l = 0; l < m_n; ++l) r[u][l] = m_F[((size_t)u * m_n + l) * m_n];
        return r;
    }
    // GetF_inv_coli (mntru-privatekey.h:87-101): column j of every F_u^-1
    std::vector<NativeVector> GetF_inv_coli(uint32_t j) const {
        std::vector<NativeVector> r(m_k, NativeVector(m_n));
        for (uint32_t u = 0; u < m_k; ++u)
            for (uint32_t l = 0; l < m_n; ++l) r[u][l] = m_Finv[((size_t)u * m_n + l) * m_n + j];
        return r;
    }

private:
    uint32_t m_k, m_n;
    uint64_t m_mod;
    std::vector<uint32_t> m_F, m_Finv;
};
using MNTRUPrivateKey = std::shared_ptr<const MNTRUPrivateKeyImpl>;
using ConstMNTRUPrivateKey = const std::shared_ptr<const MNTRUPrivateKeyImpl>;

// MKLWEPrivateKeyImpl (mklwe-privatekey.h): k binary vectors of length n
class MKLWEPrivateKeyImpl {
public:
    MKLWEPrivateKeyImpl(uint32_t k, uint32_t n, uint64_t mod, std::vector<uint32_t> s)
        : m_k(k), m_n(n), m_mod(mod), m_s(std::move(s)) {}
    uint32_t Getk() const { return m_k; }
    uint32_t GetLength() const { return m_n; }
    uint64_t GetModulus() const { return m_mod; }
    const std::vector<uint32_t>& flat() const { return m_s; }
    std::vector<NativeVector> GetElement() const {
        std::vector<NativeVector> r(m_k, NativeVector(m_n));
        for (uint32_t u = 0; u < m_k; ++u)
            for (uint32_t i = 0; i < m_n; ++i) r[u][i] = m_s[(size_t)u * m_n + i];
        return r;
    }

private:
    uint32_t m_k, m_n;
    uint64_t m_mod;
    std::vector<uint32_t> m_s;
};
using MKLWEPrivateKey = std::shared_ptr<const MKLWEPrivateKeyImpl>;
using ConstMKLWEPrivateKey = const std::shared_ptr<const MKLWEPrivateKeyImpl>;

// The fields of the reference UniEncBTKey (binfhe-base-scheme.h:65-83) the
// gate path reads.  BTKeyLoad takes the reference-shaped members; MKBTKeyGen
// fills the flat members (the C-ABI layouts of mkfhe_amd.h / mkfhe_keys.h)
// and uploads them without building the nested objects.
struct UniEncBTKey {
    UniEncACCKey BSkey;
    MNTRUSwitchingKey2 KSkey2;
    MKLWESwitchingKey LKSkey;
    std::vector<std::vector<NativePoly>> Pkey;
    std::vector<NativePoly> f;
    // flat key material from MKBTKeyGen
    std::vector<uint32_t> crs, fvec, f_eval, finv_eval, pkey, evk, ksk, ksk_a, ksk_b;
};

// BinFHEContext for multi-key NAND gates on one MI355X, with the reference's
// key-generation / encryption / decryption calls (binfhecontext.h:98-338) over
// libmkfhe_keys.so and the gates over libmkfhe_amd.so.  The device context is
// created on first use, so key generation, encryption and decryption run on a
// host without a GPU.
class BinFHEContext {
public:
    void GenerateBinFHEContext(BINFHE_PARAMSET set, BINFHE_METHOD method, int device = 0) {
        GenerateBinFHEContext(set, method, std::vector<int>{device});
    }
    // Multi-device extension: batches of gates (EvalBinGate over vectors) shard
    // across `devices` (one GPU each, a device may repeat); keys are converted
    // once and copied device to device (mkacc_group).  Results are bit-identical.
    void GenerateBinFHEContext(BINFHE_PARAMSET set, BINFHE_METHOD method, const std::vector<int>& devices) {
        if (method != MKNTRU && method != MKNTRU_B && method != MKNTRU_LWE)
            throw config_error("method is invalid");
        if (devices.empty()) throw config_error("no device");
        m_method = method;
        m_params = UniEncCryptoParams::FromParamSet(ParamSetName(set), method);
        checkk(mkkg_paramset(ParamSetName(set), to_abi_method(method), &m_kp));
        m_have_kp = true;
        reset(devices);
    }
    // custom parameters (the reference's explicit-parameter overload, binfhecontext.h:94);
    // key generation then needs SetKeyParams.
    void GenerateBinFHEContext(const UniEncCryptoParams& params, int device = 0) {
        m_method = params.GetMethod();
        m_params = std::make_shared<UniEncCryptoParams>(params);
        m_have_kp = false;
        reset(std::vector<int>{device});
        dc();  // validates the parameters and derives digitsG / root (mkacc_create)
    }
    void SetKeyParams(const mkkg_params& kp) {
        m_kp = kp;
        m_have_kp = true;
    }
    // Extension: seed of the key/encryption sampler (0 = random, the reference's behaviour).
    void SetSeed(uint64_t seed) { m_seed = seed; }
    // Extension: the seed-0 entropy journal of this process (mkfhe_keys.h).
    // Whoever holds the master holds every seed-0 key of the process, so it is
    // exported only after EnableEntropyReplay(), which also takes the master
    // from MKFHE_ENTROPY when that is set (config_error if it is malformed).  A
    // run that enabled replay with MKFHE_ENTROPY=<master> repeats every seed-0
    // key and encryption of a run that made the same calls
    // (tools/fresh_key_rate.py --replay recomputes its gates on the CPU oracle).
    static void EnableEntropyReplay(bool enable = true) { checkk(mkkg_entropy_replay(enable ? 1 : 0)); }
    // The 64-hex-digit master and the number of seed-0 calls made under it;
    // config_error unless EnableEntropyReplay() ran first.
    static std::string GetEntropy(uint64_t* calls = nullptr) {
        uint32_t m[8];
        checkk(mkkg_entropy_get(m, calls));
        char buf[65];
        for (int i = 0; i < 8; ++i) std::snprintf(buf + 8 * i, 9, "%08x", m[i]);
        return std::string(buf, 64);
    }
    const std::shared_ptr<UniEncCryptoParams>& GetParams() const { return m_params; }
    // modKS = mod and baseKS = 32 in every MK set (binfhecontext.cpp:129-144)
    mkacc_ks_params GetKSParams() const {
        if (m_have_kp) return m_kp.ks;
        return mkacc_ks_params{m_params->Getq(), 32, m_params->GetLatticeParam()};
    }

    // ---- key generation (binfhecontext.cpp:235-250, 520-575) ----
    MNTRUPrivateKey MNTRU_KeyGen() const {
        need_keyparams();
        const uint32_t k = m_kp.acc.k, n = m_kp.acc.n;
        std::vector<uint32_t> F((size_t)k * n * n), Fi((size_t)k * n * n);
        checkk(mkkg_mntru_keygen(&m_kp, next_seed(), F.data(), Fi.data()));
        return std::make_shared<const MNTRUPrivateKeyImpl>(k, n, m_kp.ks.qKS, std::move(F), std::move(Fi));
    }
    MKLWEPrivateKey MKLWE_KeyGen() const {
        need_keyparams();
        if (m_kp.lwe_keydist != MKKG_DIST_BINARY) throw config_error("Support BINARY PrivateKey Only");
        const uint32_t k = m_kp.acc.k, n = m_kp.acc.n;
        std::vector<uint32_t> s((size_t)k * n);
        checkk(mkkg_mklwe_keygen(&m_kp, next_seed(), s.data()));
        return std::make_shared<const MKLWEPrivateKeyImpl>(k, n, m_kp.ks.qKS, std::move(s));
    }
    // policy (extension): the reference's r-defect handling (RDefectPolicy); the
    // default keeps its keys bit for bit and counts the defective ones (GetRDefects).
    void MKBTKeyGen(ConstMNTRUPrivateKey& sk, RDefectPolicy policy = RDefectPolicy::KEEP) {
        if (m_method == MKNTRU_LWE) throw config_error("MK-NTRU key for an MKNTRU_LWE context");
        std::vector<uint32_t> col0((size_t)sk->Getk() * sk->GetLength());
        const auto c = sk->GetF_col0();
        for (uint32_t u = 0; u < sk->Getk(); ++u)
            for (uint32_t l = 0; l < sk->GetLength(); ++l) col0[(size_t)u * sk->GetLength() + l] = (uint32_t)c[u][l];
        UniEncBTKey ek = common_btkey(col0, policy);
        ek.ksk.resize(mkkg_ksk_mntru_words(&m_kp));
        checkk(mkkg_ksk_mntru(&m_kp, next_seed(), ek.fvec.data(), sk->Finv().data(), ek.ksk.data()));
        up_ksk_mntru(ek.ksk.data());
        m_BTKey = std::move(ek);
        m_keys = true;
    }
    void MKBTKeyGen(ConstMKLWEPrivateKey& sk, RDefectPolicy policy = RDefectPolicy::KEEP) {
        if (m_method != MKNTRU_LWE) throw config_error("MK-LWE key for an MK-NTRU context");
        UniEncBTKey ek = common_btkey(sk->flat(), policy);
        ek.ksk_a.resize(mkkg_ksk_mklwe_a_words(&m_kp));
        ek.ksk_b.resize(mkkg_ksk_mklwe_b_words(&m_kp));
        checkk(mkkg_ksk_mklwe(&m_kp, next_seed(), ek.fvec.data(), sk->flat().data(), ek.ksk_a.data(),
                             ek.ksk_b.data()));
        up_ksk_mklwe(ek.ksk_a.data(), ek.ksk_b.data());
        m_BTKey = std::move(ek);
        m_keys = true;
    }
    // Extension: bootstrapping keys of the last MKBTKeyGen that drew DggR r != 0
    // (under RESAMPLE: the slots that were redrawn).  Nonzero means gates using
    // them may decrypt wrong (the reference's KeyGenXZW defect).
    uint64_t GetRDefects() const { return m_rdefects; }
    // ctGateGen (binfhe-base-scheme.cpp:340-376)
    void ctGateGen(ConstMNTRUPrivateKey& sk, BINGATE gate) {
        if (gate != NAND) throw config_error("Support NAND gate Only");
        need_keyparams();
        std::vector<uint32_t> c((size_t)sk->Getk() * sk->GetLength());
        checkk(mkkg_mntru_ctgate(&m_kp, next_seed(), sk->Finv().data(), c.data()));
        m_ctNAND = unpack_mntru(c.data(), sk->Getk(), sk->GetLength(), m_kp.acc.q);
    }
    const UniEncBTKey& GetBTKey() const { return m_BTKey; }

    // ---- key files (mkfhe_keys.h wire format; the reference has none for MK keys) ----
    void SaveBTKey(const std::string& path) const {
        need_keyparams();
        const UniEncBTKey& k = m_BTKey;
        if (k.evk.empty()) throw config_error("no bootstrapping key generated by MKBTKeyGen");
        std::vector<mkkg_section> s;
        auto add = [&](const char* nm, const std::vector<uint32_t>& v) {
            if (v.empty()) return;
            mkkg_section x{};
            std::strncpy(x.name, nm, 15);
            x.words = v.size();
            x.data = v.data();
            s.push_back(x);
        };
        add("crs", k.crs); add("skN", k.fvec); add("skN_eval", k.f_eval); add("skNinv_eval", k.finv_eval);
        add("pkey", k.pkey); add("evk", k.evk); add("ksk", k.ksk); add("ksk_a", k.ksk_a); add("ksk_b", k.ksk_b);
        checkk(mkkg_file_write(path.c_str(), MKKG_FILE_BTKEY, &m_kp, s.data(), (uint32_t)s.size()));
    }
    // Load a bootstrapping key written by SaveBTKey (or mkfhe_amd.keys.save_btkey) and upload it.
    void LoadBTKey(const std::string& path) {
        need_keyparams();
        uint32_t kind = 0;
        mkkg_params fp{};
        checkk(mkkg_file_info(path.c_str(), &kind, &fp, nullptr));
        if (kind != MKKG_FILE_BTKEY) throw config_error(path + " is not a bootstrapping-key file");
        if (fp.acc.method != m_kp.acc.method || fp.acc.k != m_kp.acc.k || fp.acc.n != m_kp.acc.n ||
            fp.acc.Q != m_kp.acc.Q || fp.acc.baseG != m_kp.acc.baseG || fp.ks.qKS != m_kp.ks.qKS)
            throw config_error(path + " was generated for a different context");
        UniEncBTKey ek;
        // a section the file does not have stays empty; a damaged file (a size past
        // its end, truncation, a checksum) throws
        auto get = [&](const char* nm, std::vector<uint32_t>& v) {
            v.resize(mkkg_file_section_words(path.c_str(), nm));
            if (!v.empty()) {
                checkk(mkkg_file_read_section(path.c_str(), nm, v.data(), v.size()));
            } else if (mkkg_file_read_section(path.c_str(), nm, nullptr, 0) != MKACC_OK) {
                const std::string e = mkkg_last_error();
                if (e.find("has no section") == std::string::npos) throw config_error(path + ": " + e);
            }
        };
        get("crs", ek.crs); get("skN", ek.fvec); get("skN_eval", ek.f_eval); get("skNinv_eval", ek.finv_eval);
        get("pkey", ek.pkey); get("evk", ek.evk); get("ksk", ek.ksk); get("ksk_a", ek.ksk_a); get("ksk_b", ek.ksk_b);
        const bool lwe = m_method == MKNTRU_LWE;
        if (ek.evk.size() != mkkg_evk_words(&m_kp) || ek.pkey.size() != mkkg_pkey_words(&m_kp) ||
            (lwe ? ek.ksk_a.size() != mkkg_ksk_mklwe_a_words(&m_kp) || ek.ksk_b.size() != mkkg_ksk_mklwe_b_words(&m_kp)
                 : ek.ksk.size() != mkkg_ksk_mntru_words(&m_kp)))
            throw config_error(path + ": key sizes do not match the context");
        up_keys(ek.evk.data(), ek.pkey.data());
        if (m_method == MKNTRU_LWE)
            up_ksk_mklwe(ek.ksk_a.data(), ek.ksk_b.data());
        else
            up_ksk_mntru(ek.ksk.data());
        m_BTKey = std::move(ek);
        m_keys = true;
    }
    void SaveSecretKey(const std::string& path, ConstMNTRUPrivateKey& sk) const {
        need_keyparams();
        mkkg_section s[2] = {};
        std::strncpy(s[0].name, "F", 15);
        s[0].words = sk->F().size();
        s[0].data = sk->F().data();
        std::strncpy(s[1].name, "Finv", 15);
        s[1].words = sk->Finv().size();
        s[1].data = sk->Finv().data();
        checkk(mkkg_file_write(path.c_str(), MKKG_FILE_MNTRU_SK, &m_kp, s, 2));
    }
    MNTRUPrivateKey LoadMNTRUSecretKey(const std::string& path) const {
        need_keyparams();
        const uint32_t k = m_kp.acc.k, n = m_kp.acc.n;
        std::vector<uint32_t> F((size_t)k * n * n), Fi((size_t)k * n * n);
        checkk(mkkg_file_read_section(path.c_str(), "F", F.data(), F.size()));
        checkk(mkkg_file_read_section(path.c_str(), "Finv", Fi.data(), Fi.size()));
        return std::make_shared<const MNTRUPrivateKeyImpl>(k, n, m_kp.ks.qKS, std::move(F), std::move(Fi));
    }

    // ---- encryption / decryption (binfhecontext.cpp:276-292, 330-375) ----
    MNTRUCiphertext Encrypt(ConstMNTRUPrivateKey& sk, MNTRUPlaintext m, BINFHE_OUTPUT output = BOOTSTRAPPED,
                            uint32_t p = 4, uint64_t mod = 0) const {
        (void)output;  // obsolete in the reference too (binfhecontext.cpp:268-272)
        need_keyparams();
        mkkg_params kp = m_kp;
        if (mod) kp.acc.q = mod;
        const uint32_t mm = (uint32_t)m;
        std::vector<uint32_t> c((size_t)sk->Getk() * sk->GetLength());
        checkk(mkkg_mntru_encrypt(&kp, next_seed(), sk->Finv().data(), &mm, p, 1, c.data()));
        auto ct = unpack_mntru(c.data(), sk->Getk(), sk->GetLength(), kp.acc.q);
        ct->SetptModulus(p);
        return ct;
    }
    MKLWECiphertext Encrypt(ConstMKLWEPrivateKey& sk, MKLWEPlaintext m, BINFHE_OUTPUT output = BOOTSTRAPPED,
                            uint32_t p = 4, uint64_t mod = 0) const {
        (void)output;
        need_keyparams();
        mkkg_params kp = m_kp;
        if (mod) kp.acc.q = mod;
        const uint32_t mm = (uint32_t)m, k = sk->Getk(), n = sk->GetLength();
        std::vector<uint32_t> a((size_t)k * n);
        uint32_t b = 0;
        checkk(mkkg_mklwe_encrypt(&kp, next_seed(), sk->flat().data(), &mm, p, 1, a.data(), &b));
        std::vector<NativeVector> av(k, NativeVector(n));
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t i = 0; i < n; ++i) av[u][i] = a[(size_t)u * n + i];
        auto ct = std::make_shared<MKLWECiphertextImpl>(std::move(av), b, kp.acc.q);
        ct->SetptModulus(p);
        return ct;
    }
    void Decrypt(ConstMNTRUPrivateKey& sk, ConstMNTRUCiphertext& ct, MNTRUPlaintext* result, uint32_t p = 4) const {
        decrypt_mntru(sk, ct, result, p, MKKG_DECRYPT);
    }
    void Decrypt2(ConstMNTRUPrivateKey& sk, ConstMNTRUCiphertext& ct, MNTRUPlaintext* result, uint32_t p = 4) const {
        decrypt_mntru(sk, ct, result, p, MKKG_DECRYPT2);
    }
    void DecryptNAND(ConstMNTRUPrivateKey& sk, ConstMNTRUCiphertext& ct, MNTRUPlaintext* result,
                     uint32_t p = 4) const {
        decrypt_mntru(sk, ct, result, p, MKKG_DECRYPT_NAND);
    }
    void Decrypt(ConstMKLWEPrivateKey& sk, ConstMKLWECiphertext& ct, MKLWEPlaintext* result, uint32_t p = 4) const {
        decrypt_mklwe(sk, ct, result, p, MKKG_DECRYPT);
    }
    void DecryptNAND(ConstMKLWEPrivateKey& sk, ConstMKLWECiphertext& ct, MKLWEPlaintext* result,
                     uint32_t p = 4) const {
        decrypt_mklwe(sk, ct, result, p, MKKG_DECRYPT_NAND);
    }

    // ---- reference-shaped key loading (keys produced elsewhere) ----
    void BTKeyLoad(const UniEncBTKey& ek) {
        need_context();
        if (!ek.BSkey) throw config_error("BSkey is empty");
        if (grouped()) {
            const std::vector<uint32_t> evk = UniEncAccumulator::flatten_evk(gc().params(), ek.BSkey);
            const std::vector<uint32_t> pk = UniEncAccumulator::flatten_pkey(gc().params(), ek.Pkey);
            up_keys(evk.data(), pk.data());
        } else {
            UniEncAccumulator::upload(dc(), ek.BSkey, ek.Pkey);
        }
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
            up_ksk_mntru(h.data());
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
            up_ksk_mklwe(ha.data(), hb.data());
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
        if (grouped())
            check(mkacc_group_eval_nand_mntru(gc().get(), nand.data(), a1.data(), a2.data(), out.data(), B));
        else
            check(mkacc_eval_nand_mntru(dc().get(), nand.data(), a1.data(), a2.data(), out.data(), B));
        std::vector<MNTRUCiphertext> res(B);
        for (size_t b = 0; b < B; ++b) res[b] = unpack_mntru(out.data() + b * k * n, k, n, GetKSParams().qKS);
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
        if (grouped())
            check(mkacc_group_eval_nand_mklwe(gc().get(), a1.data(), b1.data(), a2.data(), b2.data(), oa.data(),
                                              ob.data(), B));
        else
            check(mkacc_eval_nand_mklwe(dc().get(), a1.data(), b1.data(), a2.data(), b2.data(), oa.data(), ob.data(),
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
    void reset(const std::vector<int>& devices) {
        m_devices = devices;
        m_dc.reset();
        m_gc.reset();
        m_keys = false;
        m_ctNAND.reset();
        m_BTKey = UniEncBTKey{};
    }
    bool grouped() const { return m_devices.size() > 1; }
    DeviceContext& dc() const {
        need_context();
        if (grouped()) throw config_error("a multi-device context has no single device context");
        if (!m_dc) {
            m_dc = std::make_unique<DeviceContext>(m_params->abi(), m_devices[0]);
            m_params->set_abi(m_dc->params());
        }
        return *m_dc;
    }
    GroupContext& gc() const {
        need_context();
        if (!m_gc) {
            m_gc = std::make_unique<GroupContext>(m_params->abi(), m_devices);
            m_params->set_abi(m_gc->params());
        }
        return *m_gc;
    }
    // uploads through the single context or the group
    void up_keys(const uint32_t* evk, const uint32_t* pkey) const {
        if (grouped())
            check(mkacc_group_upload_keys(gc().get(), evk, pkey));
        else
            check(mkacc_upload_keys(dc().get(), evk, pkey));
    }
    void up_ksk_mntru(const uint32_t* ksk) const {
        const mkacc_ks_params ks = GetKSParams();
        if (grouped())
            check(mkacc_group_upload_ksk_mntru(gc().get(), &ks, ksk));
        else
            check(mkacc_upload_ksk_mntru(dc().get(), &ks, ksk));
    }
    void up_ksk_mklwe(const uint32_t* A, const uint32_t* B) const {
        const mkacc_ks_params ks = GetKSParams();
        if (grouped())
            check(mkacc_group_upload_ksk_mklwe(gc().get(), &ks, A, B));
        else
            check(mkacc_upload_ksk_mklwe(dc().get(), &ks, A, B));
    }
    void need_context() const {
        if (!m_params) throw config_error("call GenerateBinFHEContext first");
    }
    void need_keyparams() const {
        need_context();
        if (!m_have_kp) throw config_error("key parameters are not set (GenerateBinFHEContext(set) or SetKeyParams)");
    }
    uint64_t next_seed() const { return m_seed ? m_seed + (m_calls++) * 0x9E3779B97F4A7C15ull : 0; }
    // CRS, ring secrets, P and the accumulator key (binfhe-base-scheme.cpp:198-338), uploaded
    UniEncBTKey common_btkey(const std::vector<uint32_t>& lwe_sk, RDefectPolicy policy) {
        need_keyparams();
        const uint32_t k = m_kp.acc.k, N = m_kp.acc.N;
        const uint32_t dg = (m_kp.acc.digitsG ? m_kp.acc.digitsG : m_params->GetDigitsG()) - 1;
        UniEncBTKey ek;
        ek.crs.resize((size_t)dg * N);
        ek.fvec.resize((size_t)k * N);
        ek.f_eval.resize((size_t)k * N);
        ek.finv_eval.resize((size_t)k * N);
        ek.pkey.resize(mkkg_pkey_words(&m_kp));
        ek.evk.resize(mkkg_evk_words(&m_kp));
        checkk(mkkg_crs(&m_kp, next_seed(), ek.crs.data()));
        checkk(mkkg_ring_secrets(&m_kp, next_seed(), ek.fvec.data(), ek.f_eval.data(), ek.finv_eval.data()));
        checkk(mkkg_pkey(&m_kp, next_seed(), ek.crs.data(), ek.f_eval.data(), ek.pkey.data()));
        uint64_t ndef = 0;
        m_rdefects = 0;
        const int rc = mkkg_acc_keygen_ex(&m_kp, next_seed(), ek.crs.data(), ek.finv_eval.data(), lwe_sk.data(),
                                          ek.evk.data(), static_cast<uint32_t>(policy), &ndef);
        m_rdefects = ndef;   // also after a REJECT: GetRDefects() reports the rejected draw
        checkk(rc);
        up_keys(ek.evk.data(), ek.pkey.data());
        return ek;
    }
    static MNTRUCiphertext unpack_mntru(const uint32_t* c, uint32_t k, uint32_t n, uint64_t q) {
        std::vector<NativeVector> e(k, NativeVector(n));
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t i = 0; i < n; ++i) e[u][i] = c[(size_t)u * n + i];
        return std::make_shared<MNTRUCiphertextImpl>(std::move(e), q);
    }
    void decrypt_mntru(ConstMNTRUPrivateKey& sk, ConstMNTRUCiphertext& ct, MNTRUPlaintext* result, uint32_t p,
                       uint32_t variant) const {
        need_keyparams();
        if (!result) throw config_error("null result");
        const uint32_t k = sk->Getk(), n = sk->GetLength();
        std::vector<uint32_t> c((size_t)k * n);
        pack(*ct, c.data(), k, n);
        uint32_t m = 0;
        checkk(mkkg_mntru_decrypt(&m_kp, sk->F().data(), c.data(), ct->GetModulus(), p, variant, 1, &m));
        *result = m;
    }
    void decrypt_mklwe(ConstMKLWEPrivateKey& sk, ConstMKLWECiphertext& ct, MKLWEPlaintext* result, uint32_t p,
                       uint32_t variant) const {
        need_keyparams();
        if (!result) throw config_error("null result");
        const uint32_t k = sk->Getk(), n = sk->GetLength();
        std::vector<uint32_t> a((size_t)k * n);
        packA(*ct, a.data(), k, n);
        const uint32_t b = (uint32_t)ct->GetB();
        uint32_t m = 0;
        checkk(mkkg_mklwe_decrypt(&m_kp, sk->flat().data(), a.data(), &b, ct->GetModulus(), p, variant, 1, &m));
        *result = m;
    }
    void need_gate(BINGATE gate, BINFHE_METHOD family) const {
        need_context();
        if (gate != NAND) throw not_implemented_error("only NAND is supported (ctGateGen, binfhe-base-scheme.cpp:341-342)");
        // the reference's MKNTRU_B gate feeds mod-q MNTRU words to XZW_B as monomial
        // exponents (binfhecontext.cpp:174, binfhe-base-scheme.cpp:1127,
        // mk-acc-xzw_B.cpp:120,290): an out-of-range GetMonomial, i.e. undefined
        if (m_method == MKNTRU_B)
            throw config_error("MKNTRU_B NAND gates are undefined in the reference; use MKNTRU or MKNTRU_LWE");
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
    mutable std::unique_ptr<DeviceContext> m_dc;
    mutable std::unique_ptr<GroupContext> m_gc;
    std::vector<int> m_devices{0};
    bool m_keys = false;
    MNTRUCiphertext m_ctNAND;
    mkkg_params m_kp{};
    bool m_have_kp = false;
    uint64_t m_seed = 0;
    uint64_t m_rdefects = 0;
    mutable uint64_t m_calls = 1;
    UniEncBTKey m_BTKey;
};

}  // namespace mkfhe_amd

#endif  // MKFHE_AMD_BINFHE_HPP
