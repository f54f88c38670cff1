// Compile check of integration/mk-acc-amd.h against the reference's headers
// (tests/test_integration_adapter.py runs `g++ -fsyntax-only` on this file).
// Nothing here runs: it instantiates every member the way BinFHEScheme would
// reach it, so a signature that drifts from the reference's fails to compile.
#include "mk-acc-amd.h"

namespace lbcrypto {

// BinFHEScheme(BINFHE_METHOD) registration (binfhe-base-scheme.h:137-151)
std::shared_ptr<UniEncAccumulator> MakeAccumulator(BINFHE_METHOD method) {
    if (method == MKNTRU)
        return std::make_shared<UniEncAccumulatorAMD>(MKNTRU);
    return std::make_shared<UniEncAccumulatorAMD>(method);
}

// ... over the eight GPUs of a node: the batches shard across them
std::shared_ptr<UniEncAccumulator> MakeNodeAccumulator(BINFHE_METHOD method) {
    return std::make_shared<UniEncAccumulatorAMD>(method, std::vector<int>{0, 1, 2, 3, 4, 5, 6, 7});
}

// BinFHEScheme::MKKeyGen -> UniEncACCscheme->KeyGenAcc (binfhe-base-scheme.cpp:272, :334)
UniEncACCKey KeyGenThroughSeam(const std::shared_ptr<UniEncAccumulator>& acc,
                               const std::shared_ptr<UniEncCryptoParams>& params,
                               const std::vector<NativePoly>& invskNTT, const ConstMNTRUPrivateKey& ntru_sk,
                               const ConstMKLWEPrivateKey& lwe_sk, bool lwe) {
    return lwe ? acc->KeyGenAcc(params, invskNTT, lwe_sk, params->GetCRS())
               : acc->KeyGenAcc(params, invskNTT, ntru_sk, params->GetCRS());
}

// BootstrapGateCore -> UniEncACCscheme->EvalAcc (binfhe-base-scheme.cpp:1065, :1127)
void EvalAccThroughSeam(const std::shared_ptr<UniEncAccumulator>& acc,
                        const std::shared_ptr<UniEncCryptoParams>& params, ConstUniEncACCKey& ek,
                        const std::vector<std::vector<NativePoly>>& Pkey, const std::vector<NativePoly>& skf,
                        MKACCCiphertext& a, const std::vector<NativeVector>& ct) {
    acc->EvalAcc(params, ek, Pkey, skf, a, ct);
}

// The batch extensions, reached through a dynamic_pointer_cast as in INTEGRATION.md §3.
void BatchThroughSeam(const std::shared_ptr<UniEncAccumulator>& acc,
                      const std::shared_ptr<UniEncCryptoParams>& params, ConstUniEncACCKey& ek,
                      const std::vector<std::vector<NativePoly>>& Pkey, std::vector<MKACCCiphertext>& accs,
                      const std::vector<std::vector<NativeVector>>& cts,
                      const std::shared_ptr<MNTRUCryptoParams>& ntru, ConstMNTRUSwitchingKey2& ksk2,
                      ConstMNTRUCiphertext& ctNAND, const std::vector<MNTRUCiphertext>& n1,
                      const std::vector<MNTRUCiphertext>& n2, const std::shared_ptr<MKLWECryptoParams>& lwe,
                      ConstMKLWESwitchingKey& lksk, const std::vector<MKLWECiphertext>& l1,
                      const std::vector<MKLWECiphertext>& l2, std::vector<MNTRUCiphertext>& nout,
                      std::vector<MKLWECiphertext>& lout) {
    auto amd = std::dynamic_pointer_cast<UniEncAccumulatorAMD>(acc);
    if (!amd)
        return;
    amd->EvalAccBatch(params, ek, Pkey, accs, cts);
    nout = amd->EvalNANDBatch(params, ntru, ek, Pkey, ksk2, ctNAND, n1, n2);
    lout = amd->EvalNANDBatch(params, lwe, ek, Pkey, lksk, l1, l2);
}

// The scheme-side batch gate of INTEGRATION.md §3 (BinFHEScheme holds a BinFHECryptoParams).
void SchemeBatch(const std::shared_ptr<UniEncAccumulator>& acc, const std::shared_ptr<BinFHECryptoParams>& params,
                 ConstUniEncACCKey& ek, const std::vector<std::vector<NativePoly>>& Pkey,
                 ConstMNTRUSwitchingKey2& ksk2, ConstMNTRUCiphertext& ctNAND, const std::vector<MNTRUCiphertext>& n1,
                 const std::vector<MNTRUCiphertext>& n2, ConstMKLWESwitchingKey& lksk,
                 const std::vector<MKLWECiphertext>& l1, const std::vector<MKLWECiphertext>& l2,
                 std::vector<MNTRUCiphertext>& nout, std::vector<MKLWECiphertext>& lout) {
    if (auto amd = std::dynamic_pointer_cast<UniEncAccumulatorAMD>(acc)) {
        nout = amd->EvalNANDBatch(params, ek, Pkey, ksk2, ctNAND, n1, n2);
        lout = amd->EvalNANDBatch(params, ek, Pkey, lksk, l1, l2);
    }
}

}  // namespace lbcrypto
