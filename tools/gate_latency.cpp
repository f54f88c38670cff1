// gate_latency: EvalBinGate latency of the drop-in at small batches, through
// the C++ mirror of the reference API (include/mkfhe_amd_binfhe.hpp), i.e.
// what the reference's own examples time (boolean-mkntru.cpp:36-38 times one
// EvalBinGate with clock()).  B = 1 uses the single-gate overload; larger B
// the batch overload.  Every output is decrypted and checked against NAND.
//
//   g++ -std=c++17 -O2 -Iinclude tools/gate_latency.cpp -Lmkfhe_amd/lib -lmkfhe_amd
//       -lmkfhe_keys -Wl,-rpath,$PWD/mkfhe_amd/lib -o tools/bin/gate_latency
//   tools/bin/gate_latency [PARAMSET] [B ...]        one JSON line per B
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "mkfhe_amd_binfhe.hpp"

using namespace mkfhe_amd;

static BINFHE_PARAMSET parse(const char* s) {
    for (int i = STD128_MKNTRU; i <= STD100_MKNTRU_LWE_4; ++i)
        if (!strcmp(ParamSetName((BINFHE_PARAMSET)i), s)) return (BINFHE_PARAMSET)i;
    throw config_error(std::string("unknown parameter set ") + s);
}

using clk = std::chrono::steady_clock;

template <class Ctx, class SK, class CT, class PT, class Dec>
static int run(Ctx& cc, const SK& sk, const char* ps, const std::vector<size_t>& batches, Dec decrypt) {
    std::mt19937 rng(7);
    int bad = 0;
    for (size_t B : batches) {
        std::vector<CT> c1(B), c2(B);
        std::vector<int> m1(B), m2(B);
        for (size_t b = 0; b < B; ++b) {
            m1[b] = rng() & 1;
            m2[b] = rng() & 1;
            c1[b] = cc.Encrypt(sk, m1[b]);
            c2[b] = cc.Encrypt(sk, m2[b]);
        }
        const int reps = B <= 8 ? 5 : 3;
        std::vector<CT> out;
        double best = 1e30, sum = 0;
        for (int r = 0; r < reps; ++r) {
            const auto t0 = clk::now();
            if (B == 1)
                out = {cc.EvalBinGate(NAND, c1[0], c2[0])};
            else
                out = cc.EvalBinGate(NAND, c1, c2);
            const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
            best = ms < best ? ms : best;
            sum += ms;
        }
        int wrong = 0;
        for (size_t b = 0; b < B; ++b) wrong += decrypt(out[b]) != !(m1[b] & m2[b]);
        bad += wrong;
        std::printf("{\"paramset\": \"%s\", \"B\": %zu, \"reps\": %d, \"ms_per_call_best\": %.3f, "
                    "\"ms_per_call_mean\": %.3f, \"gates_per_s\": %.1f, \"wrong\": %d}\n",
                    ps, B, reps, best, sum / reps, 1000.0 * B / best, wrong);
        std::fflush(stdout);
    }
    return bad;
}

int main(int argc, char** argv) {
    const char* ps = argc > 1 ? argv[1] : "STD128_MKNTRU";
    std::vector<size_t> batches;
    for (int i = 2; i < argc; ++i) batches.push_back((size_t)std::strtoul(argv[i], nullptr, 10));
    if (batches.empty()) batches = {1, 8, 64};
    const BINFHE_PARAMSET set = parse(ps);
    const bool lwe = std::string(ps).find("LWE") != std::string::npos;
    BinFHEContext cc;
    cc.GenerateBinFHEContext(set, lwe ? MKNTRU_LWE : MKNTRU);
    cc.SetSeed(1234);
    int bad;
    if (lwe) {
        auto sk = cc.MKLWE_KeyGen();
        cc.MKBTKeyGen(sk);
        // warm-up: first call sizes the staging buffers and loads the code objects
        (void)cc.EvalBinGate(NAND, cc.Encrypt(sk, 0), cc.Encrypt(sk, 1));
        bad = run<BinFHEContext, MKLWEPrivateKey, MKLWECiphertext, MKLWEPlaintext>(
            cc, sk, ps, batches, [&](const MKLWECiphertext& c) {
                MKLWEPlaintext p;
                cc.Decrypt(sk, c, &p);
                return (int)p;
            });
    } else {
        auto sk = cc.MNTRU_KeyGen();
        cc.MKBTKeyGen(sk);
        cc.ctGateGen(sk, NAND);
        (void)cc.EvalBinGate(NAND, cc.Encrypt(sk, 0), cc.Encrypt(sk, 1));
        bad = run<BinFHEContext, MNTRUPrivateKey, MNTRUCiphertext, MNTRUPlaintext>(
            cc, sk, ps, batches, [&](const MNTRUCiphertext& c) {
                MNTRUPlaintext p;
                cc.Decrypt(sk, c, &p);
                return (int)p;
            });
    }
    return bad ? 1 : 0;
}
