// boolean-mklwe on the MI355X engine: the reference example
// (src/binfhe/examples/boolean-mklwe.cpp) against the C++ mirror
// include/mkfhe_amd_binfhe.hpp, for all four input pairs.  Exit status 0 iff
// every NAND decrypts correctly.
//
//   g++ -std=c++17 -O2 -Iinclude examples/boolean-mklwe.cpp -Lmkfhe_amd/lib
//       -lmkfhe_amd -lmkfhe_keys -Wl,-rpath,$PWD/mkfhe_amd/lib -o boolean-mklwe
//   ./boolean-mklwe [STD100_MKNTRU_LWE|...] [--replay] [--resample]
//   --resample: MKBTKeyGen under RDefectPolicy::RESAMPLE (redraw a key whose DggR sample r is
//   nonzero; the default keeps the reference's keys, defect included)
//   --replay: record the seed-0 entropy master so a run with a wrong gate can be
//   replayed (prints it on failure; whoever holds it holds every key of the run)
#include <cstdio>
#include <cstring>
#include <ctime>
#include <iostream>

#include "mkfhe_amd_binfhe.hpp"

using namespace mkfhe_amd;
using namespace std;

static BINFHE_PARAMSET parse(const char* s) {
    for (int i = STD128_MKNTRU; i <= STD100_MKNTRU_LWE_4; ++i)
        if (!strcmp(ParamSetName((BINFHE_PARAMSET)i), s)) return (BINFHE_PARAMSET)i;
    throw config_error(string("unknown parameter set ") + s);
}

int main(int argc, char** argv) {
    const char* set = nullptr;
    bool replay = false, resample = false;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--replay"))
            replay = true;
        else if (!strcmp(argv[i], "--resample"))
            resample = true;
        else
            set = argv[i];
    }
    if (replay) BinFHEContext::EnableEntropyReplay();   // opt-in: the master is secret material

    // Sample Program: Step 1: Set CryptoContext
    auto cc = BinFHEContext();
    cc.GenerateBinFHEContext(set ? parse(set) : STD100_MKNTRU_LWE, MKNTRU_LWE);
    cout << "Generating sk" << endl;
    auto sk = cc.MKLWE_KeyGen();

    // Generate the bootstrapping keys (refresh and switching keys)
    std::cout << "Generating the bootstrapping keys..." << std::endl;
    cc.MKBTKeyGen(sk, resample ? RDefectPolicy::RESAMPLE : RDefectPolicy::KEEP);
    if (cc.GetRDefects())   // the reference's KeyGenXZW r-defect (mk-acc-xzw.cpp:160-167), reported here
        std::cout << "warning: " << cc.GetRDefects()
                  << " bootstrapping key(s) drew a nonzero DggR sample r; gates using them may decrypt wrong "
                     "(regenerate the keys, or MKBTKeyGen(sk, RDefectPolicy::RESAMPLE))"
                  << std::endl;
    std::cout << "Completed the key generation." << std::endl;

    int bad = 0;
    for (int m0 = 0; m0 < 2; ++m0)
        for (int m1 = 0; m1 < 2; ++m1) {
            MKLWECiphertext ct1 = cc.Encrypt(sk, m0);
            MKLWECiphertext ct2 = cc.Encrypt(sk, m1);
            MKLWEPlaintext result;

            clock_t start = clock();
            MKLWECiphertext ctOUT = cc.EvalBinGate(NAND, ct1, ct2);
            std::cout << "Time of gate bootstrapping:\t" << float(clock() - start) * 1000 / CLOCKS_PER_SEC << "ms"
                      << std::endl;

            cc.Decrypt(sk, ctOUT, &result);
            std::cout << "Result of encrypted computation of ( " << m0 << " NAND " << m1 << " ) = " << result
                      << std::endl;
            bad += result != !(m0 & m1);
        }
    if (bad) {
        if (replay) {
            // seed material of every key and ciphertext above (seed-0 entropy journal):
            // MKFHE_ENTROPY=<master> with --replay replays this run, and
            // tools/fresh_key_rate.py --replay <master> recomputes its gates on the CPU oracle
            uint64_t calls = 0;
            const std::string master = BinFHEContext::GetEntropy(&calls);
            std::cout << "replay: MKFHE_ENTROPY=" << master << " (" << calls << " seed-0 calls)" << std::endl;
        } else {
            std::cout << "run with --replay to record the key material of a failing run" << std::endl;
        }
        return 1;
    }
    return 0;
}
