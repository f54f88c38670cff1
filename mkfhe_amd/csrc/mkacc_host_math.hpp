// mkacc_host_math.hpp -- host-side parameter derivation for the engine:
// modular helpers, primality, the reference's Q / root-of-unity choice and
// the MK parameter-set table.  Init-time only (never on the hot path).
#pragma once
#include <stdint.h>

#include <cmath>
#include <cstring>

namespace mkacc {

inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t Q) {
    return (uint64_t)(((unsigned __int128)a * b) % Q);
}
inline uint64_t powmod(uint64_t a, uint64_t e, uint64_t Q) {
    uint64_t r = 1 % Q;
    a %= Q;
    for (; e; e >>= 1) {
        if (e & 1) r = mulmod(r, a, Q);
        a = mulmod(a, a, Q);
    }
    return r;
}
inline uint64_t modinv(uint64_t a, uint64_t Q) {
    __int128 t = 0, nt = 1, r = Q, nr = a % Q;
    while (nr) {
        __int128 q = r / nr, x;
        x = t - q * nt; t = nt; nt = x;
        x = r - q * nr; r = nr; nr = x;
    }
    if (t < 0) t += Q;
    return (uint64_t)t;
}
// RoundqQ (mntru-pke.cpp:11-16): floor(0.5 + v*q/Q) in IEEE double, mod q
inline uint32_t round_qQ_host(uint64_t v, uint64_t q, uint64_t Q) {
    const double x = std::floor(0.5 + (double)v * (double)q / (double)Q);
    return (uint32_t)((uint64_t)x % q);
}
// digitCount of KeySwitch2 / KeySwitch: ceil(log qKS / log baseKS)  (mntru-pke.cpp:771)
inline uint32_t ks_digit_count(uint64_t qKS, uint32_t baseKS) {
    return (uint32_t)std::ceil(std::log((double)qKS) / std::log((double)baseKS));
}
inline uint32_t bit_reverse(uint32_t x, uint32_t bits) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}

// Deterministic Miller-Rabin for 64-bit n.
inline bool is_prime(uint64_t n) {
    static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (n < 2) return false;
    for (uint64_t b : bases) {
        if (n == b) return true;
        if (n % b == 0) return false;
    }
    uint64_t d = n - 1;
    int s = 0;
    while (!(d & 1)) { d >>= 1; ++s; }
    for (uint64_t b : bases) {
        uint64_t x = powmod(b, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int i = 1; i < s && comp; ++i) {
            x = mulmod(x, x, n);
            if (x == n - 1) comp = false;
        }
        if (comp) return false;
    }
    return true;
}

// FirstPrime / PreviousPrime (reference nbtheory-impl.h:334-377)
inline uint64_t first_prime(uint32_t nbits, uint64_t m) {
    uint64_t q = 1ull << nbits, r = q % m, c = q + 1;
    if (r) c += m - r;
    while (!is_prime(c)) c += m;
    return c;
}
inline uint64_t previous_prime(uint64_t q, uint64_t m) {
    uint64_t c = q - m;
    while (!is_prime(c)) c -= m;
    return c;
}

inline bool is_primitive_root(uint64_t w, uint64_t m, uint64_t Q) {
    // m a power of two: w^m == 1 and w^(m/2) == -1
    return w > 1 && w < Q && powmod(w, m, Q) == 1 && powmod(w, m / 2, Q) == Q - 1;
}

// RootOfUnity (nbtheory-impl.h:183-231): the minimal primitive m-th root.
inline uint64_t root_of_unity(uint64_t m, uint64_t Q) {
    uint64_t g = 2;
    while (!is_primitive_root(powmod(g, (Q - 1) / m, Q), m, Q)) ++g;
    const uint64_t w = powmod(g, (Q - 1) / m, Q), w2 = mulmod(w, w, Q);
    uint64_t x = w, best = w;
    for (uint64_t e = 1; e < m; e += 2) {
        if (x < best && x != 1) best = x;
        x = mulmod(x, w2, Q);
    }
    return best;
}

// digitsG = ceil(log(Q) / log(baseG)) (mk-cryptoparameters.h:141-142)
inline uint32_t digits_g(uint64_t Q, uint32_t baseG) {
    return (uint32_t)std::ceil(std::log((double)Q) / std::log((double)baseG));
}

// MK rows of BinFHEContext::GenerateBinFHEContext's paramsMap (binfhecontext.cpp:129-144)
struct ParamRow {
    const char* name;
    uint32_t numUser, numberBits, cyclOrder, latticeParam, mod, modKS, baseKS, gadgetBase, baseRK;
    double stdDev;     // STD_NTRU 0.5 / STD_NTRU2 0.75 / STD_DEV 1.9 (binfhecontext.cpp:85-87)
    uint32_t keyDist;  // 0 UNIFORM_TERNARY, 1 GAUSSIAN, 2 BINARY
};
inline const ParamRow* find_paramset(const char* name) {
    static const ParamRow rows[] = {
        {"STD128_MKNTRU", 2, 27, 4096, 765, 45181, 45181, 32, 1u << 7, 32, 0.5, 0},
        {"STD128_MKNTRU_2", 4, 27, 4096, 765, 45181, 45181, 32, 1u << 7, 32, 0.5, 0},
        {"STD128_MKNTRU_3", 8, 27, 4096, 765, 45181, 45181, 32, 1u << 6, 32, 0.5, 0},
        {"STD128_MKNTRU_4", 16, 27, 4096, 765, 45181, 45181, 32, 1u << 5, 32, 0.5, 0},
        {"STD128_MKNTRU_LWE", 2, 27, 4096, 635, 32749, 32749, 32, 1u << 9, 2, 1.9, 2},
        {"STD128_MKNTRU_LWE_2", 4, 27, 4096, 635, 32749, 32749, 32, 1u << 9, 2, 1.9, 2},
        {"STD128_MKNTRU_LWE_3", 8, 27, 4096, 635, 32749, 32749, 32, 1u << 9, 2, 1.9, 2},
        {"STD128_MKNTRU_LWE_4", 16, 27, 4096, 635, 32749, 32749, 32, 1u << 7, 2, 1.9, 2},
        {"STD100_MKNTRU", 2, 27, 4096, 560, 45181, 45181, 32, 1u << 9, 32, 0.75, 0},
        {"STD100_MKNTRU_2", 4, 27, 4096, 560, 45181, 45181, 32, 1u << 9, 32, 0.75, 0},
        {"STD100_MKNTRU_3", 8, 27, 4096, 560, 45181, 45181, 32, 1u << 9, 32, 0.75, 0},
        {"STD100_MKNTRU_4", 16, 27, 4096, 560, 45181, 45181, 32, 1u << 9, 32, 0.75, 0},
        {"STD100_MKNTRU_LWE", 2, 27, 4096, 500, 32749, 32749, 32, 1u << 9, 2, 1.9, 2},
        {"STD100_MKNTRU_LWE_2", 4, 27, 4096, 500, 32749, 32749, 32, 1u << 9, 2, 1.9, 2},
        {"STD100_MKNTRU_LWE_3", 8, 27, 4096, 500, 32749, 32749, 32, 1u << 9, 2, 1.9, 2},
        {"STD100_MKNTRU_LWE_4", 16, 27, 4096, 500, 32749, 32749, 32, 1u << 9, 2, 1.9, 2},
    };
    for (const auto& r : rows)
        if (std::strcmp(r.name, name) == 0) return &r;
    return nullptr;
}

}  // namespace mkacc
