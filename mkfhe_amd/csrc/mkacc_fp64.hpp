// mkacc_fp64.hpp -- exact FP64 modular arithmetic of the 64-bit word path when
// Q < 2^50 (SURVEY.md s8 config 5 stress: Q = 1125899906826241 = 2^50 - 16383),
// used by the register-resident step kernel (mkacc_widereg2.hpp).
//
// Residues are exact integers in IEEE binary64 words, signed ("balanced"), and
// the modular product is
//
//   mm(a, b) = fma(-q, Q, h) + l,   h = a*b,  l = fma(a, b, -h),  q = rint(h / Q)
//
// 6 double-precision ops where the integer path needs 11 32-bit multiply-adds
// plus carries (tools/ubench_wide.hip, profiles/r2/ubench_wide.txt: butterfly
// 3,971 vs 1,841 G butterflies/s on the chip, 2.16x).  Exactness (checked on
// 2 x 10^6 random operands per bound at the config-5 modulus,
// tools/fp64_modmul_check.c): h + l = a b exactly; for |a b| <= P Q^2, P <= 4,
// the computed quotient is within 0.5 + 0.38 P of a b / Q, so
// |a b - q Q| <= (0.5 + 0.38 P) Q and |l| <= ulp(P Q^2) / 2 <= 0.125 P Q;
// h - q Q is an integer below 2^53, so the first fma is exact, and
//   |mm(a, b)| <= (0.5 + 0.5 P) Q.
// Every value stays below 8 Q < 2^53 in magnitude, so every add is exact too.
// The results are congruent to the reference's canonical residues mod Q and are
// made canonical where they leave the engine, so the path is bit-exact.
//
// Value bounds are planned at compile time (FPlan below): a butterfly maps
// |a|, |b| <= X_a Q, X_b Q to <= (X_a + 0.5 + X_b / 4) Q (balanced twiddles,
// |w| <= Q/2), and a reduction red() is inserted exactly where a value could
// otherwise reach 7.8 Q.
#pragma once

namespace {

namespace fp64 {

struct FMod {
    double Q, Qi;     // Q and 1/Q (rounded)
    double qhalf;     // (Q - 1) / 2 = Q >> 1
};

// exact a*b - q*Q, |.| <= (0.5 + 0.5 P) Q for |a b| <= P Q^2, P <= 4
__device__ __forceinline__ double mm(double a, double b, const FMod& m) {
    const double h = __dmul_rn(a, b);
    const double l = __fma_rn(a, b, -h);
    const double q = rint(__dmul_rn(h, m.Qi));
    return __dadd_rn(__fma_rn(-q, m.Q, h), l);
}
// x - rint(x / Q) Q for |x| <= 8 Q: |.| <= Q/2 + 2
__device__ __forceinline__ double red(double x, const FMod& m) {
    return __fma_rn(-rint(__dmul_rn(x, m.Qi)), m.Q, x);
}
// canonical residue in [0, Q) as a 64-bit word
__device__ __forceinline__ uint64_t canon(double x, const FMod& m) {
    double c = red(x, m);
    c = c < 0.0 ? c + m.Q : c;
    c = c >= m.Q ? c - m.Q : c;
    return (uint64_t)c;
}
// canonical word -> balanced double (|.| <= Q/2)
__device__ __forceinline__ double balanced(uint64_t x, const FMod& m) {
    const double d = (double)x;
    return d > m.qhalf ? d - m.Q : d;
}

// d_i / f_i of AddToAccXZW{0,} for one slot (xzw.cpp:322-325, 375-378;
// xzw_B.cpp:311-314, 368-371).  Keys and monomials balanced (|.| <= Q/2), so
// each product is below 0.625 Q and the result below 2.75 Q (1.13 Q after the
// first step).
template <int METHOD, bool FIRST>
__device__ __forceinline__ double key_eff(double k1, double k2, double ks, double tp, double tn, const FMod& m) {
    if (METHOD == XZW) {
        if (FIRST) return ks + (mm(k1, tp, m) - k1) + (mm(k2, tn, m) - k2);
        return k1 - mm(k2, tn, m);   // ev1 - ev2 X^-c
    }
    if (FIRST) return ks + (mm(k1, tp, m) - k1);
    return k1;
}

// ---- compile-time bound plans (units of Q / 1000) ----------------------------
constexpr int kLim = 7800;    // |value| < 7.8 Q (< 8 Q <= 2^53)
constexpr int kRedB = 502;    // after red(): |x| <= Q/2 + 2
constexpr int tbound(int xb) { return 500 + (xb + 3) / 4 + 1; }   // |mm(b, w)|, |w| <= Q/2

// Forward (and inverse passes 2-3): every element has the same bound at a stage.
struct FPlan {
    bool redA[12] = {};
    bool redB[12] = {};
    int out = 0;
};
constexpr FPlan make_plan(int x0, int s0, int s1) {
    FPlan p{};
    int X = x0;
    for (int s = s0; s < s1; ++s) {
        int xa = X, xb = X;
        if (xb > 8000) {
            p.redB[s] = true;
            xb = kRedB;
        }
        const int T = tbound(xb);
        if (xa + T > kLim) {
            p.redA[s] = true;
            xa = kRedB;
        }
        X = xa + T;
    }
    p.out = X;
    return p;
}
// forward: balanced residues (primitive kernel), and the step's digits
// (|x| <= 2^(b-1) <= 2^25, below Q / 1000 at the config-5 modulus): starting the
// plan from 0.001 Q drops one of the two 16-element reductions per digit NTT
constexpr FPlan kFwd = make_plan(510, 0, 11);
constexpr FPlan kFwdDig = make_plan(1, 0, 11);
static_assert(kFwd.out <= kLim && kFwdDig.out <= kLim, "forward bounds");

__device__ __forceinline__ void bfly(double& a, double& b, double w, const FMod& m, bool ra, bool rb) {
    if (rb) b = red(b, m);
    if (ra) a = red(a, m);
    const double T = mm(b, w, m);
    const double X = a;
    a = __dadd_rn(X, T);
    b = __dsub_rn(X, T);
}

// The offset word D = centred(t) + C of the closed-form digits (mkacc_device.hpp
// sdd_offset), with centred(t) in [L, L + Q), L = -(Q + 1) / 2 (mk-acc.cpp:60-64),
// in 9 FP64 operations and no integer conversion:
//   s = t - L, y = s - Q floor(s / Q) in [0, Q)   (|t| <= 2.5 Q, so |s / Q| < 3.5 and the
//       product s * RN(1/Q) is within 3.5 * 2^-52 < 1/Q of s / Q: floor is exact except
//       when s is a multiple of Q, where it can come out one short -- y = Q, mapped to 0)
//   D = y + (C + L): added to 2^52 the sum is an exact double in [2^52, 2^53) whose
//       low 52 bits ARE D (C + L >= 0 and D < 2^52 when b * digitsG <= 52, host-checked),
//       and every digit field lies below bit 52
__device__ __forceinline__ uint64_t offset_word(double t, const FMod& m, double cL, double Cm) {
    const double s = __dadd_rn(t, cL);
    const double q = floor(__dmul_rn(s, m.Qi));
    double y = __fma_rn(-q, m.Q, s);
    y = y >= m.Q ? __dsub_rn(y, m.Q) : y;
    return __builtin_bit_cast(uint64_t, __dadd_rn(y, Cm));   // 2^52 + D
}
// balanced digit i (1..dg) as a small signed double (the reference's r, before r < 0 ? r + Q)
__device__ __forceinline__ double digit_of(uint64_t D, uint32_t i, const wide::Sdd64& s) {
    const uint32_t f = (uint32_t)(D >> (s.gbits * i)) & (uint32_t)((s.half << 1) - 1);
    return (double)f - (double)s.half;
}

}  // namespace fp64

}  // namespace
