// mkacc_widereg.hpp -- register-resident FP64 step kernel of the 64-bit word
// path (Q < 2^50; SURVEY.md s8 config 5 stress, Q = 2^50 - 16383).
// Included after mkacc_widefp.hpp, whose exact FP64 modular product it uses:
//   mm(a, b) = fma(-q, Q, h) + l,  h = a b, l = fma(a, b, -h), q = rint(h / Q),
// exact with |mm| <= (0.5 + 0.5 P) Q for |a b| <= P Q^2, P <= 4, while every
// value stays below 8 Q <= 2^53 in magnitude (mkacc_widefp.hpp).
//
// widefp::step_kernel runs one gate per 256-thread workgroup and every transform
// through a 16 KiB LDS tile in six radix-4 passes separated by workgroup
// barriers (90 per gate-step; PMC: 41 % of wave cycles waiting, 2.9 LDS
// bank-conflict cycles per LDS instruction).  Here one
// WAVEFRONT owns one gate, as in the 27-bit kernels: a polynomial is 32 doubles
// per lane in VGPRs, a transform is three register passes separated by two
// wave-local LDS transposes (mkacc_device.hpp layouts A/B/C/D, the same index
// maps and padding), no barriers.  The step's live state -- the offset words of
// the digit decomposition, one digit-NTT output, the running sums uj and sumV
// and X^-c, 32 slots each -- needs the whole 512-entry register file: one wave
// per SIMD, four gates per workgroup, one workgroup per CU looping over its
// gates, with every twiddle and the psi table in LDS (copied once per launch).
//
// Value bounds are planned at compile time (FPlan / InvPlan1 below): a butterfly
// maps |a|, |b| <= X_a Q, X_b Q to <= (X_a + 0.5 + X_b / 4) Q (balanced twiddles,
// |w| <= Q/2), and a reduction red() is inserted exactly where a value could
// otherwise reach 7.8 Q; inverse butterflies with twiddle 1 skip the product
// while their sum stays below the limit.  Every result is congruent to the
// reference's residue and made canonical where it leaves the engine, so the
// path is bit-exact (tests/test_wide.py).
#pragma once

namespace {

namespace widereg {

using widefp::FMod;
using widefp::mm;
using widefp::red;

constexpr int kWaves = 4;                    // gates per workgroup (one wave per SIMD)
constexpr int kScrD = kN + kN / 32;          // per-wave transpose scratch, doubles (padded)
// LDS image (doubles), built by the host (wide_setup):
//   [kImgFwd,   + kTwlPairs)  forward per-lane twiddles, mkacc_device.hpp's twl layout
//   [kImgInv,   + kTwlPairs)  inverse per-lane twiddles (bits 5..10)
//   [kImgTwist, + N)          psi^-i * N^-1 at kImgTwist + 64 r + lane (i = (r << 6) | lane)
//   [kImgPsi,   + 2N)         psi^e, e in [0, 2N)
constexpr int kImgFwd = 0;
constexpr int kImgInv = kTwlPairs;
constexpr int kImgTwist = 2 * kTwlPairs;
constexpr int kImgPsi = kImgTwist + kN;
constexpr int kImgD = kImgPsi + 2 * kN;
constexpr size_t kLdsBytes = (size_t)(kImgD + kWaves * kScrD) * 8;
static_assert(kLdsBytes <= 160 * 1024, "one workgroup per CU");
static_assert(kImgD % 2 == 0, "image copied in 16-byte units");

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
// inverse pass 1 (bits 0..4, layout C): twiddle index t = r mod 2^b, t = 0 is 1
struct InvPlan1 {
    bool skip[5][kRegs] = {};
    bool redA[5][kRegs] = {};
    bool redB[5][kRegs] = {};
    bool redOut[kRegs] = {};   // reduced before the transpose to layout D
    int out = 0;               // bound entering pass 2
};
constexpr InvPlan1 make_inv1(int x0, int thr) {
    InvPlan1 p{};
    int bd[kRegs] = {};
    for (int r = 0; r < kRegs; ++r) bd[r] = x0;
    for (int b = 0; b < 5; ++b) {
        const int h = 1 << b;
        for (int r = 0; r < kRegs; ++r) {
            if (r & h) continue;
            if ((r & (h - 1)) == 0 && bd[r] + bd[r + h] <= kLim) {
                p.skip[b][r] = true;
                bd[r] = bd[r + h] = bd[r] + bd[r + h];
                continue;
            }
            int xa = bd[r], xb = bd[r + h];
            if (xb > 8000) {
                p.redB[b][r] = true;
                xb = kRedB;
            }
            const int T = tbound(xb);
            if (xa + T > kLim) {
                p.redA[b][r] = true;
                xa = kRedB;
            }
            bd[r] = bd[r + h] = xa + T;
        }
    }
    int mx = 0;
    for (int r = 0; r < kRegs; ++r) {
        if (bd[r] > thr) {
            p.redOut[r] = true;
            bd[r] = kRedB;
        }
        mx = bd[r] > mx ? bd[r] : mx;
    }
    p.out = mx;
    return p;
}

// forward: balanced residues (primitive kernel), and the step's digits
// (|x| <= 2^(b-1) <= 2^25, below Q / 1000 at the config-5 modulus): starting the
// plan from 0.001 Q drops one of the two 16-element reductions per digit NTT
constexpr FPlan kFwd = make_plan(510, 0, 11);
constexpr FPlan kFwdDig = make_plan(1, 0, 11);
static_assert(kFwd.out <= kLim && kFwdDig.out <= kLim, "forward bounds");
// inverse: the rotated accumulator (< 1.14 Q) or sumV (< 0.51 Q)
constexpr InvPlan1 kInv1 = make_inv1(1140, 1200);
constexpr FPlan kInv23 = make_plan(kInv1.out, 5, 11);
static_assert(kInv23.out <= 8000, "inverse bounds (the twist product needs |x| <= 8 Q)");

__device__ __forceinline__ void bfly(double& a, double& b, double w, const FMod& m, bool ra, bool rb) {
    if (rb) b = red(b, m);
    if (ra) a = red(a, m);
    const double T = mm(b, w, m);
    const double X = a;
    a = __dadd_rn(X, T);
    b = __dsub_rn(X, T);
}

// ---- wave-local LDS transposes of 32 doubles per lane --------------------------
// Same maps and padding as the 27-bit transposes (pad(j) = j + j / 32 elements):
// for 8-byte elements each half-wave's 32 lanes hit 32 distinct bank pairs in
// every layout (derivation: DESIGN.md s4.5c).
template <int SRC, int DST>
__device__ __forceinline__ void transpose(double (&x)[kRegs], double* lds, uint32_t l) {
    double* ws = lds + lbase<SRC>(l);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) ws[loff<SRC>(r)] = x[r];
    wave_lds_sync();
    const double* rs = lds + lbase<DST>(l);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = rs[loff<DST>(r)];
    wave_lds_sync();
}

typedef const __attribute__((address_space(4))) double const_f64;
__device__ __forceinline__ const_f64* opaque_c(const double* p) {
    uint64_t v = (uint64_t)p;
    asm volatile("" : "+s"(v));
    return (const_f64*)v;
}

// Forward negacyclic NTT, reference EVAL order: coefficients in layout A ->
// EVAL slots in layout C (slot j = (lane << 5) | r).
//   tws: reference forward table (balanced doubles), wave-uniform indices 1..31
//   F:   LDS per-lane table (twl layout: stage s in 5..9 at twl_off(s) + 32 m + lane/2,
//        stage 10 at kTwlC + 64 m + lane)
template <const FPlan& P>
__device__ __forceinline__ void ntt_fwd(double (&x)[kRegs], double* scr, const double* tws, const double* F,
                                        uint32_t l, const FMod& m) {
    const_f64* tw = opaque_c(tws);
    // pass A: stages 0..4 on bits 10..6 (layout A), twiddle (1 << s) + (r >> (5 - s))
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int H = 16 >> s;
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & H) continue;
            bfly(x[r], x[r + H], tw[(1 << s) + (r >> (5 - s))], m, P.redA[s], P.redB[s]);
        }
    }
    const uint32_t lo = opaque_v(l);
    transpose<0, 1>(x, scr, l);
    // pass B: stages 5..9 on bits 5..1 (layout B), per-lane twiddles
    const double* tb = F + (lo >> 1);
#pragma unroll
    for (int s = 5; s < 10; ++s) {
        const int H = 1 << (9 - s), SH = 10 - s;
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & H) continue;
            bfly(x[r], x[r + H], tb[twl_off(s) + 32 * (r >> SH)], m, P.redA[s], P.redB[s]);
        }
    }
    transpose<1, 2>(x, scr, l);
    // pass C: stage 10 on bit 0 (layout C)
    const double* tc = F + kTwlC + lo;
#pragma unroll
    for (int j = 0; j < 16; ++j) bfly(x[2 * j], x[2 * j + 1], tc[64 * j], m, P.redA[10], P.redB[10]);
}

// Inverse without the reference's separate N^-1 (folded into the twist table):
// EVAL slots in layout C -> coefficients in layout A, |.| <= 2.5 Q.  The DIT
// form of mkacc_device.hpp's ntt_inv: bits 0..4 (C, wave-uniform twiddles
// psi^-(t 2^(11-b)) from tis[(1 << b) + t]), bits 5..9 (D, per-lane), bit 10 (A,
// per-lane), then x_i *= psi^-i N^-1.
__device__ __forceinline__ void ntt_inv(double (&x)[kRegs], double* scr, const double* tis, const double* I,
                                        const double* tws, uint32_t l, const FMod& m) {
    const_f64* ti = opaque_c(tis);
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        const int H = 1 << b;
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & H) continue;
            if (kInv1.skip[b][r]) {
                const double X = x[r], Y = x[r + H];
                x[r] = __dadd_rn(X, Y);
                x[r + H] = __dsub_rn(X, Y);
            } else {
                bfly(x[r], x[r + H], ti[(1 << b) + (r & (H - 1))], m, kInv1.redA[b][r], kInv1.redB[b][r]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < kRegs; ++r)
        if (kInv1.redOut[r]) x[r] = red(x[r], m);
    const uint32_t lo = opaque_v(l);
    transpose<2, 3>(x, scr, l);
    const double* t31 = I + (lo & 31u);
#pragma unroll
    for (int b = 5; b < 10; ++b) {
        const int H = 1 << (b - 5);
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & H) continue;
            bfly(x[r], x[r + H], t31[twl_off(b) + 32 * (r & (H - 1))], m, kInv23.redA[b], kInv23.redB[b]);
        }
    }
    transpose<3, 0>(x, scr, l);
    const double* t64 = I + kTwlC + lo;
#pragma unroll
    for (int j = 0; j < 16; ++j) bfly(x[j], x[j + 16], t64[64 * j], m, kInv23.redA[10], kInv23.redB[10]);
    const double* tw = tws + lo;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = mm(x[r], tw[64 * r], m);
}

// ---- device layout of accumulators and keys ("C8") ------------------------------
// EVAL slot j = (lane << 5) | r of a polynomial lives at double index
// ((r >> 1) << 7) | (lane << 1) | (r & 1): a wave moves a whole polynomial with 16
// dwordx4 accesses of 1 KiB each.
__host__ __device__ __forceinline__ uint32_t c8_index(uint32_t j) {
    const uint32_t l = j >> 5, r = j & 31u;
    return ((r >> 1) << 7) | (l << 1) | (r & 1u);
}
__device__ __forceinline__ void load_poly(double (&x)[kRegs], __amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t so) {
#pragma unroll
    for (int g = 0; g < kRegs / 2; ++g) {
        const u32x4 v = bload4(rs, vo, so + (uint32_t)g * 1024u);
        x[2 * g] = __builtin_bit_cast(double, u32x2{v.x, v.y});
        x[2 * g + 1] = __builtin_bit_cast(double, u32x2{v.z, v.w});
    }
}
__device__ __forceinline__ void store_poly(const double (&x)[kRegs], __amdgpu_buffer_rsrc_t rs, uint32_t vo,
                                           uint32_t so) {
#pragma unroll
    for (int g = 0; g < kRegs / 2; ++g) {
        const u32x2 a = __builtin_bit_cast(u32x2, x[2 * g]), b = __builtin_bit_cast(u32x2, x[2 * g + 1]);
        bstore4(u32x4{a.x, a.y, b.x, b.y}, rs, vo, so + (uint32_t)g * 1024u);
    }
}

// The offset word D = centred(t) + C of the closed-form digits (widefp::sdd_offset),
// with centred(t) in [L, L + Q), L = -(Q + 1) / 2 (mk-acc.cpp:60-64), in 9 FP64
// operations and no integer conversion:
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
__device__ __forceinline__ double digit_of(uint64_t D, uint32_t i, const wide::Sdd64& s) {
    const uint32_t f = (uint32_t)(D >> (s.gbits * i)) & (uint32_t)((s.half << 1) - 1);
    return (double)f - (double)s.half;
}

struct StepArgs {
    const double* acc_in;     // [B][k][N] C8, balanced, reduced (|.| <= Q/2 + 2)
    double* acc_out;
    const uint32_t* cvals;    // [B] exponents c of this step, in [0, 2N)
    const double* key1;       // ev1 = (*ek)[u][0][i] : [dg][2][N] C8, balanced
    const double* key2;       // ev2 = (*ek)[u][1][i] (XZW)
    const double* keys;       // evs = (*ek)[0][0][n]
    const double* pkey;       // [k][dg][N] C8
    const double* img;        // LDS image (kImgD doubles)
    const double* twf;        // forward table, reference order (pass A reads [1, 32))
    const double* tis;        // inverse pass-1 table [(1 << b) + t]
    uint32_t B, k, index, dg;
    double cL;                // (Q + 1) / 2 = -L
    double Cm;                // 2^52 + C + L (C: SDD offset constant)
    FMod m;
    wide::Sdd64 sd;
};

// X^e at this lane's slot of register r: psi^(e (2 brv11(j) + 1)), j = (lane << 5) | r,
// brv11(j) = (brv5(r) << 6) | brv6(lane): lane part w = e (2 brv6(lane) + 1), register
// part 128 e brv5(r), both mod 2N
struct Mono {
    uint32_t w, e;
    __device__ __forceinline__ double at(const double* psi, int r) const {
        const uint32_t br = __brev((uint32_t)r) >> 27;
        return psi[(w + ((e * br) << 7)) & (2u * kN - 1u)];
    }
};
__device__ __forceinline__ Mono make_mono(uint32_t e, uint32_t l) {
    const uint32_t b6 = __brev(l) >> 26;
    return Mono{(e * (2u * b6 + 1u)) & (2u * kN - 1u), e};
}

// d_i / f_i of AddToAccXZW{0,} for one slot: widefp::key_eff (xzw.cpp:322-325,
// 375-378; xzw_B.cpp:311-314, 368-371), |.| <= 1.13 Q (later steps), 2.75 Q (first)

// Key stream of one digit's MAC: 16 groups of 2 slots (one dwordx4 per key array),
// kPf groups in flight.  One wave per SIMD has no other wave to hide a load behind,
// so the first kPf groups are issued before the digit's NTT and every later group
// kPf groups ahead of its use (the first build waited for each group right after
// issuing it: 192 exposed L2 round trips per gate-step, 602 us per launch).
#ifndef MKACC_WREG_PF
#define MKACC_WREG_PF 4
#endif
constexpr int kPf = MKACC_WREG_PF;
// X^-c at the slots: hoisted into 64 registers once per step (1) or gathered from the
// LDS psi table at every use (0: 64 registers free for the key stream)
#ifndef MKACC_WREG_MN
#define MKACC_WREG_MN 1
#endif
constexpr bool kHoistMn = MKACC_WREG_MN;
struct KGrp {
    u32x4 a1, a2, as, ap;
};
struct KeySrc {
    __amdgpu_buffer_rsrc_t rk1, rk2, rks, rpk;
    uint32_t vo, ko, po;
};
template <int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void kissue(KGrp& t, const KeySrc& k, int gq) {
    const uint32_t so = (uint32_t)gq * 1024u;
    t.a1 = bload4(k.rk1, k.vo, k.ko + so);
    if (METHOD == XZW) t.a2 = bload4(k.rk2, k.vo, k.ko + so);
    if (FIRST) t.as = bload4(k.rks, k.vo, k.ko + so);
    if (!F) t.ap = bload4(k.rpk, k.vo, k.po + so);
}

// One digit's MAC:  party (F = false): uj += g d_i, sv += g P[u][i];
// f-part (F = true): uj += g f_i.  Digit-NTT outputs are reduced first
// (|g| <= Q/2 + 2), so each product is below 0.8 Q (1.2 Q in the first step) and
// four digits keep every sum below 5.3 Q.
template <int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void mac(const double (&g)[kRegs], double (&uj)[kRegs], double (&sv)[kRegs],
                                    const double (&mn)[kRegs], const Mono& mc, const Mono& mneg, const double* psi,
                                    KGrp (&kq)[kPf],
                                    const KeySrc& ks, const FMod& m) {
#pragma unroll
    for (int gq = 0; gq < kRegs / 2; ++gq) {
        const KGrp t = kq[gq % kPf];
        if (gq + kPf < kRegs / 2) kissue<METHOD, FIRST, F>(kq[gq % kPf], ks, gq + kPf);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = 2 * gq + h;
            const double k1 = __builtin_bit_cast(double, h ? u32x2{t.a1.z, t.a1.w} : u32x2{t.a1.x, t.a1.y});
            const double k2 = METHOD == XZW ? __builtin_bit_cast(double, h ? u32x2{t.a2.z, t.a2.w} : u32x2{t.a2.x, t.a2.y}) : 0.0;
            const double kst = FIRST ? __builtin_bit_cast(double, h ? u32x2{t.as.z, t.as.w} : u32x2{t.as.x, t.as.y}) : 0.0;
            const double gr = red(g[r], m);
            const double tp = FIRST ? mc.at(psi, r) : 0.0;
            const double tn = METHOD != XZW ? 0.0 : (kHoistMn ? mn[r] : mneg.at(psi, r));
            const double d = widefp::key_eff<METHOD, FIRST>(k1, k2, kst, tp, tn, m);
            uj[r] = __dadd_rn(uj[r], mm(gr, d, m));
            if (!F) {
                const double pk = __builtin_bit_cast(double, h ? u32x2{t.ap.z, t.ap.w} : u32x2{t.ap.x, t.ap.y});
                sv[r] = __dadd_rn(sv[r], mm(gr, pk, m));
            }
        }
    }
}

// iNTT(x) -> offset words -> for each digit: NTT, MAC.  uj / sv reduced every
// kRedEvery digits and at the end: from |.| <= Q/2 + 2, a later step's products stay
// below 0.78 Q (d_i, |d| <= 1.13 Q) and 0.63 Q (P), so seven digits keep the sums
// below 6 Q; the first step's d_i (<= 2.75 Q) gives 1.19 Q per product: four digits.
template <int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void digits_pass(double (&x)[kRegs], double (&uj)[kRegs], double (&sv)[kRegs],
                                            const double (&mn)[kRegs], const Mono& mc, const Mono& mneg,
                                            const StepArgs& a,
                                            double* scr, const double* lds, uint32_t l, __amdgpu_buffer_rsrc_t rk1,
                                            __amdgpu_buffer_rsrc_t rk2, __amdgpu_buffer_rsrc_t rks,
                                            __amdgpu_buffer_rsrc_t rpk, uint32_t u) {
    const FMod& m = a.m;
    const uint32_t polyB = kN * 8u;
    constexpr uint32_t kRedEvery = FIRST ? 4u : 7u;
    ntt_inv(x, scr, a.tis, lds + kImgInv, lds + kImgTwist, l, m);
    uint64_t D[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) D[r] = offset_word(x[r], m, a.cL, a.Cm);
#pragma unroll 1
    for (uint32_t i = 0; i < a.dg; ++i) {
        // key words of digit i: d-half (2i) for the parties, f-half (2i + 1) for the f-part
        const KeySrc ks{rk1, rk2, rks, rpk, l * 16u, (2u * i + (F ? 1u : 0u)) * polyB, (u * a.dg + i) * polyB};
        KGrp kq[kPf];
#pragma unroll
        for (int j = 0; j < kPf; ++j) kissue<METHOD, FIRST, F>(kq[j], ks, j);
        sched_fence();   // in flight during the transform
        double g[kRegs];
#pragma unroll
        for (int r = 0; r < kRegs; ++r) g[r] = digit_of(D[r], i + 1, a.sd);
        ntt_fwd<kFwdDig>(g, scr, a.twf, lds + kImgFwd, l, m);
        mac<METHOD, FIRST, F>(g, uj, sv, mn, mc, mneg, lds + kImgPsi, kq, ks, m);
        if (i % kRedEvery == kRedEvery - 1) {
#pragma unroll
            for (int r = 0; r < kRegs; ++r) {
                uj[r] = red(uj[r], m);
                if (!F) sv[r] = red(sv[r], m);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        uj[r] = red(uj[r], m);
        if (!F) sv[r] = red(sv[r], m);
    }
}

// One accumulator step of gate `gate` on this wave (the algebra of widefp::step_kernel:
// HbProd, mk-acc-xzw.cpp:231-290, fused with AddToAccXZW{,0}, xzw.cpp:292-381).
template <int METHOD, bool FIRST>
__device__ __forceinline__ void one_gate(const StepArgs& a, uint32_t gate, double* scr, const double* lds,
                                         uint32_t l) {
    const FMod& m = a.m;
    const uint32_t k = a.k, index = a.index;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    constexpr uint32_t polyB = kN * 8u;
    const uint32_t vo = l * 16u;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB);
    const __amdgpu_buffer_rsrc_t rk1 = make_rsrc(a.key1, a.dg * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rk2 = make_rsrc(a.key2, a.dg * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rks = make_rsrc(a.keys, a.dg * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rpk = make_rsrc(a.pkey, k * a.dg * polyB);
    const double* psi = lds + kImgPsi;
    const Mono mc = make_mono(c, l);
    // X^-c at this lane's slots: the same for every digit and pass of the step
    const Mono mneg = make_mono(cneg, l);
    double mn[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) mn[r] = METHOD == XZW && kHoistMn ? mneg.at(psi, r) : 0.0;
    double sv[kRegs], uj[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) sv[r] = 0.0;
    // parties index + 1, ..., index: the index party's result stays in uj for the f-part
#pragma unroll 1
    for (uint32_t tt = 1; tt <= k; ++tt) {
        const uint32_t u = index + tt < k ? index + tt : index + tt - k;
        double x[kRegs];
        load_poly(x, rin, vo, u * polyB);
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            uj[r] = FIRST ? 0.0 : x[r];
            // acctemp = acc (X^c - 1)      (xzw.cpp:336-338); the first step overwrites acc
            if (!FIRST) x[r] = __dsub_rn(mm(x[r], mc.at(psi, r), m), x[r]);
        }
        digits_pass<METHOD, FIRST, false>(x, uj, sv, mn, mc, mneg, a, scr, lds, l, rk1, rk2, rks, rpk, u);
        if (tt < k) store_poly(uj, rout, vo, u * polyB);
    }
    // f-part: iNTT(sumV) -> SDD -> NTT -> acc[index] += <., f>      (xzw.cpp:272-289)
    digits_pass<METHOD, FIRST, true>(sv, uj, sv, mn, mc, mneg, a, scr, lds, l, rk1, rk2, rks, rpk, index);
    store_poly(uj, rout, vo, index * polyB);
}

template <int METHOD, bool FIRST>
__global__ __launch_bounds__(64 * kWaves, 1) void step_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    {   // the table image, once per workgroup (the workgroup loops over gates)
        const u32x4* src = reinterpret_cast<const u32x4*>(a.img);
        u32x4* dst = reinterpret_cast<u32x4*>(smem);
        for (int i = threadIdx.x; i < kImgD / 2; i += 64 * kWaves) dst[i] = src[i];
    }
    __syncthreads();
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double* scr = smem + kImgD + wv * kScrD;
    for (uint32_t g0 = blockIdx.x * kWaves; g0 < a.B; g0 += gridDim.x * kWaves) {
        const uint32_t gate = g0 + wv;
        if (gate >= a.B) break;   // no barrier follows: the other waves finish their gates
        one_gate<METHOD, FIRST>(a, gate, scr, smem, l);
    }
}

// primitive kernels for parity tests: one polynomial per wave, canonical u64 in
// the reference's order in and out
__global__ __launch_bounds__(64 * kWaves, 1) void ntt_fwd_kernel(const uint64_t* __restrict__ in,
                                                                 uint64_t* __restrict__ out, uint32_t count,
                                                                 const double* img, const double* twf, FMod m) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    for (int i = threadIdx.x; i < kImgD; i += 64 * kWaves) smem[i] = img[i];
    __syncthreads();
    const uint32_t l = threadIdx.x & 63u, p = blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (p >= count) return;
    double* scr = smem + kImgD + (threadIdx.x >> 6) * kScrD;
    const uint64_t* src = in + (size_t)p * kN;
    double x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = widefp::balanced(src[(r << 6) | l], m);   // layout A
    ntt_fwd<kFwd>(x, scr, twf, smem + kImgFwd, l, m);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) out[(size_t)p * kN + ((l << 5) | r)] = widefp::canon(x[r], m);   // layout C
}
__global__ __launch_bounds__(64 * kWaves, 1) void ntt_inv_kernel(const uint64_t* __restrict__ in,
                                                                 uint64_t* __restrict__ out, uint32_t count,
                                                                 const double* img, const double* tis, FMod m) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    for (int i = threadIdx.x; i < kImgD; i += 64 * kWaves) smem[i] = img[i];
    __syncthreads();
    const uint32_t l = threadIdx.x & 63u, p = blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (p >= count) return;
    double* scr = smem + kImgD + (threadIdx.x >> 6) * kScrD;
    const uint64_t* src = in + (size_t)p * kN;
    double x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = widefp::balanced(src[(l << 5) | r], m);   // layout C (EVAL)
    ntt_inv(x, scr, tis, smem + kImgInv, smem + kImgTwist, l, m);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) out[(size_t)p * kN + ((r << 6) | l)] = widefp::canon(x[r], m);   // layout A
}

// batch prologue / epilogue with the C8 permutation: canonical u64 words (reference
// EVAL order) <-> balanced doubles (C8); a word >= Q raises `bad` and reads as 0
__global__ void to_c8_kernel(const uint64_t* __restrict__ in, double* __restrict__ out, size_t count, FMod m,
                             uint64_t Q, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    uint64_t x = in[idx];
    if (x >= Q) {
        *bad = 1u;
        x = 0;
    }
    const size_t poly = idx / kN;
    out[poly * kN + c8_index((uint32_t)(idx % kN))] = widefp::balanced(x, m);
}
__global__ void from_c8_kernel(const double* __restrict__ in, uint64_t* __restrict__ out, size_t count, FMod m) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    const size_t poly = idx / kN;
    out[idx] = widefp::canon(in[poly * kN + c8_index((uint32_t)(idx % kN))], m);
}

}  // namespace widereg

}  // namespace
