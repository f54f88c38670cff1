// mkacc_widereg2.hpp -- config-5 FP64 step kernel with TWO waves per gate
// (Q < 2^50; SURVEY.md s8 config 5 stress).  Included after mkacc_fp64.hpp,
// whose exact FP64 product, bound plans and butterfly it uses.
//
// One wave per gate (round 4's widereg::step_kernel, retired in round 5; git
// history) needs 32 doubles per lane for each of the offset words, the digit NTT,
// uj, sumV and X^-c -- the whole 512-entry register file, ONE wave per SIMD, and a
// single FP64 instruction stream reaches only ~70-78 % of the issue rate even
// with 16 independent products in flight (tools/ubench_dp_ilp.hip,
// profiles/r4/ubench_dp_ilp.txt; two waves per SIMD: 83-91 %).  Here a gate is
// split over two waves of one 128-thread workgroup, 16 doubles per lane each, so
// the per-wave state halves and two waves share a SIMD.
//
// A transform is still three register passes and two LDS transposes: one across
// the gate's two waves (s_barrier of the 2-wave workgroup, two ping-pong buffers),
// one inside each wave's half of the buffer (no barrier; mkacc_layout2.hpp Bufs).  Position p (11 bits) of a polynomial sits at
// (wave w, lane l, register r) in one of four layouts:
//   A2  r = p10..p7, w = p6,  l = p5..p0                  coefficients
//   B2  r = p6..p3,  w = p10, l = (p9, p8, p7, p2, p1, p0)
//   C2  r = p3..p0,  w = p10, l = (p8, p4, p7, p9, p6, p5) EVAL slots
//   D2  r = p7..p4,  w = p10, l = (p9, p8, p3, p2, p1, p0)
// (l written l5..l0).  Forward: A2 stages 0-3 (wave-uniform twiddles) -> B2 stages
// 4-6 -> C2 stages 7-10; inverse: C2 bits 0-3 (wave-uniform) -> D2 bits 4-7 ->
// A2 bits 8-10, then the psi^-p N^-1 twist.  The LDS word of position p is
// sum_k W_k p_k with W = 1, 2, 4, 8, 16, 33, 66, 136, 272, 548, 1088: additive in
// every bit (a per-lane base plus a compile-time register offset), injective, and
// in every layout the 32 lanes of a half-wave hit 32 distinct bank pairs (checked
// exhaustively by tools/widereg2_model.py, which also runs the whole transform
// pair in exact integers against the oracle).  Per-lane twiddles (7 + 15 forward,
// 15 + 14 inverse, 16 twist values per lane) come from one HBM table through L1,
// loaded a pass ahead; there is no LDS table image.
#pragma once

namespace {

namespace widereg2 {

using fp64::FMod;
using fp64::mm;
using fp64::red;
using fp64::bfly;
using fp64::FPlan;
using fp64::kLim;
using fp64::kRedB;
using fp64::tbound;
using fp64::make_plan;

using lay2::kR;
using lay2::Lane;
using lay2::LA;
using lay2::LB;
using lay2::LC;
using lay2::LD;
using lay2::pos_a;
using lay2::pos_c;
using lay2::tload;
using lay2::transpose;
using lay2::transpose_local;
using Bufs = lay2::Bufs<double>;
// the LB -> LC and LC -> LD transposes stay inside each wave (no barrier; every
// transpose crossing the barrier measured 351-352 against 349-350 us per config-5
// launch, profiles/r4/ab_c5_widereg2.txt)
template <int SRC, int DST>
__device__ __forceinline__ void transpose2(double (&x)[kR], Bufs& b, uint32_t l, uint32_t w) {
    transpose_local<SRC, DST>(x, b.cur(), l, w);
}
using lay2::TFB;
using lay2::TFC;
using lay2::TID;
using lay2::TIA;
using lay2::TTW;
constexpr int kBufD = lay2::kBufE;                 // doubles of one transpose buffer
constexpr size_t kLdsBytes = 2 * kBufD * 8;        // two ping-pong buffers per gate
static_assert(4 * kLdsBytes <= 160 * 1024, "four gates (eight waves) per CU");
constexpr int kTabD = lay2::kTabE;

// device ("C16") word of EVAL slot p: wave half, then register pair, lane, pair element
// -- a wave moves its half of a polynomial with 8 dwordx4 accesses of 1 KiB
__host__ __device__ __forceinline__ uint32_t c16_index(uint32_t p) {
    const uint32_t r = p & 15u;
    const uint32_t l = ((p >> 5) & 1u) | (((p >> 6) & 1u) << 1) | (((p >> 9) & 1u) << 2) | (((p >> 7) & 1u) << 3) |
                       (((p >> 4) & 1u) << 4) | (((p >> 8) & 1u) << 5);   // lay2 LC lane of p
    return ((p >> 10) << 10) | ((r >> 1) << 7) | (l << 1) | (r & 1u);
}

template <int NP>
struct TwPairs : lay2::TwPairs<NP> {
    __device__ __forceinline__ double at(int k) const { return __builtin_bit_cast(double, this->raw(k)); }
};

// ---- inverse pass-1 plan (bits 0..3, 16 registers) ------------------------------------
struct InvPlan1 {
    bool skip[4][kR] = {};
    bool redA[4][kR] = {};
    bool redB[4][kR] = {};
    bool redOut[kR] = {};
    int out = 0;
};
constexpr InvPlan1 make_inv1(int x0, int thr) {
    InvPlan1 p{};
    int bd[kR] = {};
    for (int r = 0; r < kR; ++r) bd[r] = x0;
    for (int b = 0; b < 4; ++b) {
        const int h = 1 << b;
        for (int r = 0; r < kR; ++r) {
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
    for (int r = 0; r < kR; ++r) {
        if (bd[r] > thr) {
            p.redOut[r] = true;
            bd[r] = kRedB;
        }
        mx = bd[r] > mx ? bd[r] : mx;
    }
    p.out = mx;
    return p;
}
constexpr InvPlan1 kInv1 = make_inv1(1140, 1200);
constexpr FPlan kInv23 = make_plan(kInv1.out, 4, 11);
static_assert(kInv23.out <= 8000, "inverse bounds (the twist product needs |x| <= 8 Q)");
using fp64::kFwd;
using fp64::kFwdDig;

typedef const __attribute__((address_space(4))) double const_f64;
__device__ __forceinline__ const_f64* opaque_c(const double* p) {
    uint64_t v = (uint64_t)p;
    asm volatile("" : "+s"(v));
    return (const_f64*)v;
}

// Forward negacyclic NTT (reference EVAL order): coefficients in A2 -> slots in C2.
//   tws: reference forward table (balanced), wave-uniform indices 1..15
template <const FPlan& P>
__device__ __forceinline__ void ntt_fwd(double (&x)[kR], Bufs& bufs, const double* tws, __amdgpu_buffer_rsrc_t rt,
                                        const Lane& ln, const FMod& m) {
    TwPairs<4> fb;
    tload<TFB>(fb, rt, ln.vt);
    const_f64* tw = opaque_c(tws);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int H = 8 >> s;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            bfly(x[r], x[r + H], tw[(1 << s) + (r >> (4 - s))], m, P.redA[s], P.redB[s]);
        }
    }
    transpose<LA, LB>(x, bufs.cross(), ln.l, ln.w);
    TwPairs<8> fc;
    tload<TFC>(fc, rt, ln.vt);
#pragma unroll
    for (int s = 4; s < 7; ++s) {
        const int H = 8 >> (s - 4);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            bfly(x[r], x[r + H], fb.at(((1 << (s - 4)) - 1) + (r >> (8 - s))), m, P.redA[s], P.redB[s]);
        }
    }
    transpose2<LB, LC>(x, bufs, ln.l, ln.w);
#pragma unroll
    for (int s = 7; s < 11; ++s) {
        const int H = 8 >> (s - 7);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            bfly(x[r], x[r + H], fc.at(((1 << (s - 7)) - 1) + (r >> (11 - s))), m, P.redA[s], P.redB[s]);
        }
    }
}

// Inverse without the reference's separate N^-1 (in the twist): slots in C2 ->
// coefficients in A2, |.| <= 2.5 Q.  DIT over the slot bits, twiddle
// psi^-(t 2^(11-b)) with t = p mod 2^b: bits 0-3 wave-uniform (tis[(1 << b) + t]),
// bits 4-7 and 8-10 per lane, then x_p *= psi^-p N^-1.
__device__ __forceinline__ void ntt_inv(double (&x)[kR], Bufs& bufs, const double* tis, __amdgpu_buffer_rsrc_t rt,
                                        const Lane& ln, const FMod& m) {
    TwPairs<8> id;
    tload<TID>(id, rt, ln.vt);
    const_f64* ti = opaque_c(tis);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int H = 1 << b;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
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
    for (int r = 0; r < kR; ++r)
        if (kInv1.redOut[r]) x[r] = red(x[r], m);
    TwPairs<7> ia;
    tload<TIA>(ia, rt, ln.vt);
    transpose2<LC, LD>(x, bufs, ln.l, ln.w);
#pragma unroll
    for (int b = 4; b < 8; ++b) {
        const int H = 1 << (b - 4);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            bfly(x[r], x[r + H], id.at((H - 1) + (r & (H - 1))), m, kInv23.redA[b], kInv23.redB[b]);
        }
    }
    TwPairs<8> tt;
    tload<TTW>(tt, rt, ln.vt);
    transpose<LD, LA>(x, bufs.cross(), ln.l, ln.w);
#pragma unroll
    for (int b = 8; b < 11; ++b) {
        const int H = 1 << (b - 7);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            bfly(x[r], x[r + H], ia.at((H - 2) + (r & (H - 1))), m, kInv23.redA[b], kInv23.redB[b]);
        }
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) x[r] = mm(x[r], tt.at(r), m);
}

// ---- polynomials in HBM (C16) -------------------------------------------------------
__device__ __forceinline__ void load_poly(double (&x)[kR], __amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t so) {
#pragma unroll
    for (int g = 0; g < kR / 2; ++g) {
        const u32x4 v = bload4(rs, vo, so + (uint32_t)g * 1024u);
        x[2 * g] = __builtin_bit_cast(double, u32x2{v.x, v.y});
        x[2 * g + 1] = __builtin_bit_cast(double, u32x2{v.z, v.w});
    }
}
__device__ __forceinline__ void store_poly(const double (&x)[kR], __amdgpu_buffer_rsrc_t rs, uint32_t vo,
                                           uint32_t so) {
#pragma unroll
    for (int g = 0; g < kR / 2; ++g) {
        const u32x2 a = __builtin_bit_cast(u32x2, x[2 * g]), b = __builtin_bit_cast(u32x2, x[2 * g + 1]);
        bstore4(u32x4{a.x, a.y, b.x, b.y}, rs, vo, so + (uint32_t)g * 1024u);
    }
}

// X^e at slot p = pos_c(w, l, r): psi^(e (2 brv11(p) + 1)); brv11(p) = (brv4(r) << 7) + Lw,
// Lw = 32 l0 + 16 l1 + 2 l2 + 8 l3 + 64 l4 + 4 l5 + w (p5, p6, p9, p7, p4, p8), so the exponent is
// e (2 Lw + 1) + (e brv4(r) << 8) mod 2N.  psi: the balanced psi^e table in HBM.
struct Mono {
    uint32_t wp, e;
    __device__ __forceinline__ uint32_t word(int r) const {   // byte offset of the table entry
        const uint32_t br = __brev((uint32_t)r) >> 28;
        return ((wp + ((e * br) << 8)) & (2u * kN - 1u)) * 8u;
    }
};
__device__ __forceinline__ Mono make_mono(uint32_t e, uint32_t l, uint32_t w) {
    const uint32_t Lw = ((l & 1u) << 5) | (((l >> 1) & 1u) << 4) | (((l >> 2) & 1u) << 1) | (((l >> 3) & 1u) << 3) |
                        (((l >> 4) & 1u) << 6) | (((l >> 5) & 1u) << 2) | w;
    return Mono{(e * (2u * Lw + 1u)) & (2u * kN - 1u), e};
}
__device__ __forceinline__ double ldd(__amdgpu_buffer_rsrc_t r, uint32_t vo) {
    return __builtin_bit_cast(double, bload2(r, vo, 0));
}

struct StepArgs {
    const double* acc_in;     // [B][k][N] C16, balanced, reduced (|.| <= Q/2 + 2)
    double* acc_out;
    const uint32_t* cvals;    // [B] exponents c of this step, in [0, 2N)
    const double* key1;       // ev1 = (*ek)[u][0][i] : [dg][2][N] C16, balanced
    const double* key2;       // ev2 = (*ek)[u][1][i] (XZW)
    const double* keys;       // evs = (*ek)[0][0][n]
    const double* pkey;       // [k][dg][N] C16
    const double* tab;        // per-lane twiddle table (kTabD doubles)
    const double* psi;        // psi^e, e in [0, 2N), balanced
    const double* twf;        // forward table, reference order (pass A2 reads [1, 16))
    const double* tis;        // inverse pass-1 table [(1 << b) + t]
    uint32_t B, k, index, dg;
    double cL, Cm;            // fp64::offset_word constants
    FMod m;
    wide::Sdd64 sd;
};

// key stream of one digit's MAC: 8 groups of 2 slots, kPf groups in flight (the
// first kPf issued before the digit's NTT).  1: spill-free at 2 waves per SIMD; 2
// spilled 3 VGPRs and measured the same (362.3 against 362.8 us per config-5
// launch, profiles/r4/ab_c5_widereg2.txt): the other wave on the SIMD hides the loads
constexpr int kPf = 1;
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

// One digit's MAC: party (F = false): uj += g d_i,
// sv += g P[u][i]; f-part (F = true): uj += g f_i.  g reduced first (|g| <= Q/2 + 2).
template <int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void mac(const double (&g)[kR], double (&uj)[kR], double (&sv)[kR], const double (&mn)[kR],
                                    const double (&mcv)[kR], KGrp (&kq)[kPf], const KeySrc& ks, const FMod& m) {
#pragma unroll
    for (int gq = 0; gq < kR / 2; ++gq) {
        const KGrp t = kq[gq % kPf];
        if (gq + kPf < kR / 2) kissue<METHOD, FIRST, F>(kq[gq % kPf], ks, gq + kPf);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = 2 * gq + h;
            const double k1 = __builtin_bit_cast(double, h ? u32x2{t.a1.z, t.a1.w} : u32x2{t.a1.x, t.a1.y});
            const double k2 = METHOD == XZW ? __builtin_bit_cast(double, h ? u32x2{t.a2.z, t.a2.w} : u32x2{t.a2.x, t.a2.y}) : 0.0;
            const double kst = FIRST ? __builtin_bit_cast(double, h ? u32x2{t.as.z, t.as.w} : u32x2{t.as.x, t.as.y}) : 0.0;
            const double gr = red(g[r], m);
            const double d = fp64::key_eff<METHOD, FIRST>(k1, k2, kst, FIRST ? mcv[r] : 0.0, METHOD == XZW ? mn[r] : 0.0, m);
            uj[r] = __dadd_rn(uj[r], mm(gr, d, m));
            if (!F) {
                const double pk = __builtin_bit_cast(double, h ? u32x2{t.ap.z, t.ap.w} : u32x2{t.ap.x, t.ap.y});
                sv[r] = __dadd_rn(sv[r], mm(gr, pk, m));
            }
        }
    }
}

// iNTT(x) -> offset words -> per digit: NTT, MAC.  uj / sv reduced every kRedEvery
// digits and at the end: from |.| <= Q/2 + 2, a later step's products stay below
// 0.78 Q (d_i, |d| <= 1.13 Q) and 0.63 Q (P), so seven digits keep the sums below
// 6 Q; the first step's d_i (<= 2.75 Q) gives 1.19 Q per product: four digits.
template <int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void digits_pass(double (&x)[kR], double (&uj)[kR], double (&sv)[kR], const double (&mn)[kR],
                                            const double (&mcv)[kR], const StepArgs& a, Bufs& bufs,
                                            __amdgpu_buffer_rsrc_t rt, const Lane& ln, const KeySrc& ks0, uint32_t u) {
    const FMod& m = a.m;
    constexpr uint32_t polyB = kN * 8u;
    constexpr uint32_t kRedEvery = FIRST ? 4u : 7u;
    ntt_inv(x, bufs, a.tis, rt, ln, m);
    uint64_t D[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) D[r] = fp64::offset_word(x[r], m, a.cL, a.Cm);
#pragma unroll 1
    for (uint32_t i = 0; i < a.dg; ++i) {
        KeySrc ks = ks0;
        ks.ko = (2u * i + (F ? 1u : 0u)) * polyB;
        ks.po = (u * a.dg + i) * polyB;
        KGrp kq[kPf];
#pragma unroll
        for (int j = 0; j < kPf; ++j) kissue<METHOD, FIRST, F>(kq[j], ks, j);
        sched_fence();
        double g[kR];
#pragma unroll
        for (int r = 0; r < kR; ++r) g[r] = fp64::digit_of(D[r], i + 1, a.sd);
        ntt_fwd<kFwdDig>(g, bufs, a.twf, rt, ln, m);
        mac<METHOD, FIRST, F>(g, uj, sv, mn, mcv, kq, ks, m);
        if (i % kRedEvery == kRedEvery - 1) {
#pragma unroll
            for (int r = 0; r < kR; ++r) {
                uj[r] = red(uj[r], m);
                if (!F) sv[r] = red(sv[r], m);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
        uj[r] = red(uj[r], m);
        if (!F) sv[r] = red(sv[r], m);
    }
}

// One accumulator step of gate `gate`, this wave's half of every polynomial
// (HbProd, mk-acc-xzw.cpp:231-290, fused with AddToAccXZW{,0},
// xzw.cpp:292-381; parties index + 1, ..., index, the index party's sum kept for
// the f-part).
template <int METHOD, bool FIRST>
__device__ __forceinline__ void one_gate(const StepArgs& a, uint32_t gate, Bufs& bufs, const Lane& ln) {
    const FMod& m = a.m;
    const uint32_t k = a.k, index = a.index;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    constexpr uint32_t polyB = kN * 8u;
    const uint32_t vo = ln.w * (polyB / 2u) + ln.l * 16u;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB);
    const __amdgpu_buffer_rsrc_t rt = make_rsrc(a.tab, kTabD * 8u);
    const __amdgpu_buffer_rsrc_t rp = make_rsrc(a.psi, 2u * kN * 8u);
    const KeySrc ks0{make_rsrc(a.key1, a.dg * 2 * polyB), make_rsrc(a.key2, a.dg * 2 * polyB),
                     make_rsrc(a.keys, a.dg * 2 * polyB), make_rsrc(a.pkey, k * a.dg * polyB), vo, 0u, 0u};
    const Mono mc = make_mono(c, ln.l, ln.w), mneg = make_mono(cneg, ln.l, ln.w);
    // X^-c at this lane's slots, once per step; X^c too in the first step (its d_i,
    // f_i use it in every MAC), per party for the later steps' rotation only (32 VGPRs
    // fewer across the digit loop)
    double mn[kR], mcv[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) {
        mn[r] = METHOD == XZW ? ldd(rp, mneg.word(r)) : 0.0;
        mcv[r] = FIRST ? ldd(rp, mc.word(r)) : 0.0;
    }
    double sv[kR], uj[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) sv[r] = 0.0;
#pragma unroll 1
    for (uint32_t tt = 1; tt <= k; ++tt) {
        const uint32_t u = index + tt < k ? index + tt : index + tt - k;
        double x[kR], mw[kR];
        load_poly(x, rin, vo, u * polyB);
#pragma unroll
        for (int r = 0; r < kR; ++r) mw[r] = FIRST ? 0.0 : ldd(rp, mc.word(r));
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            uj[r] = FIRST ? 0.0 : x[r];
            // acctemp = acc (X^c - 1)      (xzw.cpp:336-338); the first step overwrites acc
            if (!FIRST) x[r] = __dsub_rn(mm(x[r], mw[r], m), x[r]);
        }
        digits_pass<METHOD, FIRST, false>(x, uj, sv, mn, mcv, a, bufs, rt, ln, ks0, u);
        if (tt < k) store_poly(uj, rout, vo, u * polyB);
    }
    // f-part: iNTT(sumV) -> SDD -> NTT -> acc[index] += <., f>      (xzw.cpp:272-289)
    digits_pass<METHOD, FIRST, true>(sv, uj, sv, mn, mcv, a, bufs, rt, ln, ks0, index);
    store_poly(uj, rout, vo, index * polyB);
}

// two waves per gate, four gates (eight waves, two per SIMD: launch bounds in waves
// per SIMD, so up to 256 registers per wave) per CU, looping over the batch
template <int METHOD, bool FIRST>
__global__ __launch_bounds__(128, 2) void step_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Lane ln{l, w, (w * 64u + l) * 16u};
    Bufs bufs{smem, 0u};
    for (uint32_t gate = blockIdx.x; gate < a.B; gate += gridDim.x) one_gate<METHOD, FIRST>(a, gate, bufs, ln);
}

// primitive kernels for parity tests: one polynomial per 2-wave workgroup, canonical
// u64 words in the reference's order in and out
__global__ __launch_bounds__(128, 2) void ntt_fwd_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                         const double* tab, const double* twf, FMod m) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const uint32_t l = threadIdx.x & 63u, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Lane ln{l, w, (w * 64u + l) * 16u};
    const uint64_t* src = in + (size_t)blockIdx.x * kN;
    double x[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) x[r] = fp64::balanced(src[pos_a(w, l, r)], m);
    Bufs bufs{smem, 0u};
    ntt_fwd<kFwd>(x, bufs, twf, make_rsrc(tab, kTabD * 8u), ln, m);
#pragma unroll
    for (int r = 0; r < kR; ++r) out[(size_t)blockIdx.x * kN + pos_c(w, l, r)] = fp64::canon(x[r], m);
}
__global__ __launch_bounds__(128, 2) void ntt_inv_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                         const double* tab, const double* tis, FMod m) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const uint32_t l = threadIdx.x & 63u, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Lane ln{l, w, (w * 64u + l) * 16u};
    const uint64_t* src = in + (size_t)blockIdx.x * kN;
    double x[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) x[r] = fp64::balanced(src[pos_c(w, l, r)], m);
    Bufs bufs{smem, 0u};
    ntt_inv(x, bufs, tis, make_rsrc(tab, kTabD * 8u), ln, m);
#pragma unroll
    for (int r = 0; r < kR; ++r) out[(size_t)blockIdx.x * kN + pos_a(w, l, r)] = fp64::canon(x[r], m);
}

// batch prologue / epilogue with the C16 permutation: canonical u64 words (reference
// EVAL order) <-> balanced doubles (C16); a word >= Q raises `bad` and reads as 0
__global__ void to_c16_kernel(const uint64_t* __restrict__ in, double* __restrict__ out, size_t count, FMod m,
                              uint64_t Q, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    uint64_t x = in[idx];
    if (x >= Q) {
        *bad = 1u;
        x = 0;
    }
    const size_t poly = idx / kN;
    out[poly * kN + c16_index((uint32_t)(idx % kN))] = fp64::balanced(x, m);
}
__global__ void from_c16_kernel(const double* __restrict__ in, uint64_t* __restrict__ out, size_t count, FMod m) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    const size_t poly = idx / kN;
    out[idx] = fp64::canon(in[poly * kN + c16_index((uint32_t)(idx % kN))], m);
}

}  // namespace widereg2

}  // namespace
