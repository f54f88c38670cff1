// mkacc_engine.hip -- MI355X (gfx950) engine for the multi-key blind-rotation
// accumulator UniEncAccumulatorXZW{,_B}::EvalAcc and its C ABI
// (include/mkfhe_amd.h).
//
// Execution model:
//   * a batch of B independent gates advances one accumulator step (u, i) per
//     kernel launch, so the step's key block is read from HBM once and served
//     from L2 to every gate;
//   * one wavefront owns one gate for the whole step: all of HbProd's NTTs,
//     digit decompositions and MACs run out of that wave's VGPRs plus an
//     8 KiB LDS transpose scratch -- no workgroup barriers;
//   * the accumulator lives in HBM between steps in the "C4" EVAL layout,
//     pre-scaled by N^-1 (keys too), which removes every N^-1 multiply from the
//     inverse NTTs while keeping all results exact mod Q.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mkfhe_amd.h"
#include "mkacc_device.hpp"
#include "mkacc_host_math.hpp"

using namespace mkacc;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return fail(MKACC_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));    \
    } while (0)

// 256-thread workgroups, two per CU (2 waves / SIMD, LDS 65.8 KB each).
// The round-1 wrong results in waves 4-7 of 512-thread workgroups were the
// co-resident-wave store-data hazard of 16-byte buffer stores (DESIGN.md s2;
// fixed by bstore4, guarded by tools/isa_audit.py), not the workgroup shape;
// two 4-wave workgroups per CU stay because they were measured faster than
// one 8-wave workgroup sharing a single LDS table image.
constexpr int kWavesPerBlock = 4;
constexpr int kThreads = 64 * kWavesPerBlock;

// Table image (built once per context, HBM), in uint2 pairs:
//   [0, kTwlPairs)              forward per-lane twiddles (mkacc_device.hpp layout)
//   [kTwlPairs, +kInvImgPairs)  inverse per-lane twiddles and the psi^-i twist (ntt_inv)
//   [kPsiOff, + 2N)             psi^e (e in [0, 2N)) with Shoup companion, at psi_pos(e)
//   [kPsm1Off, + 2N)            psi^e - 1 with Shoup companion, at psi_pos(e)
// The NTTs read the twiddle runs from HBM/L2 (L1-resident, coalesced); the
// psi^e - 1 table, gathered at data-dependent slots, is copied into LDS at kernel
// start, followed by one transpose scratch of kLdsWords per wave.
constexpr int kPsiPairs = 2 * kN;
constexpr int kPsiOff = kTwlPairs + kInvImgPairs;
constexpr int kPsm1Off = kPsiOff + kPsiPairs;
constexpr int kImgPairs = kPsm1Off + kPsiPairs;
constexpr int kImgWords = 2 * kImgPairs;
static_assert(kPsm1Off % 2 == 0 && kTwlC % 2 == 0, "LDS tables are copied with dwordx4");
// LDS: [forward stage-10 twiddles, 1024 pairs][psi^e - 1 table, 2N pairs][scratch]
constexpr int kLdsTabWords = 2 * (1024 + kPsiPairs);
constexpr size_t kStepLdsBytes = (size_t)(kLdsTabWords + kWavesPerBlock * kLdsWords) * 4;
static_assert(kLdsTabWords % 4 == 0, "LDS tables are copied with dwordx4");
static_assert(2 * kStepLdsBytes <= 160 * 1024, "two workgroups per CU");

// Bank-spreading position of psi^e in the LDS table.  A wave gathers
// e = c (2 brv6(lane) + 1) + 128 c brv5(r) mod 2N (Mono): the low 7 bits are
// the lane's alone, the register part only moves bits 7..11.  Xor-ing bits 5..6
// into bits 0..1 touches the low 7 bits only, so the gather address stays
// additive in r (Mono::at: one add and one and), and it spreads the 64 lanes
// over all 32 bank pairs of a ds_read_b64 when c is odd or 2 mod 4 -- the best
// any swizzle of the low bits can do.  Exhaustively over all c and r (model:
// most distinct dwords per bank, 2 = conflict-free) this averages 3.83 LDS
// cycles per gather against 4.28 for the earlier e ^ ((e >> 5) & 31), which
// also cost 6 VALU of address arithmetic per gather instead of 2.
// MKACC_PSI_HI=1 (A/B): the earlier e ^ ((e >> 5) & 31), gathered with 4 VALU
#ifndef MKACC_PSI_HI
#define MKACC_PSI_HI 0
#endif
__host__ __device__ __forceinline__ uint32_t psi_pos(uint32_t e) {
    return MKACC_PSI_HI ? e ^ ((e >> 5) & 31u) : e ^ ((e >> 5) & 3u);
}

enum { XZW = 0, XZW_B = 1 };

// Device key words (upload_keys_impl / key_layout_kernel): every evk / pkey word
// is stored times N^-1 * 2^32 mod Q -- N^-1 because the accumulator lives scaled by
// N^-1 (the inverse NTT then needs no N^-1), 2^32 so that one Montgomery reduction
// (redc) of a lazy sum of key products returns the plain sum.  For MKNTRU the
// ev1 block of every step i < n holds ev1 + ev2 (both the d- and f-halves), so
// ev1 - ev2 X^-c = (ev1 + ev2) + ev2 (X^(N-c) - 1) is one product with a
// psi^e - 1 table entry (key_eff).
struct StepArgs {
    const uint32_t* acc_in;    // [B][k][N] C4, scaled by N^-1, residues in [0, 2Q)
    uint32_t* acc_out;         // [B][k][N]
    const uint32_t* cvals;     // [B] monomial exponents c of this step, in [0, 2N)
    const uint32_t* key1;      // ev1 (+ ev2 for MKNTRU) of step (u, i) : [dg][2][N] C4
    const uint32_t* key2;      // ev2 = (*ek)[u][1][i] (XZW)
    const uint32_t* keys;      // evs = (*ek)[0][0][n] (first step)
    const uint32_t* pkey;      // [k][dg][N]
    const uint32_t* img;       // table image [kImgWords]
    const uint2* tw_fwd;       // [N] reference forward table (pass A, scalar reads)
    const uint2* tw_inv;       // [32] inverse pass-1 table (ntt_inv)
    uint32_t* dscr;            // [B][dg][N] C4 scratch of the step's d_i (mk_step_kernel DSCR) or null
    uint32_t B, k, index;
    Mod m;
    SddConsts sd;
};

// Copy the forward stage-10 twiddles (the largest per-lane run, used by 3/4
// of the NTTs) and the psi^e - 1 table of the image into this workgroup's LDS.
__device__ __forceinline__ void load_image(uint32_t* smem, const uint32_t* img) {
    const uint4* src = reinterpret_cast<const uint4*>(img);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) dst[i] = src[kTwlC / 2 + i];
    for (int i = threadIdx.x; i < kN; i += blockDim.x) dst[512 + i] = src[kPsm1Off / 2 + i];
    __syncthreads();
}

struct Tables {
    const uint2* twf;    // HBM image: forward per-lane twiddles
    const uint2* twi;    // HBM image: inverse per-lane twiddles + twist
    const uint2* twfc;   // LDS: forward stage-10 twiddles
    const uint2* psi;    // LDS: psi^e - 1
};
__device__ __forceinline__ Tables tables(uint32_t* smem, const uint32_t* img) {
    const uint2* g = reinterpret_cast<const uint2*>(img);
    const uint2* t = reinterpret_cast<const uint2*>(smem);
    return Tables{g, g + kTwlPairs, t, t + 1024};
}

// Monomial X^e at EVAL slot j = (lane << 5) | r: the reference stores
// a(psi^(2 brv(j) + 1)) at position j (transformnat-impl.h:705-760), so
// X^c -> psi^(c (2 brv(j) + 1)), with 2 brv(j) + 1 = 128 brv5(r) + (2 brv6(lane) + 1).
// co = c * (2 brv6(lane) + 1) per lane; the r part 128 c brv5(r) is
// wave-uniform and moves only bits 7..11 of e, which psi_pos leaves in place, so
// the byte offset of psi_pos(e) is (w + 1024 c brv5(r)) & 0x7fff with the per-lane
// w = psi_pos(co mod 2N) * 8.  at() returns the LDS pair of psi^e - 1, i.e. the
// EVAL slot of X^c - 1.
struct Mono {
    uint32_t w;         // per lane: 8 psi_pos(c (2 brv6(l) + 1) mod 2N)
    uint32_t c;         // wave-uniform exponent
    __device__ __forceinline__ uint2 at(const uint2* psi, int r) const {
        constexpr uint32_t kBr5[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                       1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};
        // the wave-uniform part is recomputed per use (one s_mul) rather than
        // kept as 32 hoisted SGPR constants per monomial; the add is volatile asm
        // so the 32 per-slot addresses are not hoisted out of the party / digit
        // loops (they would stay live in VGPRs across the NTTs)
        uint32_t cs = c;
        asm volatile("" : "+s"(cs));
        uint32_t a;
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(a) : "s"(cs * (1024u * kBr5[r])), "v"(w));
        a &= 0x7fffu;
        if (MKACC_PSI_HI) a ^= (a >> 5) & 0xf8u;   // 8 psi_pos(e) from 8 e
        return *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(psi) + a);
    }
};
__device__ __forceinline__ Mono make_mono(uint32_t c, uint32_t l) {
    const uint32_t o = ((__brev(l) >> 26) << 1) | 1u;   // 2 brv6(l) + 1
    const uint32_t co = __umul24(c, o) & (2u * kN - 1u);
    return Mono{(MKACC_PSI_HI ? co : psi_pos(co)) << 3, c};
}

// Lazy Shoup product x*w in [0, 2Q) (x < 2^32)
__device__ __forceinline__ uint32_t mul_shoup_lazy(uint32_t x, uint2 w, uint32_t Q) {
    const uint32_t q = __umulhi(x, w.y);
    return (uint32_t)mad64_pin<true>(q, 0u - Q, mul64_pin<false>(x, w.x));   // x*w - q*Q in [0, 2Q)
}

// Ranges of the lazy Montgomery sums, in units of Q (values) and Q^2 (sums).
// redc needs a sum below Q * 2^32 > 32 Q^2.  Digit-NTT outputs are < kG Q
// (digit_range), effective key words from key_eff < kD Q, and the previous
// accumulator joins the party sum as acc * (2^32 mod Q) < 2 Q^2 when it fits
// (kAccInSum), otherwise it is added after the reduction.
template <int DG, int METHOD, bool FIRST>
struct Bounds {
    static constexpr int kG = DG > 4 ? 2 : 4;
    static constexpr int kD = DG * kG * 3 + 2 <= 32 ? 3 : (DG * kG * 2 <= 32 ? 2 : 1);
    // the d-words the party sums actually see: XZW_B steps after the first use ev1 itself
    static constexpr int kDSum = (METHOD == XZW_B && !FIRST) ? 1 : kD;
    static constexpr bool kAccInSum = !FIRST && DG * kG * kDSum + 2 <= 32;
    static_assert(DG * kG * kDSum + (kAccInSum ? 2 : 0) <= 32, "party sum bound");
    // sumV gains DG * kG per party (pkey canonical); fold64 leaves < 2
    static constexpr int kSvParty = DG * kG;
    // f-part: the index party's folded sum (< 2, < 4 with the accumulator added
    // there) plus DG products with canonical f-words (split form) or, in the
    // first step, with f-words reduced to canonical
    static_assert(4 + DG * kG <= 32, "f-part bound");
};

// [0, 3Q) -> [0, KD Q)
template <int KD>
__device__ __forceinline__ uint32_t from3q(uint32_t d, uint32_t Q) {
    if (KD <= 2) d = min(d, d - 2u * Q);
    if (KD <= 1) d = min(d, d - Q);
    return d;
}

// Effective key word d_i / f_i of mk-acc-xzw(_B).cpp AddToAccXZW{,0}, below KD Q.
// k1 is the stored ev1 word (ev1 + ev2 for MKNTRU, StepArgs), k2 = ev2, ks = evs.
template <int METHOD, bool FIRST, int KD>
__device__ __forceinline__ uint32_t key_eff(uint32_t k1, uint32_t k2, uint32_t ks, const uint2* psi,
                                            const Mono& mp, const Mono& mn, int r, uint32_t Q) {
    if (METHOD == XZW) {
        if (FIRST) {
            // evs + ev1*(X^c-1) + ev2*(X^-c-1)          (xzw.cpp:375-378)
            const uint32_t e1 = k1 + Q - k2;                         // ev1, (0, 2Q)
            uint32_t d = ks + mul_shoup_lazy(e1, mp.at(psi, r), Q) + mul_shoup_lazy(k2, mn.at(psi, r), Q);
            d = min(d, d - 2u * Q);                                  // [0, 5Q) -> [0, 3Q)
            return from3q<KD>(d, Q);
        }
        // ev1 - ev2*(X^-c - 1) - ev2  ==  ev1 - ev2*X^-c  ==  (ev1 + ev2) + ev2*(X^(N-c) - 1)
        // (xzw.cpp:322-325); mn is the monomial X^(N-c) = -X^-c here
        return from3q<KD>(k1 + mul_shoup_lazy(k2, mn.at(psi, r), Q), Q);
    } else {
        if (FIRST) {
            // evs + ev1*(X^c-1)                            (xzw_B.cpp:368-371)
            return from3q<KD>(ks + mul_shoup_lazy(k1, mp.at(psi, r), Q), Q);
        }
        return k1;                                        // (xzw_B.cpp:311-314)
    }
}

// digit NTT outputs: [0, 4Q) for DG <= 4, brought to [0, 2Q) at DG = 5 (Bounds::kG)
template <int DG>
__device__ __forceinline__ void digit_range(uint32_t (&x)[kRegs], uint32_t Q) {
    if (DG > 4) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) x[r] = min(x[r], x[r] - 2u * Q);
    }
}

// Key words of one 4-register group of a MAC: software-pipelined kPrefetch
// groups ahead so the L2 latency of the step's key block overlaps the arithmetic.
template <int DG>
#ifndef MKACC_PF3
#define MKACC_PF3 1
#endif
struct Prefetch { static constexpr int value = DG <= 3 ? MKACC_PF3 : 0; };
// accumulator loads: each gate's own rows, written by the previous step launch
__device__ __forceinline__ u32x4 aload4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
}
// key-block loads (shared by every gate of the launch, streamed from L2)
__device__ __forceinline__ u32x4 kload4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    // default cache policy: the 8 waves of a CU share the key lines through L1
    // (non-temporal loads measured 11% slower, profiles/r2/ab_series1.txt)
    return __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
}
struct KeyGroup {
    u32x4 k1, k2, ks, pk, acc;
    uint2 mono[4];   // X^(N-c) - 1 at the group's slots (XZW after the first step)
};
// per-wave resources of the MAC helpers
struct StepRes {
    __amdgpu_buffer_rsrc_t rin, rk1, rk2, rks, rpk, rds;
    const uint2* psi;
    Mono mp, mn;
    Mod m;
    uint32_t vo;
};

// uj_u += g * d_i ; sv += g * P[u][i]          (xzw.cpp:263-269)
// START (digit 0): uj_u starts from acc_u * 2^32 (AddToAccXZW's acc + acctemp,
// xzw.cpp:342-344; in Montgomery form, redc divides by 2^32) when the bound
// allows, streamed in with the keys; 0 in the FIRST step, where AddToAccXZW0
// overwrites acc (xzw.cpp:380).
// The caller issues the first kPrefetch key groups (issue()), run() streams
// the rest kPrefetch groups ahead.  (Issuing the first group before the digit
// NTT spilled 23 VGPRs and measured 4% slower, profiles/r2/ab_series1.txt.)
// DS (XZW after the first step, mk_step_kernel DSCR): d_i is the same for every
// party of the step, so the first party pass computes it and stores it to the
// gate's HBM scratch (DS = 1) and the later passes load it (DS = 2) instead of
// the ev1'/ev2 words and the psi^e - 1 gathers; DS = 0 computes it per party.
template <int DG, int METHOD, bool FIRST, bool START, int DS = 0>
struct DigitMac {
    using Bd = Bounds<DG, METHOD, FIRST>;
    static_assert(DS == 0 || (METHOD == XZW && !FIRST), "d_i scratch: XZW steps after the first");
    static constexpr bool kAcc = START && Bd::kAccInSum;
    // MKACC_MONO_PF=0 (A/B): gather X^(N-c) - 1 at use instead of with the key group
#ifndef MKACC_MONO_PF
#define MKACC_MONO_PF 1
#endif
    static constexpr bool kMonoPf = MKACC_MONO_PF && METHOD == XZW && !FIRST && DS != 2;
    // a d_i reload comes from HBM and frees the k2 / psi registers: prefetched
    // 3 groups ahead at DG <= 3, 2 at DG >= 4 (3 spill 10 VGPRs there); 1 group measured
    // 1-4% slower (profiles/r2/ab_dscr.txt)
#ifndef MKACC_DSCR_PF
#define MKACC_DSCR_PF 0
#endif
#ifndef MKACC_DSCR_WAIT
#define MKACC_DSCR_WAIT 0
#endif
    static constexpr int kPrefetch = DS == 2 ? (MKACC_DSCR_PF ? MKACC_DSCR_PF : (DG <= 3 ? 3 : 2)) : Prefetch<DG>::value;
    static constexpr int kBuf = kPrefetch + 1;
    const StepRes& sr;
    uint32_t koff, poff, aoff, doff;
    __device__ __forceinline__ DigitMac(const StepRes& r, int i, uint32_t u)
        : sr(r), koff((uint32_t)(2 * i) * (kN * 4u)), poff((u * DG + (uint32_t)i) * (kN * 4u)), aoff(u * (kN * 4u)),
          doff((uint32_t)i * (kN * 4u)) {}
    __device__ __forceinline__ void issue(KeyGroup& t, int gq) const {
        const uint32_t go = gq * 1024u;
        if (DS == 2)
            t.k1 = aload4(sr.rds, sr.vo, doff + go);   // d_i of the first party pass
        else
            t.k1 = kload4(sr.rk1, sr.vo, koff + go);
        t.pk = kload4(sr.rpk, sr.vo, poff + go);
        if (METHOD == XZW && DS != 2) t.k2 = kload4(sr.rk2, sr.vo, koff + go);
        if (FIRST) t.ks = kload4(sr.rks, sr.vo, koff + go);
        if (kAcc) t.acc = aload4(sr.rin, sr.vo, aoff + go);
        if (kMonoPf) {
#pragma unroll
            for (int e = 0; e < 4; ++e) t.mono[e] = sr.mn.at(sr.psi, 4 * gq + e);
        }
    }
    __device__ __forceinline__ void run(const uint32_t (&g)[kRegs], uint64_t (&uj)[kRegs], uint64_t (&sv)[kRegs],
                                        KeyGroup (&kg)[kBuf]) const {
        const uint32_t Q = sr.m.Q;
#pragma unroll
        for (int gq = 0; gq < 8; ++gq) {
            if (gq + kPrefetch < 8) issue(kg[(gq + kPrefetch) % kBuf], gq + kPrefetch);
            const KeyGroup& t = kg[gq % kBuf];
            u32x4 dv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * gq + e;
                const uint32_t deff =
                    DS == 2 ? t.k1[e]
                    : kMonoPf ? from3q<Bd::kD>(t.k1[e] + mul_shoup_lazy(t.k2[e], t.mono[e], Q), Q)   // = key_eff
                              : key_eff<METHOD, FIRST, Bd::kD>(t.k1[e], t.k2[e], t.ks[e], sr.psi, sr.mp, sr.mn, r, Q);
                dv[e] = deff;
                const uint64_t base = kAcc ? mad64(t.acc[e], sr.m.r32, 0) : (START ? 0ull : uj[r]);
                uj[r] = mad64(g[r], deff, base);
                sv[r] = mad64(g[r], t.pk[e], sv[r]);
            }
            if (DS == 1) bstore4(dv, sr.rds, sr.vo, doff + gq * 1024u);
            sched_fence();
        }
    }
};

// w += h * f_i                                  (xzw.cpp:281-288)
// (first step, and XZW_B: f-words reduced to canonical, Bounds' f-part bound)
template <int DG, int METHOD, bool FIRST>
__device__ __forceinline__ void mac_index(const uint32_t (&h)[kRegs], int i, uint64_t (&w)[kRegs],
                                          __amdgpu_buffer_rsrc_t rk1, __amdgpu_buffer_rsrc_t rk2,
                                          __amdgpu_buffer_rsrc_t rks, const uint2* psi, const Mono& mp,
                                          const Mono& mn, uint32_t vo, uint32_t Q) {
    const uint32_t polyB = kN * 4u;
    const uint32_t koff = (uint32_t)(2 * i + 1) * polyB;
    constexpr int kPrefetch = Prefetch<DG>::value;
    KeyGroup kg[kPrefetch + 1];
    auto issue = [&](KeyGroup& t, int gq) {
        const uint32_t go = gq * 1024u;
        t.k1 = kload4(rk1, vo, koff + go);
        if (METHOD == XZW) t.k2 = kload4(rk2, vo, koff + go);
        if (FIRST) t.ks = kload4(rks, vo, koff + go);
    };
#pragma unroll
    for (int j = 0; j < kPrefetch; ++j) issue(kg[j], j);
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) {
        if (gq + kPrefetch < 8) issue(kg[(gq + kPrefetch) % (kPrefetch + 1)], gq + kPrefetch);
        const KeyGroup& t = kg[gq % (kPrefetch + 1)];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * gq + e;
            const uint32_t feff = key_eff<METHOD, FIRST, 1>(t.k1[e], t.k2[e], t.ks[e], psi, mp, mn, r, Q);
            w[r] = mad64(h[r], feff, w[r]);
        }
        sched_fence();
    }
}

// XZW steps after the first: f_i = ev1'_i - ev2'_i X^-c (xzw.cpp:322-325) is
// linear in the keys, so with the stored ev1 + ev2:
//   sum_i h_i f_i = sum_i h_i (ev1 + ev2)'_i + (X^(N-c) - 1) sum_i h_i ev2'_i
// two lazy sums per slot here and ONE monomial product per slot after the last
// digit (step_body) instead of one per slot and digit.
template <int DG>
struct SplitMac {
    static constexpr int kPrefetch = Prefetch<DG>::value;
    static constexpr int kBuf = kPrefetch + 1;
    const StepRes& sr;
    uint32_t koff;
    __device__ __forceinline__ SplitMac(const StepRes& r, int i) : sr(r), koff((uint32_t)(2 * i + 1) * (kN * 4u)) {}
    __device__ __forceinline__ void issue(KeyGroup& t, int gq) const {
        const uint32_t go = gq * 1024u;
        t.k1 = kload4(sr.rk1, sr.vo, koff + go);
        t.k2 = kload4(sr.rk2, sr.vo, koff + go);
    }
    __device__ __forceinline__ void run(const uint32_t (&h)[kRegs], uint64_t (&w)[kRegs], uint64_t (&w2)[kRegs],
                                        KeyGroup (&kg)[kBuf]) const {
#pragma unroll
        for (int gq = 0; gq < 8; ++gq) {
            if (gq + kPrefetch < 8) issue(kg[(gq + kPrefetch) % kBuf], gq + kPrefetch);
            const KeyGroup& t = kg[gq % kBuf];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * gq + e;
                w[r] = mad64(h[r], t.k1[e], w[r]);
                w2[r] = mad64(h[r], t.k2[e], w2[r]);
            }
            sched_fence();
        }
    }
};

// Per-wave state shared by the passes of one step.
struct StepCtx {
    const Tables tb;
    uint32_t* lds;
    const uint2* tw_fwd;
    const uint2* tw_inv;
    Mod m;
    SddConsts sd;
    Mono mp, mn;
    uint32_t l, vo;
    __amdgpu_buffer_rsrc_t rin, rout, rk1, rk2, rks, rpk, rds;
    __device__ __forceinline__ StepRes res() const { return StepRes{rin, rk1, rk2, rks, rpk, rds, tb.psi, mp, mn, m, vo}; }
};

// One party u of HbProd (mk-acc-xzw.cpp:245-270) fused with AddToAccXZW's
// rotation and final add (xzw.cpp:336-344):
//   uj_u = (FIRST ? 0 : acc_u) + sum_i NTT(g_i) * d_i,   g = SDD(iNTT(acc_u * (X^c - 1)))
//   sv  += sum_i NTT(g_i) * P[u][i]
// Party `index` is processed last (LAST): its lazy sum stays in registers
// (`uj`, folded) and receives the f-part of HbProd before the single store.
template <int DG, int METHOD, bool FIRST, bool LAST, int DS = 0>
__device__ __forceinline__ void party_pass(const StepCtx& s, uint32_t u, uint64_t (&sv)[kRegs],
                                           uint64_t (&uj)[kRegs]) {
    using Bd = Bounds<DG, METHOD, FIRST>;
    const uint32_t Q = s.m.Q, polyB = kN * 4u;
    uint32_t x[kRegs];
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) {
        const u32x4 t = aload4(s.rin, s.vo, u * polyB + gq * 1024u);
        x[4 * gq] = t.x; x[4 * gq + 1] = t.y; x[4 * gq + 2] = t.z; x[4 * gq + 3] = t.w;
    }
    if (!FIRST) {
        // acctemp = acc * (X^c - 1)                     (xzw.cpp:336-338)
        // one Shoup product with the psi^e - 1 table entry: [0, 2Q) for any x;
        // the 32 table reads are issued while the accumulator loads are in flight
        uint2 mw[kRegs];
#pragma unroll
        for (int r = 0; r < kRegs; ++r) mw[r] = s.mp.at(s.tb.psi, r);
        sched_fence();
#pragma unroll
        for (int r = 0; r < kRegs; ++r) x[r] = mul_shoup_lazy(x[r], mw[r], Q);
    }
    ntt_inv(x, s.lds, s.tw_inv, s.tb.twi, s.l, Q);
    // SignedDigitDecompose (mk-acc.cpp:54-80): digit 1 -> x, digits 2.. packed
    PackedDigits<DG> pd;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        x[r] = pd.put(r, sdd_offset(x[r], s.sd), s.sd);
        if ((r & 7) == 7) sched_fence();
    }
    const StepRes sr = s.res();
    {
        const DigitMac<DG, METHOD, FIRST, true, DS> mac(sr, 0, u);
        KeyGroup kg[mac.kBuf];
        ntt_fwd(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
        digit_range<DG>(x, Q);
        // MKACC_DSCR_WAIT=1: the d_i scratch stores of the first pass are waited for
        // here, just before the first reload, instead of right after that pass
        if (DS == 2 && MKACC_DSCR_WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < mac.kPrefetch; ++j) mac.issue(kg[j], j);
        mac.run(x, uj, sv, kg);
    }
#pragma unroll 1
    for (int i = 1; i < DG; ++i) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) x[r] = pd.get(r, i + 1, s.sd);
        const DigitMac<DG, METHOD, FIRST, false, DS> mac(sr, i, u);
        KeyGroup kg[mac.kBuf];
        ntt_fwd(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
        digit_range<DG>(x, Q);
#pragma unroll
        for (int j = 0; j < mac.kPrefetch; ++j) mac.issue(kg[j], j);
        mac.run(x, uj, sv, kg);
    }
    if (LAST) {
        // the index party's sum continues into the f-part (step_body)
#pragma unroll
        for (int r = 0; r < kRegs; ++r) uj[r] = fold64(uj[r], s.m.r32);
        return;
    }
    // acc_u <- redc(uj_u) (+ acc_u when it is not in the sum), in [0, 2Q)
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) {
        u32x4 t;
        if constexpr (!Bd::kAccInSum && !FIRST) t = aload4(s.rin, s.vo, u * polyB + gq * 1024u);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * gq + e;
            uint32_t v = redc(uj[r], Q, s.m.qinv);
            if constexpr (!Bd::kAccInSum && !FIRST) {
                v += t[e];
                v = min(v, v - 2u * Q);
            }
            t[e] = v;
        }
        bstore4(t, s.rout, s.vo, u * polyB + gq * 1024u);
    }
}

template <int DG, int METHOD, bool FIRST, bool DSCR>
__device__ __forceinline__ void step_body(const StepCtx& s, uint32_t k, uint32_t index);
template <int DG, int METHOD, bool FIRST>
__device__ __forceinline__ void f_part(const StepCtx& s, uint32_t index, uint64_t (&w)[kRegs], uint32_t (&x)[kRegs]);

// DSCR: d_i computed once per step and gate (first party pass) and reloaded from
// a.dscr by the other k - 1 passes (DigitMac DS); the host picks it by k.
template <int DG, int METHOD, bool FIRST, bool DSCR = false>
__global__ __launch_bounds__(kThreads, 2) void mk_step_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image(smem, a.img);
    const uint32_t l = threadIdx.x & 63u;
    // wave-uniform (SGPR) gate index: the per-gate buffer descriptors must be
    // scalar, otherwise every load through them becomes a waterfall loop
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gate = blockIdx.x * kWavesPerBlock + wv;
    if (gate >= a.B) return;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k;
    const uint32_t polyB = kN * 4u;
    const StepCtx s{tables(smem, a.img),
                    smem + kLdsTabWords + wv * kLdsWords,
                    a.tw_fwd,
                    a.tw_inv,
                    a.m,
                    a.sd,
                    make_mono(c, l),
                    // X^-c in the first step; X^(N-c) = -X^-c in the later XZW steps (key_eff)
                    make_mono(FIRST || METHOD != XZW ? cneg : (cneg + kN) & (2u * kN - 1u), l),
                    l,
                    l * 16u,
                    make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB),
                    make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB),
                    make_rsrc(a.key1, DG * 2 * polyB),
                    make_rsrc(a.key2, DG * 2 * polyB),
                    make_rsrc(a.keys, DG * 2 * polyB),
                    make_rsrc(a.pkey, k * DG * polyB),
                    make_rsrc(DSCR ? a.dscr + (size_t)gate * DG * kN : a.acc_in, DSCR ? DG * polyB : 0u)};
    step_body<DG, METHOD, FIRST, DSCR>(s, k, a.index);
}

// Small batches (host: use_lat): one workgroup per gate and one wave per party,
// so the k party passes of a step run concurrently and only the f-part is
// serial -- 2 (dg + 1) transforms on a step's critical path instead of
// (k + 1)(dg + 1).  The same party_pass / f_part code as mk_step_kernel: each
// wave's sumV covers its own party; it is reduced to [0, 2Q), summed through
// LDS by the wave of party `index`, which then runs the f-part alone (the
// sums are exact mod Q, so the grouping is bit-exact).
constexpr uint32_t kLatMaxK = 8;
constexpr size_t lat_lds_bytes(uint32_t k) { return (size_t)(kLdsTabWords + k * kLdsWords) * 4; }
template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(64 * kLatMaxK, 1) void mk_lat_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image(smem, a.img);
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t u = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // this wave's party
    const uint32_t gate = blockIdx.x;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k, index = a.index;
    const uint32_t polyB = kN * 4u;
    uint32_t* scratch = smem + kLdsTabWords + u * kLdsWords;
    const StepCtx s{tables(smem, a.img),
                    scratch,
                    a.tw_fwd,
                    a.tw_inv,
                    a.m,
                    a.sd,
                    make_mono(c, l),
                    make_mono(FIRST || METHOD != XZW ? cneg : (cneg + kN) & (2u * kN - 1u), l),
                    l,
                    l * 16u,
                    make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB),
                    make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB),
                    make_rsrc(a.key1, DG * 2 * polyB),
                    make_rsrc(a.key2, DG * 2 * polyB),
                    make_rsrc(a.keys, DG * 2 * polyB),
                    make_rsrc(a.pkey, k * DG * polyB),
                    make_rsrc(a.acc_in, 0u)};
    const uint32_t Q = s.m.Q;
    uint64_t sv[kRegs], w[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) sv[r] = 0;
    if (u == index)
        party_pass<DG, METHOD, FIRST, true>(s, u, sv, w);
    else
        party_pass<DG, METHOD, FIRST, false>(s, u, sv, w);
    // this party's sumV share, [0, 2Q), into the wave's own (now idle) scratch
#pragma unroll
    for (int r = 0; r < kRegs; ++r) scratch[r * 64 + l] = redc(sv[r], Q, s.m.qinv);
    // redc's multiply-add is inline asm that writes its carry-out to VCC; hipcc
    // does not count it as a VALU write of VCC and computed the branch below with
    // an SALU write of VCC on the very next instruction.  The late VALU write
    // could land after it, zero VCC and send every wave down the index-party path
    // (intermittent wrong acc[index]; tools/isa_audit.py checks the distance).
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7" ::: "vcc");
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if (u != index) return;
    uint32_t x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        uint32_t v = 0;
        for (uint32_t p = 0; p < k; ++p) v += smem[kLdsTabWords + p * kLdsWords + r * 64 + l];   // < 16 Q
        v = min(v, v - 8u * Q);
        v = min(v, v - 4u * Q);
        x[r] = min(v, v - 2u * Q);                                                               // [0, 2Q)
    }
    f_part<DG, METHOD, FIRST>(s, index, w, x);
}

// One accumulator step for one gate per wavefront.
//   FIRST:  AddToAccXZW0 (mk-acc-xzw.cpp:347-381 / xzw_B.cpp:333-381): acc <- HbProd(acc)
//   else:   AddToAccXZW  (mk-acc-xzw.cpp:292-345 / xzw_B.cpp:281-330):
//           acc <- acc + HbProd(acc * (X^c - 1))
// HbProd is mk-acc-xzw.cpp:231-290, register resident: the per-slot sums
// uj_u = sum_i g_i d_i, sumV = sum_u sum_i g_i P[u][i] and w = sum_i h_i f_i are
// lazy 64-bit accumulators (v_mad_u64_u32) reduced once (Montgomery); all sums
// are exact mod Q, so the reordering (parties in the order index+1, ..., index)
// is bit-exact.
template <int DG, int METHOD, bool FIRST, bool DSCR>
__device__ __forceinline__ void step_body(const StepCtx& s, uint32_t k, uint32_t index) {
    using Bd = Bounds<DG, METHOD, FIRST>;
    const uint32_t Q = s.m.Q;
    uint64_t sv[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) sv[r] = 0;
    uint64_t w[kRegs];
    // sumV grows by kSvParty (units of Q^2) per party; fold it before it could
    // pass 32 (fold64 leaves < 2)
    int svb = 0;
    auto grow_sv = [&]() {
        svb += Bd::kSvParty;
        if (svb + Bd::kSvParty > 32) {
#pragma unroll
            for (int r = 0; r < kRegs; ++r) sv[r] = fold64(sv[r], s.m.r32);
            svb = 2;
        }
    };
    uint32_t t0 = 1;
    if constexpr (DSCR) {   // k >= 2 (host: use_dscr)
        party_pass<DG, METHOD, FIRST, false, 1>(s, index + 1 < k ? index + 1 : 0, sv, w);
        grow_sv();
        t0 = 2;
        // the scratch stores complete before the later passes read them back
        if (!MKACC_DSCR_WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (uint32_t t = t0; t < k; ++t) {
        party_pass<DG, METHOD, FIRST, false, DSCR ? 2 : 0>(s, index + t < k ? index + t : index + t - k, sv, w);
        grow_sv();
    }
    party_pass<DG, METHOD, FIRST, true, DSCR ? 2 : 0>(s, index, sv, w);
    uint32_t x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = redc(sv[r], Q, s.m.qinv);
    f_part<DG, METHOD, FIRST>(s, index, w, x);
}

// Second half of HbProd for party `index` (mk-acc-xzw.cpp:272-289) and the
// final store of acc[index]: w = its folded party sum (party_pass LAST),
// x = sumV in [0, 2Q).  iNTT(sumV) -> SDD -> NTT -> acc[index] += <., f>.
template <int DG, int METHOD, bool FIRST>
__device__ __forceinline__ void f_part(const StepCtx& s, uint32_t index, uint64_t (&w)[kRegs], uint32_t (&x)[kRegs]) {
    using Bd = Bounds<DG, METHOD, FIRST>;
    const uint32_t Q = s.m.Q;
    const uint32_t l = s.l;
    const uint32_t polyB = kN * 4u;
    if constexpr (!Bd::kAccInSum && !FIRST) {
        // acc[index] joins the f-part sum (Bounds: < 4 Q^2 with the folded party sum)
#pragma unroll
        for (int gq = 0; gq < 8; ++gq) {
            const u32x4 t = aload4(s.rin, s.vo, index * polyB + gq * 1024u);
#pragma unroll
            for (int e = 0; e < 4; ++e) w[4 * gq + e] = mad64(t[e], s.m.r32, w[4 * gq + e]);
        }
    }

    const StepRes sr = s.res();
    ntt_inv(x, s.lds, s.tw_inv, s.tb.twi, l, Q);
    PackedDigits<DG> pd;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        x[r] = pd.put(r, sdd_offset(x[r], s.sd), s.sd);
        if ((r & 7) == 7) sched_fence();
    }
    constexpr bool kSplit = METHOD == XZW && !FIRST;
    uint64_t w2[kSplit ? kRegs : 1];
    if constexpr (kSplit) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) w2[r] = 0;
    }
#pragma unroll 1
    for (int i = 0; i < DG; ++i) {
        if (i > 0) {
#pragma unroll
            for (int r = 0; r < kRegs; ++r) x[r] = pd.get(r, i + 1, s.sd);
        }
        if constexpr (kSplit) {
            const SplitMac<DG> mac(sr, i);
            KeyGroup kg[mac.kBuf];
            ntt_fwd(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, l, Q, s.m.m1);
            digit_range<DG>(x, Q);
#pragma unroll
            for (int j = 0; j < mac.kPrefetch; ++j) mac.issue(kg[j], j);
            mac.run(x, w, w2, kg);
        } else {
            ntt_fwd(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, l, Q, s.m.m1);
            digit_range<DG>(x, Q);
            mac_index<DG, METHOD, FIRST>(x, i, w, s.rk1, s.rk2, s.rks, s.tb.psi, s.mp, s.mn, s.vo, Q);
        }
    }
    const uint32_t ioff = index * polyB;
    uint2 mw[kSplit ? kRegs : 1];
    if constexpr (kSplit) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) mw[r] = s.mn.at(s.tb.psi, r);
    }
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) {
        u32x4 t;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * gq + e;
            uint32_t v = redc(w[r], Q, s.m.qinv);                                   // [0, 2Q)
            if constexpr (kSplit) {
                // + (X^(N-c) - 1) * sum_i h_i ev2'_i
                v += mul_shoup_lazy(redc(w2[r], Q, s.m.qinv), mw[r], Q);             // [0, 4Q)
                v = min(v, v - 2u * Q);
            }
            t[e] = v;
        }
        bstore4(t, s.rout, s.vo, ioff + gq * 1024u);
    }
}

// ---- batch prologue / epilogue kernels --------------------------------------

// c = floor(ct * 2N / q) (mk-acc-xzw.cpp:110,125) or c = ct (mk-acc-xzw_B.cpp:119,124),
// with c == 2N mapped to 0 (xzw.cpp:301).  Output layout [k*n][B].
// Device entry points validate their inputs where a kernel reads them anyway:
// a word outside its range raises the context's `bad` flag (reported by
// mkacc_sync as MKACC_E_RANGE); the monomial exponent stays masked to [0, 2N).
__global__ void prep_c_kernel(const uint32_t* __restrict__ ct, uint32_t* __restrict__ cvals, uint32_t B,
                              uint32_t kn, uint32_t method, uint32_t q, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)B * kn) return;
    const uint32_t s = (uint32_t)(idx / B), b = (uint32_t)(idx % B);
    const uint32_t raw = ct[(size_t)b * kn + s];
    if (raw >= (method == XZW ? q : 2u * kN + 1u)) *bad = 1u;   // XZW_B: c <= 2N (2N -> 0)
    uint32_t c = method == XZW ? (uint32_t)(((uint64_t)raw * (2u * kN)) / q) : raw;
    if (c >= 2u * kN) c -= 2u * kN;
    cvals[idx] = c;
}

// reference EVAL order -> C4, multiplied by a constant (N^-1 on the way in, N on the way out)
__global__ void eval_to_c4_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t npoly,
                                  uint32_t s, uint32_t sp, uint32_t Q, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= npoly * kN) return;
    const size_t p = idx / kN;
    const uint32_t j = (uint32_t)(idx % kN);
    const uint32_t x = in[idx];
    if (bad && x >= Q) *bad = 1u;
    out[p * kN + c4_index(j)] = mul_shoup(x, s, sp, Q);
}

// Key upload from device memory: reference layout [k][nk][n+1][dg][2][N] (EVAL,
// u32 or u64 words) -> device layout [k][n+1][nk][dg][2][N] in C4 order, times
// N^-1 2^32 (s, sp; StepArgs).  MKNTRU (nk = 2): the ev1 words of the steps i < n
// become ev1 + ev2.  pkey [k][dg][N] is the same map with nk = n1 = 1.
template <typename W>
__global__ void key_layout_kernel(const W* __restrict__ src, uint32_t* __restrict__ dst, size_t npolys, uint32_t nk,
                                  uint32_t n1, uint32_t dg2, uint32_t Q, uint32_t s, uint32_t sp,
                                  uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= npolys * kN) return;
    size_t p = idx / kN;
    const uint32_t j = (uint32_t)(idx % kN);
    const uint32_t dp = (uint32_t)(p % dg2); p /= dg2;
    const uint32_t i = (uint32_t)(p % n1); p /= n1;
    const uint32_t jj = (uint32_t)(p % nk);
    const size_t u = p / nk;
    const size_t dpoly = ((u * n1 + i) * nk + jj) * dg2 + dp;
    const uint64_t x = (uint64_t)src[idx];
    if (x >= Q) *bad = 1u;
    uint32_t v = (uint32_t)x;
    if (nk == 2 && jj == 0 && i + 1 < n1) {
        // ev1 + ev2 (the ev2 word is range-checked by its own thread)
        const uint64_t y = (uint64_t)src[idx + (size_t)n1 * dg2 * kN];
        v = (uint32_t)((x + (y < Q ? y : 0)) % Q);
    }
    dst[dpoly * kN + c4_index(j)] = mul_shoup(v, s, sp, Q);
}
__global__ void c4_to_eval_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t npoly,
                                  uint32_t s, uint32_t sp, uint32_t Q) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= npoly * kN) return;
    const size_t p = idx / kN;
    const uint32_t j = (uint32_t)(idx % kN);
    out[idx] = mul_shoup(in[p * kN + c4_index(j)], s, sp, Q);
}

// ---- primitive kernels (parity tests of the NTT / SDD building blocks) -------

__global__ __launch_bounds__(kThreads) void ntt_fwd_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                            uint32_t count, const uint32_t* img, const uint2* twf,
                                                            uint32_t Q, uint32_t m1) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image(smem, img);
    const Tables tb = tables(smem, img);
    const uint32_t l = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t p = blockIdx.x * kWavesPerBlock + wv;
    if (p >= count) return;
    const uint32_t* src = in + (size_t)p * kN;
    uint32_t x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = src[jA(l, r)];
    ntt_fwd(x, smem + kLdsTabWords + wv * kLdsWords, twf, tb.twf, tb.twfc, l, Q, m1);
    uint32_t* dst = out + (size_t)p * kN;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) dst[jC(l, r)] = canon4(x[r], Q);
}

__global__ __launch_bounds__(kThreads) void ntt_inv_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                            uint32_t count, const uint32_t* img, const uint2* twi,
                                                            uint32_t Q, uint32_t ninv, uint32_t ninvp) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image(smem, img);
    const Tables tb = tables(smem, img);
    const uint32_t l = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t p = blockIdx.x * kWavesPerBlock + wv;
    if (p >= count) return;
    const uint32_t* src = in + (size_t)p * kN;
    uint32_t x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = src[jC(l, r)];
    ntt_inv(x, smem + kLdsTabWords + wv * kLdsWords, twi, tb.twi, l, Q);
    uint32_t* dst = out + (size_t)p * kN;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) dst[jA(l, r)] = mul_shoup(x[r], ninv, ninvp, Q);
}

// SignedDigitDecompose through the same offset-word digits the step kernel
// feeds its NTTs, reduced to the reference's canonical residues.
__global__ void sdd_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t count, uint32_t dg,
                           uint32_t Q, SddConsts sd) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)count * kN) return;
    const size_t p = idx / kN, j = idx % kN;
    const uint32_t D = sdd_offset(in[idx], sd);
    for (uint32_t i = 0; i < dg; ++i) {
        const uint32_t v = sdd_digit(D, i + 1, sd);
        out[(p * dg + i) * kN + j] = v >= Q ? v - Q : v;
    }
}

// ---- kernel table -------------------------------------------------------------

using StepFn = void (*)(StepArgs);

template <int DG>
StepFn pick_step(int method, bool first, bool dscr) {
    if (method == XZW) {
        if (first) return mk_step_kernel<DG, XZW, true>;
        return dscr ? mk_step_kernel<DG, XZW, false, true> : mk_step_kernel<DG, XZW, false>;
    }
    return first ? mk_step_kernel<DG, XZW_B, true> : mk_step_kernel<DG, XZW_B, false>;
}

StepFn step_fn(int dg, int method, bool first, bool dscr);

template <int DG>
StepFn pick_lat(int method, bool first) {
    if (method == XZW) return first ? mk_lat_kernel<DG, XZW, true> : mk_lat_kernel<DG, XZW, false>;
    return first ? mk_lat_kernel<DG, XZW_B, true> : mk_lat_kernel<DG, XZW_B, false>;
}
StepFn lat_fn(int dg, int method, bool first);

}  // namespace

#include "mkacc_gate.hpp"
#include "mkacc_wide.hpp"
#include "mkacc_widefp.hpp"

namespace {

// Device key upload for the 64-bit word path: reference layout -> [k][n+1][nk][dg][2][N]
// (EVAL order), each word in Montgomery form K * 2^64 mod Q (r, rp: 2^64 mod Q and its
// Shoup companion), or for the FP64 variant (fp) the bits of the balanced double.
template <typename W>
__global__ void wide_key_layout_kernel(const W* __restrict__ src, uint64_t* __restrict__ dst, size_t npolys,
                                       uint32_t nk, uint32_t n1, uint32_t dg2, uint64_t Q, uint64_t r, uint64_t rp,
                                       bool fp, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= npolys * kN) return;
    size_t p = idx / kN;
    const uint32_t j = (uint32_t)(idx % kN);
    const uint32_t dp = (uint32_t)(p % dg2); p /= dg2;
    const uint32_t i = (uint32_t)(p % n1); p /= n1;
    const uint32_t jj = (uint32_t)(p % nk);
    const size_t u = p / nk;
    const size_t dpoly = ((u * n1 + i) * nk + jj) * dg2 + dp;
    const uint64_t x = (uint64_t)src[idx];
    if (x >= Q) *bad = 1u;
    if (fp) {
        const double d = (double)(x < Q ? x : 0) - (x > (Q >> 1) && x < Q ? (double)Q : 0.0);
        dst[dpoly * kN + j] = (uint64_t)__double_as_longlong(d);
    } else {
        dst[dpoly * kN + j] = wide::mul_shoup(x, r, rp, Q);
    }
}

// Every digit count is instantiated.  (Round 2's MKACC_ONLY_DG=3 A/B builds
// returned null here for other digit counts and the launch of a null kernel
// produced the segfault / all-wrong records of ab_l1, lat_l1 and ab_d1,
// DESIGN.md s2; a null kernel is now refused at mkacc_create and launch.)
StepFn step_fn(int dg, int method, bool first, bool dscr) {
    switch (dg) {
        case 2: return pick_step<2>(method, first, dscr);
        case 3: return pick_step<3>(method, first, dscr);
        case 4: return pick_step<4>(method, first, dscr);
        case 5: return pick_step<5>(method, first, dscr);
        default: return nullptr;
    }
}
StepFn lat_fn(int dg, int method, bool first) {
    switch (dg) {
        case 2: return pick_lat<2>(method, first);
        case 3: return pick_lat<3>(method, first);
        case 4: return pick_lat<4>(method, first);
        default: return nullptr;
    }
}

// Key-switching keys from device memory (mkacc_upload_ksk_*_device): the host
// conversions of mkacc_upload_ksk_mntru / _mklwe on the GPU.  MNTRU: reference row
// l = j dks + t of [k][N dks][n] -> device row t N + j of [k][dks N][n_pad], u16;
// MK-LWE: u32 -> u16 in place order.  A word >= qKS raises `bad`.
__global__ void ksk_mntru_layout_kernel(const uint32_t* __restrict__ src, uint16_t* __restrict__ dst, uint32_t k,
                                        uint32_t dks, uint32_t n, uint32_t npad, uint32_t qKS,
                                        uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t L = (size_t)dks * kN;
    if (idx >= (size_t)k * L * npad) return;
    const uint32_t i = (uint32_t)(idx % npad);
    const size_t row = (idx / npad) % L, u = idx / npad / L;
    const uint32_t t = (uint32_t)(row / kN), j = (uint32_t)(row % kN);
    uint32_t v = 0;
    if (i < n) {
        v = src[((u * kN + j) * dks + t) * n + i];
        if (v >= qKS) {
            *bad = 1u;
            v = 0;
        }
    }
    dst[idx] = (uint16_t)v;
}
__global__ void ksk_narrow_kernel(const uint32_t* __restrict__ src, uint16_t* __restrict__ dst, size_t count,
                                  uint32_t qKS, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    uint32_t v = src[idx];
    if (v >= qKS) {
        *bad = 1u;
        v = 0;
    }
    dst[idx] = (uint16_t)v;
}

__global__ void wide_copy_check_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, size_t count,
                                       uint64_t Q, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    uint64_t x = in[idx];
    if (x >= Q) {
        *bad = 1u;
        x = 0;
    }
    out[idx] = x;
}

}  // namespace

// ---- context --------------------------------------------------------------------

struct mkacc_ctx {
    mkacc_params p{};
    int device = 0;
    int cus = 256;                // compute units of the device (mk_lat_kernel residency)
    int method_class = XZW;   // XZW or XZW_B
    uint32_t dg = 0, nk = 0;
    Mod mod{};
    SddConsts sd{};
    uint32_t ninv = 0, ninvp = 0, nval = 0, nvalp = 0;
    uint32_t kscale = 0, kscalep = 0;   // key words: N^-1 2^32 mod Q and its companion
    hipStream_t stream = nullptr;
    uint2* d_twf = nullptr;
    uint2* d_twi = nullptr;
    uint32_t* d_img = nullptr;    // LDS image: per-lane twiddles + psi table
    uint32_t* d_keys = nullptr;   // [k][n+1][nk][dg][2][N] C4, scaled
    uint32_t* d_pkey = nullptr;   // [k][dg][N] C4, scaled
    bool have_keys = false;
    // batch workspace
    size_t ws_B = 0;
    uint32_t* d_acc0 = nullptr;
    uint32_t* d_acc1 = nullptr;
    uint32_t* d_cvals = nullptr;
    uint32_t* d_dscr = nullptr;   // [B][dg][N] d_i scratch (use_dscr), sized with the workspace
    // host-pointer API staging
    size_t io_B = 0;
    uint32_t* d_ct = nullptr;
    uint32_t* d_io = nullptr;
    // gate head / tail (mkacc_gate.hpp)
    mkacc_ks_params ks{};
    uint32_t dks = 0, n_pad = 0;
    bool have_ksk = false;
    uint16_t* d_ksk = nullptr;     // MNTRU: [k][dks*N][n_pad], row l = t*N + j
    uint16_t* d_lweA = nullptr;    // MK-LWE: [k][N][Bks][dks][n_out]
    uint16_t* d_lweB = nullptr;    // MK-LWE: [k][N][Bks][dks]
    uint32_t* d_tv = nullptr;      // test vector NTT(Rx) * N^-1, C4 [N]
    size_t gate_B = 0;
    uint8_t* d_digits = nullptr;   // [B][k][dks][N]
    uint32_t* d_bh = nullptr;      // [B] MK-LWE rotation b
    uint32_t* d_gin = nullptr;     // host API staging of gate inputs (grow-only)
    uint32_t* d_gout = nullptr;
    size_t gin_words = 0, gout_words = 0;
    // 64-bit word path (mkacc_wide.hpp), used when Q does not fit the 27-bit kernel
    bool wide = false;
    wide::Mod64 wm{};
    wide::Sdd64 wsd{};
    uint64_t wninv = 0, wninvp = 0;
    ulonglong2* d_wtwf = nullptr;  // forward table {w, w'} (reference order)
    ulonglong2* d_wtwi = nullptr;
    ulonglong2* d_wpsi = nullptr;  // psi^e, e < 2N
    uint64_t* d_wkeys = nullptr;   // [k][n+1][nk][dg][2][N] EVAL (FP64 variant: balanced doubles)
    uint64_t* d_wpkey = nullptr;   // [k][dg][N]
    // FP64 variant of the wide path (mkacc_widefp.hpp), Q < 2^50
    bool wfp = false;
    widefp::FMod wfm{};
    double wfninv = 0, wfC = 0;
    double* d_ftwf = nullptr;      // forward / inverse twiddles and psi^e, balanced
    double* d_ftwi = nullptr;
    double* d_fpsi = nullptr;
    size_t wws_B = 0, wio_B = 0;
    uint64_t* d_wacc0 = nullptr;
    uint64_t* d_wacc1 = nullptr;
    uint32_t* d_wcvals = nullptr;
    uint32_t* d_wct = nullptr;     // host-pointer API staging
    uint64_t* d_wio = nullptr;
    uint32_t* d_bad = nullptr;     // [0] input-range flag of the device batches (mkacc_sync), [1] device key upload
    std::mutex mu;
};

namespace {

size_t key_block_words(const mkacc_ctx* c) { return (size_t)c->nk * c->dg * 2 * kN; }

// device key block of step (u, i) (i == n: the KDM key evs)
const uint32_t* key_step(const mkacc_ctx* c, uint32_t u, uint32_t i, uint32_t j) {
    return c->d_keys + ((size_t)u * (c->p.n + 1) + i) * key_block_words(c) + (size_t)j * c->dg * 2 * kN;
}

// d_i scratch (mk_step_kernel DSCR): the XZW steps after the first compute the
// step's d_i once per gate instead of once per party pass.  It trades
// (k - 1) dg N Shoup products and psi gathers per gate-step for an HBM round
// trip of dg N words; default on from k >= kDscrMinK,
// MKACC_DSCR=0/1 overrides.
constexpr uint32_t kDscrMinK = 4;
bool use_dscr(const mkacc_ctx* c) {
    if (c->method_class != XZW || c->p.k < 2) return false;
    const char* e = std::getenv("MKACC_DSCR");
    if (e && *e) return e[0] != '0';
    return c->p.k >= kDscrMinK;
}

// Small batches take mk_lat_kernel (one wave per party) while the whole batch
// is resident in one round: its workgroups are LDS-bound (tables + k
// scratches: 2 per CU at k = 2..4, 1 at k = 8), and a second round costs more
// than the shorter critical path saves (B = 1024, k = 2: 160 ms against 109 ms
// for the batch kernel, profiles/r2/latency_v2_*.jsonl).  MKACC_LAT=0/1
// overrides.  Not built for dg = 5 or k > kLatMaxK.
constexpr size_t kLdsPerCu = 160 * 1024;
bool use_lat(const mkacc_ctx* c, size_t B) {
    if (c->p.k < 2 || c->p.k > kLatMaxK || c->dg > 4) return false;
    const char* e = std::getenv("MKACC_LAT");
    if (e && *e) return e[0] != '0';
    return B <= (size_t)c->cus * (kLdsPerCu / lat_lds_bytes(c->p.k));
}

int ensure_ws(mkacc_ctx* c, size_t B) {
    if (B <= c->ws_B) return MKACC_OK;
    if (c->d_acc0) HIP_TRY(hipFree(c->d_acc0));
    if (c->d_acc1) HIP_TRY(hipFree(c->d_acc1));
    if (c->d_cvals) HIP_TRY(hipFree(c->d_cvals));
    if (c->d_dscr) HIP_TRY(hipFree(c->d_dscr));
    c->d_acc0 = c->d_acc1 = c->d_cvals = c->d_dscr = nullptr;
    c->ws_B = 0;
    const size_t accw = B * c->p.k * (size_t)kN;
    HIP_TRY(hipMalloc(&c->d_acc0, accw * 4));
    HIP_TRY(hipMalloc(&c->d_acc1, accw * 4));
    HIP_TRY(hipMalloc(&c->d_cvals, B * c->p.k * (size_t)c->p.n * 4));
    if (use_dscr(c)) HIP_TRY(hipMalloc(&c->d_dscr, B * c->dg * (size_t)kN * 4));
    c->ws_B = B;
    return MKACC_OK;
}

// The k*n accumulator steps over a batch whose monomial exponents are in
// d_cvals and whose C4 accumulators are in d_acc0; returns the buffer holding
// the result (nullptr if the build has no kernel for the context's digit count).
uint32_t* launch_steps(mkacc_ctx* c, size_t B) {
    const uint32_t k = c->p.k, n = c->p.n;
    uint32_t* cur = c->d_acc0;
    uint32_t* nxt = c->d_acc1;
    const dim3 grid((unsigned)((B + kWavesPerBlock - 1) / kWavesPerBlock)), block(kThreads);
    // MKACC_DBG_LDS=<bytes> (diagnosis, tools/dbg/determ2.py): extra dynamic LDS per
    // workgroup; 10240 leaves one workgroup per CU, the co-residency reference
    const char* dl = std::getenv("MKACC_DBG_LDS");
    const size_t lds = kStepLdsBytes + (dl ? std::strtoul(dl, nullptr, 0) : 0);
    const bool lat = use_lat(c, B);
    for (uint32_t u = 0; u < k; ++u) {
        for (uint32_t i = 0; i < n; ++i) {
            const bool first = (u == 0 && i == 0);
            StepArgs a;
            a.acc_in = cur;
            a.acc_out = nxt;
            a.cvals = c->d_cvals + ((size_t)u * n + i) * B;
            a.key1 = key_step(c, u, i, 0);
            a.key2 = c->nk == 2 ? key_step(c, u, i, 1) : a.key1;
            a.keys = key_step(c, 0, n, 0);
            a.pkey = c->d_pkey;
            a.tw_fwd = c->d_twf;
            a.tw_inv = c->d_twi;
            a.img = c->d_img;
            a.B = (uint32_t)B;
            a.k = k;
            a.index = u;
            a.m = c->mod;
            a.sd = c->sd;
            a.dscr = c->d_dscr;
            // a null kernel must never reach hipLaunchKernelGGL (mkacc_create checks the set)
            if (lat) {
                const StepFn fn = lat_fn((int)c->dg, c->method_class, first);
                if (!fn) return nullptr;
                hipLaunchKernelGGL(fn, dim3((unsigned)B), dim3(64 * k), lat_lds_bytes(k), c->stream, a);
            } else {
                const StepFn fn = step_fn((int)c->dg, c->method_class, first, !first && c->d_dscr != nullptr);
                if (!fn) return nullptr;
                hipLaunchKernelGGL(fn, grid, block, lds, c->stream, a);
            }
            std::swap(cur, nxt);
        }
    }
    return cur;
}

void launch_prep_c(mkacc_ctx* c, const uint32_t* d_ct, size_t B) {
    const size_t tot = B * (size_t)c->p.k * c->p.n;
    hipLaunchKernelGGL(prep_c_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, d_ct,
                       c->d_cvals, (uint32_t)B, c->p.k * c->p.n, (uint32_t)c->method_class, (uint32_t)c->p.q,
                       c->d_bad);
}

int launch_batch(mkacc_ctx* c, const uint32_t* d_ct, const uint32_t* d_in, uint32_t* d_out, size_t B) {
    if (!c->have_keys) return fail(MKACC_E_NOKEYS, "Bootstrapping keys have not been generated/uploaded");
    if (B == 0) return MKACC_OK;
    int rc = ensure_ws(c, B);
    if (rc) return rc;
    const size_t npoly = B * c->p.k;
    const int tpb = 256;
    launch_prep_c(c, d_ct, B);
    {
        const size_t tw = npoly * kN;
        hipLaunchKernelGGL(eval_to_c4_kernel, dim3((unsigned)((tw + tpb - 1) / tpb)), dim3(tpb), 0, c->stream, d_in,
                           c->d_acc0, npoly, c->ninv, c->ninvp, c->mod.Q, c->d_bad);
    }
    uint32_t* cur = launch_steps(c, B);
    if (!cur) return fail(MKACC_E_UNSUPPORTED, "no step kernel for this digit count in this build");
    {
        const size_t tw = npoly * kN;
        hipLaunchKernelGGL(c4_to_eval_kernel, dim3((unsigned)((tw + tpb - 1) / tpb)), dim3(tpb), 0, c->stream, cur,
                           d_out, npoly, c->nval, c->nvalp, c->mod.Q);
    }
    HIP_TRY(hipGetLastError());
    return MKACC_OK;
}

// ---- gate level (head + EvalAcc + tail) -------------------------------------------

int ensure_gate_ws(mkacc_ctx* c, size_t B) {
    int rc = ensure_ws(c, B);
    if (rc) return rc;
    if (B <= c->gate_B) return MKACC_OK;
    if (c->d_digits) HIP_TRY(hipFree(c->d_digits));
    if (c->d_bh) HIP_TRY(hipFree(c->d_bh));
    c->d_digits = nullptr;
    c->d_bh = nullptr;
    c->gate_B = 0;
    HIP_TRY(hipMalloc(&c->d_digits, B * c->p.k * (size_t)c->dks * kN));
    HIP_TRY(hipMalloc(&c->d_bh, B * c->p.k * 4));   // MK-LWE head rotation b [B], then partial b sums [B][k]
    c->gate_B = B;
    return MKACC_OK;
}

// Test vector of BootstrapGateCore (binfhe-base-scheme.cpp:1093-1115 MNTRU,
// :1017-1021 MK-LWE; plaintext modulus p = 4, mntru-ciphertext.h:30), NTT'd on
// the device and stored C4 * N^-1.
int ensure_test_vector(mkacc_ctx* c) {
    if (c->d_tv) return MKACC_OK;
    const uint64_t Q = c->p.Q, p = 4, Q2p = Q / (2 * p) + 1, Q2pNeg = Q - Q2p;
    std::vector<uint32_t> rx(kN);
    for (uint32_t j = 0; j < (uint32_t)kN; ++j) {
        const bool lo = j < (uint32_t)kN / 2;
        rx[j] = (uint32_t)(c->method_class == XZW ? (lo ? Q2pNeg : Q2p) : (lo ? Q2p : Q2pNeg));
    }
    uint32_t *din = nullptr, *dev = nullptr;
    HIP_TRY(hipMalloc(&din, kN * 4));
    HIP_TRY(hipMalloc(&dev, kN * 4));
    HIP_TRY(hipMalloc(&c->d_tv, kN * 4));
    HIP_TRY(hipMemcpyAsync(din, rx.data(), kN * 4, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(ntt_fwd_kernel, dim3(1), dim3(kThreads), kStepLdsBytes, c->stream, din, dev, 1u, c->d_img,
                       c->d_twf, c->mod.Q, c->mod.m1);
    hipLaunchKernelGGL(eval_to_c4_kernel, dim3(kN / 256), dim3(256), 0, c->stream, dev, c->d_tv, (size_t)1, c->ninv,
                       c->ninvp, c->mod.Q, (uint32_t*)nullptr);
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(din));
    HIP_TRY(hipFree(dev));
    return MKACC_OK;
}

TailConsts tail_consts(const mkacc_ctx* c) {
    return TailConsts{c->mod.Q, (uint32_t)c->ks.qKS, c->ks.baseKS, c->dks};
}

const uint2* psi_image(const mkacc_ctx* c) { return reinterpret_cast<const uint2*>(c->d_img) + kPsiOff; }

// tail on the C4 accumulators `acc`: extraction + ModSwitch + digits, then the
// method's key switch into out_a (and out_b for MK-LWE)
void launch_tail(mkacc_ctx* c, const uint32_t* acc, uint32_t* out_a, uint32_t* out_b, size_t B) {
    const uint32_t k = c->p.k;
    const uint32_t npoly = (uint32_t)(B * k);
    const uint2* twl_inv = reinterpret_cast<const uint2*>(c->d_img) + kTwlPairs;
    hipLaunchKernelGGL(extract_kernel, dim3((npoly + 3) / 4), dim3(256), 0, c->stream, acc, c->d_digits, npoly,
                       c->d_twi, twl_inv, tail_consts(c));
    const uint32_t L = c->dks * kN;
    if (c->method_class == XZW) {
        const uint32_t qinv = (uint32_t)((1ull << 32) / c->ks.qKS);
        const dim3 grid(c->n_pad / kKsTile, (unsigned)((B + kKsTile - 1) / kKsTile), k);
        hipLaunchKernelGGL(ks_mntru_kernel, grid, dim3(256), 0, c->stream, c->d_digits, c->d_ksk, out_a,
                           (uint32_t)B, k, L, c->ks.n_out, c->n_pad, (uint32_t)c->ks.qKS, qinv);
    } else {
        const uint32_t b0 = round_qQ_host((c->p.Q >> 3) + 1, c->ks.qKS, c->p.Q);
        hipLaunchKernelGGL(ks_mklwe_kernel, dim3((unsigned)(B * k)), dim3(256), 0, c->stream, c->d_digits,
                           c->d_lweA, c->d_lweB, out_a, c->d_bh, k, c->ks.n_out, c->ks.baseKS, c->dks,
                           (uint32_t)c->ks.qKS);
        hipLaunchKernelGGL(ks_mklwe_b_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, c->stream, c->d_bh,
                           out_b, (uint32_t)B, k, (uint32_t)c->ks.qKS, b0);
    }
}

// full NAND gates on device buffers
int launch_gates(mkacc_ctx* c, const uint32_t* d_nand, const uint32_t* d_a1, const uint32_t* d_b1,
                 const uint32_t* d_a2, const uint32_t* d_b2, uint32_t* d_out_a, uint32_t* d_out_b, size_t B) {
    if (!c->have_keys) return fail(MKACC_E_NOKEYS, "Bootstrapping keys have not been generated. Please call MKBTKeyGen before calling bootstrapping.");
    if (!c->have_ksk) return fail(MKACC_E_NOKEYS, "Key-switching keys have not been uploaded");
    if (B == 0) return MKACC_OK;
    int rc = ensure_gate_ws(c, B);
    if (!rc) rc = ensure_test_vector(c);
    if (rc) return rc;
    const uint32_t k = c->p.k, kn = k * c->p.n;
    const size_t tot = B * (size_t)kn;
    // head: the raw accumulator exponents go through d_ct
    if (B > c->io_B) {
        if (c->d_ct) HIP_TRY(hipFree(c->d_ct));
        if (c->d_io) HIP_TRY(hipFree(c->d_io));
        c->d_ct = c->d_io = nullptr;
        c->io_B = 0;
        HIP_TRY(hipMalloc(&c->d_ct, tot * 4));
        HIP_TRY(hipMalloc(&c->d_io, B * k * (size_t)kN * 4));
        c->io_B = B;
    }
    const unsigned g1 = (unsigned)((tot + 255) / 256);
    if (c->method_class == XZW)
        hipLaunchKernelGGL(mntru_head_kernel, dim3(g1), dim3(256), 0, c->stream, d_nand, d_a1, d_a2, c->d_ct,
                           (uint32_t)B, kn, (uint32_t)c->p.q, c->d_bad);
    else
        hipLaunchKernelGGL(mklwe_head_kernel, dim3(g1), dim3(256), 0, c->stream, d_a1, d_b1, d_a2, d_b2, c->d_ct,
                           c->d_bh, (uint32_t)B, kn, (uint32_t)c->p.q, c->d_bad);
    launch_prep_c(c, c->d_ct, B);
    const size_t tw = B * k * (size_t)kN;
    hipLaunchKernelGGL(acc_init_kernel, dim3((unsigned)((tw + 255) / 256)), dim3(256), 0, c->stream, c->d_acc0,
                       c->d_tv, c->method_class == XZW ? nullptr : c->d_bh, psi_image(c), (uint32_t)B, k, c->mod.Q);
    uint32_t* cur = launch_steps(c, B);
    if (!cur) return fail(MKACC_E_UNSUPPORTED, "no step kernel for this digit count in this build");
    launch_tail(c, cur, d_out_a, d_out_b, B);
    HIP_TRY(hipGetLastError());
    return MKACC_OK;
}

template <typename W>
int upload_keys_impl(mkacc_ctx* c, const W* evk, const W* pkey) {
    if (!evk || !pkey) return fail(MKACC_E_ARG, "null key pointer");
    const uint64_t Q = c->p.Q;
    const uint32_t k = c->p.k, n = c->p.n, nk = c->nk, dg = c->dg;
    const size_t npolys = (size_t)k * nk * (n + 1) * dg * 2;
    std::vector<uint32_t> host((size_t)k * (n + 1) * key_block_words(c));
    // reference [k][nk][n+1][dg][2][N]  ->  device [k][n+1][nk][dg][2][N] (C4, * N^-1 2^32;
    // MKNTRU: ev1 + ev2 in the ev1 blocks of the steps i < n, StepArgs)
    bool bad = false;
    const uint64_t ks = c->kscale;
    const size_t ev2_stride = (size_t)(n + 1) * dg * 2 * kN;
    auto worker = [&](size_t p0, size_t p1) {
        for (size_t p = p0; p < p1; ++p) {
            size_t t = p;
            const size_t dp = t % (dg * 2); t /= (dg * 2);
            const size_t i = t % (n + 1); t /= (n + 1);
            const size_t j = t % nk; t /= nk;
            const size_t u = t;
            const W* src = evk + p * kN;
            uint32_t* dst = host.data() + (((u * (n + 1) + i) * nk + j) * dg * 2 + dp) * kN;
            const bool comb = nk == 2 && j == 0 && i < n;
            for (uint32_t s = 0; s < (uint32_t)kN; ++s) {
                uint64_t x = (uint64_t)src[s];
                if (x >= Q) bad = true;
                if (comb) {
                    const uint64_t y = (uint64_t)src[ev2_stride + s];
                    if (y >= Q) bad = true;
                    x = (x + y) % Q;
                }
                dst[c4_index(s)] = (uint32_t)((x % Q) * ks % Q);
            }
        }
    };
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back(worker, npolys * t / nt, npolys * (t + 1) / nt);
    for (auto& x : th) x.join();
    if (bad) return fail(MKACC_E_RANGE, "evk word not a canonical residue mod Q");
    std::vector<uint32_t> hp((size_t)k * dg * kN);
    for (size_t p = 0; p < (size_t)k * dg; ++p)
        for (uint32_t s = 0; s < (uint32_t)kN; ++s) {
            const uint64_t x = (uint64_t)pkey[p * kN + s];
            if (x >= Q) return fail(MKACC_E_RANGE, "pkey word not a canonical residue mod Q");
            hp[p * kN + c4_index(s)] = (uint32_t)((x * ks) % Q);
        }
    HIP_TRY(hipSetDevice(c->device));
    if (!c->d_keys) HIP_TRY(hipMalloc(&c->d_keys, host.size() * 4));
    if (!c->d_pkey) HIP_TRY(hipMalloc(&c->d_pkey, hp.size() * 4));
    HIP_TRY(hipMemcpy(c->d_keys, host.data(), host.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_pkey, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    c->have_keys = true;
    return MKACC_OK;
}

// keys already in device memory (e.g. the RCCL-broadcast buffer of bench.py):
// one layout kernel per array on the context stream, no host round trip
template <typename W>
int upload_keys_device_impl(mkacc_ctx* c, const W* d_evk, const W* d_pkey) {
    const uint32_t k = c->p.k, n1 = c->p.n + 1, nk = c->nk, dg = c->dg;
    const size_t ep = (size_t)k * nk * n1 * dg * 2, pp = (size_t)k * dg;
    const unsigned tpb = 256;
    auto grid = [&](size_t np) { return dim3((unsigned)((np * kN + tpb - 1) / tpb)); };
    HIP_TRY(hipSetDevice(c->device));
    // the key check has its own flag word (d_bad[1]): a pending input-range error
    // of an earlier device batch (d_bad[0]) stays for mkacc_sync to report
    uint32_t* kbad = c->d_bad + 1;
    HIP_TRY(hipMemsetAsync(kbad, 0, 4, c->stream));
    c->have_keys = false;
    if (c->wide) {
        const uint64_t Q = c->p.Q, R = (uint64_t)(((unsigned __int128)1 << 64) % Q);
        const uint64_t Rp = (uint64_t)(((unsigned __int128)R << 64) / Q);
        if (!c->d_wkeys) HIP_TRY(hipMalloc(&c->d_wkeys, ep * kN * 8));
        if (!c->d_wpkey) HIP_TRY(hipMalloc(&c->d_wpkey, pp * kN * 8));
        hipLaunchKernelGGL(wide_key_layout_kernel<W>, grid(ep), dim3(tpb), 0, c->stream, d_evk, c->d_wkeys, ep, nk,
                           n1, dg * 2, Q, R, Rp, c->wfp, kbad);
        hipLaunchKernelGGL(wide_key_layout_kernel<W>, grid(pp), dim3(tpb), 0, c->stream, d_pkey, c->d_wpkey, pp, 1u,
                           1u, dg, Q, R, Rp, c->wfp, kbad);
    } else {
        if (!c->d_keys) HIP_TRY(hipMalloc(&c->d_keys, ep * kN * 4));
        if (!c->d_pkey) HIP_TRY(hipMalloc(&c->d_pkey, pp * kN * 4));
        hipLaunchKernelGGL(key_layout_kernel<W>, grid(ep), dim3(tpb), 0, c->stream, d_evk, c->d_keys, ep, nk, n1,
                           dg * 2, c->mod.Q, c->kscale, c->kscalep, kbad);
        hipLaunchKernelGGL(key_layout_kernel<W>, grid(pp), dim3(tpb), 0, c->stream, d_pkey, c->d_pkey, pp, 1u, 1u,
                           dg, c->mod.Q, c->kscale, c->kscalep, kbad);
    }
    HIP_TRY(hipGetLastError());
    uint32_t bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, kbad, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (bad) return fail(MKACC_E_RANGE, "evk/pkey word not a canonical residue mod Q");
    c->have_keys = true;
    return MKACC_OK;
}

int prim_launch(mkacc_ctx* c, const uint32_t* in, uint32_t* out, size_t count, size_t out_mul, int which) {
    if (!c || !in || !out) return fail(MKACC_E_ARG, "null argument");
    if (count == 0) return MKACC_OK;
    HIP_TRY(hipSetDevice(c->device));
    for (size_t s = 0; s < count * kN; ++s)
        if (in[s] >= c->p.Q) return fail(MKACC_E_RANGE, "input word not a canonical residue mod Q");
    uint32_t *din = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc(&din, count * kN * 4));
    HIP_TRY(hipMalloc(&dout, count * kN * 4 * out_mul));
    HIP_TRY(hipMemcpyAsync(din, in, count * kN * 4, hipMemcpyHostToDevice, c->stream));
    const size_t lds = kStepLdsBytes;
    const dim3 grid((unsigned)((count + kWavesPerBlock - 1) / kWavesPerBlock)), block(kThreads);
    if (which == 0)
        hipLaunchKernelGGL(ntt_fwd_kernel, grid, block, lds, c->stream, din, dout, (uint32_t)count, c->d_img, c->d_twf,
                           c->mod.Q, c->mod.m1);
    else if (which == 1)
        hipLaunchKernelGGL(ntt_inv_kernel, grid, block, lds, c->stream, din, dout, (uint32_t)count, c->d_img, c->d_twi,
                           c->mod.Q, c->ninv, c->ninvp);
    else {
        const size_t tot = count * kN;
        hipLaunchKernelGGL(sdd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, din, dout,
                           (uint32_t)count, c->dg, c->mod.Q, c->sd);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, dout, count * kN * 4 * out_mul, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(din));
    HIP_TRY(hipFree(dout));
    return MKACC_OK;
}

// ---- 64-bit word path (mkacc_wide.hpp) --------------------------------------------

int wide_setup(mkacc_ctx* c) {
    using u128 = unsigned __int128;
    const uint64_t Q = c->p.Q;
    const uint32_t L = 64u - (uint32_t)__builtin_clzll(Q);
    uint64_t qi = Q;                       // Q^-1 mod 2^64 by Newton (Q odd)
    for (int it = 0; it < 6; ++it) qi *= 2 - Q * qi;
    c->wm = wide::Mod64{Q, (uint64_t)(((u128)1 << (2 * L)) / Q), L, 0 - qi};
    const uint32_t b = (uint32_t)__builtin_ctz(c->p.baseG);
    uint64_t C = 0;
    for (uint32_t i = 0; i < c->p.digitsG; ++i) C += (1ull << (b - 1)) << (b * i);
    c->wsd = wide::Sdd64{Q >> 1, C, C - Q, 1ull << (b - 1), b};
    auto comp = [Q](uint64_t w) { return (uint64_t)(((u128)w << 64) / Q); };
    c->wninv = modinv(kN, Q);
    c->wninvp = comp(c->wninv);
    std::vector<ulonglong2> tf(kN), ti(kN), pw(2 * kN);
    const uint64_t psi = c->p.root, psii = modinv(psi, Q);
    uint64_t x = 1, xi = 1;
    for (uint32_t i = 0; i < (uint32_t)kN; ++i) {
        const uint32_t r = bit_reverse(i, kLogN);
        tf[r] = make_ulonglong2(x, comp(x));
        ti[r] = make_ulonglong2(xi, comp(xi));
        x = mulmod(x, psi, Q);
        xi = mulmod(xi, psii, Q);
    }
    uint64_t e = 1;
    for (uint32_t i = 0; i < 2u * kN; ++i) {
        pw[i] = make_ulonglong2(e, comp(e));
        e = mulmod(e, psi, Q);
    }
    HIP_TRY(hipMalloc(&c->d_wtwf, kN * sizeof(ulonglong2)));
    HIP_TRY(hipMalloc(&c->d_wtwi, kN * sizeof(ulonglong2)));
    HIP_TRY(hipMalloc(&c->d_wpsi, 2 * kN * sizeof(ulonglong2)));
    HIP_TRY(hipMemcpy(c->d_wtwf, tf.data(), kN * sizeof(ulonglong2), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_wtwi, ti.data(), kN * sizeof(ulonglong2), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_wpsi, pw.data(), 2 * kN * sizeof(ulonglong2), hipMemcpyHostToDevice));
    // FP64 variant (mkacc_widefp.hpp): exact while every value stays below 8 Q <= 2^53
    // and the SDD offset word below 2^53; MKACC_WIDE_FP=0 keeps the integer kernels
    const char* fe = std::getenv("MKACC_WIDE_FP");
    c->wfp = Q < (1ull << 50) && b * c->p.digitsG <= 52 && !(fe && fe[0] == '0');
    if (c->wfp) {
        const double Qd = (double)Q;
        c->wfm = widefp::FMod{Qd, 1.0 / Qd, (double)(Q >> 1)};
        auto bal = [Q](uint64_t x) { return x > (Q >> 1) ? (double)x - (double)Q : (double)x; };
        c->wfninv = bal(c->wninv);
        c->wfC = (double)C;
        std::vector<double> ftf(kN), fti(kN), fpw(2 * kN);
        for (uint32_t i = 0; i < (uint32_t)kN; ++i) {
            ftf[i] = bal(tf[i].x);
            fti[i] = bal(ti[i].x);
        }
        for (uint32_t i = 0; i < 2u * kN; ++i) fpw[i] = bal(pw[i].x);
        HIP_TRY(hipMalloc(&c->d_ftwf, kN * sizeof(double)));
        HIP_TRY(hipMalloc(&c->d_ftwi, kN * sizeof(double)));
        HIP_TRY(hipMalloc(&c->d_fpsi, 2 * kN * sizeof(double)));
        HIP_TRY(hipMemcpy(c->d_ftwf, ftf.data(), kN * sizeof(double), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_ftwi, fti.data(), kN * sizeof(double), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_fpsi, fpw.data(), 2 * kN * sizeof(double), hipMemcpyHostToDevice));
    }
    return MKACC_OK;
}

// reference [k][nk][n+1][dg][2][N] -> device [k][n+1][nk][dg][2][N] (same EVAL
// order), every word in Montgomery form K * 2^64 mod Q (wide::montmul)
template <typename W>
int wide_upload_keys(mkacc_ctx* c, const W* evk, const W* pkey) {
    if (!evk || !pkey) return fail(MKACC_E_ARG, "null key pointer");
    const uint64_t Q = c->p.Q;
    const uint64_t R = (uint64_t)(((unsigned __int128)1 << 64) % Q);
    const bool fp = c->wfp;   // FP64 variant: the bits of the balanced double
    auto mont = [Q, R, fp](uint64_t x) {
        if (fp) {
            const double d = x > (Q >> 1) ? (double)x - (double)Q : (double)x;
            uint64_t bits;
            std::memcpy(&bits, &d, 8);
            return bits;
        }
        return (uint64_t)((unsigned __int128)x * R % Q);
    };
    const uint32_t k = c->p.k, n = c->p.n, nk = c->nk, dg = c->dg;
    const size_t blk = (size_t)dg * 2 * kN;
    std::vector<uint64_t> host((size_t)k * (n + 1) * nk * blk);
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < nk; ++j)
            for (uint32_t i = 0; i <= n; ++i) {
                const W* src = evk + (((size_t)u * nk + j) * (n + 1) + i) * blk;
                uint64_t* dst = host.data() + (((size_t)u * (n + 1) + i) * nk + j) * blk;
                for (size_t s = 0; s < blk; ++s) {
                    if ((uint64_t)src[s] >= Q) return fail(MKACC_E_RANGE, "evk word not a canonical residue mod Q");
                    dst[s] = mont((uint64_t)src[s]);
                }
            }
    const size_t pw = (size_t)k * dg * kN;
    std::vector<uint64_t> hp(pw);
    for (size_t s = 0; s < pw; ++s) {
        if ((uint64_t)pkey[s] >= Q) return fail(MKACC_E_RANGE, "pkey word not a canonical residue mod Q");
        hp[s] = mont((uint64_t)pkey[s]);
    }
    HIP_TRY(hipSetDevice(c->device));
    if (!c->d_wkeys) HIP_TRY(hipMalloc(&c->d_wkeys, host.size() * 8));
    if (!c->d_wpkey) HIP_TRY(hipMalloc(&c->d_wpkey, pw * 8));
    HIP_TRY(hipMemcpy(c->d_wkeys, host.data(), host.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_wpkey, hp.data(), pw * 8, hipMemcpyHostToDevice));
    c->have_keys = true;
    return MKACC_OK;
}

int wide_ensure_ws(mkacc_ctx* c, size_t B) {
    if (B <= c->wws_B) return MKACC_OK;
    for (void* p : {(void*)c->d_wacc0, (void*)c->d_wacc1, (void*)c->d_wcvals})
        if (p) HIP_TRY(hipFree(p));
    c->d_wacc0 = c->d_wacc1 = nullptr;
    c->d_wcvals = nullptr;
    c->wws_B = 0;
    const size_t accw = B * c->p.k * (size_t)kN;
    HIP_TRY(hipMalloc(&c->d_wacc0, accw * 8));
    HIP_TRY(hipMalloc(&c->d_wacc1, accw * 8));
    HIP_TRY(hipMalloc(&c->d_wcvals, B * c->p.k * (size_t)c->p.n * 4));
    c->wws_B = B;
    return MKACC_OK;
}

// k*n wide steps over a batch on device buffers (d_in may alias d_out)
int wide_launch_batch(mkacc_ctx* c, const uint32_t* d_ct, const uint64_t* d_in, uint64_t* d_out, size_t B) {
    if (!c->have_keys) return fail(MKACC_E_NOKEYS, "Bootstrapping keys have not been generated/uploaded");
    if (B == 0) return MKACC_OK;
    int rc = wide_ensure_ws(c, B);
    if (rc) return rc;
    const uint32_t k = c->p.k, n = c->p.n;
    const size_t tot = B * (size_t)k * n, accb = B * (size_t)k * kN * 8;
    hipLaunchKernelGGL(prep_c_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, d_ct, c->d_wcvals,
                       (uint32_t)B, k * n, (uint32_t)c->method_class, (uint32_t)c->p.q, c->d_bad);
    const size_t blk = (size_t)c->dg * 2 * kN;
    auto key = [&](uint32_t u, uint32_t i, uint32_t j) {
        return c->d_wkeys + (((size_t)u * (n + 1) + i) * c->nk + j) * blk;
    };
    if (c->wfp) {   // FP64 variant: balanced doubles between the prologue and the epilogue
        const size_t words = B * (size_t)k * kN;
        const dim3 g((unsigned)((words + 255) / 256));
        double* cur = reinterpret_cast<double*>(c->d_wacc0);
        double* nxt = reinterpret_cast<double*>(c->d_wacc1);
        hipLaunchKernelGGL(widefp::to_balanced_kernel, g, dim3(256), 0, c->stream, d_in, cur, words, c->wfm,
                           c->p.Q, c->d_bad);
        auto dk = [](const uint64_t* p) { return reinterpret_cast<const double*>(p); };
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t i = 0; i < n; ++i) {
                const bool first = (u == 0 && i == 0);
                widefp::StepArgs a;
                a.acc_in = cur;
                a.acc_out = nxt;
                a.cvals = c->d_wcvals + ((size_t)u * n + i) * B;
                a.key1 = dk(key(u, i, 0));
                a.key2 = dk(c->nk == 2 ? key(u, i, 1) : key(u, i, 0));
                a.keys = dk(key(0, n, 0));
                a.pkey = dk(c->d_wpkey);
                a.twf = c->d_ftwf;
                a.twi = c->d_ftwi;
                a.psi = c->d_fpsi;
                a.k = k;
                a.index = u;
                a.dg = c->dg;
                a.ninv = c->wfninv;
                a.C = c->wfC;
                a.m = c->wfm;
                a.sd = c->wsd;
                void (*fn)(widefp::StepArgs);
                if (c->method_class == XZW) fn = first ? widefp::step_kernel<XZW, true> : widefp::step_kernel<XZW, false>;
                else fn = first ? widefp::step_kernel<XZW_B, true> : widefp::step_kernel<XZW_B, false>;
                hipLaunchKernelGGL(fn, dim3((unsigned)B), dim3(widefp::kThreads), 0, c->stream, a);
                std::swap(cur, nxt);
            }
        hipLaunchKernelGGL(widefp::to_canonical_kernel, g, dim3(256), 0, c->stream, cur, d_out, words, c->wfm);
        HIP_TRY(hipGetLastError());
        return MKACC_OK;
    }
    {   // copy into the working buffer with the range check of the device entry point
        const size_t words = accb / 8;
        hipLaunchKernelGGL(wide_copy_check_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, c->stream, d_in,
                           c->d_wacc0, words, c->p.Q, c->d_bad);
    }
    uint64_t* cur = c->d_wacc0;
    uint64_t* nxt = c->d_wacc1;
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t i = 0; i < n; ++i) {
            const bool first = (u == 0 && i == 0);
            wide::StepArgs a;
            a.acc_in = cur;
            a.acc_out = nxt;
            a.cvals = c->d_wcvals + ((size_t)u * n + i) * B;
            a.key1 = key(u, i, 0);
            a.key2 = c->nk == 2 ? key(u, i, 1) : a.key1;
            a.keys = key(0, n, 0);
            a.pkey = c->d_wpkey;
            a.twf = c->d_wtwf;
            a.twi = c->d_wtwi;
            a.psi = c->d_wpsi;
            a.k = k;
            a.index = u;
            a.dg = c->dg;
            a.ninv = c->wninv;
            a.ninvp = c->wninvp;
            a.m = c->wm;
            a.sd = c->wsd;
            void (*fn)(wide::StepArgs);
            if (c->method_class == XZW) fn = first ? wide::step_kernel<XZW, true> : wide::step_kernel<XZW, false>;
            else fn = first ? wide::step_kernel<XZW_B, true> : wide::step_kernel<XZW_B, false>;
            hipLaunchKernelGGL(fn, dim3((unsigned)B), dim3(wide::kThreads), 0, c->stream, a);
            std::swap(cur, nxt);
        }
    HIP_TRY(hipMemcpyAsync(d_out, cur, accb, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipGetLastError());
    return MKACC_OK;
}

// host-pointer batch through the wide path
int wide_eval_host(mkacc_ctx* c, const uint32_t* ct, const uint64_t* acc_in, uint64_t* acc_out, size_t B) {
    const size_t ctw = B * c->p.k * (size_t)c->p.n, accw = B * c->p.k * (size_t)kN;
    HIP_TRY(hipSetDevice(c->device));
    if (B > c->wio_B) {
        if (c->d_wct) HIP_TRY(hipFree(c->d_wct));
        if (c->d_wio) HIP_TRY(hipFree(c->d_wio));
        c->d_wct = nullptr;
        c->d_wio = nullptr;
        c->wio_B = 0;
        HIP_TRY(hipMalloc(&c->d_wct, ctw * 4));
        HIP_TRY(hipMalloc(&c->d_wio, accw * 8));
        c->wio_B = B;
    }
    HIP_TRY(hipMemcpyAsync(c->d_wct, ct, ctw * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_wio, acc_in, accw * 8, hipMemcpyHostToDevice, c->stream));
    int rc = wide_launch_batch(c, c->d_wct, c->d_wio, c->d_wio, B);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(acc_out, c->d_wio, accw * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MKACC_OK;
}

int wide_prim(mkacc_ctx* c, const uint64_t* in, uint64_t* out, size_t count, int which) {
    if (count == 0) return MKACC_OK;
    HIP_TRY(hipSetDevice(c->device));
    const uint64_t Q = c->p.Q;
    for (size_t s = 0; s < count * kN; ++s)
        if (in[s] >= Q) return fail(MKACC_E_RANGE, "input word not a canonical residue mod Q");
    const size_t out_mul = which == 2 ? c->dg : 1;
    uint64_t *din = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc(&din, count * kN * 8));
    HIP_TRY(hipMalloc(&dout, count * kN * 8 * out_mul));
    HIP_TRY(hipMemcpyAsync(din, in, count * kN * 8, hipMemcpyHostToDevice, c->stream));
    if (which == 0 && c->wfp)
        hipLaunchKernelGGL(widefp::ntt_fwd_kernel, dim3((unsigned)count), dim3(widefp::kThreads), 0, c->stream, din,
                           dout, c->d_ftwf, c->wfm);
    else if (which == 1 && c->wfp)
        hipLaunchKernelGGL(widefp::ntt_inv_kernel, dim3((unsigned)count), dim3(widefp::kThreads), 0, c->stream, din,
                           dout, c->d_ftwi, c->wfm, c->wfninv);
    else if (which == 0)
        hipLaunchKernelGGL(wide::ntt_fwd_kernel, dim3((unsigned)count), dim3(wide::kThreads), 0, c->stream, din, dout,
                           c->d_wtwf, Q);
    else if (which == 1)
        hipLaunchKernelGGL(wide::ntt_inv_kernel, dim3((unsigned)count), dim3(wide::kThreads), 0, c->stream, din, dout,
                           c->d_wtwi, Q, c->wninv, c->wninvp);
    else
        hipLaunchKernelGGL(wide::sdd_kernel, dim3((unsigned)((count * kN + 255) / 256)), dim3(256), 0, c->stream, din,
                           dout, (uint32_t)count, c->dg, c->wsd, Q);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, dout, count * kN * 8 * out_mul, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(din));
    HIP_TRY(hipFree(dout));
    return MKACC_OK;
}

int check_batch_inputs(const mkacc_ctx* c, const uint32_t* ct, size_t B) {
    const size_t ctw = B * c->p.k * (size_t)c->p.n;
    const uint64_t lim = c->method_class == XZW ? c->p.q : 2ull * kN + 1;  // XZW_B: c <= 2N (2N -> 0)
    for (size_t s = 0; s < ctw; ++s)
        if (ct[s] >= lim) return fail(MKACC_E_RANGE, "ciphertext word out of range");
    return MKACC_OK;
}

// The reference's MKNTRU_B gate is undefined: GenerateBinFHEContext builds an
// MNTRU context for it (binfhecontext.cpp:174), EvalBinGate hands the unscaled
// mod-q MNTRU words to BootstrapGateCore (binfhe-base-scheme.cpp:1127), and
// XZW_B uses them directly as monomial exponents (mk-acc-xzw_B.cpp:120,126,290),
// i.e. GetMonomial(c) with c up to q - 1 > 2N -- an out-of-range table read.
// The gate API rejects it (config_error); EvalAcc itself stays available for
// MKNTRU_B with exponents in [0, 2N].
int reject_mkntru_b(const mkacc_ctx* c) {
    if (c->p.method == MKACC_METHOD_MKNTRU_B)
        return fail(MKACC_E_ARG, "MKNTRU_B NAND gates are undefined in the reference (MNTRU words mod q used as "
                                 "XZW_B monomial exponents, binfhe-base-scheme.cpp:1127, mk-acc-xzw_B.cpp:120); "
                                 "use MKNTRU or MKNTRU_LWE");
    return MKACC_OK;
}

}  // namespace

// ---- C ABI ------------------------------------------------------------------------

extern "C" {

int mkacc_abi_version(void) { return MKACC_ABI_VERSION; }

// Build identity (mkfhe_amd/build.py passes the ids): SHA-256 prefixes of
// include/mkfhe_amd.h and of every engine source, and the extra -D switches of
// an A/B build.  mkfhe_amd._lib.load refuses a library whose abi or header id
// does not match the tree it runs in.
#ifndef MKACC_HEADER_ID
#define MKACC_HEADER_ID "unknown"
#endif
#ifndef MKACC_SOURCE_ID
#define MKACC_SOURCE_ID "unknown"
#endif
#ifndef MKACC_BUILD_FLAGS
#define MKACC_BUILD_FLAGS ""
#endif
const char* mkacc_build_info(void) {
    static const std::string info = [] {
        std::string dgs;
        for (int dg = 2; dg <= 5; ++dg)
            if (step_fn(dg, XZW, true, false) && step_fn(dg, XZW_B, false, false))
                dgs += (dgs.empty() ? "" : ",") + std::to_string(dg);
        return "abi=" + std::to_string(MKACC_ABI_VERSION) + ";header=" MKACC_HEADER_ID ";source=" MKACC_SOURCE_ID
               ";dg=" + dgs + ";flags=" MKACC_BUILD_FLAGS;
    }();
    return info.c_str();
}

const char* mkacc_last_error(void) { return g_last_error.c_str(); }

int mkacc_paramset(const char* name, uint32_t method, mkacc_params* out) {
    if (!name || !out) return fail(MKACC_E_ARG, "null argument");
    const ParamRow* row = find_paramset(name);
    if (!row) return fail(MKACC_E_ARG, std::string("unknown parameter set ") + name);
    if (method > MKACC_METHOD_MKNTRU_LWE) return fail(MKACC_E_ARG, "bad method");
    mkacc_params p{};
    p.method = method;
    p.k = row->numUser;
    p.n = row->latticeParam;
    p.N = row->cyclOrder / 2;
    p.Q = previous_prime(first_prime(row->numberBits, row->cyclOrder), row->cyclOrder);
    p.q = row->mod;
    p.baseG = row->gadgetBase;
    p.digitsG = digits_g(p.Q, p.baseG);
    p.root = root_of_unity(2ull * p.N, p.Q);
    *out = p;
    return MKACC_OK;
}

int mkacc_create(const mkacc_params* pin, int device, mkacc_ctx** out) {
    if (!pin || !out) return fail(MKACC_E_ARG, "null argument");
    *out = nullptr;
    mkacc_params p = *pin;
    if (p.method > MKACC_METHOD_MKNTRU_LWE) return fail(MKACC_E_ARG, "method is invalid");
    if (p.N != (uint32_t)kN) return fail(MKACC_E_UNSUPPORTED, "engine supports ring dimension N = 2048 only");
    // Q < 2^61: the 64-bit path's lazy butterflies keep words below 6Q < 2^64
    // (the reference's NATIVE_SIZE=64 limit MAX_MODULUS_SIZE is 60 bits)
    if (!(p.Q > (1ull << 26) && p.Q < (1ull << 61)))
        return fail(MKACC_E_UNSUPPORTED, "engine supports 2^26 < Q < 2^61");
    if ((p.Q - 1) % (2ull * p.N) != 0 || !is_prime(p.Q)) return fail(MKACC_E_ARG, "Q must be a prime = 1 mod 2N");
    if (p.k == 0 || p.k > 64 || p.n == 0) return fail(MKACC_E_ARG, "bad k or n");
    if (p.baseG < 2 || (p.baseG & (p.baseG - 1))) return fail(MKACC_E_ARG, "Gadget base should be a power of two.");
    if (p.method == MKACC_METHOD_MKNTRU && (p.q == 0 || p.q > (1u << 20)))
        return fail(MKACC_E_ARG, "bad ciphertext modulus q");
    if (p.digitsG == 0) p.digitsG = digits_g(p.Q, p.baseG);
    if (p.root == 0) p.root = root_of_unity(2ull * p.N, p.Q);
    if (p.digitsG < 2) return fail(MKACC_E_ARG, "digitsG must be at least 2");
    const uint32_t dg = p.digitsG - 1;
    const uint32_t gb = (uint32_t)__builtin_ctz(p.baseG);
    // the 27-bit register-resident kernel, or the 64-bit LDS-tile path (mkacc_wide.hpp)
    std::string why;
    if (!(p.Q < (1ull << 27))) why = "Q >= 2^27";
    else if (dg < 2 || dg > 5) why = "dg outside 2..5";
    else if (gb * p.digitsG > 32) why = "log2(baseG) * digitsG > 32";
    else if (gb * (dg - 1) > (dg <= 3 ? 16u : 20u) || (dg > 3 && 2u * gb + 20u > 32u))
        why = "digits 2..dg do not pack into 16 (dg <= 3) or 20 bits";
    const char* eng = std::getenv("MKACC_ENGINE");
    if (eng && !std::strcmp(eng, "wide")) why = "MKACC_ENGINE=wide";
    const bool wide = !why.empty();
    if (wide && (dg > 8 || gb * p.digitsG > 63))
        return fail(MKACC_E_UNSUPPORTED, "engine supports dg <= 8 and log2(baseG) * digitsG <= 63 (" + why + ")");
    if (!is_primitive_root(p.root, 2ull * p.N, p.Q)) return fail(MKACC_E_ARG, "root is not a primitive 2N-th root");

    auto c = std::make_unique<mkacc_ctx>();
    c->p = p;
    c->device = device;
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
            c->cus = ncu;
    }
    c->method_class = p.method == MKACC_METHOD_MKNTRU ? XZW : XZW_B;
    c->dg = dg;
    c->nk = c->method_class == XZW ? 2 : 1;
    c->wide = wide;
    if (!wide && !step_fn((int)dg, c->method_class, true, false))
        return fail(MKACC_E_UNSUPPORTED, "this build has no step kernel for dg = " + std::to_string(dg));
    if (wide) {
        HIP_TRY(hipSetDevice(device));
        HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        HIP_TRY(hipMalloc(&c->d_bad, 8));   // [0] batch inputs, [1] device key upload
        HIP_TRY(hipMemset(c->d_bad, 0, 8));
        const int rc = wide_setup(c.get());
        if (rc) {
            mkacc_destroy(c.release());
            return rc;
        }
        *out = c.release();
        return MKACC_OK;
    }
    c->mod.Q = (uint32_t)p.Q;
    c->mod.mu = (uint32_t)((1ull << 58) / p.Q);
    c->mod.r32 = (uint32_t)((1ull << 32) % p.Q);
    {
        uint32_t qi = (uint32_t)p.Q;          // Q^-1 mod 2^32 by Newton (Q odd)
        for (int it = 0; it < 5; ++it) qi *= 2u - (uint32_t)p.Q * qi;
        c->mod.qinv = 0u - qi;
        c->mod.m1 = (uint32_t)((1ull << 32) / p.Q);
    }
    {
        // offset-word digit decomposition constants (mkacc_device.hpp)
        const uint32_t b = (uint32_t)__builtin_ctz(p.baseG);
        uint64_t C = 0;
        for (uint32_t i = 0; i < p.digitsG; ++i) C += (1ull << (b - 1)) << (b * i);
        c->sd.qhalf = (uint32_t)(p.Q >> 1);
        c->sd.cpos = (uint32_t)C;
        c->sd.cneg = (uint32_t)(C - p.Q);
        c->sd.gbits = b;
        c->sd.qm = (uint32_t)(p.Q - (1ull << (b - 1)));
    }
    const uint64_t ninv = modinv(p.N, p.Q);
    c->ninv = (uint32_t)ninv;
    c->ninvp = (uint32_t)(((unsigned __int128)ninv << 32) / p.Q);
    c->kscale = (uint32_t)(ninv * c->mod.r32 % p.Q);
    c->kscalep = (uint32_t)(((unsigned __int128)c->kscale << 32) / p.Q);
    c->nval = p.N;
    c->nvalp = (uint32_t)(((unsigned __int128)p.N << 32) / p.Q);

    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_TRY(hipMalloc(&c->d_bad, 8));   // [0] batch inputs, [1] device key upload
    HIP_TRY(hipMemset(c->d_bad, 0, 8));
    // forward NTT table in the reference's order (transformnat-impl.h:705-760),
    // powers psi^e and psi^-e (e < 2N) for the inverse transform and the monomials
    const uint64_t Q = p.Q, psi = p.root, psii = modinv(psi, Q);
    std::vector<uint64_t> tf(kN), pw(2 * kN), pwi(2 * kN);
    {
        uint64_t x = 1;
        for (uint32_t i = 0; i < (uint32_t)kN; ++i) {
            tf[bit_reverse(i, kLogN)] = x;
            x = mulmod(x, psi, Q);
        }
        uint64_t e = 1, ei = 1;
        for (uint32_t i = 0; i < 2u * kN; ++i) {
            pw[i] = e;
            pwi[i] = ei;
            e = mulmod(e, psi, Q);
            ei = mulmod(ei, psii, Q);
        }
    }
    auto pair = [Q](uint64_t w) { return make_uint2((uint32_t)w, (uint32_t)(((unsigned __int128)w << 32) / Q)); };
    auto npair = [&](uint64_t w) { uint2 t = pair(w); t.x = 0u - t.x; return t; };   // ct_bfly_lazy's -w
    std::vector<uint2> htf(kN), hti(32, make_uint2(0, 0));
    for (int i = 0; i < kN; ++i) htf[i] = npair(tf[i]);
    // inverse pass 1 (ntt_inv): bit b < 5, t < 2^b -> psi^-(t 2^(11-b))
    for (int b = 0; b < 5; ++b)
        for (int t = 0; t < (1 << b); ++t) hti[(1 << b) + t] = npair(pwi[(size_t)t << (11 - b)]);
    HIP_TRY(hipMalloc(&c->d_twf, htf.size() * sizeof(uint2)));
    HIP_TRY(hipMalloc(&c->d_twi, hti.size() * sizeof(uint2)));
    // table image (kImgPairs, layout at StepArgs / ntt_inv)
    std::vector<uint2> img(kImgPairs);
    {
        uint2* F = img.data();
        for (int st = 5; st <= 9; ++st) {
            const int NP = 1 << (st - 5);
            for (int lhi = 0; lhi < 32; ++lhi)
                for (int m = 0; m < NP; ++m) F[twl_off(st) + 32 * m + lhi] = htf[(1 << st) + lhi * NP + m];
        }
        for (int ln = 0; ln < 64; ++ln)
            for (int m = 0; m < 16; ++m) F[kTwlC + 64 * m + ln] = htf[1024 + 16 * ln + m];
        uint2* I = img.data() + kTwlPairs;
        for (int b = 5; b <= 9; ++b)
            for (int m = 0; m < (1 << (b - 5)); ++m)
                for (int l31 = 0; l31 < 32; ++l31)
                    I[twl_off(b) + 32 * m + l31] = npair(pwi[(size_t)(l31 | (m << 5)) << (11 - b)]);
        for (int m = 0; m < 16; ++m)
            for (int ln = 0; ln < 64; ++ln) I[kTwlC + 64 * m + ln] = npair(pwi[(size_t)((m << 6) | ln) << 1]);
        for (int r = 0; r < 32; ++r)
            for (int ln = 0; ln < 64; ++ln) I[kTwlPairs + 64 * r + ln] = pair(pwi[(r << 6) | ln]);
        for (uint32_t e = 0; e < 2u * kN; ++e) {
            img[kPsiOff + psi_pos(e)] = pair(pw[e]);
            img[kPsm1Off + psi_pos(e)] = pair((pw[e] + Q - 1) % Q);
        }
    }
    HIP_TRY(hipMalloc(&c->d_img, img.size() * sizeof(uint2)));
    HIP_TRY(hipMemcpy(c->d_twf, htf.data(), htf.size() * sizeof(uint2), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_twi, hti.data(), hti.size() * sizeof(uint2), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_img, img.data(), img.size() * sizeof(uint2), hipMemcpyHostToDevice));
    *out = c.release();
    return MKACC_OK;
}

void mkacc_destroy(mkacc_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void* p : {(void*)c->d_twf, (void*)c->d_twi, (void*)c->d_img, (void*)c->d_keys, (void*)c->d_pkey,
                    (void*)c->d_acc0, (void*)c->d_acc1, (void*)c->d_cvals, (void*)c->d_dscr, (void*)c->d_ct,
                    (void*)c->d_io, (void*)c->d_ksk, (void*)c->d_lweA, (void*)c->d_lweB, (void*)c->d_tv,
                    (void*)c->d_digits, (void*)c->d_bh, (void*)c->d_gin, (void*)c->d_gout, (void*)c->d_wtwf,
                    (void*)c->d_wtwi, (void*)c->d_wpsi, (void*)c->d_ftwf, (void*)c->d_ftwi, (void*)c->d_fpsi,
                    (void*)c->d_wkeys, (void*)c->d_wpkey, (void*)c->d_wacc0,
                    (void*)c->d_wacc1, (void*)c->d_wcvals, (void*)c->d_wct, (void*)c->d_wio, (void*)c->d_bad})
        if (p) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int mkacc_get_params(const mkacc_ctx* c, mkacc_params* out) {
    if (!c || !out) return fail(MKACC_E_ARG, "null argument");
    *out = c->p;
    return MKACC_OK;
}

size_t mkacc_evk_words(const mkacc_ctx* c) {
    return c ? (size_t)c->p.k * c->nk * (c->p.n + 1) * c->dg * 2 * kN : 0;
}
size_t mkacc_pkey_words(const mkacc_ctx* c) { return c ? (size_t)c->p.k * c->dg * kN : 0; }

int mkacc_upload_keys(mkacc_ctx* c, const uint32_t* evk, const uint32_t* pkey) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return wide_upload_keys<uint32_t>(c, evk, pkey);
    return upload_keys_impl<uint32_t>(c, evk, pkey);
}
int mkacc_upload_keys_u64(mkacc_ctx* c, const uint64_t* evk, const uint64_t* pkey) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return wide_upload_keys<uint64_t>(c, evk, pkey);
    return upload_keys_impl<uint64_t>(c, evk, pkey);
}

int mkacc_upload_keys_device(mkacc_ctx* c, const void* d_evk, const void* d_pkey, uint32_t word_bytes) {
    if (!c || !d_evk || !d_pkey) return fail(MKACC_E_ARG, "null argument");
    if (word_bytes != 4 && word_bytes != 8) return fail(MKACC_E_ARG, "word_bytes must be 4 or 8");
    if (word_bytes == 4 && c->p.Q > 0xFFFFFFFFull) return fail(MKACC_E_ARG, "Q >= 2^32 needs 8-byte key words");
    std::lock_guard<std::mutex> g(c->mu);
    if (word_bytes == 4)
        return upload_keys_device_impl(c, (const uint32_t*)d_evk, (const uint32_t*)d_pkey);
    return upload_keys_device_impl(c, (const uint64_t*)d_evk, (const uint64_t*)d_pkey);
}

int mkacc_is_wide(const mkacc_ctx* c) { return c && c->wide ? (c->wfp ? 2 : 1) : 0; }

int mkacc_eval_batch_u64(mkacc_ctx* c, const uint32_t* ct, const uint64_t* acc_in, uint64_t* acc_out, size_t B) {
    if (!c || !ct || !acc_in || !acc_out) return fail(MKACC_E_ARG, "null argument");
    if (!c->have_keys) return fail(MKACC_E_NOKEYS, "Bootstrapping keys have not been generated. Please call MKBTKeyGen before calling bootstrapping.");
    if (B == 0) return MKACC_OK;
    const size_t accw = B * c->p.k * (size_t)kN;
    for (size_t s = 0; s < accw; ++s)
        if (acc_in[s] >= c->p.Q) return fail(MKACC_E_RANGE, "accumulator word not a canonical residue mod Q");
    if (!c->wide) {   // 27-bit kernel: narrow, run, widen
        std::vector<uint32_t> a32(acc_in, acc_in + accw);
        const int rc = mkacc_eval_batch(c, ct, a32.data(), a32.data(), B);
        if (rc) return rc;
        for (size_t s = 0; s < accw; ++s) acc_out[s] = a32[s];
        return MKACC_OK;
    }
    std::lock_guard<std::mutex> g(c->mu);
    const int rc = check_batch_inputs(c, ct, B);
    if (rc) return rc;
    return wide_eval_host(c, ct, acc_in, acc_out, B);
}

int mkacc_eval_batch(mkacc_ctx* c, const uint32_t* ct, const uint32_t* acc_in, uint32_t* acc_out, size_t B) {
    if (!c || !ct || !acc_in || !acc_out) return fail(MKACC_E_ARG, "null argument");
    if (c->wide) {
        if (c->p.Q > 0xFFFFFFFFull)
            return fail(MKACC_E_UNSUPPORTED, "Q >= 2^32 does not fit 32-bit words: use mkacc_eval_batch_u64");
        const size_t accw = B * c->p.k * (size_t)kN;
        std::vector<uint64_t> a64(acc_in, acc_in + accw);
        const int rc = mkacc_eval_batch_u64(c, ct, a64.data(), a64.data(), B);
        if (rc) return rc;
        for (size_t s = 0; s < accw; ++s) acc_out[s] = (uint32_t)a64[s];
        return MKACC_OK;
    }
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->have_keys) return fail(MKACC_E_NOKEYS, "Bootstrapping keys have not been generated. Please call MKBTKeyGen before calling bootstrapping.");
    if (B == 0) return MKACC_OK;
    const size_t ctw = B * c->p.k * (size_t)c->p.n, accw = B * c->p.k * (size_t)kN;
    int rc0 = check_batch_inputs(c, ct, B);
    if (rc0) return rc0;
    for (size_t s = 0; s < accw; ++s)
        if (acc_in[s] >= c->p.Q) return fail(MKACC_E_RANGE, "accumulator word not a canonical residue mod Q");
    HIP_TRY(hipSetDevice(c->device));
    if (B > c->io_B) {
        if (c->d_ct) HIP_TRY(hipFree(c->d_ct));
        if (c->d_io) HIP_TRY(hipFree(c->d_io));
        c->d_ct = c->d_io = nullptr;
        c->io_B = 0;
        HIP_TRY(hipMalloc(&c->d_ct, ctw * 4));
        HIP_TRY(hipMalloc(&c->d_io, accw * 4));
        c->io_B = B;
    }
    HIP_TRY(hipMemcpyAsync(c->d_ct, ct, ctw * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_io, acc_in, accw * 4, hipMemcpyHostToDevice, c->stream));
    int rc = launch_batch(c, c->d_ct, c->d_io, c->d_io, B);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(acc_out, c->d_io, accw * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MKACC_OK;
}

int mkacc_eval_batch_device(mkacc_ctx* c, const uint32_t* d_ct, const uint32_t* d_in, uint32_t* d_out, size_t B) {
    if (!c || !d_ct || !d_in || !d_out) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    if (c->wide)   // 64-bit words: d_in / d_out hold [B][k][N] uint64_t
        return wide_launch_batch(c, d_ct, reinterpret_cast<const uint64_t*>(d_in), reinterpret_cast<uint64_t*>(d_out),
                                 B);
    return launch_batch(c, d_ct, d_in, d_out, B);
}

uint32_t mkacc_ks_digits(const mkacc_ks_params* ks) {
    if (!ks || ks->qKS < 2 || ks->baseKS < 2) return 0;
    return ks_digit_count(ks->qKS, ks->baseKS);
}

namespace {
int check_ks(mkacc_ctx* c, const mkacc_ks_params* ks) {
    if (!ks) return fail(MKACC_E_ARG, "null key-switching parameters");
    if (ks->qKS < 2 || ks->qKS > 65535) return fail(MKACC_E_UNSUPPORTED, "engine supports qKS < 2^16");
    if (ks->baseKS < 2 || ks->baseKS > 256) return fail(MKACC_E_UNSUPPORTED, "engine supports baseKS <= 256");
    if (ks->n_out == 0 || ks->n_out > 4096) return fail(MKACC_E_ARG, "bad output dimension");
    c->ks = *ks;
    c->dks = ks_digit_count(ks->qKS, ks->baseKS);
    c->n_pad = (ks->n_out + kKsTile - 1) / kKsTile * kKsTile;
    return MKACC_OK;
}
}  // namespace

int mkacc_upload_ksk_mntru(mkacc_ctx* c, const mkacc_ks_params* ks, const uint32_t* ksk) {
    if (!c || !ksk) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW) return fail(MKACC_E_ARG, "KeySwitch2 keys belong to the MKNTRU method");
    int rc = check_ks(c, ks);
    if (rc) return rc;
    const uint32_t k = c->p.k, dks = c->dks, n = ks->n_out, npad = c->n_pad;
    const size_t L = (size_t)dks * kN;
    // reference row l = j*dks + t  ->  device row t*N + j, columns padded to n_pad
    std::vector<uint16_t> h((size_t)k * L * npad, 0);
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < (uint32_t)kN; ++j)
            for (uint32_t t = 0; t < dks; ++t) {
                const uint32_t* src = ksk + (((size_t)u * kN + j) * dks + t) * n;
                uint16_t* dst = h.data() + ((size_t)u * L + (size_t)t * kN + j) * npad;
                for (uint32_t i = 0; i < n; ++i) {
                    if (src[i] >= ks->qKS) return fail(MKACC_E_RANGE, "ksk word not a canonical residue mod qKS");
                    dst[i] = (uint16_t)src[i];
                }
            }
    HIP_TRY(hipSetDevice(c->device));
    if (c->d_ksk) HIP_TRY(hipFree(c->d_ksk));
    c->d_ksk = nullptr;
    HIP_TRY(hipMalloc(&c->d_ksk, h.size() * 2));
    HIP_TRY(hipMemcpy(c->d_ksk, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    c->have_ksk = true;
    return MKACC_OK;
}

int mkacc_upload_ksk_mklwe(mkacc_ctx* c, const mkacc_ks_params* ks, const uint32_t* A, const uint32_t* B) {
    if (!c || !A || !B) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW_B) return fail(MKACC_E_ARG, "MK-LWE KeySwitch keys belong to the MKNTRU_LWE method");
    if (int rc = reject_mkntru_b(c)) return rc;
    int rc = check_ks(c, ks);
    if (rc) return rc;
    const size_t rows = (size_t)c->p.k * kN * ks->baseKS * c->dks;
    std::vector<uint16_t> ha(rows * ks->n_out), hb(rows);
    for (size_t i = 0; i < ha.size(); ++i) {
        if (A[i] >= ks->qKS) return fail(MKACC_E_RANGE, "A word not a canonical residue mod qKS");
        ha[i] = (uint16_t)A[i];
    }
    for (size_t i = 0; i < rows; ++i) {
        if (B[i] >= ks->qKS) return fail(MKACC_E_RANGE, "B word not a canonical residue mod qKS");
        hb[i] = (uint16_t)B[i];
    }
    HIP_TRY(hipSetDevice(c->device));
    if (c->d_lweA) HIP_TRY(hipFree(c->d_lweA));
    if (c->d_lweB) HIP_TRY(hipFree(c->d_lweB));
    c->d_lweA = nullptr;
    c->d_lweB = nullptr;
    HIP_TRY(hipMalloc(&c->d_lweA, ha.size() * 2));
    HIP_TRY(hipMalloc(&c->d_lweB, hb.size() * 2));
    HIP_TRY(hipMemcpy(c->d_lweA, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_lweB, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    c->have_ksk = true;
    return MKACC_OK;
}

}  // extern "C"

namespace {
// the device key-switching uploads: layout kernel(s) on the context stream, then
// the range flag (d_bad[1]) read back; no keys are kept if a word is out of range
template <class L>
int ksk_device_finish(mkacc_ctx* c, L&& launch) {
    uint32_t* kbad = c->d_bad + 1;
    HIP_TRY(hipMemsetAsync(kbad, 0, 4, c->stream));
    c->have_ksk = false;
    int rc = launch(kbad);
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    uint32_t bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, kbad, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (bad) return fail(MKACC_E_RANGE, "key-switching key word not a canonical residue mod qKS");
    c->have_ksk = true;
    return MKACC_OK;
}
}  // namespace

extern "C" {

int mkacc_upload_ksk_mntru_device(mkacc_ctx* c, const mkacc_ks_params* ks, const void* d_ksk) {
    if (!c || !d_ksk) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW) return fail(MKACC_E_ARG, "KeySwitch2 keys belong to the MKNTRU method");
    int rc = check_ks(c, ks);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    const size_t w = (size_t)c->p.k * c->dks * kN * c->n_pad;
    if (c->d_ksk) HIP_TRY(hipFree(c->d_ksk));
    c->d_ksk = nullptr;
    HIP_TRY(hipMalloc(&c->d_ksk, w * 2));
    return ksk_device_finish(c, [&](uint32_t* kbad) {
        hipLaunchKernelGGL(ksk_mntru_layout_kernel, dim3((unsigned)((w + 255) / 256)), dim3(256), 0, c->stream,
                           (const uint32_t*)d_ksk, c->d_ksk, c->p.k, c->dks, c->ks.n_out, c->n_pad,
                           (uint32_t)c->ks.qKS, kbad);
        return MKACC_OK;
    });
}

int mkacc_upload_ksk_mklwe_device(mkacc_ctx* c, const mkacc_ks_params* ks, const void* d_A, const void* d_B) {
    if (!c || !d_A || !d_B) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW_B) return fail(MKACC_E_ARG, "MK-LWE KeySwitch keys belong to the MKNTRU_LWE method");
    if (int rc = reject_mkntru_b(c)) return rc;
    int rc = check_ks(c, ks);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    const size_t rows = (size_t)c->p.k * kN * ks->baseKS * c->dks, wa = rows * ks->n_out;
    if (c->d_lweA) HIP_TRY(hipFree(c->d_lweA));
    if (c->d_lweB) HIP_TRY(hipFree(c->d_lweB));
    c->d_lweA = c->d_lweB = nullptr;
    HIP_TRY(hipMalloc(&c->d_lweA, wa * 2));
    HIP_TRY(hipMalloc(&c->d_lweB, rows * 2));
    return ksk_device_finish(c, [&](uint32_t* kbad) {
        hipLaunchKernelGGL(ksk_narrow_kernel, dim3((unsigned)((wa + 255) / 256)), dim3(256), 0, c->stream,
                           (const uint32_t*)d_A, c->d_lweA, wa, (uint32_t)ks->qKS, kbad);
        hipLaunchKernelGGL(ksk_narrow_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, c->stream,
                           (const uint32_t*)d_B, c->d_lweB, rows, (uint32_t)ks->qKS, kbad);
        return MKACC_OK;
    });
}

namespace {
// host-buffer gate staging: [ct_nand | a1 | a2 | b1 | b2] in, [out_a | out_b] out
int gate_host(mkacc_ctx* c, const uint32_t* nand, const uint32_t* a1, const uint32_t* b1, const uint32_t* a2,
              const uint32_t* b2, uint32_t* out_a, uint32_t* out_b, size_t B) {
    const bool lwe = c->method_class == XZW_B;
    const size_t kn = (size_t)c->p.k * c->p.n, kno = (size_t)c->p.k * c->ks.n_out;
    const uint64_t q = c->p.q;
    for (size_t i = 0; i < B * kn; ++i)
        if (a1[i] >= q || a2[i] >= q) return fail(MKACC_E_RANGE, "ciphertext word not a canonical residue mod q");
    if (!lwe)
        for (size_t i = 0; i < kn; ++i)
            if (nand[i] >= q) return fail(MKACC_E_RANGE, "ctNAND word not a canonical residue mod q");
    if (lwe)
        for (size_t i = 0; i < B; ++i)
            if (b1[i] >= q || b2[i] >= q) return fail(MKACC_E_RANGE, "ciphertext b not a canonical residue mod q");
    HIP_TRY(hipSetDevice(c->device));
    // staging buffers grow only: a single-gate caller (the reference's
    // EvalBinGate, boolean-mkntru.cpp:36-38) pays no allocation per gate
    const size_t in_words = kn + 2 * B * kn + 2 * B, out_words = B * kno + B;
    if (in_words > c->gin_words || out_words > c->gout_words) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->d_gin) HIP_TRY(hipFree(c->d_gin));
        if (c->d_gout) HIP_TRY(hipFree(c->d_gout));
        c->d_gin = c->d_gout = nullptr;
        c->gin_words = c->gout_words = 0;
        HIP_TRY(hipMalloc(&c->d_gin, in_words * 4));
        HIP_TRY(hipMalloc(&c->d_gout, out_words * 4));
        c->gin_words = in_words;
        c->gout_words = out_words;
    }
    uint32_t* dn = c->d_gin;
    uint32_t* d1 = dn + kn;
    uint32_t* d2 = d1 + B * kn;
    uint32_t* db1 = d2 + B * kn;
    uint32_t* db2 = db1 + B;
    if (!lwe) HIP_TRY(hipMemcpyAsync(dn, nand, kn * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d1, a1, B * kn * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d2, a2, B * kn * 4, hipMemcpyHostToDevice, c->stream));
    if (lwe) {
        HIP_TRY(hipMemcpyAsync(db1, b1, B * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(db2, b2, B * 4, hipMemcpyHostToDevice, c->stream));
    }
    int rc = launch_gates(c, dn, d1, db1, d2, db2, c->d_gout, c->d_gout + B * kno, B);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out_a, c->d_gout, B * kno * 4, hipMemcpyDeviceToHost, c->stream));
    if (lwe) HIP_TRY(hipMemcpyAsync(out_b, c->d_gout + B * kno, B * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MKACC_OK;
}
}  // namespace

int mkacc_eval_nand_mntru(mkacc_ctx* c, const uint32_t* ct_nand, const uint32_t* ct1, const uint32_t* ct2,
                          uint32_t* out, size_t B) {
    if (!c || !ct_nand || !ct1 || !ct2 || !out) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW) return fail(MKACC_E_ARG, "method is not MKNTRU");
    if (ct1 == ct2) return fail(MKACC_E_ARG, "Input ciphertexts should be independant");
    if (B == 0) return MKACC_OK;
    return gate_host(c, ct_nand, ct1, nullptr, ct2, nullptr, out, nullptr, B);
}

int mkacc_eval_nand_mklwe(mkacc_ctx* c, const uint32_t* a1, const uint32_t* b1, const uint32_t* a2,
                          const uint32_t* b2, uint32_t* out_a, uint32_t* out_b, size_t B) {
    if (!c || !a1 || !b1 || !a2 || !b2 || !out_a || !out_b) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW_B) return fail(MKACC_E_ARG, "method is not MKNTRU_LWE");
    if (int rc = reject_mkntru_b(c)) return rc;
    if (a1 == a2) return fail(MKACC_E_ARG, "Input ciphertexts should be independant");
    if (B == 0) return MKACC_OK;
    return gate_host(c, nullptr, a1, b1, a2, b2, out_a, out_b, B);
}

int mkacc_eval_nand_device(mkacc_ctx* c, const uint32_t* d_ct_nand, const uint32_t* d_a1, const uint32_t* d_b1,
                           const uint32_t* d_a2, const uint32_t* d_b2, uint32_t* d_out_a, uint32_t* d_out_b,
                           size_t B) {
    if (!c || !d_a1 || !d_a2 || !d_out_a) return fail(MKACC_E_ARG, "null argument");
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    std::lock_guard<std::mutex> g(c->mu);
    if (int rc = reject_mkntru_b(c)) return rc;
    if (c->method_class == XZW && !d_ct_nand) return fail(MKACC_E_ARG, "null ctNAND");
    if (c->method_class == XZW_B && (!d_b1 || !d_b2 || !d_out_b)) return fail(MKACC_E_ARG, "null b");
    HIP_TRY(hipSetDevice(c->device));
    return launch_gates(c, d_ct_nand, d_a1, d_b1, d_a2, d_b2, d_out_a, d_out_b, B);
}

int mkacc_gate_tail(mkacc_ctx* c, const uint32_t* acc, uint32_t* out_a, uint32_t* out_b, size_t B) {
    if (!c || !acc || !out_a || (c->method_class == XZW_B && !out_b)) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (!c->have_ksk) return fail(MKACC_E_NOKEYS, "Key-switching keys have not been uploaded");
    if (B == 0) return MKACC_OK;
    const size_t npoly = B * c->p.k, kno = (size_t)c->p.k * c->ks.n_out;
    for (size_t i = 0; i < npoly * kN; ++i)
        if (acc[i] >= c->p.Q) return fail(MKACC_E_RANGE, "accumulator word not a canonical residue mod Q");
    HIP_TRY(hipSetDevice(c->device));
    int rc = ensure_gate_ws(c, B);
    if (rc) return rc;
    uint32_t *din = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc(&din, npoly * kN * 4));
    HIP_TRY(hipMalloc(&dout, (B * kno + B) * 4));
    HIP_TRY(hipMemcpyAsync(din, acc, npoly * kN * 4, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(eval_to_c4_kernel, dim3((unsigned)((npoly * kN + 255) / 256)), dim3(256), 0, c->stream, din,
                       c->d_acc0, npoly, c->ninv, c->ninvp, c->mod.Q, (uint32_t*)nullptr);
    launch_tail(c, c->d_acc0, dout, dout + B * kno, B);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out_a, dout, B * kno * 4, hipMemcpyDeviceToHost, c->stream));
    if (out_b) HIP_TRY(hipMemcpyAsync(out_b, dout + B * kno, B * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(din));
    HIP_TRY(hipFree(dout));
    return MKACC_OK;
}

int mkacc_sync(mkacc_ctx* c) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    uint32_t bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, c->d_bad, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (bad) {
        HIP_TRY(hipMemset(c->d_bad, 0, 4));
        return fail(MKACC_E_RANGE, "an input word passed to a device entry point was out of range "
                                   "(ciphertext not mod q / 2N, accumulator or ciphertext not canonical)");
    }
    return MKACC_OK;
}

void* mkacc_stream(mkacc_ctx* c) { return c ? (void*)c->stream : nullptr; }

int mkacc_ntt_forward(mkacc_ctx* c, const uint32_t* in, uint32_t* out, size_t count) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "64-bit word context: use the _u64 primitive");
    return prim_launch(c, in, out, count, 1, 0);
}
int mkacc_ntt_inverse(mkacc_ctx* c, const uint32_t* in, uint32_t* out, size_t count) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "64-bit word context: use the _u64 primitive");
    return prim_launch(c, in, out, count, 1, 1);
}
int mkacc_sdd(mkacc_ctx* c, const uint32_t* in, uint32_t* out, size_t count) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "64-bit word context: use the _u64 primitive");
    return prim_launch(c, in, out, count, c->dg, 2);
}

namespace {
// 64-bit primitives: the wide kernels, or the 27-bit ones through narrowed words
int prim_u64(mkacc_ctx* c, const uint64_t* in, uint64_t* out, size_t count, int which) {
    if (!c || !in || !out) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return wide_prim(c, in, out, count, which);
    const size_t w = count * kN, out_mul = which == 2 ? c->dg : 1;
    std::vector<uint32_t> i32(w), o32(w * out_mul);
    for (size_t s = 0; s < w; ++s) {
        if (in[s] >= c->p.Q) return fail(MKACC_E_RANGE, "input word not a canonical residue mod Q");
        i32[s] = (uint32_t)in[s];
    }
    const int rc = prim_launch(c, i32.data(), o32.data(), count, out_mul, which);
    if (rc) return rc;
    for (size_t s = 0; s < o32.size(); ++s) out[s] = o32[s];
    return MKACC_OK;
}
}  // namespace

int mkacc_ntt_forward_u64(mkacc_ctx* c, const uint64_t* in, uint64_t* out, size_t count) {
    return prim_u64(c, in, out, count, 0);
}
int mkacc_ntt_inverse_u64(mkacc_ctx* c, const uint64_t* in, uint64_t* out, size_t count) {
    return prim_u64(c, in, out, count, 1);
}
int mkacc_sdd_u64(mkacc_ctx* c, const uint64_t* in, uint64_t* out, size_t count) {
    return prim_u64(c, in, out, count, 2);
}

}  // extern "C"

// ---- multi-device groups (include/mkfhe_amd.h) -------------------------------------

struct mkacc_group {
    std::vector<mkacc_ctx*> m;
};

extern "C" void mkacc_shard_range(size_t B, uint32_t parts, uint32_t i, size_t* begin, size_t* end) {
    // the split of mkfhe_amd/shard.py:shard_range: contiguous, sizes differ by at most one
    size_t b = 0, e = 0;
    if (parts && i < parts) {
        const size_t q = B / parts, r = B % parts;
        b = (size_t)i * q + std::min<size_t>(i, r);
        e = b + q + (i < r ? 1 : 0);
    }
    if (begin) *begin = b;
    if (end) *end = e;
}

namespace {

// dst <- src device buffer (bytes), on dst's stream: a peer copy over xGMI
// between devices, a device-to-device copy within one device
int dev_copy(mkacc_ctx* dst, void* d, const mkacc_ctx* src, const void* s, size_t bytes) {
    if (!bytes) return MKACC_OK;
    HIP_TRY(hipSetDevice(dst->device));
    if (dst->device == src->device)
        HIP_TRY(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, dst->stream));
    else
        HIP_TRY(hipMemcpyPeerAsync(d, dst->device, s, src->device, bytes, dst->stream));
    return MKACC_OK;
}
template <typename T>
int ensure_like(mkacc_ctx* dst, T*& d, size_t words) {
    if (d) return MKACC_OK;
    HIP_TRY(hipSetDevice(dst->device));
    HIP_TRY(hipMalloc(&d, words * sizeof(T)));
    return MKACC_OK;
}

// member i > 0 takes member 0's converted keys (device layout) by device copy
int share_keys(mkacc_ctx* dst, const mkacc_ctx* src) {
    const size_t kw = (size_t)src->p.k * (src->p.n + 1) * key_block_words(src), pw = (size_t)src->p.k * src->dg * kN;
    int rc;
    if (src->wide) {
        if ((rc = ensure_like(dst, dst->d_wkeys, kw)) || (rc = ensure_like(dst, dst->d_wpkey, pw))) return rc;
        if ((rc = dev_copy(dst, dst->d_wkeys, src, src->d_wkeys, kw * 8)) ||
            (rc = dev_copy(dst, dst->d_wpkey, src, src->d_wpkey, pw * 8)))
            return rc;
    } else {
        if ((rc = ensure_like(dst, dst->d_keys, kw)) || (rc = ensure_like(dst, dst->d_pkey, pw))) return rc;
        if ((rc = dev_copy(dst, dst->d_keys, src, src->d_keys, kw * 4)) ||
            (rc = dev_copy(dst, dst->d_pkey, src, src->d_pkey, pw * 4)))
            return rc;
    }
    HIP_TRY(hipStreamSynchronize(dst->stream));
    dst->have_keys = true;
    return MKACC_OK;
}

int share_ksk(mkacc_ctx* dst, const mkacc_ctx* src) {
    dst->ks = src->ks;
    dst->dks = src->dks;
    dst->n_pad = src->n_pad;
    const size_t L = (size_t)src->dks * kN;
    int rc;
    if (src->method_class == XZW) {
        const size_t w = (size_t)src->p.k * L * src->n_pad;
        if (dst->d_ksk) HIP_TRY(hipFree(dst->d_ksk));
        dst->d_ksk = nullptr;
        if ((rc = ensure_like(dst, dst->d_ksk, w)) || (rc = dev_copy(dst, dst->d_ksk, src, src->d_ksk, w * 2)))
            return rc;
    } else {
        const size_t rows = (size_t)src->p.k * kN * src->ks.baseKS * src->dks;
        if (dst->d_lweA) HIP_TRY(hipFree(dst->d_lweA));
        if (dst->d_lweB) HIP_TRY(hipFree(dst->d_lweB));
        dst->d_lweA = dst->d_lweB = nullptr;
        if ((rc = ensure_like(dst, dst->d_lweA, rows * src->ks.n_out)) || (rc = ensure_like(dst, dst->d_lweB, rows)) ||
            (rc = dev_copy(dst, dst->d_lweA, src, src->d_lweA, rows * src->ks.n_out * 2)) ||
            (rc = dev_copy(dst, dst->d_lweB, src, src->d_lweB, rows * 2)))
            return rc;
    }
    HIP_TRY(hipStreamSynchronize(dst->stream));
    dst->have_ksk = true;
    return MKACC_OK;
}

// upload through member 0 (its host-side conversion and checks), then share
template <class F, class S>
int group_upload(mkacc_group* g, F&& upload0, S&& share) {
    if (!g || g->m.empty()) return fail(MKACC_E_ARG, "null group");
    int rc = upload0(g->m[0]);
    if (rc) return rc;
    for (size_t i = 1; i < g->m.size(); ++i) {
        std::lock_guard<std::mutex> lk(g->m[i]->mu);
        if ((rc = share(g->m[i], g->m[0]))) return rc;
    }
    return MKACC_OK;
}

// run f(member, begin, count) for every non-empty shard, one host thread per
// member; the first failure (status and its message) is reported
template <class F>
int group_run(mkacc_group* g, size_t B, F&& f) {
    if (!g || g->m.empty()) return fail(MKACC_E_ARG, "null group");
    const uint32_t P = (uint32_t)g->m.size();
    std::vector<int> rcs(P, MKACC_OK);
    std::vector<std::string> msgs(P);
    std::vector<std::thread> th;
    for (uint32_t i = 0; i < P; ++i) {
        size_t b, e;
        mkacc_shard_range(B, P, i, &b, &e);
        if (e == b) continue;
        th.emplace_back([&, i, b, e] {
            rcs[i] = f(g->m[i], b, e - b);
            if (rcs[i]) msgs[i] = mkacc_last_error();
        });
    }
    for (auto& t : th) t.join();
    for (uint32_t i = 0; i < P; ++i)
        if (rcs[i]) return fail(rcs[i], "group member " + std::to_string(i) + ": " + msgs[i]);
    return MKACC_OK;
}

}  // namespace

extern "C" {

int mkacc_group_create(const mkacc_params* p, const int* devices, uint32_t count, mkacc_group** out) {
    if (!p || !devices || !out || count == 0) return fail(MKACC_E_ARG, "null argument or empty device list");
    *out = nullptr;
    auto g = std::make_unique<mkacc_group>();
    for (uint32_t i = 0; i < count; ++i) {
        mkacc_ctx* c = nullptr;
        const int rc = mkacc_create(p, devices[i], &c);
        if (rc) {
            const std::string msg = mkacc_last_error();
            mkacc_group_destroy(g.release());
            return fail(rc, msg);
        }
        g->m.push_back(c);
    }
    // direct xGMI access between the member devices where the runtime offers it
    for (uint32_t i = 0; i < count; ++i)
        for (uint32_t j = 0; j < count; ++j) {
            int can = 0;
            if (devices[i] != devices[j] && hipDeviceCanAccessPeer(&can, devices[i], devices[j]) == hipSuccess && can) {
                (void)hipSetDevice(devices[i]);
                (void)hipDeviceEnablePeerAccess(devices[j], 0);   // "already enabled" is fine
                (void)hipGetLastError();
            }
        }
    *out = g.release();
    return MKACC_OK;
}

void mkacc_group_destroy(mkacc_group* g) {
    if (!g) return;
    for (mkacc_ctx* c : g->m) mkacc_destroy(c);
    delete g;
}

uint32_t mkacc_group_size(const mkacc_group* g) { return g ? (uint32_t)g->m.size() : 0; }

mkacc_ctx* mkacc_group_member(mkacc_group* g, uint32_t i) { return g && i < g->m.size() ? g->m[i] : nullptr; }

int mkacc_group_upload_keys(mkacc_group* g, const uint32_t* evk, const uint32_t* pkey) {
    return group_upload(g, [&](mkacc_ctx* c) { return mkacc_upload_keys(c, evk, pkey); }, share_keys);
}
int mkacc_group_upload_keys_u64(mkacc_group* g, const uint64_t* evk, const uint64_t* pkey) {
    return group_upload(g, [&](mkacc_ctx* c) { return mkacc_upload_keys_u64(c, evk, pkey); }, share_keys);
}
int mkacc_group_upload_ksk_mntru(mkacc_group* g, const mkacc_ks_params* ks, const uint32_t* ksk) {
    return group_upload(g, [&](mkacc_ctx* c) { return mkacc_upload_ksk_mntru(c, ks, ksk); }, share_ksk);
}
int mkacc_group_upload_ksk_mklwe(mkacc_group* g, const mkacc_ks_params* ks, const uint32_t* A, const uint32_t* B) {
    return group_upload(g, [&](mkacc_ctx* c) { return mkacc_upload_ksk_mklwe(c, ks, A, B); }, share_ksk);
}

int mkacc_group_eval_batch(mkacc_group* g, const uint32_t* ct, const uint32_t* acc_in, uint32_t* acc_out, size_t B) {
    if (!g || g->m.empty() || !ct || !acc_in || !acc_out) return fail(MKACC_E_ARG, "null argument");
    const size_t ctw = (size_t)g->m[0]->p.k * g->m[0]->p.n, accw = (size_t)g->m[0]->p.k * kN;
    return group_run(g, B, [&](mkacc_ctx* c, size_t b, size_t cnt) {
        return mkacc_eval_batch(c, ct + b * ctw, acc_in + b * accw, acc_out + b * accw, cnt);
    });
}
int mkacc_group_eval_batch_u64(mkacc_group* g, const uint32_t* ct, const uint64_t* acc_in, uint64_t* acc_out,
                               size_t B) {
    if (!g || g->m.empty() || !ct || !acc_in || !acc_out) return fail(MKACC_E_ARG, "null argument");
    const size_t ctw = (size_t)g->m[0]->p.k * g->m[0]->p.n, accw = (size_t)g->m[0]->p.k * kN;
    return group_run(g, B, [&](mkacc_ctx* c, size_t b, size_t cnt) {
        return mkacc_eval_batch_u64(c, ct + b * ctw, acc_in + b * accw, acc_out + b * accw, cnt);
    });
}
int mkacc_group_eval_nand_mntru(mkacc_group* g, const uint32_t* ct_nand, const uint32_t* ct1, const uint32_t* ct2,
                                uint32_t* out, size_t B) {
    if (!g || g->m.empty() || !ct_nand || !ct1 || !ct2 || !out) return fail(MKACC_E_ARG, "null argument");
    if (ct1 == ct2) return fail(MKACC_E_ARG, "Input ciphertexts should be independant");
    const size_t kn = (size_t)g->m[0]->p.k * g->m[0]->p.n, kno = (size_t)g->m[0]->p.k * g->m[0]->ks.n_out;
    return group_run(g, B, [&](mkacc_ctx* c, size_t b, size_t cnt) {
        return mkacc_eval_nand_mntru(c, ct_nand, ct1 + b * kn, ct2 + b * kn, out + b * kno, cnt);
    });
}
int mkacc_group_eval_nand_mklwe(mkacc_group* g, const uint32_t* a1, const uint32_t* b1, const uint32_t* a2,
                                const uint32_t* b2, uint32_t* out_a, uint32_t* out_b, size_t B) {
    if (!g || g->m.empty() || !a1 || !b1 || !a2 || !b2 || !out_a || !out_b) return fail(MKACC_E_ARG, "null argument");
    if (a1 == a2) return fail(MKACC_E_ARG, "Input ciphertexts should be independant");
    const size_t kn = (size_t)g->m[0]->p.k * g->m[0]->p.n, kno = (size_t)g->m[0]->p.k * g->m[0]->ks.n_out;
    return group_run(g, B, [&](mkacc_ctx* c, size_t b, size_t cnt) {
        return mkacc_eval_nand_mklwe(c, a1 + b * kn, b1 + b, a2 + b * kn, b2 + b, out_a + b * kno, out_b + b, cnt);
    });
}

}  // extern "C"
