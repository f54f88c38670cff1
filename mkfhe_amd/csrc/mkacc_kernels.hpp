// mkacc_kernels.hpp -- device side of the 27-bit engine: constants, StepArgs,
// the step kernels (mk_step_kernel, mk_lat_kernel) and the batch / primitive
// kernels.  Included by the host translation unit (mkacc_engine.hip) and by the
// kernel translation units (mkacc_steps.hip, compiled once per digit count and
// for the 64-bit kernels), which hipcc builds in parallel; the host unit reaches
// the step kernels through the table below (mkacc_tu::*), so it instantiates
// none of them itself.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "../../include/mkfhe_amd.h"
#include "mkacc_device.hpp"
#include "mkacc_host_math.hpp"

using namespace mkacc;

namespace {
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
// mk_step2_kernel workgroup: kS2Waves gates sharing one LDS table image, two
// workgroups per CU (one 8-wave workgroup with one table copy per CU measured 2 %
// slower, profiles/r3/ab_step2.txt)
constexpr int kS2Waves = 4;
constexpr size_t kStep2LdsBytes = (size_t)(kLdsTabWords + kS2Waves * kLdsWords) * 4;
static_assert((8 / kS2Waves) * kStep2LdsBytes <= 160 * 1024, "8 waves per CU");

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
__host__ __device__ __forceinline__ uint32_t psi_pos(uint32_t e) { return e ^ ((e >> 5) & 3u); }

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
        return *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(psi) + a);
    }
};
__device__ __forceinline__ Mono make_mono(uint32_t c, uint32_t l) {
    const uint32_t o = ((__brev(l) >> 26) << 1) | 1u;   // 2 brv6(l) + 1
    const uint32_t co = __umul24(c, o) & (2u * kN - 1u);
    return Mono{psi_pos(co) << 3, c};
}

// MKACC_BFLY_C = 2 (forward transforms in C) for the MK-NTRU step kernels only
template <int METHOD>
constexpr bool fwd_c = kFwdC && !(MKACC_BFLY_C == 2 && METHOD != XZW);

// Lazy Shoup product x*w in [0, 2Q) (x < 2^32)
__device__ __forceinline__ uint32_t mul_shoup_lazy(uint32_t x, uint2 w, uint32_t Q) {
    const uint32_t q = __umulhi(x, w.y);
    if constexpr (MKACC_BFLY_C == 1) return (uint32_t)((uint64_t)q * (0u - Q) + (uint64_t)(x * w.x));
    return (uint32_t)mad64_pin<true>(q, 0u - Q, mul64_pin<false>(x, w.x));   // x*w - q*Q in [0, 2Q)
}

// Ranges of the lazy Montgomery sums, in units of Q (values) and Q^2 (sums).
// redc needs a sum below Q * 2^32 > 32 Q^2.  Digit-NTT outputs are < kG Q
// (digit_range), effective key words from key_eff < kD Q, and the previous
// accumulator joins the party sum as acc * (2^32 mod Q) < 2 Q^2 when it fits
// (kAccInSum), otherwise it is added after the reduction.
// CANON: the party sum's d-words are canonical (< Q): the d_i scratch (party_pass).
template <int DG, int METHOD, bool FIRST, bool CANON = false>
struct Bounds {
    static constexpr int kG = DG > 4 ? 2 : 4;
    static constexpr int kD = DG * kG * 3 + 2 <= 32 ? 3 : (DG * kG * 2 <= 32 ? 2 : 1);
    // the d-words the party sums actually see: XZW_B steps after the first use ev1 itself
    static constexpr int kDSum = ((METHOD == XZW_B && !FIRST) || CANON) ? 1 : kD;
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
template <int METHOD, bool FIRST, int KD, class M>
__device__ __forceinline__ uint32_t key_eff(uint32_t k1, uint32_t k2, uint32_t ks, const uint2* psi,
                                            const M& mp, const M& mn, int r, uint32_t Q) {
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
template <int DG, int R>
__device__ __forceinline__ void digit_range(uint32_t (&x)[R], uint32_t Q) {
    if (DG > 4) {
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = min(x[r], x[r] - 2u * Q);
    }
}

// Key words of one 4-register group of a MAC: software-pipelined kPrefetch
// groups ahead so the L2 latency of the step's key block overlaps the arithmetic.
template <int DG>
struct Prefetch { static constexpr int value = DG <= 3 ? 1 : 0; };
// accumulator loads: each gate's own rows, written by the previous step launch
// (default cache policy: non-temporal accumulator accesses cost 6 % and
// non-temporal d_i scratch accesses 16 % per config-4 step,
// profiles/r4/ab_c4_cpol.txt)
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
// The first pass stores the d_i scratch canonical (< Q), so the passes other than the
// index party's (CANON) fit the previous accumulator into the party sum
// (Bounds::kAccInSum at dg = 4): acc_u is read again at digit 0, shortly after the
// rotation read, instead of after the last digit (+3.4 % at config 4,
// profiles/r4/ab_c4_canon.txt; the index party's pass too measured the same, run v36).
// PF >= 0 overrides the prefetch depth (the small-batch kernels: one wave per SIMD,
// register file to spare, every key group an exposed L2 / HBM latency).
template <int DG, int METHOD, bool FIRST, bool START, int DS = 0, bool CANON = false, int PF = -1>
struct DigitMac {
    using Bd = Bounds<DG, METHOD, FIRST, CANON>;
    static_assert(DS == 0 || (METHOD == XZW && !FIRST), "d_i scratch: XZW steps after the first");
    static constexpr bool kAcc = START && Bd::kAccInSum;
    // X^(N-c) - 1 gathered with the key group
    static constexpr bool kMonoPf = METHOD == XZW && !FIRST && DS != 2;
    // a d_i reload comes from HBM and frees the k2 / psi registers: prefetched
    // 3 groups ahead at DG <= 3, 2 at DG >= 4 (3 spill 10 VGPRs there); 1 group measured
    // 1-4% slower (profiles/r2/ab_dscr.txt)
    static constexpr int kPrefetch = PF >= 0 ? PF : DS == 2 ? (DG <= 3 ? 3 : 2) : Prefetch<DG>::value;
    static_assert(kPrefetch < 8, "a MAC streams 8 key groups");
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
                const uint32_t dc = DS == 1 ? from3q<1>(deff, Q) : deff;
                dv[e] = dc;
                const uint64_t base = kAcc ? mad64(t.acc[e], sr.m.r32, 0) : (START ? 0ull : uj[r]);
                uj[r] = mad64(g[r], (DS == 1 && CANON) ? dc : deff, base);
                sv[r] = mad64(g[r], t.pk[e], sv[r]);
            }
            if (DS == 1) bstore4(dv, sr.rds, sr.vo, doff + gq * 1024u);
            sched_fence();
        }
    }
};

// w += h * f_i                                  (xzw.cpp:281-288)
// (first step, and XZW_B: f-words reduced to canonical, Bounds' f-part bound)
template <int DG, int METHOD, bool FIRST, int PF = -1>
__device__ __forceinline__ void mac_index(const uint32_t (&h)[kRegs], int i, uint64_t (&w)[kRegs],
                                          __amdgpu_buffer_rsrc_t rk1, __amdgpu_buffer_rsrc_t rk2,
                                          __amdgpu_buffer_rsrc_t rks, const uint2* psi, const Mono& mp,
                                          const Mono& mn, uint32_t vo, uint32_t Q) {
    const uint32_t polyB = kN * 4u;
    const uint32_t koff = (uint32_t)(2 * i + 1) * polyB;
    constexpr int kPrefetch = PF >= 0 ? PF : Prefetch<DG>::value;
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
template <int DG, int PF = -1>
struct SplitMac {
    static constexpr int kPrefetch = PF >= 0 ? PF : Prefetch<DG>::value;
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
// d_i reload passes (DS = 2) alternate the order of digits 1..DG-1 (rev: DG-1 down
// to 1), so a pass starts its reloads with the digit the previous pass read last
// (shorter reuse distance of the scratch lines in L2; +0.3 %, profiles/r4/ab_c4_alt.txt).
// Every digit's products are the same exact lazy sums in another order: bit-exact.
template <int DG, int METHOD, bool FIRST, bool LAST, int DS = 0>
__device__ __forceinline__ void party_pass(const StepCtx& s, uint32_t u, uint64_t (&sv)[kRegs],
                                           uint64_t (&uj)[kRegs], bool rev = false) {
    constexpr bool kCanon = !LAST && DS != 0;
    using Bd = Bounds<DG, METHOD, FIRST, kCanon>;
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
        const DigitMac<DG, METHOD, FIRST, true, DS, kCanon> mac(sr, 0, u);
        KeyGroup kg[mac.kBuf];
        ntt_fwd<fwd_c<METHOD>>(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
        digit_range<DG>(x, Q);
#pragma unroll
        for (int j = 0; j < mac.kPrefetch; ++j) mac.issue(kg[j], j);
        mac.run(x, uj, sv, kg);
    }
#pragma unroll 1
    for (int i = 1; i < DG; ++i) {
        const int j = (DS == 2 && rev) ? DG - i : i;
#pragma unroll
        for (int r = 0; r < kRegs; ++r) x[r] = pd.get(r, j + 1, s.sd);
        const DigitMac<DG, METHOD, FIRST, false, DS, kCanon> mac(sr, j, u);
        KeyGroup kg[mac.kBuf];
        ntt_fwd<fwd_c<METHOD>>(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
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
__device__ __forceinline__ void lat_step(const StepArgs a, uint32_t* smem) {
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
    if (u == index) {
        party_pass<DG, METHOD, FIRST, true>(s, u, sv, w);
    } else {
        party_pass<DG, METHOD, FIRST, false>(s, u, sv, w);
        vcc_fence();   // the branches' join follows the party's last reductions
    }
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
template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(64 * kLatMaxK, 1) void mk_lat_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image(smem, a.img);
    lat_step<DG, METHOD, FIRST>(a, smem);
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
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (uint32_t t = t0; t < k; ++t) {
        party_pass<DG, METHOD, FIRST, false, DSCR ? 2 : 0>(s, index + t < k ? index + t : index + t - k, sv, w,
                                                           (t & 1u) == 0);
        grow_sv();
    }
    party_pass<DG, METHOD, FIRST, true, DSCR ? 2 : 0>(s, index, sv, w, (k & 1u) == 0);
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
            ntt_fwd<fwd_c<METHOD>>(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, l, Q, s.m.m1);
            digit_range<DG>(x, Q);
#pragma unroll
            for (int j = 0; j < mac.kPrefetch; ++j) mac.issue(kg[j], j);
            mac.run(x, w, w2, kg);
        } else {
            ntt_fwd<fwd_c<METHOD>>(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, l, Q, s.m.m1);
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

// ---- two-party small batches with the digits split over waves (mk_latd_kernel) ----
// mk_lat_kernel's step has 2 (dg + 1) transforms on its critical path: a party
// pass (iNTT + dg digit NTTs) on every party's wave at once, then the f-part on
// one wave.  For k = 2 this kernel runs each party on two waves and the f-part on
// dg waves (one workgroup of four waves per gate, one per SIMD): every wave of a
// party recomputes its iNTT (no exchange, off the critical path) and transforms
// and multiplies only its share of the digits; the lazy sums are reduced once per
// wave and added through LDS.  Critical path: iNTT + ceil(dg / 2) digit NTTs, then
// iNTT + one digit NTT.  Sums exact mod Q, so bit-exact like the other kernels.
constexpr uint32_t kLatdWaves = 4;
// Latency switches of the split-digit kernel (one wave per SIMD: the wave's own
// memory latency is exposed, not hidden by other waves):
//   MKACC_LATD_PFD    key groups a MAC streams ahead (-1: the batch kernels' depth)
//   MKACC_LATD_KPF    1: the waves the f-part leaves idle pull the next step's key
//                     block into L2 while it runs (mk_latd_run_kernel)
//   MKACC_LATD_TWLDS  1: the per-lane NTT twiddles of both directions in LDS
//                     (the batch kernels read them from L1/L2 behind other waves)
#ifndef MKACC_LATD_PFD
#define MKACC_LATD_PFD -1
#endif
#ifndef MKACC_LATD_KPF
#define MKACC_LATD_KPF 0
#endif
#ifndef MKACC_LATD_TWLDS
#define MKACC_LATD_TWLDS 0
#endif
constexpr int kLatdPfd = MKACC_LATD_PFD;
// LDS: [forward + inverse per-lane twiddle image][psi^e - 1][4 transpose scratches]
// with MKACC_LATD_TWLDS, else the batch kernels' [stage-10 twiddles][psi^e - 1][...]
constexpr int kLatdImgPairs = kTwlPairs + kInvImgPairs;   // image pairs [0, kLatdImgPairs): both directions
constexpr int kLatdTabWords = MKACC_LATD_TWLDS ? 2 * (kLatdImgPairs + kPsiPairs) : kLdsTabWords;
constexpr size_t latd_lds_bytes() { return (size_t)(kLatdTabWords + kLatdWaves * kLdsWords) * 4; }
static_assert(latd_lds_bytes() <= 160 * 1024, "one split-digit workgroup per CU");
static_assert(kLatdImgPairs % 2 == 0 && kLatdImgPairs == kPsiOff, "both directions' images are contiguous, dwordx4 copy");
__device__ __forceinline__ void load_image_latd(uint32_t* smem, const uint32_t* img) {
    if constexpr (MKACC_LATD_TWLDS) {
        const uint4* src = reinterpret_cast<const uint4*>(img);
        uint4* dst = reinterpret_cast<uint4*>(smem);
        for (int i = threadIdx.x; i < kLatdImgPairs / 2; i += blockDim.x) dst[i] = src[i];
        for (int i = threadIdx.x; i < kN; i += blockDim.x) dst[kLatdImgPairs / 2 + i] = src[kPsm1Off / 2 + i];
        __syncthreads();
    } else {
        load_image(smem, img);
    }
}
__device__ __forceinline__ Tables tables_latd(uint32_t* smem, const uint32_t* img) {
    if constexpr (MKACC_LATD_TWLDS) {
        const uint2* t = reinterpret_cast<const uint2*>(smem);
        return Tables{t, t + kTwlPairs, t + kTwlC, t + kLatdImgPairs};
    } else {
        return tables(smem, img);
    }
}
// Pull [p, p + BYTES) into L2: one dword per 64-byte line, PARTS waves sharing the
// lines.  The loads are consumed only by an empty asm, so the wave waits for them
// once, at its next barrier, and nothing else waits behind them.
template <uint32_t BYTES, uint32_t PARTS>
__device__ __forceinline__ void l2_touch(const uint32_t* p, uint32_t part, uint32_t l) {
    constexpr uint32_t kChunks = BYTES / 4096u;   // 64 lanes x 64 B per load
    static_assert(BYTES % 4096u == 0, "whole chunks");
    constexpr uint32_t kPer = (kChunks + PARTS - 1) / PARTS;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(p, BYTES);   // a chunk past the end loads 0, no access
    uint32_t v[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b32(r, l * 64u, (j * PARTS + part) * 4096u, 0);
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) acc |= v[j];
    asm volatile("" ::"v"(acc));
}
// digits [d0, d1) of party u: uj (its partial party sum, from acc_u * 2^32 at digit 0
// when the bound allows) and sv (its share of sumV) as lazy 64-bit sums
template <int DG, int METHOD, bool FIRST>
__device__ __forceinline__ void party_digits(const StepCtx& s, uint32_t u, uint32_t d0, uint32_t d1,
                                             uint64_t (&sv)[kRegs], uint64_t (&uj)[kRegs]) {
    const uint32_t Q = s.m.Q, polyB = kN * 4u;
    uint32_t x[kRegs];
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) {
        const u32x4 t = aload4(s.rin, s.vo, u * polyB + gq * 1024u);
        x[4 * gq] = t.x; x[4 * gq + 1] = t.y; x[4 * gq + 2] = t.z; x[4 * gq + 3] = t.w;
    }
    if (!FIRST) {
        // acctemp = acc * (X^c - 1)                     (xzw.cpp:336-338)
        uint2 mw[kRegs];
#pragma unroll
        for (int r = 0; r < kRegs; ++r) mw[r] = s.mp.at(s.tb.psi, r);
        sched_fence();
#pragma unroll
        for (int r = 0; r < kRegs; ++r) x[r] = mul_shoup_lazy(x[r], mw[r], Q);
    }
    ntt_inv(x, s.lds, s.tw_inv, s.tb.twi, s.l, Q);
    PackedDigits<DG> pd;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        x[r] = pd.put(r, sdd_offset(x[r], s.sd), s.sd);
        if ((r & 7) == 7) sched_fence();
    }
    const StepRes sr = s.res();
#pragma unroll 1
    for (uint32_t i = d0; i < d1; ++i) {
        if (i > 0) {
#pragma unroll
            for (int r = 0; r < kRegs; ++r) x[r] = pd.get(r, (int)i + 1, s.sd);
        }
        ntt_fwd<fwd_c<METHOD>>(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
        digit_range<DG>(x, Q);
        vcc_fence();   // the digit-0 branch follows the last butterflies
        if (i == 0) {
            const DigitMac<DG, METHOD, FIRST, true, 0, false, kLatdPfd> mac(sr, 0, u);
            KeyGroup kg[mac.kBuf];
#pragma unroll
            for (int j = 0; j < mac.kPrefetch; ++j) mac.issue(kg[j], j);
            mac.run(x, uj, sv, kg);
        } else {
            const DigitMac<DG, METHOD, FIRST, false, 0, false, kLatdPfd> mac(sr, (int)i, u);
            KeyGroup kg[mac.kBuf];
#pragma unroll
            for (int j = 0; j < mac.kPrefetch; ++j) mac.issue(kg[j], j);
            mac.run(x, uj, sv, kg);
        }
        vcc_fence();   // the loop branch follows the MAC's reductions
    }
}
// f-part digit f of party `index` (mk-acc-xzw.cpp:272-289): x = sumV in [0, 2Q);
// w enters with the index party's sum (digit 0's wave) or 0 and leaves as its
// share of acc'[index] in [0, 2Q)
template <int DG, int METHOD, bool FIRST>
__device__ __forceinline__ void f_digit(const StepCtx& s, uint32_t f, uint64_t (&w)[kRegs], uint32_t (&x)[kRegs]) {
    const uint32_t Q = s.m.Q;
    const StepRes sr = s.res();
    ntt_inv(x, s.lds, s.tw_inv, s.tb.twi, s.l, Q);
    PackedDigits<DG> pd;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        x[r] = pd.put(r, sdd_offset(x[r], s.sd), s.sd);
        if ((r & 7) == 7) sched_fence();
    }
    if (f > 0) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) x[r] = pd.get(r, (int)f + 1, s.sd);
    }
    constexpr bool kSplit = METHOD == XZW && !FIRST;
    uint64_t w2[kSplit ? kRegs : 1];
    ntt_fwd<fwd_c<METHOD>>(x, s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
    digit_range<DG>(x, Q);
    if constexpr (kSplit) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) w2[r] = 0;
        const SplitMac<DG, kLatdPfd> mac(sr, (int)f);
        KeyGroup kg[mac.kBuf];
#pragma unroll
        for (int j = 0; j < mac.kPrefetch; ++j) mac.issue(kg[j], j);
        mac.run(x, w, w2, kg);
    } else {
        mac_index<DG, METHOD, FIRST, kLatdPfd>(x, (int)f, w, s.rk1, s.rk2, s.rks, s.tb.psi, s.mp, s.mn, s.vo, Q);
    }
    uint2 mw[kSplit ? kRegs : 1];
    if constexpr (kSplit) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) mw[r] = s.mn.at(s.tb.psi, r);
    }
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        uint32_t v = redc(w[r], Q, s.m.qinv);                                       // [0, 2Q)
        if constexpr (kSplit) {
            v += mul_shoup_lazy(redc(w2[r], Q, s.m.qinv), mw[r], Q);                 // [0, 4Q)
            v = min(v, v - 2u * Q);
        }
        x[r] = v;
    }
}

// pf: the next step's key block (the run kernel), pulled into L2 by the waves the
// f-part leaves idle (MKACC_LATD_KPF); null for none
template <int DG, int METHOD, bool FIRST>
__device__ __forceinline__ void latd_step(const StepArgs a, uint32_t* smem, const uint32_t* pf = nullptr) {
    using Bd = Bounds<DG, METHOD, FIRST>;
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // this wave
    const uint32_t gate = blockIdx.x;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = 2u, index = a.index;
    const uint32_t polyB = kN * 4u;
    uint32_t* const scratch = smem + kLatdTabWords + wv * kLdsWords;
    const StepCtx s{tables_latd(smem, a.img),
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
    // party p = wv / 2 takes digits [0, dh) (half 0) or [dh, DG) (half 1)
    const uint32_t p = wv >> 1, half = wv & 1u;
    constexpr uint32_t kDh = (DG + 1) / 2;
    uint64_t sv[kRegs], uj[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) sv[r] = uj[r] = 0;
    party_digits<DG, METHOD, FIRST>(s, p, half ? kDh : 0u, half ? (uint32_t)DG : kDh, sv, uj);
    // (1) party sums: acc'_p = the two halves (+ acc_p when it was not in the sum)
#pragma unroll
    for (int r = 0; r < kRegs; ++r) scratch[r * 64 + l] = redc(uj[r], Q, s.m.qinv);
    vcc_fence();   // the branches below follow the reductions' multiply-adds
    __syncthreads();
    uint64_t w[kRegs];
    // the f-part: wave 2 index takes digit 0 (it holds the index party's sum), the
    // others digits 1, 2, ... in wave order after it
    const uint32_t f = (wv + kLatdWaves - 2u * index) % kLatdWaves;
    if (half == 0) {
        const uint32_t* o = smem + kLatdTabWords + (wv + 1u) * kLdsWords;
        uint32_t t4[kRegs];
#pragma unroll
        for (int r = 0; r < kRegs; ++r) t4[r] = scratch[r * 64 + l] + o[r * 64 + l];   // < 4Q
        if constexpr (!Bd::kAccInSum && !FIRST) {
#pragma unroll
            for (int gq = 0; gq < 8; ++gq) {
                const u32x4 t = aload4(s.rin, s.vo, p * polyB + gq * 1024u);
#pragma unroll
                for (int e = 0; e < 4; ++e) t4[4 * gq + e] += t[e];                      // < 6Q
            }
        }
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            uint32_t v = min(t4[r], t4[r] - 4u * Q);
            t4[r] = min(v, v - 2u * Q);                                                 // [0, 2Q)
        }
        if (p != index) {
#pragma unroll
            for (int gq = 0; gq < 8; ++gq)
                bstore4(u32x4{t4[4 * gq], t4[4 * gq + 1], t4[4 * gq + 2], t4[4 * gq + 3]}, s.rout, s.vo,
                        p * polyB + gq * 1024u);
        } else {
#pragma unroll
            for (int r = 0; r < kRegs; ++r) w[r] = mad64(t4[r], s.m.r32, 0);           // < 2 Q^2
        }
    }
    if (f != 0) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) w[r] = 0;
    }
    __syncthreads();
    // (2) sumV: every wave's share, [0, 2Q) each
#pragma unroll
    for (int r = 0; r < kRegs; ++r) scratch[r * 64 + l] = redc(sv[r], Q, s.m.qinv);
    vcc_fence();
    __syncthreads();
    uint32_t x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        uint32_t v = 0;
        for (uint32_t q = 0; q < kLatdWaves; ++q) v += smem[kLatdTabWords + q * kLdsWords + r * 64 + l];   // < 8Q
        v = min(v, v - 4u * Q);
        x[r] = min(v, v - 2u * Q);                                                      // [0, 2Q)
    }
    __syncthreads();   // every wave has read the shares before the transforms reuse the scratch
    // (3) f-part digit f on waves f < DG, then acc'[index] = the sum of their shares
    if (f < DG) f_digit<DG, METHOD, FIRST>(s, f, w, x);
    vcc_fence();
    if constexpr (MKACC_LATD_KPF && DG < (int)kLatdWaves) {
        if (f >= DG && pf) l2_touch<(METHOD == XZW ? 2u : 1u) * DG * 2u * kN * 4u, kLatdWaves - DG>(pf, f - DG, l);
    }
    if (f < DG) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) scratch[r * 64 + l] = x[r];
    }
    __syncthreads();
    if (f != 0) return;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        uint32_t v = 0;
        for (uint32_t q = 0; q < kLatdWaves; ++q) {
            const uint32_t fq = (q + kLatdWaves - 2u * index) % kLatdWaves;
            if (fq < DG) v += smem[kLatdTabWords + q * kLdsWords + r * 64 + l];              // < 2 DG Q <= 8Q
        }
        v = min(v, v - 4u * Q);
        x[r] = min(v, v - 2u * Q);
    }
#pragma unroll
    for (int gq = 0; gq < 8; ++gq)
        bstore4(u32x4{x[4 * gq], x[4 * gq + 1], x[4 * gq + 2], x[4 * gq + 3]}, s.rout, s.vo, index * polyB + gq * 1024u);
}

template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(64 * kLatdWaves, 1) void mk_latd_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image_latd(smem, a.img);
    latd_step<DG, METHOD, FIRST>(a, smem);
}

// Steps [t0, t1) (t = u n + i, none of them the first) of a batch of at most one
// gate per CU in ONE launch: each workgroup runs its gate's steps back to back,
// with the LDS tables loaded once and no launch between steps.  A step's
// accumulator stores are complete (vmcnt) and the workgroup has passed a barrier
// before the next step's waves read them: the waves of a workgroup share the CU's
// write-through L1, so no cache maintenance is needed at workgroup scope.
struct LatdRun {
    const uint32_t* keys;   // key blocks [k][n + 1] of kbw words (mkacc_engine key_step)
    const uint32_t* cvals;  // [k n][cstride] exponents, this launch's gates at column 0
    uint32_t* acc0;         // step t0's input; t0 + 1's input in acc1, and so on
    uint32_t* acc1;
    uint64_t kbw;           // words per key block
    uint32_t cstride, n, t0, t1, key2off;
};
// key block of step t
__device__ __forceinline__ const uint32_t* run_keys(const LatdRun& r, uint32_t t) {
    const uint32_t u = t / r.n, i = t - u * r.n;
    return r.keys + ((uint64_t)u * (r.n + 1) + i) * r.kbw;
}
// step t's arguments from the launch's first-step arguments
__device__ __forceinline__ StepArgs run_args(const StepArgs& a, const LatdRun& r, uint32_t t) {
    const uint32_t u = t / r.n;
    StepArgs b = a;
    b.key1 = run_keys(r, t);
    b.key2 = b.key1 + r.key2off;
    b.cvals = r.cvals + (uint64_t)t * r.cstride;
    b.index = u;
    const bool odd = ((t - r.t0) & 1u) != 0;
    b.acc_in = odd ? r.acc1 : r.acc0;
    b.acc_out = odd ? r.acc0 : r.acc1;
    return b;
}
template <int DG, int METHOD>
__global__ __launch_bounds__(64 * kLatdWaves, 1) void mk_latd_run_kernel(StepArgs a, LatdRun r) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image_latd(smem, a.img);
#pragma unroll 1
    for (uint32_t t = r.t0; t < r.t1; ++t) {
        latd_step<DG, METHOD, false>(run_args(a, r, t), smem, t + 1 < r.t1 ? run_keys(r, t + 1) : nullptr);
        vcc_fence();   // the loop branch follows the step's last reductions
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}
// the same for mk_lat_kernel (one wave per party) at k <= kLatRunMaxK: the register
// file of one wave per SIMD (VGPRs + AGPRs; at 256 the loop spills), so the host takes
// it only for batches whose k B waves are resident at once (one wave per SIMD)
constexpr uint32_t kLatRunMaxK = 4;
// workgroups per CU the loop is built for: two at dg = 2 (spill-free at 256 VGPRs;
// k = 4, B = 512: 90.6 -> 82.8 ms, B <= 256 within 1 %, profiles/r5/ab_lat_run_occ_v28.txt),
// one above (two would spill 20-52 B per lane)
constexpr uint32_t lat_run_occ(uint32_t dg) { return dg == 2 ? 2 : 1; }
// parties the loop is built for: up to kLatMaxK at dg = 2 (eight waves of 256 VGPRs
// are the same register budget as two four-wave workgroups), kLatRunMaxK above
constexpr uint32_t lat_run_max_k(uint32_t dg) { return dg == 2 ? kLatMaxK : kLatRunMaxK; }
template <int DG, int METHOD>
__global__ __launch_bounds__(64 * lat_run_max_k(DG), DG == 2 ? 1 : lat_run_occ(DG)) void mk_lat_run_kernel(StepArgs a,
                                                                                                       LatdRun r) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image(smem, a.img);
#pragma unroll 1
    for (uint32_t t = r.t0; t < r.t1; ++t) {
        lat_step<DG, METHOD, false>(run_args(a, r, t), smem);
        vcc_fence();   // the loop branch follows the step's last reductions
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
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


#include "mkacc_step2.hpp"
#include "mkacc_layout2.hpp"
#include "mkacc_quad.hpp"

template <int DG, bool FIRST>
StepFn pick_step2(int method) {
    return method == XZW ? mk_step2_kernel<DG, XZW, FIRST> : mk_step2_kernel<DG, XZW_B, FIRST>;
}

template <int DG>
StepFn pick_lat(int method, bool first) {
    if (method == XZW) return first ? mk_lat_kernel<DG, XZW, true> : mk_lat_kernel<DG, XZW, false>;
    return first ? mk_lat_kernel<DG, XZW_B, true> : mk_lat_kernel<DG, XZW_B, false>;
}
template <int DG>
StepFn pick_latd(int method, bool first) {
    if (method == XZW) return first ? mk_latd_kernel<DG, XZW, true> : mk_latd_kernel<DG, XZW, false>;
    return first ? mk_latd_kernel<DG, XZW_B, true> : mk_latd_kernel<DG, XZW_B, false>;
}
template <int DG>
const void* pick_latd_run(int method) {
    return method == XZW ? (const void*)mk_latd_run_kernel<DG, XZW> : (const void*)mk_latd_run_kernel<DG, XZW_B>;
}
template <int DG>
const void* pick_lat_run(int method) {
    return method == XZW ? (const void*)mk_lat_run_kernel<DG, XZW> : (const void*)mk_lat_run_kernel<DG, XZW_B>;
}

}  // namespace

// Kernel table across translation units: host-stub addresses of the step kernel
// instantiations (launched with hipLaunchKernel), null for a combination that
// does not exist.
namespace mkacc_tu {
using KernelPtr = const void*;
#define MKACC_TU_API __attribute__((visibility("hidden")))
MKACC_TU_API KernelPtr step_dg4(int method, bool first, bool dscr);   // mk_step_kernel (dg >= 4)
MKACC_TU_API KernelPtr step_dg5(int method, bool first, bool dscr);
MKACC_TU_API KernelPtr step2_dg2(int method);    // mk_step2_kernel (mkacc_step2.hpp, dg <= 3), later steps
MKACC_TU_API KernelPtr step2_dg3(int method);
MKACC_TU_API KernelPtr step2f_dg2(int method);   // its first (KDM) step, a unit of its own (build.py STEP2_BFLY)
MKACC_TU_API KernelPtr step2f_dg3(int method);
MKACC_TU_API KernelPtr lat_dg2(int method, bool first);
MKACC_TU_API KernelPtr lat_dg3(int method, bool first);
MKACC_TU_API KernelPtr lat_dg4(int method, bool first);
MKACC_TU_API KernelPtr latd_dg2(int method, bool first);   // mk_latd_kernel (k = 2, digits split over waves)
MKACC_TU_API KernelPtr latd_dg3(int method, bool first);
MKACC_TU_API KernelPtr latd_dg4(int method, bool first);
MKACC_TU_API KernelPtr latdrun_dg2(int method);   // mk_latd_run_kernel (the later steps in one launch)
MKACC_TU_API KernelPtr latdrun_dg3(int method);
MKACC_TU_API KernelPtr latdrun_dg4(int method);
MKACC_TU_API KernelPtr latrun_dg2(int method);    // mk_lat_run_kernel (the later steps in one launch)
MKACC_TU_API KernelPtr latrun_dg3(int method);
MKACC_TU_API KernelPtr latrun_dg4(int method);
MKACC_TU_API KernelPtr quad_dg2(int method, bool first, int occ);   // mk_quad_kernel (a gate per workgroup, quarter polynomials)
MKACC_TU_API KernelPtr quad_dg3(int method, bool first, int occ);
MKACC_TU_API KernelPtr quad_dg4(int method, bool first, int occ);
MKACC_TU_API KernelPtr quad_dg5(int method, bool first, int occ);
MKACC_TU_API KernelPtr quadrun_dg2(int method, int occ);            // mk_quad_run_kernel (the later steps in one launch)
MKACC_TU_API KernelPtr quadrun_dg3(int method, int occ);
MKACC_TU_API KernelPtr quadrun_dg4(int method, int occ);
MKACC_TU_API KernelPtr quadrun_dg5(int method, int occ);
MKACC_TU_API KernelPtr wide_step(int method, bool first);     // mkacc_wide.hpp (integer 64-bit words)
MKACC_TU_API KernelPtr widereg2_step(int method, bool first);  // mkacc_widereg2.hpp (FP64, Q < 2^50)
}  // namespace mkacc_tu
