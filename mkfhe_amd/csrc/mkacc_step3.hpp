// mkacc_step3.hpp -- the 27-bit batch step kernel with TWO waves per gate
// (mk_step3_kernel).  Included inside mkacc_kernels.hpp's anonymous namespace,
// after mkacc_step2.hpp and mkacc_layout2.hpp.
//
// The algebra and pass structure are mk_step2_kernel's (HbProd, mk-acc-xzw.cpp:
// 231-290, fused with AddToAccXZW{,0}, xzw.cpp:292-381; digit NTTs first, then
// one streaming pass over the step's key words per party and for the f-part, the
// split form acc' = redc(a1) + (X^(N-c) - 1) redc(a2); every sum exact mod Q, so
// bit-exact).  What changes is the data split: a gate's polynomials are spread
// over the two waves of a 128-thread workgroup, 16 words per lane
// (mkacc_layout2.hpp), so every per-wave array halves -- at dg = 4 the digit-NTT
// outputs are 4 x 16 registers instead of 4 x 32, which lets two waves share a
// SIMD without the per-gate d_i scratch of mk_step_kernel (config 4,
// STD128_MKNTRU_3).  The EVAL layout LC4 is the one-wave layout C split at slot
// bit 4, so the C4 key and accumulator words of every other 27-bit kernel serve
// unchanged (a wave's base offset is 4 KiB further).  Transforms cross the two
// waves through LDS (one 2-wave barrier per transpose); per-lane twiddles and the
// psi^e - 1 table are read from HBM through L1 (no LDS table image).
#pragma once

namespace s3 {

using lay2::kR;
using lay2::Lane;
using lay2::TwPairs;
using lay2::tload;
constexpr size_t kLdsBytes = 2 * lay2::kBufE * 4;   // two ping-pong u32 buffers per gate

__device__ __forceinline__ uint2 tw(const u32x2 v) { return make_uint2(v.x, v.y); }

// Inverse pass 1 (bits 0..3, 16 registers): bounds in units of Q per register;
// a twiddle-1 butterfly skips its product while the doubled bound leaves room for
// the remaining pass-1 stages (+2 each); everything entering pass 2 stays below
// 18 Q, so the seven per-lane stages end below 32 Q <= 2^32 (Q < 2^27).
struct InvPlan3 {
    bool skip[4][kR];
    int bound[4][kR];
    int maxb;
    constexpr explicit InvPlan3(int b0) : skip{}, bound{}, maxb(0) {
        int bd[kR] = {};
        for (int r = 0; r < kR; ++r) bd[r] = b0;
        for (int b = 0; b < 4; ++b) {
            const int h = 1 << b;
            for (int r = 0; r < kR; ++r) bound[b][r] = bd[r];
            for (int r = 0; r < kR; ++r) {
                if (r & h) continue;
                const int s = bd[r] + bd[r + h];
                if ((r & (h - 1)) == 0 && s + 2 * (3 - b) <= 18) {
                    skip[b][r] = true;
                    bd[r] = bd[r + h] = s;
                } else {
                    bd[r] = bd[r + h] = bd[r] + 2;
                }
            }
        }
        for (int r = 0; r < kR; ++r) maxb = bd[r] > maxb ? bd[r] : maxb;
    }
};
constexpr InvPlan3 kInvPlan3(2);   // inputs in [0, 2Q)
static_assert(kInvPlan3.maxb + 2 * 7 <= 32, "inverse NTT bounds");

// Forward negacyclic NTT (reference EVAL order): coefficients in LA, [0, 2Q) ->
// slots in LC4, [0, 4Q).  Lazy Shoup butterflies as ntt_fwd (mkacc_device.hpp):
// a stage adds < 2Q, stage 10 (ct_bfly_last) brings a under 2Q first.
//   tw_g: reference forward table {-w, w'} (scalar reads, indices 1..15)
__device__ __forceinline__ void ntt_fwd(uint32_t (&x)[kR], uint32_t* bufs, const uint2* tw_g,
                                        __amdgpu_buffer_rsrc_t rt, const Lane& ln, uint32_t Q, uint32_t m1) {
    TwPairs<4> fb;
    tload<lay2::TFB>(fb, rt, ln.vt);
    const ConstTable twc{(const_u64*)opaque(tw_g)};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int H = 8 >> s;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            ct_bfly_lazy<true>(x[r], x[r + H], twc[(1 << s) + (r >> (4 - s))], Q);
        }
    }
    lay2::transpose<lay2::LA, lay2::LB>(x, bufs, ln.l, ln.w);
    TwPairs<8> fc;
    tload<lay2::TFC>(fc, rt, ln.vt);
#pragma unroll
    for (int s = 4; s < 7; ++s) {
        const int H = 8 >> (s - 4);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            ct_bfly_lazy(x[r], x[r + H], tw(fb.raw(((1 << (s - 4)) - 1) + (r >> (8 - s)))), Q);
        }
    }
    lay2::transpose<lay2::LB, lay2::LC4>(x, bufs + lay2::kBufE, ln.l, ln.w);
#pragma unroll
    for (int s = 7; s < 10; ++s) {
        const int H = 8 >> (s - 7);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            ct_bfly_lazy(x[r], x[r + H], tw(fc.raw(((1 << (s - 7)) - 1) + (r >> (11 - s)))), Q);
        }
    }
#pragma unroll
    for (int j = 0; j < kR / 2; ++j) ct_bfly_last(x[2 * j], x[2 * j + 1], tw(fc.raw(7 + j)), Q, m1);
}

// Inverse without N^-1 (folded into keys and accumulators): slots
// in LC4, [0, 2Q) -> canonical coefficients in LA.  DIT over the slot bits
// (ntt_inv, mkacc_device.hpp): bits 0-3 wave-uniform ({-w, w'} from tis[(1 << b) + t]),
// bits 4-7 and 8-10 per lane, then the psi^-p Shoup twist (canonical output).
__device__ __forceinline__ void ntt_inv(uint32_t (&x)[kR], uint32_t* bufs, const uint2* tis,
                                        __amdgpu_buffer_rsrc_t rt, const Lane& ln, uint32_t Q) {
    TwPairs<8> id;
    tload<lay2::TID>(id, rt, ln.vt);
    const ConstTable twc{(const_u64*)opaque(tis)};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int H = 1 << b;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            if (kInvPlan3.skip[b][r]) {
                const uint32_t X = x[r], Y = x[r + H];
                x[r] = X + Y;
                x[r + H] = X - Y + (uint32_t)kInvPlan3.bound[b][r + H] * Q;
            } else {
                ct_bfly_lazy<true>(x[r], x[r + H], twc[(1 << b) + (r & (H - 1))], Q);
            }
        }
    }
    TwPairs<7> ia;
    tload<lay2::TIA>(ia, rt, ln.vt);
    lay2::transpose<lay2::LC4, lay2::LD>(x, bufs, ln.l, ln.w);
#pragma unroll
    for (int b = 4; b < 8; ++b) {
        const int H = 1 << (b - 4);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            ct_bfly_lazy(x[r], x[r + H], tw(id.raw((H - 1) + (r & (H - 1)))), Q);
        }
    }
    TwPairs<8> tt;
    tload<lay2::TTW>(tt, rt, ln.vt);
    lay2::transpose<lay2::LD, lay2::LA>(x, bufs + lay2::kBufE, ln.l, ln.w);
#pragma unroll
    for (int b = 8; b < 11; ++b) {
        const int H = 1 << (b - 7);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (r & H) continue;
            ct_bfly_lazy(x[r], x[r + H], tw(ia.raw((H - 2) + (r & (H - 1)))), Q);
        }
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
        const uint2 t = tw(tt.raw(r));
        x[r] = mul_shoup(x[r], t.x, t.y, Q);
    }
}

// X^c - 1 at slot (l << 5) | (w << 4) | r (Mono, mkacc_kernels.hpp): 2 brv11 + 1 =
// 256 brv4(r) + 128 w + 2 brv6(l) + 1; the register part moves bits >= 8 of the
// exponent only, which psi_pos leaves in place.  psi: the HBM image's psi^e - 1 pairs.
struct Mono3 {
    uint32_t w;         // per lane: 8 psi_pos(c (2 brv6(l) + 128 wave + 1) mod 2N)
    uint32_t c;         // wave-uniform exponent
    __device__ __forceinline__ uint2 at(const uint2* psi, int r) const {
        constexpr uint32_t kBr4[16] = {0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15};
        uint32_t cs = c;
        asm volatile("" : "+s"(cs));
        uint32_t a;
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(a) : "s"(cs * (2048u * kBr4[r])), "v"(w));
        a &= 0x7fffu;
        return *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(psi) + a);
    }
};
static_assert(!MKACC_PSI_HI, "Mono3 assumes psi_pos permutes exponent bits 0..6 only");
__device__ __forceinline__ Mono3 make_mono3(uint32_t c, uint32_t l, uint32_t w) {
    const uint32_t o = ((__brev(l) >> 26) << 1) + (w << 7) + 1u;
    const uint32_t co = __umul24(c, o) & (2u * kN - 1u);
    return Mono3{psi_pos(co) << 3, c};
}

struct Ctx {
    const uint2* psi;     // HBM: psi^e - 1 pairs at psi_pos(e)
    const uint2* tw_fwd;
    const uint2* tw_inv;
    __amdgpu_buffer_rsrc_t rt;
    Mod m;
    SddConsts sd;
    Mono3 mp, mn;
    Lane ln;
    uint32_t vo;          // C4 byte offset of this lane: l * 16 + wave * 4 KiB
    __amdgpu_buffer_rsrc_t rin, rout, rk1, rk2, rks, rpk;
};

// key-stream shape: kGS slots per load group (C4: one dwordx4 per lane for 4), kPf in flight
template <int DG, int METHOD, bool FIRST>
struct Cfg {
    static constexpr bool kSplit = METHOD == XZW && !FIRST;
    static constexpr bool kK2 = METHOD == XZW;
#ifndef MKACC_S3_GS
#define MKACC_S3_GS 4
#endif
#ifndef MKACC_S3_PF
#define MKACC_S3_PF 1
#endif
    static constexpr int kGS = MKACC_S3_GS;
    static constexpr int kPf = MKACC_S3_PF;
    static constexpr int kGroups = kR / kGS;
    static constexpr int kBuf = kPf + 1;
    __device__ __forceinline__ static constexpr uint32_t soff(int g) {
        return (uint32_t)(((g * kGS) >> 2) * 1024 + ((g * kGS) & 3) * 4);
    }
    static constexpr int kG = DG > 4 ? 2 : 4;
    static_assert(2 + DG * kG <= 32, "step3 sum bound");
};
template <int DG, int METHOD, bool FIRST>
struct Grp {
    using C = Cfg<DG, METHOD, FIRST>;
    using V = typename VecLd<C::kGS>::T;
    V k1[DG];
    V k2[C::kK2 ? DG : 1];
    V ks[FIRST ? DG : 1];
    V pk[DG];
    V st;
};

// Streaming MAC of one pass (mac2 with this wave's 16 slots).
//   F = false (party u): keys d-half (2i), P[u][i]; start = acc_in[u]; out -> acc_out[u];
//                        sv <- redc(sv r32 + sum G P)   (svf = 0 for the first party)
//   F = true  (f-part):  keys f-half (2i + 1); start = acc_out[index]; out -> acc_out[index]
template <int DG, int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void mac(const Ctx& s, uint32_t u, const uint32_t (&G)[DG][kR], uint32_t (&sv)[kR],
                                    uint32_t svf) {
    using C = Cfg<DG, METHOD, FIRST>;
    using L = VecLd<C::kGS>;
    using Gp = Grp<DG, METHOD, FIRST>;
    const uint32_t Q = s.m.Q, polyB = kN * 4u, vo = s.vo;
    const uint32_t half = F ? polyB : 0u;
    const uint32_t uoff = u * polyB;
    const uint32_t poff = u * DG * polyB;
    auto issue = [&](Gp& t, int g) {
        const uint32_t so = C::soff(g);
#pragma unroll
        for (int i = 0; i < DG; ++i) {
            const uint32_t ko = (uint32_t)(2 * i) * polyB + half + so;
            t.k1[i] = L::ld(s.rk1, vo, ko);
            if (C::kK2) t.k2[i] = L::ld(s.rk2, vo, ko);
            if (FIRST) t.ks[i] = L::ld(s.rks, vo, ko);
            if (!F) t.pk[i] = L::ld(s.rpk, vo, poff + (uint32_t)i * polyB + so);
        }
        if (F) t.st = L::ld(s.rout, vo, uoff + so);
        else if (!FIRST) t.st = L::ld(s.rin, vo, uoff + so);
    };
    Gp kg[C::kBuf];
#pragma unroll
    for (int j = 0; j < C::kPf; ++j) issue(kg[j], j);
#pragma unroll
    for (int g = 0; g < C::kGroups; ++g) {
        if (g + C::kPf < C::kGroups) issue(kg[(g + C::kPf) % C::kBuf], g + C::kPf);
        const Gp& t = kg[g % C::kBuf];
        typename L::T ov;
#pragma unroll
        for (int e = 0; e < C::kGS; ++e) {
            const int r = g * C::kGS + e;
            uint64_t a1 = (F || !FIRST) ? mad64(t.st[e], s.m.r32, 0) : 0ull;
            uint64_t a2 = 0, sa = F ? 0ull : mad64(sv[r], svf, 0);
#pragma unroll
            for (int i = 0; i < DG; ++i) {
                if constexpr (C::kSplit) {
                    a1 = mad64(G[i][r], t.k1[i][e], a1);
                    a2 = mad64(G[i][r], t.k2[i][e], a2);
                } else {
                    const uint32_t ke = key_eff<METHOD, FIRST, 1>(t.k1[i][e], C::kK2 ? t.k2[i][e] : 0u,
                                                                 FIRST ? t.ks[i][e] : 0u, s.psi, s.mp, s.mn, r, Q);
                    a1 = mad64(G[i][r], ke, a1);
                }
                if (!F) sa = mad64(G[i][r], t.pk[i][e], sa);
            }
            uint32_t v = redc(a1, Q, s.m.qinv);                                       // [0, 2Q)
            if constexpr (C::kSplit) {
                v += mul_shoup_lazy(redc(a2, Q, s.m.qinv), s.mn.at(s.psi, r), Q);   // [0, 4Q)
                v = min(v, v - 2u * Q);
            }
            ov[e] = v;
            if (!F) sv[r] = redc(sa, Q, s.m.qinv);
        }
        L::st(ov, s.rout, vo, uoff + C::soff(g));
        sched_fence();
    }
    vcc_fence();   // the caller's branches follow the last reductions
}

// iNTT -> SDD -> dg forward NTTs: x (LC4, [0, 2Q)) -> G[i] = NTT(digit i + 1)
template <int DG>
__device__ __forceinline__ void digit_ntts(const Ctx& s, uint32_t (&x)[kR], uint32_t (&G)[DG][kR], uint32_t* bufs) {
    const uint32_t Q = s.m.Q;
    ntt_inv(x, bufs, s.tw_inv, s.rt, s.ln, Q);
    PackedDigits<DG, kR> pd;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
        G[0][r] = pd.put(r, sdd_offset(x[r], s.sd), s.sd);
        if ((r & 7) == 7) sched_fence();
    }
    ntt_fwd(G[0], bufs, s.tw_fwd, s.rt, s.ln, Q, s.m.m1);
    digit_range<DG>(G[0], Q);
#pragma unroll
    for (int i = 1; i < DG; ++i) {
#pragma unroll
        for (int r = 0; r < kR; ++r) G[i][r] = pd.get(r, i + 1, s.sd);
        ntt_fwd(G[i], bufs, s.tw_fwd, s.rt, s.ln, Q, s.m.m1);
        digit_range<DG>(G[i], Q);
    }
}

// waves per SIMD the register budget is sized for (launch bounds count waves per SIMD)
#ifndef MKACC_S3_WPS
#define MKACC_S3_WPS 2
#endif

}  // namespace s3

// One gate per 128-thread workgroup (two waves), grid = B.
template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(128, MKACC_S3_WPS) void mk_step3_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gate = blockIdx.x;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k, index = a.index;
    const uint32_t polyB = kN * 4u;
    const s3::Ctx s{reinterpret_cast<const uint2*>(a.img) + kPsm1Off,
                    a.tw_fwd,
                    a.tw_inv,
                    make_rsrc(a.tab3, lay2::kTabE * 8u),
                    a.m,
                    a.sd,
                    s3::make_mono3(c, l, wv),
                    // X^-c in the first step; X^(N-c) = -X^-c in the later XZW steps (key_eff)
                    s3::make_mono3(FIRST || METHOD != XZW ? cneg : (cneg + kN) & (2u * kN - 1u), l, wv),
                    lay2::Lane{l, wv, (wv * 64u + l) * 16u},
                    l * 16u + wv * 4096u,
                    make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB),
                    make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB),
                    make_rsrc(a.key1, DG * 2 * polyB),
                    make_rsrc(a.key2, DG * 2 * polyB),
                    make_rsrc(a.keys, DG * 2 * polyB),
                    make_rsrc(a.pkey, k * DG * polyB)};
    const uint32_t Q = s.m.Q;
    uint32_t sv[s3::kR];
#pragma unroll
    for (int r = 0; r < s3::kR; ++r) sv[r] = 0;
    // passes t = 0 .. k-1: parties index + 1, ..., index; t = k: the f-part of party index
#pragma unroll 1
    for (uint32_t t = 0; t <= k; ++t) {
        const bool fpart = __builtin_amdgcn_readfirstlane(t) == k;
        const uint32_t u = index + 1 + t < k ? index + 1 + t : index + 1 + t - k;
        uint32_t x[s3::kR];
        if (!fpart) {
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const u32x4 v = aload4(s.rin, s.vo, u * polyB + gq * 1024u);
                x[4 * gq] = v.x; x[4 * gq + 1] = v.y; x[4 * gq + 2] = v.z; x[4 * gq + 3] = v.w;
            }
            if (!FIRST) {
                // acctemp = acc * (X^c - 1)                 (xzw.cpp:336-338)
                uint2 mw[s3::kR];
#pragma unroll
                for (int r = 0; r < s3::kR; ++r) mw[r] = s.mp.at(s.psi, r);
                sched_fence();
#pragma unroll
                for (int r = 0; r < s3::kR; ++r) x[r] = mul_shoup_lazy(x[r], mw[r], Q);
                vcc_fence();
            }
        } else {
#pragma unroll
            for (int r = 0; r < s3::kR; ++r) x[r] = sv[r];
            // the index party's output (acc_out[index], this wave's own stores) is
            // read back by the f-part's MAC
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        vcc_fence();
        uint32_t G[DG][s3::kR];
        s3::digit_ntts<DG>(s, x, G, smem);
        vcc_fence();
        if (!fpart)
            s3::mac<DG, METHOD, FIRST, false>(s, u, G, sv, t == 0 ? 0u : s.m.r32);
        else
            s3::mac<DG, METHOD, FIRST, true>(s, index, G, sv, 0u);
    }
}

template <int DG>
StepFn pick_step3(int method, bool first) {
    if (method == XZW) return first ? mk_step3_kernel<DG, XZW, true> : mk_step3_kernel<DG, XZW, false>;
    return first ? mk_step3_kernel<DG, XZW_B, true> : mk_step3_kernel<DG, XZW_B, false>;
}
