// mkacc_step2.hpp -- the batch step kernel, round-3 form (mk_step2_kernel).
// Included inside mkacc_kernels.hpp's anonymous namespace.
//
// Same algebra as mk_step_kernel (HbProd, mk-acc-xzw.cpp:231-290, fused with
// AddToAccXZW{,0}, xzw.cpp:292-381; every sum exact mod Q, so bit-exact), but
// each of the k + 1 passes of a step runs its dg digit NTTs FIRST and keeps
// their outputs G_i in registers, then makes ONE streaming pass over the key
// words in which every slot's sums are short-lived temporaries:
//
//   party u:  G = NTT(SDD(iNTT(acc_u (X^c - 1))))
//             acc'_u = acc_u + sum_i G_i ev1'_i + (X^(N-c) - 1) sum_i G_i ev2_i
//             sv     = sv + sum_i G_i P[u][i]                 (32-bit between parties)
//   f-part:   G = NTT(SDD(iNTT(sv)))
//             acc'_index += sum_i G_i f1'_i + (X^(N-c) - 1) sum_i G_i f2_i
//
// Against mk_step_kernel this
//   * drops the 64-bit per-slot sums that lived across the digit NTTs
//     (uj and sumV: 128 VGPRs) for dg x 32 G registers, so the kernel runs
//     without spills and with deeper key prefetch;
//   * never forms d_i = ev1' + ev2 (X^(N-c) - 1) per slot and digit: the
//     monomial product is applied once per slot to the reduced ev2 sum (the
//     f-part's split form, now also for the parties): (dg - 1) fewer psi
//     gathers and Shoup products per slot and party, and no per-gate d_i
//     scratch at large k (mk_step_kernel DSCR);
//   * runs the parties and the f-part through ONE copy of the transform code
//     (k + 1 iterations of a rolled loop; the index party's output goes to
//     acc_out and the f-part reads it back), (dg + 1) NTTs of code instead of
//     2 (dg + 1) + 1.
// The first (KDM) step and XZW_B form the per-slot effective key inline
// (key_eff, one sum), as mk_step_kernel does.
#pragma once

template <int GS>
struct VecLd;
// cache policy of the accumulator stores (aux; 16 = sc1: the line leaves the XCD's L2,
// MI355X_MICROARCH.md, so the streamed outputs do not evict the inputs that the
// MAC reads a second time): HBM traffic 243 -> 223 MB per STD128_MKNTRU launch
// at unchanged time (profiles/r3/pmc_sc1.txt, ab_step2.txt)
constexpr int kS2StAux = 16;
template <>
struct VecLd<4> {
    using T = u32x4;
    __device__ __forceinline__ static T ld(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) { return bload4(r, vo, so); }
    __device__ __forceinline__ static T ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        return __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 16);
    }
    __device__ __forceinline__ static void st(T v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        __builtin_amdgcn_raw_buffer_store_b128(v, r, vo, so, kS2StAux);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 1");   // store-data hazard (bstore4)
        __builtin_amdgcn_sched_barrier(0);
    }
};
template <>
struct VecLd<2> {
    using T = u32x2;
    __device__ __forceinline__ static T ld(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) { return bload2(r, vo, so); }
    __device__ __forceinline__ static T ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        return __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 16);
    }
    // 8-byte stores carry no store-data hazard (bstore4)
    __device__ __forceinline__ static void st(T v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        __builtin_amdgcn_raw_buffer_store_b64(v, r, vo, so, kS2StAux);
    }
};

struct u32x1 {
    uint32_t v;
    __device__ __forceinline__ uint32_t operator[](int) const { return v; }
    __device__ __forceinline__ uint32_t& operator[](int) { return v; }
};
template <>
struct VecLd<1> {
    using T = u32x1;
    __device__ __forceinline__ static T ld(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        return T{__builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0)};
    }
    __device__ __forceinline__ static T ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        return T{__builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 16)};
    }
    __device__ __forceinline__ static void st(T v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        __builtin_amdgcn_raw_buffer_store_b32(v.v, r, vo, so, kS2StAux);
    }
};

// Key-stream shape of one pass.  kGS slots per load group (C4 layout: slot r of
// lane l at byte (r >> 2) * 1024 + l * 16 + (r & 3) * 4), kPf groups in flight.
// Measured and not kept (profiles/r3/ab_step2.txt, r4/ab_r4_v14.txt): 8-byte groups,
// no prefetch, the monomials gathered with the key loads, sumV in an HBM scratch, the
// next party's accumulator copied into LDS during the stream.
template <int DG, int METHOD, bool FIRST>
struct Step2Cfg {
    static_assert(DG <= 3, "mk_step2_kernel is built for dg <= 3 (dg >= 4: mk_step_kernel)");
    static constexpr bool kSplit = METHOD == XZW && !FIRST;   // two sums + one monomial product per slot
    static constexpr bool kK2 = METHOD == XZW;                // ev2 words needed
    static constexpr int kGS = 4;
    static constexpr int kPf = 1;                             // load groups in flight ahead of the one summed
    static constexpr int kGroups = kRegs / kGS;
    static constexpr int kBuf = kPf + 1;
    __device__ __forceinline__ static constexpr uint32_t soff(int g) {
        return (uint32_t)(((g * kGS) >> 2) * 1024 + ((g * kGS) & 3) * 4);
    }
    // redc bound (units of Q^2, below 32): digit-NTT outputs < kG Q, canonical keys,
    // plus a 32-bit start value in [0, 2Q) times 2^32 mod Q (< 2 Q^2)
    static constexpr int kG = DG > 4 ? 2 : 4;
    static_assert(2 + DG * kG <= 32, "step2 sum bound");
};

// One load group: the key words of kGS slots for every digit, the start value
// (previous accumulator / index party output) and the slots' X^(N-c) - 1.
template <int DG, int METHOD, bool FIRST>
struct Grp2 {
    using C = Step2Cfg<DG, METHOD, FIRST>;
    using V = typename VecLd<C::kGS>::T;
    V k1[DG];
    V k2[C::kK2 ? DG : 1];
    V ks[FIRST ? DG : 1];
    V pk[DG];
    V st;
};

// Streaming MAC of one pass over the step's key block.
//   F = false (party u): keys d-half of ev1'/ev2 (2i), P[u][i]; start = acc_in[u];
//                        out -> acc_out[u]; sv <- redc(sv r32 + sum G P)
//   F = true  (f-part):  keys f-half (2i + 1); start = acc_out[index] (the index
//                        party's output); out -> acc_out[index]
template <int DG, int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void mac2(const StepCtx& s, uint32_t u, const uint32_t (&G)[DG][kRegs],
                                     uint32_t (&sv)[kRegs]) {
    using C = Step2Cfg<DG, METHOD, FIRST>;
    using L = VecLd<C::kGS>;
    using Grp = Grp2<DG, METHOD, FIRST>;
    const uint32_t Q = s.m.Q, polyB = kN * 4u, vo = s.vo;
    const uint32_t half = F ? polyB : 0u;           // f-half of each digit's key pair
    const uint32_t uoff = u * polyB;
    const uint32_t poff = u * DG * polyB;
    auto issue = [&](Grp& t, int g) {
        const uint32_t so = C::soff(g);
#pragma unroll
        for (int i = 0; i < DG; ++i) {
            const uint32_t ko = (uint32_t)(2 * i) * polyB + half + so;
            t.k1[i] = L::ld(s.rk1, vo, ko);
            if (C::kK2) t.k2[i] = L::ld(s.rk2, vo, ko);
            if (FIRST) t.ks[i] = L::ld(s.rks, vo, ko);
            if (!F) t.pk[i] = L::ld(s.rpk, vo, poff + (uint32_t)i * polyB + so);
        }
        // party: acc_u (not in the first step, which overwrites acc); f-part: the
        // index party's output, written by this wave earlier in the step
        if (F) t.st = L::ld(s.rout, vo, uoff + so);
        else if (!FIRST) t.st = L::ld(s.rin, vo, uoff + so);
    };
    Grp kg[C::kBuf];
#pragma unroll
    for (int j = 0; j < C::kPf; ++j) issue(kg[j], j);
#pragma unroll
    for (int g = 0; g < C::kGroups; ++g) {
        if (g + C::kPf < C::kGroups) issue(kg[(g + C::kPf) % C::kBuf], g + C::kPf);
        const Grp& t = kg[g % C::kBuf];
        typename L::T ov;
#pragma unroll
        for (int e = 0; e < C::kGS; ++e) {
            const int r = g * C::kGS + e;
            uint64_t a1 = (F || !FIRST) ? mad64(t.st[e], s.m.r32, 0) : 0ull;
            uint64_t a2 = 0, sa = F ? 0ull : mad64(sv[r], s.m.r32, 0);
#pragma unroll
            for (int i = 0; i < DG; ++i) {
                if constexpr (C::kSplit) {
                    a1 = mad64(G[i][r], t.k1[i][e], a1);
                    a2 = mad64(G[i][r], t.k2[i][e], a2);
                } else {
                    const uint32_t ke = key_eff<METHOD, FIRST, 1>(t.k1[i][e], C::kK2 ? t.k2[i][e] : 0u,
                                                                 FIRST ? t.ks[i][e] : 0u, s.tb.psi, s.mp, s.mn, r, Q);
                    a1 = mad64(G[i][r], ke, a1);
                }
                if (!F) sa = mad64(G[i][r], t.pk[i][e], sa);
            }
            uint32_t v = redc(a1, Q, s.m.qinv);                                       // [0, 2Q)
            if constexpr (C::kSplit) {
                v += mul_shoup_lazy(redc(a2, Q, s.m.qinv), s.mn.at(s.tb.psi, r), Q);   // [0, 4Q)
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

// digits I .. DG - 1 (unrolled by recursion: an unroll pragma over two whole
// transforms is dropped when the body passes the unroller's threshold, and a G[i]
// with a run-time i puts the whole G array in scratch memory)
template <int DG, int I>
__device__ __forceinline__ void digit_ntts_from(const StepCtx& s, const PackedDigits<DG>& pd,
                                                uint32_t (&G)[DG][kRegs]) {
    if constexpr (I < DG) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) G[I][r] = pd.get(r, I + 1, s.sd);
        ntt_fwd(G[I], s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, s.m.Q, s.m.m1);
        digit_range<DG>(G[I], s.m.Q);
        digit_ntts_from<DG, I + 1>(s, pd, G);
    }
}

// iNTT -> SDD -> dg forward NTTs: x (layout C, [0, 2Q)) -> G[i] = NTT(digit i + 1)
template <int DG>
__device__ __forceinline__ void digit_ntts(const StepCtx& s, uint32_t (&x)[kRegs], uint32_t (&G)[DG][kRegs]) {
    const uint32_t Q = s.m.Q;
    ntt_inv(x, s.lds, s.tw_inv, s.tb.twi, s.l, Q);
    // SignedDigitDecompose (mk-acc.cpp:54-80): digit 1 -> G[0], digits 2.. packed
    PackedDigits<DG> pd;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        G[0][r] = pd.put(r, sdd_offset(x[r], s.sd), s.sd);
        if ((r & 7) == 7) sched_fence();
    }
    ntt_fwd(G[0], s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
    digit_range<DG>(G[0], Q);
    digit_ntts_from<DG, 1>(s, pd, G);
}

// two waves per SIMD (256 VGPRs): two 4-wave workgroups per CU
template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(64 * kS2Waves, 2) void mk_step2_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    load_image(smem, a.img);
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gate = blockIdx.x * kS2Waves + wv;
    if (gate >= a.B) return;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k, index = a.index;
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
                    make_rsrc(a.acc_in, 0u)};
    const uint32_t Q = s.m.Q;
    uint32_t sv[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) sv[r] = 0;
    // passes t = 0 .. k-1: party t; t = k: the f-part of party `index`
    // (prefetching the next party's accumulator in the previous pass's stream kept
    // 32 more VGPRs live: 53 spills, 206 us per launch against 168)
    // Parties in the order index + 1, ..., index: the index party's output, read back
    // by the f-part, is written last (shortest time in L2)
#pragma unroll 1
    for (uint32_t t = 0; t <= k; ++t) {
        const bool fpart = __builtin_amdgcn_readfirstlane(t) == k;
        const uint32_t u = index + 1 + t < k ? index + 1 + t : index + 1 + t - k;
        uint32_t x[kRegs];
        if (!fpart) {
#pragma unroll
            for (int gq = 0; gq < 8; ++gq) {
                const u32x4 v = aload4(s.rin, s.vo, u * polyB + gq * 1024u);
                x[4 * gq] = v.x; x[4 * gq + 1] = v.y; x[4 * gq + 2] = v.z; x[4 * gq + 3] = v.w;
            }
            if (!FIRST) {
                // acctemp = acc * (X^c - 1)                 (xzw.cpp:336-338)
                uint2 mw[kRegs];
#pragma unroll
                for (int r = 0; r < kRegs; ++r) mw[r] = s.mp.at(s.tb.psi, r);
                sched_fence();
#pragma unroll
                for (int r = 0; r < kRegs; ++r) x[r] = mul_shoup_lazy(x[r], mw[r], Q);
                vcc_fence();   // the jump over the f-part branch follows the rotation
            }
        } else {
            // sumV of every party, [0, 2Q)
#pragma unroll
            for (int r = 0; r < kRegs; ++r) x[r] = sv[r];
            // the index party's output (acc_out[index], this wave's own stores) is
            // read back by the f-part's MAC
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        vcc_fence();   // the branch above follows the rotation's multiply-adds
        uint32_t G[DG][kRegs];
        digit_ntts<DG>(s, x, G);
        vcc_fence();   // the MAC branch follows the last butterflies
        if (!fpart)
            mac2<DG, METHOD, FIRST, false>(s, u, G, sv);
        else
            mac2<DG, METHOD, FIRST, true>(s, index, G, sv);
        // the f-part is the last pass: no back edge from it, so nothing a party
        // pass leaves for the next one (xn) is live across the f-part's transforms
        if (fpart) break;
    }
}
