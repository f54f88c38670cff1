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
#ifndef MKACC_S2_STAUX
#define MKACC_S2_STAUX 16
#endif
template <>
struct VecLd<4> {
    using T = u32x4;
    __device__ __forceinline__ static T ld(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) { return bload4(r, vo, so); }
    __device__ __forceinline__ static T ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        return __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 16);
    }
    __device__ __forceinline__ static void st(T v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        __builtin_amdgcn_raw_buffer_store_b128(v, r, vo, so, MKACC_S2_STAUX);
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
        __builtin_amdgcn_raw_buffer_store_b64(v, r, vo, so, MKACC_S2_STAUX);
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
        __builtin_amdgcn_raw_buffer_store_b32(v.v, r, vo, so, MKACC_S2_STAUX);
    }
};

// MKACC_S2_NXPF / MKACC_S2_NXAT: the accumulator copy of mac2 (below)
#ifndef MKACC_S2_NXPF
#define MKACC_S2_NXPF 0
#endif
#ifndef MKACC_S2_NXAT
#define MKACC_S2_NXAT 5
#endif

// Key-stream shape of one pass.  kGS slots per load group (C4 layout: slot r of
// lane l at byte (r >> 2) * 1024 + l * 16 + (r & 3) * 4), kPf groups in flight.
template <int DG, int METHOD, bool FIRST>
struct Step2Cfg {
    static constexpr bool kSplit = METHOD == XZW && !FIRST;   // two sums + one monomial product per slot
    static constexpr bool kK2 = METHOD == XZW;                // ev2 words needed
#ifndef MKACC_S2_GS
#define MKACC_S2_GS 0
#endif
    static constexpr int kGS = MKACC_S2_GS ? MKACC_S2_GS : 4;
    // load groups in flight ahead of the one being summed: 1 at dg <= 3; at dg >= 4
    // the 4 x 32 G registers need the whole 512-entry file (one wave per SIMD,
    // kWavesPerSimd), which leaves room for two
#ifndef MKACC_S2_PF
#define MKACC_S2_PF -1
#endif
    static constexpr int kPf = MKACC_S2_PF >= 0 ? MKACC_S2_PF : (DG <= 3 ? 1 : 2);
    // X^(N-c) - 1 gathered with the group's key loads (1) or at use (0)
#ifndef MKACC_S2_MONO
#define MKACC_S2_MONO 0
#endif
    static constexpr bool kMonoPf = kSplit && MKACC_S2_MONO;
    // sumV between the party passes: in the gate's HBM scratch (StepArgs::dscr),
    // streamed in with the keys, instead of 32 VGPRs live across every transform
#ifndef MKACC_S2_SVMEM
#define MKACC_S2_SVMEM 0
#endif
    static constexpr bool kSvMem = MKACC_S2_SVMEM;

    static constexpr int kGroups = kRegs / kGS;
    static constexpr int kBuf = kPf + 1;
    __device__ __forceinline__ static constexpr uint32_t soff(int g) {
        return (uint32_t)(((g * kGS) >> 2) * 1024 + ((g * kGS) & 3) * 4);
    }
    // MKACC_S2_NXPF: vector memory ops a party stream issues after its accumulator copies
    // (group MKACC_S2_NXAT): that group's store, then per later group its key loads
    // (if any) and its store
    static constexpr int kLoadsPerGroup = DG * (1 + (kK2 ? 1 : 0) + (FIRST ? 1 : 0) + 1) + (FIRST ? 0 : 1) +
                                          (kSvMem ? 1 : 0);
    static constexpr int young() {
        int n = 1 + (kSvMem ? 1 : 0);
        for (int g = MKACC_S2_NXAT + 1; g < kGroups; ++g) n += (g + kPf < kGroups ? kLoadsPerGroup : 0) + 1 + (kSvMem ? 1 : 0);
        return n;
    }
    static constexpr int kNxYoung = young();
    static_assert(!MKACC_S2_NXPF || (MKACC_S2_NXAT < kGroups && kNxYoung <= 63), "accumulator copy placement");
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
    V sv;   // kSvMem: sumV of the earlier parties
    uint2 mono[C::kMonoPf ? C::kGS : 1];
};

// Streaming MAC of one pass over the step's key block.
//   F = false (party u): keys d-half of ev1'/ev2 (2i), P[u][i]; start = acc_in[u];
//                        out -> acc_out[u]; sv <- redc(sv r32 + sum G P)
//                        (kSvMem: the earlier parties' sv is read from the gate's
//                        scratch, scaled by svf = 0 for the first party, r32 after;
//                        sv is returned in registers and also stored)
//   F = true  (f-part):  keys f-half (2i + 1); start = acc_out[index] (the index
//                        party's output); out -> acc_out[index]
// MKACC_S2_NXPF=1 (A/B): a party pass also copies the NEXT pass's accumulator (party
// nu) from HBM straight into the wave's LDS transpose scratch (idle during the key
// stream) with direct-to-LDS buffer loads, so the next pass reads it from LDS instead
// of starting with an exposed HBM load, and no VGPR is spent (prefetching it into
// registers spilled 53-60 VGPRs).  The last party reloads its own, L2-resident, words
// (no branch in the stream); every pass waits for the copies before its first transform.
template <int DG, int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void mac2(const StepCtx& s, uint32_t u, const uint32_t (&G)[DG][kRegs],
                                     uint32_t (&sv)[kRegs], uint32_t svf = 0, uint32_t nu = 0) {
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
        if (!F && C::kSvMem) t.sv = L::ld(s.rds, vo, so);
        if (C::kMonoPf) {
#pragma unroll
            for (int e = 0; e < C::kGS; ++e) t.mono[e] = s.mn.at(s.tb.psi, g * C::kGS + e);
        }
    };
    Grp kg[C::kBuf];
#pragma unroll
    for (int j = 0; j < C::kPf; ++j) issue(kg[j], j);
#pragma unroll
    for (int g = 0; g < C::kGroups; ++g) {
        if (g + C::kPf < C::kGroups) issue(kg[(g + C::kPf) % C::kBuf], g + C::kPf);
        if (MKACC_S2_NXPF && !F && g == MKACC_S2_NXAT) {
#pragma unroll
            for (int gq = 0; gq < 8; ++gq)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    s.rin, (__attribute__((address_space(3))) void*)(s.lds + gq * 256), 16, vo,
                    nu * polyB + gq * 1024u, 0, 0);
        }
        const Grp& t = kg[g % C::kBuf];
        typename L::T ov;
#pragma unroll
        for (int e = 0; e < C::kGS; ++e) {
            const int r = g * C::kGS + e;
            uint64_t a1 = (F || !FIRST) ? mad64(t.st[e], s.m.r32, 0) : 0ull;
            uint64_t a2 = 0, sa = F ? 0ull : mad64(C::kSvMem ? t.sv[e] : sv[r], C::kSvMem ? svf : s.m.r32, 0);
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
                const uint2 mo = C::kMonoPf ? t.mono[e] : s.mn.at(s.tb.psi, r);
                v += mul_shoup_lazy(redc(a2, Q, s.m.qinv), mo, Q);                  // [0, 4Q)
                v = min(v, v - 2u * Q);
            }
            ov[e] = v;
            if (!F) sv[r] = redc(sa, Q, s.m.qinv);
        }
        L::st(ov, s.rout, vo, uoff + C::soff(g));
        if (!F && C::kSvMem) {   // (also after the last party: no branch in the stream)
            typename L::T sw;
#pragma unroll
            for (int e = 0; e < C::kGS; ++e) sw[e] = sv[g * C::kGS + e];
            L::st(sw, s.rds, vo, C::soff(g));
        }
#ifndef MKACC_S2_FENCE
#define MKACC_S2_FENCE 1
#endif
        if (MKACC_S2_FENCE) sched_fence();
    }
    vcc_fence();   // the caller's branches follow the last reductions
}

// ---- dg = 4 in two halves (config 4, STD128_MKNTRU_3) ----------------------------
// The 4 x 32 digit-NTT registers of the one-stream form need the whole register
// file (one wave per SIMD, 1.46 ms per launch against 1.19 ms for mk_step_kernel).
// Two streams of two digits each keep 2 x 32 G registers and two waves per SIMD:
//   half 0: G = NTT(digits 1, 2); a1 = start + sum G ev1', a2 = sum G ev2 (split form)
//           -> p1 = redc(a1) into acc_out[u], p2 = redc(a2) into the gate's scratch
//   half 1: G = NTT(digits 3, 4); a1 = p1 r32 + sum G ev1', a2 = p2 r32 + sum G ev2
//           -> acc_out[u] = redc(a1) + (X^(N-c) - 1) redc(a2)
// sumV is reduced after each stream as in mac2.  Same sums mod Q, so bit-exact.
#ifndef MKACC_S2_HALVES
#define MKACC_S2_HALVES 1
#endif
template <int DG>
constexpr bool s2_halves() { return DG == 4 && MKACC_S2_HALVES; }

template <int METHOD, bool FIRST>
struct HalfCfg {
    static constexpr bool kSplit = METHOD == XZW && !FIRST;
    static constexpr bool kK2 = METHOD == XZW;
#ifndef MKACC_S2H_GS
#define MKACC_S2H_GS 2
#endif
#ifndef MKACC_S2H_PF
#define MKACC_S2H_PF 2
#endif
    static constexpr int kGS = MKACC_S2H_GS;
    static constexpr int kPf = MKACC_S2H_PF;
    static constexpr int kGroups = kRegs / kGS;
    static constexpr int kBuf = kPf + 1;
    __device__ __forceinline__ static constexpr uint32_t soff(int g) {
        return (uint32_t)(((g * kGS) >> 2) * 1024 + ((g * kGS) & 3) * 4);
    }
};
template <int METHOD, bool FIRST>
struct GrpH {
    using L = VecLd<HalfCfg<METHOD, FIRST>::kGS>;
    using V = typename L::T;
    V k1[2];
    V k2[HalfCfg<METHOD, FIRST>::kK2 ? 2 : 1];
    V ks[FIRST ? 2 : 1];
    V pk[2];
    V st, st2;
};

__device__ __forceinline__ void hstore(u32x4 v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) { bstore4(v, r, vo, so); }
__device__ __forceinline__ void hstore(u32x2 v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
    __builtin_amdgcn_raw_buffer_store_b64(v, r, vo, so, 0);
}
__device__ __forceinline__ void hstore(u32x1 v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
    __builtin_amdgcn_raw_buffer_store_b32(v.v, r, vo, so, 0);
}
// One stream of half H (digits 2H + 1, 2H + 2) of party u (F = false) or the f-part (F = true).
template <int METHOD, bool FIRST, bool F, int H>
__device__ __forceinline__ void mac2h(const StepCtx& s, uint32_t u, const uint32_t (&G)[2][kRegs],
                                      uint32_t (&sv)[kRegs]) {
    using C = HalfCfg<METHOD, FIRST>;
    using Grp = GrpH<METHOD, FIRST>;
    using L = typename Grp::L;
    const uint32_t Q = s.m.Q, polyB = kN * 4u, vo = s.vo;
    const uint32_t half = F ? polyB : 0u;
    const uint32_t uoff = u * polyB;
    const uint32_t poff = (u * 4u + 2u * H) * polyB;
    // start value: half 0 -- acc_u (party; none in the first step, which overwrites
    // acc) or the index party's output (f-part); half 1 -- the parked p1 (+ p2)
    constexpr bool kStart = H == 1 || F || !FIRST;
    auto issue = [&](Grp& t, int g) {
        const uint32_t so = C::soff(g);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t ko = (uint32_t)(2 * (2 * H + j)) * polyB + half + so;
            t.k1[j] = L::ld(s.rk1, vo, ko);
            if (C::kK2) t.k2[j] = L::ld(s.rk2, vo, ko);
            if (FIRST) t.ks[j] = L::ld(s.rks, vo, ko);
            if (!F) t.pk[j] = L::ld(s.rpk, vo, poff + (uint32_t)j * polyB + so);
        }
        // this wave's own earlier stores are read back L1-bypassing (sc1): p1 / p2 are
        // rewritten every pass, and acc_out[index] is read as p1 before the f-part reads
        // it again, so correctness does not rest on the vector L1's write policy.  (The
        // 4-slot-group build's 14 of 16 wrong gates at full size were a store-data
        // hazard instead: under its 60+ spilled VGPRs the register allocator put a copy
        // into a dwordx4 store's data registers ahead of bstore4's s_nop -- found by
        // tools/isa_audit.py, which tools/build_variant.sh now runs on every variant.)
        if (kStart) t.st = (H == 1 || F) ? L::ld_sc1(s.rout, vo, uoff + so) : L::ld(s.rin, vo, uoff + so);
        if (H == 1 && C::kSplit) t.st2 = L::ld_sc1(s.rds, vo, so);
    };
    Grp kg[C::kBuf];
#pragma unroll
    for (int j = 0; j < C::kPf; ++j) issue(kg[j], j);
#pragma unroll
    for (int g = 0; g < C::kGroups; ++g) {
        if (g + C::kPf < C::kGroups) issue(kg[(g + C::kPf) % C::kBuf], g + C::kPf);
        const Grp& t = kg[g % C::kBuf];
        typename L::T ov, o2;
#pragma unroll
        for (int e = 0; e < C::kGS; ++e) {
            const int r = g * C::kGS + e;
            uint64_t a1 = kStart ? mad64(t.st[e], s.m.r32, 0) : 0ull;
            uint64_t a2 = (H == 1 && C::kSplit) ? mad64(t.st2[e], s.m.r32, 0) : 0ull;
            uint64_t sa = F ? 0ull : mad64(sv[r], s.m.r32, 0);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if constexpr (C::kSplit) {
                    a1 = mad64(G[j][r], t.k1[j][e], a1);
                    a2 = mad64(G[j][r], t.k2[j][e], a2);
                } else {
                    const uint32_t ke = key_eff<METHOD, FIRST, 1>(t.k1[j][e], C::kK2 ? t.k2[j][e] : 0u,
                                                                 FIRST ? t.ks[j][e] : 0u, s.tb.psi, s.mp, s.mn, r, Q);
                    a1 = mad64(G[j][r], ke, a1);
                }
                if (!F) sa = mad64(G[j][r], t.pk[j][e], sa);
            }
            uint32_t v = redc(a1, Q, s.m.qinv);                                   // [0, 2Q)
            if constexpr (C::kSplit) {
                const uint32_t v2 = redc(a2, Q, s.m.qinv);                        // [0, 2Q)
                if (H == 0) {
                    o2[e] = v2;                                                   // parked p2
                } else {
                    v += mul_shoup_lazy(v2, s.mn.at(s.tb.psi, r), Q);             // [0, 4Q)
                    v = min(v, v - 2u * Q);
                }
            }
            ov[e] = v;
            if (!F) sv[r] = redc(sa, Q, s.m.qinv);
        }
        // default write policy for the parked p1 / p2 (read back by this wave after
        // two digit NTTs); VecLd::st's L2-bypassing policy for the final outputs
        if (H == 0) {
            hstore(ov, s.rout, vo, uoff + C::soff(g));
            if (C::kSplit) hstore(o2, s.rds, vo, C::soff(g));
        } else {
            L::st(ov, s.rout, vo, uoff + C::soff(g));
        }
        sched_fence();
    }
    vcc_fence();
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
#pragma unroll
    for (int i = 1; i < DG; ++i) {
#pragma unroll
        for (int r = 0; r < kRegs; ++r) G[i][r] = pd.get(r, i + 1, s.sd);
        ntt_fwd(G[i], s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
        digit_range<DG>(G[i], Q);
    }
}

// waves per SIMD the register budget is sized for: 2 (256 VGPRs) at dg <= 3;
// 1 at dg >= 4 (512: the dg x 32 digit-NTT registers, the sumV and the key prefetch)
template <int DG>
constexpr int s2_waves_per_simd() {
#ifdef MKACC_S2_WPS
    return MKACC_S2_WPS;
#else
    return DG <= 3 || s2_halves<DG>() ? 2 : 1;
#endif
}
template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(64 * kS2Waves, 4 * s2_waves_per_simd<DG>() / kS2Waves) void mk_step2_kernel(StepArgs a) {
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
                    make_rsrc(Step2Cfg<DG, METHOD, FIRST>::kSvMem || s2_halves<DG>() ? a.dscr + (size_t)gate * kN
                                                                                    : a.acc_in,
                              Step2Cfg<DG, METHOD, FIRST>::kSvMem || s2_halves<DG>() ? polyB : 0u)};
    const uint32_t Q = s.m.Q;
    uint32_t sv[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) sv[r] = 0;
    // passes t = 0 .. k-1: party t; t = k: the f-part of party `index`
    // (prefetching the next party's accumulator in the previous pass's stream kept
    // 32 more VGPRs live: 53 spills, 206 us per launch against 168)
    // Parties in the order index + 1, ..., index (MKACC_S2_ORDER=1): the index
    // party's output, read back by the f-part, is written last (shortest time in L2)
#ifndef MKACC_S2_ORDER
#define MKACC_S2_ORDER 1
#endif
#pragma unroll 1
    for (uint32_t t = 0; t <= k; ++t) {
        const bool fpart = __builtin_amdgcn_readfirstlane(t) == k;
        const uint32_t u = MKACC_S2_ORDER ? (index + 1 + t < k ? index + 1 + t : index + 1 + t - k) : t;
        uint32_t x[kRegs];
        if (!fpart) {
            if (MKACC_S2_NXPF && !s2_halves<DG>() && t > 0) {
                // copied into this wave's scratch by the previous pass's stream (C4 order):
                // wait for those copies only -- the stream issued kNxYoung memory ops after them
                // (vector memory returns in issue order).  The reads are inline asm: for a
                // compiled LDS read after LDS-DMA writes hipcc inserts s_waitcnt vmcnt(0),
                // i.e. waits for every store of the previous stream as well.
                // (the lane term recomputed here, opaque to hoisting: a loop-invariant address
                // kept live across the pass was the one VGPR the kernel spilled)
                const uint32_t la = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)(s.lds) + opaque_v(s.l) * 16u;
                u32x4 v0, v1, v2, v3, v4, v5, v6, v7;
                asm volatile(
                    "s_waitcnt vmcnt(%8)\n\t"
                    "ds_read_b128 %0, %9\n\t"
                    "ds_read_b128 %1, %9 offset:1024\n\t"
                    "ds_read_b128 %2, %9 offset:2048\n\t"
                    "ds_read_b128 %3, %9 offset:3072\n\t"
                    "ds_read_b128 %4, %9 offset:4096\n\t"
                    "ds_read_b128 %5, %9 offset:5120\n\t"
                    "ds_read_b128 %6, %9 offset:6144\n\t"
                    "ds_read_b128 %7, %9 offset:7168\n\t"
                    "s_waitcnt lgkmcnt(0)"
                    : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(v4), "=&v"(v5), "=&v"(v6), "=&v"(v7)
                    : "n"(Step2Cfg<DG, METHOD, FIRST>::kNxYoung), "v"(la)
                    : "memory");
                const u32x4 vv[8] = {v0, v1, v2, v3, v4, v5, v6, v7};
#pragma unroll
                for (int gq = 0; gq < 8; ++gq) {
                    x[4 * gq] = vv[gq].x; x[4 * gq + 1] = vv[gq].y; x[4 * gq + 2] = vv[gq].z; x[4 * gq + 3] = vv[gq].w;
                }
            } else {
#pragma unroll
                for (int gq = 0; gq < 8; ++gq) {
                    const u32x4 v = aload4(s.rin, s.vo, u * polyB + gq * 1024u);
                    x[4 * gq] = v.x; x[4 * gq + 1] = v.y; x[4 * gq + 2] = v.z; x[4 * gq + 3] = v.w;
                }
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
        if constexpr (s2_halves<DG>()) {
            const uint32_t Q = s.m.Q;
            ntt_inv(x, s.lds, s.tw_inv, s.tb.twi, s.l, Q);
            PackedDigits<DG> pd;
            uint32_t G[2][kRegs];
#pragma unroll
            for (int r = 0; r < kRegs; ++r) {
                G[0][r] = pd.put(r, sdd_offset(x[r], s.sd), s.sd);
                if ((r & 7) == 7) sched_fence();
            }
            ntt_fwd(G[0], s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
#pragma unroll
            for (int r = 0; r < kRegs; ++r) G[1][r] = pd.get(r, 2, s.sd);
            ntt_fwd(G[1], s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
            vcc_fence();
            if (!fpart)
                mac2h<METHOD, FIRST, false, 0>(s, u, G, sv);
            else
                mac2h<METHOD, FIRST, true, 0>(s, index, G, sv);
#pragma unroll
            for (int r = 0; r < kRegs; ++r) G[0][r] = pd.get(r, 3, s.sd);
            ntt_fwd(G[0], s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
#pragma unroll
            for (int r = 0; r < kRegs; ++r) G[1][r] = pd.get(r, 4, s.sd);
            ntt_fwd(G[1], s.lds, s.tw_fwd, s.tb.twf, s.tb.twfc, s.l, Q, s.m.m1);
            vcc_fence();
            // the parked p1 / p2 of this wave are read back in the next stream
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (!fpart)
                mac2h<METHOD, FIRST, false, 1>(s, u, G, sv);
            else
                mac2h<METHOD, FIRST, true, 1>(s, index, G, sv);
        } else {
            uint32_t G[DG][kRegs];
            digit_ntts<DG>(s, x, G);
            vcc_fence();   // the MAC branch follows the last butterflies
            // next pass: party u + 1 (mod k), or u itself after the last party (unused)
            const uint32_t nu = t + 1 < k ? (u + 1 < k ? u + 1 : 0u) : u;
            if (!fpart)
                mac2<DG, METHOD, FIRST, false>(s, u, G, sv, t == 0 ? 0u : s.m.r32, nu);
            else
                mac2<DG, METHOD, FIRST, true>(s, index, G, sv);
        }
        // the f-part is the last pass: no back edge from it, so nothing a party
        // pass leaves for the next one (xn) is live across the f-part's transforms
        if (fpart) break;
    }
}
