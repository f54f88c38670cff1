// mkacc_quad.hpp -- small batches, one gate per workgroup with every ring polynomial
// spread over the workgroup's four waves (mk_quad_kernel).  Included inside
// mkacc_kernels.hpp's anonymous namespace, after mkacc_step2.hpp.
//
// The split-digit kernel (mk_latd_kernel) gives each wave a whole polynomial, so a
// step's critical path is ceil(dg/2) + 3 transforms run by one wave per SIMD -- and
// one wave per SIMD issues a dependent VALU op every ~10 cycles and v_mad_u64_u32
// every ~8.5 (tools/ubench_lat.hip, profiles/r6/v4_ubench_lat.txt), so a transform
// takes ~3 us.  Here wave q of the gate's workgroup holds residues
// j = f(q, lane, r), 8 per lane, of EVERY polynomial of the step, and all four waves
// run the whole step together with mk_step2_kernel's algebra (HbProd,
// mk-acc-xzw.cpp:231-290, fused with AddToAccXZW{,0}, xzw.cpp:292-381):
//
//   party u:  G = NTT(SDD(iNTT(acc_u (X^c - 1))))
//             acc'_u = acc_u + sum_i G_i ev1'_i + (X^(N-c) - 1) sum_i G_i ev2_i
//             sv     = sv + sum_i G_i P[u][i]
//   f-part:   G = NTT(SDD(iNTT(sv)));  acc'_index += sum_i G_i f1'_i + (X^(N-c) - 1) sum_i G_i f2_i
//
// The (k + 1)(dg + 1) transforms of a step are each a quarter per wave (no transform
// is repeated, no wave idles), every per-slot sum is wave-local (a wave owns the same
// EVAL slots of every polynomial), and the only cross-wave traffic is one LDS exchange
// with one workgroup barrier per transform.  All sums are exact mod Q: bit-exact with
// the other kernels.
//
// Layouts (j = coefficient / EVAL index, bits listed MSB first; tools/quad_model.py
// runs the transforms through them in exact integers against the oracle):
//   QA  reg 10,9,8   wave 1,0   lane 7..2          coefficients (inverse out, forward in)
//   QB  reg 7,6,5    wave 1,0   lane 10,9,8,4,3,2
//   QC  reg 4,3,2    wave 1,0   lane 10..5
//   QD  reg 2,1,0    wave 4,3   lane 10..5         EVAL slots: j = lane << 5 | wave << 3 | r
//   IB  reg 5,4,3    wave 1,0   lane 10..6,2
//   IC  reg 8,7,6    wave 1,0   lane 10,9,5..2
// Forward (CT, bits 10 -> 0): QA [10,9,8] -> QB [7,6,5] -> QC [4,3,2] =x=> QD [1,0].
// Inverse (DIT, bits 0 -> 10, then psi^-i): QD [0,1,2] =x=> IB [3,4,5] -> IC [6,7,8] -> QA [9,10].
// "->" is a wave-local LDS transpose (wave bits unchanged), "=x=>" the cross-wave
// exchange (ping-pong buffers, one barrier).  In QD a wave's slots are C4 groups
// 2q, 2q + 1 of every lane: the key and accumulator streams are 1 KiB per load.
#pragma once

#ifndef MKACC_QUAD_KEEP
// the same in the one-workgroup-per-gate kernels (quad_step): +1.1 % at B = 256, +1.4 %
// for the two-per-CU form at B = 1024 (profiles/r6/v37)
#define MKACC_QUAD_KEEP 1
#endif
#ifndef MKACC_QUADP_KEEP
// 1: the party-parallel kernel keeps the index party's pass output in registers for the
// f-part (no store and reload through acc_out on the critical path): -2.2 % for one
// STD128_MKNTRU gate, -1.6 % at B = 128 (profiles/r6/v36)
#define MKACC_QUADP_KEEP 1
#endif
#ifndef MKACC_QUAD_PF
#define MKACC_QUAD_PF 1   // the MAC's key groups issued at the start of the pass (before its transforms)
#endif

namespace quad {

constexpr int kR = 8;                // residues per lane
constexpr uint32_t kWaves = 4;

// ---- layouts and LDS maps --------------------------------------------------------
enum { QA = 0, QB, QC, QD, IB, IC };
struct Lay {
    int r[3], w[2], l[6];
};
__host__ __device__ constexpr Lay lay(int id) {
    return id == QA   ? Lay{{10, 9, 8}, {1, 0}, {7, 6, 5, 4, 3, 2}}
           : id == QB ? Lay{{7, 6, 5}, {1, 0}, {10, 9, 8, 4, 3, 2}}
           : id == QC ? Lay{{4, 3, 2}, {1, 0}, {10, 9, 8, 7, 6, 5}}
           : id == QD ? Lay{{2, 1, 0}, {4, 3}, {10, 9, 8, 7, 6, 5}}
           : id == IB ? Lay{{5, 4, 3}, {1, 0}, {10, 9, 8, 7, 6, 2}}
                      : Lay{{8, 7, 6}, {1, 0}, {10, 9, 5, 4, 3, 2}};
}
// LDS word maps, additive in the bits of j (so a register's word is the lane's base plus
// an immediate): word(j) = sum_k W[k] bit_k(j).  Intra-wave maps act on j >> 2 inside the
// wave's own region (wave bits 1, 0 weigh 0).  Half-wave bank multiplicity of each
// exchange's write / read (tools/quad_model.py): QA->QB 2/1, QB->QC 1/1, IB->IC 1/2,
// IC->QA 1/1 (intra), QC->QD 1/1, QD->IB 1/2 (cross).
enum { MI3 = 0, MICA, MX5 };
__host__ __device__ constexpr uint32_t wgt(int map, int k) {
    if (map == MX5) return (1u << k) + (k >= 5 ? 1u << (k - 5) : 0u);   // j + (j >> 5)
    if (k < 2) return 0u;
    const int b = k - 2;                                             // bit of j >> 2
    if (map == MI3) return (1u << b) + (b >= 3 ? 1u << (b - 3) : 0u);   // j' + (j' >> 3)
    return (1u << b) + (b >= 7 ? 16u : 0u);                          // j' + 16 bit7 + 16 bit8
}
constexpr uint32_t kIntraWords = 576;   // >= every intra map's span (575, 544)
constexpr uint32_t kCrossWords = 2112;  // >= the cross map's span (2111)
// immediate (word) offset of register r of layout L under map M
__host__ __device__ constexpr uint32_t roff(int L, int M, int r) {
    return ((r >> 2) & 1) * wgt(M, lay(L).r[0]) + ((r >> 1) & 1) * wgt(M, lay(L).r[1]) + (r & 1) * wgt(M, lay(L).r[2]);
}
// lane and wave part (words) of layout L under map M
template <int L, int M>
__device__ __forceinline__ uint32_t lbase(uint32_t l, uint32_t q) {
    constexpr Lay y = lay(L);
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) b += ((l >> (5 - i)) & 1u) * wgt(M, y.l[i]);
#pragma unroll
    for (int i = 0; i < 2; ++i) b += ((q >> (1 - i)) & 1u) * wgt(M, y.w[i]);
    return b;
}

// LDS layout of the workgroup (words): [psi^e - 1 (Mono), 2N pairs][TF: forward table,
// N pairs][TI: inverse table, N pairs][TW: psi^-i, N pairs][2 cross buffers][4 intra regions]
constexpr uint32_t kPsiW = 2 * 2 * kN;
constexpr uint32_t kTfW = kPsiW;
constexpr uint32_t kTiW = kTfW + 2 * kN;
constexpr uint32_t kTwW = kTiW + 2 * kN;
constexpr uint32_t kXW = kTwW + 2 * kN;
constexpr uint32_t kIW = kXW + 2 * kCrossWords;
constexpr uint32_t kLdsWordsQ = kIW + kWaves * kIntraWords;
constexpr size_t kLdsBytes = (size_t)kLdsWordsQ * 4;
static_assert(kLdsBytes <= 160 * 1024, "one quad workgroup per CU");
static_assert(kTfW % 4 == 0 && kXW % 4 == 0, "dwordx4 table copies");
// the two-workgroups-per-CU form (mk_quad2_kernel): the TF / TI / TW tables stay in
// HBM (read through L1 / L2), LDS holds [psi^e - 1][2 cross buffers][4 intra regions]
constexpr uint32_t kXW2 = kPsiW;
constexpr uint32_t kIW2 = kXW2 + 2 * kCrossWords;
constexpr size_t kLdsBytes2 = (size_t)(kIW2 + kWaves * kIntraWords) * 4;
static_assert(2 * kLdsBytes2 <= 160 * 1024, "two quad2 workgroups per CU");

// Table image in HBM (mkacc_ctx::d_qimg, mkacc_create): TF (= the reference forward
// table, negated pairs), TI[2^b + t] = psi^-(t 2^(11-b)) (negated pairs), TW[i] =
// psi^-i (Shoup pairs), 3N pairs, copied behind the psi^e - 1 table
template <bool LDSTAB>
__device__ __forceinline__ void load_tables(uint32_t* smem, const uint32_t* img, const uint32_t* qimg) {
    const uint4* s1 = reinterpret_cast<const uint4*>(img) + kPsm1Off / 2;
    const uint4* s2 = reinterpret_cast<const uint4*>(qimg);
    uint4* d = reinterpret_cast<uint4*>(smem);
    for (int i = threadIdx.x; i < kN; i += blockDim.x) d[i] = s1[i];
    if constexpr (LDSTAB)
        for (int i = threadIdx.x; i < 3 * kN / 2; i += blockDim.x) d[kN + i] = s2[i];
    __syncthreads();
}

// ---- per-wave context -------------------------------------------------------------
struct Ctx {
    const uint2* psi;    // LDS psi^e - 1
    const uint2* tf;     // LDS tables
    const uint2* ti;
    const uint2* tw;
    uint32_t* xb;        // LDS cross buffers (2 x kCrossWords)
    uint32_t* ib;        // LDS intra region of this wave
    const uint2* tws;    // HBM: forward table (scalar reads, stages on bits 10..8)
    const uint2* tis;    // HBM: inverse table, b < 5 (scalar reads, bits 0..2)
    uint32_t l, q;
    Mod m;
    SddConsts sd;
    // exchange bases (words): E1 QA->QB, E2 QB->QC (MI3), E3 QC->QD, E4 QD->IB (MX5),
    // E5 IB->IC (MI3), E6 IC->QA (MICA)
    uint32_t a_mi3, b_mi3, c_mi3, c_mx5, d_mx5, ib_mx5, ib_mi3, ic_mi3, ic_mica, a_mica;
};
__device__ __forceinline__ void init_bases(Ctx& s) {
    const uint32_t l = s.l, q = s.q;
    s.a_mi3 = lbase<QA, MI3>(l, q);
    s.b_mi3 = lbase<QB, MI3>(l, q);
    s.c_mi3 = lbase<QC, MI3>(l, q);
    s.c_mx5 = lbase<QC, MX5>(l, q);
    s.d_mx5 = lbase<QD, MX5>(l, q);
    s.ib_mx5 = lbase<IB, MX5>(l, q);
    s.ib_mi3 = lbase<IB, MI3>(l, q);
    s.ic_mi3 = lbase<IC, MI3>(l, q);
    s.ic_mica = lbase<IC, MICA>(l, q);
    s.a_mica = lbase<QA, MICA>(l, q);
}

// wave-local transpose SRC -> DST through the wave's own region
template <int SRC, int DST, int M>
__device__ __forceinline__ void xintra(uint32_t (&x)[kR], uint32_t* ib, uint32_t bs, uint32_t bd) {
#pragma unroll
    for (int r = 0; r < kR; ++r) ib[bs + roff(SRC, M, r)] = x[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < kR; ++r) x[r] = ib[bd + roff(DST, M, r)];
    wave_lds_sync();
}
// cross-wave exchange through cross buffer `buf` (alternating per exchange): the
// barrier orders every wave's writes before any read; a buffer is written again two
// exchanges later, after every wave has passed the barrier in between (so its reads
// of it are done: s_waitcnt lgkmcnt(0) precedes each barrier)
template <int SRC, int DST>
__device__ __forceinline__ void xcross(uint32_t (&x)[kR], uint32_t* buf, uint32_t bs, uint32_t bd) {
#pragma unroll
    for (int r = 0; r < kR; ++r) buf[bs + roff(SRC, MX5, r)] = x[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kR; ++r) x[r] = buf[bd + roff(DST, MX5, r)];
}

// ---- transforms ----------------------------------------------------------------------
// per-register butterfly with a per-lane twiddle from an LDS table: t = tab[base + o]
template <bool C>
__device__ __forceinline__ void bfly_lds(uint32_t& a, uint32_t& b, const uint2* tab, uint32_t base, uint32_t o,
                                         uint32_t Q) {
    ct_bfly_lazy<false, C>(a, b, tab[base + o], Q);
}

// Forward negacyclic NTT of NP quarter polynomials at once: QA (coefficients, < 4Q) ->
// QD (EVAL, [0, 4Q)); the reference's table and order (transformnat-impl.h:300-354)
// with the lazy Shoup butterflies of ntt_fwd (values grow by < 2Q per stage, the last
// one reduces).  The NP transforms (a pass's digit NTTs) run stage by stage together:
// NP x 4 independent butterflies per stage for a lone wave per SIMD, each stage's
// twiddles read once; the exchanges go polynomial by polynomial (a wave's LDS
// operations execute in order, so one region serves them all), each cross exchange
// on the next cross buffer.
template <int NP, bool C>
__device__ __forceinline__ void ntt_fwd_q(uint32_t (&x)[NP][kR], const Ctx& s, uint32_t& xs) {
    const uint32_t Q = s.m.Q, l = s.l, q = s.q;
    {   // QA: bits 10, 9, 8 -- twiddle 2^st + (j >> (b + 1)) depends on register bits only
        const ConstTable twc{(const_u64*)opaque(s.tws)};
        const uint2 w0 = twc[1], w1a = twc[2], w1b = twc[3], w2[4] = {twc[4], twc[5], twc[6], twc[7]};
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 4; ++r) ct_bfly_lazy<true, C>(x[p][r], x[p][r + 4], w0, Q);
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) ct_bfly_lazy<true, C>(x[p][r], x[p][r + 2], (r & 4) ? w1b : w1a, Q);
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 8; r += 2) ct_bfly_lazy<true, C>(x[p][r], x[p][r + 1], w2[r >> 1], Q);
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) xintra<QA, QB, MI3>(x[p], s.ib, s.a_mi3, s.b_mi3);
    {   // QB: bits 7, 6, 5; lane bits 5..3 = j bits 10..8
        const uint32_t lb = (l >> 3) & 7u;
        const uint2 w7 = s.tf[8u + lb];
        const uint2 w6[2] = {s.tf[16u + 2u * lb], s.tf[17u + 2u * lb]};
        const uint2 w5[4] = {s.tf[32u + 4u * lb], s.tf[33u + 4u * lb], s.tf[34u + 4u * lb], s.tf[35u + 4u * lb]};
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 4; ++r) ct_bfly_lazy<false, C>(x[p][r], x[p][r + 4], w7, Q);
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) ct_bfly_lazy<false, C>(x[p][r], x[p][r + 2], w6[r >> 2], Q);
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 8; r += 2) ct_bfly_lazy<false, C>(x[p][r], x[p][r + 1], w5[r >> 1], Q);
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) xintra<QB, QC, MI3>(x[p], s.ib, s.b_mi3, s.c_mi3);
    {   // QC: bits 4, 3, 2; lane = j bits 10..5
        const uint2 w4 = s.tf[64u + l];
        const uint2 w3[2] = {s.tf[128u + 2u * l], s.tf[129u + 2u * l]};
        const uint2 w2[4] = {s.tf[256u + 4u * l], s.tf[257u + 4u * l], s.tf[258u + 4u * l], s.tf[259u + 4u * l]};
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 4; ++r) ct_bfly_lazy<false, C>(x[p][r], x[p][r + 4], w4, Q);
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) ct_bfly_lazy<false, C>(x[p][r], x[p][r + 2], w3[r >> 2], Q);
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 8; r += 2) ct_bfly_lazy<false, C>(x[p][r], x[p][r + 1], w2[r >> 1], Q);
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        xcross<QC, QD>(x[p], s.xb + xs * kCrossWords, s.c_mx5, s.d_mx5);
        xs ^= 1u;
    }
    {   // QD: bits 1, 0; j = lane << 5 | q << 3 | r
        const uint32_t t1 = 512u + 8u * l + 2u * q, t0 = 1024u + 16u * l + 4u * q;
        const uint2 w1[2] = {s.tf[t1], s.tf[t1 + 1u]};
        const uint2 w0[4] = {s.tf[t0], s.tf[t0 + 1u], s.tf[t0 + 2u], s.tf[t0 + 3u]};
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) ct_bfly_lazy<false, C>(x[p][r], x[p][r + 2], w1[r >> 2], Q);
        const uint32_t m1 = s.m.m1;
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int r = 0; r < 8; r += 2) ct_bfly_last<C>(x[p][r], x[p][r + 1], w0[r >> 1], Q, m1);
    }
}

// Inverse without N^-1 (folded into keys and accumulators): QD (EVAL,
// [0, 2Q)) -> QA (canonical coefficients).  DIT butterflies on bits 0..10 with
// psi^-(t 2^(11-b)), t = j mod 2^b, then psi^-i per coefficient -- the map of the
// reference's GS inverse (transformnat-impl.h:492-552), as ntt_inv.  Every stage is
// the lazy butterfly: < 2Q + 11 x 2Q = 24Q < 2^32; the twist's Shoup product takes
// any 32-bit word.
template <bool C>
__device__ __forceinline__ void ntt_inv_q(uint32_t (&x)[kR], const Ctx& s, uint32_t& xs) {
    const uint32_t Q = s.m.Q, l = s.l, q = s.q;
    {   // QD: bits 0, 1, 2 -- t = j mod 2^b from register bits only
        const ConstTable twc{(const_u64*)opaque(s.tis)};
        const uint2 w0 = twc[1], w1[2] = {twc[2], twc[3]}, w2[4] = {twc[4], twc[5], twc[6], twc[7]};
#pragma unroll
        for (int r = 0; r < 8; r += 2) ct_bfly_lazy<true, C>(x[r], x[r + 1], w0, Q);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) ct_bfly_lazy<true, C>(x[r], x[r + 2], w1[r & 1], Q);
#pragma unroll
        for (int r = 0; r < 4; ++r) ct_bfly_lazy<true, C>(x[r], x[r + 4], w2[r & 3], Q);
    }
    xcross<QD, IB>(x, s.xb + xs * kCrossWords, s.d_mx5, s.ib_mx5);
    xs ^= 1u;
    {   // IB: bits 3, 4, 5; j bit 2 = lane bit 0, bits 1, 0 = q
        const uint32_t t = ((l & 1u) << 2) | q;
        const uint32_t b3 = 8u + t, b4 = 16u + t, b5 = 32u + t;
#pragma unroll
        for (int r = 0; r < 8; r += 2) bfly_lds<C>(x[r], x[r + 1], s.ti, b3, 0, Q);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) bfly_lds<C>(x[r], x[r + 2], s.ti, b4, (uint32_t)(r & 1) << 3, Q);
#pragma unroll
        for (int r = 0; r < 4; ++r) bfly_lds<C>(x[r], x[r + 4], s.ti, b5, (uint32_t)(r & 3) << 3, Q);
    }
    xintra<IB, IC, MI3>(x, s.ib, s.ib_mi3, s.ic_mi3);
    {   // IC: bits 6, 7, 8; j bits 5..2 = lane bits 3..0, bits 1, 0 = q
        const uint32_t t = ((l & 15u) << 2) | q;
        const uint32_t b6 = 64u + t, b7 = 128u + t, b8 = 256u + t;
#pragma unroll
        for (int r = 0; r < 8; r += 2) bfly_lds<C>(x[r], x[r + 1], s.ti, b6, 0, Q);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) bfly_lds<C>(x[r], x[r + 2], s.ti, b7, (uint32_t)(r & 1) << 6, Q);
#pragma unroll
        for (int r = 0; r < 4; ++r) bfly_lds<C>(x[r], x[r + 4], s.ti, b8, (uint32_t)(r & 3) << 6, Q);
    }
    xintra<IC, QA, MICA>(x, s.ib, s.ic_mica, s.a_mica);
    {   // QA: bits 9, 10 and the twist; j = r << 8 | lane << 2 | q
        const uint32_t t = (l << 2) | q;
        const uint32_t b9 = 512u + t, b10 = 1024u + t;
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) bfly_lds<C>(x[r], x[r + 2], s.ti, b9, (uint32_t)(r & 1) << 8, Q);
#pragma unroll
        for (int r = 0; r < 4; ++r) bfly_lds<C>(x[r], x[r + 4], s.ti, b10, (uint32_t)(r & 3) << 8, Q);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint2 w = s.tw[t + ((uint32_t)r << 8)];
            x[r] = mul_shoup(x[r], w.x, w.y, Q);
        }
    }
}

// ---- monomials at this wave's EVAL slots ------------------------------------------
// slot j = lane << 5 | q << 3 | r is Mono's (lane, R = q << 3 | r) with
// brv5(R) = brv3(r) << 2 | brv2(q): the wave part joins the per-lane word once
struct QMono {
    uint32_t w, c;
    __device__ __forceinline__ uint2 at(const uint2* psi, int r) const {
        constexpr uint32_t kBr3[8] = {0, 4, 2, 6, 1, 5, 3, 7};
        uint32_t cs = c;
        asm volatile("" : "+s"(cs));
        uint32_t a;
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(a) : "s"(cs * (4096u * kBr3[r])), "v"(w));
        a &= 0x7fffu;
        return *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(psi) + a);
    }
};
__device__ __forceinline__ QMono make_qmono(uint32_t c, uint32_t l, uint32_t q) {
    const Mono m = make_mono(c, l);
    const uint32_t bq = ((q & 1u) << 1) | (q >> 1);   // brv2(q)
    return QMono{m.w + ((c * bq) << 10), c};
}

// ---- one accumulator step ----------------------------------------------------------
template <int DG, int METHOD, bool FIRST>
struct QCfg {
    static constexpr bool kSplit = METHOD == XZW && !FIRST;
    static constexpr bool kK2 = METHOD == XZW;
    static constexpr int kG = DG > 4 ? 2 : 4;
    static_assert(2 + DG * kG <= 32, "quad sum bound");
};
// key words of this wave's slots: group g (0, 1) = C4 group 2q + g of every lane
template <int DG, int METHOD, bool FIRST>
struct QKeys {
    u32x4 k1[2][DG];
    u32x4 k2[2][QCfg<DG, METHOD, FIRST>::kK2 ? DG : 1];
    u32x4 ks[2][FIRST ? DG : 1];
    u32x4 pk[2][DG];
};
struct QRes {
    __amdgpu_buffer_rsrc_t rin, rout, rk1, rk2, rks, rpk;
    uint32_t vo, so;   // lane offset (l * 16), this wave's group offset (2q * 1024)
};
// issue the pass's key loads (F: f-part, keys' f-half, no P)
template <int DG, int METHOD, bool FIRST, bool F>
__device__ __forceinline__ void issue_keys(QKeys<DG, METHOD, FIRST>& kk, const QRes& rs, uint32_t u) {
    using Cf = QCfg<DG, METHOD, FIRST>;
    const uint32_t polyB = kN * 4u, half = F ? polyB : 0u, poff = u * DG * polyB;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const uint32_t so = rs.so + (uint32_t)g * 1024u;
#pragma unroll
        for (int i = 0; i < DG; ++i) {
            const uint32_t ko = (uint32_t)(2 * i) * polyB + half + so;
            kk.k1[g][i] = bload4(rs.rk1, rs.vo, ko);
            if (Cf::kK2) kk.k2[g][i] = bload4(rs.rk2, rs.vo, ko);
            if (FIRST) kk.ks[g][i] = bload4(rs.rks, rs.vo, ko);
            if (!F) kk.pk[g][i] = bload4(rs.rpk, rs.vo, poff + (uint32_t)i * polyB + so);
        }
    }
}

// iNTT -> SDD -> dg forward NTTs of the quarter: x (QD, [0, 2Q)) -> G[i] (QD); the
// digit NTTs run together (ntt_fwd_q<DG>)
template <int DG, bool C>
__device__ __forceinline__ void digits_q(const Ctx& s, uint32_t (&x)[kR], uint32_t (&G)[DG][kR], uint32_t& xs) {
    ntt_inv_q<C>(x, s, xs);
    PackedDigits<DG, kR> pd;
#pragma unroll
    for (int r = 0; r < kR; ++r) G[0][r] = pd.put(r, sdd_offset(x[r], s.sd), s.sd);
#pragma unroll
    for (int i = 1; i < DG; ++i)
#pragma unroll
        for (int r = 0; r < kR; ++r) G[i][r] = pd.get(r, i + 1, s.sd);
    ntt_fwd_q<DG, C>(G, s, xs);
#pragma unroll
    for (int i = 0; i < DG; ++i) digit_range<DG>(G[i], s.m.Q);
}

// the MAC of one pass over this wave's 8 slots (mac2's algebra):
//   F = false (party u): start = acc_u (st), out -> acc_out[u], sv <- redc(sv r32 + sum G P)
//   F = true  (f-part):  start = the index party's output (st), out -> acc_out[index]
// KEEP: the outputs stay in keep[] instead of going to acc_out (the index party's pass,
// whose output only the f-part reads)
// KEEP 2: keep[] gets the outputs and acc_out too (the f-part output the index party's
// next pass starts from, MKACC_QUADP_CARRY)
template <int DG, int METHOD, bool FIRST, bool F, int KEEP = 0>
__device__ __forceinline__ void mac_q(const Ctx& s, const QRes& rs, const QKeys<DG, METHOD, FIRST>& kk,
                                      const uint32_t (&G)[DG][kR], const uint32_t (&st)[kR], uint32_t (&sv)[kR],
                                      const QMono& mp, const QMono& mn, uint32_t u, uint32_t* keep = nullptr) {
    using Cf = QCfg<DG, METHOD, FIRST>;
    const uint32_t Q = s.m.Q;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        u32x4 ov;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * g + e;
            uint64_t a1 = (F || !FIRST) ? mad64(st[r], s.m.r32, 0) : 0ull;
            uint64_t a2 = 0, sa = F ? 0ull : mad64(sv[r], s.m.r32, 0);
#pragma unroll
            for (int i = 0; i < DG; ++i) {
                if constexpr (Cf::kSplit) {
                    a1 = mad64(G[i][r], kk.k1[g][i][e], a1);
                    a2 = mad64(G[i][r], kk.k2[g][i][e], a2);
                } else {
                    // key_eff with this wave's monomials (r is the register index of QMono)
                    uint32_t ke;
                    if (METHOD == XZW) {
                        const uint32_t k1 = kk.k1[g][i][e], k2 = Cf::kK2 ? kk.k2[g][i][e] : 0u;
                        const uint32_t e1 = k1 + Q - k2;   // FIRST: evs + ev1 (X^c-1) + ev2 (X^-c-1)
                        uint32_t d = (FIRST ? kk.ks[g][i][e] : 0u) + mul_shoup_lazy(e1, mp.at(s.psi, r), Q) +
                                     mul_shoup_lazy(k2, mn.at(s.psi, r), Q);
                        d = min(d, d - 2u * Q);
                        ke = from3q<1>(d, Q);
                    } else if (FIRST) {
                        ke = from3q<1>(kk.ks[g][i][e] + mul_shoup_lazy(kk.k1[g][i][e], mp.at(s.psi, r), Q), Q);
                    } else {
                        ke = kk.k1[g][i][e];
                    }
                    a1 = mad64(G[i][r], ke, a1);
                }
                if (!F) sa = mad64(G[i][r], kk.pk[g][i][e], sa);
            }
            uint32_t v = redc(a1, Q, s.m.qinv);                                    // [0, 2Q)
            if constexpr (Cf::kSplit) {
                v += mul_shoup_lazy(redc(a2, Q, s.m.qinv), mn.at(s.psi, r), Q);   // [0, 4Q)
                v = min(v, v - 2u * Q);
            }
            ov[e] = v;
            if (!F) sv[r] = redc(sa, Q, s.m.qinv);
        }
        if constexpr (KEEP != 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) keep[4 * g + e] = ov[e];
        }
        if constexpr (KEEP != 1) bstore4(ov, rs.rout, rs.vo, u * (kN * 4u) + rs.so + (uint32_t)g * 1024u);
    }
    vcc_fence();
}

// xs: the cross buffer of the next exchange, carried from step to step ((k + 1)(dg + 1)
// exchanges per step may be odd: two exchanges in a row must never share a buffer)
template <int DG, int METHOD, bool FIRST>
__device__ __forceinline__ void quad_step(const StepArgs& a, const Ctx& s0, uint32_t& xs) {
    constexpr bool C = true;   // C Shoup products in every transform
    Ctx s = s0;
    const uint32_t l = s.l, q = s.q;
    const uint32_t gate = blockIdx.x;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k, index = a.index;
    const uint32_t polyB = kN * 4u;
    const QMono mp = make_qmono(c, l, q);
    // X^-c in the first step; X^(N-c) = -X^-c in the later XZW steps (key_eff, mac2)
    const QMono mn = make_qmono(FIRST || METHOD != XZW ? cneg : (cneg + kN) & (2u * kN - 1u), l, q);
    const QRes rs{make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB),
                  make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB),
                  make_rsrc(a.key1, DG * 2 * polyB),
                  make_rsrc(a.key2, DG * 2 * polyB),
                  make_rsrc(a.keys, DG * 2 * polyB),
                  make_rsrc(a.pkey, k * DG * polyB),
                  l * 16u,
                  q * 2048u};
    const uint32_t Q = s.m.Q;
    uint32_t sv[kR];
    uint32_t keep[kR];   // the index party's pass output, the f-part's start (MKACC_QUADP_KEEP)
    // not in the first (KDM) step: it runs once per gate, and at dg = 5 the kept words
    // pushed a 16-byte store's data registers into a store-data hazard (isa_audit)
    constexpr bool kKeep = MKACC_QUAD_KEEP && !FIRST;
#pragma unroll
    for (int r = 0; r < kR; ++r) sv[r] = 0;
    // passes t = 0 .. k - 1: party index + 1 + t (mod k), the index party last; t = k: the f-part
#pragma unroll 1
    for (uint32_t t = 0; t <= k; ++t) {
        const bool fpart = __builtin_amdgcn_readfirstlane(t) == k;
        const uint32_t u = index + 1 + t < k ? index + 1 + t : index + 1 + t - k;
        uint32_t x[kR], st[kR];
        QKeys<DG, METHOD, FIRST> kk;
        // keys issued before the transforms, except in the first (KDM) step: its four
        // key words per digit would hold 32 dg VGPRs across them (it runs once per gate)
        constexpr bool kPf = MKACC_QUAD_PF && !FIRST;
        if (!fpart) {
            if (kPf) issue_keys<DG, METHOD, FIRST, false>(kk, rs, u);
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const u32x4 v = bload4(rs.rin, rs.vo, u * polyB + rs.so + (uint32_t)g * 1024u);
#pragma unroll
                for (int e = 0; e < 4; ++e) st[4 * g + e] = v[e];
            }
            if (!FIRST) {
                // acctemp = acc * (X^c - 1)                 (xzw.cpp:336-338)
#pragma unroll
                for (int r = 0; r < kR; ++r) x[r] = mul_shoup_lazy(st[r], mp.at(s.psi, r), Q);
            } else {
#pragma unroll
                for (int r = 0; r < kR; ++r) x[r] = st[r];
            }
            vcc_fence();   // the jump over the f-part branch follows the rotation
        } else {
            if (kKeep) {
                if (kPf) issue_keys<DG, METHOD, FIRST, true>(kk, rs, index);
#pragma unroll
                for (int r = 0; r < kR; ++r) st[r] = keep[r];
            } else {
                // the index party's output: this wave's own stores earlier in the step
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (kPf) issue_keys<DG, METHOD, FIRST, true>(kk, rs, index);
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    const u32x4 v = bload4(rs.rout, rs.vo, index * polyB + rs.so + (uint32_t)g * 1024u);
#pragma unroll
                    for (int e = 0; e < 4; ++e) st[4 * g + e] = v[e];
                }
            }
#pragma unroll
            for (int r = 0; r < kR; ++r) x[r] = sv[r];
        }
        vcc_fence();   // the branch joins after the rotation's multiply-adds
        uint32_t G[DG][kR];
        digits_q<DG, C>(s, x, G, xs);
        vcc_fence();   // the MAC branch follows the last butterflies
        if (!fpart) {
            if (!kPf) issue_keys<DG, METHOD, FIRST, false>(kk, rs, u);
            if (kKeep && u == index)
                mac_q<DG, METHOD, FIRST, false, 1>(s, rs, kk, G, st, sv, mp, mn, u, keep);
            else
                mac_q<DG, METHOD, FIRST, false>(s, rs, kk, G, st, sv, mp, mn, u);
        } else {
            if (!kPf) issue_keys<DG, METHOD, FIRST, true>(kk, rs, index);
            mac_q<DG, METHOD, FIRST, true>(s, rs, kk, G, st, sv, mp, mn, index);
        }
        if (fpart) break;
    }
}

// ---- party-parallel steps (mk_quadp_run_kernel) ------------------------------------
// A batch of B <= CUs / k gates runs B k workgroups, one per CU: workgroup g k + t runs
// party t's pass of every step of gate g (its accumulator polynomial is touched by no
// other workgroup), and the index party's workgroup also runs the step's f-part.  The
// f-part needs sumV = sum over the parties of their sv shares; the other parties publish
// theirs through a per-gate HBM ring of kSlots slots and run on into their next steps
// (which need only their own polynomial), so a step's critical path is the index
// party's pass plus the f-part: 2 (dg + 1) transforms instead of (k + 1)(dg + 1).
// Synchronisation is per wave: wave q of the index workgroup reads only the slots wave
// q of every other workgroup wrote (the same EVAL slots), so no workgroup barrier is
// added.  Shares and counters move with system-coherent accesses (sc0 sc1: written
// through to memory, read past both cache levels) ordered by s_waitcnt, never by
// whole-cache write-backs or invalidates: agent-scope release / acquire pairs
// (buffer_wbl2 / buffer_inv) ran 18.4 ms per STD128_MKNTRU gate at B = 1 but tripled
// the step at 256 workgroups, where every CU's waits flushed its XCD's L2
// (profiles/r6/v15).  A share carries its step in the free top bits of every word
// (a residue below 2Q < 2^28; tag 1 + rel mod 8, a zeroed slot never matches), so the
// index party loads the shares without a flag round trip, after its own pass, and
// reloads only what is not there yet.  One counter
// per wave, `used`, orders the ring: the index party's wave q posts rel + 1 once it has
// taken step rel's shares (and, in the last kSlots steps of its turn as index, written
// its own share of rel to its slot, so no slot keeps a share from 8 steps back); a writer
// waits for used >= rel + 1 - kSlots before reusing a slot, and a party that takes over
// as index waits for the same before (re)loading, so every slot it reads holds step rel
// or rel - kSlots, whose tags differ (tools/quadp_protocol.py checks this under random
// schedules, and that each of the three rules is needed).  Every wait is bounded: a timeout sets *abort, after which no wave waits
// again (the kernel drains, the engine reports MKACC_E_DEVICE).
constexpr uint32_t kSlots = 4;
constexpr uint32_t kBatch = 4;              // shares per load batch of the index workgroup
#ifndef MKACC_QUADP_CARRY
// 1: a one-party workgroup that stays index keeps its f-part output in registers for the
// next step's pass (no reload through acc_in, no drain of the step's stores).  Off:
// 3 % slower for one STD128_MKNTRU gate, 1.4 % for STD128_MKNTRU_3 (profiles/r6/v39)
#define MKACC_QUADP_CARRY 0
#endif
#ifndef MKACC_QUADP_PRELOAD
// 1: the index workgroup's first share batch in flight across its pass.  Off: the
// system-coherent loads queued behind the pass's accumulator loads delayed its keys
// (vector loads return in order): loading after the pass was 1.5-3 % faster at k = 2,
// 8 and 16 (profiles/r6/v32)
#define MKACC_QUADP_PRELOAD 0
#endif
constexpr uint32_t kSpinLimit = 1u << 20;   // polls of ~1 us: far beyond any step
constexpr int kSysCoherent = 1 | 16;        // buffer cache policy sc0 | sc1
struct PSync {
    uint32_t* used;    // this gate's [4]: steps whose shares wave q of the index workgroup has taken
    __amdgpu_buffer_rsrc_t rsv;   // this gate's [kSlots][groups][N] tagged sv shares, C4 order
    uint32_t* abort;
    uint32_t gate, wg;            // this workgroup's gate and its place among the gate's
    uint32_t groups, ppw;         // workgroups per gate; parties per workgroup (wg owns
                                  // parties wg ppw .. wg ppw + ppw - 1)
};
// words of the synchronisation area for B gates of G workgroups: the counters, then the
// 16-byte aligned slot ring (all zeroed before every launch)
__host__ __device__ constexpr size_t psync_counter_words(size_t B) { return (B * 4 + 3) & ~size_t(3); }
__host__ __device__ constexpr size_t psync_words(size_t B, size_t G) {
    return psync_counter_words(B) + B * kSlots * G * (size_t)kN;
}
__device__ __forceinline__ PSync make_psync(uint32_t* sync, uint32_t* abort, uint32_t B, uint32_t G, uint32_t ppw) {
    PSync p;
    p.gate = __builtin_amdgcn_readfirstlane(blockIdx.x / G);
    p.wg = __builtin_amdgcn_readfirstlane(blockIdx.x - p.gate * G);
    p.groups = G;
    p.ppw = ppw;
    p.used = sync + p.gate * 4;
    p.rsv = make_rsrc(sync + psync_counter_words(B) + (size_t)p.gate * kSlots * G * kN, kSlots * G * kN * 4u);
    p.abort = abort;
    return p;
}
__device__ __forceinline__ uint32_t share_tag(uint32_t rel) { return (rel & 7u) + 1u; }
__device__ __forceinline__ bool aborted(uint32_t* abort) {
    return __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}
__device__ __forceinline__ void set_abort(uint32_t* abort) {
    __hip_atomic_store(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// wait until *p >= want; false after a timeout here or elsewhere
__device__ __forceinline__ bool wait_at_least(const uint32_t* p, uint32_t want, uint32_t* abort) {
    asm volatile("" ::: "memory");
    bool ok = true;
    for (uint32_t n = 0;; ++n) {
        if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= want) break;
        if (aborted(abort)) { ok = false; break; }
        if (n >= kSpinLimit) {
            set_abort(abort);
            ok = false;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    asm volatile("" ::: "memory");
    return ok;
}
// set a counter once the loads whose values the caller consumed have completed
__device__ __forceinline__ void post(uint32_t* p, uint32_t v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("" ::: "memory");
}
// the index party's loads of shares o0 .. o0 + nb - 1 (party index + o) of this step
template <uint32_t NB>
struct ShareBatch {
    u32x4 v[NB][2];
};
template <uint32_t NB>
__device__ __forceinline__ void load_shares(ShareBatch<NB>& sb, const PSync& ps, uint32_t slot, uint32_t k,
                                            uint32_t index, uint32_t o0, uint32_t nb, uint32_t vo, uint32_t so) {
    const uint32_t polyB = kN * 4u;
#pragma unroll
    for (uint32_t b = 0; b < NB; ++b) {
        if (b < nb) {
            const uint32_t o = o0 + b, u = index + o < k ? index + o : index + o - k;
#pragma unroll
            for (int g = 0; g < 2; ++g)
                sb.v[b][g] = __builtin_amdgcn_raw_buffer_load_b128(ps.rsv, vo, (slot * k + u) * polyB + so +
                                                                   (uint32_t)g * 1024u, kSysCoherent);
        }
    }
}
// check the batch's tags (reloading until every word of the wave carries this step's),
// then add its shares into sum ([0, 2Q))
template <uint32_t NB>
__device__ __forceinline__ void take_shares(ShareBatch<NB>& sb, const PSync& ps, uint32_t slot, uint32_t k,
                                            uint32_t index, uint32_t o0, uint32_t nb, uint32_t vo, uint32_t so,
                                            uint32_t tag, uint32_t Q, uint32_t (&sum)[kR]) {
    for (uint32_t n = 0;; ++n) {
        bool ok = true;
#pragma unroll
        for (uint32_t b = 0; b < NB; ++b)
            if (b < nb)
#pragma unroll
                for (int g = 0; g < 2; ++g)
#pragma unroll
                    for (int e = 0; e < 4; ++e) ok = ok && (sb.v[b][g][e] >> 28) == tag;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;   // wave-uniform
        if (aborted(ps.abort)) break;
        if (n >= kSpinLimit) {
            set_abort(ps.abort);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
        asm volatile("" ::: "memory");
        load_shares(sb, ps, slot, k, index, o0, nb, vo, so);
    }
#pragma unroll
    for (uint32_t b = 0; b < NB; ++b)
        if (b < nb)
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t y = sum[4 * g + e] + (sb.v[b][g][e] & 0x0fffffffu);
                    sum[4 * g + e] = min(y, y - 2u * Q);
                }
}

// publish this wave's tagged share of step rel in its slot (system-coherent stores)
__device__ __forceinline__ void put_share(const PSync& ps, const uint32_t (&sv)[kR], uint32_t slot, uint32_t k,
                                          uint32_t t, uint32_t tag, uint32_t vo, uint32_t so) {
    const uint32_t polyB = kN * 4u, tg = tag << 28;
    asm volatile("" ::: "memory");
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{sv[4 * g] | tg, sv[4 * g + 1] | tg, sv[4 * g + 2] | tg, sv[4 * g + 3] | tg}, ps.rsv, vo,
            (slot * k + t) * polyB + so + (uint32_t)g * 1024u, kSysCoherent);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 1");   // store-data hazard (bstore4)
        __builtin_amdgcn_sched_barrier(0);
    }
}

// one later step (rel = steps since the launch's first) of workgroup ps.wg of gate
// ps.gate: the passes of its parties (the index party's last), then -- the index
// workgroup -- the f-part.  takeover: the index workgroup of this step was not the
// previous step's; last: this step is one of the last kSlots of the index workgroup's turn
// carry_in: the index party's accumulator is carry[] (this workgroup's f-part output of
// the previous step, the same index party); carry_out: keep this step's f-part output
template <int DG, int METHOD, uint32_t NB>
__device__ __forceinline__ void quadp_step(const StepArgs& a, const Ctx& s0, uint32_t& xs, const PSync& ps,
                                           uint32_t rel, bool takeover, bool last, bool carry_in, bool carry_out,
                                           uint32_t (&carry)[kR]) {
    constexpr bool C = true, FIRST = false;
    constexpr bool kPf = MKACC_QUAD_PF;
    Ctx s = s0;
    const uint32_t l = s.l, q = s.q;
    const uint32_t gate = ps.gate, w = ps.wg, G = ps.groups;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k, index = a.index;
    const uint32_t polyB = kN * 4u;
    const QMono mp = make_qmono(c, l, q);
    const QMono mn = make_qmono(METHOD != XZW ? cneg : (cneg + kN) & (2u * kN - 1u), l, q);
    const QRes rs{make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB),
                  make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB),
                  make_rsrc(a.key1, DG * 2 * polyB),
                  make_rsrc(a.key2, DG * 2 * polyB),
                  make_rsrc(a.keys, DG * 2 * polyB),
                  make_rsrc(a.pkey, k * DG * polyB),
                  l * 16u,
                  q * 2048u};
    const uint32_t Q = s.m.Q;
    const uint32_t slot = rel % kSlots, tag = share_tag(rel);
    const uint32_t lo = w * ps.ppw, cnt = min(k, lo + ps.ppw) - lo, iw = index / ps.ppw;
    const bool is_index = w == iw;
    // pass order lo + (base - lo + j) mod cnt, j = 1 .. cnt: the index party last
    const uint32_t base = is_index ? index : lo + cnt - 1u;
    ShareBatch<NB> sb;
    const uint32_t nb0 = is_index ? min(G - 1u, NB) : 0u;
    uint32_t sv[kR];   // the workgroup's share: redc-summed over its parties' passes (mac_q)
    uint32_t keep[kR];   // the index party's pass output, the f-part's start (MKACC_QUADP_KEEP)
#pragma unroll
    for (int r = 0; r < kR; ++r) sv[r] = 0;
#pragma unroll 1
    for (uint32_t j = 1; j <= cnt; ++j) {   // party u's pass: acc_out[u] and its sv share
        const uint32_t o = base - lo + j, u = __builtin_amdgcn_readfirstlane(lo + (o < cnt ? o : o % cnt));
        uint32_t x[kR], st[kR];
        QKeys<DG, METHOD, FIRST> kk;
        // loads in the order they are needed (vector loads return in order): the party's
        // accumulator for the rotation, then -- the index party -- the first batch of the
        // other workgroups' shares, in flight across the pass, then the keys for the MAC
        if (carry_in && u == index) {
#pragma unroll
            for (int r = 0; r < kR; ++r) st[r] = carry[r];
        } else {
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const u32x4 v = bload4(rs.rin, rs.vo, u * polyB + rs.so + (uint32_t)g * 1024u);
#pragma unroll
                for (int e = 0; e < 4; ++e) st[4 * g + e] = v[e];
            }
        }
        asm volatile("" ::: "memory");
        if (MKACC_QUADP_PRELOAD && is_index && j == cnt) load_shares(sb, ps, slot, G, iw, 1u, nb0, rs.vo, rs.so);
        asm volatile("" ::: "memory");
        if (kPf) issue_keys<DG, METHOD, FIRST, false>(kk, rs, u);
#pragma unroll
        for (int r = 0; r < kR; ++r) x[r] = mul_shoup_lazy(st[r], mp.at(s.psi, r), Q);   // xzw.cpp:336-338
        vcc_fence();
        uint32_t Gd[DG][kR];
        digits_q<DG, C>(s, x, Gd, xs);
        vcc_fence();
        if (!kPf) issue_keys<DG, METHOD, FIRST, false>(kk, rs, u);
        if (MKACC_QUADP_KEEP && is_index && j == cnt)
            mac_q<DG, METHOD, FIRST, false, 1>(s, rs, kk, Gd, st, sv, mp, mn, u, keep);
        else
            mac_q<DG, METHOD, FIRST, false>(s, rs, kk, Gd, st, sv, mp, mn, u);
    }
    if (!is_index) {
        // publish the tagged share once the index workgroup has taken what the slot held
        if (rel + 1u > kSlots) wait_at_least(ps.used + q, rel + 1u - kSlots, ps.abort);
        put_share(ps, sv, slot, G, w, tag, rs.vo, rs.so);
        return;
    }
    // the index workgroup: sumV = its own share + the others', then the f-part.  Taking
    // over from another workgroup, it first waits for the ring to hold nothing older than
    // rel - kSlots (as index of the previous step it posted used = rel itself)
    if (takeover || !MKACC_QUADP_PRELOAD) {
        // the batch loaded before the pass may hold a share from 2 kSlots steps back
        // (same tag): load it again once the ring is known to be recent
        if (takeover && rel + 1u > kSlots) wait_at_least(ps.used + q, rel + 1u - kSlots, ps.abort);
        load_shares(sb, ps, slot, G, iw, 1u, nb0, rs.vo, rs.so);
    }
    uint32_t x[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) x[r] = sv[r];
    take_shares(sb, ps, slot, G, iw, 1u, nb0, rs.vo, rs.so, tag, Q, x);
#pragma unroll 1
    for (uint32_t o0 = 1u + NB; o0 < G; o0 += NB) {
        const uint32_t nb = min(G - o0, NB);
        load_shares(sb, ps, slot, G, iw, o0, nb, rs.vo, rs.so);
        take_shares(sb, ps, slot, G, iw, o0, nb, rs.vo, rs.so, tag, Q, x);
    }
    vcc_fence();
    // the shares have landed: outside the last kSlots steps of its turn (no slot write of
    // its own) the index workgroup frees the slots now, not behind the f-part
    if (!last) post(ps.used + q, rel + 1u);
    {
        uint32_t st[kR];
        QKeys<DG, METHOD, FIRST> kk;
        if (MKACC_QUADP_KEEP) {
            if (kPf) issue_keys<DG, METHOD, FIRST, true>(kk, rs, index);
#pragma unroll
            for (int r = 0; r < kR; ++r) st[r] = keep[r];
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's acc_out[index] stores
            if (kPf) issue_keys<DG, METHOD, FIRST, true>(kk, rs, index);
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const u32x4 v = bload4(rs.rout, rs.vo, index * polyB + rs.so + (uint32_t)g * 1024u);
#pragma unroll
                for (int e = 0; e < 4; ++e) st[4 * g + e] = v[e];
            }
        }
        // the index workgroup refreshes its slots in the last kSlots steps of its turn (a
        // share of its last turn as writer could alias the tag later): issued behind the
        // f-part's loads (vmcnt counts stores too, in order), so no wait before the MAC
        // covers the write-through store
        if (last) put_share(ps, sv, slot, G, w, tag, rs.vo, rs.so);
        uint32_t Gd[DG][kR];
        digits_q<DG, C>(s, x, Gd, xs);
        vcc_fence();
        if (!kPf) issue_keys<DG, METHOD, FIRST, true>(kk, rs, index);
        if (carry_out)
            mac_q<DG, METHOD, FIRST, true, 2>(s, rs, kk, Gd, st, sv, mp, mn, index, carry);
        else
            mac_q<DG, METHOD, FIRST, true>(s, rs, kk, Gd, st, sv, mp, mn, index);
    }
    // in the last steps of its turn: the shares have landed and its own is written (long
    // since, behind the f-part: the wait for the write-through store is off the critical path)
    if (last) post(ps.used + q, rel + 1u);
}

}  // namespace quad

// Zeroes the synchronisation area before a party-parallel launch with system-coherent
// stores: a zeroed slot must read as "no share" through the whole launch, and an
// ordinary fill could leave dirty L2 lines whose later write-back lands on top of a
// share written through to memory (the shares bypass the L2s).
__global__ void psync_clear_kernel(uint32_t* p, uint32_t vec4s) {
    const __amdgpu_buffer_rsrc_t r = make_rsrc(p, vec4s * 16u);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < vec4s; i += gridDim.x * blockDim.x)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, r, i * 16u, 0, quad::kSysCoherent);
}

namespace quad {
template <bool LDSTAB>
__device__ __forceinline__ Ctx make_ctx(const StepArgs& a, uint32_t* smem, const uint32_t* qimg) {
    Ctx s;
    const uint2* t = reinterpret_cast<const uint2*>(smem);
    const uint2* g = reinterpret_cast<const uint2*>(qimg);
    s.psi = t;
    s.tf = LDSTAB ? t + kTfW / 2 : g;
    s.ti = LDSTAB ? t + kTiW / 2 : g + kN;
    s.tw = LDSTAB ? t + kTwW / 2 : g + 2 * kN;
    s.xb = smem + (LDSTAB ? kXW : kXW2);
    s.l = threadIdx.x & 63u;
    s.q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    s.ib = smem + (LDSTAB ? kIW : kIW2) + s.q * kIntraWords;
    s.tws = a.tw_fwd;
    s.tis = a.tw_inv;
    s.m = a.m;
    s.sd = a.sd;
    init_bases(s);
    (void)qimg;
    return s;
}

}  // namespace quad

struct QuadArgs {
    const uint32_t* qimg;   // TF, TI, TW tables (mkacc_ctx::d_qimg), 3N pairs
    uint32_t* sync;         // mk_quadp_run_kernel: counters and sv slots (quad::psync_words)
    uint32_t* abort;        // mk_quadp_run_kernel: non-zero after a synchronisation timeout
    uint32_t groups, ppw;   // mk_quadp_run_kernel: workgroups per gate, parties per workgroup
};

// one accumulator step (the first, KDM, or any other) for B gates, one workgroup each.
// OCC = 1: the twiddle tables in LDS, one workgroup per CU (B <= CUs: every gate
// resident at once, the kernel the engine takes); OCC = 2: the tables in HBM, two
// workgroups per CU (mk_quad2_kernel, MKACC_QUAD=2)
template <int DG, int METHOD, bool FIRST, int OCC>
__device__ __forceinline__ void quad_one(const StepArgs& a, const QuadArgs& qa, uint32_t* smem) {
    quad::load_tables<OCC == 1>(smem, a.img, qa.qimg);
    const quad::Ctx s = quad::make_ctx<OCC == 1>(a, smem, qa.qimg);
    uint32_t xs = 0;
    quad::quad_step<DG, METHOD, FIRST>(a, s, xs);
}
// steps [t0, t1) (none the first) in one launch: each workgroup runs its gate's steps
// back to back; a wave reads only the accumulator slots it wrote itself, so a step's
// stores drain (vmcnt) before the next step's loads and no workgroup barrier is needed
// between steps beyond those inside the transforms
template <int DG, int METHOD, int OCC>
__device__ __forceinline__ void quad_run(const StepArgs& a, const LatdRun& r, const QuadArgs& qa, uint32_t* smem) {
    quad::load_tables<OCC == 1>(smem, a.img, qa.qimg);
    const quad::Ctx s = quad::make_ctx<OCC == 1>(a, smem, qa.qimg);
    uint32_t xs = 0;
#pragma unroll 1
    for (uint32_t t = r.t0; t < r.t1; ++t) {
        quad::quad_step<DG, METHOD, false>(run_args(a, r, t), s, xs);
        vcc_fence();   // the loop branch follows the step's last reductions
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}
template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(256, 1) void mk_quad_kernel(StepArgs a, QuadArgs qa) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    quad_one<DG, METHOD, FIRST, 1>(a, qa, smem);
}
template <int DG, int METHOD>
__global__ __launch_bounds__(256, 1) void mk_quad_run_kernel(StepArgs a, LatdRun r, QuadArgs qa) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    quad_run<DG, METHOD, 1>(a, r, qa, smem);
}
template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(256, 2) void mk_quad2_kernel(StepArgs a, QuadArgs qa) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    quad_one<DG, METHOD, FIRST, 2>(a, qa, smem);
}
template <int DG, int METHOD>
__global__ __launch_bounds__(256, 2) void mk_quad2_run_kernel(StepArgs a, LatdRun r, QuadArgs qa) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    quad_run<DG, METHOD, 2>(a, r, qa, smem);
}

// steps [t0, t1) party-parallel: B G workgroups, all resident (cooperative launch).
// OCC = 1: tables in LDS, one workgroup per CU (B <= CUs / 2); OCC = 2: tables in HBM,
// two per CU (mk_quadp2_run_kernel, CUs / 2 < B <= CUs, dg <= 4)
template <int DG, int METHOD, int OCC>
__device__ __forceinline__ void quadp_run(const StepArgs& a, const LatdRun& r, const QuadArgs& qa, uint32_t* smem) {
    quad::load_tables<OCC == 1>(smem, a.img, qa.qimg);
    const quad::Ctx s = quad::make_ctx<OCC == 1>(a, smem, qa.qimg);
    const quad::PSync ps = quad::make_psync(qa.sync, qa.abort, a.B, qa.groups, qa.ppw);
    uint32_t xs = 0;
    uint32_t carry[quad::kR];
    bool carried = false;
#pragma unroll 1
    for (uint32_t t = r.t0; t < r.t1; ++t) {
        // the index workgroup of step t is (t / n) / ppw (run_args: index = t / n)
        const uint32_t iw = t / r.n / ps.ppw;
        // a workgroup of one party that stays index for the next step keeps its f-part
        // output in registers: no reload, and no drain of its stores between the steps
        const bool carry_out = MKACC_QUADP_CARRY && ps.ppw == 1u && iw == ps.wg && t + 1u < r.t1 &&
                               (t + 1u) / r.n == t / r.n;
        // the two-per-CU form at dg = 4 loads one share at a time (a batch of four would
        // spill at 256 VGPRs)
        constexpr uint32_t kNb = OCC == 2 && DG >= 4 ? 1u : quad::kBatch;
        quad::quadp_step<DG, METHOD, kNb>(run_args(a, r, t), s, xs, ps, t - r.t0, (t - 1u) / r.n / ps.ppw != iw,
                                     (t + quad::kSlots) / r.n / ps.ppw != iw, carried, carry_out, carry);
        vcc_fence();   // the loop branch follows the step's last reductions
        if (!carry_out) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        carried = carry_out;
    }
}
template <int DG, int METHOD>
__global__ __launch_bounds__(256, 1) void mk_quadp_run_kernel(StepArgs a, LatdRun r, QuadArgs qa) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    quadp_run<DG, METHOD, 1>(a, r, qa, smem);
}
template <int DG, int METHOD>
__global__ __launch_bounds__(256, 2) void mk_quadp2_run_kernel(StepArgs a, LatdRun r, QuadArgs qa) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    quadp_run<DG, METHOD, 2>(a, r, qa, smem);
}

template <int DG>
const void* pick_quad(int method, bool first, int occ) {
    if (occ == 2) {
        // dg = 5 needs more than 256 registers per lane (it would spill); the first step
        // runs mk_quad_kernel at either occupancy (the engine's StepChain::step)
        if constexpr (DG > 4) {
            return nullptr;
        } else {
            if (first) return nullptr;
            return method == XZW ? (const void*)mk_quad2_kernel<DG, XZW, false> : (const void*)mk_quad2_kernel<DG, XZW_B, false>;
        }
    }
    if (method == XZW) return first ? (const void*)mk_quad_kernel<DG, XZW, true> : (const void*)mk_quad_kernel<DG, XZW, false>;
    return first ? (const void*)mk_quad_kernel<DG, XZW_B, true> : (const void*)mk_quad_kernel<DG, XZW_B, false>;
}
template <int DG>
const void* pick_quad_run(int method, int occ) {
    if (occ == 3) return method == XZW ? (const void*)mk_quadp_run_kernel<DG, XZW> : (const void*)mk_quadp_run_kernel<DG, XZW_B>;
    if (occ == 4) {
        if constexpr (DG > 4) {
            return nullptr;
        } else {
            return method == XZW ? (const void*)mk_quadp2_run_kernel<DG, XZW> : (const void*)mk_quadp2_run_kernel<DG, XZW_B>;
        }
    }
    if (occ == 2) {
        if constexpr (DG > 4) {
            return nullptr;
        } else {
            return method == XZW ? (const void*)mk_quad2_run_kernel<DG, XZW> : (const void*)mk_quad2_run_kernel<DG, XZW_B>;
        }
    }
    return method == XZW ? (const void*)mk_quad_run_kernel<DG, XZW> : (const void*)mk_quad_run_kernel<DG, XZW_B>;
}
