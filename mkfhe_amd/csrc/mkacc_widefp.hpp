// mkacc_widefp.hpp -- FP64 arithmetic for the 64-bit word path when Q < 2^50
// (SURVEY.md s8 config 5 stress: Q = 1125899906826241 = 2^50 - 16383).
// Included by mkacc_engine.hip after mkacc_wide.hpp; same structure as
// wide::step_kernel (one 256-thread workgroup per gate, 8 EVAL slots per
// thread, transforms in a 16 KiB LDS tile, radix-4 passes), but residues are
// held as exact integers in IEEE binary64 words, signed ("balanced"), and the
// modular product is
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
// made canonical where they leave the kernel, so the path is bit-exact.
#pragma once

namespace {

namespace widefp {

constexpr int kThreads = 256;
constexpr int kPer = kN / kThreads;   // 8 slots per thread

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
// the reference's centred coefficient (mk-acc.cpp:60-64): t < Q/2 ? t : t - Q for
// the canonical t == x (mod Q), i.e. the representative in [-(Q+1)/2, (Q-3)/2]
__device__ __forceinline__ double centred(double x, const FMod& m) {
    double d = red(x, m);
    d = d >= m.qhalf ? d - m.Q : d;
    return d < -m.qhalf - 1.0 ? d + m.Q : d;
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

// Forward NTT of the LDS tile, reference order (transformnat-impl.h:300-354),
// radix-4 passes as wide::ntt_fwd.  Twiddles balanced (|w| <= Q/2).  Each pass
// reduces its two first-stage a-inputs; with pass inputs below X Q the outputs
// stay below (1.75 + 5X/16) Q, whose fixed point is 2.55 Q; the last stage
// (a reduced) leaves < 1.7 Q.
__device__ __forceinline__ void ct(double& a, double& b, double w, const FMod& m) {
    const double T = mm(b, w, m);
    const double X = a;
    a = __dadd_rn(X, T);
    b = __dsub_rn(X, T);
}
// (the lane index is opaque to the optimiser: otherwise the twiddle addresses of
// every pass of every transform of the step are hoisted into registers and spilled)
__device__ __forceinline__ void ntt_fwd(double* a, const double* __restrict__ tw, const FMod& m) {
    const uint32_t tid = opaque_v(threadIdx.x);
    uint32_t mb = 1, logt = kLogN - 1;
    for (; logt >= 2; mb <<= 2, logt -= 2) {
        const uint32_t h = 1u << (logt - 1);
#pragma unroll
        for (int r = 0; r < kN / 4 / kThreads; ++r) {
            const uint32_t g = tid + r * kThreads;
            const uint32_t i = g >> (logt - 1), j0 = (i << (logt + 1)) + (g & (h - 1));
            double x0 = red(a[j0], m), x1 = red(a[j0 + h], m), x2 = a[j0 + 2 * h], x3 = a[j0 + 3 * h];
            const double w1 = tw[mb + i];
            ct(x0, x2, w1, m);
            ct(x1, x3, w1, m);
            ct(x0, x1, tw[2 * mb + 2 * i], m);
            ct(x2, x3, tw[2 * mb + 2 * i + 1], m);
            a[j0] = x0; a[j0 + h] = x1; a[j0 + 2 * h] = x2; a[j0 + 3 * h] = x3;
        }
        __syncthreads();
    }
    for (; mb < (uint32_t)kN; mb <<= 1, --logt) {
        const uint32_t t = 1u << logt;
#pragma unroll
        for (int r = 0; r < kN / 2 / kThreads; ++r) {
            const uint32_t b = tid + r * kThreads;
            const uint32_t i = b >> logt, j = (i << (logt + 1)) + (b & (t - 1));
            double x0 = red(a[j], m), x1 = a[j + t];
            ct(x0, x1, tw[mb + i], m);
            a[j] = x0;
            a[j + t] = x1;
        }
        __syncthreads();
    }
}

// Inverse GS without N^-1 (transformnat-impl.h:492-552 up to the scaling),
// radix-4 passes as wide::ntt_inv_noscale.  With pass inputs below X Q the
// outputs are x0 < 4X, x1 < 1 + X, x2 < 0.5 + X, x3 < 0.5 + (1 + X)/4; x0..x2
// are reduced, so the pass inputs stay below max(X0, 1.04) Q for an input
// bound X0 <= 1.13 (the rotated accumulator), and the second-stage difference
// below 4.5 Q.  Output of the last stage < 2.3 Q.
__device__ __forceinline__ void gs(double& a, double& b, double w, const FMod& m) {
    const double d = __dsub_rn(a, b);
    a = __dadd_rn(a, b);
    b = mm(d, w, m);
}
__device__ __forceinline__ void ntt_inv_noscale(double* a, const double* __restrict__ tw, const FMod& m) {
    const uint32_t tid = opaque_v(threadIdx.x);
    uint32_t mb = kN >> 1, logt = 0;
    for (; mb >= 2; mb >>= 2, logt += 2) {
        const uint32_t t = 1u << logt;
#pragma unroll
        for (int r = 0; r < kN / 4 / kThreads; ++r) {
            const uint32_t g = tid + r * kThreads;
            const uint32_t b = g >> logt, j0 = (b << (logt + 2)) + (g & (t - 1));
            double x0 = a[j0], x1 = a[j0 + t], x2 = a[j0 + 2 * t], x3 = a[j0 + 3 * t];
            gs(x0, x1, tw[mb + 2 * b], m);
            gs(x2, x3, tw[mb + 2 * b + 1], m);
            const double w2 = tw[(mb >> 1) + b];
            gs(x0, x2, w2, m);
            gs(x1, x3, w2, m);
            a[j0] = red(x0, m); a[j0 + t] = red(x1, m); a[j0 + 2 * t] = red(x2, m); a[j0 + 3 * t] = x3;
        }
        __syncthreads();
    }
    for (; mb >= 1; mb >>= 1, ++logt) {
        const uint32_t t = 1u << logt;
#pragma unroll
        for (int r = 0; r < kN / 2 / kThreads; ++r) {
            const uint32_t b = tid + r * kThreads;
            const uint32_t i = b >> logt, j = (i << (logt + 1)) + (b & (t - 1));
            double x0 = a[j], x1 = a[j + t];
            gs(x0, x1, tw[mb + i], m);
            a[j] = x0;
            a[j + t] = x1;
        }
        __syncthreads();
    }
}

// SignedDigitDecompose (mk-acc.cpp:54-80) through the offset word of
// wide::sdd_offset: D = centred(t) + C, 0 <= D < 2^53 (host: b * digitsG <= 52)
__device__ __forceinline__ uint64_t sdd_offset(double t, const FMod& m, double C) {
    return (uint64_t)__dadd_rn(centred(t, m), C);
}
// balanced digit i (1..dg) as a small signed double (the reference's r, before r < 0 ? r + Q)
__device__ __forceinline__ double sdd_digit(uint64_t D, uint32_t i, const wide::Sdd64& s) {
    const int64_t f = (int64_t)((D >> (s.gbits * i)) & ((s.half << 1) - 1));
    return (double)(f - (int64_t)s.half);
}

struct StepArgs {
    const double* acc_in;     // [B][k][N] EVAL (reference order), balanced
    double* acc_out;
    const uint32_t* cvals;    // [B] exponents c of this step, in [0, 2N)
    const double* key1;       // ev1 = (*ek)[u][0][i] : [dg][2][N], balanced
    const double* key2;       // ev2 = (*ek)[u][1][i] (XZW)
    const double* keys;       // evs = (*ek)[0][0][n]
    const double* pkey;       // [k][dg][N]
    const double* twf;        // forward table
    const double* twi;        // inverse table
    const double* psi;        // psi^e, e in [0, 2N)
    uint32_t k, index, dg;
    double ninv;              // N^-1, balanced
    double C;                 // SDD offset constant
    FMod m;
    wide::Sdd64 sd;
};

// d_i / f_i of AddToAccXZW{0,} for one slot (xzw.cpp:322-325, 375-378;
// xzw_B.cpp:311-314, 368-371).  Keys and monomials balanced (|.| <= Q/2), so
// each product is below 0.625 Q and the result below 2.75 Q.
template <int METHOD, bool FIRST>
__device__ __forceinline__ double key_eff(double k1, double k2, double ks, double tp, double tn, const FMod& m) {
    if (METHOD == XZW) {
        if (FIRST) return ks + (mm(k1, tp, m) - k1) + (mm(k2, tn, m) - k2);
        return k1 - mm(k2, tn, m);   // ev1 - ev2 X^-c
    }
    if (FIRST) return ks + (mm(k1, tp, m) - k1);
    return k1;
}

// One accumulator step of one gate per workgroup (the algebra of
// wide::step_kernel).  Stored accumulators are reduced (|.| <= Q/2 + 2); the
// digit-NTT outputs are reduced before the MACs (one reduction serves the d_i
// and the P products), so every product has P <= 1.4 and every running sum is
// reduced after each add.
// Memory goes through buffer resources: a slot's byte offset is the lane part
// t * 8 (one VGPR) plus a wave-uniform part (slot, digit, party) in an SGPR, so
// no 64-bit address is kept per slot and array (with plain pointers the
// compiler hoisted ~60 of them and spilled at 4 workgroups per CU).
__device__ __forceinline__ uint32_t odd_exp(uint32_t j) { return 2u * (__brev(j) >> (32 - kLogN)) + 1u; }
__device__ __forceinline__ double ldd(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(double, bload2(r, voff, soff));
}
__device__ __forceinline__ void std8(__amdgpu_buffer_rsrc_t r, double x, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x), r, voff, soff, 0);
}
__device__ __forceinline__ double mono(__amdgpu_buffer_rsrc_t psi, uint32_t e, uint32_t oj) {
    return ldd(psi, ((e * opaque_v(oj)) & (2u * kN - 1u)) * 8u, 0);   // recomputed per use, not hoisted
}

#ifndef MKACC_WFP_WG_PER_CU
#define MKACC_WFP_WG_PER_CU 4
#endif
template <int METHOD, bool FIRST>
__global__ __launch_bounds__(kThreads, MKACC_WFP_WG_PER_CU) void step_kernel(StepArgs a) {
    __shared__ double tile[kN];
    __shared__ uint64_t dtile[kN];
    const uint32_t gate = blockIdx.x, t = threadIdx.x;
    const FMod& m = a.m;
    const uint32_t c = a.cvals[gate], cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k, index = a.index, dg = a.dg;
    constexpr uint32_t polyB = kN * 8u, slotB = kThreads * 8u;
    const uint32_t vo = t * 8u;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB);
    const __amdgpu_buffer_rsrc_t rk1 = make_rsrc(a.key1, dg * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rk2 = make_rsrc(a.key2, dg * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rks = make_rsrc(a.keys, dg * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rpk = make_rsrc(a.pkey, k * dg * polyB);
    const __amdgpu_buffer_rsrc_t rpsi = make_rsrc(a.psi, 2 * polyB);
    double sv[kPer];
#pragma unroll
    for (int e = 0; e < kPer; ++e) sv[e] = 0.0;
#ifndef MKACC_WFP_HOIST_MONO
#define MKACC_WFP_HOIST_MONO 1
#endif
    // X^-c at this thread's slots: the same for every digit and party of the step,
    // gathered once (instead of (k+1) dg times) and kept in 16 VGPRs
    double mn[kPer];
    if (METHOD == XZW && MKACC_WFP_HOIST_MONO) {
#pragma unroll
        for (int e = 0; e < kPer; ++e) mn[e] = mono(rpsi, cneg, odd_exp(t + kThreads * e));
    }
#ifndef MKACC_WFP_HOIST_MC
#define MKACC_WFP_HOIST_MC 1
#endif
    // X^c likewise (the k rotations; the KDM step's key combination)
    double mc[kPer];
    if (MKACC_WFP_HOIST_MC) {
#pragma unroll
        for (int e = 0; e < kPer; ++e) mc[e] = mono(rpsi, c, odd_exp(t + kThreads * e));
    }

    for (uint32_t tt = 1; tt <= k; ++tt) {
        const uint32_t u = index + tt < k ? index + tt : index + tt - k;
        double uj[kPer];
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const uint32_t j = t + kThreads * e;
            double x = ldd(rin, vo, u * polyB + e * slotB);
            uj[e] = FIRST ? 0.0 : x;
            if (!FIRST) x = mm(x, MKACC_WFP_HOIST_MC ? mc[e] : mono(rpsi, c, odd_exp(j)), m) - x;   // acc (X^c - 1)  (xzw.cpp:336-338)
            tile[j] = x;
        }
        __syncthreads();
        ntt_inv_noscale(tile, a.twi, m);
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const uint32_t j = t + kThreads * e;
            dtile[j] = sdd_offset(mm(tile[j], a.ninv, m), m, a.C);
        }
        for (uint32_t i = 0; i < dg; ++i) {
            __syncthreads();
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint32_t j = t + kThreads * e;
                tile[j] = sdd_digit(dtile[j], i + 1, a.sd);
            }
            __syncthreads();
            ntt_fwd(tile, a.twf, m);
            const uint32_t ko = i * 2 * polyB, po = (u * dg + i) * polyB;
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint32_t j = t + kThreads * e, so = e * slotB;
                const double g = red(tile[j], m);
                const double tp = FIRST ? (MKACC_WFP_HOIST_MC ? mc[e] : mono(rpsi, c, odd_exp(j))) : 0.0;
                const double tn = METHOD == XZW ? (MKACC_WFP_HOIST_MONO ? mn[e] : mono(rpsi, cneg, odd_exp(j))) : 0.0;
                const double d = key_eff<METHOD, FIRST>(ldd(rk1, vo, ko + so), METHOD == XZW ? ldd(rk2, vo, ko + so) : 0.0,
                                                        FIRST ? ldd(rks, vo, ko + so) : 0.0, tp, tn, m);
                uj[e] = red(uj[e] + mm(g, d, m), m);                    // <g^-1(c), d_i>
                sv[e] = red(sv[e] + mm(g, ldd(rpk, vo, po + so), m), m);   // <g^-1(c), P[u]_i>
            }
        }
#pragma unroll
        for (int e = 0; e < kPer; ++e) std8(rout, uj[e], vo, u * polyB + e * slotB);
    }

    // second half of HbProd: iNTT(sumV) -> SDD -> NTT -> acc[index] += <., f>  (xzw.cpp:272-289)
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kPer; ++e) tile[t + kThreads * e] = sv[e];
    __syncthreads();
    ntt_inv_noscale(tile, a.twi, m);
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
        const uint32_t j = t + kThreads * e;
        dtile[j] = sdd_offset(mm(tile[j], a.ninv, m), m, a.C);
    }
    // acc[index] was stored by this thread in its party pass
    double keep[kPer];
#pragma unroll
    for (int e = 0; e < kPer; ++e) keep[e] = ldd(rout, vo, index * polyB + e * slotB);
    for (uint32_t i = 0; i < dg; ++i) {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const uint32_t j = t + kThreads * e;
            tile[j] = sdd_digit(dtile[j], i + 1, a.sd);
        }
        __syncthreads();
        ntt_fwd(tile, a.twf, m);
        const uint32_t ko = i * 2 * polyB + polyB;   // f_i follows d_i inside [dg][2][N]
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const uint32_t j = t + kThreads * e, so = e * slotB;
            const double tp = FIRST ? (MKACC_WFP_HOIST_MC ? mc[e] : mono(rpsi, c, odd_exp(j))) : 0.0;
            const double tn = METHOD == XZW ? (MKACC_WFP_HOIST_MONO ? mn[e] : mono(rpsi, cneg, odd_exp(j))) : 0.0;
            const double f = key_eff<METHOD, FIRST>(ldd(rk1, vo, ko + so), METHOD == XZW ? ldd(rk2, vo, ko + so) : 0.0,
                                                    FIRST ? ldd(rks, vo, ko + so) : 0.0, tp, tn, m);
            keep[e] = red(keep[e] + mm(red(tile[j], m), f, m), m);
        }
    }
#pragma unroll
    for (int e = 0; e < kPer; ++e) std8(rout, keep[e], vo, index * polyB + e * slotB);
}

// batch prologue / epilogue: canonical u64 words <-> balanced doubles
// device entry point: a word >= Q raises `bad` (mkacc_sync reports MKACC_E_RANGE)
// and is replaced by 0, so every value stays inside the exactness bounds
__global__ void to_balanced_kernel(const uint64_t* __restrict__ in, double* __restrict__ out, size_t count, FMod m,
                                   uint64_t Q, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    uint64_t x = in[idx];
    if (x >= Q) {
        *bad = 1u;
        x = 0;
    }
    out[idx] = balanced(x, m);
}
__global__ void to_canonical_kernel(const double* __restrict__ in, uint64_t* __restrict__ out, size_t count, FMod m) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < count) out[idx] = canon(in[idx], m);
}

// primitive kernels for parity tests: one polynomial per workgroup, canonical in/out
__global__ __launch_bounds__(kThreads) void ntt_fwd_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                            const double* __restrict__ tw, FMod m) {
    __shared__ double tile[kN];
    const size_t base = (size_t)blockIdx.x * kN;
    for (int e = 0; e < kPer; ++e) tile[threadIdx.x + kThreads * e] = balanced(in[base + threadIdx.x + kThreads * e], m);
    __syncthreads();
    ntt_fwd(tile, tw, m);
    for (int e = 0; e < kPer; ++e) out[base + threadIdx.x + kThreads * e] = canon(tile[threadIdx.x + kThreads * e], m);
}
__global__ __launch_bounds__(kThreads) void ntt_inv_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                            const double* __restrict__ tw, FMod m, double ninv) {
    __shared__ double tile[kN];
    const size_t base = (size_t)blockIdx.x * kN;
    for (int e = 0; e < kPer; ++e) tile[threadIdx.x + kThreads * e] = balanced(in[base + threadIdx.x + kThreads * e], m);
    __syncthreads();
    ntt_inv_noscale(tile, tw, m);
    for (int e = 0; e < kPer; ++e) {
        const uint32_t j = threadIdx.x + kThreads * e;
        out[base + j] = canon(mm(tile[j], ninv, m), m);
    }
}

}  // namespace widefp

}  // namespace
