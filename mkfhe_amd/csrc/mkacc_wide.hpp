// mkacc_wide.hpp -- the 64-bit-word accumulator path: EvalAcc for a ring
// modulus 2^27 <= Q < 2^61 (the reference at NATIVE_SIZE=64, where
// MAX_MODULUS_SIZE is 60; SURVEY.md s8 config 5 stress: Q = 1125899906826241,
// B_g = 2^10).  Included by mkacc_engine.hip.
//
// A residue no longer fits a 32-bit lane word, so the register-resident
// one-wave-per-gate design of the 27-bit kernel (mkacc_device.hpp) does not
// carry over: here one 256-thread workgroup owns one gate, each thread holds
// 8 EVAL slots (j = t + 256 e, coalesced key/accumulator streams), and every
// transform runs in a 16 KiB LDS tile (two stages per barrier).
// Products are 64 x 64 -> 128-bit: Shoup with precomputed companions for the
// fixed operands (twiddles, monomial powers psi^e, N^-1; built from 32-bit
// limb multiply-adds, lazy butterflies) and Montgomery for
// the data x key products (keys stored as K * 2^64 mod Q at upload; the key
// combinations are linear, so d_i, f_i stay in that form).  Every stored result is a canonical
// residue, so the same reorderings as the 27-bit kernel are bit-exact.
#pragma once

namespace {

namespace wide {

constexpr int kThreads = 256;
constexpr int kPer = kN / kThreads;   // 8 slots per thread

struct Mod64 {
    uint64_t Q;
    uint64_t mu;    // floor(2^(2L) / Q)
    uint32_t L;     // 2^(L-1) <= Q < 2^L
    uint64_t qp;    // -Q^-1 mod 2^64 (Montgomery, R = 2^64)
};

__device__ __forceinline__ uint64_t add(uint64_t a, uint64_t b, uint64_t Q) {
    const uint64_t s = a + b;
    return s >= Q ? s - Q : s;
}
__device__ __forceinline__ uint64_t sub(uint64_t a, uint64_t b, uint64_t Q) {
    return a >= b ? a - b : a + Q - b;
}
// Shoup product from 32-bit limbs with a truncated quotient.  For any 64-bit x,
// w < Q and wp = floor(w 2^64 / Q): q~ = xh*ph + hi(xh*pl) + hi(xl*ph + lo(xh*pl))
// drops only the xl*pl partial product and one low carry, so q~ = q - delta with
// q = floor(x wp / 2^64) and delta in {0, 1}; exact Shoup gives x w - q Q in
// [0, 2Q), hence T = x w - q~ Q lies in [0, 3Q).  T is formed as the low 64 bits
// of x w + q~ (2^64 - Q): two full products for the low word, four low-word
// products (one v_mad_u64_u32 each) for the high word.  11 multiply-adds in all,
// against ~4 wide products plus corrections for the 128-bit form.
__device__ __forceinline__ uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint64_t shoup3(uint64_t x, uint64_t w, uint64_t wp, uint64_t nQ) {
    const uint32_t xl = lo32(x), xh = hi32(x);
    const uint64_t t1 = mad64(xh, lo32(wp), 0);
    const uint64_t s = mad64(xl, hi32(wp), lo32(t1));
    const uint64_t q = mad64(xh, hi32(wp), hi32(t1)) + hi32(s);
    const uint64_t A = mad64(lo32(q), lo32(nQ), mad64(xl, lo32(w), 0));
    uint64_t h = mad64_pin<false>(xh, lo32(w), hi32(A));
    h = mad64_pin<false>(xl, hi32(w), h);
    h = mad64_pin<true>(hi32(q), lo32(nQ), h);
    h = mad64_pin<true>(lo32(q), hi32(nQ), h);
    return ((uint64_t)lo32(h) << 32) | lo32(A);
}
__device__ __forceinline__ uint64_t csub(uint64_t x, uint64_t m) { return x >= m ? x - m : x; }
// x * w mod Q, canonical (any 64-bit x)
__device__ __forceinline__ uint64_t mul_shoup(uint64_t x, uint64_t w, uint64_t wp, uint64_t Q) {
    return csub(csub(shoup3(x, w, wp, 0 - Q), Q), Q);
}
// a * b mod Q for a, b < Q (Barrett, HAC 14.42 with base 2)
__device__ __forceinline__ uint64_t mulmod(uint64_t a, uint64_t b, const Mod64& m) {
    const unsigned __int128 x = (unsigned __int128)a * b;
    const uint64_t q1 = (uint64_t)(x >> (m.L - 1));
    const uint64_t q2 = (uint64_t)(((unsigned __int128)q1 * m.mu) >> (m.L + 1));
    uint64_t r = (uint64_t)x - q2 * m.Q;   // [0, 3Q)
    r = r >= m.Q ? r - m.Q : r;
    return r >= m.Q ? r - m.Q : r;
}

// a * b * 2^-64 mod Q for a < 6Q, b < Q (Montgomery reduction of the 128-bit
// product): the keys are stored as K * 2^64 mod Q, so montmul(g, K') = g * K.
// t + m Q is divisible by 2^64, its low word is 0 iff t's is, and the quotient
// is below Q + 6Q^2 / 2^64 < 2Q (Q < 2^61), so one subtraction makes it canonical.
__device__ __forceinline__ uint64_t montmul(uint64_t a, uint64_t b, const Mod64& m) {
    const uint64_t lo = a * b, hi = __umul64hi(a, b);
    const uint64_t mq = lo * m.qp;
    const uint64_t r = hi + __umul64hi(mq, m.Q) + (lo != 0);
    return r >= m.Q ? r - m.Q : r;
}

struct Sdd64 {
    uint64_t qhalf;   // Q >> 1
    uint64_t cpos;    // C = sum_{i < digitsG} 2^(b-1) 2^(b i)
    uint64_t cneg;    // C - Q (mod 2^64)
    uint64_t half;    // 2^(b-1)
    uint32_t gbits;   // b
};
// offset word D = centred(t) + C; balanced digit i = bfe(D, b i, b) - 2^(b-1)
// (closed form of mk-acc.cpp:54-80, proof in mkacc_device.hpp; b * digitsG <= 63)
__device__ __forceinline__ uint64_t sdd_offset(uint64_t t, const Sdd64& s) {
    return t + (t < s.qhalf ? s.cpos : s.cneg);
}
// digit i (1..dg) as the reference emits it: r < 0 ? r + Q : r
__device__ __forceinline__ uint64_t sdd_digit(uint64_t D, uint32_t i, const Sdd64& s, uint64_t Q) {
    const uint64_t f = (D >> (s.gbits * i)) & ((s.half << 1) - 1);
    return f >= s.half ? f - s.half : f + Q - s.half;
}

// Lazy CT / GS butterflies (Q < 2^61, so 6Q < 2^64).  Forward: values stay
// in [0, 6Q) -- a is brought under 3Q, T = shoup3(b) < 3Q, outputs X + T and
// X + 3Q - T.  Inverse: values stay in [0, 3Q) -- a + b reduced once by 3Q,
// b' = shoup3(a - b + 3Q) < 3Q.  One 64-bit conditional subtraction per
// butterfly instead of three; results are reduced where they are consumed
// (montmul accepts g < 6Q, mul_shoup any word, canon6 for the primitives).
struct Lazy {
    uint64_t Q3, nQ;
};
__device__ __forceinline__ void ct(uint64_t& a, uint64_t& b, ulonglong2 w, const Lazy& z) {
    const uint64_t X = csub(a, z.Q3);
    const uint64_t T = shoup3(b, w.x, w.y, z.nQ);
    a = X + T;
    b = X + z.Q3 - T;
}
__device__ __forceinline__ void gs(uint64_t& a, uint64_t& b, ulonglong2 w, const Lazy& z) {
    const uint64_t d = a + z.Q3 - b;
    a = csub(a + b, z.Q3);
    b = shoup3(d, w.x, w.y, z.nQ);
}
// [0, 6Q) -> [0, Q)
__device__ __forceinline__ uint64_t canon6(uint64_t x, uint64_t Q) {
    return csub(csub(csub(x, 3 * Q), Q), Q);
}

// NTT of the LDS tile a[N], reference order (transformnat-impl.h:300-354):
// stage m: butterfly (j, j+t) with table[m + i], t = N / 2m.  tw = {w, w'}.
// Stages are taken two at a time (radix-4 groups j0 + {0, t/2, t, 3t/2}: one
// barrier per pair), the last stage alone.
__device__ __forceinline__ void ntt_fwd(uint64_t* a, const ulonglong2* __restrict__ tw, uint64_t Q) {
    const Lazy z{3 * Q, 0 - Q};
    uint32_t m = 1, logt = kLogN - 1;                 // stage s: m = 2^s, t = 2^logt
    for (; logt >= 2; m <<= 2, logt -= 2) {          // stages (s, s+1), t >= 4
        const uint32_t h = 1u << (logt - 1);          // t / 2 = groups per block
#pragma unroll
        for (int r = 0; r < kN / 4 / kThreads; ++r) {
            const uint32_t g = threadIdx.x + r * kThreads;
            const uint32_t i = g >> (logt - 1), j0 = (i << (logt + 1)) + (g & (h - 1));
            uint64_t x0 = a[j0], x1 = a[j0 + h], x2 = a[j0 + 2 * h], x3 = a[j0 + 3 * h];
            const ulonglong2 w1 = tw[m + i];
            ct(x0, x2, w1, z);
            ct(x1, x3, w1, z);
            ct(x0, x1, tw[2 * m + 2 * i], z);
            ct(x2, x3, tw[2 * m + 2 * i + 1], z);
            a[j0] = x0; a[j0 + h] = x1; a[j0 + 2 * h] = x2; a[j0 + 3 * h] = x3;
        }
        __syncthreads();
    }
    // remaining stages with t = 2 then t = 1 (N = 2^11: one pair above leaves t = 1 only)
    for (; m < (uint32_t)kN; m <<= 1, --logt) {
        const uint32_t t = 1u << logt;
#pragma unroll
        for (int r = 0; r < kN / 2 / kThreads; ++r) {
            const uint32_t b = threadIdx.x + r * kThreads;
            const uint32_t i = b >> logt, j = (i << (logt + 1)) + (b & (t - 1));
            ct(a[j], a[j + t], tw[m + i], z);
        }
        __syncthreads();
    }
}
// Inverse GS without the N^-1 factor (transformnat-impl.h:492-552 up to the
// scaling): stage pairs (t, 2t) as radix-4 groups j0 + {0, t, 2t, 3t}.
__device__ __forceinline__ void ntt_inv_noscale(uint64_t* a, const ulonglong2* __restrict__ tw, uint64_t Q) {
    const Lazy z{3 * Q, 0 - Q};
    uint32_t m = kN >> 1, logt = 0;                   // stage: m blocks, t = 2^logt
    for (; m >= 2; m >>= 2, logt += 2) {
        const uint32_t t = 1u << logt;
#pragma unroll
        for (int r = 0; r < kN / 4 / kThreads; ++r) {
            const uint32_t g = threadIdx.x + r * kThreads;
            const uint32_t b = g >> logt, j0 = (b << (logt + 2)) + (g & (t - 1));
            uint64_t x0 = a[j0], x1 = a[j0 + t], x2 = a[j0 + 2 * t], x3 = a[j0 + 3 * t];
            gs(x0, x1, tw[m + 2 * b], z);
            gs(x2, x3, tw[m + 2 * b + 1], z);
            const ulonglong2 w2 = tw[(m >> 1) + b];
            gs(x0, x2, w2, z);
            gs(x1, x3, w2, z);
            a[j0] = x0; a[j0 + t] = x1; a[j0 + 2 * t] = x2; a[j0 + 3 * t] = x3;
        }
        __syncthreads();
    }
    for (; m >= 1; m >>= 1, ++logt) {
        const uint32_t t = 1u << logt;
#pragma unroll
        for (int r = 0; r < kN / 2 / kThreads; ++r) {
            const uint32_t b = threadIdx.x + r * kThreads;
            const uint32_t i = b >> logt, j = (i << (logt + 1)) + (b & (t - 1));
            gs(a[j], a[j + t], tw[m + i], z);
        }
        __syncthreads();
    }
}

struct StepArgs {
    const uint64_t* acc_in;    // [B][k][N] EVAL (reference order)
    uint64_t* acc_out;
    const uint32_t* cvals;     // [B] exponents c of this step, in [0, 2N)
    const uint64_t* key1;      // ev1 = (*ek)[u][0][i] : [dg][2][N]
    const uint64_t* key2;      // ev2 = (*ek)[u][1][i] (XZW)
    const uint64_t* keys;      // evs = (*ek)[0][0][n]
    const uint64_t* pkey;      // [k][dg][N]
    const ulonglong2* twf;     // forward table {w, w'}
    const ulonglong2* twi;     // inverse table
    const ulonglong2* psi;     // psi^e, e in [0, 2N), with companions
    uint32_t k, index, dg;
    uint64_t ninv, ninvp;
    Mod64 m;
    Sdd64 sd;
};

// X^e at EVAL slot j: psi^(e (2 brv(j) + 1) mod 2N)  (transformnat-impl.h:705-760)
__device__ __forceinline__ ulonglong2 mono(const ulonglong2* psi, uint32_t e, uint32_t oj) {
    return psi[(e * oj) & (2u * kN - 1u)];
}

// d_i / f_i of AddToAccXZW{0,} for one slot (xzw.cpp:322-325, 375-378; xzw_B.cpp:311-314, 368-371)
template <int METHOD, bool FIRST>
__device__ __forceinline__ uint64_t key_eff(uint64_t k1, uint64_t k2, uint64_t ks, ulonglong2 tp, ulonglong2 tn,
                                            uint64_t Q) {
    if (METHOD == XZW) {
        if (FIRST) {
            const uint64_t t1 = sub(mul_shoup(k1, tp.x, tp.y, Q), k1, Q);
            const uint64_t t2 = sub(mul_shoup(k2, tn.x, tn.y, Q), k2, Q);
            return add(add(ks, t1, Q), t2, Q);
        }
        return sub(k1, mul_shoup(k2, tn.x, tn.y, Q), Q);   // ev1 - ev2 X^-c
    }
    if (FIRST) return add(ks, sub(mul_shoup(k1, tp.x, tp.y, Q), k1, Q), Q);
    return k1;
}

// One accumulator step of one gate per workgroup (same algebra as mk_step_kernel):
//   FIRST: acc <- HbProd(acc);  else acc <- acc + HbProd(acc (X^c - 1))
// Four workgroups per CU (<= 128 VGPRs): the offset words D of the digit
// decomposition live in a second LDS tile (each thread touches only its own
// slots, so it needs no barrier) and the EVAL exponents 2 brv(j) + 1 are
// recomputed where they are used.
__device__ __forceinline__ uint32_t odd_exp(uint32_t j) { return 2u * (__brev(j) >> (32 - kLogN)) + 1u; }

template <int METHOD, bool FIRST>
__global__ __launch_bounds__(kThreads, 4) void step_kernel(StepArgs a) {
    __shared__ uint64_t tile[kN];
    __shared__ uint64_t dtile[kN];
    const uint32_t gate = blockIdx.x, t = threadIdx.x;
    const uint64_t Q = a.m.Q;
    const uint32_t c = a.cvals[gate], cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k, index = a.index, dg = a.dg;
    const size_t key_f = (size_t)kN;   // f_i follows d_i inside [dg][2][N]
    uint64_t sv[kPer];
#pragma unroll
    for (int e = 0; e < kPer; ++e) sv[e] = 0;

    for (uint32_t tt = 1; tt <= k; ++tt) {
        const uint32_t u = index + tt < k ? index + tt : index + tt - k;
        const uint64_t* accu = a.acc_in + ((size_t)gate * k + u) * kN;
        uint64_t uj[kPer];
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const uint32_t j = t + kThreads * e;
            uint64_t x = accu[j];
            uj[e] = FIRST ? 0 : x;
            if (!FIRST) {   // acctemp = acc * (X^c - 1)   (xzw.cpp:336-338)
                const ulonglong2 w = mono(a.psi, c, odd_exp(j));
                x = sub(mul_shoup(x, w.x, w.y, Q), x, Q);
            }
            tile[j] = x;
        }
        __syncthreads();
        ntt_inv_noscale(tile, a.twi, Q);
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const uint32_t j = t + kThreads * e;
            dtile[j] = sdd_offset(mul_shoup(tile[j], a.ninv, a.ninvp, Q), a.sd);
        }
        for (uint32_t i = 0; i < dg; ++i) {
            __syncthreads();
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint32_t j = t + kThreads * e;
                tile[j] = sdd_digit(dtile[j], i + 1, a.sd, Q);
            }
            __syncthreads();
            ntt_fwd(tile, a.twf, Q);
            const size_t ko = (size_t)i * 2 * kN;
            const uint64_t* P = a.pkey + ((size_t)u * dg + i) * kN;
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint32_t j = t + kThreads * e;
                const uint64_t g = tile[j];   // [0, 6Q): montmul's range
                const ulonglong2 tp = FIRST ? mono(a.psi, c, odd_exp(j)) : ulonglong2{0, 0};
                const ulonglong2 tn = METHOD == XZW ? mono(a.psi, cneg, odd_exp(j)) : ulonglong2{0, 0};
                const uint64_t d = key_eff<METHOD, FIRST>(a.key1[ko + j], METHOD == XZW ? a.key2[ko + j] : 0,
                                                          FIRST ? a.keys[ko + j] : 0, tp, tn, Q);
                uj[e] = add(uj[e], montmul(g, d, a.m), Q);                // <g^-1(c), d_i>
                sv[e] = add(sv[e], montmul(g, P[j], a.m), Q);             // <g^-1(c), P[u]_i>
            }
        }
        // acc[index] is stored here too and read back by this thread for the f-part
        uint64_t* out = a.acc_out + ((size_t)gate * k + u) * kN;
#pragma unroll
        for (int e = 0; e < kPer; ++e) out[t + kThreads * e] = uj[e];
    }

    // second half of HbProd: iNTT(sumV) -> SDD -> NTT -> acc[index] += <., f>  (xzw.cpp:272-289)
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kPer; ++e) tile[t + kThreads * e] = sv[e];
    __syncthreads();
    ntt_inv_noscale(tile, a.twi, Q);
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
        const uint32_t j = t + kThreads * e;
        dtile[j] = sdd_offset(mul_shoup(tile[j], a.ninv, a.ninvp, Q), a.sd);
    }
    uint64_t* out = a.acc_out + ((size_t)gate * k + index) * kN;
    uint64_t keep[kPer];
#pragma unroll
    for (int e = 0; e < kPer; ++e) keep[e] = out[t + kThreads * e];
    for (uint32_t i = 0; i < dg; ++i) {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const uint32_t j = t + kThreads * e;
            tile[j] = sdd_digit(dtile[j], i + 1, a.sd, Q);
        }
        __syncthreads();
        ntt_fwd(tile, a.twf, Q);
        const size_t ko = (size_t)i * 2 * kN + key_f;
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            const uint32_t j = t + kThreads * e;
            const ulonglong2 tp = FIRST ? mono(a.psi, c, odd_exp(j)) : ulonglong2{0, 0};
            const ulonglong2 tn = METHOD == XZW ? mono(a.psi, cneg, odd_exp(j)) : ulonglong2{0, 0};
            const uint64_t f = key_eff<METHOD, FIRST>(a.key1[ko + j], METHOD == XZW ? a.key2[ko + j] : 0,
                                                      FIRST ? a.keys[ko + j] : 0, tp, tn, Q);
            keep[e] = add(keep[e], montmul(tile[j], f, a.m), Q);
        }
    }
#pragma unroll
    for (int e = 0; e < kPer; ++e) out[t + kThreads * e] = keep[e];
}

// primitive kernels for parity tests: one polynomial per workgroup
__global__ __launch_bounds__(kThreads) void ntt_fwd_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                            const ulonglong2* __restrict__ tw, uint64_t Q) {
    __shared__ uint64_t tile[kN];
    const size_t base = (size_t)blockIdx.x * kN;
    for (int e = 0; e < kPer; ++e) tile[threadIdx.x + kThreads * e] = in[base + threadIdx.x + kThreads * e];
    __syncthreads();
    ntt_fwd(tile, tw, Q);
    for (int e = 0; e < kPer; ++e) out[base + threadIdx.x + kThreads * e] = canon6(tile[threadIdx.x + kThreads * e], Q);
}
__global__ __launch_bounds__(kThreads) void ntt_inv_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                            const ulonglong2* __restrict__ tw, uint64_t Q,
                                                            uint64_t ninv, uint64_t ninvp) {
    __shared__ uint64_t tile[kN];
    const size_t base = (size_t)blockIdx.x * kN;
    for (int e = 0; e < kPer; ++e) tile[threadIdx.x + kThreads * e] = in[base + threadIdx.x + kThreads * e];
    __syncthreads();
    ntt_inv_noscale(tile, tw, Q);
    for (int e = 0; e < kPer; ++e) {
        const uint32_t j = threadIdx.x + kThreads * e;
        out[base + j] = mul_shoup(tile[j], ninv, ninvp, Q);
    }
}
__global__ void sdd_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint32_t count, uint32_t dg,
                           Sdd64 sd, uint64_t Q) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)count * kN) return;
    const size_t p = idx / kN, j = idx % kN;
    const uint64_t D = sdd_offset(in[idx], sd);
    for (uint32_t i = 0; i < dg; ++i) out[(p * dg + i) * kN + j] = sdd_digit(D, i + 1, sd, Q);
}

}  // namespace wide

}  // namespace
