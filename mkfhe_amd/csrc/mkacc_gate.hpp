// mkacc_gate.hpp -- gate head and tail kernels around EvalAcc: the rest of
// BinFHEScheme::EvalBinGate for MK-NTRU (binfhe-base-scheme.cpp:467-515) and
// MK-LWE (binfhe-base-scheme.cpp:380-463).  Included by mkacc_engine.hip.
//
//   head (element-wise):  MNTRU  ct = ctNAND - (ct1 + ct2) mod q
//                         MK-LWE ct = (0, 5q/8) - (ct1 + ct2) mod q, ModSwitch to 2N,
//                                c = -a mod 2N, test vector rotated by b
//   EvalAcc (the step kernels)
//   tail:  extract_kernel   Transpose + iNTT + ModSwitch(qKS) + base-Bks digits
//          ks_mntru_kernel  KeySwitch2 as a digit x key GEMM (mntru-pke.cpp:763-823)
//          ks_mklwe_kernel  KeySwitch as a digit-selected row gather (mklwe-pke.cpp:260-298)
#pragma once

namespace {

// RoundqQ (mntru-pke.cpp:11-16, mklwe-pke.cpp): floor(0.5 + v*q/Q) in IEEE
// double, evaluated left to right exactly as the reference, then mod q.
__device__ __forceinline__ uint32_t round_qQ(uint32_t v, uint32_t q, uint32_t Q) {
    const double x = __dadd_rn(0.5, __ddiv_rn(__dmul_rn((double)v, (double)q), (double)Q));
    const uint32_t r = (uint32_t)floor(x);
    return r >= q ? r - q : r;
}

// MNTRU head: out[b][s] = ctNAND[s] - (ct1[b][s] + ct2[b][s]) mod q  (EvalAddEq/EvalSubEq,
// mntru-pke.cpp:826-838).  s over k*n.
__global__ void mntru_head_kernel(const uint32_t* __restrict__ ct_nand, const uint32_t* __restrict__ ct1,
                                  const uint32_t* __restrict__ ct2, uint32_t* __restrict__ out, uint32_t B,
                                  uint32_t kn, uint32_t q, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)B * kn) return;
    const uint32_t s = (uint32_t)(idx % kn);
    const uint32_t x1 = ct1[idx], x2 = ct2[idx], a = ct_nand[s];
    if (x1 >= q || x2 >= q || a >= q) *bad = 1u;
    uint32_t t = x1 + x2;
    t = t >= q ? t - q : t;
    out[idx] = a >= t ? a - t : a + q - t;
}

// MK-LWE head (binfhe-base-scheme.cpp:394-406, 1026, mklwe-ciphertext.h:86-96):
//   a' = RoundqQ(0 - (a1 + a2), 2N, q),  c = (2N - a') mod 2N      -> c   [B][k][n]
//   b' = RoundqQ(5q/8 - (b1 + b2), 2N, q)                          -> bh  [B]
__global__ void mklwe_head_kernel(const uint32_t* __restrict__ a1, const uint32_t* __restrict__ b1,
                                  const uint32_t* __restrict__ a2, const uint32_t* __restrict__ b2,
                                  uint32_t* __restrict__ c, uint32_t* __restrict__ bh, uint32_t B, uint32_t kn,
                                  uint32_t q, uint32_t* __restrict__ bad) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t M = 2u * kN;
    if (idx < (size_t)B * kn) {
        if (a1[idx] >= q || a2[idx] >= q) *bad = 1u;
        uint32_t t = a1[idx] + a2[idx];
        t = t >= q ? t - q : t;
        const uint32_t at = t == 0 ? 0 : q - t;
        const uint32_t ams = round_qQ(at, M, q);
        c[idx] = ams == 0 ? 0 : M - ams;
    }
    if (idx < B) {
        if (b1[idx] >= q || b2[idx] >= q) *bad = 1u;
        uint32_t t = b1[idx] + b2[idx];
        t = t >= q ? t - q : t;
        const uint32_t b5 = (5u * q / 8u) % q;
        const uint32_t bt = b5 >= t ? b5 - t : b5 + q - t;
        bh[idx] = round_qQ(bt, M, q);
    }
}

// Accumulator initialisation in the device C4 layout (values pre-scaled by N^-1):
// party 0 = test vector NTT(Rx) (binfhe-base-scheme.cpp:1093-1115), times X^bh
// for MK-LWE (the reference rotates Rx in the coefficient domain, :1024-1043;
// multiplying the EVAL vector by psi^(bh (2 brv(j) + 1)) is the same product),
// parties u > 0 = 0.
__global__ void acc_init_kernel(uint32_t* __restrict__ acc, const uint32_t* __restrict__ tv,
                                const uint32_t* __restrict__ bh, const uint2* __restrict__ psi_img, uint32_t B,
                                uint32_t k, uint32_t Q) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)B * k * kN) return;
    const uint32_t pidx = (uint32_t)(idx % kN);
    const size_t poly = idx / kN;
    const uint32_t u = (uint32_t)(poly % k), b = (uint32_t)(poly / k);
    if (u != 0) {
        acc[idx] = 0;
        return;
    }
    uint32_t v = tv[pidx];
    if (bh) {
        // physical C4 index -> EVAL slot j = (lane << 5) | r
        const uint32_t r = ((pidx >> 8) << 2) | (pidx & 3u), ln = (pidx >> 2) & 63u;
        const uint32_t j = (ln << 5) | r;
        const uint32_t odd = ((__brev(j) >> 21) << 1) | 1u;
        const uint32_t e = (bh[b] * odd) & (2u * kN - 1u);
        const uint2 w = psi_img[psi_pos(e)];
        v = mul_shoup(v, w.x, w.y, Q);
    }
    acc[idx] = v;
}

struct TailConsts {
    uint32_t Q, qKS, baseKS, dks;
};

// Extraction (binfhe-base-scheme.cpp:498-506): per gate and party, Transpose
// (automorphism X -> X^-1) then iNTT of the accumulator; ModSwitch(qKS)
// (mntru-pke.cpp:359-374); base-Bks digits of every coefficient
// (KeySwitch2/KeySwitch loop, mntru-pke.cpp:784-790).  One wave per polynomial.
// Since the automorphism commutes with the transform, it is applied to the
// coefficients: b[0] = a[0], b[N - j] = -a[j].  The device accumulator is
// scaled by N^-1, so iNTT without N^-1 yields the true coefficients.
//   digits [B][k][dks][N] (u8)
__global__ __launch_bounds__(256) void extract_kernel(const uint32_t* __restrict__ acc, uint8_t* __restrict__ digits,
                                                      uint32_t npoly, const uint2* __restrict__ tw_inv,
                                                      const uint2* __restrict__ twl_inv, TailConsts tc) {
    __shared__ __attribute__((aligned(16))) uint32_t smem[4 * kLdsWords];
    const uint32_t l = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t p = blockIdx.x * 4 + wv;
    if (p >= npoly) return;
    uint32_t x[kRegs];
    load_c4(x, acc + (size_t)p * kN, l);
    ntt_inv(x, smem + wv * kLdsWords, tw_inv, twl_inv, l, tc.Q);
    uint8_t* dp = digits + (size_t)p * tc.dks * kN;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        const uint32_t j = jA(l, (uint32_t)r);                 // coefficient index of x[r]
        const uint32_t i = (kN - j) & (kN - 1u);
        const uint32_t v = (j == 0 || x[r] == 0) ? x[r] : tc.Q - x[r];
        uint32_t y = round_qQ(v, tc.qKS, tc.Q);
        for (uint32_t t = 0; t < tc.dks; ++t) {
            dp[(size_t)t * kN + i] = (uint8_t)(y % tc.baseKS);
            y /= tc.baseKS;
        }
    }
}

// MNTRU KeySwitch2 (mntru-pke.cpp:763-823) as a GEMM per party u:
//   out[b][u][i] = sum_l D[b][u][l] * K[u][l][i]  mod qKS,   l = t*N + j
// which equals the reference's sum of the pre-multiplied rows KSK2[u][D][l]
// because KeySwitchGen2 stores KSK2[u][d][l] = d * KSK2[u][1][l] mod qKS
// (mntru-pke.cpp:744-755).  64 gates x 64 outputs per 256-thread block, 4x4
// per thread, 32-bit sums (digits < 2^8, keys < 2^16) reduced every 128 l.
// Small batches split l over slices (blockIdx.z = u + k slice, lper l each, a multiple
// of 128): a slice writes its sums mod qKS to part[slice] and ks_sum_kernel adds them
// -- one STD128_MKNTRU gate had 24 blocks for 36.7 MB of key rows.
constexpr int kKsTile = 64, kKsChunk = 32;
__global__ __launch_bounds__(256) void ks_mntru_kernel(const uint8_t* __restrict__ D, const uint16_t* __restrict__ K,
                                                       uint32_t* __restrict__ out, uint32_t B, uint32_t k,
                                                       uint32_t L, uint32_t n_out, uint32_t n_pad, uint32_t qKS,
                                                       uint32_t qinv, uint32_t lper, uint32_t* __restrict__ part) {
    __shared__ uint32_t sD[kKsChunk][kKsTile + 1];   // [l][gate]
    __shared__ uint32_t sK[kKsChunk][kKsTile];       // [l][col]
    const uint32_t u = blockIdx.z % k, sl = blockIdx.z / k;
    const uint32_t lb = sl * lper, le = min(L, lb + lper);
    uint32_t* dst = part ? part + (size_t)sl * B * k * n_out : out;
    const uint32_t g0 = blockIdx.y * kKsTile, c0 = blockIdx.x * kKsTile;
    const uint32_t tx = threadIdx.x & 15u, ty = threadIdx.x >> 4;    // 16 x 16
    uint32_t acc[4][4] = {};
    const uint8_t* Du = D + (size_t)u * L;
    const uint16_t* Ku = K + (size_t)u * L * n_pad;
    for (uint32_t l0 = lb; l0 < le; l0 += kKsChunk) {
        // D tile: 64 gates x 32 l (bytes), one byte per thread-iteration
        for (uint32_t e = threadIdx.x; e < kKsTile * kKsChunk; e += 256) {
            const uint32_t g = e / kKsChunk, ll = e % kKsChunk;
            const uint32_t gb = g0 + g;
            sD[ll][g] = (gb < B && l0 + ll < le) ? Du[(size_t)gb * k * L + l0 + ll] : 0u;
        }
        for (uint32_t e = threadIdx.x; e < kKsChunk * kKsTile; e += 256) {
            const uint32_t ll = e / kKsTile, cc = e % kKsTile;
            sK[ll][cc] = (l0 + ll < le) ? Ku[(size_t)(l0 + ll) * n_pad + c0 + cc] : 0u;
        }
        __syncthreads();
#pragma unroll 8
        for (int ll = 0; ll < kKsChunk; ++ll) {
            uint32_t dv[4], kv[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) dv[a] = sD[ll][ty * 4 + a];
#pragma unroll
            for (int bq = 0; bq < 4; ++bq) kv[bq] = sK[ll][tx * 4 + bq];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int bq = 0; bq < 4; ++bq) acc[a][bq] = __umul24(dv[a], kv[bq]) + acc[a][bq];
        }
        __syncthreads();
        if ((((l0 - lb) / kKsChunk) & 3u) == 3u || l0 + kKsChunk >= le) {
            // every 128 l: sums stay below 128 * 2^8 * 2^16 = 2^31
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int bq = 0; bq < 4; ++bq) {
                    uint32_t v = acc[a][bq];
                    v -= __umulhi(v, qinv) * qKS;
                    acc[a][bq] = v >= qKS ? v - qKS : v;
                }
        }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const uint32_t gb = g0 + ty * 4 + a;
        if (gb >= B) continue;
#pragma unroll
        for (int bq = 0; bq < 4; ++bq) {
            const uint32_t col = c0 + tx * 4 + bq;
            if (col < n_out) dst[((size_t)gb * k + u) * n_out + col] = acc[a][bq];
        }
    }
}

// sum of the slices' partial sums (each < qKS) mod qKS into out
__global__ void ks_sum_kernel(const uint32_t* __restrict__ part, uint32_t* __restrict__ out, uint32_t slices,
                              uint32_t total, uint32_t qKS) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    uint32_t s = 0;
    for (uint32_t sl = 0; sl < slices; ++sl) s += part[(size_t)sl * total + i];   // slices x 2^16 < 2^32
    out[i] = s % qKS;
}

// MK-LWE KeySwitch (mklwe-pke.cpp:260-298): for every party u, coefficient j
// and digit t the row (u, j, D, t) of A is subtracted from a[u] and the entry
// of B from b.  One block per (gate, party); threads run over the n output
// columns and stream the dks*N digit-selected rows, 16 independent row loads
// in flight per thread (digits fetched 16 at a time, wave-uniform).  Sums of
// dks*N words < 2^16 stay below 2^32 (dks*N <= 2^16).  Small batches split l over
// slices (blockIdx.x = (b k + u) slices + slice, lper l each, a multiple of 16): a
// slice writes its sums mod qKS (not negated) to pa[slice] / pb[slice] and
// ks_mklwe_sum_kernel finishes them.
//   A [k][N][Bks][dks][n] u16, Bv [k][N][Bks][dks] u16, partial_b [B][k]
__global__ __launch_bounds__(256) void ks_mklwe_kernel(const uint8_t* __restrict__ D, const uint16_t* __restrict__ A,
                                                       const uint16_t* __restrict__ Bv, uint32_t* __restrict__ out_a,
                                                       uint32_t* __restrict__ partial_b, uint32_t k, uint32_t n_out,
                                                       uint32_t baseKS, uint32_t dks, uint32_t qKS, uint32_t B,
                                                       uint32_t slices, uint32_t lper, uint32_t* __restrict__ pa,
                                                       uint32_t* __restrict__ pb) {
    const uint32_t sl = blockIdx.x % slices, bu = blockIdx.x / slices;
    const uint32_t u = bu % k, b = bu / k;
    const uint32_t L = dks * kN, lb = sl * lper, le = min(L, lb + lper);
    const uint4* Dp = reinterpret_cast<const uint4*>(D + ((size_t)b * k + u) * L);
    const size_t rowbase = (size_t)u * kN * baseKS;     // row of (u, j=0, d=0, t=0) / dks
    for (uint32_t c0 = 0; c0 < n_out; c0 += 256) {
        const uint32_t c = c0 + threadIdx.x;
        const bool on = c < n_out;
        uint32_t s = 0, sb = 0;
        for (uint32_t l0 = lb; l0 < le; l0 += 16) {
            const uint4 dv = Dp[l0 >> 4];
            const uint32_t dw[4] = {(uint32_t)__builtin_amdgcn_readfirstlane(dv.x),
                                    (uint32_t)__builtin_amdgcn_readfirstlane(dv.y),
                                    (uint32_t)__builtin_amdgcn_readfirstlane(dv.z),
                                    (uint32_t)__builtin_amdgcn_readfirstlane(dv.w)};
            uint32_t v[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const uint32_t l = l0 + e, t = l / kN, j = l % kN;     // digits stored [t][j]
                const uint32_t d = (dw[e >> 2] >> (8 * (e & 3))) & 0xFFu;
                const size_t row = ((rowbase + (size_t)j * baseKS + d) * dks) + t;
                v[e] = on ? A[row * n_out + c] : 0u;
                if (c0 == 0 && threadIdx.x == 0) sb += Bv[row];
            }
#pragma unroll
            for (int e = 0; e < 16; ++e) s += v[e];
        }
        s %= qKS;
        if (pa) {
            if (on) pa[((size_t)sl * B * k + (size_t)b * k + u) * n_out + c] = s;
            if (c0 == 0 && threadIdx.x == 0) pb[(size_t)sl * B * k + (size_t)b * k + u] = sb % qKS;
            continue;
        }
        if (on) out_a[((size_t)b * k + u) * n_out + c] = s == 0 ? 0 : qKS - s;
        if (c0 == 0 && threadIdx.x == 0) partial_b[(size_t)b * k + u] = sb % qKS;
    }
}

// the slices of ks_mklwe_kernel: out_a = -(sum of pa) and partial_b = sum of pb, mod qKS
__global__ void ks_mklwe_sum_kernel(const uint32_t* __restrict__ pa, const uint32_t* __restrict__ pb,
                                    uint32_t* __restrict__ out_a, uint32_t* __restrict__ partial_b, uint32_t slices,
                                    uint32_t Bk, uint32_t n_out, uint32_t qKS) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, total = Bk * n_out;
    if (i < total) {
        uint32_t s = 0;
        for (uint32_t sl = 0; sl < slices; ++sl) s += pa[(size_t)sl * total + i];
        s %= qKS;
        out_a[i] = s == 0 ? 0 : qKS - s;
    }
    if (i < Bk) {
        uint32_t s = 0;
        for (uint32_t sl = 0; sl < slices; ++sl) s += pb[(size_t)sl * Bk + i];
        partial_b[i] = s % qKS;
    }
}

// b = b0 - sum_u partial_b[g][u] mod qKS
__global__ void ks_mklwe_b_kernel(const uint32_t* __restrict__ partial_b, uint32_t* __restrict__ out_b, uint32_t B,
                                  uint32_t k, uint32_t qKS, uint32_t b0) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= B) return;
    uint32_t sb = 0;
    for (uint32_t u = 0; u < k; ++u) {
        sb += partial_b[(size_t)g * k + u];
        sb = sb >= qKS ? sb - qKS : sb;
    }
    out_b[g] = b0 >= sb ? b0 - sb : b0 + qKS - sb;
}

}  // namespace
