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

constexpr int kWavesPerBlock = 4;
constexpr int kThreads = 64 * kWavesPerBlock;

enum { XZW = 0, XZW_B = 1 };

struct StepArgs {
    const uint32_t* acc_in;    // [B][k][N] C4, scaled by N^-1
    uint32_t* acc_out;         // [B][k][N]
    const uint32_t* cvals;     // [B] monomial exponents c of this step, in [0, 2N)
    const uint32_t* key1;      // ev1 = (*ek)[u][0][i] : [dg][2][N] C4
    const uint32_t* key2;      // ev2 = (*ek)[u][1][i] (XZW)
    const uint32_t* keys;      // evs = (*ek)[0][0][n] (first step)
    const uint32_t* pkey;      // [k][dg][N]
    uint32_t* sumv;            // [B][N] scratch: sumV of HbProd
    const uint2* tw_fwd;       // [N]
    const uint2* tw_inv;       // [N]
    const uint2* psi_pow;      // [2N] psi^e with Shoup companion
    uint32_t B, k, index;
    Mod m;
    uint32_t qhalf, gbits;
};

// EVAL exponent base of slot j = (lane << 5) | r: the reference stores
// a(psi^(2*brv(j)+1)) at position j (transformnat-impl.h:705-760).
__device__ __forceinline__ uint32_t slot_odd(uint32_t l, uint32_t r) {
    uint32_t j = (l << 5) | r;
    return ((__brev(j) >> 21) << 1) | 1u;
}

// One accumulator step for one gate per wavefront.
//   FIRST:  AddToAccXZW0 (mk-acc-xzw.cpp:347-381 / xzw_B.cpp:333-381): acc <- HbProd(acc)
//   else:   AddToAccXZW  (mk-acc-xzw.cpp:292-345 / xzw_B.cpp:281-330):
//           acc <- acc + HbProd(acc * (X^c - 1))
// HbProd is mk-acc-xzw.cpp:231-290.  All sums are exact mod Q, so the
// reordering below (d/f formed per slot, sums reduced lazily) is bit-exact.

// monomial value X^e at this lane's slot r (EVAL) with its Shoup companion
__device__ __forceinline__ uint2 mono_at(__amdgpu_buffer_rsrc_t pp, uint32_t c, uint32_t l, int r) {
    const uint32_t e = __umul24(c, slot_odd(l, (uint32_t)r)) & (2u * kN - 1u);
    const u32x2 t = bload2(pp, e * 8u, 0);
    return make_uint2(t.x, t.y);
}

// effective key word d_i / f_i of mk-acc-xzw(_B).cpp AddToAccXZW{,0}
template <int METHOD, bool FIRST>
__device__ __forceinline__ uint32_t key_eff(uint32_t k1, uint32_t k2, uint32_t ks, __amdgpu_buffer_rsrc_t pp,
                                            uint32_t c, uint32_t cneg, uint32_t l, int r, uint32_t Q) {
    if (METHOD == XZW) {
        const uint2 tn = mono_at(pp, cneg, l, r);
        if (FIRST) {
            // evs + ev1*(X^c-1) + ev2*(X^-c-1)          (xzw.cpp:375-378)
            const uint2 tp = mono_at(pp, c, l, r);
            const uint32_t t1 = sub_mod(mul_shoup(k1, tp.x, tp.y, Q), k1, Q);
            const uint32_t t2 = sub_mod(mul_shoup(k2, tn.x, tn.y, Q), k2, Q);
            return add_mod(add_mod(ks, t1, Q), t2, Q);
        }
        // ev1 - ev2*(X^-c - 1) - ev2  ==  ev1 - ev2*X^-c   (xzw.cpp:322-325)
        return sub_mod(k1, mul_shoup(k2, tn.x, tn.y, Q), Q);
    } else {
        if (FIRST) {
            // evs + ev1*(X^c-1)                            (xzw_B.cpp:368-371)
            const uint2 tp = mono_at(pp, c, l, r);
            return add_mod(ks, sub_mod(mul_shoup(k1, tp.x, tp.y, Q), k1, Q), Q);
        }
        return k1;                                        // (xzw_B.cpp:311-314)
    }
}

// Register-resident HbProd (mk-acc-xzw.cpp:231-290) for one gate per wave.
// The per-slot sums uj_u = sum_i g_i d_i, sumV = sum_u sum_i g_i P[u][i] and
// w = sum_i h_i f_i are kept as lazy 64-bit accumulators (v_mad_u64_u32) and
// reduced once; every operand is canonical, so a sum of up to 16 products
// stays below 2^58 (reduce58).
template <int DG, int METHOD, bool FIRST>
__device__ __forceinline__ void mac_digit(const uint32_t (&g)[kRegs], int i, uint32_t u, const StepArgs& a,
                                          uint64_t (&uj)[kRegs], uint64_t (&sv)[kRegs],
                                          __amdgpu_buffer_rsrc_t rk1, __amdgpu_buffer_rsrc_t rk2,
                                          __amdgpu_buffer_rsrc_t rks, __amdgpu_buffer_rsrc_t rpk,
                                          __amdgpu_buffer_rsrc_t rpp, uint32_t c, uint32_t cneg, uint32_t l) {
    const uint32_t Q = a.m.Q;
    const uint32_t polyB = kN * 4u, vo = l * 16u;
    const uint32_t koff = (uint32_t)(2 * i) * polyB;
    const uint32_t poff = (u * DG + (uint32_t)i) * polyB;
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) {
        const uint32_t go = gq * 1024u;
        const uint32_t lq = opaque_v(l);   // keep slot exponents from being hoisted (VGPR pressure)
        const u32x4 k1 = bload4(rk1, vo, koff + go);
        const u32x4 pk = bload4(rpk, vo, poff + go);
        u32x4 k2 = {0, 0, 0, 0}, ks = {0, 0, 0, 0};
        if (METHOD == XZW) k2 = bload4(rk2, vo, koff + go);
        if (FIRST) ks = bload4(rks, vo, koff + go);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * gq + e;
            const uint32_t deff = key_eff<METHOD, FIRST>(k1[e], k2[e], ks[e], rpp, c, cneg, lq, r, Q);
            uj[r] = mad64(g[r], deff, uj[r]);
            sv[r] = mad64(g[r], pk[e], sv[r]);
        }
        sched_fence();
    }
}

template <int METHOD, bool FIRST>
__device__ __forceinline__ void mac_index(const uint32_t (&h)[kRegs], int i, const StepArgs& a, uint64_t (&w)[kRegs],
                                          __amdgpu_buffer_rsrc_t rk1, __amdgpu_buffer_rsrc_t rk2,
                                          __amdgpu_buffer_rsrc_t rks, __amdgpu_buffer_rsrc_t rpp, uint32_t c,
                                          uint32_t cneg, uint32_t l) {
    const uint32_t Q = a.m.Q;
    const uint32_t polyB = kN * 4u, vo = l * 16u;
    const uint32_t koff = (uint32_t)(2 * i + 1) * polyB;
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) {
        const uint32_t go = gq * 1024u;
        const uint32_t lq = opaque_v(l);
        const u32x4 k1 = bload4(rk1, vo, koff + go);
        u32x4 k2 = {0, 0, 0, 0}, ks = {0, 0, 0, 0};
        if (METHOD == XZW) k2 = bload4(rk2, vo, koff + go);
        if (FIRST) ks = bload4(rks, vo, koff + go);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * gq + e;
            const uint32_t feff = key_eff<METHOD, FIRST>(k1[e], k2[e], ks[e], rpp, c, cneg, lq, r, Q);
            w[r] = mad64(h[r], feff, w[r]);
        }
        sched_fence();
    }
}

template <int DG, int METHOD, bool FIRST>
__global__ __launch_bounds__(kThreads, 2) void mk_step_kernel(StepArgs a) {
    // register allocation fits without spills when the digit loop is unrolled
    // for DG = 2 and kept rolled for DG >= 3 (measured, hipcc ROCm 7.2)
    constexpr int kDigitUnroll = DG == 2 ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t gate = blockIdx.x * kWavesPerBlock + wv;
    if (gate >= a.B) return;
    uint32_t* lds = smem + wv * kLdsWords;
    const Mod m = a.m;
    const uint32_t Q = m.Q;
    const uint32_t c = __builtin_amdgcn_readfirstlane(a.cvals[gate]);
    const uint32_t cneg = (2u * kN - c) & (2u * kN - 1u);
    const uint32_t k = a.k;
    const uint32_t polyB = kN * 4u;
    const uint32_t vo = l * 16u;   // lane offset of a C4 dwordx4

    const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.acc_in + (size_t)gate * k * kN, k * polyB);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(a.acc_out + (size_t)gate * k * kN, k * polyB);
    const __amdgpu_buffer_rsrc_t rk1 = make_rsrc(a.key1, DG * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rk2 = make_rsrc(a.key2, DG * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rks = make_rsrc(a.keys, DG * 2 * polyB);
    const __amdgpu_buffer_rsrc_t rpk = make_rsrc(a.pkey, k * DG * polyB);
    const __amdgpu_buffer_rsrc_t rpp = make_rsrc(a.psi_pow, 2u * kN * 8u);

    uint64_t sv[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) sv[r] = 0;

    for (uint32_t u = 0; u < k; ++u) {
        uint32_t x[kRegs];
#pragma unroll
        for (int gq = 0; gq < 8; ++gq) {
            const u32x4 t = bload4(rin, vo, u * polyB + gq * 1024u);
            x[4 * gq] = t.x; x[4 * gq + 1] = t.y; x[4 * gq + 2] = t.z; x[4 * gq + 3] = t.w;
        }
        if (!FIRST) {
            // acctemp = acc * (X^c - 1)                     (xzw.cpp:336-338)
#pragma unroll
            for (int r0 = 0; r0 < kRegs; r0 += 8) {
                const uint32_t lq = opaque_v(l);
#pragma unroll
                for (int r = r0; r < r0 + 8; ++r) {
                    const uint2 t = mono_at(rpp, c, lq, r);
                    x[r] = sub_mod(mul_shoup(x[r], t.x, t.y, Q), x[r], Q);
                }
                sched_fence();
            }
        }
        ntt_inv_noscale(x, lds, a.tw_inv, l, Q);
        // SignedDigitDecompose (mk-acc.cpp:54-80): digit 0 -> x, digits 1.. packed
        PackedDigits<DG> pd;
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            x[r] = pd.put(r, x[r], Q, a.qhalf, a.gbits);
            if ((r & 7) == 7) sched_fence();
        }
        uint64_t uj[kRegs];
#pragma unroll
        for (int r = 0; r < kRegs; ++r) uj[r] = 0;
#pragma unroll kDigitUnroll
        for (int i = 0; i < DG; ++i) {
            if (i > 0) {
#pragma unroll
                for (int r = 0; r < kRegs; ++r) x[r] = pd.get(r, i, Q);
            }
            ntt_fwd(x, lds, a.tw_fwd, l, Q);
#pragma unroll
            for (int r = 0; r < kRegs; ++r) x[r] = canon4(x[r], Q);
            mac_digit<DG, METHOD, FIRST>(x, i, u, a, uj, sv, rk1, rk2, rks, rpk, rpp, c, cneg, l);
        }
        // acc_u <- (FIRST ? 0 : acc_u) + uj_u   (xzw.cpp:270, 342-344); sumV reduced per party
#pragma unroll
        for (int gq = 0; gq < 8; ++gq) {
            u32x4 t = {0, 0, 0, 0};
            if (!FIRST) t = bload4(rin, vo, u * polyB + gq * 1024u);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * gq + e;
                t[e] = reduce58(uj[r] + t[e], m);
                sv[r] = reduce58(sv[r], m);
            }
            bstore4(t, rout, vo, u * polyB + gq * 1024u);
        }
    }

    // second half of HbProd: iNTT(sumV) -> SDD -> NTT -> acc[index] += <., f>
    uint32_t x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = (uint32_t)sv[r];
    ntt_inv_noscale(x, lds, a.tw_inv, l, Q);
    PackedDigits<DG> pd;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
        x[r] = pd.put(r, x[r], Q, a.qhalf, a.gbits);
        if ((r & 7) == 7) sched_fence();
    }
    uint64_t w[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) w[r] = 0;
#pragma unroll kDigitUnroll
    for (int i = 0; i < DG; ++i) {
        if (i > 0) {
#pragma unroll
            for (int r = 0; r < kRegs; ++r) x[r] = pd.get(r, i, Q);
        }
        ntt_fwd(x, lds, a.tw_fwd, l, Q);
#pragma unroll
        for (int r = 0; r < kRegs; ++r) x[r] = canon4(x[r], Q);
        mac_index<METHOD, FIRST>(x, i, a, w, rk1, rk2, rks, rpp, c, cneg, l);
    }
    const uint32_t ioff = a.index * polyB;
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) {
        u32x4 t = bload4(rout, vo, ioff + gq * 1024u);
#pragma unroll
        for (int e = 0; e < 4; ++e) t[e] = reduce58(w[4 * gq + e] + t[e], m);
        bstore4(t, rout, vo, ioff + gq * 1024u);
    }
}

// ---- batch prologue / epilogue kernels --------------------------------------

// c = floor(ct * 2N / q) (mk-acc-xzw.cpp:110,125) or c = ct (mk-acc-xzw_B.cpp:119,124),
// with c == 2N mapped to 0 (xzw.cpp:301).  Output layout [k*n][B].
__global__ void prep_c_kernel(const uint32_t* __restrict__ ct, uint32_t* __restrict__ cvals, uint32_t B,
                              uint32_t kn, uint32_t method, uint32_t q) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)B * kn) return;
    const uint32_t s = (uint32_t)(idx / B), b = (uint32_t)(idx % B);
    const uint32_t raw = ct[(size_t)b * kn + s];
    uint32_t c = method == XZW ? (uint32_t)(((uint64_t)raw * (2u * kN)) / q) : raw;
    if (c >= 2u * kN) c -= 2u * kN;
    cvals[idx] = c;
}

// reference EVAL order -> C4, multiplied by a constant (N^-1 on the way in, N on the way out)
__global__ void eval_to_c4_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t npoly,
                                  uint32_t s, uint32_t sp, uint32_t Q) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= npoly * kN) return;
    const size_t p = idx / kN;
    const uint32_t j = (uint32_t)(idx % kN);
    out[p * kN + c4_index(j)] = mul_shoup(in[idx], s, sp, Q);
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
                                                            uint32_t count, const uint2* __restrict__ twf, uint32_t Q) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t l = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t p = blockIdx.x * kWavesPerBlock + wv;
    if (p >= count) return;
    const uint32_t* src = in + (size_t)p * kN;
    uint32_t x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = src[jA(l, r)];
    ntt_fwd(x, smem + wv * kLdsWords, twf, l, Q);
    uint32_t* dst = out + (size_t)p * kN;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) dst[jC(l, r)] = canon4(x[r], Q);
}

__global__ __launch_bounds__(kThreads) void ntt_inv_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                            uint32_t count, const uint2* __restrict__ twi, uint32_t Q,
                                                            uint32_t ninv, uint32_t ninvp) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t l = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t p = blockIdx.x * kWavesPerBlock + wv;
    if (p >= count) return;
    const uint32_t* src = in + (size_t)p * kN;
    uint32_t x[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = src[jC(l, r)];
    ntt_inv_noscale(x, smem + wv * kLdsWords, twi, l, Q);
    uint32_t* dst = out + (size_t)p * kN;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) dst[jA(l, r)] = mul_shoup(x[r], ninv, ninvp, Q);
}

__global__ void sdd_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t count, uint32_t dg,
                           uint32_t Q, uint32_t qhalf, uint32_t gbits) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)count * kN) return;
    const size_t p = idx / kN, j = idx % kN;
    int32_t d = sdd_start(in[idx], Q, qhalf, gbits);
    for (uint32_t i = 0; i < dg; ++i) out[(p * dg + i) * kN + j] = sdd_next(d, Q, gbits);
}

// ---- kernel table -------------------------------------------------------------

using StepFn = void (*)(StepArgs);

template <int DG>
StepFn pick_step(int method, bool first) {
    if (method == XZW) return first ? mk_step_kernel<DG, XZW, true> : mk_step_kernel<DG, XZW, false>;
    return first ? mk_step_kernel<DG, XZW_B, true> : mk_step_kernel<DG, XZW_B, false>;
}

StepFn step_fn(int dg, int method, bool first) {
    switch (dg) {
        case 2: return pick_step<2>(method, first);
        case 3: return pick_step<3>(method, first);
        case 4: return pick_step<4>(method, first);
        case 5: return pick_step<5>(method, first);
        default: return nullptr;
    }
}

}  // namespace

// ---- context --------------------------------------------------------------------

struct mkacc_ctx {
    mkacc_params p{};
    int device = 0;
    int method_class = XZW;   // XZW or XZW_B
    uint32_t dg = 0, nk = 0;
    Mod mod{};
    uint32_t qhalf = 0, gbits = 0;
    uint32_t ninv = 0, ninvp = 0, nval = 0, nvalp = 0;
    hipStream_t stream = nullptr;
    uint2* d_twf = nullptr;
    uint2* d_twi = nullptr;
    uint2* d_psi = nullptr;
    uint32_t* d_keys = nullptr;   // [k][n+1][nk][dg][2][N] C4, scaled
    uint32_t* d_pkey = nullptr;   // [k][dg][N] C4, scaled
    bool have_keys = false;
    // batch workspace
    size_t ws_B = 0;
    uint32_t* d_acc0 = nullptr;
    uint32_t* d_acc1 = nullptr;
    uint32_t* d_cvals = nullptr;
    uint32_t* d_sumv = nullptr;
    // host-pointer API staging
    size_t io_B = 0;
    uint32_t* d_ct = nullptr;
    uint32_t* d_io = nullptr;
    std::mutex mu;
};

namespace {

size_t key_block_words(const mkacc_ctx* c) { return (size_t)c->nk * c->dg * 2 * kN; }

// device key block of step (u, i) (i == n: the KDM key evs)
const uint32_t* key_step(const mkacc_ctx* c, uint32_t u, uint32_t i, uint32_t j) {
    return c->d_keys + ((size_t)u * (c->p.n + 1) + i) * key_block_words(c) + (size_t)j * c->dg * 2 * kN;
}

int ensure_ws(mkacc_ctx* c, size_t B) {
    if (B <= c->ws_B) return MKACC_OK;
    if (c->d_acc0) HIP_TRY(hipFree(c->d_acc0));
    if (c->d_acc1) HIP_TRY(hipFree(c->d_acc1));
    if (c->d_cvals) HIP_TRY(hipFree(c->d_cvals));
    if (c->d_sumv) HIP_TRY(hipFree(c->d_sumv));
    c->d_acc0 = c->d_acc1 = c->d_cvals = c->d_sumv = nullptr;
    c->ws_B = 0;
    const size_t accw = B * c->p.k * (size_t)kN;
    HIP_TRY(hipMalloc(&c->d_acc0, accw * 4));
    HIP_TRY(hipMalloc(&c->d_acc1, accw * 4));
    HIP_TRY(hipMalloc(&c->d_cvals, B * c->p.k * (size_t)c->p.n * 4));
    HIP_TRY(hipMalloc(&c->d_sumv, B * (size_t)kN * 4));
    c->ws_B = B;
    return MKACC_OK;
}

int launch_batch(mkacc_ctx* c, const uint32_t* d_ct, const uint32_t* d_in, uint32_t* d_out, size_t B) {
    if (!c->have_keys) return fail(MKACC_E_NOKEYS, "Bootstrapping keys have not been generated/uploaded");
    if (B == 0) return MKACC_OK;
    int rc = ensure_ws(c, B);
    if (rc) return rc;
    const uint32_t k = c->p.k, n = c->p.n;
    const size_t npoly = B * k;
    const int tpb = 256;
    {
        const size_t tot = B * (size_t)k * n;
        hipLaunchKernelGGL(prep_c_kernel, dim3((unsigned)((tot + tpb - 1) / tpb)), dim3(tpb), 0, c->stream, d_ct,
                           c->d_cvals, (uint32_t)B, k * n, (uint32_t)c->method_class, (uint32_t)c->p.q);
        const size_t tw = npoly * kN;
        hipLaunchKernelGGL(eval_to_c4_kernel, dim3((unsigned)((tw + tpb - 1) / tpb)), dim3(tpb), 0, c->stream, d_in,
                           c->d_acc0, npoly, c->ninv, c->ninvp, c->mod.Q);
    }
    uint32_t* cur = c->d_acc0;
    uint32_t* nxt = c->d_acc1;
    const dim3 grid((unsigned)((B + kWavesPerBlock - 1) / kWavesPerBlock)), block(kThreads);
    const size_t lds = kWavesPerBlock * kLdsWords * sizeof(uint32_t);
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
            a.sumv = c->d_sumv;
            a.tw_fwd = c->d_twf;
            a.tw_inv = c->d_twi;
            a.psi_pow = c->d_psi;
            a.B = (uint32_t)B;
            a.k = k;
            a.index = u;
            a.m = c->mod;
            a.qhalf = c->qhalf;
            a.gbits = c->gbits;
            StepFn fn = step_fn((int)c->dg, c->method_class, first);
            hipLaunchKernelGGL(fn, grid, block, lds, c->stream, a);
            std::swap(cur, nxt);
        }
    }
    {
        const size_t tw = npoly * kN;
        hipLaunchKernelGGL(c4_to_eval_kernel, dim3((unsigned)((tw + tpb - 1) / tpb)), dim3(tpb), 0, c->stream, cur,
                           d_out, npoly, c->nval, c->nvalp, c->mod.Q);
    }
    HIP_TRY(hipGetLastError());
    return MKACC_OK;
}

std::vector<uint2> shoup_table(const std::vector<uint64_t>& vals, uint64_t Q) {
    std::vector<uint2> t(vals.size());
    for (size_t i = 0; i < vals.size(); ++i)
        t[i] = make_uint2((uint32_t)vals[i], (uint32_t)(((unsigned __int128)vals[i] << 32) / Q));
    return t;
}

template <typename W>
int upload_keys_impl(mkacc_ctx* c, const W* evk, const W* pkey) {
    if (!evk || !pkey) return fail(MKACC_E_ARG, "null key pointer");
    const uint64_t Q = c->p.Q;
    const uint32_t k = c->p.k, n = c->p.n, nk = c->nk, dg = c->dg;
    const size_t npolys = (size_t)k * nk * (n + 1) * dg * 2;
    std::vector<uint32_t> host((size_t)k * (n + 1) * key_block_words(c));
    // reference [k][nk][n+1][dg][2][N]  ->  device [k][n+1][nk][dg][2][N] (C4, * N^-1)
    bool bad = false;
    const uint64_t ninv = c->ninv;
    auto worker = [&](size_t p0, size_t p1) {
        for (size_t p = p0; p < p1; ++p) {
            size_t t = p;
            const size_t dp = t % (dg * 2); t /= (dg * 2);
            const size_t i = t % (n + 1); t /= (n + 1);
            const size_t j = t % nk; t /= nk;
            const size_t u = t;
            const W* src = evk + p * kN;
            uint32_t* dst = host.data() + (((u * (n + 1) + i) * nk + j) * dg * 2 + dp) * kN;
            for (uint32_t s = 0; s < (uint32_t)kN; ++s) {
                const uint64_t x = (uint64_t)src[s];
                if (x >= Q) bad = true;
                dst[c4_index(s)] = (uint32_t)((x * ninv) % Q);
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
            hp[p * kN + c4_index(s)] = (uint32_t)((x * ninv) % Q);
        }
    HIP_TRY(hipSetDevice(c->device));
    if (!c->d_keys) HIP_TRY(hipMalloc(&c->d_keys, host.size() * 4));
    if (!c->d_pkey) HIP_TRY(hipMalloc(&c->d_pkey, hp.size() * 4));
    HIP_TRY(hipMemcpy(c->d_keys, host.data(), host.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_pkey, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
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
    const size_t lds = kWavesPerBlock * kLdsWords * sizeof(uint32_t);
    const dim3 grid((unsigned)((count + kWavesPerBlock - 1) / kWavesPerBlock)), block(kThreads);
    if (which == 0)
        hipLaunchKernelGGL(ntt_fwd_kernel, grid, block, lds, c->stream, din, dout, (uint32_t)count, c->d_twf,
                           c->mod.Q);
    else if (which == 1)
        hipLaunchKernelGGL(ntt_inv_kernel, grid, block, lds, c->stream, din, dout, (uint32_t)count, c->d_twi,
                           c->mod.Q, c->ninv, c->ninvp);
    else {
        const size_t tot = count * kN;
        hipLaunchKernelGGL(sdd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, din, dout,
                           (uint32_t)count, c->dg, c->mod.Q, c->qhalf, c->gbits);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, dout, count * kN * 4 * out_mul, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(din));
    HIP_TRY(hipFree(dout));
    return MKACC_OK;
}

}  // namespace

// ---- C ABI ------------------------------------------------------------------------

extern "C" {

int mkacc_abi_version(void) { return MKACC_ABI_VERSION; }

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
    if (!(p.Q > (1ull << 26) && p.Q < (1ull << 27))) return fail(MKACC_E_UNSUPPORTED, "engine supports 2^26 < Q < 2^27");
    if ((p.Q - 1) % (2ull * p.N) != 0 || !is_prime(p.Q)) return fail(MKACC_E_ARG, "Q must be a prime = 1 mod 2N");
    if (p.k == 0 || p.k > 64 || p.n == 0) return fail(MKACC_E_ARG, "bad k or n");
    if (p.baseG < 2 || (p.baseG & (p.baseG - 1))) return fail(MKACC_E_ARG, "Gadget base should be a power of two.");
    if (p.method == MKACC_METHOD_MKNTRU && (p.q == 0 || p.q > (1u << 20)))
        return fail(MKACC_E_ARG, "bad ciphertext modulus q");
    if (p.digitsG == 0) p.digitsG = digits_g(p.Q, p.baseG);
    if (p.root == 0) p.root = root_of_unity(2ull * p.N, p.Q);
    const uint32_t dg = p.digitsG - 1;
    if (dg < 2 || dg > 5) return fail(MKACC_E_UNSUPPORTED, "engine supports 2..5 used gadget digits");
    if (!is_primitive_root(p.root, 2ull * p.N, p.Q)) return fail(MKACC_E_ARG, "root is not a primitive 2N-th root");

    auto c = std::make_unique<mkacc_ctx>();
    c->p = p;
    c->device = device;
    c->method_class = p.method == MKACC_METHOD_MKNTRU ? XZW : XZW_B;
    c->dg = dg;
    c->nk = c->method_class == XZW ? 2 : 1;
    c->mod.Q = (uint32_t)p.Q;
    c->mod.mu = (uint32_t)((1ull << 58) / p.Q);
    c->qhalf = (uint32_t)(p.Q >> 1);
    c->gbits = (uint32_t)__builtin_ctz(p.baseG);
    const uint64_t ninv = modinv(p.N, p.Q);
    c->ninv = (uint32_t)ninv;
    c->ninvp = (uint32_t)(((unsigned __int128)ninv << 32) / p.Q);
    c->nval = p.N;
    c->nvalp = (uint32_t)(((unsigned __int128)p.N << 32) / p.Q);

    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    // NTT tables in the reference's order (transformnat-impl.h:705-760)
    std::vector<uint64_t> tf(kN), ti(kN), pw(2 * kN);
    {
        const uint64_t Q = p.Q, psi = p.root, psii = modinv(psi, Q);
        uint64_t x = 1, xi = 1;
        for (uint32_t i = 0; i < (uint32_t)kN; ++i) {
            const uint32_t r = bit_reverse(i, kLogN);
            tf[r] = x;
            ti[r] = xi;
            x = mulmod(x, psi, Q);
            xi = mulmod(xi, psii, Q);
        }
        uint64_t e = 1;
        for (uint32_t i = 0; i < 2u * kN; ++i) { pw[i] = e; e = mulmod(e, psi, Q); }
    }
    auto htf = shoup_table(tf, p.Q), hti = shoup_table(ti, p.Q), hpw = shoup_table(pw, p.Q);
    HIP_TRY(hipMalloc(&c->d_twf, htf.size() * sizeof(uint2)));
    HIP_TRY(hipMalloc(&c->d_twi, hti.size() * sizeof(uint2)));
    HIP_TRY(hipMalloc(&c->d_psi, hpw.size() * sizeof(uint2)));
    HIP_TRY(hipMemcpy(c->d_twf, htf.data(), htf.size() * sizeof(uint2), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_twi, hti.data(), hti.size() * sizeof(uint2), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_psi, hpw.data(), hpw.size() * sizeof(uint2), hipMemcpyHostToDevice));
    *out = c.release();
    return MKACC_OK;
}

void mkacc_destroy(mkacc_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    for (void* p : {(void*)c->d_twf, (void*)c->d_twi, (void*)c->d_psi, (void*)c->d_keys, (void*)c->d_pkey,
                    (void*)c->d_acc0, (void*)c->d_acc1, (void*)c->d_cvals, (void*)c->d_sumv, (void*)c->d_ct, (void*)c->d_io})
        if (p) hipFree(p);
    if (c->stream) hipStreamDestroy(c->stream);
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
    return upload_keys_impl<uint32_t>(c, evk, pkey);
}
int mkacc_upload_keys_u64(mkacc_ctx* c, const uint64_t* evk, const uint64_t* pkey) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    return upload_keys_impl<uint64_t>(c, evk, pkey);
}

int mkacc_eval_batch(mkacc_ctx* c, const uint32_t* ct, const uint32_t* acc_in, uint32_t* acc_out, size_t B) {
    if (!c || !ct || !acc_in || !acc_out) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->have_keys) return fail(MKACC_E_NOKEYS, "Bootstrapping keys have not been generated. Please call MKBTKeyGen before calling bootstrapping.");
    if (B == 0) return MKACC_OK;
    const size_t ctw = B * c->p.k * (size_t)c->p.n, accw = B * c->p.k * (size_t)kN;
    const uint64_t lim = c->method_class == XZW ? c->p.q : 2ull * kN + 1;  // XZW_B: c <= 2N (2N -> 0)
    for (size_t s = 0; s < ctw; ++s)
        if (ct[s] >= lim) return fail(MKACC_E_RANGE, "ciphertext word out of range");
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
    return launch_batch(c, d_ct, d_in, d_out, B);
}

int mkacc_sync(mkacc_ctx* c) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MKACC_OK;
}

void* mkacc_stream(mkacc_ctx* c) { return c ? (void*)c->stream : nullptr; }

int mkacc_ntt_forward(mkacc_ctx* c, const uint32_t* in, uint32_t* out, size_t count) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    return prim_launch(c, in, out, count, 1, 0);
}
int mkacc_ntt_inverse(mkacc_ctx* c, const uint32_t* in, uint32_t* out, size_t count) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    return prim_launch(c, in, out, count, 1, 1);
}
int mkacc_sdd(mkacc_ctx* c, const uint32_t* in, uint32_t* out, size_t count) {
    if (!c) return fail(MKACC_E_ARG, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    return prim_launch(c, in, out, count, c->dg, 2);
}

}  // extern "C"
