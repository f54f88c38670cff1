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

}  // namespace

#include "mkacc_kernels.hpp"


#include "mkacc_gate.hpp"
#include "mkacc_wide.hpp"
#include "mkacc_fp64.hpp"
#include "mkacc_widereg2.hpp"

namespace {

// Device key upload for the 64-bit word path: reference layout -> [k][n+1][nk][dg][2][N]
// (EVAL order), each word in Montgomery form K * 2^64 mod Q (r, rp: 2^64 mod Q and its
// Shoup companion), or for the FP64 kernel (fp) the bits of the balanced double in the
// C16 layout.
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
    // the register-resident FP64 kernel reads its words in the C16 layout
    const uint32_t jd = fp ? widereg2::c16_index(j) : j;
    if (fp) {
        const double d = (double)(x < Q ? x : 0) - (x > (Q >> 1) && x < Q ? (double)Q : 0.0);
        dst[dpoly * kN + jd] = (uint64_t)__double_as_longlong(d);
    } else {
        dst[dpoly * kN + jd] = wide::mul_shoup(x, r, rp, Q);
    }
}

// Every digit count is instantiated.  (Round 2's MKACC_ONLY_DG=3 A/B builds
// returned null here for other digit counts and the launch of a null kernel
// produced the segfault / all-wrong records of ab_l1, lat_l1 and ab_d1,
// DESIGN.md s2; a null kernel is now refused at mkacc_create and launch.)
// Batch step kernel generation: 2 = mk_step2_kernel (mkacc_step2.hpp, digit NTTs
// first, one key stream per pass) at dg <= 3, 1 = mk_step_kernel (with its d_i
// scratch from k >= 4) at dg >= 4.  (STD128_MKNTRU 163.8 -> 158.5 us per launch,
// STD100_MKNTRU 132.6 -> 126.2, STD100_MKNTRU_LWE_2 187.4 -> 183.7 for the step2
// form; at dg = 4 the 4 x 32 digit-NTT registers leave no room for the key prefetch
// and every step2 form measured slower than mk_step_kernel)
int step_version(int dg) { return dg <= 3 ? 2 : 1; }

const void* step_fn(int dg, int method, bool first, bool dscr, int ver) {
    if (ver == 2) {
        switch (dg) {
            case 2: return first ? mkacc_tu::step2f_dg2(method) : mkacc_tu::step2_dg2(method);
            case 3: return first ? mkacc_tu::step2f_dg3(method) : mkacc_tu::step2_dg3(method);
            default: return nullptr;
        }
    }
    switch (dg) {
        case 4: return mkacc_tu::step_dg4(method, first, dscr);
        case 5: return mkacc_tu::step_dg5(method, first, dscr);
        default: return nullptr;
    }
}
const void* latd_fn(int dg, int method, bool first) {
    switch (dg) {
        case 2: return mkacc_tu::latd_dg2(method, first);
        case 3: return mkacc_tu::latd_dg3(method, first);
        case 4: return mkacc_tu::latd_dg4(method, first);
        default: return nullptr;
    }
}
const void* latdrun_fn(int dg, int method) {
    switch (dg) {
        case 2: return mkacc_tu::latdrun_dg2(method);
        case 3: return mkacc_tu::latdrun_dg3(method);
        case 4: return mkacc_tu::latdrun_dg4(method);
        default: return nullptr;
    }
}
const void* latrun_fn(int dg, int method) {
    switch (dg) {
        case 2: return mkacc_tu::latrun_dg2(method);
        case 3: return mkacc_tu::latrun_dg3(method);
        case 4: return mkacc_tu::latrun_dg4(method);
        default: return nullptr;
    }
}
const void* quad_fn(int dg, int method, bool first, int occ) {
    switch (dg) {
        case 2: return mkacc_tu::quad_dg2(method, first, occ);
        case 3: return mkacc_tu::quad_dg3(method, first, occ);
        case 4: return mkacc_tu::quad_dg4(method, first, occ);
        case 5: return mkacc_tu::quad_dg5(method, first, occ);
        default: return nullptr;
    }
}
const void* quadrun_fn(int dg, int method, int occ) {
    switch (dg) {
        case 2: return mkacc_tu::quadrun_dg2(method, occ);
        case 3: return mkacc_tu::quadrun_dg3(method, occ);
        case 4: return mkacc_tu::quadrun_dg4(method, occ);
        case 5: return mkacc_tu::quadrun_dg5(method, occ);
        default: return nullptr;
    }
}
// quad modes (use_quad): 1 one workgroup per gate, 2 the same two per CU, 3 party-parallel,
// 4 party-parallel two per CU; modes 2 and 4 keep the twiddle tables in HBM
size_t quad_lds(int mode) { return mode == 2 || mode == 4 ? quad::kLdsBytes2 : quad::kLdsBytes; }
const void* lat_fn(int dg, int method, bool first) {
    switch (dg) {
        case 2: return mkacc_tu::lat_dg2(method, first);
        case 3: return mkacc_tu::lat_dg3(method, first);
        case 4: return mkacc_tu::lat_dg4(method, first);
        default: return nullptr;
    }
}

// launch of a kernel reached through the mkacc_tu table (one by-value argument);
// a launch error is left for the caller's hipGetLastError
template <class A>
void launch_ptr(const void* fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, A a) {
    void* args[] = {&a};
    (void)hipLaunchKernel(fn, grid, block, args, lds, s);
}
template <class A, class R>
void launch_ptr2(const void* fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, A a, R r) {
    void* args[] = {&a, &r};
    (void)hipLaunchKernel(fn, grid, block, args, lds, s);
}
template <class A, class R, class T>
void launch_ptr3(const void* fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, A a, R r, T t) {
    void* args[] = {&a, &r, &t};
    (void)hipLaunchKernel(fn, grid, block, args, lds, s);
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
    int step_ver = 1;         // batch step kernel generation (step_version)
    // kernel-choice overrides, read once at mkacc_create (-1: unset, 0 / 1 forced):
    // MKACC_LAT (small-batch kernels), MKACC_LATD (split-digit kernel), MKACC_DSCR
    // (d_i scratch), so every launch and mkacc_step_kernel_name agree for the
    // context's lifetime
    int env_lat = -1, env_latd = -1, env_dscr = -1, env_quad = -1;
    uint32_t* d_qimg = nullptr;   // mk_quad_kernel tables: TF, TI, TW (mkacc_quad.hpp), 3N pairs
    uint32_t* d_psync = nullptr;  // mk_quadp_run_kernel flags, counters and sv slots (quad::psync_words)
    size_t psync_words = 0;
    bool psync_pending = false;   // a party-parallel launch since its timeout word was last read
    uint32_t h_abort = 0;
    uint32_t dg = 0, nk = 0;
    Mod mod{};
    SddConsts sd{};
    uint32_t ninv = 0, ninvp = 0, nval = 0, nvalp = 0;
    uint32_t kscale = 0, kscalep = 0;   // key words: N^-1 2^32 mod Q and its companion
    hipStream_t stream = nullptr;
    // step chains of batch slices on streams of their own (launch_steps)
    static constexpr int kMaxStreams = 4;
    int nstreams = 1;
    hipStream_t xs[kMaxStreams - 1] = {};   // extra streams
    hipEvent_t ev_fork = nullptr, ev_join[kMaxStreams - 1] = {};
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
    uint32_t* d_dscr = nullptr;   // per-gate step scratch, sized with the workspace (step_scratch_words)
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
    uint32_t gate_dks = 0;         // dks d_digits was sized for
    uint8_t* d_digits = nullptr;   // [B][k][dks][N]
    uint32_t* d_kspart = nullptr;  // key-switch slice sums of small batches (ks_slices)
    size_t kspart_words = 0;
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
    // FP64 register-resident kernel of the wide path (mkacc_widereg2.hpp), Q < 2^50,
    // balanced doubles in the C16 layout
    bool wfp = false;
    fp64::FMod wfm{};
    double wfcL = 0, wfCm = 0;     // offset-word constants (fp64::offset_word)
    double* d_r2tab = nullptr;     // per-lane twiddle table (widereg2::kTabD doubles)
    double* d_rtis = nullptr;      // inverse pass-1 table [32]
    double* d_ftwf = nullptr;      // forward twiddles (reference order) and psi^e, balanced
    double* d_fpsi = nullptr;
    size_t wws_B = 0, wio_B = 0;
    uint64_t* d_wacc0 = nullptr;
    uint64_t* d_wacc1 = nullptr;
    uint32_t* d_wcvals = nullptr;
    uint32_t* d_wct = nullptr;     // host-pointer API staging
    uint64_t* d_wio = nullptr;
    uint32_t* d_bad = nullptr;     // [0] input-range flag of the device batches (mkacc_sync), [1] device key upload,
                                   // [2] party-parallel synchronisation timeout (mk_quadp_run_kernel)
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
    if (c->method_class != XZW || c->p.k < 2 || c->step_ver != 1) return false;
    if (c->env_dscr >= 0) return c->env_dscr != 0;
    return c->p.k >= kDscrMinK;
}
// an environment switch: -1 unset, else 0 (value starting with '0') or 1
int env_switch(const char* name) {
    const char* e = std::getenv(name);
    return e && *e ? (e[0] != '0') : -1;
}

// Two-party batches of at most one gate per CU split each party's digits over two
// waves (mk_latd_kernel: four waves of up to 256 VGPRs, one workgroup per CU);
// MKACC_LATD=0 keeps one wave per party (mk_lat_kernel).
bool use_latd(const mkacc_ctx* c, size_t B) {
    if (c->p.k != 2 || B > (size_t)c->cus) return false;
    return c->env_latd != 0;
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
    if (c->env_lat >= 0) return c->env_lat != 0;
    return B <= (size_t)c->cus * (kLdsPerCu / lat_lds_bytes(c->p.k));
}

// The party-parallel form (mk_quadp_run_kernel: each gate's parties spread over G >= 2
// workgroups, one per CU, the steps after the first) needs all B G workgroups resident
// (a cooperative launch): G = k where B k <= CUs, fewer -- ceil(k / G) parties each --
// for larger batches up to CUs / 2 gates.  It is the default wherever it fits:
// STD128_MKNTRU one gate 24.1 -> 17.1 ms, B = 128 5.24 k -> 7.30 k gates/s;
// STD128_MKNTRU_3 one gate 319.5 -> 95.2 ms, B = 32 101 -> 340 gates/s
// (profiles/r6/v16_ab_*).  MKACC_QUAD=1 keeps one workgroup per gate.
struct QuadpShape {
    uint32_t groups = 0, ppw = 0;   // workgroups per gate, parties per workgroup
};
// occ: workgroups per CU (2: mk_quadp2_run_kernel, dg <= 4)
QuadpShape quadp_shape(const mkacc_ctx* c, size_t B, int occ = 1) {
    const uint32_t k = c->p.k;
    // shares carry their step tag in bits 28..31: residues below 2Q < 2^28
    if (k < 2 || B == 0 || k * c->p.n < 2 || c->p.Q >= (1ull << 27)) return {};
    if (occ == 2 && c->dg > 4) return {};
    const size_t gmax = std::min<size_t>(k, (size_t)occ * c->cus / B);
    if (gmax < 2) return {};
    QuadpShape sh;
    sh.ppw = (uint32_t)((k + gmax - 1) / gmax);
    sh.groups = (k + sh.ppw - 1) / sh.ppw;
    return sh;
}
bool use_quadp(const mkacc_ctx* c, size_t B, int occ = 1) { return quadp_shape(c, B, occ).groups >= 2; }

// Small batches of at most one gate per CU take mk_quad_kernel (every polynomial
// spread over the four waves of the gate's workgroup, mkacc_quad.hpp) for every k and
// dg: one STD128_MKNTRU gate 43.7 -> 24.2 ms against the split-digit kernel, B = 256
// 5.87 k -> 10.5 k gates/s, STD128_MKNTRU_3 one gate 486 -> 323 ms, B = 256 491 ->
// 794 gates/s (profiles/r6/v5_ab_*, v6_ab_*).  MKACC_QUAD=0 keeps the older kernels.
// Above one gate per CU and up to four per CU, mk_quad2_kernel (the twiddle tables in
// HBM, two workgroups per CU, dg <= 4; batches above 2 x CUs in rounds) beats the
// per-party and the batch kernels: STD128_MKNTRU B = 384 6.8 k -> 11.0 k gates/s,
// 512 8.7 k -> 14.7 k, 1024 12.0 k -> 15.3 k; STD100_MKNTRU_LWE_2 B = 512 6.2 k -> 8.5 k,
// 1024 7.3 k -> 8.8 k; STD128_MKNTRU_3 B = 512 409 -> 992, 1024 773 -> 1,022.  From 8
// gates per CU the batch kernels win (STD128_MKNTRU B = 2048: 18.2 k against 15.8 k,
// 4096: 19.2 k against 16.0 k; config 3 at 4096 11.3 k against 9.2 k; config 4 at 8192
// 1,282 against 1,059) -- profiles/r6/v11_ab_*, v12_ab_*.  MKACC_QUAD=2 forces it for
// any batch (A/B runs).  Returns the workgroups per CU of the quad kernel, 0 for none.
int use_quad(const mkacc_ctx* c, size_t B) {
    if (c->wide || c->dg < 2 || c->dg > 5 || c->env_quad == 0) return 0;
    if (c->env_quad == 2) return c->dg <= 4 ? 2 : 0;
    if (c->env_quad != 1 && use_quadp(c, B)) return 3;
    if (c->env_quad == 4 && use_quadp(c, B, 2)) return 4;
    if (B <= (size_t)c->cus) return 1;
    return B <= 4 * (size_t)c->cus && c->dg <= 4 ? 2 : 0;
}

// Per-gate scratch words of the batch step kernel: mk_step_kernel DSCR keeps the
// step's d_i ([dg][N]).
size_t step_scratch_words(const mkacc_ctx* c) { return use_dscr(c) ? (size_t)c->dg * kN : 0; }

int ensure_psync(mkacc_ctx* c, size_t B);
int ensure_ws(mkacc_ctx* c, size_t B) {
    if (use_quad(c, B) >= 3) {
        const int rc = ensure_psync(c, B);
        if (rc) return rc;
    }
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
    if (const size_t sw = step_scratch_words(c)) HIP_TRY(hipMalloc(&c->d_dscr, B * sw * 4));
    c->ws_B = B;
    return MKACC_OK;
}
// the party-parallel kernel's synchronisation area for B gates
int ensure_psync(mkacc_ctx* c, size_t B) {
    const int mode = use_quad(c, B);
    const size_t w = quad::psync_words(B, quadp_shape(c, B, mode == 4 ? 2 : 1).groups);
    if (w <= c->psync_words) return MKACC_OK;
    if (c->d_psync) HIP_TRY(hipFree(c->d_psync));
    c->d_psync = nullptr;
    c->psync_words = 0;
    HIP_TRY(hipMalloc(&c->d_psync, w * 4));
    c->psync_words = w;
    return MKACC_OK;
}
// After the final synchronisation of an entry point: a party-parallel launch whose
// waits timed out (d_bad[2], read back with the results by psync_enqueue) fails it.
int psync_enqueue(mkacc_ctx* c) {
    if (c->psync_pending) HIP_TRY(hipMemcpyAsync(&c->h_abort, c->d_bad + 2, 4, hipMemcpyDeviceToHost, c->stream));
    return MKACC_OK;
}
int psync_result(mkacc_ctx* c) {
    if (!c->psync_pending) return MKACC_OK;
    c->psync_pending = false;
    if (!c->h_abort) return MKACC_OK;
    c->h_abort = 0;
    HIP_TRY(hipMemset(c->d_bad + 2, 0, 4));
    return fail(MKACC_E_DEVICE, "party-parallel step kernel: a synchronisation wait timed out (results are invalid)");
}

// The k*n accumulator steps over a batch whose monomial exponents are in
// d_cvals and whose C4 accumulators are in d_acc0; returns the buffer holding
// the result (nullptr if the build has no kernel for the context's digit count).
// Gates [g0, g0 + Bh) of a batch of B on stream st: the k*n accumulator steps, one
// launch per step() call, ping-ponging between d_acc0 and d_acc1 at this half's offset.
struct StepChain {
    mkacc_ctx* c;
    size_t B, g0, Bh, ao;
    hipStream_t st;
    uint32_t* cur;
    uint32_t* nxt;
    bool lat;
    int quad;   // use_quad: 0, or the quad kernel's workgroups per CU
    StepChain(mkacc_ctx* c_, size_t B_, size_t g0_, size_t Bh_, hipStream_t st_)
        : c(c_), B(B_), g0(g0_), Bh(Bh_), ao(g0_ * c_->p.k * kN), st(st_), cur(c_->d_acc0 + ao), nxt(c_->d_acc1 + ao),
          lat(use_lat(c_, Bh_)), quad(use_quad(c_, Bh_)) {}
    StepArgs args(uint32_t u, uint32_t i) const {
        const uint32_t k = c->p.k, n = c->p.n;
        StepArgs a;
        a.acc_in = cur;
        a.acc_out = nxt;
        a.cvals = c->d_cvals + ((size_t)u * n + i) * B + g0;
        a.key1 = key_step(c, u, i, 0);
        a.key2 = c->nk == 2 ? key_step(c, u, i, 1) : a.key1;
        a.keys = key_step(c, 0, n, 0);
        a.pkey = c->d_pkey;
        a.tw_fwd = c->d_twf;
        a.tw_inv = c->d_twi;
        a.img = c->d_img;
        a.B = (uint32_t)Bh;
        a.k = k;
        a.index = u;
        a.m = c->mod;
        a.sd = c->sd;
        a.dscr = c->d_dscr ? c->d_dscr + g0 * step_scratch_words(c) : nullptr;
        return a;
    }
    // one accumulator step (u, i); false if the build has no kernel for it
    bool step(uint32_t u, uint32_t i, size_t lds) {
        const uint32_t k = c->p.k;
        const bool first = (u == 0 && i == 0);
        const StepArgs a = args(u, i);
        // a null kernel must never reach hipLaunchKernelGGL (mkacc_create checks the set)
        if (quad) {
            // the first (KDM) step, once per gate, runs the one-workgroup-per-CU form for
            // either occupancy: its four key words per digit do not fit 256 VGPRs at dg = 4
            const int occ = first ? 1 : quad;   // modes 3 and 4 have no step kernel of their own
            const void* fn = quad_fn((int)c->dg, c->method_class, first, occ);
            if (!fn) return false;
            launch_ptr2(fn, dim3((unsigned)Bh), dim3(64 * quad::kWaves), quad_lds(occ), st, a, QuadArgs{c->d_qimg});
        } else if (lat) {
            const bool split = use_latd(c, Bh);
            const void* fn = split ? latd_fn((int)c->dg, c->method_class, first) : lat_fn((int)c->dg, c->method_class, first);
            if (!fn) return false;
            const uint32_t waves = split ? kLatdWaves : k;
            launch_ptr(fn, dim3((unsigned)Bh), dim3(64 * waves), split ? latd_lds_bytes() : lat_lds_bytes(waves), st, a);
        } else {
            const void* fn = step_fn((int)c->dg, c->method_class, first, !first && use_dscr(c), c->step_ver);
            if (!fn) return false;
            if (c->step_ver == 2)
                launch_ptr(fn, dim3((unsigned)((Bh + kS2Waves - 1) / kS2Waves)), dim3(64 * kS2Waves),
                           kStep2LdsBytes + (lds - kStepLdsBytes), st, a);
            else
                launch_ptr(fn, dim3((unsigned)((Bh + kWavesPerBlock - 1) / kWavesPerBlock)), dim3(kThreads), lds, st,
                           a);
        }
        std::swap(cur, nxt);
        return true;
    }
    // steps [t0, t1) (t = u n + i, t0 >= 1) in one mk_latd_run_kernel (use_latd
    // batches) or mk_lat_run_kernel launch; false if the build has no kernel for it
    bool run(uint32_t t0, uint32_t t1) {
        const uint32_t n = c->p.n;
        const bool split = use_latd(c, Bh);
        const uint32_t waves = quad ? quad::kWaves : split ? kLatdWaves : c->p.k;
        const void* fn = quad    ? quadrun_fn((int)c->dg, c->method_class, quad)
                         : split ? latdrun_fn((int)c->dg, c->method_class)
                                 : latrun_fn((int)c->dg, c->method_class);
        if (!fn || t0 == 0 || t0 >= t1) return false;
        const StepArgs a = args(t0 / n, t0 % n);
        LatdRun r;
        r.keys = c->d_keys;
        r.cvals = c->d_cvals + g0;
        r.acc0 = cur;
        r.acc1 = nxt;
        r.kbw = key_block_words(c);
        r.cstride = (uint32_t)B;
        r.n = n;
        r.t0 = t0;
        r.t1 = t1;
        r.key2off = c->nk == 2 ? (uint32_t)(c->dg * 2 * kN) : 0u;
        if (quad >= 3) {
            // every workgroup of the batch resident at once: the cooperative launch refuses
            // a grid the device cannot hold instead of leaving waits without a producer
            const QuadpShape sh = quadp_shape(c, Bh, quad == 4 ? 2 : 1);
            const uint32_t v4 = (uint32_t)(quad::psync_words(Bh, sh.groups) / 4);
            hipLaunchKernelGGL(psync_clear_kernel, dim3(std::min<uint32_t>((v4 + 255) / 256, 1024u)), dim3(256), 0, st,
                               c->d_psync, v4);
            QuadArgs qa{c->d_qimg, c->d_psync, c->d_bad + 2, sh.groups, sh.ppw};
            void* args[] = {(void*)&a, (void*)&r, (void*)&qa};
            if (hipLaunchCooperativeKernel(fn, dim3((unsigned)(Bh * sh.groups)), dim3(64 * waves), args,
                                           (unsigned)quad_lds(quad), st) != hipSuccess)
                return false;
            c->psync_pending = true;
        } else if (quad)
            launch_ptr3(fn, dim3((unsigned)Bh), dim3(64 * waves), quad_lds(quad), st, a, r, QuadArgs{c->d_qimg});
        else
            launch_ptr2(fn, dim3((unsigned)Bh), dim3(64 * waves), split ? latd_lds_bytes() : lat_lds_bytes(waves), st, a,
                        r);
        if ((t1 - t0) & 1u) std::swap(cur, nxt);
        return true;
    }
    uint32_t* result() const { return cur - ao; }   // the full-batch buffer holding the result
};

// Small batches run the steps after the first in one launch: every batch of the
// split-digit kernel (mk_latd_run_kernel: -9 % at B = 1, -22 % at B = 256,
// profiles/r5/ab_latd_run_v24.txt) and those of the one-wave-per-party kernel whose
// k B waves are resident at once at k <= 4 (mk_lat_run_kernel, ab_lat_run_v25.txt).
// Residency counts whole workgroups: a CU holds 4 SIMDs x lat_run_occ waves of the
// loop's register budget, i.e. floor(4 occ / k) workgroups of k waves, and no more
// than its LDS allows (k = 5..7 fit once per CU, not 8 occ / k times).
bool use_run(const mkacc_ctx* c, size_t B) {
    const size_t k = c->p.k;
    if (k * c->p.n < 2) return false;
    if (use_quad(c, B)) return true;
    if (!use_lat(c, B)) return false;
    if (use_latd(c, B)) return true;
    if (k > lat_run_max_k(c->dg)) return false;
    const size_t wgs = std::min<size_t>(4 * lat_run_occ(c->dg) / k, kLdsPerCu / lat_lds_bytes((uint32_t)k));
    return wgs > 0 && B <= (size_t)c->cus * wgs;
}

// Joins the slice streams a batch forked from the context stream back into it on
// every exit path: later work on c->stream -- a key upload's
// hipStreamSynchronize, a workspace free -- must stay ordered after every slice
// launch, also when a launch helper returns early.
struct SliceJoin {
    mkacc_ctx* c;
    size_t ns = 0;   // slices forked (streams xs[0 .. ns-2] wait on ev_fork)
    bool ok = true;  // every join recorded and waited for
    ~SliceJoin() { join(); }
    void join() {
        for (size_t j = 1; j < ns; ++j)
            if (hipEventRecord(c->ev_join[j - 1], c->xs[j - 1]) != hipSuccess ||
                hipStreamWaitEvent(c->stream, c->ev_join[j - 1], 0) != hipSuccess)
                ok = false;
        ns = 0;
    }
};

// The k*n accumulator steps over a batch whose monomial exponents are in
// d_cvals and whose C4 accumulators are in d_acc0; returns the buffer holding
// the result (nullptr if the build has no kernel for the context's digit count).
// A batch of at least two units of cus x 4 gates (one 4-gate workgroup per CU, half
// a round of resident gates) is cut into up to nstreams slices of whole units
// (MKACC_STREAMS, default 2), each slice's launches
// on a stream of its own, enqueued step by step and forked after / joined before
// the main stream's work.  Gates are independent, so the slices need no other
// ordering, and one slice's next launch takes the CUs another slice's tail leaves
// idle: STD128_MKNTRU 238.4 -> 211.1 ms per batch, STD128_MKNTRU_3 7.27 -> 6.65 s
// (profiles/r4/ab_streams.txt).
uint32_t* launch_steps(mkacc_ctx* c, size_t B) {
    const uint32_t k = c->p.k, n = c->p.n;
    // MKACC_DBG_LDS=<bytes> (diagnosis, tools/dbg/determ2.py): extra dynamic LDS per
    // workgroup; 10240 leaves one workgroup per CU, the co-residency reference
    const char* dl = std::getenv("MKACC_DBG_LDS");
    const size_t lds = kStepLdsBytes + (dl ? std::strtoul(dl, nullptr, 0) : 0);
    const size_t unit = (size_t)c->cus * 4;
    // a quad batch runs its later steps in one launch: one chain, no slices
    const size_t ns = use_quad(c, B) ? 1 : std::min<size_t>((size_t)c->nstreams, B / unit);
    if (ns < 2) {
        StepChain ch(c, B, 0, B, c->stream);
        if (use_run(c, B)) {
            if (!ch.step(0, 0, lds) || !ch.run(1, k * n)) return nullptr;
            return ch.result();
        }
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t i = 0; i < n; ++i)
                if (!ch.step(u, i, lds)) return nullptr;
        return ch.result();
    }
    // slices of whole units, the remainder in the last one
    const size_t per = (B / unit / ns) * unit;
    if (hipEventRecord(c->ev_fork, c->stream) != hipSuccess) return nullptr;
    SliceJoin join{c};
    std::vector<StepChain> ch;
    ch.reserve(ns);
    for (size_t j = 0; j < ns; ++j) {
        hipStream_t st = j == 0 ? c->stream : c->xs[j - 1];
        if (j > 0 && hipStreamWaitEvent(st, c->ev_fork, 0) != hipSuccess) return nullptr;
        join.ns = j + 1;
        ch.emplace_back(c, B, j * per, j + 1 < ns ? per : B - j * per, st);
    }
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t i = 0; i < n; ++i)
            for (auto& h : ch)
                if (!h.step(u, i, lds)) return nullptr;
    join.join();
    return join.ok ? ch[0].result() : nullptr;
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

// Key-switch slices of a small batch: the sum over l = (digit, coefficient) split into
// slices of lper (a multiple of the kernel's reduction / digit-fetch granule) so the
// blocks cover the CUs about twice; 1 for batches with blocks enough.  One STD128_MKNTRU
// gate's KeySwitch2 ran 24 blocks (1.38 ms of a 17.7 ms gate, profiles/r6/v25).
uint32_t ks_slices(const mkacc_ctx* c, size_t B, uint32_t& lper) {
    const size_t L = (size_t)c->dks * kN;
    const bool mntru = c->method_class == XZW;
    const size_t blocks = mntru ? (size_t)(c->n_pad / kKsTile) * ((B + kKsTile - 1) / kKsTile) * c->p.k : B * c->p.k;
    const size_t gran = mntru ? 4 * kKsChunk : 16;
    size_t S = blocks >= 2 * (size_t)c->cus ? 1 : (2 * (size_t)c->cus + blocks - 1) / blocks;
    S = std::max<size_t>(1, std::min<size_t>(S, std::min<size_t>(64, L / gran)));
    lper = (uint32_t)(((L + S - 1) / S + gran - 1) / gran * gran);
    return (uint32_t)((L + lper - 1) / lper);
}
size_t kspart_words(const mkacc_ctx* c, size_t B) {
    uint32_t lper;
    const size_t S = ks_slices(c, B, lper);
    return S > 1 ? S * B * c->p.k * ((size_t)c->ks.n_out + 1) : 0;
}

int ensure_gate_ws(mkacc_ctx* c, size_t B) {
    int rc = ensure_ws(c, B);
    if (rc) return rc;
    if (const size_t w = kspart_words(c, B); w > c->kspart_words) {
        if (c->d_kspart) HIP_TRY(hipFree(c->d_kspart));
        c->d_kspart = nullptr;
        c->kspart_words = 0;
        HIP_TRY(hipMalloc(&c->d_kspart, w * 4));
        c->kspart_words = w;
    }
    // d_digits is sized for the key-switching digit count it was allocated with;
    // a re-upload (or share_ksk) with a different dks must reallocate it
    if (B <= c->gate_B && c->dks == c->gate_dks) return MKACC_OK;
    if (c->d_digits) HIP_TRY(hipFree(c->d_digits));
    if (c->d_bh) HIP_TRY(hipFree(c->d_bh));
    c->d_digits = nullptr;
    c->d_bh = nullptr;
    c->gate_B = 0;
    HIP_TRY(hipMalloc(&c->d_digits, B * c->p.k * (size_t)c->dks * kN));
    HIP_TRY(hipMalloc(&c->d_bh, B * c->p.k * 4));   // MK-LWE head rotation b [B], then partial b sums [B][k]
    c->gate_B = B;
    c->gate_dks = c->dks;
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
    uint32_t lper = 0;
    uint32_t S = ks_slices(c, B, lper);
    // the slice sums need ensure_gate_ws's buffer (every gate entry point sizes it)
    if (S > 1 && c->kspart_words < kspart_words(c, B)) {
        S = 1;
        lper = L;
    }
    uint32_t* part = S > 1 ? c->d_kspart : nullptr;
    const uint32_t total = (uint32_t)(B * k * c->ks.n_out);
    if (c->method_class == XZW) {
        const uint32_t qinv = (uint32_t)((1ull << 32) / c->ks.qKS);
        const dim3 grid(c->n_pad / kKsTile, (unsigned)((B + kKsTile - 1) / kKsTile), k * S);
        hipLaunchKernelGGL(ks_mntru_kernel, grid, dim3(256), 0, c->stream, c->d_digits, c->d_ksk, out_a,
                           (uint32_t)B, k, L, c->ks.n_out, c->n_pad, (uint32_t)c->ks.qKS, qinv, lper, part);
        if (part)
            hipLaunchKernelGGL(ks_sum_kernel, dim3((total + 255) / 256), dim3(256), 0, c->stream, part, out_a, S, total,
                               (uint32_t)c->ks.qKS);
    } else {
        const uint32_t b0 = round_qQ_host((c->p.Q >> 3) + 1, c->ks.qKS, c->p.Q);
        uint32_t* pb = part ? part + (size_t)S * total : nullptr;
        hipLaunchKernelGGL(ks_mklwe_kernel, dim3((unsigned)(B * k * S)), dim3(256), 0, c->stream, c->d_digits,
                           c->d_lweA, c->d_lweB, out_a, c->d_bh, k, c->ks.n_out, c->ks.baseKS, c->dks,
                           (uint32_t)c->ks.qKS, (uint32_t)B, S, lper, part, pb);
        if (part)
            hipLaunchKernelGGL(ks_mklwe_sum_kernel, dim3((total + 255) / 256), dim3(256), 0, c->stream, part, pb, out_a,
                               c->d_bh, S, (uint32_t)(B * k), c->ks.n_out, (uint32_t)c->ks.qKS);
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
    // an earlier device batch may still read the old keys on the context stream
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->have_keys = false;
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

// MKACC_STREAMS=1..4 (default 2): the streams of the batch slices (launch_steps,
// wide_launch_batch)
hipError_t create_slice_streams(mkacc_ctx* c) {
    const char* e = std::getenv("MKACC_STREAMS");
    const int ns = e && e[0] >= '1' && e[0] <= '4' && !e[1] ? e[0] - '0' : 2;
    hipError_t r = hipSuccess;
    if (ns > 1 && (r = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming)) != hipSuccess) return r;
    for (int j = 0; j + 1 < ns; ++j) {
        if ((r = hipStreamCreateWithFlags(&c->xs[j], hipStreamNonBlocking)) != hipSuccess) return r;
        if ((r = hipEventCreateWithFlags(&c->ev_join[j], hipEventDisableTiming)) != hipSuccess) return r;
    }
    c->nstreams = ns;
    return r;
}

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
    // FP64 register-resident kernel (mkacc_widereg2.hpp): exact while every value stays
    // below 8 Q <= 2^53; the offset word's 2^52 form (fp64::offset_word) needs
    // C + L >= 0 and C + (Q - 1) / 2 < 2^52.  MKACC_WIDE_FP=0 keeps the integer kernels.
    const char* fe = std::getenv("MKACC_WIDE_FP");
    const uint64_t cL = (Q + 1) / 2;
    c->wfp = Q < (1ull << 50) && b * c->p.digitsG <= 52 && C >= cL && C + (Q >> 1) < (1ull << 52) &&
             !(fe && fe[0] == '0');
    if (c->wfp) {
        const double Qd = (double)Q;
        c->wfm = fp64::FMod{Qd, 1.0 / Qd, (double)(Q >> 1)};
        auto bal = [Q](uint64_t x) { return x > (Q >> 1) ? (double)x - (double)Q : (double)x; };
        c->wfcL = (double)cL;
        c->wfCm = (double)((1ull << 52) + (C - std::min(C, cL)));
        std::vector<double> ftf(kN), fpw(2 * kN), tis(32, 0.0);
        for (uint32_t i = 0; i < (uint32_t)kN; ++i) ftf[i] = bal(tf[i].x);
        for (uint32_t i = 0; i < 2u * kN; ++i) fpw[i] = bal(pw[i].x);
        // psi^-e for e in [0, 2N) in natural order
        std::vector<uint64_t> pwi(2 * kN);
        {
            uint64_t ei = 1;
            for (uint32_t i = 0; i < 2u * kN; ++i) {
                pwi[i] = ei;
                ei = mulmod(ei, psii, Q);
            }
        }
        // inverse pass 1: bit b, t < 2^b -> psi^-(t 2^(11-b)) (the kernel reads b < 4)
        for (int b = 0; b < 5; ++b)
            for (int t = 0; t < (1 << b); ++t) tis[(1 << b) + t] = bal(pwi[(size_t)t << (11 - b)]);
        // per-lane twiddle table: value k of sub-table T for (w, l) at
        // ((kTG0[T] + k / 2) * 128 + w * 64 + l) * 2 + k % 2 (index maps checked against
        // the oracle by tools/widereg2_model.py)
        using namespace lay2;
        std::vector<double> tab(kTabE, 0.0);
        auto put = [&](int T, uint32_t w, uint32_t l, int k, double v) { tab[tab_index(T, w, l, k)] = v; };
        auto lg = [](int v) { int b = 0; while ((2 << b) <= v) ++b; return b; };   // floor(log2 v)
        for (uint32_t w = 0; w < 2; ++w)
            for (uint32_t l = 0; l < 64; ++l) {
                const uint32_t l3 = (l >> 3) & 1u, l4 = (l >> 4) & 1u, l5 = (l >> 5) & 1u;
                auto pb = [&](uint32_t r) { return (r << 3) | (l & 7u) | (l3 << 7) | (l4 << 8) | (l5 << 9) | (w << 10); };
                auto pd = [&](uint32_t r) { return (r << 4) | (l & 15u) | (l4 << 8) | (l5 << 9) | (w << 10); };
                for (int k = 0; k < 7; ++k) {          // forward B2, stages 4..6
                    const int st = 4 + lg(k + 1), m = k - ((1 << (st - 4)) - 1);
                    put(TFB, w, l, k, ftf[(1u << st) + (pb((uint32_t)m << (8 - st)) >> (11 - st))]);
                }
                for (int k = 0; k < 15; ++k) {         // forward C2, stages 7..10
                    const int st = 7 + lg(k + 1), m = k - ((1 << (st - 7)) - 1);
                    put(TFC, w, l, k, ftf[(1u << st) + (pos_c(w, l, (uint32_t)m << (11 - st)) >> (11 - st))]);
                }
                for (int k = 0; k < 15; ++k) {         // inverse D2, bits 4..7
                    const int b = 4 + lg(k + 1), H = 1 << (b - 4);
                    const uint32_t t = pd((uint32_t)(k - (H - 1))) & ((1u << b) - 1u);
                    put(TID, w, l, k, bal(pwi[(size_t)t << (11 - b)]));
                }
                for (int k = 0; k < 14; ++k) {         // inverse A2, bits 8..10
                    const int b = k < 2 ? 8 : (k < 6 ? 9 : 10), H = 1 << (b - 7);
                    const uint32_t t = pos_a(w, l, (uint32_t)(k - (H - 2))) & ((1u << b) - 1u);
                    put(TIA, w, l, k, bal(pwi[(size_t)t << (11 - b)]));
                }
                for (int k = 0; k < 16; ++k)           // twist psi^-p N^-1
                    put(TTW, w, l, k, bal(mulmod(pwi[pos_a(w, l, (uint32_t)k)], c->wninv, Q)));
            }
        HIP_TRY(hipMalloc(&c->d_ftwf, kN * sizeof(double)));
        HIP_TRY(hipMalloc(&c->d_fpsi, 2 * kN * sizeof(double)));
        HIP_TRY(hipMalloc(&c->d_rtis, tis.size() * sizeof(double)));
        HIP_TRY(hipMalloc(&c->d_r2tab, tab.size() * sizeof(double)));
        HIP_TRY(hipMemcpy(c->d_ftwf, ftf.data(), kN * sizeof(double), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_fpsi, fpw.data(), 2 * kN * sizeof(double), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_rtis, tis.data(), tis.size() * sizeof(double), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_r2tab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
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
    const bool fp = c->wfp;   // FP64 kernel: the bits of the balanced double
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
    // the register-resident FP64 kernel reads every polynomial in the C16 layout
    auto pos = [fp](size_t s) {
        const uint32_t j = (uint32_t)(s & (kN - 1));
        return (s & ~(size_t)(kN - 1)) | (fp ? widereg2::c16_index(j) : j);
    };
    std::vector<uint64_t> host((size_t)k * (n + 1) * nk * blk);
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t j = 0; j < nk; ++j)
            for (uint32_t i = 0; i <= n; ++i) {
                const W* src = evk + (((size_t)u * nk + j) * (n + 1) + i) * blk;
                uint64_t* dst = host.data() + (((size_t)u * (n + 1) + i) * nk + j) * blk;
                for (size_t s = 0; s < blk; ++s) {
                    if ((uint64_t)src[s] >= Q) return fail(MKACC_E_RANGE, "evk word not a canonical residue mod Q");
                    dst[pos(s)] = mont((uint64_t)src[s]);
                }
            }
    const size_t pw = (size_t)k * dg * kN;
    std::vector<uint64_t> hp(pw);
    for (size_t s = 0; s < pw; ++s) {
        if ((uint64_t)pkey[s] >= Q) return fail(MKACC_E_RANGE, "pkey word not a canonical residue mod Q");
        hp[pos(s)] = mont((uint64_t)pkey[s]);
    }
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->have_keys = false;
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
    if (c->wfp) {   // FP64, two waves per gate: balanced doubles in the C16 layout
        const size_t words = B * (size_t)k * kN;
        const dim3 g((unsigned)((words + 255) / 256));
        double* cur = reinterpret_cast<double*>(c->d_wacc0);
        double* nxt = reinterpret_cast<double*>(c->d_wacc1);
        hipLaunchKernelGGL(widereg2::to_c16_kernel, g, dim3(256), 0, c->stream, d_in, cur, words, c->wfm, c->p.Q,
                           c->d_bad);
        auto dk = [](const uint64_t* p) { return reinterpret_cast<const double*>(p); };
        // four 2-wave workgroups per CU, each looping over its slice of the batch; a
        // batch of at least two units of cus x 4 gates is cut into slices on streams of
        // their own, as launch_steps does for the 27-bit kernels
        const size_t unit = (size_t)c->cus * 4;
        const size_t ns = std::max<size_t>(1, std::min<size_t>((size_t)c->nstreams, B / unit));
        const size_t per = ns > 1 ? (B / unit / ns) * unit : B;
        SliceJoin join{c};
        if (ns > 1) {
            HIP_TRY(hipEventRecord(c->ev_fork, c->stream));
            for (size_t j = 1; j < ns; ++j) {
                HIP_TRY(hipStreamWaitEvent(c->xs[j - 1], c->ev_fork, 0));
                join.ns = j + 1;
            }
        }
        for (uint32_t u = 0; u < k; ++u)
            for (uint32_t i = 0; i < n; ++i)
            for (size_t j = 0; j < ns; ++j) {
                const size_t g0 = j * per, Bh = j + 1 < ns ? per : B - g0;
                const size_t ao = g0 * k * kN;
                const bool first = (u == 0 && i == 0);
                widereg2::StepArgs a;
                a.acc_in = cur + ao;
                a.acc_out = nxt + ao;
                a.cvals = c->d_wcvals + ((size_t)u * n + i) * B + g0;
                a.key1 = dk(key(u, i, 0));
                a.key2 = dk(c->nk == 2 ? key(u, i, 1) : key(u, i, 0));
                a.keys = dk(key(0, n, 0));
                a.pkey = dk(c->d_wpkey);
                a.tab = c->d_r2tab;
                a.psi = c->d_fpsi;
                a.twf = c->d_ftwf;
                a.tis = c->d_rtis;
                a.B = (uint32_t)Bh;
                a.k = k;
                a.index = u;
                a.dg = c->dg;
                a.cL = c->wfcL;
                a.Cm = c->wfCm;
                a.m = c->wfm;
                a.sd = c->wsd;
                launch_ptr(mkacc_tu::widereg2_step(c->method_class, first),
                           dim3((unsigned)std::min<size_t>(Bh, unit)), dim3(128), widereg2::kLdsBytes,
                           j == 0 ? c->stream : c->xs[j - 1], a);
                if (j + 1 == ns) std::swap(cur, nxt);
            }
        join.join();
        if (!join.ok) return fail(MKACC_E_DEVICE, "joining the batch slice streams failed");
        hipLaunchKernelGGL(widereg2::from_c16_kernel, g, dim3(256), 0, c->stream, cur, d_out, words, c->wfm);
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
            launch_ptr(mkacc_tu::wide_step(c->method_class, first), dim3((unsigned)B), dim3(wide::kThreads), 0, c->stream,
                       a);
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
        hipLaunchKernelGGL(widereg2::ntt_fwd_kernel, dim3((unsigned)count), dim3(128), widereg2::kLdsBytes, c->stream,
                           din, dout, c->d_r2tab, c->d_ftwf, c->wfm);
    else if (which == 1 && c->wfp)
        hipLaunchKernelGGL(widereg2::ntt_inv_kernel, dim3((unsigned)count), dim3(128), widereg2::kLdsBytes, c->stream,
                           din, dout, c->d_r2tab, c->d_rtis, c->wfm);
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
            if (step_fn(dg, XZW, true, false, step_version(dg)) && step_fn(dg, XZW_B, false, false, step_version(dg)))
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
    c->env_lat = env_switch("MKACC_LAT");
    c->env_latd = env_switch("MKACC_LATD");
    c->env_dscr = env_switch("MKACC_DSCR");
    {
        // 0 (no quad kernel), 1 (one workgroup per gate, no party-parallel form),
        // 2 (two workgroups per CU, any B), 3 / unset (the policy of use_quad), 4 (the
        // policy with the two-per-CU party-parallel form up to CUs gates)
        const char* e = std::getenv("MKACC_QUAD");
        c->env_quad = e && *e ? (e[0] == '0' ? 0 : e[0] == '2' ? 2 : e[0] == '3' ? 3 : e[0] == '4' ? 4 : 1) : -1;
    }
    c->dg = dg;
    c->step_ver = step_version((int)dg);
    c->nk = c->method_class == XZW ? 2 : 1;
    c->wide = wide;
    if (!wide && !step_fn((int)dg, c->method_class, true, false, c->step_ver))
        return fail(MKACC_E_UNSUPPORTED, "this build has no step kernel for dg = " + std::to_string(dg));
    if (wide) {
        HIP_TRY(hipSetDevice(device));
        HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        HIP_TRY(create_slice_streams(c.get()));
        HIP_TRY(hipMalloc(&c->d_bad, 12));   // [0] batch inputs, [1] device key upload, [2] sync timeout
        HIP_TRY(hipMemset(c->d_bad, 0, 12));
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
    HIP_TRY(create_slice_streams(c.get()));
    HIP_TRY(hipMalloc(&c->d_bad, 12));   // [0] batch inputs, [1] device key upload, [2] sync timeout
    HIP_TRY(hipMemset(c->d_bad, 0, 12));
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
    // mk_quad_kernel tables (mkacc_quad.hpp): TF = the forward table, TI[2^b + t] =
    // psi^-(t 2^(11-b)) for every bit b (negated pairs), TW[i] = psi^-i.  (Lane-major
    // copies of the per-lane blocks, free of LDS bank conflicts, measured -0.5 % for one
    // gate and +1 % at B = 1024: profiles/r6/v14)
    std::vector<uint2> qimg(3 * kN, make_uint2(0, 0));
    for (int i = 0; i < kN; ++i) qimg[i] = htf[i];
    for (int b = 0; b < kLogN; ++b)
        for (int t = 0; t < (1 << b); ++t) qimg[kN + (1 << b) + t] = npair(pwi[(size_t)t << (11 - b)]);
    for (int i = 0; i < kN; ++i) qimg[2 * kN + i] = pair(pwi[i]);
    HIP_TRY(hipMalloc(&c->d_qimg, qimg.size() * sizeof(uint2)));
    HIP_TRY(hipMemcpy(c->d_qimg, qimg.data(), qimg.size() * sizeof(uint2), hipMemcpyHostToDevice));
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
    for (void* p : {(void*)c->d_twf, (void*)c->d_twi, (void*)c->d_img, (void*)c->d_qimg, (void*)c->d_keys, (void*)c->d_pkey,
                    (void*)c->d_acc0, (void*)c->d_acc1, (void*)c->d_cvals, (void*)c->d_dscr, (void*)c->d_ct,
                    (void*)c->d_io, (void*)c->d_ksk, (void*)c->d_lweA, (void*)c->d_lweB, (void*)c->d_tv,
                    (void*)c->d_digits, (void*)c->d_kspart, (void*)c->d_bh, (void*)c->d_gin, (void*)c->d_gout, (void*)c->d_wtwf,
                    (void*)c->d_wtwi, (void*)c->d_wpsi, (void*)c->d_ftwf, (void*)c->d_fpsi, (void*)c->d_rtis,
                    (void*)c->d_r2tab,
                    (void*)c->d_wkeys, (void*)c->d_wpkey, (void*)c->d_wacc0,
                    (void*)c->d_wacc1, (void*)c->d_wcvals, (void*)c->d_wct, (void*)c->d_wio, (void*)c->d_bad,
                    (void*)c->d_psync})
        if (p) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    for (int j = 0; j < mkacc_ctx::kMaxStreams - 1; ++j) {
        if (c->xs[j]) (void)hipStreamDestroy(c->xs[j]);
        if (c->ev_join[j]) (void)hipEventDestroy(c->ev_join[j]);
    }
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
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

const char* mkacc_step_kernel_name(const mkacc_ctx* c, size_t B) {
    if (!c) return "";
    if (c->wide)
        return c->wfp ? "widereg2::step_kernel" : "wide::step_kernel";
    // small batches: the kernel that runs the steps after the first (all but one of
    // the k n steps; the first is one launch of mk_latd_kernel / mk_lat_kernel)
    if (const int qo = use_quad(c, B))
        return qo == 4   ? "mk_quadp2_run_kernel"
               : qo == 3 ? "mk_quadp_run_kernel"
               : qo == 2 ? (use_run(c, B) ? "mk_quad2_run_kernel" : "mk_quad2_kernel")
                       : (use_run(c, B) ? "mk_quad_run_kernel" : "mk_quad_kernel");
    if (use_lat(c, B)) {
        if (use_run(c, B)) return use_latd(c, B) ? "mk_latd_run_kernel" : "mk_lat_run_kernel";
        return use_latd(c, B) ? "mk_latd_kernel" : "mk_lat_kernel";
    }
    return c->step_ver == 2 ? "mk_step2_kernel" : "mk_step_kernel";
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
    if (const int prc = psync_enqueue(c)) return prc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return psync_result(c);
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
// Key-switching shape of an upload.  Validated first and committed to the
// context (ks_commit) only once the new key is on the device, so a failed
// upload never leaves have_ksk set with a key of another shape.
struct KsPlan {
    mkacc_ks_params ks;
    uint32_t dks, n_pad;
};
int check_ks(const mkacc_ks_params* ks, KsPlan& plan) {
    if (!ks) return fail(MKACC_E_ARG, "null key-switching parameters");
    if (ks->qKS < 2 || ks->qKS > 65535) return fail(MKACC_E_UNSUPPORTED, "engine supports qKS < 2^16");
    if (ks->baseKS < 2 || ks->baseKS > 256) return fail(MKACC_E_UNSUPPORTED, "engine supports baseKS <= 256");
    if (ks->n_out == 0 || ks->n_out > 4096) return fail(MKACC_E_ARG, "bad output dimension");
    plan.ks = *ks;
    plan.dks = ks_digit_count(ks->qKS, ks->baseKS);
    plan.n_pad = (ks->n_out + kKsTile - 1) / kKsTile * kKsTile;
    return MKACC_OK;
}
// the old key is gone from here on: no gate may run until ks_commit
void ks_drop(mkacc_ctx* c) { c->have_ksk = false; }
void ks_commit(mkacc_ctx* c, const KsPlan& plan) {
    c->ks = plan.ks;
    c->dks = plan.dks;
    c->n_pad = plan.n_pad;
}
}  // namespace

int mkacc_upload_ksk_mntru(mkacc_ctx* c, const mkacc_ks_params* ks, const uint32_t* ksk) {
    if (!c || !ksk) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW) return fail(MKACC_E_ARG, "KeySwitch2 keys belong to the MKNTRU method");
    KsPlan plan;
    int rc = check_ks(ks, plan);
    if (rc) return rc;
    const uint32_t k = c->p.k, dks = plan.dks, n = ks->n_out, npad = plan.n_pad;
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
    ks_drop(c);
    if (c->d_ksk) HIP_TRY(hipFree(c->d_ksk));
    c->d_ksk = nullptr;
    HIP_TRY(hipMalloc(&c->d_ksk, h.size() * 2));
    HIP_TRY(hipMemcpy(c->d_ksk, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    ks_commit(c, plan);
    c->have_ksk = true;
    return MKACC_OK;
}

int mkacc_upload_ksk_mklwe(mkacc_ctx* c, const mkacc_ks_params* ks, const uint32_t* A, const uint32_t* B) {
    if (!c || !A || !B) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW_B) return fail(MKACC_E_ARG, "MK-LWE KeySwitch keys belong to the MKNTRU_LWE method");
    if (int rc = reject_mkntru_b(c)) return rc;
    KsPlan plan;
    int rc = check_ks(ks, plan);
    if (rc) return rc;
    const size_t rows = (size_t)c->p.k * kN * ks->baseKS * plan.dks;
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
    ks_drop(c);
    if (c->d_lweA) HIP_TRY(hipFree(c->d_lweA));
    if (c->d_lweB) HIP_TRY(hipFree(c->d_lweB));
    c->d_lweA = nullptr;
    c->d_lweB = nullptr;
    HIP_TRY(hipMalloc(&c->d_lweA, ha.size() * 2));
    HIP_TRY(hipMalloc(&c->d_lweB, hb.size() * 2));
    HIP_TRY(hipMemcpy(c->d_lweA, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_lweB, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    ks_commit(c, plan);
    c->have_ksk = true;
    return MKACC_OK;
}

}  // extern "C"

namespace {
// the device key-switching uploads: layout kernel(s) on the context stream, then
// the range flag (d_bad[1]) read back; no keys are kept if a word is out of range
template <class L>
int ksk_device_finish(mkacc_ctx* c, const KsPlan& plan, L&& launch) {
    uint32_t* kbad = c->d_bad + 1;
    HIP_TRY(hipMemsetAsync(kbad, 0, 4, c->stream));
    int rc = launch(kbad);
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    uint32_t bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, kbad, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (bad) return fail(MKACC_E_RANGE, "key-switching key word not a canonical residue mod qKS");
    ks_commit(c, plan);
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
    KsPlan plan;
    int rc = check_ks(ks, plan);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    const size_t w = (size_t)c->p.k * plan.dks * kN * plan.n_pad;
    ks_drop(c);
    if (c->d_ksk) HIP_TRY(hipFree(c->d_ksk));
    c->d_ksk = nullptr;
    HIP_TRY(hipMalloc(&c->d_ksk, w * 2));
    return ksk_device_finish(c, plan, [&](uint32_t* kbad) {
        hipLaunchKernelGGL(ksk_mntru_layout_kernel, dim3((unsigned)((w + 255) / 256)), dim3(256), 0, c->stream,
                           (const uint32_t*)d_ksk, c->d_ksk, c->p.k, plan.dks, plan.ks.n_out, plan.n_pad,
                           (uint32_t)plan.ks.qKS, kbad);
        return MKACC_OK;
    });
}

int mkacc_upload_ksk_mklwe_device(mkacc_ctx* c, const mkacc_ks_params* ks, const void* d_A, const void* d_B) {
    if (!c || !d_A || !d_B) return fail(MKACC_E_ARG, "null argument");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->wide) return fail(MKACC_E_UNSUPPORTED, "the 64-bit word path covers EvalAcc only; NAND gates need Q < 2^27");
    if (c->method_class != XZW_B) return fail(MKACC_E_ARG, "MK-LWE KeySwitch keys belong to the MKNTRU_LWE method");
    if (int rc = reject_mkntru_b(c)) return rc;
    KsPlan plan;
    int rc = check_ks(ks, plan);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    const size_t rows = (size_t)c->p.k * kN * ks->baseKS * plan.dks, wa = rows * ks->n_out;
    ks_drop(c);
    if (c->d_lweA) HIP_TRY(hipFree(c->d_lweA));
    if (c->d_lweB) HIP_TRY(hipFree(c->d_lweB));
    c->d_lweA = c->d_lweB = nullptr;
    HIP_TRY(hipMalloc(&c->d_lweA, wa * 2));
    HIP_TRY(hipMalloc(&c->d_lweB, rows * 2));
    return ksk_device_finish(c, plan, [&](uint32_t* kbad) {
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
    if (const int prc = psync_enqueue(c)) return prc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return psync_result(c);
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
    if (const int prc = psync_enqueue(c)) return prc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (const int rc = psync_result(c)) return rc;
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

// Member i > 0 takes member 0's converted keys (device layout) by device copy.
// Two phases so the copies to all members run concurrently (one xGMI link per
// peer on a fully connected node): *_enqueue allocates and enqueues the copy on
// the member's stream, *_finish waits for it and marks the keys present.
int share_keys_enqueue(mkacc_ctx* dst, const mkacc_ctx* src) {
    const size_t kw = (size_t)src->p.k * (src->p.n + 1) * key_block_words(src), pw = (size_t)src->p.k * src->dg * kN;
    int rc;
    HIP_TRY(hipSetDevice(dst->device));
    HIP_TRY(hipStreamSynchronize(dst->stream));   // no batch of this member still reads the old keys
    dst->have_keys = false;
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
    return MKACC_OK;
}
int share_keys_finish(mkacc_ctx* dst, const mkacc_ctx*) {
    HIP_TRY(hipSetDevice(dst->device));
    HIP_TRY(hipStreamSynchronize(dst->stream));
    dst->have_keys = true;
    return MKACC_OK;
}

int share_ksk_enqueue(mkacc_ctx* dst, const mkacc_ctx* src) {
    HIP_TRY(hipSetDevice(dst->device));
    HIP_TRY(hipStreamSynchronize(dst->stream));
    ks_drop(dst);
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
    return MKACC_OK;
}
int share_ksk_finish(mkacc_ctx* dst, const mkacc_ctx* src) {
    HIP_TRY(hipSetDevice(dst->device));
    HIP_TRY(hipStreamSynchronize(dst->stream));
    ks_commit(dst, KsPlan{src->ks, src->dks, src->n_pad});
    dst->have_ksk = true;
    return MKACC_OK;
}

// Upload through member 0 (its host-side conversion and checks), wait for
// member 0's stream (the layout conversion may run there), then copy to every
// other member concurrently: all copies are enqueued before the first wait.
template <class F, class E, class W>
int group_upload(mkacc_group* g, F&& upload0, E&& enqueue, W&& finish) {
    if (!g || g->m.empty()) return fail(MKACC_E_ARG, "null group");
    int rc = upload0(g->m[0]);
    if (rc) return rc;
    mkacc_ctx* src = g->m[0];
    {
        std::lock_guard<std::mutex> lk(src->mu);
        HIP_TRY(hipSetDevice(src->device));
        HIP_TRY(hipStreamSynchronize(src->stream));
    }
    std::vector<std::unique_lock<std::mutex>> locks;
    for (size_t i = 1; i < g->m.size(); ++i) locks.emplace_back(g->m[i]->mu);
    int first = MKACC_OK;
    std::string msg;
    size_t started = 1;
    for (; started < g->m.size(); ++started)
        if ((rc = enqueue(g->m[started], src))) {
            first = rc;
            msg = mkacc_last_error();
            break;
        }
    // wait for every copy that was enqueued, even after a failure
    for (size_t i = 1; i < started; ++i)
        if ((rc = finish(g->m[i], src)) && !first) {
            first = rc;
            msg = mkacc_last_error();
        }
    if (first) return fail(first, msg);
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
    return group_upload(g, [&](mkacc_ctx* c) { return mkacc_upload_keys(c, evk, pkey); }, share_keys_enqueue,
                        share_keys_finish);
}
int mkacc_group_upload_keys_u64(mkacc_group* g, const uint64_t* evk, const uint64_t* pkey) {
    return group_upload(g, [&](mkacc_ctx* c) { return mkacc_upload_keys_u64(c, evk, pkey); }, share_keys_enqueue,
                        share_keys_finish);
}
int mkacc_group_upload_ksk_mntru(mkacc_group* g, const mkacc_ks_params* ks, const uint32_t* ksk) {
    return group_upload(g, [&](mkacc_ctx* c) { return mkacc_upload_ksk_mntru(c, ks, ksk); }, share_ksk_enqueue,
                        share_ksk_finish);
}
int mkacc_group_upload_ksk_mklwe(mkacc_group* g, const mkacc_ks_params* ks, const uint32_t* A, const uint32_t* B) {
    return group_upload(g, [&](mkacc_ctx* c) { return mkacc_upload_ksk_mklwe(c, ks, A, B); }, share_ksk_enqueue,
                        share_ksk_finish);
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
