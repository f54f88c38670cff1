// ubench_lat.hip -- the transforms at the small-batch kernels' occupancy: one wave
// per SIMD (four waves per CU, one workgroup per CU), the shape of mk_latd_kernel at
// B = 1.  Times ITERS back-to-back transforms per wave (us per transform), and the
// dependent-issue latency of the VALU ops the butterflies are built from.
// Build (tools/ubench_lat.sh): hipcc --offload-arch=gfx950 -O3 [-DMKACC_TW_FENCE=0]
//                              [-mllvm -amdgpu-sched-strategy=...] ubench_lat.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../mkfhe_amd/csrc/mkacc_device.hpp"

using namespace mkacc;

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);        \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int kImgPairs = kTwlPairs + kInvImgPairs;   // forward image, inverse image + twist

// MODE 0: ntt_fwd, 1: ntt_inv, 2: ntt_fwd with the per-lane image in LDS, 3: ntt_inv
// with it in LDS, 4: fwd + inv back to back (one round trip), 5: two polynomials per
// wave, fwd on each (the interleaving the compiler finds across two calls)
template <int MODE>
__global__ __launch_bounds__(256, 1) void chain(uint32_t* data, const uint2* tws, const uint2* img, int iters,
                                                uint32_t Q, uint32_t m1) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t l = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint2* limg = reinterpret_cast<uint2*>(smem);
    for (int i = threadIdx.x; i < kImgPairs; i += blockDim.x) limg[i] = img[i];
    __syncthreads();
    uint32_t* lds = smem + 2 * kImgPairs + wv * kLdsWords;
    const uint2* twf = (MODE == 2 || MODE == 3) ? limg : img;
    const uint2* twi = twf + kTwlPairs;
    const uint32_t p = blockIdx.x * 4 + wv;
    uint32_t x[kRegs], y[kRegs];
    load_c4(x, data + (size_t)p * kN, l);
    if (MODE == 5) load_c4(y, data + (size_t)(p ^ 1) * kN, l);
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0 || MODE == 2 || MODE == 4 || MODE == 5) {
            ntt_fwd(x, lds, tws, twf, twf + kTwlC, l, Q, m1);
#pragma unroll
            for (int r = 0; r < kRegs; ++r) x[r] = min(x[r], x[r] - 2 * Q);
        }
        if (MODE == 5) {
            ntt_fwd(y, lds + kLdsWords * 4, tws, twf, twf + kTwlC, l, Q, m1);
#pragma unroll
            for (int r = 0; r < kRegs; ++r) y[r] = min(y[r], y[r] - 2 * Q);
        }
        if (MODE == 1 || MODE == 3 || MODE == 4) ntt_inv(x, lds, tws, twi, l, Q);
    }
    store_c4(x, data + (size_t)p * kN, l);
    if (MODE == 5) store_c4(y, data + (size_t)(p ^ 1) * kN, l);
}

// dependent chains: OP 0 v_add_u32, 1 v_mul_hi_u32, 2 v_mad_u64_u32 (low word fed back),
// 3 v_mul_lo_u32; CH independent chains interleaved
template <int OP, int CH>
__global__ __launch_bounds__(256, 1) void dep(uint32_t* out, int iters, uint32_t c) {
    uint32_t v[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) v[j] = threadIdx.x + j;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[j]) : "s"(c));
                if (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[j]) : "s"(c));
                if (OP == 2) {
                    uint64_t r;
                    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(v[j]), "s"(c) : "vcc");
                    v[j] = (uint32_t)r;
                }
                if (OP == 3) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[j]) : "s"(c));
            }
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) s += v[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char** argv) {
    const uint32_t Q = 134176769;
    const uint32_t m1 = (uint32_t)((1ull << 32) / Q);
    const int blocks = 256, iters = 200;
    std::vector<uint2> himg(kImgPairs), hts(kN);
    uint64_t s = 88172645463325252ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (auto& t : himg) {
        const uint32_t w = (uint32_t)(rnd() % Q);
        t = make_uint2(w, (uint32_t)(((uint64_t)w << 32) / Q));
    }
    for (auto& t : hts) {
        const uint32_t w = (uint32_t)(rnd() % Q);
        t = make_uint2(0u - w, (uint32_t)(((uint64_t)w << 32) / Q));
    }
    std::vector<uint32_t> h((size_t)blocks * 4 * kN);
    for (auto& v : h) v = (uint32_t)(rnd() % Q);
    uint32_t* d;
    uint2 *dimg, *dts;
    CHK(hipMalloc(&d, h.size() * 4));
    CHK(hipMalloc(&dimg, himg.size() * 8));
    CHK(hipMalloc(&dts, hts.size() * 8));
    CHK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dimg, himg.data(), himg.size() * 8, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dts, hts.data(), hts.size() * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    // LDS: the image + four transpose scratches + 4 more for MODE 5 (> 80 KB: one block per CU)
    const size_t lds = (size_t)(2 * kImgPairs + 8 * kLdsWords) * 4;
    auto run = [&](auto fn, const char* name, double per_iter) -> int {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            CHK(hipEventRecord(e0));
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), lds, 0, d, dts, dimg, iters, Q, m1);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-34s %8.3f us per transform per wave (1 wave/SIMD)\n", name, best * 1e3 / iters / per_iter);
        return 0;
    };
    const char* tag = argc > 1 ? argv[1] : "";
    printf("-- build %s\n", tag);
    if (run(chain<0>, "ntt_fwd (image in HBM/L2)", 1)) return 1;
    if (run(chain<1>, "ntt_inv (image in HBM/L2)", 1)) return 1;
    if (run(chain<2>, "ntt_fwd (image in LDS)", 1)) return 1;
    if (run(chain<3>, "ntt_inv (image in LDS)", 1)) return 1;
    if (run(chain<4>, "ntt_fwd + ntt_inv", 2)) return 1;
    if (run(chain<5>, "two polys per wave, fwd each", 2)) return 1;
    uint32_t* o;
    CHK(hipMalloc(&o, blocks * 256 * 4));
    auto dep_run = [&](auto fn, const char* name, int ch) -> int {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            CHK(hipEventRecord(e0));
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), lds, 0, o, 2000, 12345u);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        // cycles per instruction at 2.4 GHz: ms * 2.4e6 / (2000 * 16 * ch)
        printf("%-34s %6.2f cycles per instruction (%d chain%s)\n", name, best * 2.4e6 / (2000.0 * 16 * ch), ch,
               ch > 1 ? "s" : "");
        return 0;
    };
    if (dep_run(dep<0, 1>, "v_add_u32 dependent", 1)) return 1;
    if (dep_run(dep<1, 1>, "v_mul_hi_u32 dependent", 1)) return 1;
    if (dep_run(dep<2, 1>, "v_mad_u64_u32 dependent", 1)) return 1;
    if (dep_run(dep<3, 1>, "v_mul_lo_u32 dependent", 1)) return 1;
    if (dep_run(dep<1, 4>, "v_mul_hi_u32 x4", 4)) return 1;
    if (dep_run(dep<2, 4>, "v_mad_u64_u32 x4", 4)) return 1;
    if (dep_run(dep<2, 8>, "v_mad_u64_u32 x8", 8)) return 1;
    return 0;
}
