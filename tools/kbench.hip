// kbench.hip -- component timing of the accumulator building blocks on gfx950.
// Each wave runs ITERS back-to-back NTTs on its own polynomial (4096 waves,
// the step kernel's occupancy), so the time per NTT-wave is the cost the step
// kernel pays per transform.  Build: hipcc --offload-arch=gfx950 -O3 -I../include
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../mkfhe_amd/csrc/mkacc_device.hpp"
#include "../mkfhe_amd/csrc/mkacc_host_math.hpp"

using namespace mkacc;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(256, 4) void chain(uint32_t* data, const uint2* twf, const uint2* twi, int iters, uint32_t Q) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t l = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t p = blockIdx.x * 4 + wv;
    uint32_t* lds = smem + wv * kLdsWords;
    uint32_t x[kRegs];
    load_c4(x, data + (size_t)p * kN, l);
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {
            ntt_fwd(x, lds, twf, twf, twf + kTwlC, l, Q);
#pragma unroll
            for (int r = 0; r < kRegs; ++r) x[r] = min(x[r], x[r] - 2 * Q);
        } else if (MODE == 1) {
            ntt_inv_noscale(x, lds, twi, twi, l, Q);
        } else {
            transpose<0, 1>(x, lds, l);
            transpose<1, 2>(x, lds, l);
        }
    }
    store_c4(x, data + (size_t)p * kN, l);
}

int main() {
    const uint64_t Q = 134176769, psi = 100530;
    std::vector<uint64_t> tf(kN), ti(kN);
    uint64_t x = 1, xi = 1, psii = modinv(psi, Q);
    for (uint32_t i = 0; i < (uint32_t)kN; ++i) {
        uint32_t r = bit_reverse(i, 11);
        tf[r] = x; ti[r] = xi;
        x = mulmod(x, psi, Q); xi = mulmod(xi, psii, Q);
    }
    std::vector<uint2> htf(kN), hti(kN);
    for (int i = 0; i < kN; ++i) {
        htf[i] = make_uint2((uint32_t)tf[i], (uint32_t)(((unsigned __int128)tf[i] << 32) / Q));
        hti[i] = make_uint2((uint32_t)ti[i], (uint32_t)(((unsigned __int128)ti[i] << 32) / Q));
    }
    const int waves = 4096, iters = 24;
    std::vector<uint32_t> h((size_t)waves * kN);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)((i * 2654435761u) % Q);
    uint32_t* d; uint2 *dtf, *dti;
    CHK(hipMalloc(&d, h.size() * 4)); CHK(hipMalloc(&dtf, kN * 8)); CHK(hipMalloc(&dti, kN * 8));
    CHK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dtf, htf.data(), kN * 8, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dti, hti.data(), kN * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    const char* names[] = {"ntt_fwd", "ntt_inv", "2 transposes"};
    // occupancy forced through the dynamic LDS size: 4 waves per block,
    // blocks per CU = 160 KiB / lds  ->  waves per SIMD = blocks per CU
    for (int occ : {4, 2, 1})
    for (int mode = 0; mode < 3; ++mode) {
        auto fn = mode == 0 ? chain<0> : (mode == 1 ? chain<1> : chain<2>);
        const size_t lds = occ == 4 ? 4 * kLdsWords * 4 : (occ == 2 ? 64 * 1024 : 100 * 1024);
        if (mode == 0) printf("-- %d waves/SIMD\n", occ);
        for (int rep = 0; rep < 3; ++rep) {
            CHK(hipEventRecord(e0));
            hipLaunchKernelGGL(fn, dim3(waves / 4), dim3(256), lds, 0, d, dtf, dti, iters, (uint32_t)Q);
            CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            double per = ms * 1e3 / iters;   // us per "one op on every wave"
            if (rep == 2)
                printf("%-14s %8.2f us per op over %d waves = %7.1f G polys/s (%.1f ns/poly)\n", names[mode], per, waves,
                       waves / per / 1e3, per * 1e3 / waves);
        }
    }
    return 0;
}
