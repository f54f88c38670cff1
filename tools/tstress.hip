// tstress.hip -- stress the per-wave LDS transposes of mkacc_device.hpp in the
// step kernel's geometry (512-thread workgroups, 2 waves / SIMD, ~132 KiB LDS):
// each wave round-trips its polynomial through the four transposes many times
// and counts words that come back wrong, per wave slot.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../mkfhe_amd/csrc/mkacc_device.hpp"
using namespace mkacc;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kImg = 16256;
template <int WAIT>
__global__ __launch_bounds__(512, 2) void tstress(unsigned* bad, int iters) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t l = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* lds = smem + kImg + wv * kLdsWords;
    uint32_t x[kRegs];
    for (int r = 0; r < kRegs; ++r) x[r] = (blockIdx.x << 20) ^ (wv << 16) ^ (l << 8) ^ r;
    unsigned nb = 0;
    for (int it = 0; it < iters; ++it) {
        transpose<0, 1>(x, lds, l);
        for (int r = 0; r < kRegs; ++r) x[r] = x[r] * 3u + 1u;      // VALU work between transposes
        transpose<1, 2>(x, lds, l);
        for (int r = 0; r < kRegs; ++r) x[r] = (x[r] - 1u) * 2863311531u;   // inverse of *3+1
        transpose<2, 1>(x, lds, l);
        transpose<1, 0>(x, lds, l);
        for (int r = 0; r < kRegs; ++r) nb += x[r] != ((blockIdx.x << 20) ^ (wv << 16) ^ (l << 8) ^ (uint32_t)r);
    }
    if (nb) atomicAdd(&bad[wv], nb);
}

int main() {
    unsigned* d;
    CHK(hipMalloc(&d, 64));
    const size_t lds = (kImg + 8 * kLdsWords) * 4;
    for (int rep = 0; rep < 3; ++rep) {
        CHK(hipMemset(d, 0, 64));
        hipLaunchKernelGGL(tstress<0>, dim3(2048), dim3(512), lds, 0, d, 200);
        CHK(hipDeviceSynchronize());
        unsigned h[8];
        CHK(hipMemcpy(h, d, 32, hipMemcpyDeviceToHost));
        printf("rep %d bad words per wave slot:", rep);
        for (int i = 0; i < 8; ++i) printf(" %u", h[i]);
        printf("\n");
    }
    return 0;
}
