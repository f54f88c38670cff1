// vgpr_stress.hip -- is register state of a wave preserved when two waves
// using ~256 VGPRs each share a SIMD?  Every thread runs a deterministic
// integer mixing chain over NV live registers (v_mad_u64_u32-heavy, like the
// step kernel) and stores a digest; the host recomputes every digest.
//   hipcc --offload-arch=gfx950 -O3 -o vgpr_stress vgpr_stress.hip
//   ./vgpr_stress [rounds] [blocks] [lds_bytes]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef NV
#define NV 232
#endif

__host__ __device__ inline uint32_t mix(uint32_t a, uint32_t b, uint32_t c) {
    const uint64_t p = (uint64_t)a * 0x9E3779B1u + b;
    return (uint32_t)(p >> 32) ^ (uint32_t)p ^ (c >> 3);
}

#ifndef LDS_RT
#define LDS_RT 0
#endif
__global__ __launch_bounds__(256, 2) void stress(uint32_t* out, int rounds) {
    extern __shared__ uint32_t lds[];
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t* mine = lds + (threadIdx.x >> 6) * (NV * 64 + 64) + (threadIdx.x & 63);
    uint32_t x[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) x[i] = t * 2654435761u + (uint32_t)i * 40503u;
    uint32_t acc = t;
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            acc = mix(acc, x[i], (uint32_t)r);
            x[i] = mix(x[i], acc, (uint32_t)i);
        }
        if (LDS_RT) {
            // round trip of every live register through this wave's LDS scratch
#pragma unroll
            for (int i = 0; i < NV; ++i) mine[i * 64] = x[i];
            asm volatile("" ::: "memory");
#pragma unroll
            for (int i = 0; i < NV; ++i) x[i] = ((volatile uint32_t*)mine)[i * 64];
            asm volatile("" ::: "memory");
        }
    }
    uint32_t h = acc;
#pragma unroll
    for (int i = 0; i < NV; ++i) h = h * 31u + x[i];
    out[t] = h;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
    const int blocks = argc > 2 ? atoi(argv[2]) : 2048;
    const size_t ldsb = argc > 3 ? (size_t)atol(argv[3]) : 74752;
    const size_t n = (size_t)blocks * 256;
    uint32_t* d;
    if (hipMalloc(&d, n * 4) != hipSuccess) return 2;
    hipLaunchKernelGGL(stress, dim3(blocks), dim3(256), ldsb, 0, d, rounds);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
    std::vector<uint32_t> h(n);
    hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    // expected digest per thread (in-place sequential update, the device loop's order)
    auto digest = [&](uint32_t t) {
        std::vector<uint32_t> x(NV);
        for (int i = 0; i < NV; ++i) x[i] = t * 2654435761u + (uint32_t)i * 40503u;
        uint32_t acc = t;
        for (int r = 0; r < rounds; ++r)
            for (int i = 0; i < NV; ++i) {
                acc = mix(acc, x[i], (uint32_t)r);
                x[i] = mix(x[i], acc, (uint32_t)i);
            }
        uint32_t hh = acc;
        for (int i = 0; i < NV; ++i) hh = hh * 31u + x[i];
        return hh;
    };
    long bad_lo = 0, bad_hi = 0, checked = 0;
    for (int b = 0; b < blocks; b += (b < 1024 ? 37 : 7)) {
        for (uint32_t k = 0; k < 256; k += 5) {
            const uint32_t t = (uint32_t)b * 256 + k;
            const uint32_t want = digest(t);
            ++checked;
            if (h[t] != want) (b < 256 ? bad_lo : bad_hi)++;
        }
    }
    printf("rounds %d blocks %d lds %zu: checked %ld threads, bad in first 256 blocks %ld, later %ld\n", rounds,
           blocks, ldsb, checked, bad_lo, bad_hi);
    return 0;
}
