// vgpr_lds.hip -- two ~256-VGPR waves per SIMD (two 4-wave workgroups per CU),
// each wave doing deterministic integer mixing on NX registers that make an
// LDS round trip every round (like the step kernel's transposes) plus NY
// registers that stay in VGPRs.  The host recomputes every thread's digest.
//   ./vgpr_lds [rounds] [blocks] [lds_bytes]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef NX
#define NX 32
#endif
#ifndef NY
#define NY 80
#endif
#ifndef PERM
#define PERM 1   // read back through a lane permutation (lane ^ 1), like a transpose
#endif

__host__ __device__ inline uint32_t mix(uint32_t a, uint32_t b, uint32_t c) {
    const uint64_t p = (uint64_t)a * 0x9E3779B1u + b;
    return (uint32_t)(p >> 32) ^ (uint32_t)p ^ (c >> 3);
}

#ifndef VMEM
#define VMEM 0
#endif
#ifndef GATHER
#define GATHER 0
#endif
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256, 2) void stress(uint32_t* out, int rounds, const uint32_t* tab) {
    extern __shared__ uint32_t lds[];
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(tab), (short)0, 1 << 20, 0x00020000);
    uint32_t* gt = lds + 4 * (NX * 64);   // 8 KB gather table after the wave scratch
    for (int i = threadIdx.x; i < 2048; i += 256) gt[i] = tab[i] * 7u + 1u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t* ws = lds + wv * (NX * 64);
    uint32_t x[NX], y[NY];
    // each lane's state depends only on its wave (the host replays whole waves)
#pragma unroll
    for (int i = 0; i < NX; ++i) x[i] = t * 2654435761u + (uint32_t)i * 40503u;
#pragma unroll
    for (int i = 0; i < NY; ++i) y[i] = t * 2246822519u + (uint32_t)i * 3266489917u;
    uint32_t acc = t;
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int i = 0; i < NY; ++i) {
            acc = mix(acc, y[i], (uint32_t)r);
            y[i] = mix(y[i], acc, (uint32_t)i);
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            acc = mix(acc, x[i], (uint32_t)r);
            x[i] = mix(x[i], acc, (uint32_t)i);
        }
        if (VMEM) {
            // shared-table dwordx4 loads (L1/L2), offset depends on the round
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rt, lane * 16u, ((r * 4 + g) & 255) * 1024u, 0);
                x[4 * g] ^= v.x; x[4 * g + 1] ^= v.y; x[4 * g + 2] ^= v.z; x[4 * g + 3] ^= v.w;
            }
        }
        if (GATHER) {
#pragma unroll
            for (int i = 16; i < NX; ++i) x[i] += gt[(x[i] ^ acc) & 2047u];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) ws[i * 64 + lane] = x[i];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < NX; ++i) x[i] = ws[i * 64 + (PERM ? (lane ^ 1) : lane)];
        asm volatile("" ::: "memory");
    }
    uint32_t h = acc;
#pragma unroll
    for (int i = 0; i < NX; ++i) h = h * 31u + x[i];
#pragma unroll
    for (int i = 0; i < NY; ++i) h = h * 31u + y[i];
    out[t] = h;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 500;
    const int blocks = argc > 2 ? atoi(argv[2]) : 2048;
    const size_t ldsb = argc > 3 ? (size_t)atol(argv[3]) : 74752;
    const size_t n = (size_t)blocks * 256;
    uint32_t* d;
    if (hipMalloc(&d, n * 4) != hipSuccess) return 2;
    std::vector<uint32_t> tab(1 << 18);
    for (size_t i = 0; i < tab.size(); ++i) tab[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;
    uint32_t* dt;
    hipMalloc(&dt, tab.size() * 4);
    hipMemcpy(dt, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(stress, dim3(blocks), dim3(256), ldsb, 0, d, rounds, dt);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
    std::vector<uint32_t> h(n);
    hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    // replay one wave (64 lanes) on the host
    auto wave = [&](uint32_t t0, std::vector<uint32_t>& res) {
        std::vector<uint32_t> x(64 * NX), y(64 * NY), acc(64), tmp(64 * NX);
        for (int l = 0; l < 64; ++l) {
            const uint32_t t = t0 + l;
            for (int i = 0; i < NX; ++i) x[l * NX + i] = t * 2654435761u + (uint32_t)i * 40503u;
            for (int i = 0; i < NY; ++i) y[l * NY + i] = t * 2246822519u + (uint32_t)i * 3266489917u;
            acc[l] = t;
        }
        for (int r = 0; r < rounds; ++r) {
            for (int l = 0; l < 64; ++l) {
                uint32_t a = acc[l];
                for (int i = 0; i < NY; ++i) { a = mix(a, y[l * NY + i], (uint32_t)r); y[l * NY + i] = mix(y[l * NY + i], a, (uint32_t)i); }
                for (int i = 0; i < NX; ++i) { a = mix(a, x[l * NX + i], (uint32_t)r); x[l * NX + i] = mix(x[l * NX + i], a, (uint32_t)i); }
                acc[l] = a;
            }
            for (int l = 0; l < 64; ++l) {
                if (VMEM)
                    for (int g = 0; g < 4; ++g)
                        for (int c = 0; c < 4; ++c)
                            x[l * NX + 4 * g + c] ^= tab[(((r * 4 + g) & 255) * 1024u + l * 16u) / 4 + c];
                if (GATHER)
                    for (int i = 16; i < NX; ++i) x[l * NX + i] += tab[(x[l * NX + i] ^ acc[l]) & 2047u] * 7u + 1u;
            }
            tmp = x;
            for (int l = 0; l < 64; ++l)
                for (int i = 0; i < NX; ++i) x[l * NX + i] = tmp[(PERM ? (l ^ 1) : l) * NX + i];
        }
        res.resize(64);
        for (int l = 0; l < 64; ++l) {
            uint32_t hh = acc[l];
            for (int i = 0; i < NX; ++i) hh = hh * 31u + x[l * NX + i];
            for (int i = 0; i < NY; ++i) hh = hh * 31u + y[l * NY + i];
            res[l] = hh;
        }
    };
    long bad_lo = 0, bad_hi = 0, waves = 0;
    std::vector<uint32_t> res;
    for (int b = 0; b < blocks; b += (b < 256 ? 17 : 5)) {
        for (int w = 0; w < 4; ++w) {
            const uint32_t t0 = (uint32_t)b * 256 + 64 * w;
            wave(t0, res);
            ++waves;
            int bad = 0;
            for (int l = 0; l < 64; ++l) bad += h[t0 + l] != res[l];
            if (bad) (b < 256 ? bad_lo : bad_hi)++;
        }
    }
    printf("NX %d NY %d rounds %d blocks %d lds %zu: checked %ld waves, bad waves in first 256 blocks %ld, later %ld\n",
           NX, NY, rounds, blocks, ldsb, waves, bad_lo, bad_hi);
    return 0;
}
