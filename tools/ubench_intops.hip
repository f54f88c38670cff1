// Microbenchmark: VALU throughput of the integer / fp64 primitives that a
// 27-bit modular multiply can be built from on gfx950.  Decides which
// reduction the accumulator kernels use (see DESIGN.md "Modular arithmetic").
//
// Each kernel runs R rounds over 8 independent chains per lane so the result
// is issue-bound, not latency-bound.  Reports G lane-ops/s per primitive and
// the rate of three complete mod-mul formulations (Shoup, Barrett, fp64).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int R = 4096;
constexpr uint32_t Q = 134176769u;

__global__ void k_mullo(uint32_t* out, uint32_t s) {
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j * 7 + s;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[j] * (a[j] | 1u);
    uint32_t x = 0; for (int j = 0; j < 8; ++j) x ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_mulhi(uint32_t* out, uint32_t s) {
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j * 7 + s;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = __umulhi(a[j], 0x9E3779B9u) + a[j];
    uint32_t x = 0; for (int j = 0; j < 8; ++j) x ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_mad64(uint32_t* out, uint32_t s) {
    uint64_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j * 7 + s;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = (uint64_t)(uint32_t)a[j] * 0x9E3779B9u + (a[j] >> 32);
    uint32_t x = 0; for (int j = 0; j < 8; ++j) x ^= (uint32_t)a[j] ^ (uint32_t)(a[j] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_mul24(uint32_t* out, uint32_t s) {
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j * 7 + s;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = __umul24(a[j], 0x5A5A5Au) + 1u;
    uint32_t x = 0; for (int j = 0; j < 8; ++j) x ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_add(uint32_t* out, uint32_t s) {
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j * 7 + s;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = (a[j] + 0x3779B9u) ^ s;
    uint32_t x = 0; for (int j = 0; j < 8; ++j) x ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_fma64(uint32_t* out, uint32_t s) {
    double a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j * 7 + s;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = fma(a[j], 0.999999, 1.0);
    double x = 0; for (int j = 0; j < 8; ++j) x += a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)x;
}
__global__ void k_fma32(uint32_t* out, uint32_t s) {
    float a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j * 7 + s;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = fmaf(a[j], 0.999999f, 1.0f);
    float x = 0; for (int j = 0; j < 8; ++j) x += a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)x;
}
// Shoup mod-mul by a constant: 1 mulhi + 2 mullo + sub + min
__global__ void k_shoup(uint32_t* out, uint32_t s) {
    uint32_t a[8];
    const uint32_t w = 100530u, wp = (uint32_t)(((uint64_t)w << 32) / Q);
    for (int j = 0; j < 8; ++j) a[j] = (threadIdx.x + j * 7 + s) % Q;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t qh = __umulhi(a[j], wp);
            uint32_t t = a[j] * w - qh * Q;
            a[j] = min(t, t - Q);
        }
    uint32_t x = 0; for (int j = 0; j < 8; ++j) x ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// Barrett mod-mul of two variables: mad64 product, alignbit, mulhi, mullo, 2x(sub,min)
__global__ void k_barrett(uint32_t* out, uint32_t s) {
    uint32_t a[8];
    const uint32_t mu = (uint32_t)((1ull << 58) / Q);
    const uint32_t b = 77777777u;
    for (int j = 0; j < 8; ++j) a[j] = (threadIdx.x + j * 7 + s) % Q;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint64_t p = (uint64_t)a[j] * b;
            uint32_t sh = (uint32_t)(p >> 26);
            uint32_t qh = __umulhi(sh, mu);
            uint32_t t = (uint32_t)p - qh * Q;
            t = min(t, t - Q);
            a[j] = min(t, t - Q);
        }
    uint32_t x = 0; for (int j = 0; j < 8; ++j) x ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// fp64 Barrett: exact for Q < 2^27 (product < 2^54 handled by hi/lo split)
__global__ void k_fp64mm(uint32_t* out, uint32_t s) {
    double a[8];
    const double Qd = (double)Q, Qi = 1.0 / (double)Q, b = 77777777.0;
    for (int j = 0; j < 8; ++j) a[j] = (double)((threadIdx.x + j * 7 + s) % Q);
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            double hi = a[j] * b;
            double lo = fma(a[j], b, -hi);
            double qq = rint(hi * Qi);
            double t = fma(-qq, Qd, hi) + lo;
            t = t < 0 ? t + Qd : t;
            a[j] = t >= Qd ? t - Qd : t;
        }
    double x = 0; for (int j = 0; j < 8; ++j) x += a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)x;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
    printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
    const int blocks = prop.multiProcessorCount * 16, threads = 256;
    uint32_t* d; CHK(hipMalloc(&d, (size_t)blocks * threads * 4));
    struct { const char* name; kfn f; double ops_per_iter; } ks[] = {
        {"v_add_u32+xor (2 ops)", k_add, 2}, {"v_mul_lo_u32", k_mullo, 1}, {"v_mul_hi_u32 (+add)", k_mulhi, 1},
        {"v_mad_u64_u32", k_mad64, 1}, {"v_mul_u32_u24 (+add)", k_mul24, 1}, {"v_fma_f32", k_fma32, 1},
        {"v_fma_f64", k_fma64, 1}, {"shoup mulmod", k_shoup, 1}, {"barrett mulmod", k_barrett, 1},
        {"fp64 mulmod", k_fp64mm, 1}};
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0));
        for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)it);
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        double ops = 5.0 * blocks * threads * (double)R * 8 * k.ops_per_iter;
        printf("%-24s %9.1f G lane-ops/s  (%.3f ms)\n", k.name, ops / (ms * 1e-3) / 1e9, ms / 5);
    }
    CHK(hipFree(d));
    return 0;
}
