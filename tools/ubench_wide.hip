// ubench_wide.hip -- issue rate of the 64-bit word path's butterflies at the
// config-5 modulus (Q = 1125899906826241 < 2^50): the integer lazy CT
// butterfly of mkacc_wide.hpp (limb-built Shoup, 11 multiply-adds) against an
// exact FP64 butterfly (tools/fp64_modmul_check.c: h = a w, l = fma(a, w, -h),
// q = rint(h / Q), T = fma(-q, Q, h) + l), with the a-input reduced every
// stage or every second stage.  8 independent butterflies per lane, 2 waves
// per SIMD (the wide kernel runs 4 workgroups of 256 threads per CU).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_wide tools/ubench_wide.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int R = 1024;
constexpr uint64_t Q = 1125899906826241ull;

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
    return (uint64_t)a * b + c;
}
__device__ __forceinline__ uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
// mkacc_wide.hpp shoup3 (same formula, no pinning)
__device__ __forceinline__ uint64_t shoup3(uint64_t x, uint64_t w, uint64_t wp, uint64_t nQ) {
    const uint32_t xl = lo32(x), xh = hi32(x);
    const uint64_t t1 = (uint64_t)xh * lo32(wp);
    const uint64_t s = (uint64_t)xl * hi32(wp) + lo32(t1);
    const uint64_t q = (uint64_t)xh * hi32(wp) + hi32(t1) + hi32(s);
    const uint64_t A = (uint64_t)lo32(q) * lo32(nQ) + (uint64_t)xl * lo32(w);
    uint64_t h = (uint64_t)xh * lo32(w) + hi32(A);
    h = (uint64_t)xl * hi32(w) + h;
    h = (uint64_t)hi32(q) * lo32(nQ) + h;
    h = (uint64_t)lo32(q) * hi32(nQ) + h;
    return ((uint64_t)lo32(h) << 32) | lo32(A);
}
__device__ __forceinline__ uint64_t csub(uint64_t x, uint64_t m) { return x >= m ? x - m : x; }

// integer lazy CT butterfly of mkacc_wide.hpp: values in [0, 6Q)
__global__ __launch_bounds__(256, 2) void k_int(uint64_t* out, uint64_t w, uint64_t wp) {
    uint64_t a[8], b[8];
    for (int j = 0; j < 8; ++j) { a[j] = (threadIdx.x * 977 + j * 7919) % Q; b[j] = (threadIdx.x * 131 + j) % Q; }
    const uint64_t Q3 = 3 * Q, nQ = 0 - Q;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t X = csub(a[j], Q3);
            const uint64_t T = shoup3(b[j], w, wp, nQ);
            a[j] = X + T;
            b[j] = X + Q3 - T;
        }
    uint64_t x = 0;
    for (int j = 0; j < 8; ++j) x ^= a[j] ^ b[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ double mmw(double b, double w, double Qd, double Qi) {
    const double h = b * w;
    const double l = fma(b, w, -h);
    const double q = rint(h * Qi);
    return fma(-q, Qd, h) + l;
}
__device__ __forceinline__ double red(double x, double Qd, double Qi) { return fma(-rint(x * Qi), Qd, x); }

// FP64 CT butterfly, a reduced every stage (|a| <= Q/2, T <= 2Q, outputs <= 2.5Q)
__global__ __launch_bounds__(256, 2) void k_fp1(uint64_t* out, double w) {
    double a[8], b[8];
    const double Qd = (double)Q, Qi = 1.0 / Qd;
    for (int j = 0; j < 8; ++j) { a[j] = (double)((threadIdx.x * 977 + j * 7919) % 1000003); b[j] = (double)j; }
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const double X = red(a[j], Qd, Qi);
            const double T = mmw(b[j], w, Qd, Qi);
            a[j] = X + T;
            b[j] = X - T;
        }
    double x = 0;
    for (int j = 0; j < 8; ++j) x += a[j] - b[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(int64_t)x;
}
// FP64 CT butterfly, a reduced every second stage (outputs <= 4.5Q, b input <= 8Q)
__global__ __launch_bounds__(256, 2) void k_fp2(uint64_t* out, double w) {
    double a[8], b[8];
    const double Qd = (double)Q, Qi = 1.0 / Qd;
    for (int j = 0; j < 8; ++j) { a[j] = (double)((threadIdx.x * 977 + j * 7919) % 1000003); b[j] = (double)j; }
    for (int r = 0; r < R; r += 2)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const double X = s == 0 ? red(a[j], Qd, Qi) : a[j];
                const double T = mmw(b[j], w, Qd, Qi);
                a[j] = X + T;
                b[j] = X - T;
            }
    double x = 0;
    for (int j = 0; j < 8; ++j) x += a[j] - b[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(int64_t)x;
}
// the bare FP64 product (6 ops) and the integer Shoup product alone
__global__ __launch_bounds__(256, 2) void k_fpmm(uint64_t* out, double w) {
    double a[8];
    const double Qd = (double)Q, Qi = 1.0 / Qd;
    for (int j = 0; j < 8; ++j) a[j] = (double)((threadIdx.x * 977 + j * 7919) % 1000003);
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = mmw(a[j], w, Qd, Qi);
    double x = 0;
    for (int j = 0; j < 8; ++j) x += a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(int64_t)x;
}
__global__ __launch_bounds__(256, 2) void k_intmm(uint64_t* out, uint64_t w, uint64_t wp) {
    uint64_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = (threadIdx.x * 977 + j * 7919) % Q;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = shoup3(a[j], w, wp, 0 - Q);
    uint64_t x = 0;
    for (int j = 0; j < 8; ++j) x ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 8, threads = 256;
    uint64_t* d;
    CHK(hipMalloc(&d, (size_t)blocks * threads * 8));
    const uint64_t w = 1080667890455ull % Q;
    const uint64_t wp = (uint64_t)(((unsigned __int128)w << 64) / Q);
    const double wd = (double)(int64_t)(w > Q / 2 ? w - Q : w);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) -> int {
        launch();
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0));
        for (int it = 0; it < 5; ++it) launch();
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        const double n = 5.0 * blocks * threads * (double)R * 8;
        printf("%-44s %8.1f G/s  (%.3f ms per launch)\n", name, n / (ms * 1e-3) / 1e9, ms / 5);
        return 0;
    };
    printf("device %s CUs=%d, Q = %llu\n", prop.gcnArchName, prop.multiProcessorCount, (unsigned long long)Q);
    run("int Shoup product (shoup3, [0,3Q))", [&] { hipLaunchKernelGGL(k_intmm, dim3(blocks), dim3(threads), 0, 0, d, w, wp); });
    run("fp64 exact product (6 ops, |r|<=2Q)", [&] { hipLaunchKernelGGL(k_fpmm, dim3(blocks), dim3(threads), 0, 0, d, wd); });
    run("int lazy CT butterfly (mkacc_wide.hpp)", [&] { hipLaunchKernelGGL(k_int, dim3(blocks), dim3(threads), 0, 0, d, w, wp); });
    run("fp64 CT butterfly, a reduced every stage", [&] { hipLaunchKernelGGL(k_fp1, dim3(blocks), dim3(threads), 0, 0, d, wd); });
    run("fp64 CT butterfly, a reduced every 2nd stage", [&] { hipLaunchKernelGGL(k_fp2, dim3(blocks), dim3(threads), 0, 0, d, wd); });
    CHK(hipFree(d));
    return 0;
}
