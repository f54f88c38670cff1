// ubench_dp_ilp.hip -- how much independent work one wave per SIMD needs to keep
// the FP64 pipe busy (config 5's register-resident kernel runs one wave per SIMD).
// Each lane runs R rounds of ILP independent exact modular products
// (mkacc_widefp.hpp mm: h = a b, l = fma(a, b, -h), q = rint(h / Q),
// fma(-q, Q, h) + l) chained through their outputs; 256 CUs x WPS waves per SIMD.
// Reported: ns per wave-level mm instruction group and the implied fraction of the
// 4-cycle-per-instruction FP64 issue rate.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_dp_ilp tools/ubench_dp_ilp.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int R = 4096;
constexpr double Qd = 1125899906826241.0;

__device__ __forceinline__ double mm(double a, double b, double Q, double Qi) {
    const double h = __dmul_rn(a, b);
    const double l = __fma_rn(a, b, -h);
    const double q = rint(__dmul_rn(h, Qi));
    return __dadd_rn(__fma_rn(-q, Q, h), l);
}

template <int ILP>
__global__ __launch_bounds__(256, 1) void chain(double* out, double w, double Q, double Qi) {
    double x[ILP];
#pragma unroll
    for (int j = 0; j < ILP; ++j) x[j] = (double)(threadIdx.x * 131 + j * 7919 + blockIdx.x);
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int j = 0; j < ILP; ++j) x[j] = mm(x[j], w, Q, Qi);
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < ILP; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ILP>
int run(double* d, int blocks, int threads) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const double w = 123456789012345.0, Qi = 1.0 / Qd;
    hipLaunchKernelGGL(chain<ILP>, dim3(blocks), dim3(threads), 0, 0, d, w, Qd, Qi);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    const int reps = 5;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(chain<ILP>, dim3(blocks), dim3(threads), 0, 0, d, w, Qd, Qi);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double t = ms * 1e-3 / reps;
    const double waves = (double)blocks * threads / 64;
    const double instr = waves * R * ILP * 6.0;            // 6 FP64 instructions per mm
    const double simds = 256.0 * 4;
    const double cyc = t * 2.4e9;                          // cycles at 2.4 GHz
    const double busy = instr / simds * 4.0 / cyc;          // 4 cycles per wave64 FP64 instruction
    printf("ILP %2d waves/SIMD %.0f : %.3f ms, %.2f T mm/s, FP64 issue fraction %.3f\n", ILP, waves / simds, t * 1e3,
           waves * 64 * R * ILP / t * 1e-12, busy);
    return 0;
}

int main() {
    double* d;
    CHK(hipMalloc(&d, 256 * 1024 * sizeof(double) * 2));
    for (int wps : {1, 2}) {
        const int blocks = 256 * wps;   // 256 threads = 4 waves: one per SIMD per block
        if (run<1>(d, blocks, 256) || run<2>(d, blocks, 256) || run<3>(d, blocks, 256) || run<4>(d, blocks, 256) ||
            run<6>(d, blocks, 256) || run<8>(d, blocks, 256) || run<16>(d, blocks, 256))
            return 1;
    }
    CHK(hipFree(d));
    return 0;
}
