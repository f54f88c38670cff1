// Microbenchmark: issue cost (SIMD cycles per wave64 instruction) of single
// gfx950 VALU opcodes, measured with inline asm on 8 independent register
// chains so the loop is throughput-bound.  Run at 2 and 8 waves/SIMD (the
// step kernel runs at 2).  Used to price the mod-mul formulations in
// DESIGN.md "Modular arithmetic".
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int R = 2048;

#define REP8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

#define K32(NAME, ASM)                                                                  \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                  \
        uint32_t a0 = threadIdx.x + s, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;          \
        uint32_t a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                   \
        const uint32_t b = s * 0x9E3779B9u + 77u;                                      \
        for (int r = 0; r < R; ++r) {                                                  \
            _Pragma("unroll") for (int u = 0; u < 4; ++u) {                            \
                asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a1) : "v"(b)); \
                asm volatile(ASM : "+v"(a2) : "v"(b)); asm volatile(ASM : "+v"(a3) : "v"(b)); \
                asm volatile(ASM : "+v"(a4) : "v"(b)); asm volatile(ASM : "+v"(a5) : "v"(b)); \
                asm volatile(ASM : "+v"(a6) : "v"(b)); asm volatile(ASM : "+v"(a7) : "v"(b)); \
            }                                                                          \
        }                                                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    }

K32(k_add, "v_add_u32 %0, %0, %1")
K32(k_add3, "v_add3_u32 %0, %0, %1, %0")
K32(k_min, "v_min_u32 %0, %0, %1")
K32(k_lshladd, "v_lshl_add_u32 %0, %0, 3, %1")
K32(k_bfe, "v_bfe_u32 %0, %0, %1, 5")
K32(k_mullo, "v_mul_lo_u32 %0, %0, %1")
K32(k_mulhi, "v_mul_hi_u32 %0, %0, %1")
K32(k_mul24, "v_mul_u32_u24 %0, %0, %1")
K32(k_mulhi24, "v_mul_hi_u32_u24 %0, %0, %1")
K32(k_mad24, "v_mad_u32_u24 %0, %0, %1, %0")

// 64-bit destination ops: a 64-bit chain register, 32-bit sources
#define K64(NAME, ASM)                                                                  \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                  \
        uint64_t a0 = threadIdx.x + s, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;          \
        uint64_t a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                   \
        const uint32_t b = s * 0x9E3779B9u + 77u, c = b ^ 0x55u;                       \
        for (int r = 0; r < R; ++r) {                                                  \
            _Pragma("unroll") for (int u = 0; u < 4; ++u) {                            \
                asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c) : "s40", "s41"); asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c) : "s40", "s41"); \
                asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c) : "s40", "s41"); asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c) : "s40", "s41"); \
                asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c) : "s40", "s41"); asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c) : "s40", "s41"); \
                asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c) : "s40", "s41"); asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c) : "s40", "s41"); \
            }                                                                          \
        }                                                                              \
        uint64_t x = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)x ^ (uint32_t)(x >> 32);  \
    }

K64(k_mad64, "v_mad_u64_u32 %0, s[40:41], %1, %2, %0")
K64(k_lshladd64, "v_lshl_add_u64 %0, %0, 3, %0")
K64(k_add64, "v_lshl_add_u64 %0, %0, 0, %0")

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const double clk = prop.clockRate * 1e3;
    printf("device %s CUs=%d clock=%.0f MHz\n", prop.gcnArchName, prop.multiProcessorCount, clk / 1e6);
    uint32_t* d;
    CHK(hipMalloc(&d, (size_t)prop.multiProcessorCount * 32 * 256 * 4));
    struct {
        const char* name;
        kfn f;
    } ks[] = {{"v_add_u32", k_add},          {"v_add3_u32", k_add3},       {"v_min_u32", k_min},
              {"v_lshl_add_u32", k_lshladd}, {"v_bfe_u32", k_bfe},         {"v_mul_lo_u32", k_mullo},
              {"v_mul_hi_u32", k_mulhi},     {"v_mul_u32_u24", k_mul24},   {"v_mul_hi_u32_u24", k_mulhi24},
              {"v_mad_u32_u24", k_mad24},    {"v_mad_u64_u32", k_mad64},   {"v_lshl_add_u64", k_lshladd64},
              {"v_lshl_add_u64 (s=0)", k_add64}};
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int wps : {2, 8}) {
        // wps waves per SIMD: 4 SIMDs per CU, 256 threads = 4 waves per block
        const int blocks = prop.multiProcessorCount * wps, threads = 256;
        printf("-- %d waves/SIMD --\n", wps);
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0));
            for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)it);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const double instr_per_simd = 5.0 * wps * (double)R * 32;   // wave instructions per SIMD
            const double cyc = ms * 1e-3 * clk / instr_per_simd;
            printf("%-24s %6.2f cycles/wave-instr\n", k.name, cyc);
        }
    }
    CHK(hipFree(d));
    return 0;
}
