// ldscheck.hip -- does a 512-thread workgroup with >64 KiB of DYNAMIC LDS see
// all of it?  Each thread fills a strided slice with a (block, word) pattern,
// barrier, then every thread reads the slice written by a thread of the
// opposite half of the block and counts mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(512) void fill_check(unsigned* bad, unsigned words, unsigned salt) {
    extern __shared__ unsigned lds[];
    const unsigned t = threadIdx.x, nt = blockDim.x;
    for (unsigned w = t; w < words; w += nt) lds[w] = (blockIdx.x * 2654435761u) ^ (w * 40503u) ^ salt;
    __syncthreads();
    const unsigned src = (t + nt / 2) % nt;  // a thread of the other half
    unsigned nbad = 0;
    for (unsigned w = src; w < words; w += nt)
        nbad += lds[w] != ((blockIdx.x * 2654435761u) ^ (w * 40503u) ^ salt);
    if (nbad) atomicAdd(&bad[t >> 6], nbad);
}

int main() {
    unsigned* d;
    CHK(hipMalloc(&d, 64 * 4));
    for (unsigned kb : {48u, 64u, 96u, 128u, 132u, 160u}) {
        const unsigned bytes = kb * 1024u - (kb == 160 ? 0 : 0);
        CHK(hipMemset(d, 0, 64 * 4));
        hipLaunchKernelGGL(fill_check, dim3(1024), dim3(512), bytes, 0, d, bytes / 4, kb);
        hipError_t e = hipGetLastError();
        CHK(hipDeviceSynchronize());
        unsigned h[8];
        CHK(hipMemcpy(h, d, 32, hipMemcpyDeviceToHost));
        printf("dyn LDS %3u KiB launch=%s bad per wave:", kb, hipGetErrorString(e));
        for (int i = 0; i < 8; ++i) printf(" %u", h[i]);
        printf("\n");
    }
    int v = 0;
    CHK(hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, 0));
    printf("hipDeviceAttributeMaxSharedMemoryPerBlock = %d\n", v);
    return 0;
}
