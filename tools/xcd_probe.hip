// Records which XCD (HW_REG_XCC_ID) and CU each block of a 1-block-per-CU grid
// lands on, to check the round-robin placement the scan's block mapping uses.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ __launch_bounds__(256, 1) void probe(int* out, long long spin) {
    extern __shared__ char lds[];
    if (threadIdx.x == 0) {
        unsigned xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        long long t0 = clock64();
        while (clock64() - t0 < spin) {}
        out[blockIdx.x * 3 + 0] = xcc & 0xf;
        out[blockIdx.x * 3 + 1] = hw;
        out[blockIdx.x * 3 + 2] = (int)(wall_clock64() & 0x7fffffff);
    }
    lds[threadIdx.x] = 0;
}
int main(int argc, char** argv) {
    int grid = argc > 1 ? atoi(argv[1]) : 1280;
    int* d; hipMalloc(&d, grid * 12);
    hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 150000);
    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 150000, 0, d, 2000000LL);
    int* h = (int*)malloc(grid * 12);
    hipMemcpy(h, d, grid * 12, hipMemcpyDeviceToHost);
    int mism = 0;
    for (int b = 0; b < grid; ++b) if (h[b * 3] != h[(b % 8) * 3]) ++mism;
    printf("grid %d: blocks whose XCC differs from block (b%%8): %d\n", grid, mism);
    for (int b = 0; b < 40; ++b) printf("%d:%d ", b, h[b * 3]);
    printf("\n");
    for (int b = 256; b < 280; ++b) printf("%d:%d ", b, h[b * 3]);
    printf("\n");
    return 0;
}
