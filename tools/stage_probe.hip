// stage_probe.hip -- microbenchmark of one scan pipeline stage on gfx950.
//
// Question: what does a stage of the fused scan cost when every wave issues
// its own corpus LDS-DMA pieces beside its MFMAs, at one wave per SIMD (the
// k_scan_q3 shape: 32 MFMA + 4 DMA + 16 ds_read_b128 per wave per stage) vs
// two waves per SIMD (16 MFMA + 2 DMA + 8 ds_read_b128 per wave)?  Each
// workgroup streams its own 16 MiB window of a 4 GiB buffer through a 5-slot
// LDS ring; one counted vmcnt + s_barrier per stage, as in the scan kernel.
// Prints shader cycles per stage (s_memtime) and the in-kernel clock.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/stage_probe tools/stage_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;

constexpr int NSLOT = 5;
constexpr int STAGE = 16384;
constexpr size_t BUF = 4ull << 30;
static size_t WIN_H = 16ull << 20;  // per-block streamed window (host-set)
__constant__ size_t WIN;
__constant__ int NWIN;  // stages per window
constexpr int ROWB = 1536;

__device__ __forceinline__ uint32_t lds_off(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int NW, int NMFMA, int NDMA, int NRD, int CONTIG, int NODMA>
__global__ __launch_bounds__(NW * 64, 1) void probe(const char* buf, int nstage, unsigned long long* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t lbase = lds_off(smem);
    const char* win = buf + ((size_t)blockIdx.x * WIN) % BUF;
    bf16x8 b0, b1;
    for (int i = 0; i < 8; ++i) {
        b0[i] = (__bf16)(0.01f * (lane + i));
        b1[i] = (__bf16)(0.02f * (lane - i));
    }
    asm volatile("" ::"a"(b0), "a"(b1));
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[2][8];
    for (int s = 0; s < 2; ++s)
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 8; ++j) a[s][i][j] = (__bf16)(0.001f * (lane * 3 + i + j + s));

    // per-lane offsets of this wave's pieces inside a stage (fragment-ordered
    // image as in fx_scan.hip), scalar stage base: no vector address math
    uint32_t voff[4];
    for (int p = 0; p < 4; ++p) {
        const int piece = wave * NDMA + p;
        voff[p] = CONTIG ? (uint32_t)(piece * 1024 + lane * 16)
                         : (uint32_t)((((piece >> 1) & 7) * 16 + (lane & 15)) * ROWB + (piece & 1) * 64 +
                                      (lane >> 4) * 16);
    }
    auto dma = [&](int g, int p) {
        if (NODMA) return;
        const int piece = wave * NDMA + p;  // 0..15 per stage per CU
        const uint64_t b = (uint64_t)(win + (size_t)(g % NWIN) * (CONTIG ? STAGE : 128 * ROWB));
        // readfirstlane returns int: go through uint32_t (no sign extension)
        const uint32_t bhi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
        const uint32_t blo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
        const char* sb = (const char*)(((uint64_t)bhi << 32) | blo);
        const uint32_t m0 = lbase + 4096 + (g % NSLOT) * STAGE + piece * 1024;
        asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff[p]), "s"(sb),
                     "{m0}"(__builtin_amdgcn_readfirstlane(m0))
                     : "memory");
    };
    auto rd = [&](int g, bf16x8(&d)[8], int half) {
        const uint32_t base = lbase + 4096 + (g % NSLOT) * STAGE + lane * 16 + half * 1024;
        asm volatile(
            "ds_read_b128 %0, %8\n\t"
            "ds_read_b128 %1, %8 offset:2048\n\t"
            "ds_read_b128 %2, %8 offset:4096\n\t"
            "ds_read_b128 %3, %8 offset:6144\n\t"
            "ds_read_b128 %4, %8 offset:8192\n\t"
            "ds_read_b128 %5, %8 offset:10240\n\t"
            "ds_read_b128 %6, %8 offset:12288\n\t"
            "ds_read_b128 %7, %8 offset:14336"
            : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7])
            : "v"(base)
            : "memory");
    };
    auto mm = [&](int i, const bf16x8& x) {
        if (i & 1)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i & 15]) : "v"(x), "a"(b1));
        else
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i & 15]) : "v"(x), "a"(b0));
    };
    for (int st = 0; st < NSLOT - 1; ++st)
        for (int p = 0; p < NDMA; ++p) dma(st, p);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int g = 0; g < nstage; g += 2) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            bf16x8(&X)[8] = a[u];
            bf16x8(&Y)[8] = a[u ^ 1];
            if (NODMA)
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            else if (NDMA == 4)
                asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            else if (NDMA == 2)
                asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            // next stage's operands: NRD reads (8 or 16)
            rd(g + u + 1, Y, 0);
            constexpr int per = NMFMA / (NDMA + 1);
            int p = 0;
#pragma unroll
            for (int i = 0; i < NMFMA; ++i) {
                mm(i, X[i & 7]);
                if ((i + 1) % per == 0 && p < NDMA) {
                    __builtin_amdgcn_sched_barrier(0);
                    dma(g + u + NSLOT - 1, p++);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (NRD == 16 && i == NMFMA / 2) {
                    __builtin_amdgcn_sched_barrier(0);
                    rd(g + u + 1, Y, 1);  // (reuses Y: timing only)
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (lane == 0) {
        out[(blockIdx.x * NW + wave) * 3 + 0] = t1 - t0;
        out[(blockIdx.x * NW + wave) * 3 + 1] = r1 - r0;
        out[(blockIdx.x * NW + wave) * 3 + 2] = (unsigned long long)(s != 12345.f);
    }
}

template <int NW, int NMFMA, int NDMA, int NRD, int CONTIG, int NODMA>
void run(const char* name, const char* buf, int nstage) {
    unsigned long long* d;
    const int grid = 256;
    hipMalloc(&d, (size_t)grid * NW * 24);
    auto k = probe<NW, NMFMA, NDMA, NRD, CONTIG, NODMA>;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 150000);
    std::vector<unsigned long long> h((size_t)grid * NW * 3);
    double best = 1e30, clk = 0;
    for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), 150000, 0, buf, nstage, d);
        hipError_t e0 = hipGetLastError(), e1 = hipDeviceSynchronize();
        if (e0 != hipSuccess || e1 != hipSuccess) {
            printf("%s: launch %s / sync %s\n", name, hipGetErrorString(e0), hipGetErrorString(e1));
            exit(1);
        }
        hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
        std::vector<double> cyc, ghz;
        for (int i = 0; i < grid * NW; ++i) {
            cyc.push_back((double)h[i * 3] / nstage);
            ghz.push_back((double)h[i * 3] / ((double)h[i * 3 + 1] / 100e6) / 1e9);
        }
        std::sort(cyc.begin(), cyc.end());
        std::sort(ghz.begin(), ghz.end());
        if (rep > 0 && cyc[cyc.size() / 2] < best) {
            best = cyc[cyc.size() / 2];
            clk = ghz[ghz.size() / 2];
        }
    }
    const double mf_per_simd = (double)NMFMA * NW / 4;  // per stage
    printf("%-44s %8.1f cyc/stage  (ideal %5.0f, MFMA util %.2f) clk %.2f GHz\n", name, best, mf_per_simd * 16,
           mf_per_simd * 16 / best, clk);
    hipFree(d);
}

int main(int argc, char** argv) {
    int nstage = argc > 1 ? atoi(argv[1]) : 4000;
    WIN_H = (argc > 2 ? (size_t)atoll(argv[2]) : 16) << 10;  // KiB
    hipMemcpyToSymbol(HIP_SYMBOL(WIN), &WIN_H, sizeof(WIN_H));
    const int nwin = (int)std::max<size_t>(1, WIN_H / (128 * ROWB));
    hipMemcpyToSymbol(HIP_SYMBOL(NWIN), &nwin, sizeof(nwin));
    printf("window per block: %zu KiB\n", WIN_H >> 10);
    char* buf;
    hipMalloc(&buf, BUF);
    hipMemset(buf, 0x3c, BUF);
    run<4, 32, 4, 16, 0, 1>("1 wave/SIMD, 32 MFMA, no DMA, 16 rd", buf, nstage);
    run<4, 32, 4, 16, 0, 0>("1 wave/SIMD, 32 MFMA, 4 DMA strided, 16 rd", buf, nstage);
    run<4, 32, 4, 16, 1, 0>("1 wave/SIMD, 32 MFMA, 4 DMA contig, 16 rd", buf, nstage);
    run<8, 16, 2, 8, 0, 1>("2 waves/SIMD, 16 MFMA, no DMA, 8 rd", buf, nstage);
    run<8, 16, 2, 8, 0, 0>("2 waves/SIMD, 16 MFMA, 2 DMA strided, 8 rd", buf, nstage);
    run<8, 16, 2, 8, 1, 0>("2 waves/SIMD, 16 MFMA, 2 DMA contig, 8 rd", buf, nstage);
    run<4, 64, 4, 16, 0, 0>("1 wave/SIMD, 64 MFMA, 4 DMA strided, 16 rd", buf, nstage);
    run<8, 32, 2, 8, 0, 0>("2 waves/SIMD, 32 MFMA, 2 DMA strided, 8 rd", buf, nstage);
    hipFree(buf);
    return 0;
}
