// fx_scan5.hip -- 8-wave K-split variant of the fused scan (k_scan_v5).
//
// Why: in k_scan_v4 (one wave per SIMD, 438 registers) every LDS-DMA piece
// stalls the only wave that could issue the SIMD's next MFMA; the ablation
// builds put that at ~30 % of the scan.  Here each SIMD holds
// TWO waves of <= 256 registers, so one wave's DMA issue (and epilogue) runs
// beside its partner's MFMAs.  Registers are halved by splitting K: the two
// waves of a pair hold the same 32 queries, each for half of the row bytes
// (96 AGPRs at d = 768 bf16), and their partial keys are exchanged through
// LDS once per 64-row tile.
//
//   workgroup 512 threads = 8 waves; wave w: pair p = w & 3 (queries
//     32p .. 32p+31 of the 128-query tile), half h = w >> 2 (row bytes
//     [h RB/2, (h+1) RB/2)); one workgroup per CU (LDS);
//   tile = 64 corpus rows; stage = 64 rows x (128 B of each half) = 16 KiB in
//     a 5-slot LDS ring; per wave per stage: 2 corpus LDS-DMA pieces, 8
//     ds_read_b128, 16 MFMAs (4 row blocks x 2 query columns x 2 K-steps);
//   once per tile each wave also moves an aux piece (h = 1: 16 row norms of
//     its row block; h = 0: its pair's 32 shared thresholds);
//   epilogue: wave (p, h) finalises queries 32p + 16h .. +15 (its column 0):
//     its own partial + the partner's (2 LDS rounds of 16 KiB) + |y|^2 (L2), then the
//     group-ballot push of k_scan_v4 into its own 16 LDS lists.
//   STAG = 1 (FX_SCAN_V5=2): one 32 KiB exchange round at tile end; waves 0-3
//     finish the tile before the next tile's first MFMAs, waves 4-7 after
//     them, so each SIMD runs one wave's epilogue beside its partner's MFMAs.
//   DT = F32S (split fp32): half h takes quarter h of each [hi | lo] plane.
//
// Not yet measured on hardware: selected only with FX_SCAN_V5=1 / 2 (the
// product path is k_scan_v4).
#include "fx_scan_common.h"

#include <stdlib.h>

namespace fx {

constexpr int V5_THREADS = 512;
constexpr int V5_TR = 64;                          // corpus rows per tile
constexpr int V5_NS = 5;                           // ring slots
constexpr int V5_STAGE = V5_TR * 256;              // 16 KiB: 64 rows x (2 halves x 128 B)
// LDS carve.  STAG = 1 (staggered epilogue) exchanges all four partner blocks
// in one round (32 KiB) and keeps 40-entry lists to stay within 160 KiB.
template <int STAG>
struct V5Lds {
    static constexpr int CAPV = STAG ? 40 : 48;            // LDS list capacity per query (> KP)
    static constexpr int AUX_B = 256 + TILE_Q * 4;         // per tile: 64 norms + 128 thresholds
    static constexpr int AUX_OFF = 0;                      // 4 tile slots of aux data
    static constexpr int RING_OFF = 4096;                  // >= any DMA instruction offset (dma_piece)
    static constexpr int XCH_OFF = RING_OFF + V5_NS * V5_STAGE;
    static constexpr int XCH_B = STAG ? 32768 : 16384;     // exchange: 8 waves x 4 (2) KiB
    static constexpr int LD_OFF = XCH_OFF + XCH_B;
    static constexpr int LI_OFF = LD_OFF + TILE_Q * CAPV * 4;
    static constexpr int CNT_OFF = LI_OFF + TILE_Q * CAPV * 4;
    static constexpr int TAU_OFF = CNT_OFF + TILE_Q * 4;
    static constexpr int BYTES = TAU_OFF + TILE_Q * 4;
    static_assert(4 * AUX_B <= RING_OFF, "aux slots");
    static_assert(BYTES <= 160 * 1024, "LDS budget");
};

// Compact the wave's full lists (16 queries from q_first) to their KP best.
template <int CAPV>
__device__ __noinline__ void compact16(float* lst_d, int* lst_i, int* cnt, float* tau, unsigned* gt_first,
                                       int q_first, int lane) {
    for (int qi = 0; qi < 16; ++qi) {
        const int q = q_first + qi;
        if (cnt[q] >= CAPV) {
            float d = lane < CAPV ? lst_d[q * CAPV + lane] : FX_INF;
            int i = lane < CAPV ? lst_i[q * CAPV + lane] : INT_MAX;
            sort64(d, i, lane);
            if (lane < KP) {
                lst_d[q * CAPV + lane] = d;
                lst_i[q * CAPV + lane] = i;
            }
            if (lane == KP - 1) {
                tau[q] = d;
                atomicMin(gt_first + qi, f2ord(d));
            }
            if (lane == 0) cnt[q] = KP;
        }
    }
}

// push the eligible entries of key group m (4 rows of this lane) into query
// q's list (capacity CAPV); list-full entries -> pend bit 4m+i
template <int CAPV>
__device__ __forceinline__ bool push4(const f32x4& key, int m, unsigned elig, float tn, int q, int row0, int rlim,
                                      float* lst_d, int* lst_i, int* cnt, unsigned& pend) {
    bool ovf = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float v = key[i];
        const int rl = row0 + i;
        if (((elig >> i) & 1u) && v <= tn && rl < rlim) {
            const int s = atomicAdd(&cnt[q], 1);
            if (s < CAPV) {
                lst_d[q * CAPV + s] = v;
                lst_i[q * CAPV + s] = rl;
            } else {
                pend |= 1u << (m * 4 + i);
                ovf = true;
            }
        }
    }
    return ovf;
}

// 48 wait states between the last (asm) MFMA and the epilogue's VALU reads
__device__ __forceinline__ void acc_fence4(f32x4 (&acc)[4][2]) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[1][0]), "+v"(acc[1][1]), "+v"(acc[2][0]),
                   "+v"(acc[2][1]), "+v"(acc[3][0]), "+v"(acc[3][1]));
}

// pinned LDS write of one accumulator block (the exchange)
template <int OFF>
__device__ __forceinline__ void ds_wr128(uint32_t addr, const f32x4& v) {
    asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(OFF) : "memory");
}

template <int DT, int METRIC, int KSTEPS, int STAG>
__global__ __launch_bounds__(V5_THREADS, 1) void k_scan_v5(ScanParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename AsmMmaV<DT>::A frag_t;
    typedef typename AsmMmaV<DT>::B bfrag_t;
    static_assert(KSTEPS % 4 == 0, "each half must hold a whole number of 128-B stages");
    // F32S (split fp32, rows [hi plane | lo plane]): wave half h takes quarter h
    // of EACH plane, so both halves run hi*x_hi + hi*x_lo + lo*x_hi on equal work
    constexpr bool SPL = DT == F32S;
    static_assert(!SPL || KSTEPS % 8 == 0, "F32S: a plane quarter must be whole 128-B stages");
    constexpr int RB = KSTEPS * 64;       // row stride (bytes)
    constexpr int HB = RB / 2;            // bytes of one K half
    constexpr int QB = RB / 4;            // F32S: bytes of one plane quarter
    constexpr int KH = KSTEPS / 2;        // 64-B K-steps per half
    constexpr int SPT = KSTEPS / 4;       // stages per tile (128 B of each half per stage)
    constexpr int NS = V5_NS;
    constexpr int M = V5_TR / 16;         // 4 row blocks
    constexpr int N = 2;                  // query columns of 16
    constexpr int64_t TB = (int64_t)V5_TR * RB;
    typedef V5Lds<STAG> L;
    constexpr int CAPV = L::CAPV;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int pr = wave & 3, h = wave >> 2;
    int qtile, split;
    map_block(blockIdx.x, p, qtile, split);
    if (qtile >= p.n_qtiles) return;
    const int n64 = (int)((p.ntotal + V5_TR - 1) / V5_TR);
    // asserted uniform: the 64-bit divisions run on the VALU, and a base pointer
    // derived from them must stay in SGPRs for the LDS-DMA (dma_piece's "s")
    const int ct0 = __builtin_amdgcn_readfirstlane((int)((int64_t)split * n64 / p.splits));
    const int ct1 = __builtin_amdgcn_readfirstlane((int)((int64_t)(split + 1) * n64 / p.splits));
    const int ntiles = ct1 - ct0;
    const int64_t q0 = (int64_t)qtile * TILE_Q;

    float* lst_d = (float*)(smem + L::LD_OFF);
    int* lst_i = (int*)(smem + L::LI_OFF);
    int* cnt = (int*)(smem + L::CNT_OFF);
    float* tau = (float*)(smem + L::TAU_OFF);
    const int qf = pr * 32 + h * 16;      // first of the 16 queries this wave finalises
    if (lane < 16) {
        cnt[qf + lane] = 0;
        tau[qf + lane] = KEY_MAX;
    }

    // the pair's 32 queries, this wave's K half -> AGPRs
    bfrag_t b[KH][N];
    {
        // column n holds queries pr*32 + (n ^ h)*16 ..: column 0 is always the
        // 16 queries this wave finalises, column 1 its partner's (no dynamic
        // register indexing in the epilogue)
        // (F32S: K-steps 0 .. KH/2-1 = quarter h of x_hi, KH/2 .. KH-1 = quarter h of x_lo)
        const char* qb = p.qop + (q0 + pr * 32 + (lane & 15)) * RB + (lane >> 4) * 16;
#pragma unroll
        for (int ks = 0; ks < KH; ++ks) {
            const int kofs = !SPL ? h * HB + ks * 64
                                  : (ks < KH / 2 ? h * QB + ks * 64 : HB + h * QB + (ks - KH / 2) * 64);
#pragma unroll
            for (int n = 0; n < N; ++n) b[ks][n] = *(const bfrag_t*)(qb + (n ^ h) * 16 * RB + kofs);
        }
#pragma unroll
        for (int ks = 0; ks < KH; ++ks)
#pragma unroll
            for (int n = 0; n < N; ++n) AsmMmaV<DT>::settle(b[ks][n]);
    }

    // ---- DMA: wave w moves LDS blocks (m = pr, h, kb = 0/1) of every stage:
    //      rows 16 pr .. 16 pr + 15, bytes h HB + 128 j + 64 kb of its half
    const uint32_t lds_base = lds_off(smem);
    const uint32_t voff = (uint32_t)((pr * 16 + (lane & 15)) * RB + h * (SPL ? QB : HB) + (lane >> 4) * 16);
    const uint32_t blk_w = (uint32_t)(((pr * 2 + h) * 2) * 1024);   // block (m = pr, h, kb = 0)
    const char* cb0 = p.codes + (int64_t)ct0 * TB;
    const char* cb_last = sgpr_ptr(p.codes + (int64_t)(ct0 + (ntiles > 0 ? ntiles - 1 : 0)) * TB);
    // aux piece of tile u: h = 1 -> 16 norms of rows 16 pr.. (64 B, lanes 0-3);
    //                      h = 0 -> the pair's 32 thresholds (128 B, lanes 0-7)
    const unsigned* gtp = p.gtau + q0 + pr * 32;
    const uint64_t aux_exec = h ? 0xFull : 0xFFull;
    const uint32_t aux_dst = h ? (uint32_t)(pr * 64) : (uint32_t)(256 + pr * 128);

    auto tile_base = [&](int u) {  // scalar base of tile u (clamped: look-ahead past the end)
        return u < ntiles ? sgpr_ptr(cb0 + (int64_t)u * TB) : cb_last;
    };
    auto aux_piece = [&](int u) {
        const int uc = u < ntiles ? u : (ntiles > 0 ? ntiles - 1 : 0);
        const char* src = h ? (const char*)(p.norms + (int64_t)(ct0 + uc) * V5_TR + pr * 16 + (lane & 3) * 4)
                            : (const char*)(gtp + (lane & 7) * 4);
        const uint32_t m0 = lds_base + L::AUX_OFF + (uint32_t)(u & 3) * L::AUX_B + aux_dst;
        uint64_t saved;
        asm volatile(
            "s_mov_b64 %0, exec\n\t"
            "s_mov_b64 exec, %3\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\t"
            "s_mov_b64 exec, %0"
            : "=&s"(saved)
            : "v"(src), "{m0}"(m0), "s"(aux_exec)
            : "memory");
    };
    // corpus piece kb (0/1) of stage jp of tile base cb into ring slot `slot`
    auto corpus_piece = [&](auto KB, auto JP, const char* cb, uint32_t slot) {
        constexpr int kb = decltype(KB)::value, jp = decltype(JP)::value;
        // NOP 4: hipcc may compute the tile base with v_readfirstlane right here
        // F32S: stages 0 .. SPT/2-1 walk the hi plane's quarter, the rest the lo plane's
        constexpr int sofs = !SPL ? jp * 128 : (jp < SPT / 2 ? jp * 128 : HB + (jp - SPT / 2) * 128);
        dma_piece<sofs + kb * 64, 4>(voff, cb, lds_base + L::RING_OFF + slot * V5_STAGE + blk_w + kb * 1024);
    };

    // prologue: stages 0 .. NS-2 (tiles 0 .. (NS-2)/SPT)
    static_for<NS - 1>([&](auto ST) {
        constexpr int st = decltype(ST)::value;
        constexpr int u = st / SPT, jp = st % SPT;
        const char* cb = tile_base(u);
        corpus_piece(std::integral_constant<int, 0>{}, std::integral_constant<int, jp>{}, cb, (uint32_t)st);
        corpus_piece(std::integral_constant<int, 1>{}, std::integral_constant<int, jp>{}, cb, (uint32_t)st);
        if constexpr (jp == 0) aux_piece(u);
    });
    // VMEM ops of the prologue after stage 0's
    constexpr int PRO_AFTER0 = 2 * (NS - 2) + (1 < NS - 1 && 1 % SPT == 0) + (2 < NS - 1 && 2 % SPT == 0) +
                               (3 < NS - 1 && 3 % SPT == 0);

    f32x4 acc[M][N];
    frag_t X[M], Y[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        acc[m][0] = acc[m][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        X[m] = Y[m] = frag_t{};
    }
    const int rl0 = 4 * (lane >> 4);
    const int ql = qf + (lane & 15);                   // the query this lane finalises
    const bool qv = q0 + ql < p.nq;
    const uint32_t tau_addr = lds_off(tau + ql);
    const uint32_t gt_lane = (uint32_t)(256 + pr * 128 + h * 64 + (lane & 15) * 4);
    // exchange: wave (pr, h) writes its column 1 (the partner's queries) into the
    // partner's region and reads its own region
    // (STAG: one round, 4 KiB per destination wave; else two rounds of 2 KiB)
    constexpr uint32_t XREG = STAG ? 4096 : 2048;
    const uint32_t xw = lds_base + L::XCH_OFF + (uint32_t)((pr * 2 + (1 - h)) * XREG + lane * 16);
    const uint32_t xr = lds_base + L::XCH_OFF + (uint32_t)((pr * 2 + h) * XREG + lane * 16);
    unsigned* gt_first = p.gtau + q0 + qf;

    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(PRO_AFTER0) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    // block (m, h, kb) of slot s at RING + s*STAGE + ((m*2 + h)*2 + kb)*1024
    const uint32_t rd_h = lds_base + L::RING_OFF + (uint32_t)(h * 2 * 1024 + lane * 16);
    uint32_t rd_addr = rd_h;  // slot 0
    if (ntiles > 0) {
        static_for<M>([&](auto MM) {
            constexpr int m = decltype(MM)::value;
            ds_rd128<m * 4096>(X[m], rd_addr);
        });
    }

    // STAG: this wave's own column of the previous tile (keyt) and its
    // thresholds wait across the next tile's first barrier; waves 0-3 finish
    // that tile before their first MFMAs of the next one, waves 4-7 after them,
    // so each SIMD overlaps one wave's epilogue with its partner's MFMAs
    // (MI355X_MICROARCH.md "two waves per SIMD", item 9)
    f32x4 keyt[M];
    float trp = 0.f;
    unsigned grp = 0u;
#pragma unroll
    for (int m = 0; m < M; ++m) keyt[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto finish = [&](int tt) {
        f32x4 key[M];
        {
            f32x4 o0, o1, o2, o3;  // the partner's partial sums of this wave's queries
            asm volatile(
                "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                : "=&v"(o0), "=&v"(o1), "=&v"(o2), "=&v"(o3)
                : "v"(xr)
                : "memory");
            key[0] = keyt[0] + o0;
            key[1] = keyt[1] + o1;
            key[2] = keyt[2] + o2;
            key[3] = keyt[3] + o3;
        }
        if (METRIC == L2) {
            const uint32_t na = lds_base + L::AUX_OFF + (uint32_t)(tt & 3) * L::AUX_B + (uint32_t)(rl0 * 4);
#pragma unroll
            for (int m = 0; m < M; ++m) {
                f32x4 y;
                asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(y)
                             : "v"(na), "i"(m * 64)
                             : "memory");
                key[m] += y;
            }
        }
        if (p.dbgbuf) {
            float* keys = (float*)p.dbgbuf;
            const int64_t ld = (int64_t)p.n_ctiles * TILE_R;
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    keys[(q0 + ql) * ld + (int64_t)(ct0 + tt) * V5_TR + rl0 + 16 * m + i] = key[m][i];
        }
        const float tn = qv ? fminf(trp, ord2f(grp)) : -FX_INF;
        float gmin[M], mn;
#pragma unroll
        for (int m = 0; m < M; ++m) gmin[m] = fminf(fminf(key[m][0], key[m][1]), fminf(key[m][2], key[m][3]));
        mn = fminf(fminf(gmin[0], gmin[1]), fminf(gmin[2], gmin[3]));
        if (__builtin_amdgcn_ballot_w64(mn <= tn)) {
            const int trow0 = (ct0 + tt) * V5_TR;
            const int rlim = p.ntotal < (int64_t)trow0 + V5_TR ? (int)p.ntotal : trow0 + V5_TR;
            unsigned pend = 0u;
            bool ovf = false;
            static_for<M>([&](auto MM) {
                constexpr int m = decltype(MM)::value;
                if (__builtin_amdgcn_ballot_w64(gmin[m] <= tn))
                    ovf |= push4<CAPV>(key[m], m, 15u, tn, ql, trow0 + rl0 + m * 16, rlim, lst_d, lst_i, cnt, pend);
            });
            while (__builtin_amdgcn_ballot_w64(ovf)) {
                compact16<CAPV>(lst_d, lst_i, cnt, tau, gt_first, qf, lane);
                ovf = false;
                const float tq = qv ? fminf(tau[ql], tn) : -FX_INF;
                const unsigned pn = pend;
                pend = 0u;
                static_for<M>([&](auto MM) {
                    constexpr int m = decltype(MM)::value;
                    const unsigned el = (pn >> (4 * m)) & 15u;
                    if (__builtin_amdgcn_ballot_w64(el != 0u))
                        ovf |= push4<CAPV>(key[m], m, el, tq, ql, trow0 + rl0 + m * 16, rlim, lst_d, lst_i, cnt, pend);
                });
            }
        }
    };

    int c = 0;
    for (int t = 0; t < ntiles; ++t) {
        float tr = 0.f;
        unsigned gr = 0u;
        static_for<SPT>([&](auto JJ) {
            constexpr int j = decltype(JJ)::value;
            constexpr bool LAST = j == SPT - 1;
            constexpr int jq = j + NS - 1;               // stage issued now: tile t + jq / SPT, stage jq % SPT
            typedef std::integral_constant<int, jq % SPT> JP;
            const uint32_t c1 = c == NS - 1 ? 0u : (uint32_t)c + 1;
            const uint32_t c4 = c == 0 ? (uint32_t)NS - 1 : (uint32_t)c - 1;
            // VMEM ops younger than stage g+1's: those issued in stages g-2, g-1
            constexpr int W = 4 + ((j + NS - 3) % SPT == 0) + ((j + NS - 2) % SPT == 0);
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(W) : "memory");
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (STAG && j == 0) {
                if (t > 0 && h == 0) finish(t - 1);  // waves 0-3: previous tile first
                __builtin_amdgcn_sched_barrier(0);
            }
            // F32S: hi stages (j < SPT/2) take x_hi then x_lo, lo stages x_hi only
            constexpr bool HI = SPL && j < SPT / 2;
            constexpr int kq = (SPL && !HI) ? 2 * (j - SPT / 2) : 2 * j;  // B K-step of half kb = 0
            // ---- kb = 0: X MFMAs; read kb = 1 (Y) of this stage after >= 6 MFMAs
            static_for<M>([&](auto MM) {
                constexpr int m = decltype(MM)::value;
                constexpr int INIT = j == 0 ? 2 : 0;  // first K-step of the tile: srcC = 0
                AsmMmaV<DT>::template mma2<INIT>(acc[m][0], acc[m][1], X[m], b[kq][0], b[kq][1], acc[m][0]);
                if constexpr (m == 1) {
                    ds_rd128<0 * 4096 + 1024>(Y[0], rd_addr);
                    ds_rd128<1 * 4096 + 1024>(Y[1], rd_addr);
                }
                if constexpr (m == 2) {
                    ds_rd128<2 * 4096 + 1024>(Y[2], rd_addr);
                    ds_rd128<3 * 4096 + 1024>(Y[3], rd_addr);
                }
                if constexpr (m == 3)
                    corpus_piece(std::integral_constant<int, 0>{}, JP{}, tile_base(t + jq / SPT), c4);
            });
            if constexpr (HI) {
                static_for<M>([&](auto MM) {
                    constexpr int m = decltype(MM)::value;
                    AsmMmaV<DT>::template mma2<0>(acc[m][0], acc[m][1], X[m], b[KH / 2 + kq][0], b[KH / 2 + kq][1],
                                                  acc[m][0]);
                });
            }
            if constexpr (LAST) {
                ds_rd32<0>(tr, tau_addr);
                const uint32_t ns = lds_base + L::AUX_OFF + (uint32_t)(t & 3) * L::AUX_B + gt_lane;
                ds_rd32<0>(gr, ns);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            // ---- kb = 1: Y MFMAs; read kb = 0 (X) of stage g+1 after >= 6 MFMAs
            const uint32_t rd_next = rd_h + c1 * V5_STAGE;
            static_for<M>([&](auto MM) {
                constexpr int m = decltype(MM)::value;
                AsmMmaV<DT>::template mma2<0>(acc[m][0], acc[m][1], Y[m], b[kq + 1][0], b[kq + 1][1], acc[m][0]);
                if constexpr (m == 1) {
                    ds_rd128<0 * 4096>(X[0], rd_next);
                    ds_rd128<1 * 4096>(X[1], rd_next);
                }
                if constexpr (m == 2) {
                    ds_rd128<2 * 4096>(X[2], rd_next);
                    ds_rd128<3 * 4096>(X[3], rd_next);
                }
                if constexpr (m == 3) {
                    corpus_piece(std::integral_constant<int, 1>{}, JP{}, tile_base(t + jq / SPT), c4);
                    if constexpr (jq % SPT == 0) aux_piece(t + jq / SPT);
                }
            });
            if constexpr (HI) {
                static_for<M>([&](auto MM) {
                    constexpr int m = decltype(MM)::value;
                    AsmMmaV<DT>::template mma2<0>(acc[m][0], acc[m][1], Y[m], b[KH / 2 + kq + 1][0],
                                                  b[KH / 2 + kq + 1][1], acc[m][0]);
                });
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (STAG && j == 0) {
                if (t > 0 && h == 1) finish(t - 1);  // waves 4-7: after this stage's MFMAs
                __builtin_amdgcn_sched_barrier(0);
            }
            rd_addr = rd_next;
            c = (int)c1;
        });

        // ---- epilogue of tile t ----------------------------------------------
        acc_fence4(acc);
        if constexpr (STAG) {
            // hand the partner its column, keep ours; finished during the next tile
            ds_wr128<0>(xw, acc[0][1]);
            ds_wr128<1024>(xw, acc[1][1]);
            ds_wr128<2048>(xw, acc[2][1]);
            ds_wr128<3072>(xw, acc[3][1]);
#pragma unroll
            for (int m = 0; m < M; ++m) keyt[m] = acc[m][0];
            trp = tr;
            grp = gr;
            continue;
        }
        // exchange the partner column in two rounds (m = 0,1 then 2,3)
        static_for<2>([&](auto RR) {
            constexpr int r = decltype(RR)::value;
            ds_wr128<0>(xw, acc[2 * r][1]);
            ds_wr128<1024>(xw, acc[2 * r + 1][1]);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            f32x4 o0, o1;
            asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(o0), "=&v"(o1)
                         : "v"(xr)
                         : "memory");
            acc[2 * r][0] += o0;
            acc[2 * r + 1][0] += o1;
            if constexpr (r == 0) asm volatile("s_barrier" ::: "memory");  // round-1 writes after round-0 reads
        });
        f32x4 key[M];
#pragma unroll
        for (int m = 0; m < M; ++m) key[m] = acc[m][0];
        if (METRIC == L2) {
            // + |y|^2 of this lane's rows (16 m + rl0 .. +3) from the tile's aux slot
            const uint32_t na = lds_base + L::AUX_OFF + (uint32_t)(t & 3) * L::AUX_B + (uint32_t)(rl0 * 4);
#pragma unroll
            for (int m = 0; m < M; ++m) {
                f32x4 y;
                asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(y)
                             : "v"(na), "i"(m * 64)
                             : "memory");
                key[m] += y;
            }
        }
        if (p.dbgbuf) {  // diagnostics (FX_SCAN_DBG & 32): every key -> [nq_pad][n_ctiles*128]
            float* keys = (float*)p.dbgbuf;
            const int64_t ld = (int64_t)p.n_ctiles * TILE_R;
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    keys[(q0 + ql) * ld + (int64_t)(ct0 + t) * V5_TR + rl0 + 16 * m + i] = key[m][i];
        }
        const float tn = qv ? fminf(tr, ord2f(gr)) : -FX_INF;
        float gmin[M], mn;
#pragma unroll
        for (int m = 0; m < M; ++m) gmin[m] = fminf(fminf(key[m][0], key[m][1]), fminf(key[m][2], key[m][3]));
        mn = fminf(fminf(gmin[0], gmin[1]), fminf(gmin[2], gmin[3]));
        if (__builtin_amdgcn_ballot_w64(mn <= tn)) {
            const int trow0 = (ct0 + t) * V5_TR;
            const int rlim = p.ntotal < (int64_t)trow0 + V5_TR ? (int)p.ntotal : trow0 + V5_TR;
            unsigned pend = 0u;
            bool ovf = false;
            static_for<M>([&](auto MM) {
                constexpr int m = decltype(MM)::value;
                if (__builtin_amdgcn_ballot_w64(gmin[m] <= tn))
                    ovf |= push4<CAPV>(key[m], m, 15u, tn, ql, trow0 + rl0 + m * 16, rlim, lst_d, lst_i, cnt, pend);
            });
            while (__builtin_amdgcn_ballot_w64(ovf)) {
                compact16<CAPV>(lst_d, lst_i, cnt, tau, gt_first, qf, lane);
                ovf = false;
                const float tq = qv ? fminf(tau[ql], tn) : -FX_INF;
                const unsigned pn = pend;
                pend = 0u;
                static_for<M>([&](auto MM) {
                    constexpr int m = decltype(MM)::value;
                    const unsigned el = (pn >> (4 * m)) & 15u;
                    if (__builtin_amdgcn_ballot_w64(el != 0u))
                        ovf |= push4<CAPV>(key[m], m, el, tq, ql, trow0 + rl0 + m * 16, rlim, lst_d, lst_i, cnt, pend);
                });
            }
        }
    }

    if constexpr (STAG) {
        if (ntiles > 0) {  // the last tile: both halves finish it after one barrier
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            finish(ntiles - 1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
    const int64_t obase = ((int64_t)qtile * p.splits + split) * TILE_Q;
    for (int qi = 0; qi < 16; ++qi) {
        const int q = qf + qi;
        if (q0 + q >= p.nq) break;
        const int cn = min(cnt[q], CAPV);
        float d = lane < cn ? lst_d[q * CAPV + lane] : FX_INF;
        int i = lane < cn ? lst_i[q * CAPV + lane] : INT_MAX;
        sort64(d, i, lane);
        if (lane < KP) {
            p.cand_d[(obase + q) * KP + lane] = d;
            p.cand_i[(obase + q) * KP + lane] = i == INT_MAX ? -1 : i;
        }
    }
}

template <int DT, int METRIC, int KSTEPS, int STAG>
static hipError_t scan_v5_t(const ScanParams& p, hipStream_t s) {
    hipError_t e = g_graph_capture ? hipSuccess : hipFuncSetAttribute((const void*)k_scan_v5<DT, METRIC, KSTEPS, STAG>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, V5Lds<STAG>::BYTES);
    if (e != hipSuccess) return e;
    const int grid = p.qt_per_xcd > 0 ? 8 * p.qt_per_xcd * p.splits : p.n_qtiles * p.splits;
    hipLaunchKernelGGL((k_scan_v5<DT, METRIC, KSTEPS, STAG>), dim3(grid), dim3(V5_THREADS), V5Lds<STAG>::BYTES, s,
                       p);
    return hipGetLastError();
}

// STAG (the staggered epilogue) is built for the 2-byte dtypes only
template <int DT, int METRIC>
static hipError_t scan5_rows(const ScanParams& p, hipStream_t s, bool stag, bool* handled) {
    *handled = true;
    constexpr bool S = DT != F32;
    switch (p.row_bytes / 64) {
        case 8: return (S && stag) ? scan_v5_t<DT, METRIC, 8, S>(p, s) : scan_v5_t<DT, METRIC, 8, 0>(p, s);
        case 12:
            if constexpr (DT == F32S) {  // a plane quarter of 192 B is not whole stages: k_scan_v4 takes it
                *handled = false;
                return hipSuccess;
            } else {
                return (S && stag) ? scan_v5_t<DT, METRIC, 12, S>(p, s) : scan_v5_t<DT, METRIC, 12, 0>(p, s);
            }
        case 16: return (S && stag) ? scan_v5_t<DT, METRIC, 16, S>(p, s) : scan_v5_t<DT, METRIC, 16, 0>(p, s);
        case 24: return (S && stag) ? scan_v5_t<DT, METRIC, 24, S>(p, s) : scan_v5_t<DT, METRIC, 24, 0>(p, s);
        default: *handled = false; return hipSuccess;
    }
}

hipError_t launch_scan_mfma5(int st_dt, int metric, const ScanParams& p, hipStream_t s, bool stag, bool* handled) {
    if (p.row_bytes % 64 != 0) {
        *handled = false;
        return hipSuccess;
    }
    if (st_dt == F32S)
        return metric == L2 ? scan5_rows<F32S, L2>(p, s, stag, handled) : scan5_rows<F32S, IP>(p, s, stag, handled);
    if (metric == L2) {
        if (st_dt == F32) return scan5_rows<F32, L2>(p, s, stag, handled);
        if (st_dt == BF16) return scan5_rows<BF16, L2>(p, s, stag, handled);
        return scan5_rows<F16, L2>(p, s, stag, handled);
    }
    if (st_dt == F32) return scan5_rows<F32, IP>(p, s, stag, handled);
    if (st_dt == BF16) return scan5_rows<BF16, IP>(p, s, stag, handled);
    return scan5_rows<F16, IP>(p, s, stag, handled);
}

}  // namespace fx
