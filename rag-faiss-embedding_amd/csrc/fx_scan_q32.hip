// fx_scan_q32.hip -- the small-batch scan (k_scan_q32): nq <= 32 per tile.
//
// The reference searches ONE query per call (faiss_store.py:61 reshapes to
// (1, d)); at such batches the scan is HBM-bound (ridge at
// nq ~ 39 fp32 / ~312 bf16), and k_scan_v4's 128-query tile would spend 4x the
// MFMA work of a 32-query tile on padding.  Here a workgroup holds 32 queries
// and its 4 waves split the corpus rows instead of the queries:
//
//   * every wave keeps the same 32 queries in AGPRs (as k_scan_v4's waves do
//     for their own 32) and owns 32 of each 128-row tile (row blocks 2w, 2w+1);
//   * a wave DMAs exactly the 4 KiB of each stage it reads itself (same LDS
//     image and pieces as k_scan_v4), so the waves never wait for each other:
//     no s_barrier, only the wave's own counted vmcnt per stage;
//   * a stage's 4 fragments are read one stage ahead into a second register
//     set, hiding the LDS latency behind the current stage's 8 MFMAs and the
//     wave's 4 DMA issues;
//   * each wave keeps its own top-KP lists for the 32 queries; after the scan
//     the 4 waves' lists are merged in LDS (one barrier) into one list per
//     (query, corpus split), in the refine's [query tile of 128][split][128][KP]
//     layout.
//
// Opt-in (FX_SCAN_Q32=1).  Measured (profiles/r2_sweep_nq.jsonl): at nq = 1 its
// scan is slower than k_scan_v4's on 10M x 768 bf16 (2.64 vs 2.48 ms) and on
// 1M x 384 fp32 (0.49 vs 0.32 ms); the search as a whole is faster on the
// latter through the refine's prefetch (0.79 vs 1.08 ms), so it stays opt-in.
#include "fx_scan_common.h"

#include <stdlib.h>

namespace fx {

constexpr int Q_NS = 5;                          // ring slots (4 stages in flight per wave)
constexpr int Q_STAGE = TILE_R * STAGE_B;        // 16 KiB: the 4 waves' 4 KiB blocks
constexpr int Q_NORM_OFF = 0;                    // [tile slot][wave][32 norms | 32 thresholds]
constexpr int Q_NSLOT_B = 4 * 256;
constexpr int Q_RING_OFF = Q_NORM_OFF + 4 * Q_NSLOT_B;  // 4 KiB: >= any DMA instruction offset
constexpr int Q_LD_OFF = Q_RING_OFF + Q_NS * Q_STAGE;
constexpr int Q_LI_OFF = Q_LD_OFF + TILE_Q * CAP * 4;     // list slot = wave * 32 + query
constexpr int Q_CNT_OFF = Q_LI_OFF + TILE_Q * CAP * 4;
constexpr int Q_TAU_OFF = Q_CNT_OFF + TILE_Q * 4;
constexpr int Q_LDS_BYTES = Q_TAU_OFF + TILE_Q * 4;
static_assert(Q_LDS_BYTES <= 160 * 1024, "LDS budget");

// 48 wait states between the last (asm) MFMA and the epilogue's VALU reads
__device__ __forceinline__ void acc_fence2(f32x4 (&acc)[2][2]) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[1][0]), "+v"(acc[1][1]));
}

template <int P, typename T>
__device__ __forceinline__ T& pick(T& a, T& b) {
    if constexpr (P == 0) return a;
    else return b;
}

template <int DT, int METRIC, int KSTEPS>
__global__ __launch_bounds__(SCAN_THREADS, 1) void k_scan_q32(ScanParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename AsmMmaV<DT>::A frag_t;
    typedef typename AsmMmaV<DT>::B bfrag_t;
    constexpr int SPT = KSTEPS / 2;  // stages per tile
    constexpr int NS = Q_NS;
    constexpr int M = 2;             // this wave's 16-row blocks per tile
    constexpr int N = 2;             // 16-query columns
    constexpr int KH = KSTEPS / 2;
    constexpr int RB = KSTEPS * 64;
    constexpr int64_t TILE_BYTES = (int64_t)TILE_R * RB;
    static_assert(SPT >= NS - 1 && SPT % 2 == 0, "prefetch within the next tile; register sets alternate per stage");

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int qt = (int)(blockIdx.x % (unsigned)p.q32_tiles), split = (int)(blockIdx.x / (unsigned)p.q32_tiles);
    const int ct0 = (int)((int64_t)split * p.n_ctiles / p.splits);
    const int ct1 = (int)((int64_t)(split + 1) * p.n_ctiles / p.splits);
    const int ntiles = ct1 - ct0;
    const int64_t q0 = (int64_t)qt * 32;  // this workgroup's 32 queries

    float* lst_d = (float*)(smem + Q_LD_OFF);
    int* lst_i = (int*)(smem + Q_LI_OFF);
    int* cnt = (int*)(smem + Q_CNT_OFF);
    float* tau = (float*)(smem + Q_TAU_OFF);
    const int sw0 = wave * 32;  // this wave's list slots
    if (lane < 32) {
        cnt[sw0 + lane] = 0;
        tau[sw0 + lane] = KEY_MAX;
    }
    unsigned* gtq = p.gtau + q0;

    // the 32 queries -> AGPRs (B fragments), settled before the ring starts
    bfrag_t b[KSTEPS][N];
    {
        const char* qb = p.qop + (q0 + (lane & 15)) * RB + (lane >> 4) * 16;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
            for (int n = 0; n < N; ++n) b[ks][n] = *(const bfrag_t*)(qb + n * 16 * RB + ks * 64);
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
            for (int n = 0; n < N; ++n) AsmMmaV<DT>::settle(b[ks][n]);
    }

    // DMA: the wave's 4 pieces of a stage = row blocks 2w, 2w+1 x the stage's
    // two 64-B K-steps (k_scan_v4's image: block (m, half) at m*2048 + half*1024)
    const uint32_t voffA = (uint32_t)((2 * wave * 16 + (lane & 15)) * RB + (lane >> 4) * 16);
    const uint32_t voffB = voffA + 16 * RB;
    const uint32_t lds_base = lds_off(smem);
    const uint32_t m0w = lds_base + Q_RING_OFF + wave * 4096;
    const uint32_t nslot_w = lds_base + Q_NORM_OFF + wave * 256;
    const char* cb_cur = sgpr_ptr(p.codes + (int64_t)ct0 * TILE_BYTES);
    const char* cb_nxt = sgpr_ptr(ntiles > 1 ? cb_cur + TILE_BYTES : cb_cur);
    const int nstep = lane < 8 ? TILE_R * 4 : 0;
    const char* nv_cur = lane < 8 ? (const char*)(p.norms + (int64_t)ct0 * TILE_R + 32 * wave + lane * 4)
                                  : (const char*)(gtq + ((lane - 8) & 7) * 4);
    const char* nv_nxt = ntiles > 1 ? nv_cur + nstep : nv_cur;

    auto piece = [&](auto W, auto JP, auto NXT, uint32_t slot, int tnext) {
        constexpr int w = decltype(W)::value, jp = decltype(JP)::value;
        const char* cb = decltype(NXT)::value ? cb_nxt : cb_cur;
        const uint32_t m0 = m0w + slot * Q_STAGE + w * 1024;
        if constexpr (w == 0) dma_piece<jp * STAGE_B>(voffA, cb, m0);
        if constexpr (w == 1) dma_piece<jp * STAGE_B + 64>(voffA, cb, m0);
        if constexpr (w == 2) dma_piece<jp * STAGE_B>(voffB, cb, m0);
        if constexpr (w == 3) dma_piece<jp * STAGE_B + 64>(voffB, cb, m0);
        if constexpr (w == 4)
            dma_norm_piece(decltype(NXT)::value ? nv_nxt : nv_cur, nslot_w + (uint32_t)(tnext & 3) * Q_NSLOT_B);
    };

    // prologue: stages 0 .. NS-2 (all in tile 0), the norm piece with stage 0
    static_for<NS - 1>([&](auto ST) {
        constexpr int st = decltype(ST)::value;
        static_for<4>([&](auto W) { piece(W, ST, std::false_type{}, (uint32_t)st, 0); });
        if constexpr (st == 0) piece(std::integral_constant<int, 4>{}, ST, std::false_type{}, 0u, 0);
    });

    f32x4 acc[M][N];
    frag_t F0[2][M], F1[2][M];  // two register sets: [K-step of the stage][row block]
    f32x4 yin[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        acc[m][0] = acc[m][1] = yin[m] = f32x4{0.f, 0.f, 0.f, 0.f};
        F0[0][m] = F0[1][m] = F1[0][m] = F1[1][m] = frag_t{};
    }
    const int rl0 = 4 * (lane >> 4);
    int qloc[N];
#pragma unroll
    for (int n = 0; n < N; ++n) qloc[n] = sw0 + n * 16 + (lane & 15);
    const bool qv0 = q0 + (lane & 15) < p.nq, qv1 = q0 + 16 + (lane & 15) < p.nq;
    const uint32_t tau_addr = lds_off(tau + qloc[0]);
    const uint32_t gt_lane = (uint32_t)(128 + (lane & 15) * 4);
    const uint32_t nrm_lane = (uint32_t)(rl0 * 4);
    // this wave's fragments of ring slot s: block (2w + m, half) at s*STAGE + (2w+m)*2048 + half*1024
    const uint32_t rd_w = lds_base + Q_RING_OFF + (uint32_t)(wave * 4096 + lane * 16);

    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // stage 0 (4 pieces + norms) landed
    __builtin_amdgcn_sched_barrier(0);
    if (ntiles > 0) {
        ds_rd128<0>(F0[0][0], rd_w);
        ds_rd128<2048>(F0[0][1], rd_w);
        ds_rd128<1024>(F0[1][0], rd_w);
        ds_rd128<3072>(F0[1][1], rd_w);
        const uint32_t na = lds_base + Q_NORM_OFF + wave * 256 + nrm_lane;
        ds_rd128<0>(yin[0], na);
        ds_rd128<64>(yin[1], na);
    }

    int c = 0;  // ring slot of the current stage
    for (int t = 0; t < ntiles; ++t) {
        float tr[N];
        unsigned gr[N];
        static_for<SPT>([&](auto JJ) {
            constexpr int j = decltype(JJ)::value;
            constexpr bool LAST = j == SPT - 1;
            constexpr int jp = (j + NS - 1) % SPT;
            constexpr bool nxt = j + NS - 1 >= SPT;
            typedef std::integral_constant<bool, nxt> NXT;
            typedef std::integral_constant<int, jp> JP;
            constexpr bool HI = DT == F32S && 2 * j < KH;
            constexpr int kq = (DT == F32S && !HI) ? 2 * j - KH : 2 * j;  // query K-step of the stage's first half
            const uint32_t c1 = c == NS - 1 ? 0u : (uint32_t)c + 1;
            const uint32_t c4 = c == 0 ? (uint32_t)NS - 1 : (uint32_t)c - 1;
            const int tnext = t + (nxt ? 1 : 0);
            auto& cur = pick<j % 2>(F0, F1);
            auto& nxf = pick<(j + 1) % 2>(F0, F1);
            // stage g+1 landed (own pieces only: VMEM younger than its = stages g+2, g+3);
            // this stage's fragments are in registers
            constexpr int W = 8 + ((j + 3) % SPT == 0) + ((j + 2) % SPT == 0);
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(W) : "memory");
            __builtin_amdgcn_sched_barrier(0);
            // next stage's fragments into the other set (its last MFMA readers were a stage ago)
            const uint32_t rd_n = rd_w + c1 * Q_STAGE;
            ds_rd128<0>(nxf[0][0], rd_n);
            ds_rd128<2048>(nxf[0][1], rd_n);
            ds_rd128<1024>(nxf[1][0], rd_n);
            ds_rd128<3072>(nxf[1][1], rd_n);
            if constexpr (LAST) {
                ds_rd32<0>(tr[0], tau_addr);
                ds_rd32<64>(tr[1], tau_addr);
                const uint32_t ns = lds_base + Q_NORM_OFF + (uint32_t)(t & 3) * Q_NSLOT_B + wave * 256 + gt_lane;
                ds_rd32<0>(gr[0], ns);
                ds_rd32<64>(gr[1], ns);
            }
            constexpr int INIT = j == 0 ? (METRIC == L2 ? 1 : 2) : 0;
            AsmMmaV<DT>::template mma2<INIT>(acc[0][0], acc[0][1], cur[0][0], b[kq][0], b[kq][1], yin[0]);
            AsmMmaV<DT>::template mma2<INIT>(acc[1][0], acc[1][1], cur[0][1], b[kq][0], b[kq][1], yin[1]);
            piece(std::integral_constant<int, 0>{}, JP{}, NXT{}, c4, tnext);
            AsmMmaV<DT>::template mma2<0>(acc[0][0], acc[0][1], cur[1][0], b[kq + 1][0], b[kq + 1][1], yin[0]);
            AsmMmaV<DT>::template mma2<0>(acc[1][0], acc[1][1], cur[1][1], b[kq + 1][0], b[kq + 1][1], yin[1]);
            piece(std::integral_constant<int, 1>{}, JP{}, NXT{}, c4, tnext);
            if constexpr (HI) {  // split fp32: hi plane x x_lo
                AsmMmaV<DT>::template mma2<0>(acc[0][0], acc[0][1], cur[0][0], b[kq + KH][0], b[kq + KH][1], yin[0]);
                AsmMmaV<DT>::template mma2<0>(acc[1][0], acc[1][1], cur[0][1], b[kq + KH][0], b[kq + KH][1], yin[1]);
                AsmMmaV<DT>::template mma2<0>(acc[0][0], acc[0][1], cur[1][0], b[kq + 1 + KH][0],
                                              b[kq + 1 + KH][1], yin[0]);
                AsmMmaV<DT>::template mma2<0>(acc[1][0], acc[1][1], cur[1][1], b[kq + 1 + KH][0],
                                              b[kq + 1 + KH][1], yin[1]);
            }
            piece(std::integral_constant<int, 2>{}, JP{}, NXT{}, c4, tnext);
            piece(std::integral_constant<int, 3>{}, JP{}, NXT{}, c4, tnext);
            if constexpr (jp == 0) piece(std::integral_constant<int, 4>{}, JP{}, NXT{}, c4, tnext);
            if constexpr (LAST) {
                // the next tile's row norms (its first MFMAs' srcC); their piece
                // came with stage g+1, which the wait above retired
                const uint32_t na = lds_base + Q_NORM_OFF + (uint32_t)((t + 1) & 3) * Q_NSLOT_B + wave * 256 + nrm_lane;
                ds_rd128<0>(yin[0], na);
                ds_rd128<64>(yin[1], na);
            }
            __builtin_amdgcn_sched_barrier(0);
            c = (int)c1;
        });

        // ---- epilogue of tile t: the accumulator holds the keys ------------
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // tr / gr (asm LDS reads) have landed
        acc_fence2(acc);
        const int trow0 = (ct0 + t) * TILE_R + 32 * wave;  // this wave's rows of the tile
        if (p.dbgbuf) {  // diagnostics (FX_SCAN_DBG & 32): every key -> [nq_pad][n_ctiles * 128]
            float* keys = (float*)p.dbgbuf;
            const int64_t ld = (int64_t)p.n_ctiles * TILE_R;
#pragma unroll
            for (int n = 0; n < N; ++n)
#pragma unroll
                for (int m = 0; m < M; ++m)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        keys[(q0 + n * 16 + (lane & 15)) * ld + trow0 + 16 * m + rl0 + i] = acc[m][n][i];
        }
        float tn[N];
        tn[0] = qv0 ? fminf(tr[0], ord2f(gr[0])) : -FX_INF;
        tn[1] = qv1 ? fminf(tr[1], ord2f(gr[1])) : -FX_INF;
        float gmin[N][M], mn[N];
#pragma unroll
        for (int n = 0; n < N; ++n) {
#pragma unroll
            for (int m = 0; m < M; ++m)
                gmin[n][m] = fminf(fminf(acc[m][n][0], acc[m][n][1]), fminf(acc[m][n][2], acc[m][n][3]));
            mn[n] = fminf(gmin[n][0], gmin[n][1]);
        }
        if (__builtin_amdgcn_ballot_w64(mn[0] <= tn[0] || mn[1] <= tn[1])) {
            const int rlim = p.ntotal < (int64_t)trow0 + 32 ? (int)p.ntotal : trow0 + 32;
            unsigned pend[N] = {0u, 0u};
            bool ovf = false;
            static_for<N>([&](auto NN) {
                constexpr int n = decltype(NN)::value;
                if (__builtin_amdgcn_ballot_w64(mn[n] <= tn[n])) {
                    static_for<M>([&](auto MM) {
                        constexpr int m = decltype(MM)::value;
                        if (__builtin_amdgcn_ballot_w64(gmin[n][m] <= tn[n]))
                            ovf |= push_group<M, N>(acc, n, m, 15u, tn[n], qloc[n], trow0 + rl0 + m * 16, rlim,
                                                    lst_d, lst_i, cnt, pend[n]);
                    });
                }
            });
            while (__builtin_amdgcn_ballot_w64(ovf)) {
                compact_wave(lst_d, lst_i, cnt, tau, p.share ? gtq : nullptr, sw0, lane);
                ovf = false;
                static_for<N>([&](auto NN) {
                    constexpr int n = decltype(NN)::value;
                    const float tq = (n == 0 ? qv0 : qv1) ? fminf(tau[qloc[n]], tn[n]) : -FX_INF;
                    const unsigned pn = pend[n];
                    pend[n] = 0u;
                    static_for<M>([&](auto MM) {
                        constexpr int m = decltype(MM)::value;
                        const unsigned el = (pn >> (4 * m)) & 15u;
                        if (__builtin_amdgcn_ballot_w64(el != 0u))
                            ovf |= push_group<M, N>(acc, n, m, el, tq, qloc[n], trow0 + rl0 + m * 16, rlim, lst_d,
                                                    lst_i, cnt, pend[n]);
                    });
                });
            }
        }
        // advance the tile bases (clamped: stages past the end re-read the last tile)
        cb_cur = sgpr_ptr(cb_nxt);
        nv_cur = nv_nxt;
        if (t + 2 < ntiles) {
            cb_nxt = sgpr_ptr(cb_nxt + TILE_BYTES);
            nv_nxt += nstep;
        }
    }

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
    // each wave: its sorted top-KP per query, in place (missing entries +inf)
    for (int qi = 0; qi < 32; ++qi) {
        const int q = sw0 + qi;
        const int cn = min(cnt[q], CAP);
        float d = lane < cn ? lst_d[q * CAP + lane] : FX_INF;
        int i = lane < cn ? lst_i[q * CAP + lane] : INT_MAX;
        sort64(d, i, lane);
        if (lane < KP) {
            lst_d[q * CAP + lane] = d;
            lst_i[q * CAP + lane] = i;
        }
    }
    __syncthreads();
    // wave w merges queries 8w .. 8w+7 over the 4 waves' lists -> one list
    // per (query, split) in the refine's [query tile of 128][split][128][KP]
    const int64_t qt128 = q0 / TILE_Q, qoff = q0 % TILE_Q;
    const int64_t obase = (qt128 * p.splits + split) * TILE_Q + qoff;
    for (int qq = 0; qq < 8; ++qq) {
        const int qi = wave * 8 + qq;
        if (q0 + qi >= p.nq) break;
        const int s0 = (lane >> 5) * 32 + qi, s1 = (2 + (lane >> 5)) * 32 + qi;  // slots of waves 0/1, 2/3
        float d = lst_d[s0 * CAP + (lane & 31)];
        int i = lst_i[s0 * CAP + (lane & 31)];
        float d2 = lst_d[s1 * CAP + (lane & 31)];
        int i2 = lst_i[s1 * CAP + (lane & 31)];
        sort64(d, i, lane);
        sort64(d2, i2, lane);
        merge_into(d, i, d2, i2, lane);
        if (lane < KP) {
            p.cand_d[(obase + qi) * KP + lane] = d;
            p.cand_i[(obase + qi) * KP + lane] = i == INT_MAX ? -1 : i;
        }
    }
}

template <int DT, int METRIC, int KSTEPS>
static hipError_t scan_q32_t(const ScanParams& p, hipStream_t s) {
    hipError_t e = g_graph_capture ? hipSuccess : hipFuncSetAttribute((const void*)k_scan_q32<DT, METRIC, KSTEPS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, Q_LDS_BYTES);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_scan_q32<DT, METRIC, KSTEPS>), dim3(p.grid), dim3(SCAN_THREADS),
                       Q_LDS_BYTES, s, p);
    return hipGetLastError();
}

template <int DT, int METRIC>
static hipError_t scan_q32_rows(const ScanParams& p, hipStream_t s, bool* handled) {
    *handled = true;
    switch (p.row_bytes / 64) {
        case 8: return scan_q32_t<DT, METRIC, 8>(p, s);
        case 12: return scan_q32_t<DT, METRIC, 12>(p, s);
        case 16: return scan_q32_t<DT, METRIC, 16>(p, s);
        case 24: return scan_q32_t<DT, METRIC, 24>(p, s);
        default: *handled = false; return hipSuccess;
    }
}

hipError_t launch_scan_q32(int st_dt, int metric, const ScanParams& p, hipStream_t s, bool* handled) {
    *handled = false;
    if (p.row_bytes % 64 != 0 || p.q32_tiles <= 0) return hipSuccess;
    if (metric == L2) {
        if (st_dt == F32) return scan_q32_rows<F32, L2>(p, s, handled);
        if (st_dt == F32S) return scan_q32_rows<F32S, L2>(p, s, handled);
        if (st_dt == BF16) return scan_q32_rows<BF16, L2>(p, s, handled);
        return scan_q32_rows<F16, L2>(p, s, handled);
    }
    if (st_dt == F32) return scan_q32_rows<F32, IP>(p, s, handled);
    if (st_dt == F32S) return scan_q32_rows<F32S, IP>(p, s, handled);
    if (st_dt == BF16) return scan_q32_rows<BF16, IP>(p, s, handled);
    return scan_q32_rows<F16, IP>(p, s, handled);
}

}  // namespace fx
