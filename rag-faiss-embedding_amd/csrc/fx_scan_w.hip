// fx_scan_w.hip -- the wide-tile search() scan for large query batches
// (BASELINE configs (d) and (e): 10k-query batches).
//
// Same contract as k_scan_v4 (fx_scan.hip): exact squared-L2 / inner-product
// keys of every (query, corpus row) pair by MFMA, fused with a per-(query,
// split) top-KP select into per-wave LDS lists, cross-split pruning through
// the shared per-query thresholds, candidate lists out in the
// [qtile128][split][128][KP] layout k_refine reads.  What changes is the
// shape of the work: k_scan_v4 keeps 32 queries per wave (128 per workgroup)
// in AGPRs and streams 128-row corpus tiles; here a wave keeps N x 16 queries
// (N = 3: 192 per workgroup) and streams 16 M-row tiles (M = 4: 64 rows).
// Per corpus byte moved into the CU the workgroup does N/2 times the MFMA
// work of k_scan_v4, so per MFMA it issues 2/N of the LDS-DMA pieces (the
// largest stall of k_scan_v4: DESIGN.md 3.1), 2/N of the fragment reads and
// barriers, and the corpus passes through L2 nq/(64 N) times instead of
// nq/128.  The register file sets N: the queries of a wave take
// KSTEPS x N x 4 AGPRs (288 at d = 768, N = 3).
//
// Pipeline per wave, per 16-KiB stage (SB bytes of K x 16 M rows):
//   * PPW LDS-DMA pieces (full-line: 8 rows x 128 B, source-side XOR swizzle of
//     the 16-B chunks by row & 7, as k_scan_v4's LN = 1 image), plus one
//     row-norm / shared-threshold piece per tile;
//   * one counted `s_waitcnt vmcnt` + s_barrier retires the next stage;
//   * K-steps of the stage alternate between two pinned fragment register sets:
//     the fragments of K-step s+1 are read during K-step s's M x N MFMAs, each
//     read >= 8 MFMAs after the register's previous MFMA reader;
//   * a tile's first MFMAs take srcC = |y|^2 of its rows (L2);
//   * epilogue per tile: as k_scan_v4 (group minima, ballot, rare pushes into
//     the wave's own lists, wave-level compaction publishing the KP-th key).
#include "fx_scan_common.h"

#include <stdlib.h>

namespace fx {

// single MFMA 16x16x32 (bf16 / f16 operands; F32S runs on the bf16 pipe),
// pinned operands as AsmMmaV (fx_device.h)
// single MFMA 16x16x32 (bf16 / f16 operands; F32S runs on the bf16 pipe),
// pinned operands as AsmMmaV (fx_device.h).  BA: the B (query) fragment is an
// AGPR operand -- the AGPR file holds 256 registers, so a wave's stationary
// queries beyond 64 fragments live in VGPRs ("v": gfx950 MFMAs read B from
// either file)
#define FX_MMA1(OP)                                                                                   \
    template <int INIT, bool BA, typename T>                                                          \
    static __device__ __forceinline__ void run(f32x4& c, const T& a, const T& b, const f32x4& ci) {    \
        if constexpr (BA) {                                                                           \
            if constexpr (INIT == 0)                                                                  \
                asm volatile(OP " %0, %1, %2, %0" : "+v"(c) : "v"(a), "a"(b));                        \
            else if constexpr (INIT == 1)                                                             \
                asm volatile(OP " %0, %1, %2, %3" : "+v"(c) : "v"(a), "a"(b), "v"(ci));               \
            else                                                                                      \
                asm volatile(OP " %0, %1, %2, 0" : "+v"(c) : "v"(a), "a"(b));                         \
        } else {                                                                                      \
            if constexpr (INIT == 0)                                                                  \
                asm volatile(OP " %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));                        \
            else if constexpr (INIT == 1)                                                             \
                asm volatile(OP " %0, %1, %2, %3" : "+v"(c) : "v"(a), "v"(b), "v"(ci));               \
            else                                                                                      \
                asm volatile(OP " %0, %1, %2, 0" : "+v"(c) : "v"(a), "v"(b));                         \
        }                                                                                             \
    }
template <int DT> struct Mma1;
template <> struct Mma1<BF16> { FX_MMA1("v_mfma_f32_16x16x32_bf16") };
template <> struct Mma1<F16> { FX_MMA1("v_mfma_f32_16x16x32_f16") };
template <> struct Mma1<F32S> : Mma1<BF16> {};
#undef FX_MMA1
constexpr int AGPR_FRAGS = 64;  // 256 AGPRs / 4 per fragment

template <int DT> struct WFrag { typedef bf16x8 T; };
template <> struct WFrag<F16> { typedef f16x8 T; };

// LDS carve (bytes), generic in the tile shape
template <int M, int N, int NS, int CAPL>
struct WLayout {
    static constexpr int TR = 16 * M, QW = 16 * N, QT = 4 * QW;
    static constexpr int NSLOT_B = (TR * 4 + QW * 4 + 255) / 256 * 256;  // [TR norms | QW thresholds]
    static constexpr int NORM_OFF = 0;                                   // [2 tile slots][4 waves]
    static constexpr int LD_OFF = NORM_OFF + 2 * 4 * NSLOT_B;
    static constexpr int LI_OFF = LD_OFF + QT * CAPL * 4;
    static constexpr int CNT_OFF = LI_OFF + QT * CAPL * 4;
    static constexpr int TAU_OFF = CNT_OFF + QT * 4;
    // ring last: every piece's LDS address is then >= 4 KiB, more than any
    // instruction offset subtracted from its M0 (dma_piece)
    static constexpr int RING_OFF = (TAU_OFF + QT * 4 + 1023) / 1024 * 1024;
    static constexpr int BYTES = RING_OFF + NS * 16384;
    static_assert(RING_OFF >= 4096, "M0 = lds - offset must not wrap");
    static_assert(BYTES <= 160 * 1024, "LDS budget");
};

// push the entries of accumulator group (m, n) selected by `elig` that pass
// `tn` into list slot q (as push_group, list capacity CAPL)
template <int M, int N, int CAPL>
__device__ __forceinline__ bool wpush(const f32x4 (&acc)[M][N], int n, int m, unsigned elig, float tn, int q,
                                      int row0, int rlim, float* lst_d, int* lst_i, int* cnt, unsigned& pend) {
    bool ovf = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float v = acc[m][n][i];
        const int rl = row0 + i;
        if (((elig >> i) & 1u) && v <= tn && rl < rlim) {
            const int s = atomicAdd(&cnt[q], 1);
            if (s < CAPL) {
                lst_d[q * CAPL + s] = v;
                lst_i[q * CAPL + s] = rl;
            } else {
                pend |= 1u << (m * 4 + i);
                ovf = true;
            }
        }
    }
    return ovf;
}

// compact this wave's full lists (cnt >= CAPL) to their KP best; tau = KP-th,
// published to the shared per-query threshold (gtq null: no sharing)
template <int QW, int CAPL>
__device__ __noinline__ void wcompact(float* lst_d, int* lst_i, int* cnt, float* tau, unsigned* gtq, int qw0,
                                      int lane) {
    for (int qi = 0; qi < QW; ++qi) {
        const int q = qw0 + qi;
        if (cnt[q] >= CAPL) {
            float d = lane < CAPL ? lst_d[q * CAPL + lane] : FX_INF;
            int i = lane < CAPL ? lst_i[q * CAPL + lane] : INT_MAX;
            sort64(d, i, lane);
            if (lane < KP) {
                lst_d[q * CAPL + lane] = d;
                lst_i[q * CAPL + lane] = i;
            }
            if (lane == KP - 1) {
                tau[q] = d;
                if (gtq) atomicMin(gtq + qi, f2ord(d));
            }
            if (lane == 0) cnt[q] = KP;
        }
    }
}

// the norm / threshold piece: lanes [0, LANES) move 16 B each (row norms,
// then the wave's thresholds); the other lanes are masked off
template <int LANES>
__device__ __forceinline__ void dma_norm_piece_w(const char* vaddr, uint32_t m0) {
    static_assert(LANES > 0 && LANES <= 64, "lanes");
    constexpr uint64_t MASK = LANES == 64 ? ~0ull : ((1ull << LANES) - 1);
    uint64_t saved;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "v"(vaddr), "{m0}"(m0), "s"(MASK)
        : "memory");
}

template <int M, int N>
__device__ __forceinline__ void acc_fence_w(f32x4 (&acc)[M][N]) {
    // 48 wait states between the last asm MFMA and the epilogue's VALU reads;
    // the "+v" ties make the compiler keep every accumulator behind them
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
        for (int n = 0; n < N; ++n) asm volatile("" : "+v"(acc[m][n]));
}

template <int DT, int METRIC, int KSTEPS, int M, int N, int SB, int NS, int CAPL>
__global__ __launch_bounds__(SCAN_THREADS, 1) void k_scan_w(ScanParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef WLayout<M, N, NS, CAPL> L;
    typedef typename WFrag<DT>::T frag_t;
    constexpr int TR = L::TR, QW = L::QW, QT = L::QT;
    constexpr int RB = KSTEPS * 64;              // row stride in bytes
    constexpr int SPT = RB / SB;                 // stages per tile
    constexpr int KPS = SB / 64;                 // K-steps per stage
    constexpr int LPS = SB / 128;                // 128-B lines per stage
    constexpr int PPL = TR / 8;                  // pieces per line
    constexpr int PPW = LPS * PPL / 4;           // corpus pieces per wave per stage
    constexpr int64_t TILE_BYTES = (int64_t)TR * RB;
    constexpr int KH = KSTEPS / 2;
    constexpr int NLANES = (TR * 4 + QW * 4) / 16;  // lanes of the norm piece
    static_assert(TR * SB == 16384, "16-KiB stages");
    static_assert(RB % SB == 0 && SPT >= NS - 1, "whole stages per row; prefetch within the next tile");
    static_assert(KPS % 2 == 0, "fragment register sets alternate within a stage");
    static_assert(PPW >= 1 && (LPS * PPL) % 4 == 0 && (4 % LPS == 0 || LPS % 4 == 0), "pieces split evenly");
    static_assert(DT != F32S || (RB / 2) % SB == 0, "F32S: a stage lies in one plane");
    static_assert(NLANES <= 64, "one norm piece");
    static_assert(CAPL <= 64 && CAPL > KP, "list capacity");
    static_assert(PPW == KPS && M * N > 5, "one corpus piece per K-step, issued after its 6th MFMA");
    // WAR/RAW distances of the fragment reads: G[r] is read after MFMA rd_at(r)
    // of a K-step, >= 8 MFMAs after its last reader (MFMA r N + N - 1 of the
    // previous K-step) and >= 8 MFMAs before its first use (MFMA r N of the next)
    constexpr auto rd_at = [](int r) constexpr { return 7 + r * N + N - M * N < 0 ? 0 : 7 + r * N + N - M * N; };
    static_assert(rd_at(M - 1) <= M * N - 1 && M * N - rd_at(M - 1) + (M - 1) * N >= 8, "fragment read schedule");

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int wt, split;
    map_tile(blockIdx.x, p, p.n_wtiles, wt, split);
    if (wt >= p.n_wtiles) return;
    const int nct = (int)((p.ntotal + TR - 1) / TR);
    const int ct0 = (int)((int64_t)split * nct / p.splits);
    const int ct1 = (int)((int64_t)(split + 1) * nct / p.splits);
    const int ntiles = ct1 - ct0;
    const int64_t q0 = (int64_t)wt * QT;

    float* lst_d = (float*)(smem + L::LD_OFF);
    int* lst_i = (int*)(smem + L::LI_OFF);
    int* cnt = (int*)(smem + L::CNT_OFF);
    float* tau = (float*)(smem + L::TAU_OFF);
    const int qw0 = wave * QW;  // this wave's queries (tile-local) and list slots
    for (int x = lane; x < QW; x += 64) {
        cnt[qw0 + x] = 0;
        tau[qw0 + x] = KEY_MAX;
    }
    unsigned* gtq = p.gtau + q0 + qw0;

    // queries -> AGPRs (B fragments), settled once before the DMA ring starts
    frag_t b[KSTEPS][N];
    {
        const char* qb = p.qop + (q0 + qw0 + (lane & 15)) * RB + (lane >> 4) * 16;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
            for (int n = 0; n < N; ++n) b[ks][n] = *(const frag_t*)(qb + n * 16 * RB + ks * 64);
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
            for (int n = 0; n < N; ++n) {
                if (ks * N + n < AGPR_FRAGS) asm volatile("" ::"a"(b[ks][n]));
                else asm volatile("" ::"v"(b[ks][n]));
            }
    }

    // ---- DMA addressing ----------------------------------------------------
    // piece p = PPW * wave + jj of a stage: line j = p / PPL, rows 8 (p % PPL)
    // .. +7; lane l -> row + (l >> 3), source chunk (l & 7) ^ (l >> 3); the
    // stage image is [line][row][128 B] (chunk c of row r at (c ^ (r & 7)) * 16)
    const int p0 = PPW * wave;
    const uint32_t voff = (uint32_t)((8 * (p0 % PPL) + (lane >> 3)) * RB + (p0 / PPL) * 128 +
                                     (((lane & 7) ^ (lane >> 3)) << 4));
    const uint32_t lds_base = lds_off(smem);
    const uint32_t m0w = lds_base + L::RING_OFF + p0 * 1024;
    const uint32_t nslot_w = lds_base + L::NORM_OFF + wave * L::NSLOT_B;
    const char* cb_cur = sgpr_ptr(p.codes + (int64_t)ct0 * TILE_BYTES);
    const char* cb_nxt = sgpr_ptr(ntiles > 1 ? cb_cur + TILE_BYTES : cb_cur);
    constexpr int NL = TR / 4;  // norm lanes
    const int nstep = lane < NL ? TR * 4 : 0;
    const char* nv_cur = lane < NL ? (const char*)(p.norms + (int64_t)ct0 * TR + lane * 4)
                                   : (const char*)(gtq + (lane < NLANES ? lane - NL : 0) * 4);
    const char* nv_nxt = ntiles > 1 ? nv_cur + nstep : nv_cur;

    // the corpus pieces of stage (t + NXT, JP) into ring slot `slot`; piece jj
    // of this wave (jj within one line: PPW <= PPL, both powers of two)
    auto piece = [&](auto JJ, auto JP, auto NXT, uint32_t slot) {
        constexpr int jj = decltype(JJ)::value, jp = decltype(JP)::value;
        const char* cb = decltype(NXT)::value ? cb_nxt : cb_cur;
        const uint32_t m0 = m0w + slot * 16384 + jj * 1024;
        dma_piece<jp * SB>(voff, cb + jj * 8 * RB, m0);
    };
    auto norm_piece = [&](auto NXT, int tnext) {
        dma_norm_piece_w<NLANES>(decltype(NXT)::value ? nv_nxt : nv_cur,
                                 nslot_w + (uint32_t)(tnext & 1) * 4 * L::NSLOT_B);
    };

    // prologue: stages 0 .. NS-2 (all in tile 0), the norm piece with stage 0
    static_for<NS - 1>([&](auto ST) {
        constexpr int st = decltype(ST)::value;
        static_for<PPW>([&](auto JJ) { piece(JJ, ST, std::false_type{}, (uint32_t)st); });
        if constexpr (st == 0) norm_piece(std::false_type{}, 0);
    });

    f32x4 acc[M][N];
    frag_t X[M], Y[M];
    f32x4 yin[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
#pragma unroll
        for (int n = 0; n < N; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        yin[m] = f32x4{0.f, 0.f, 0.f, 0.f};
        X[m] = Y[m] = frag_t{};
    }
    const int rl0 = 4 * (lane >> 4);
    int qloc[N];
    bool qv[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
        qloc[n] = qw0 + n * 16 + (lane & 15);
        qv[n] = q0 + qloc[n] < p.nq;
    }
    // fragment-read lane offsets within a stage slot: K-steps with (ks & 1) == 0
    // take chunks 0-3 of their line, odd ones chunks 4-7 (XOR-swizzled)
    const uint32_t rd_e = (uint32_t)((lane & 15) * 128 + ((((lane >> 4)) ^ (lane & 7)) << 4));
    const uint32_t rd_o = (uint32_t)((lane & 15) * 128 + ((((lane >> 4) + 4) ^ (lane & 7)) << 4));
    const uint32_t ring0 = lds_base + L::RING_OFF;

    // stage 0 landed: of the prologue's (NS - 1) PPW + 1 pieces, the younger
    // (NS - 2) PPW may be in flight
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"((NS - 2) * PPW) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (ntiles > 0) {
        // K-step 0 of stage 0 (slot 0) -> X; row norms of tile 0
        static_for<M>([&](auto MM) {
            constexpr int m = decltype(MM)::value;
            ds_rd128<m * 2048>(X[m], ring0 + rd_e);
        });
        const uint32_t na = nslot_w + rl0 * 4;
        static_for<M>([&](auto MM) {
            constexpr int m = decltype(MM)::value;
            ds_rd128<m * 64>(yin[m], na);
        });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    int c = 0;  // ring slot of the current stage
    for (int t = 0; t < ntiles; ++t) {
        float tr[N];
        unsigned gr[N];
        static_for<SPT>([&](auto JJ) {
            constexpr int j = decltype(JJ)::value;
            constexpr bool LAST = j == SPT - 1;
            constexpr int jp = (j + NS - 1) % SPT;  // stage issued now: (t + nxt, jp)
            constexpr bool nxt = j + NS - 1 >= SPT;
            typedef std::integral_constant<bool, nxt> NXT;
            typedef std::integral_constant<int, jp> JP;
            const uint32_t c1 = c == NS - 1 ? 0u : (uint32_t)c + 1;           // slot of stage g+1
            const uint32_t cw = c == 0 ? (uint32_t)NS - 1 : (uint32_t)c - 1;  // slot of stage g+NS-1
            // stage g+1 landed for every wave (its pieces were issued NS-2
            // stages ago; younger: the previous stage's PPW pieces, plus its
            // norm piece if it prefetched a tile's first stage); slot cw is no
            // longer read by anyone
            // (no LDS wait: every read of slot cw was waited for by the counted
            // waits of the K-step that used it)
            constexpr int W = (NS - 3) * PPW + ((j + NS - 2) % SPT == 0 ? 1 : 0);
            static_assert(NS == 4, "vmcnt accounting below assumes 4 ring slots");
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(W) : "memory");
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t sbase = ring0 + (uint32_t)c * 16384;
            const uint32_t snext = ring0 + c1 * 16384;
            static_for<KPS>([&](auto KS) {
                constexpr int ks = decltype(KS)::value;
                constexpr int kg = j * KPS + ks;  // K-step within the row
                // F32S: hi-plane K-steps (kg < KH) take x_hi and x_lo, lo-plane
                // ones x_hi
                constexpr bool HI = DT == F32S && kg < KH;
                constexpr int kq = (DT == F32S && !HI) ? kg - KH : kg;
                constexpr int INIT = (j == 0 && ks == 0) ? (METRIC == L2 ? 1 : 2) : 0;
                // the fragments of the next K-step: this stage's ks + 1, or
                // K-step 0 of stage g+1
                constexpr int kn = ks + 1 == KPS ? 0 : ks + 1;
                const uint32_t rbase = (ks + 1 == KPS ? snext : sbase) + ((kn & 1) ? rd_o : rd_e);
                constexpr int roff = (kn >> 1) * TR * 128;
                frag_t(&F)[M] = (ks & 1) ? Y : X;
                frag_t(&G)[M] = (ks & 1) ? X : Y;
                __builtin_amdgcn_sched_barrier(0);
                static_for<M>([&](auto MM) {
                    constexpr int m = decltype(MM)::value;
                    // F[m] landed: the previous K-step read F[0..M-1] in order
                    // (the only LDS ops since; the tile epilogue drains all)
                    asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(M - 1 - m) : "memory");
                    static_for<N>([&](auto NN) {
                        constexpr int n = decltype(NN)::value;
                        constexpr int idx = m * N + n;  // MFMA index within the K-step
                        Mma1<DT>::template run<INIT, kq * N + n < AGPR_FRAGS>(acc[m][n], F[m], b[kq][n], yin[m]);
                        // next K-step's fragment G[r]: read after MFMA rd_at(r)
                        static_for<M>([&](auto RR) {
                            constexpr int r = decltype(RR)::value;
                            if constexpr (idx == rd_at(r)) ds_rd128<roff + r * 2048>(G[r], rbase);
                        });
                        // this stage's corpus pieces: one per K-step, after its 6th MFMA
                        if constexpr (idx == 5) piece(std::integral_constant<int, ks>{}, JP{}, NXT{}, cw);
                    });
                });
                if constexpr (HI) {  // hi * x_lo
                    static_for<M>([&](auto MM) {
                        constexpr int m = decltype(MM)::value;
                        static_for<N>([&](auto NN) {
                            constexpr int n = decltype(NN)::value;
                            Mma1<DT>::template run<0, (kg + KH) * N + n < AGPR_FRAGS>(acc[m][n], F[m], b[kg + KH][n],
                                                                                       yin[m]);
                        });
                    });
                }
                if constexpr (ks == KPS - 1 && jp == 0) norm_piece(NXT{}, t + (nxt ? 1 : 0));
                if constexpr (LAST && ks == KPS - 1) {
                    // epilogue operands: the queries' thresholds; the next
                    // tile's row norms (its first MFMAs' srcC)
                    static_for<N>([&](auto NN) {
                        constexpr int n = decltype(NN)::value;
                        ds_rd32<0>(tr[n], lds_off(tau + qloc[n]));
                    });
                    const uint32_t ns = nslot_w + (uint32_t)(t & 1) * 4 * L::NSLOT_B + TR * 4 + (lane & 15) * 4;
                    static_for<N>([&](auto NN) {
                        constexpr int n = decltype(NN)::value;
                        ds_rd32<n * 64>(gr[n], ns);
                    });
                    const uint32_t na = nslot_w + (uint32_t)((t + 1) & 1) * 4 * L::NSLOT_B + rl0 * 4;
                    static_for<M>([&](auto MM) {
                        constexpr int m = decltype(MM)::value;
                        ds_rd128<m * 64>(yin[m], na);
                    });
                }
                __builtin_amdgcn_sched_barrier(0);
            });
            c = (int)c1;
        });

        // ---- epilogue of tile t: the accumulator holds the keys ------------
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        acc_fence_w<M, N>(acc);
        if (p.dbgbuf) {  // diagnostics (FX_SCAN_DBG & 32): every key -> [nq_pad][ld]
            float* keys = (float*)p.dbgbuf;
            const int64_t ld = (p.ntotal + TILE_R - 1) / TILE_R * TILE_R;
            const int64_t rows = (int64_t)(ct0 + t) * TR;
#pragma unroll
            for (int n = 0; n < N; ++n)
#pragma unroll
                for (int m = 0; m < M; ++m)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int64_t row = rows + rl0 + 16 * m + i;
                        if (qv[n] && row < ld) keys[(q0 + qloc[n]) * ld + row] = acc[m][n][i];
                    }
        }
        float tn[N], gmin[N][M], mn[N];
        bool any = false;
#pragma unroll
        for (int n = 0; n < N; ++n) {
            tn[n] = qv[n] ? fminf(tr[n], ord2f(gr[n])) : -FX_INF;
#pragma unroll
            for (int m = 0; m < M; ++m)
                gmin[n][m] = fminf(fminf(acc[m][n][0], acc[m][n][1]), fminf(acc[m][n][2], acc[m][n][3]));
            mn[n] = gmin[n][0];
#pragma unroll
            for (int m = 1; m < M; ++m) mn[n] = fminf(mn[n], gmin[n][m]);
            any |= mn[n] <= tn[n];
        }
        if (__builtin_amdgcn_ballot_w64(any)) {
            // slow path: some row beats a query's threshold
            const int trow0 = (ct0 + t) * TR;
            const int rlim = p.ntotal < (int64_t)trow0 + TR ? (int)p.ntotal : trow0 + TR;
            unsigned pend[N];
            bool ovf = false;
            static_for<N>([&](auto NN) {
                constexpr int n = decltype(NN)::value;
                pend[n] = 0u;
                if (__builtin_amdgcn_ballot_w64(mn[n] <= tn[n])) {
                    static_for<M>([&](auto MM) {
                        constexpr int m = decltype(MM)::value;
                        if (__builtin_amdgcn_ballot_w64(gmin[n][m] <= tn[n]))
                            ovf |= wpush<M, N, CAPL>(acc, n, m, 15u, tn[n], qloc[n], trow0 + rl0 + m * 16, rlim,
                                                     lst_d, lst_i, cnt, pend[n]);
                    });
                }
            });
            while (__builtin_amdgcn_ballot_w64(ovf)) {
                wcompact<QW, CAPL>(lst_d, lst_i, cnt, tau, p.share ? gtq : nullptr, qw0, lane);
                ovf = false;
                static_for<N>([&](auto NN) {
                    constexpr int n = decltype(NN)::value;
                    const float tq = qv[n] ? fminf(tau[qloc[n]], tn[n]) : -FX_INF;
                    const unsigned pn = pend[n];
                    pend[n] = 0u;
                    static_for<M>([&](auto MM) {
                        constexpr int m = decltype(MM)::value;
                        const unsigned el = (pn >> (4 * m)) & 15u;
                        if (__builtin_amdgcn_ballot_w64(el != 0u))
                            ovf |= wpush<M, N, CAPL>(acc, n, m, el, tq, qloc[n], trow0 + rl0 + m * 16, rlim, lst_d,
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

    // retire the ring's look-ahead pieces: an LDS-DMA still in flight at exit
    // would land in the LDS of the next workgroup on this CU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // final flush: sorted top-KP per query of this (wide tile, split), into the
    // [qtile128][split][128][KP] candidate layout
    for (int qi = 0; qi < QW; ++qi) {
        const int q = qw0 + qi;
        const int64_t gq = q0 + q;
        if (gq >= p.nq) break;
        const int cn = min(cnt[q], CAPL);
        float d = lane < cn ? lst_d[q * CAPL + lane] : FX_INF;
        int i = lane < cn ? lst_i[q * CAPL + lane] : INT_MAX;
        sort64(d, i, lane);
        if (lane < KP) {
            const int64_t o = ((gq / TILE_Q * p.splits + split) * TILE_Q + gq % TILE_Q) * KP + lane;
            p.cand_d[o] = d;
            p.cand_i[o] = i == INT_MAX ? -1 : i;
        }
    }
}

// stage bytes: 16 KiB stages of TR = 64 rows -> 256 B of K; narrower rows (or
// an F32S plane that is not a multiple of 256 B) would leave fewer than NS - 1
// stages per tile, so they stay on k_scan_v4
template <int DT, int METRIC, int KSTEPS>
static hipError_t scan_w_t(const ScanParams& p, hipStream_t s) {
    constexpr int M = 4, N = 3, SB = 256, NS = 4, CAPL = 60;
    typedef WLayout<M, N, NS, CAPL> L;
    hipError_t e = g_graph_capture ? hipSuccess
                                   : hipFuncSetAttribute((const void*)k_scan_w<DT, METRIC, KSTEPS, M, N, SB, NS, CAPL>,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, L::BYTES);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_scan_w<DT, METRIC, KSTEPS, M, N, SB, NS, CAPL>), dim3(p.grid), dim3(SCAN_THREADS), L::BYTES,
                       s, p);
    return hipGetLastError();
}

int scan_w_queries() { return 4 * 16 * 3; }

bool scan_w_supported(int st_dt, int row_bytes) {
    if (st_dt != BF16 && st_dt != F16 && st_dt != F32S) return false;
    if (row_bytes % 64 != 0) return false;
    const int ks = row_bytes / 64;
    if (st_dt == F32S) return ks == 16 || ks == 24;  // planes of 512 / 768 B
    return ks == 12 || ks == 16 || ks == 24;         // >= 3 stages of 256 B per row
}

template <int DT, int METRIC>
static hipError_t scan_w_rows(const ScanParams& p, hipStream_t s) {
    switch (p.row_bytes / 64) {
        case 12: if constexpr (DT != F32S) return scan_w_t<DT, METRIC, 12>(p, s); else break;
        case 16: return scan_w_t<DT, METRIC, 16>(p, s);
        case 24: return scan_w_t<DT, METRIC, 24>(p, s);
        default: break;
    }
    return hipErrorInvalidValue;
}

hipError_t launch_scan_w(int st_dt, int metric, const ScanParams& p, hipStream_t s) {
    if (!scan_w_supported(st_dt, p.row_bytes)) return hipErrorInvalidValue;
    if (st_dt == F32S) return metric == L2 ? scan_w_rows<F32S, L2>(p, s) : scan_w_rows<F32S, IP>(p, s);
    if (st_dt == BF16) return metric == L2 ? scan_w_rows<BF16, L2>(p, s) : scan_w_rows<BF16, IP>(p, s);
    return metric == L2 ? scan_w_rows<F16, L2>(p, s) : scan_w_rows<F16, IP>(p, s);
}

}  // namespace fx
