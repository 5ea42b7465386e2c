// fx_scan5.hip -- k_scan_v5: the search() scan with 64-row corpus tiles and
// NB x 16 stationary queries per wave: NB = 4 (64 queries per wave, 256 per
// workgroup) for 16-bit rows of <= 768 B (d <= 384: config (e)), NB = 3 (48
// per wave, 192 per workgroup) for 1,536-B rows (d = 768: config (d)).
//
// Same algorithm and the same per-split top-KP lists as k_scan_v4
// (fx_scan.hip: the fused MFMA distance GEMM, the LDS-DMA ring, the shared
// thresholds and the union bound; every result is certified the same way
// by k_refine), in a shape that moves half the bytes per MFMA:
//
//   * a wave's accumulator tile is 64 rows x 64 queries (k_scan_v4: 128 x
//     32; both 64 registers), so each A fragment read from LDS feeds four
//     MFMAs instead of two: LDS read bytes per MFMA halve;
//   * a workgroup consumes 64 corpus rows per tile for 256 queries: L2->LDS
//     bytes and LDS-DMA pieces per MFMA halve (two 1 KiB pieces per wave per
//     stage instead of four), and at nq <= 256 one workgroup streams a split
//     once for the whole batch (the mid-batch case of DESIGN.md §8 item 3);
//   * the per-query lists hold LC = 48 entries (256 lists must fit the LDS
//     beside the ring: 96 KiB of lists + a 40 KiB ring).
//
// The B operand takes 4 NB registers per K-step: 192 AGPRs for NB = 4 at
// K = 384 (KSTEPS = 12) -- k_scan_v4's 32 queries at K = 768 take as many --
// and 288 for NB = 3 at K = 768, so the third block's upper K-steps live in
// VGPRs (ODD_KA).  At NB = 3 the ratios are two thirds of k_scan_v4's (an A
// fragment feeds three MFMAs; 192 queries per 64-row tile).
#include "fx_scan_common.h"

namespace fx {
namespace v5 {

// A/B switches (make v5variant): ring slots, the MFMA row after which a
// half-stage issues its corpus piece, the odd block's AGPR K-steps, the list
// capacity of the 3-block instance
#ifndef FX_V5_NS3
#define FX_V5_NS3 6
#endif
#ifndef FX_V5_PIECE_M
#define FX_V5_PIECE_M 2
#endif
#ifndef FX_V5_ODD_KA
#define FX_V5_ODD_KA 14
#endif
#ifndef FX_V5_LC3
#define FX_V5_LC3 48
#endif
#ifndef FX_V5_NS4
#define FX_V5_NS4 5
#endif
#ifndef FX_V5_LC4
#define FX_V5_LC4 48
#endif

constexpr int TR = 64;                 // corpus rows per tile
constexpr int M = TR / 16;             // 16-row fragments per tile
constexpr int S_STAGE = TR * STAGE_B;  // 8 KiB: 64 rows x 128 B of K
constexpr int PPS = S_STAGE / 1024 / 4;  // corpus pieces per wave per stage (2)
// ring slots (NS - 1 stages in flight; the ring must not reach past the next
// tile): the 3-block instance has the LDS for FX_V5_NS3 slots with 48-entry
// lists (same box, profiles/r6/ab_v5_variants_*_r6k.txt: 6 slots (d) -1.2 %,
// the N = 8 shard -0.5 % against 5 slots with 64-entry lists); the 4-block
// instance's 256 lists leave room for 5
template <int KSTEPS, int NB>
constexpr int ns_for() {
    return NB == 3 && FX_V5_NS3 - 1 <= KSTEPS / 2   ? FX_V5_NS3
           : NB == 4 && FX_V5_NS4 - 1 <= KSTEPS / 2 ? FX_V5_NS4
                                                   : 5;
}
// VMEM operations issued after stage g+1's at the wait of stage j (a tile's
// stage): PPS corpus pieces per stage for stages g+2 .. g+NS-2, plus the norm
// piece of every tile's first stage among them
template <int NS, int SPT>
constexpr int younger(int j) {
    int w = PPS * (NS - 3);
    for (int d = 2; d <= NS - 2; ++d) w += (j + d) % SPT == 0;
    return w;
}

template <int NB, int LC, int NS = 5>
struct Lds {
    static constexpr int QW = 16 * NB;                             // queries per wave
    static constexpr int QT = 4 * QW;                              // per workgroup
    static constexpr int NSLOT = 64 + 4 * QW <= 256 ? 256 : 512;   // per wave: [16 row norms | QW thresholds]
    static constexpr int NORM_OFF = 0;                             // 4 tile slots x 4 waves x NSLOT
    static constexpr int RING_OFF = NORM_OFF + 4 * 4 * NSLOT;      // >= 4 KiB (dma_piece's M0 rule)
    static constexpr int UNION_OFF = RING_OFF + NS * S_STAGE;      // [4 waves][2 slots][256 keys]
    static constexpr int LST = 2 * LC;                             // list stride (words): LC keys | LC rows
    static constexpr int LST_OFF = UNION_OFF + 4 * 2 * 1024;
    static constexpr int TRASH_OFF = LST_OFF + QT * LST * 4;       // [4 waves][64 keys | 64 rows]
    static constexpr int BYTES = TRASH_OFF + 4 * 2 * 256;
    static_assert(RING_OFF >= 4096, "ring pieces need LDS offsets >= 4 KiB");
    static_assert(BYTES <= 160 * 1024, "LDS budget");
};

// a value of a per-n register array at a wave-uniform index (no dynamic
// register indexing: that would go to scratch)
template <int NB, typename T>
__device__ __forceinline__ T pick(const T (&a)[NB], int n) {
    T v = a[0];
    static_for<NB>([&](auto I) {
        if (decltype(I)::value == n) v = a[decltype(I)::value];
    });
    return v;
}

template <int NB>
struct ListRegs {
    int cnt[NB];
    float tau[NB];
};

// one (key, row) entry: ONE ds_write2_b32 (rows LC words after the keys)
template <int LC>
__device__ __forceinline__ void wr_entry(uint32_t off, float key, int row) {
    asm volatile("ds_write2_b32 %0, %1, %2 offset1:%3" ::"v"(off), "v"(key), "v"(row), "i"(LC) : "memory");
}

// fx_scan_common.h push_group with the list capacity LC
template <bool RETRY, int LC>
__device__ __forceinline__ unsigned push_group(const f32x4& a, unsigned elig, float tn, int row0, uint32_t lq,
                                               uint32_t trash, int& cntv, int lane) {
    bool p[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = (!RETRY || ((elig >> i) & 1u)) && a[i] <= tn;
    const int c = (int)p[0] + (int)p[1] + (int)p[2] + (int)p[3];
    int excl, total;
    quad_prefix(c, lane, excl, total);
    const int s = cntv + excl;
    cntv += total;
    unsigned late = 0u;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(s + c > LC) == 0, 1)) {
        uint32_t e = lq + (uint32_t)s * 4u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            wr_entry<LC>(p[i] ? e : trash, a[i], row0 + i);
            e += p[i] ? 4u : 0u;
        }
    } else {
        int slot = s;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool ok = p[i] && slot < LC;
            wr_entry<LC>(ok ? lq + (uint32_t)slot * 4u : trash, a[i], row0 + i);
            late |= (p[i] && !ok) ? (1u << i) : 0u;
            slot += (int)p[i];
        }
    }
    return late;
}

// fx_scan_common.h union_finish for NB query blocks
template <int NB>
__device__ __forceinline__ void union_finish(int (&upq)[2], const float* uslot, const ListRegs<NB>& r, unsigned* gtq,
                                             int splits, int split, int rank, int uw, int lane) {
    const int le = union_le(uw);
    const int w0 = split & ~(uw - 1);
    const int nsp = splits - w0 < uw ? splits - w0 : uw;
    const bool in_win = (lane >> (le - 2)) < nsp;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if (upq[u] < 0) continue;
        const int qi = upq[u];
        const f32x4 raw = *(const f32x4*)(uslot + u * 256 + lane * 4);
        unsigned kv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) kv[j] = in_win ? f2ord(raw[j]) : 0xFFFFFFFFu;
        const unsigned own = f2ord(readlane_f(pick<NB>(r.tau, qi >> 4), qi & 15));
        const unsigned v = union_kth_v(kv, own, rank);
        if (lane == 0 && v < own) gmin_u32(gtq + qi, v);
        upq[u] = -1;
    }
}

// fx_scan_common.h compact_regs for NB query blocks and lists of LC entries:
// every list of this wave holding `at` or more entries is sorted (packed
// 64-bit bitonic) and cut to its KP best; its threshold becomes its rank-th
// key, published to the shared threshold and (pub) to the split's published
// list; then the union bounds (deferred into the two LDS slots, or in place
// for at most inplace_max lists), exactly as k_scan_v4's.
template <int NB, int LC>
__device__ __forceinline__ ListRegs<NB> compact_regs(float* lst, ListRegs<NB> r, unsigned* gtq, int qw0, int lane,
                                                  float* pub, int splits, int split, int rank, int at, int uw,
                                                  int (&upq)[2], float* uslot, int defer, int inplace_max) {
    constexpr int LST = 2 * LC;
    float* lst_d = lst;
    int* lst_i = (int*)(lst + LC);
    uint64_t all = 0;
    static_for<NB>([&](auto N) {
        constexpr int n = decltype(N)::value;
        all |= (__builtin_amdgcn_ballot_w64(lane < 16 && r.cnt[n] >= at) & 0xffffull) << (16 * n);
    });
    uint64_t full = all;
    while (full) {
        const int qi = __builtin_ctzll(full);
        full &= full - 1;
        const int q = qw0 + qi;
        const int cq = __builtin_amdgcn_readlane(pick<NB>(r.cnt, qi >> 4), qi & 15);
        const bool live = lane < cq && lane < LC;
        uint32_t hi, lo;
        load_packed(lst_d, lst_i, q * LST + lane, live, hi, lo);
        sort64_packed(hi, lo, lane);
        const float d = ord2f(hi);
        const int i = (int)lo;
        if (lane < KP) {
            lst_d[q * LST + lane] = d;
            lst_i[q * LST + lane] = i;
        }
        const float dr = readlane_f(d, rank - 1);
        static_for<NB>([&](auto N) {
            constexpr int n = decltype(N)::value;
            if ((qi >> 4) == n && (lane & 15) == (qi & 15)) {
                r.tau[n] = dr;
                r.cnt[n] = KP;
            }
        });
        if (gtq && lane == 0) gmin_u32(gtq + qi, f2ord(dr));
        if (pub && gtq && lane < KP)
            __hip_atomic_store((gfloat*)(pub + ((int64_t)qi * splits + split) * KP + lane), d, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!(pub && gtq)) return r;
    const int le = union_le(uw);
    const int w0 = split & ~(uw - 1);
    const int nsp = splits - w0 < uw ? splits - w0 : uw;
    uint64_t rest = all;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if (rest == 0 || upq[u] >= 0 || !defer) continue;
        const int qi = __builtin_ctzll(rest);
        rest &= rest - 1;
        const int l = lane >> (le - 2), e4 = lane & ((1 << (le - 2)) - 1);
        const char* wb = sgpr_ptr((const char*)(pub + ((int64_t)qi * splits + w0) * KP));
        const uint32_t voff = (uint32_t)(((l < nsp ? l : 0) * KP + 4 * e4) * 4);
        dma_piece<0, 4>(voff, wb, lds_off(uslot + u * 256));  // s_nop 4: wb was written by VALU
        upq[u] = qi;
    }
    for (int done = 0; rest && done < inplace_max; done += 4) {
        int qs[4];
        unsigned kv[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool take = rest != 0 && done + u < inplace_max;
            qs[u] = take ? __builtin_ctzll(rest) : -1;
            if (take) rest &= rest - 1;
        }
        float raw[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const gfloat* lists = (const gfloat*)(pub + ((int64_t)(qs[u] < 0 ? 0 : qs[u]) * splits + w0) * KP);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int x = lane + 64 * j, l = x >> le, e = x & ((1 << le) - 1);
                raw[u][j] = __hip_atomic_load(lists + (l < nsp ? l : 0) * KP + e, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                kv[u][j] = (qs[u] >= 0 && ((lane + 64 * j) >> le) < nsp) ? f2ord(raw[u][j]) : 0xFFFFFFFFu;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (qs[u] < 0) break;
            const int qi = qs[u];
            const unsigned own = f2ord(readlane_f(pick<NB>(r.tau, qi >> 4), qi & 15));
            const unsigned v = union_kth_v(kv[u], own, rank);
            if (lane == 0 && v < own) gmin_u32(gtq + qi, v);
        }
    }
    return r;
}

// the per-stage row-norm / threshold piece of a wave: lanes 0-3 move its 16
// row norms, lanes 4 .. 4 + QW/4 - 1 its QW shared thresholds
template <int LANES>
__device__ __forceinline__ void dma_norm_piece(const char* vaddr, uint32_t m0) {
    constexpr uint64_t EXEC = (1ull << LANES) - 1;
    uint64_t saved;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "v"(vaddr), "{m0}"(m0), "i"(EXEC)
        : "memory");
}

__device__ __forceinline__ float min4_raw(float a, float b, float c, float d) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3\n\tv_min_f32 %0, %0, %4" : "=&v"(r) : "v"(a), "v"(b), "v"(c), "v"(d));
    return r;
}

// K-steps of the odd query block whose B fragments sit in AGPRs (the rest in
// VGPRs): 192 + 4 KA <= 256 AGPRs
constexpr int ODD_KA = FX_V5_ODD_KA;

// MFMAs of one A fragment against NB query blocks (pairs through
// AsmMmaV::mma2: B pinned in AGPRs; an odd last block through mma1)
template <int DT, int INIT, int NB, int KS>
__device__ __forceinline__ void mma_row(f32x4 (&acc)[NB], const typename AsmMmaV<DT>::A& a,
                                        const typename AsmMmaV<DT>::B (&b)[NB], const f32x4& ci) {
    static_for<NB / 2>([&](auto P) {
        constexpr int n = 2 * decltype(P)::value;
        AsmMmaV<DT>::template mma2<INIT>(acc[n], acc[n + 1], a, b[n], b[n + 1], ci);
    });
    if constexpr (NB % 2) mma1<DT, INIT, (KS < ODD_KA)>(acc[NB - 1], a, b[NB - 1], ci);
}

constexpr int RESCAN = 4096;  // (kernel name of the re-scan's instance, as in fx_scan.hip)

template <int DT, int METRIC, int KSTEPS, int NB, int LC, int ABL = 0>
__global__ __launch_bounds__(SCAN_THREADS, 1) void k_scan_v5(ScanParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename AsmMmaV<DT>::A frag_t;
    typedef typename AsmMmaV<DT>::B bfrag_t;
    constexpr int NS = ns_for<KSTEPS, NB>();
    typedef Lds<NB, LC, NS> L;
    constexpr int QW = L::QW, QT = L::QT, NSLOT = L::NSLOT, LST = L::LST;
    constexpr int SPT = KSTEPS / 2;  // stages per tile
    constexpr int RB = KSTEPS * 64;  // row stride in bytes
    constexpr int64_t TILE_BYTES = (int64_t)TR * RB;
    static_assert(SPT >= NS - 1, "prefetch distance must stay within the next tile");
    static_assert(LC > KP && LC <= 64, "list capacity");

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int qtile, split;
    map_block(blockIdx.x, p, qtile, split);
    const int64_t nq = p.nq_dev ? min((int64_t)*p.nq_dev, p.nq) : p.nq;
    if (qtile >= p.n_qtiles || (int64_t)qtile * QT >= nq) return;
    const int ct0 = (int)((int64_t)split * p.n_ctiles / p.splits);
    const int ct1 = (int)((int64_t)(split + 1) * p.n_ctiles / p.splits);
    const int ntiles = ct1 - ct0;
    const int64_t q0 = (int64_t)qtile * QT;
    if (p.trace && tid == 0) trace_block_start(p, qtile, split);

    float* lst = (float*)(smem + L::LST_OFF);
    const int qw0 = wave * QW;
    const uint32_t ld_off = lds_off(lst);
    const uint32_t trash = lds_off(smem + L::TRASH_OFF) + (uint32_t)(wave * 512 + lane * 4);
    float* uslot = (float*)(smem + L::UNION_OFF) + wave * 512;
    int upq[2] = {-1, -1};
    ListRegs<NB> lr;
#pragma unroll
    for (int n = 0; n < NB; ++n) {
        lr.cnt[n] = 0;
        lr.tau[n] = KEY_MAX;
    }
    unsigned* gtq = p.gtau + q0 + qw0;
    float* pubw = p.pub ? p.pub + (q0 + qw0) * p.splits * KP : nullptr;

    // queries -> AGPRs (B fragments)
    bfrag_t b[KSTEPS][NB];
    {
        const char* qb = p.qop + (q0 + qw0 + (lane & 15)) * RB + (lane >> 4) * 16;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
            for (int n = 0; n < NB; ++n) b[ks][n] = *(const bfrag_t*)(qb + n * 16 * RB + ks * 64);
        static_for<KSTEPS>([&](auto KS) {
            constexpr int ks = decltype(KS)::value;
            static_for<NB>([&](auto N) {
                constexpr int n = decltype(N)::value;
                if constexpr (NB % 2 && n == NB - 1 && ks >= ODD_KA) asm volatile("" ::"v"(b[ks][n]));
                else AsmMmaV<DT>::settle(b[ks][n]);
            });
        });
    }

    // ---- DMA addressing: piece w of a wave = rows 16 wave + 8 w .. +7 of the
    // stage (full 128-B lines), lane l -> row + (l >> 3), source chunk
    // (l & 7) ^ (l >> 3) (the row-linear, chunk-swizzled image of k_scan_v4 LN = 1)
    const uint32_t voffA = (uint32_t)((16 * wave + (lane >> 3)) * RB + (((lane & 7) ^ (lane >> 3)) << 4));
    const uint32_t lds_base = lds_off(smem);
    const uint32_t m0w = lds_base + L::RING_OFF + wave * (S_STAGE / 4);
    const uint32_t nslot_w = lds_base + L::NORM_OFF + wave * NSLOT;
    // convoy start: the split-relative tile another block of this split
    // published last (any value is a valid start: the block scans its
    // ntiles tiles circularly from it; results do not depend on the order).
    // Read ONCE per block and passed to the other waves through LDS (the list
    // area, not yet in use): every wave DMAs its own pieces of each shared
    // stage, so waves that each read the word -- and saw a store land between
    // their reads -- would fill one stage from two tiles (caught by
    // test_v5_clustered_certifies: rows of one split missing)
    int rel = 0;
    if (p.conv && ntiles > 1) {
        unsigned* bc = (unsigned*)(smem + L::LST_OFF);
        if (tid == 0)
            *bc = __hip_atomic_load((const guint*)(p.conv + (int64_t)split * 16), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        rel = __builtin_amdgcn_readfirstlane((int)(*bc % (unsigned)ntiles));
    }
    const char* cb_split = p.codes + (int64_t)ct0 * TILE_BYTES;
    const int rel1 = rel + 1 == ntiles ? 0 : rel + 1;
    const char* cb_cur = sgpr_ptr(cb_split + (int64_t)rel * TILE_BYTES);
    const char* cb_nxt = sgpr_ptr(ntiles > 1 ? cb_split + (int64_t)rel1 * TILE_BYTES : cb_cur);
    constexpr int NLANES = 4 + QW / 4;  // norm-piece lanes
    const int nstep = lane < 4 ? TR * 4 : 0;
    const char* nv_split = lane < 4 ? (const char*)(p.norms + (int64_t)ct0 * TR + 16 * wave + lane * 4)
                                    : (const char*)(gtq + ((lane - 4) % (QW / 4)) * 4);
    const char* nv_cur = nv_split + (int64_t)rel * nstep;
    const char* nv_nxt = ntiles > 1 ? nv_split + (int64_t)rel1 * nstep : nv_cur;

    auto piece = [&](auto W, auto JP, auto NXT, uint32_t slot, int tnext) {
        constexpr int w = decltype(W)::value, jp = decltype(JP)::value;
        const char* cb = decltype(NXT)::value ? cb_nxt : cb_cur;
        if constexpr (w < PPS) {
            dma_piece<jp * STAGE_B>(voffA, cb + w * 8 * RB, m0w + slot * S_STAGE + w * 1024);
        } else {
            dma_norm_piece<NLANES>(decltype(NXT)::value ? nv_nxt : nv_cur,
                                   nslot_w + (uint32_t)(tnext & 3) * (4 * NSLOT));
        }
    };

    // prologue: stages 0 .. NS-2 (all in tile 0)
    static_for<NS - 1>([&](auto ST) {
        constexpr int st = decltype(ST)::value;
        static_for<PPS>([&](auto W) { piece(W, ST, std::false_type{}, (uint32_t)st, 0); });
        if constexpr (st == 0) piece(std::integral_constant<int, PPS>{}, ST, std::false_type{}, 0u, 0);
        (void)st;
    });

    f32x4 acc[M][NB];
    frag_t X[M], Y[M];
    f32x4 yin[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
#pragma unroll
        for (int n = 0; n < NB; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        yin[m] = f32x4{0.f, 0.f, 0.f, 0.f};
        X[m] = Y[m] = frag_t{};
    }
    const int rl0 = 4 * (lane >> 4);
    int qloc[NB];
    bool qv[NB];
    uint64_t qm[NB];
    uint32_t lq[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
        qloc[n] = qw0 + n * 16 + (lane & 15);
        qv[n] = q0 + qloc[n] < nq;
        qm[n] = __builtin_amdgcn_ballot_w64(qv[n]);
        lq[n] = ld_off + (uint32_t)(qloc[n] * LST * 4);
    }
    const uint32_t gt_lane = (uint32_t)(64 + (lane & 15) * 4);
    const uint32_t nrm_lane = (uint32_t)(rl0 * 4);

    // stage 0 landed; younger are stages 1 .. NS-2
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(PPS * (NS - 2)) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t rd_lane = (uint32_t)((lane & 15) * 128 + ((((lane >> 4)) ^ (lane & 7)) << 4));
    const uint32_t rd_h1 = (uint32_t)((lane & 15) * 128 + ((((lane >> 4) + 4) ^ (lane & 7)) << 4)) - rd_lane;
    uint32_t rd_addr = lds_base + L::RING_OFF + rd_lane;  // slot 0
    if (ntiles > 0) {
        static_for<M>([&](auto MM) {
            constexpr int m = decltype(MM)::value;
            ds_rd128<m * 2048>(X[m], rd_addr);
        });
        // row norms of tile 0: rows 16 m + rl0 .. +3 are in wave m's norm slot
        const uint32_t na = lds_base + L::NORM_OFF + nrm_lane;
        static_for<M>([&](auto MM) {
            constexpr int m = decltype(MM)::value;
            ds_rd128<m * NSLOT>(yin[m], na);
        });
    }

    int c = 0;  // ring slot of the current stage
    for (int t = 0; t < ntiles; ++t) {
        unsigned gr[NB];
        static_for<SPT>([&](auto JJ) {
            constexpr int j = decltype(JJ)::value;
            constexpr bool LAST = j == SPT - 1;
            constexpr int jp = (j + NS - 1) % SPT;
            constexpr bool nxt = j + NS - 1 >= SPT;
            typedef std::integral_constant<bool, nxt> NXT;
            typedef std::integral_constant<int, jp> JP;
            const uint32_t c1 = c == NS - 1 ? 0u : (uint32_t)c + 1;
            const uint32_t c4 = c == 0 ? (uint32_t)NS - 1 : (uint32_t)c - 1;
            const int tnext = t + (nxt ? 1 : 0);
            // VMEM ops younger than stage g+1's: stages g+2 .. g+NS-2 (PPS
            // corpus pieces each, + the norm piece with a tile's first stage)
            constexpr int W = younger<NS, SPT>(j);
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(W) : "memory");
            __builtin_amdgcn_sched_barrier(0);
            constexpr int kq0 = 2 * j;
            // ---- half 0: X MFMAs; read half 1 (Y) of this stage meanwhile
            static_for<M>([&](auto MM) {
                constexpr int m = decltype(MM)::value;
                constexpr int INIT = j == 0 ? (METRIC == L2 ? 1 : 2) : 0;
                mma_row<DT, INIT, NB, kq0>(acc[m], X[m], b[kq0], yin[m]);
                if constexpr (m < M / 2) {
                    const uint32_t rd1 = rd_addr + rd_h1;
                    ds_rd128<(2 * m) * 2048>(Y[2 * m], rd1);
                    ds_rd128<(2 * m + 1) * 2048>(Y[2 * m + 1], rd1);
                }
                if constexpr (LAST && m >= M / 2) {
                    // the next tile's row norms (its first MFMAs' srcC)
                    const uint32_t na = lds_base + L::NORM_OFF + (uint32_t)((t + 1) & 3) * (4 * NSLOT) + nrm_lane;
                    constexpr int m0 = 2 * (m - M / 2), m1 = m0 + 1;
                    ds_rd128<m0 * NSLOT>(yin[m0], na);
                    ds_rd128<m1 * NSLOT>(yin[m1], na);
                }
                if constexpr (m == FX_V5_PIECE_M) piece(std::integral_constant<int, 0>{}, JP{}, NXT{}, c4, tnext);
            });
            if constexpr (LAST) {
                // epilogue operands of this tile: the queries' shared thresholds
                const uint32_t ns = lds_base + L::NORM_OFF + (uint32_t)(t & 3) * (4 * NSLOT) + wave * NSLOT + gt_lane;
                static_for<NB>([&](auto N) {
                    constexpr int n = decltype(N)::value;
                    ds_rd32<64 * n>(gr[n], ns);
                });
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            // ---- half 1: Y MFMAs; read half 0 (X) of stage g+1 meanwhile
            const uint32_t rd_next = lds_base + L::RING_OFF + c1 * S_STAGE + rd_lane;
            static_for<M>([&](auto MM) {
                constexpr int m = decltype(MM)::value;
                mma_row<DT, 0, NB, kq0 + 1>(acc[m], Y[m], b[kq0 + 1], yin[m]);
                if constexpr (m < M / 2) {
                    ds_rd128<(2 * m) * 2048>(X[2 * m], rd_next);
                    ds_rd128<(2 * m + 1) * 2048>(X[2 * m + 1], rd_next);
                }
                if constexpr (m == FX_V5_PIECE_M) piece(std::integral_constant<int, 1>{}, JP{}, NXT{}, c4, tnext);
                if constexpr (m == 3 && jp == 0) piece(std::integral_constant<int, PPS>{}, JP{}, NXT{}, c4, tnext);
            });
            __builtin_amdgcn_sched_barrier(0);
            rd_addr = rd_next;
            c = (int)c1;
        });

        // ---- epilogue of tile t: the accumulator holds the keys ------------
        float gmin[NB][M];
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int n = 0; n < NB; ++n) gmin[n][m] = min4(acc[m][n]);
        // (the thresholds as operands: no use of them is scheduled above the wait)
        if constexpr (NB == 4)
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(gr[0]), "+v"(gr[1]), "+v"(gr[2]), "+v"(gr[3])::"memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(gr[0]), "+v"(gr[1]), "+v"(gr[NB - 1])::"memory");
        float tn[NB], mn[NB];
#pragma unroll
        for (int n = 0; n < NB; ++n) {
            tn[n] = __builtin_bit_cast(float, sel_mask(qm[n], __builtin_bit_cast(uint32_t, -FX_INF),
                                                       __builtin_bit_cast(uint32_t, min_raw(lr.tau[n], ord2f(gr[n])))));
            mn[n] = min4_raw(gmin[n][0], gmin[n][1], gmin[n][2], gmin[n][3]);
        }
        if (__builtin_expect(upq[0] >= 0 || upq[1] >= 0, 0))
            union_finish<NB>(upq, uslot, lr, gtq, p.splits, split, p.prune_rank, p.union_w, lane);
        bool any = false;
#pragma unroll
        for (int n = 0; n < NB; ++n) any |= mn[n] <= tn[n];
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(any) != 0, 0)) {
            // slow path: some row beats a query's threshold
            const int trow0 = (ct0 + rel) * TR;
            // the index's last tile: rows past ntotal get key +inf (and the
            // group minima are re-taken: the cold-start bound counts them)
            if (__builtin_expect((int64_t)trow0 + TR > p.ntotal, 0)) {
                const int lim = (int)(p.ntotal - trow0);
#pragma unroll
                for (int m = 0; m < M; ++m)
#pragma unroll
                    for (int n = 0; n < NB; ++n) {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if (rl0 + 16 * m + i >= lim) acc[m][n][i] = FX_INF;
                        gmin[n][m] = min4(acc[m][n]);
                    }
#pragma unroll
                for (int n = 0; n < NB; ++n) mn[n] = min4_raw(gmin[n][0], gmin[n][1], gmin[n][2], gmin[n][3]);
            }
            if (p.cold_bound) {
                // an empty list's first record tile: its threshold bounded by
                // the max over the query's 4 lanes of each lane's c-th smallest
                // group minimum (4 c >= rank distinct rows at or below it),
                // published like a compaction's bound (fx_scan.hip)
                const int cc = (p.prune_rank + 3) >> 2;
                static_for<NB>([&](auto NN) {
                    constexpr int n = decltype(NN)::value;
                    if (cc <= 4 && __builtin_amdgcn_ballot_w64(qv[n] && lr.cnt[n] == 0 && mn[n] <= tn[n])) {
                        float a1 = FX_INF, a2 = FX_INF, a3 = FX_INF, a4 = FX_INF;
#pragma unroll
                        for (int m = 0; m < M; ++m) {
                            const float x = gmin[n][m];
                            a4 = __builtin_amdgcn_fmed3f(a3, x, a4);
                            a3 = __builtin_amdgcn_fmed3f(a2, x, a3);
                            a2 = __builtin_amdgcn_fmed3f(a1, x, a2);
                            a1 = fminf(a1, x);
                        }
                        float bb = cc <= 1 ? a1 : cc == 2 ? a2 : cc == 3 ? a3 : a4;
                        bb = fmaxf(bb, lane_xor<16>(bb, lane));
                        bb = fmaxf(bb, lane_xor<32>(bb, lane));
                        if (qv[n] && lr.cnt[n] == 0) {
                            tn[n] = fminf(tn[n], bb);
                            if (lane < 16 && bb < lr.tau[n]) gmin_u32(gtq + 16 * n + lane, f2ord(bb));
                            lr.tau[n] = fminf(lr.tau[n], bb);
                        }
                    }
                });
            }
            int rb = trow0 + rl0;
            unsigned pend[NB];
            unsigned ovf = 0u;
            static_for<NB>([&](auto NN) {
                constexpr int n = decltype(NN)::value;
                pend[n] = 0u;
                if (__builtin_amdgcn_ballot_w64(mn[n] <= tn[n])) {
                    static_for<M>([&](auto MM) {
                        constexpr int m = decltype(MM)::value;
                        if (__builtin_amdgcn_ballot_w64(gmin[n][m] <= tn[n])) {
                            const unsigned late =
                                push_group<false, LC>(acc[m][n], 15u, tn[n], rb + 16 * m, lq[n], trash, lr.cnt[n], lane);
                            pend[n] |= late << (4 * m);
                            ovf |= late;
                        }
                    });
                }
            });
            const int cat = min(p.compact_at, LC);
            bool need = ovf != 0u;
#pragma unroll
            for (int n = 0; n < NB; ++n) need |= lr.cnt[n] >= cat;
            while (__builtin_expect(__builtin_amdgcn_ballot_w64(need) != 0, 0)) {
                lr = compact_regs<NB, LC>(lst, lr, p.share ? gtq : nullptr, qw0, lane, p.pub ? pubw : nullptr, p.splits,
                                          split, p.prune_rank, cat, p.union_w, upq, uslot, p.union_defer,
                                          p.union_inplace);
                asm volatile("" : "+v"(rb));
                ovf = 0u;
                static_for<NB>([&](auto NN) {
                    constexpr int n = decltype(NN)::value;
                    const float tq = qv[n] ? fminf(lr.tau[n], tn[n]) : -FX_INF;
                    const unsigned pn = pend[n];
                    pend[n] = 0u;
                    static_for<M>([&](auto MM) {
                        constexpr int m = decltype(MM)::value;
                        const unsigned el = (pn >> (4 * m)) & 15u;
                        if (__builtin_amdgcn_ballot_w64(el != 0u)) {
                            const unsigned late =
                                push_group<true, LC>(acc[m][n], el, tq, rb + 16 * m, lq[n], trash, lr.cnt[n], lane);
                            pend[n] |= late << (4 * m);
                            ovf |= late;
                        }
                    });
                });
                need = ovf != 0u;
            }
        }
        // advance the tile bases (clamped: stages past the end re-read the last tile)
        cb_cur = sgpr_ptr(cb_nxt);
        nv_cur = nv_nxt;
        if (t + 2 < ntiles) {
            int rel2 = rel + 2;
            rel2 -= rel2 >= ntiles ? ntiles : 0;
            cb_nxt = sgpr_ptr(cb_split + (int64_t)rel2 * TILE_BYTES);
            nv_nxt = nv_split + (int64_t)rel2 * nstep;
        }
        rel = rel + 1 == ntiles ? 0 : rel + 1;
        // publish this block's place in the split every conv_every tiles (a
        // global store: counted with the ring's loads in issue order, so the
        // next stage wait at most also waits for one younger piece)
        if (p.conv && (t & (p.conv_every - 1)) == p.conv_every - 1 && wave == 0 && lane == 0)
            __hip_atomic_store((guint*)(p.conv + (int64_t)split * 16), (unsigned)rel, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }

    // retire the ring's look-ahead pieces before the LDS is reused
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // final flush: sorted top-KP per query of this (query tile, split)
    const int64_t obase = ((int64_t)qtile * p.splits + split) * QT;
    float* lst_d = lst;
    const int* lst_i = (const int*)(lst + LC);
    for (int qi = 0; qi < QW; ++qi) {
        const int q = qw0 + qi;
        if (q0 + q >= nq) break;
        const int cq = __builtin_amdgcn_readlane(pick<NB>(lr.cnt, qi >> 4), qi & 15);
        const int cn = min(cq, LC);
        uint32_t hi, lo;
        load_packed(lst_d, lst_i, q * LST + lane, lane < cn, hi, lo);
        sort64_packed(hi, lo, lane);
        const float d = ord2f(hi);
        const int i = (int)lo;
        if (lane < KP) {
            p.cand_d[(obase + q) * KP + lane] = d;
            p.cand_i[(obase + q) * KP + lane] = i == INT_MAX ? -1 : i;
        }
    }
    if (p.trace && tid == 0) p.trace[blockIdx.x * 4 + 3] = wall_clock64();
}

template <int DT, int METRIC, int KSTEPS, int NB, int LC, int ABL>
static hipError_t launch_t(const ScanParams& p, hipStream_t s) {
    constexpr int LDS_BYTES = Lds<NB, LC, ns_for<KSTEPS, NB>()>::BYTES;
    hipError_t e = g_graph_capture ? hipSuccess
                                   : hipFuncSetAttribute((const void*)k_scan_v5<DT, METRIC, KSTEPS, NB, LC, ABL>,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_scan_v5<DT, METRIC, KSTEPS, NB, LC, ABL>), dim3(p.grid), dim3(SCAN_THREADS), LDS_BYTES, s,
                       p);
    return hipGetLastError();
}

template <int DT, int METRIC>
static hipError_t rows(const ScanParams& p, hipStream_t s) {
#ifdef FX_V5_DEV  // kernel-development A/B builds: configs (d) and (e)'s instances only
    if constexpr (DT == BF16 && METRIC == L2)
        if (p.row_bytes == 1536)
            return p.nq_dev ? launch_t<DT, METRIC, 24, 3, FX_V5_LC3, RESCAN>(p, s)
                            : launch_t<DT, METRIC, 24, 3, FX_V5_LC3, 0>(p, s);
    if constexpr (DT == F16 && METRIC == L2)
        if (p.row_bytes == 768)
            return p.nq_dev ? launch_t<DT, METRIC, 12, 4, FX_V5_LC4, RESCAN>(p, s)
                            : launch_t<DT, METRIC, 12, 4, FX_V5_LC4, 0>(p, s);
    return hipErrorInvalidValue;
#else
    // the re-scan of uncertified queries (p.nq_dev set) runs the same code under its own name
    switch (p.row_bytes / 64) {
        case 8:
            return p.nq_dev ? launch_t<DT, METRIC, 8, 4, FX_V5_LC4, RESCAN>(p, s)
                            : launch_t<DT, METRIC, 8, 4, FX_V5_LC4, 0>(p, s);
        case 12:
            return p.nq_dev ? launch_t<DT, METRIC, 12, 4, FX_V5_LC4, RESCAN>(p, s)
                            : launch_t<DT, METRIC, 12, 4, FX_V5_LC4, 0>(p, s);
        case 24:
            return p.nq_dev ? launch_t<DT, METRIC, 24, 3, FX_V5_LC3, RESCAN>(p, s)
                            : launch_t<DT, METRIC, 24, 3, FX_V5_LC3, 0>(p, s);
        default: return hipErrorInvalidValue;
    }
#endif
}

}  // namespace v5

// k_scan_v5's shapes (ScanParams.qt queries per workgroup, 64-row tiles):
// 16-bit rows of 512 or 768 B (d <= 256 / 384): 4 query blocks per wave, 256
// queries; of 1,536 B (d = 768, config (d)): 3 blocks, 192 queries.  0: none.
int scan_v5_qt(int st_dt, int row_bytes) {
    if (st_dt != BF16 && st_dt != F16) return 0;
    if (row_bytes == 512 || row_bytes == 768) return v5::Lds<4, 48>::QT;
    if (row_bytes == 1536) return v5::Lds<3, 64>::QT;
    return 0;
}

hipError_t launch_scan_v5(int st_dt, int metric, const ScanParams& p, hipStream_t s) {
    if (scan_v5_qt(st_dt, p.row_bytes) == 0 || p.qt != scan_v5_qt(st_dt, p.row_bytes) || p.tr != v5::TR)
        return hipErrorInvalidValue;
    if (metric == L2) return st_dt == BF16 ? v5::rows<BF16, L2>(p, s) : v5::rows<F16, L2>(p, s);
    return st_dt == BF16 ? v5::rows<BF16, IP>(p, s) : v5::rows<F16, IP>(p, s);
}

}  // namespace fx
