// fx_kernels.hip -- HIP/CDNA4 (gfx950) kernels of the flat vector index.
//
// Replaces the arithmetic faiss-cpu performs behind IndexFlatL2.add/search
// (faiss_store.py:46,64; rag_datastore_manager.py:173,218):
//
//   k_convert_rows   add(): dtype conversion into the HBM-resident, 128-B
//                    row-aligned code matrix + |y|^2 per row (+ opt-in row
//                    L2 normalisation) -- one wave per row, HBM-bound.
//   k_prep_queries   search(): fp32 copy of the queries for the exact refine,
//                    storage-dtype operand for the MFMA scan, per-query
//                    certification margin.
//   k_scan_topk      search() hot loop: Y.Q^T as an MFMA-tiled GEMM
//                    (128 rows x 128 queries per workgroup tile, both operands
//                    staged global->LDS by global_load_lds, fragment-ordered
//                    LDS images, 16x16x32 bf16/f16 or 16x16x4 f32 MFMA) fused
//                    with a threshold-filtered top-KP select into per-query
//                    LDS candidate lists (no distance matrix ever hits HBM).
//   k_refine         merge the per-split candidate lists, recompute the KP
//                    best candidates' distances exactly (fp64 sum of squared
//                    differences, one rounding to fp32 -- the oracle's
//                    definition), order by (D, id), certify the top-k against
//                    the scan's error bound.
//   k_exact_scan /   fallback for uncertified queries: exact fp64 scan of every
//   k_merge_exact    row, then (D, id) top-k.
//   k_merge_shards   multi-GPU: merge G gathered per-shard top-k lists.
//   k_synth          counter-based synthetic corpus (oracle/flat_l2.c twin).
#include "fx_internal.h"

#include <float.h>
#include <limits.h>
#include <stdlib.h>

namespace fx {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define FX_INF __builtin_inff()

// ---------------------------------------------------------------------------
// scalar conversions
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even, NaN kept NaN
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float h2f(uint16_t h) {
    _Float16 x;
    __builtin_memcpy(&x, &h, 2);
    return (float)x;
}
__device__ __forceinline__ uint16_t f2h(float f) {
    _Float16 x = (_Float16)f;
    uint16_t h;
    __builtin_memcpy(&h, &x, 2);
    return h;
}

__device__ __forceinline__ float load_elem(const void* p, int64_t idx, int dt) {
    if (dt == F32) return ((const float*)p)[idx];
    uint16_t h = ((const uint16_t*)p)[idx];
    return dt == BF16 ? bf2f(h) : h2f(h);
}
// round v to dtype dt and back (the value the index stores)
__device__ __forceinline__ float round_to(float v, int dt) {
    if (dt == F32) return v;
    return dt == BF16 ? bf2f(f2bf(v)) : h2f(f2h(v));
}
__device__ __forceinline__ void store_elem(void* p, int64_t idx, int dt, float v) {
    if (dt == F32) ((float*)p)[idx] = v;
    else ((uint16_t*)p)[idx] = dt == BF16 ? f2bf(v) : f2h(v);
}

// ---------------------------------------------------------------------------
// wave-level (64-lane) bitonic helpers on (key, id) pairs, ascending,
// ties -> smaller id.  Used for LDS list compaction and every merge.
// ---------------------------------------------------------------------------
template <typename Id>
__device__ __forceinline__ bool key_lt(float d1, Id i1, float d2, Id i2) {
    return d1 < d2 || (d1 == d2 && i1 < i2);
}

template <typename Id>
__device__ __forceinline__ void cmpx(float& d, Id& i, int lane, int stride, bool asc) {
    float od = __shfl_xor(d, stride, 64);
    Id oi = __shfl_xor(i, stride, 64);
    bool lower = (lane & stride) == 0;
    bool take = (lower == asc) ? key_lt(od, oi, d, i) : key_lt(d, i, od, oi);
    d = take ? od : d;
    i = take ? oi : i;
}

template <typename Id>
__device__ __forceinline__ void sort64(float& d, Id& i, int lane) {
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) cmpx(d, i, lane, stride, (lane & size) == 0);
    }
}

template <typename Id>
__device__ __forceinline__ void merge64(float& d, Id& i, int lane) {  // bitonic -> ascending
#pragma unroll
    for (int stride = 32; stride > 0; stride >>= 1) cmpx(d, i, lane, stride, true);
}

// best (ascending, one per lane) <- the 64 smallest of best U cand (cand sorted ascending)
template <typename Id>
__device__ __forceinline__ void merge_into(float& bd, Id& bi, float cd, Id ci, int lane) {
    float rd = __shfl(cd, 63 - lane, 64);
    Id ri = __shfl(ci, 63 - lane, 64);
    if (key_lt(rd, ri, bd, bi)) { bd = rd; bi = ri; }
    merge64(bd, bi, lane);
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---------------------------------------------------------------------------
// add(): convert rows into the code matrix, compute |y|^2
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_convert_rows(const void* __restrict__ x, int x_dt, int64_t n, int d,
                                                      void* __restrict__ codes, int st_dt, int kdim,
                                                      float* __restrict__ norms, unsigned* __restrict__ max_sq_bits,
                                                      int normalize) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += nwaves) {
        float scale = 1.0f;
        if (normalize) {
            double s = 0.0;
            for (int c = lane; c < d; c += 64) {
                double v = load_elem(x, r * d + c, x_dt);
                s += v * v;
            }
            s = wave_sum_f64(s);
            scale = s > 0.0 ? (float)(1.0 / sqrt(s)) : 1.0f;
        }
        float sq = 0.0f;
        for (int c = lane; c < kdim; c += 64) {
            float v = c < d ? load_elem(x, r * d + c, x_dt) * scale : 0.0f;
            float st = round_to(v, st_dt);
            store_elem(codes, r * (int64_t)kdim + c, st_dt, st);
            sq = fmaf(st, st, sq);
        }
        sq = wave_sum_f32(sq);
        if (lane == 0) {
            norms[r] = sq;
            atomicMax(max_sq_bits, __float_as_uint(sq));  // positive floats order as uints
        }
    }
}

// ---------------------------------------------------------------------------
// search(): query preparation
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prep_queries(const void* __restrict__ q, int q_dt, int64_t nq,
                                                      int64_t nq_pad, int d, int kdim, int st_dt, int metric,
                                                      float* __restrict__ qf32, void* __restrict__ qop,
                                                      float* __restrict__ qeps, double max_norm, double gamma) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= nq_pad) return;
    const bool live = r < nq;
    double s = 0.0;
    bool inexact = false;
    for (int c = lane; c < kdim; c += 64) {
        float v = (live && c < d) ? load_elem(q, r * d + c, q_dt) : 0.0f;
        qf32[r * (int64_t)kdim + c] = v;
        {
            // scan operand: x rounded to the storage dtype, pre-scaled (exactly,
            // by a power of two) so that the MFMA accumulator is the key:
            // L2: acc = -2 x.y (+ |y|^2 from the accumulator init); IP: -x.y
            const float st = round_to(v, st_dt);
            inexact |= st != v;
            store_elem(qop, r * (int64_t)kdim + c, st_dt, st * (metric == L2 ? -2.0f : -1.0f));
        }
        s += (double)v * (double)v;
    }
    s = wave_sum_f64(s);
    inexact = __any(inexact);
    if (live && lane == 0) {
        // Worst-case bound on |approx - exact| of the scan's key for any row
        // (DESIGN.md "certification"): fp32 fma-chain dot and |y|^2 over K =
        // kdim terms (gamma = K u / (1 - K u)), one more rounding in the key
        // (u), and the query's rounding to the storage dtype (delta).
        const double u = 5.9604644775390625e-8;  // 2^-24
        const double xn = sqrt(s), M = max_norm;
        const double delta = inexact ? (st_dt == BF16 ? 3.90625e-3 : 4.8828125e-4) : 0.0;
        double eps;
        if (metric == L2) eps = (2.0 * gamma + u) * (M * M + 2.0 * xn * M) + 2.0 * delta * xn * M;
        else eps = (gamma + u) * xn * M + delta * xn * M;
        qeps[r] = (float)(eps * 1.0625 + 1e-30);
    }
}

// ---------------------------------------------------------------------------
// the fused scan kernel
// ---------------------------------------------------------------------------
template <int DT> struct Frag;
template <> struct Frag<BF16> {
    typedef bf16x8 T;
    static __device__ __forceinline__ f32x4 mma(T a, T b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};
template <> struct Frag<F16> {
    typedef f16x8 T;
    static __device__ __forceinline__ f32x4 mma(T a, T b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
};
template <> struct Frag<F32> {
    typedef f32x4 T;
    // one 1-KiB fragment block holds 16 rows x 16 k: lane l has row l&15,
    // k = 4(l>>4) .. 4(l>>4)+3.  MFMA step j sums k = 4c+j (c = l>>4): every
    // k is covered exactly once; A and B use the same permutation.
    static __device__ __forceinline__ f32x4 mma(T a, T b, f32x4 c) {
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
        return c;
    }
};

__device__ __forceinline__ void glds16(const void* gsrc, char* lds_uniform) {
    __builtin_amdgcn_global_load_lds(gsrc, (__attribute__((address_space(3))) void*)lds_uniform, 16, 0, 0);
}

// blockIdx -> (query tile, corpus split).  With >= 8 query tiles the grid is
// laid out so that, under the observed round-robin dispatch of blocks over the
// 8 XCDs, each XCD group owns a fixed set of query tiles (their operand stays
// in that XCD's L2) and all groups walk the corpus splits in the same order
// (corpus rows are fetched from HBM about once and re-read from L2/MALL).
// Placement only changes speed, never results.
__device__ __forceinline__ void map_block(int b, const ScanParams& p, int& qtile, int& split) {
    if (p.qt_per_xcd > 0) {
        int xcd = b & 7, j = b >> 3;
        qtile = xcd + 8 * (j % p.qt_per_xcd);
        split = j / p.qt_per_xcd;
    } else {
        qtile = b % p.n_qtiles;
        split = b / p.n_qtiles;
    }
}

// order-preserving float <-> uint (atomicMin on floats of either sign)
__device__ __forceinline__ unsigned f2ord(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// Compact every full list (cnt >= CAP) to its KP best entries; tau = KP-th.
__device__ __forceinline__ void compact_full(float* lst_d, int* lst_i, int* cnt, float* tau, int wave, int lane,
                                             unsigned* gtau = nullptr) {
    for (int q = wave; q < TILE_Q; q += 4) {
        if (cnt[q] >= CAP) {
            float d = lst_d[q * CAP + lane];
            int i = lst_i[q * CAP + lane];
            sort64(d, i, lane);
            if (lane < KP) { lst_d[q * CAP + lane] = d; lst_i[q * CAP + lane] = i; }
            if (lane == KP - 1) {
                tau[q] = d;
                // publish: no split needs keys above the best KP-th of any split
                if (gtau) atomicMin(gtau + q, f2ord(d));
            }
            if (lane == 0) cnt[q] = KP;
        }
    }
}

template <int DT, int METRIC>
__global__ __launch_bounds__(SCAN_THREADS, 1) void k_scan_topk(ScanParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename Frag<DT>::T frag_t;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    int qtile, split;
    map_block(blockIdx.x, p, qtile, split);
    if (qtile >= p.n_qtiles) return;
    const int ct0 = (int)((int64_t)split * p.n_ctiles / p.splits);
    const int ct1 = (int)((int64_t)(split + 1) * p.n_ctiles / p.splits);
    const int nks = p.row_bytes / STAGE_B;
    const int G = (ct1 - ct0) * nks;
    const int64_t q0 = (int64_t)qtile * TILE_Q;
    const int rb = p.row_bytes;

    float* lst_d = (float*)(smem + LDS_LD_OFF);
    int* lst_i = (int*)(smem + LDS_LI_OFF);
    int* cnt = (int*)(smem + LDS_CNT_OFF);
    float* tau = (float*)(smem + LDS_TAU_OFF);
    volatile int* flag = (volatile int*)(smem + LDS_FLAG_OFF);

    for (int x = tid; x < TILE_Q; x += SCAN_THREADS) { cnt[x] = 0; tau[x] = FX_INF; }
    if (tid == 0) *flag = 0;

    // per-lane byte offsets of this wave's 4 A blocks and 4 B blocks inside a
    // tile (fragment-ordered image: block bi = 16-row block * 2 + 64-B half)
    int offs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int bi = wave * 4 + j, rblk = bi >> 1, kb = bi & 1;
        offs[j] = (rblk * 16 + (lane & 15)) * rb + kb * 64 + (lane >> 4) * 16;
    }
    const char* qbase = p.qop + q0 * rb;

    auto issue = [&](int g) {
        const int t = g / nks, ks = g - t * nks;
        char* buf = smem + (g & 1) * ((TILE_R + TILE_Q) * STAGE_B);
        const int64_t row0 = (int64_t)(ct0 + t) * TILE_R;
        const char* abase = p.codes + row0 * rb + ks * STAGE_B;
        const char* bbase = qbase + ks * STAGE_B;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            glds16(abase + offs[j], buf + (wave * 4 + j) * 1024);
            glds16(bbase + offs[j], buf + TILE_R * STAGE_B + (wave * 4 + j) * 1024);
        }
        if (ks == 0 && wave == 0 && lane < 32)
            glds16(p.norms + row0 + lane * 4, smem + LDS_NORM_OFF + (t & 1) * (TILE_R * 4));
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (G > 0) issue(0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");

    int t = 0, ks = 0;
    for (int g = 0; g < G; ++g) {
        if (g + 1 < G) issue(g + 1);
        const char* buf = smem + (g & 1) * ((TILE_R + TILE_Q) * STAGE_B);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            frag_t a[4], b[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) a[m] = *(const frag_t*)(buf + ((wm * 4 + m) * 2 + kb) * 1024 + lane * 16);
#pragma unroll
            for (int n = 0; n < 4; ++n)
                b[n] = *(const frag_t*)(buf + TILE_R * STAGE_B + ((wn * 4 + n) * 2 + kb) * 1024 + lane * 16);
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) acc[m][n] = Frag<DT>::mma(a[m], b[n], acc[m][n]);
        }

        if (ks == nks - 1) {
            // ---------------- epilogue: filter + push into LDS lists ----------
            const float* nb = (const float*)(smem + LDS_NORM_OFF + (t & 1) * (TILE_R * 4));
            const int trow0 = (ct0 + t) * TILE_R;
            const int rlim = (int)(p.ntotal - (int64_t)trow0);  // rows of this tile that exist
            const int rl0 = wm * 64 + 4 * (lane >> 4);           // local row of (m=0, i=0)
            float yn[4][4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                float4 v = *(const float4*)(nb + rl0 + m * 16);
                yn[m][0] = v.x; yn[m][1] = v.y; yn[m][2] = v.z; yn[m][3] = v.w;
            }
            int qloc[4];
            bool qv[4];
            float tn[4];
            unsigned pend[4];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                qloc[n] = wn * 64 + n * 16 + (lane & 15);
                qv[n] = q0 + qloc[n] < p.nq;
                tn[n] = tau[qloc[n]];
                pend[n] = 0u;
            }
            int ovf = 0;
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float v = METRIC == L2 ? acc[m][n][i] + yn[m][i] : acc[m][n][i];
                        const int rl = rl0 + m * 16 + i;
                        if (qv[n] && rl < rlim && v <= tn[n]) {
                            const int s = atomicAdd(&cnt[qloc[n]], 1);
                            if (s < CAP) {
                                lst_d[qloc[n] * CAP + s] = v;
                                lst_i[qloc[n] * CAP + s] = trow0 + rl;
                            } else {
                                pend[n] |= 1u << (m * 4 + i);
                                ovf = 1;
                            }
                        }
                    }
            if (ovf) *flag = 1;
            __syncthreads();
            while (*flag) {
                __syncthreads();
                if (tid == 0) *flag = 0;
                compact_full(lst_d, lst_i, cnt, tau, wave, lane);
                __syncthreads();
                ovf = 0;
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    tn[n] = tau[qloc[n]];
#pragma unroll
                    for (int m = 0; m < 4; ++m)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const unsigned bit = 1u << (m * 4 + i);
                            if (pend[n] & bit) {
                                const float v =
                                    METRIC == L2 ? acc[m][n][i] + yn[m][i] : acc[m][n][i];
                                pend[n] &= ~bit;
                                if (v <= tn[n]) {
                                    const int s = atomicAdd(&cnt[qloc[n]], 1);
                                    if (s < CAP) {
                                        lst_d[qloc[n] * CAP + s] = v;
                                        lst_i[qloc[n] * CAP + s] = trow0 + rl0 + m * 16 + i;
                                    } else {
                                        pend[n] |= bit;
                                        ovf = 1;
                                    }
                                }
                            }
                        }
                }
                if (ovf) *flag = 1;
                __syncthreads();
            }
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
            ks = 0;
            ++t;
        } else {
            ++ks;
        }
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }

    // final flush: sorted top-KP per query of this (query tile, split)
    __syncthreads();
    const int64_t obase = ((int64_t)qtile * p.splits + split) * TILE_Q;
    for (int q = wave; q < TILE_Q; q += 4) {
        if (q0 + q >= p.nq) break;
        const int c = min(cnt[q], CAP);
        float d = lane < c ? lst_d[q * CAP + lane] : FX_INF;
        int i = lane < c ? lst_i[q * CAP + lane] : INT_MAX;
        sort64(d, i, lane);
        if (lane < KP) {
            p.cand_d[(obase + q) * KP + lane] = d;
            p.cand_i[(obase + q) * KP + lane] = i == INT_MAX ? -1 : i;
        }
    }
}

// ---------------------------------------------------------------------------
// scan kernel v2: queries stationary in VGPRs, corpus streamed through a
// 5-deep global_load_lds ring (counted vmcnt, one raw barrier per stage)
// ---------------------------------------------------------------------------
//
// Workgroup = 4 waves = 128 queries (32 per wave, held as MFMA B fragments for
// the whole K: KSTEPS x 2 fragments, <= 192 VGPRs) x a corpus split streamed in
// 128-row tiles.  Per 128-B stage every wave issues exactly 4 corpus LDS-DMA
// pieces + 1 norm piece, so `s_waitcnt vmcnt(5*(NS-2))` retires exactly the
// stage about to be read (stages past the split end re-read the last tile to
// keep the count uniform).  All 4 waves read the same 16 A fragments per stage
// (LDS: 64 KiB per 512 MFMA cycles); only the corpus crosses L2 (16 KiB/stage).

// MFMA with the (stationary) B operand pinned in AGPRs via inline asm: the
// builtin form leaves the 192 query VGPRs to the allocator, which spills them.
// hipcc does not know the latency of an asm MFMA, so (a) a tile's first MFMA
// uses the srcC = 0 form (no VALU zeroing of the accumulator -> no VALU->MFMA
// hazard) and (b) acc_fence() pads 24 wait states (>= the 19 an XDL write ->
// VALU read needs) and is tied to every accumulator before the epilogue reads.
template <int DT> struct AsmMma;
template <> struct AsmMma<BF16> {
    typedef bf16x8 A;
    typedef bf16x8 B;
    static __device__ __forceinline__ void mma(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "a"(b));
    }
    static __device__ __forceinline__ void mma0(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "a"(b));
    }
};
template <> struct AsmMma<F16> {
    typedef f16x8 A;
    typedef f16x8 B;
    static __device__ __forceinline__ void mma(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "a"(b));
    }
    static __device__ __forceinline__ void mma0(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "a"(b));
    }
};
// f32: a 64-B k-chunk is 4 k-steps of 16x16x4 (see Frag<F32>); B is kept as 4
// scalar AGPRs per chunk.
struct Bf32 { float x[4]; };
template <> struct AsmMma<F32> {
    typedef f32x4 A;
    typedef Bf32 B;
    static __device__ __forceinline__ void mma(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c) : "v"(a[0]), "a"(b.x[0]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c) : "v"(a[1]), "a"(b.x[1]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c) : "v"(a[2]), "a"(b.x[2]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c) : "v"(a[3]), "a"(b.x[3]));
    }
    static __device__ __forceinline__ void mma0(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=a"(c) : "v"(a[0]), "a"(b.x[0]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c) : "v"(a[1]), "a"(b.x[1]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c) : "v"(a[2]), "a"(b.x[2]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c) : "v"(a[3]), "a"(b.x[3]));
    }
};

// LDS byte offset of a generic pointer into the extern LDS array
__device__ __forceinline__ uint32_t lds_off(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// The epilogue's per-tile LDS reads (row norms, tau, flag) as inline asm: hipcc
// would otherwise treat them as possibly aliasing the in-flight LDS-DMA ring and
// drain it with s_waitcnt vmcnt(0) once per tile.  Their data is ordered by the
// stage's counted vmcnt + barrier (norms) or by the previous barrier (tau, flag).
// norm_base -> row rl0 of the tile's slot ([wave][32 norms | 32 gtau], 256 B
// per wave: row r lives at (r/32)*256 + (r%32)*4); gt_base -> this lane's
// query in the wave's gtau half.
__device__ __forceinline__ void lds_read_epi(const char* norm_base, const float* tau_base, const char* gt_base,
                                             f32x4 (&y)[8], float (&t)[2], unsigned (&gt)[2]) {
    asm volatile(
        "ds_read_b128 %0, %12\n\t"
        "ds_read_b128 %1, %12 offset:64\n\t"
        "ds_read_b128 %2, %12 offset:256\n\t"
        "ds_read_b128 %3, %12 offset:320\n\t"
        "ds_read_b128 %4, %12 offset:512\n\t"
        "ds_read_b128 %5, %12 offset:576\n\t"
        "ds_read_b128 %6, %12 offset:768\n\t"
        "ds_read_b128 %7, %12 offset:832\n\t"
        "ds_read_b32 %8, %13\n\t"
        "ds_read_b32 %9, %13 offset:64\n\t"
        "ds_read_b32 %10, %14\n\t"
        "ds_read_b32 %11, %14 offset:64\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3]), "=&v"(y[4]), "=&v"(y[5]), "=&v"(y[6]), "=&v"(y[7]),
          "=&v"(t[0]), "=&v"(t[1]), "=&v"(gt[0]), "=&v"(gt[1])
        : "v"(lds_off(norm_base)), "v"(lds_off(tau_base)), "v"(lds_off(gt_base))
        : "memory");
}
__device__ __forceinline__ int lds_read_flag(const volatile int* f) {
    int v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_off((const void*)f)) : "memory");
    return v;
}

template <int M>
__device__ __forceinline__ void acc_fence(f32x4 (&acc)[M][2]) {
    static_assert(M == 8, "acc_fence operand list is written for 8x2 accumulators");
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[1][0]), "+a"(acc[1][1]), "+a"(acc[2][0]),
                   "+a"(acc[2][1]), "+a"(acc[3][0]), "+a"(acc[3][1]), "+a"(acc[4][0]), "+a"(acc[4][1]),
                   "+a"(acc[5][0]), "+a"(acc[5][1]), "+a"(acc[6][0]), "+a"(acc[6][1]), "+a"(acc[7][0]),
                   "+a"(acc[7][1]));
}

constexpr int V2_NS = 5;
constexpr int V2_STAGE = TILE_R * STAGE_B;                     // 16 KiB
constexpr int V2_NORM_OFF = V2_NS * V2_STAGE;                  // 4 slots x 4 waves x 256 B
constexpr int V2_SLOT_B = 4 * 256;                              // [wave][32 norms | 32 gtau]
constexpr int V2_LD_OFF = V2_NORM_OFF + 4 * V2_SLOT_B;
constexpr int V2_LI_OFF = V2_LD_OFF + TILE_Q * CAP * 4;
constexpr int V2_CNT_OFF = V2_LI_OFF + TILE_Q * CAP * 4;
constexpr int V2_TAU_OFF = V2_CNT_OFF + TILE_Q * 4;
constexpr int V2_FLAG_OFF = V2_TAU_OFF + TILE_Q * 4;
constexpr int V2_LDS_BYTES = V2_FLAG_OFF + 16;
static_assert(V2_LDS_BYTES <= 160 * 1024, "LDS budget");

// push the tile's survivors (key <= tau) into the LDS lists; elements that
// find their list full stay pending (bit set) for the overflow path
template <int M, int N, int METRIC>
__device__ __forceinline__ bool epi_push(const f32x4 (&acc)[M][N], const float (&yn)[M][4], const int (&qloc)[N],
                                         const float (&tn)[N], int rl0, int rlim, int trow0, unsigned (&pend)[N],
                                         float* lst_d, int* lst_i, int* cnt) {
    // fast reject: per query the smallest key of the tile (padding rows carry
    // |y|^2 = +inf, so they only reach the exact checks below while tau = inf)
    bool any = false;
#pragma unroll
    for (int n = 0; n < N; ++n) {
        float mn = FX_INF;
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                mn = fminf(mn, METRIC == L2 ? acc[m][n][i] + yn[m][i] : acc[m][n][i]);
        any |= mn <= tn[n];
    }
    if (!__any(any)) return false;
    bool ovf = false;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v = METRIC == L2 ? acc[m][n][i] + yn[m][i] : acc[m][n][i];
                const int rl = rl0 + m * 16 + i;
                if (rl < rlim && v <= tn[n]) {
                    const int s = atomicAdd(&cnt[qloc[n]], 1);
                    if (s < CAP) {
                        lst_d[qloc[n] * CAP + s] = v;
                        lst_i[qloc[n] * CAP + s] = trow0 + rl;
                    } else {
                        pend[n] |= 1u << (m * 4 + i);
                        ovf = true;
                    }
                }
            }
    return ovf;
}

template <int M, int N, int METRIC>
__device__ __forceinline__ bool epi_retry(const f32x4 (&acc)[M][N], const float (&yn)[M][4], const int (&qloc)[N],
                                          const float (&tn)[N], int rl0, int trow0, unsigned (&pend)[N],
                                          float* lst_d, int* lst_i, int* cnt) {
    bool ovf = false;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const unsigned bit = 1u << (m * 4 + i);
                if (pend[n] & bit) {
                    const float v = METRIC == L2 ? acc[m][n][i] + yn[m][i] : acc[m][n][i];
                    pend[n] &= ~bit;
                    if (v <= tn[n]) {
                        const int s = atomicAdd(&cnt[qloc[n]], 1);
                        if (s < CAP) {
                            lst_d[qloc[n] * CAP + s] = v;
                            lst_i[qloc[n] * CAP + s] = trow0 + rl0 + m * 16 + i;
                        } else {
                            pend[n] |= bit;
                            ovf = true;
                        }
                    }
                }
            }
    return ovf;
}

// ABL: compile-time ablation switches for profiling builds only (0 = product):
// 2 = no corpus DMA, 4 = no MFMA, 8 = no epilogue
template <int DT, int METRIC, int KSTEPS, int ABL = 0>
__global__ __launch_bounds__(SCAN_THREADS, 1) void k_scan_qreg(ScanParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename AsmMma<DT>::A frag_t;
    constexpr int SPT = KSTEPS / 2;  // 128-B stages per tile
    constexpr int NS = V2_NS;
    constexpr int M = TILE_R / 16;   // 8 row blocks per tile
    constexpr int N = 2;             // 2 query blocks of 16 per wave

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int qtile, split;
    map_block(blockIdx.x, p, qtile, split);
    if (qtile >= p.n_qtiles) return;
    const int ct0 = (int)((int64_t)split * p.n_ctiles / p.splits);
    const int ct1 = (int)((int64_t)(split + 1) * p.n_ctiles / p.splits);
    const int ntiles = ct1 - ct0;
    const int64_t q0 = (int64_t)qtile * TILE_Q;
    constexpr int rb = KSTEPS * 64;

    float* lst_d = (float*)(smem + V2_LD_OFF);
    int* lst_i = (int*)(smem + V2_LI_OFF);
    int* cnt = (int*)(smem + V2_CNT_OFF);
    float* tau = (float*)(smem + V2_TAU_OFF);
    volatile int* flag = (volatile int*)(smem + V2_FLAG_OFF);
    for (int x = tid; x < TILE_Q; x += SCAN_THREADS) { cnt[x] = 0; tau[x] = FX_INF; }
    if (tid == 0) *flag = 0;

    // this wave's 32 queries as B fragments for every k-step (stationary, AGPRs)
    typedef typename AsmMma<DT>::B bfrag_t;
    bfrag_t b[KSTEPS][N];
    {
        const char* qb = p.qop + (q0 + wave * 32 + (lane & 15)) * rb + (lane >> 4) * 16;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
            for (int n = 0; n < N; ++n) b[ks][n] = *(const bfrag_t*)(qb + n * 16 * rb + ks * 64);
    }
    int offs[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        const int bi = wave * 4 + jj, rblk = bi >> 1, kb = bi & 1;
        offs[jj] = (rblk * 16 + (lane & 15)) * rb + kb * 64 + (lane >> 4) * 16;
    }
    const unsigned* gtq = p.gtau + q0 + wave * 32;
    auto issue = [&](int g) {
        int t = g / SPT;
        const int j = g - t * SPT;
        if (t >= ntiles) t = ntiles - 1;  // dummy stage: uniform vmcnt accounting
        int64_t row0 = (int64_t)(ct0 + t) * TILE_R;
        if (p.dbg & 1) row0 = (int64_t)(ct0 + (t & 7)) * TILE_R;  // ablation: L2-resident corpus
        char* slot = smem + (g % NS) * V2_STAGE;
        const char* src = p.codes + row0 * rb + j * STAGE_B;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) glds16(src + offs[jj], slot + (wave * 4 + jj) * 1024);
        // lanes 0-7: this wave's 32 row norms of the tile; lanes 8-15: the
        // shared thresholds of this wave's 32 queries (refreshed every stage;
        // any version is a valid bound)
        if (lane < 16) {
            const void* src = lane < 8 ? (const void*)(p.norms + row0 + wave * 32 + lane * 4)
                                       : (const void*)(gtq + (lane - 8) * 4);
            glds16(src, smem + V2_NORM_OFF + (t & 3) * V2_SLOT_B + wave * 256);
        }
    };

#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue(s);

    f32x4 acc[M][N];
    const int rl0 = 4 * (lane >> 4);
    int qloc[N];
#pragma unroll
    for (int n = 0; n < N; ++n) qloc[n] = wave * 32 + n * 16 + (lane & 15);
    const bool qv0 = q0 + qloc[0] < p.nq, qv1 = q0 + qloc[1] < p.nq;
    unsigned pend[N] = {0u, 0u};

    // slow path: compact full lists and re-push pending survivors of tile `tp`
    auto overflow = [&](int tp) {
        const char* nb = smem + V2_NORM_OFF + (tp & 3) * V2_SLOT_B;
        float yn[M][4];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int r = rl0 + m * 16;
            const float4 v = *(const float4*)(nb + (r >> 5) * 256 + (r & 31) * 4);
            yn[m][0] = v.x; yn[m][1] = v.y; yn[m][2] = v.z; yn[m][3] = v.w;
        }
        const int trow0 = (ct0 + tp) * TILE_R;
        while (*flag) {
            __syncthreads();
            if (tid == 0) *flag = 0;
            compact_full(lst_d, lst_i, cnt, tau, wave, lane, p.gtau + q0);
            __syncthreads();
            float tn[N];
#pragma unroll
            for (int n = 0; n < N; ++n) tn[n] = tau[qloc[n]];
            if (epi_retry<M, N, METRIC>(acc, yn, qloc, tn, rl0, trow0, pend, lst_d, lst_i, cnt)) *flag = 1;
            __syncthreads();
        }
    };

    // ring reads are issued one stage ahead into a second register set (aA /
    // aB by stage parity); stage g's MFMAs then overlap stage g+1's ds_reads.
    frag_t aA[2][M], aB[2][M];
    auto read_stage = [&](int g, frag_t (&a)[2][M]) {
        const char* slot = smem + (g % NS) * V2_STAGE;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int m = 0; m < M; ++m) a[kb][m] = *(const frag_t*)(slot + (m * 2 + kb) * 1024 + lane * 16);
    };
    const int G = ntiles * SPT;
    // stage 0 landed (own DMA: vmcnt leaves stages 1..NS-2 in flight) + barrier
    asm volatile("s_waitcnt vmcnt(15)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (G > 0) read_stage(0, aA);

    for (int t = 0; t < ntiles; ++t) {
        // K loop of one 128-row tile, fully unrolled (B fragments are indexed
        // by k-step: must be compile-time to stay in registers)
#pragma unroll
        for (int j = 0; j < SPT; ++j) {
            const int g = t * SPT + j;
            frag_t (&cur)[2][M] = (j & 1) ? aB : aA;
            frag_t (&nxt)[2][M] = (j & 1) ? aA : aB;
            // stage g+1 landed for every wave; every wave is done with the
            // slot the next DMA overwrites ((g-1) % NS, read two stages ago)
            asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            // (a tile's last stage defers the prefetch past the epilogue, which
            // needs the registers)
            if (j + 1 < SPT) read_stage(g + 1, nxt);
            if (!(ABL & 2)) issue(g + NS - 1);
            if (!(ABL & 4))
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int m = 0; m < M; ++m)
#pragma unroll
                    for (int n = 0; n < N; ++n) {
                        if (j == 0 && kb == 0) AsmMma<DT>::mma0(acc[m][n], cur[kb][m], b[0][n]);
                        else AsmMma<DT>::mma(acc[m][n], cur[kb][m], b[2 * j + kb][n]);
                    }
        }
        // epilogue: filter against tau, push survivors into the LDS lists
        acc_fence<M>(acc);
        if (!(ABL & 8)) {
            const char* nb = smem + V2_NORM_OFF + (t & 3) * V2_SLOT_B;
            f32x4 y4[M];
            float tn[N];
            unsigned gt[N];
            lds_read_epi(nb + rl0 * 4, tau + qloc[0], nb + wave * 256 + 128 + (lane & 15) * 4, y4, tn, gt);
            tn[0] = fminf(tn[0], ord2f(gt[0]));
            tn[1] = fminf(tn[1], ord2f(gt[1]));
            float yn[M][4];
#pragma unroll
            for (int m = 0; m < M; ++m) {
                yn[m][0] = y4[m][0]; yn[m][1] = y4[m][1]; yn[m][2] = y4[m][2]; yn[m][3] = y4[m][3];
            }
            if (!qv0) tn[0] = -FX_INF;
            if (!qv1) tn[1] = -FX_INF;
            const int trow0 = (ct0 + t) * TILE_R;
            const int rlim = (int)(p.ntotal - (int64_t)trow0);
            if (epi_push<M, N, METRIC>(acc, yn, qloc, tn, rl0, rlim, trow0, pend, lst_d, lst_i, cnt)) *flag = 1;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (lds_read_flag(flag)) overflow(t);
        if (t + 1 < ntiles) read_stage((t + 1) * SPT, aA);  // SPT is even: tile starts in aA
    }
    // final flush: sorted top-KP per query of this (query tile, split)
    __syncthreads();
    const int64_t obase = ((int64_t)qtile * p.splits + split) * TILE_Q;
    for (int q = wave; q < TILE_Q; q += 4) {
        if (q0 + q >= p.nq) break;
        const int c = min(cnt[q], CAP);
        float d = lane < c ? lst_d[q * CAP + lane] : FX_INF;
        int i = lane < c ? lst_i[q * CAP + lane] : INT_MAX;
        sort64(d, i, lane);
        if (lane < KP) {
            p.cand_d[(obase + q) * KP + lane] = d;
            p.cand_i[(obase + q) * KP + lane] = i == INT_MAX ? -1 : i;
        }
    }
}

// ---------------------------------------------------------------------------
// scan kernel v3: v2's structure with (a) the accumulator in VGPRs holding the
// KEY itself -- queries are pre-scaled by -2 (L2) / -1 (IP) and a tile's first
// MFMA takes srcC = |y|^2 of its rows (L2) -- so the epilogue is a min3 chain
// with no accumulator reads and no FMA; (b) a 3-set rotation of A-fragment
// registers (next stage's half-stage reads overlap this stage's MFMAs);
// (c) the stage's 5 LDS-DMA pieces interleaved between MFMA groups.
// ---------------------------------------------------------------------------
template <int DT> struct AsmMmaV;
template <> struct AsmMmaV<BF16> {
    typedef bf16x8 A;
    typedef bf16x8 B;
    static __device__ __forceinline__ void settle(const B& b) { asm volatile("" ::"a"(b)); }
    static __device__ __forceinline__ void mma(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "a"(b));
    }
    static __device__ __forceinline__ void mmac(f32x4& c, const A& a, const B& b, const f32x4& c0) {
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %3" : "=&v"(c) : "v"(a), "a"(b), "v"(c0));
    }
};
template <> struct AsmMmaV<F16> {
    typedef f16x8 A;
    typedef f16x8 B;
    static __device__ __forceinline__ void settle(const B& b) { asm volatile("" ::"a"(b)); }
    static __device__ __forceinline__ void mma(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "a"(b));
    }
    static __device__ __forceinline__ void mmac(f32x4& c, const A& a, const B& b, const f32x4& c0) {
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %3" : "=&v"(c) : "v"(a), "a"(b), "v"(c0));
    }
};
template <> struct AsmMmaV<F32> {
    typedef f32x4 A;
    typedef Bf32 B;
    static __device__ __forceinline__ void settle(const B& b) {
        asm volatile("" ::"a"(b.x[0]), "a"(b.x[1]), "a"(b.x[2]), "a"(b.x[3]));
    }
    static __device__ __forceinline__ void mma(f32x4& c, const A& a, const B& b) {
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a[0]), "a"(b.x[0]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a[1]), "a"(b.x[1]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a[2]), "a"(b.x[2]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a[3]), "a"(b.x[3]));
    }
    static __device__ __forceinline__ void mmac(f32x4& c, const A& a, const B& b, const f32x4& c0) {
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %3" : "=&v"(c) : "v"(a[0]), "a"(b.x[0]), "v"(c0));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a[1]), "a"(b.x[1]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a[2]), "a"(b.x[2]));
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a[3]), "a"(b.x[3]));
    }
};

__device__ __forceinline__ void acc_fence_v(f32x4 (&acc)[8][2]) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[1][0]), "+v"(acc[1][1]), "+v"(acc[2][0]),
                   "+v"(acc[2][1]), "+v"(acc[3][0]), "+v"(acc[3][1]), "+v"(acc[4][0]), "+v"(acc[4][1]),
                   "+v"(acc[5][0]), "+v"(acc[5][1]), "+v"(acc[6][0]), "+v"(acc[6][1]), "+v"(acc[7][0]),
                   "+v"(acc[7][1]));
}

// the tile's 8 row-norm quads of this lane (rows rl0 + 16m .. +3), asm so that
// hipcc does not drain the DMA ring (see lds_read_epi)
__device__ __forceinline__ void lds_read_norms(const char* base, f32x4 (&y)[8]) {
    asm volatile(
        "ds_read_b128 %0, %8\n\t"
        "ds_read_b128 %1, %8 offset:64\n\t"
        "ds_read_b128 %2, %8 offset:256\n\t"
        "ds_read_b128 %3, %8 offset:320\n\t"
        "ds_read_b128 %4, %8 offset:512\n\t"
        "ds_read_b128 %5, %8 offset:576\n\t"
        "ds_read_b128 %6, %8 offset:768\n\t"
        "ds_read_b128 %7, %8 offset:832\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3]), "=&v"(y[4]), "=&v"(y[5]), "=&v"(y[6]), "=&v"(y[7])
        : "v"(lds_off(base))
        : "memory");
}
// LDS-DMA of one 1 KiB block (16 B per lane) issued from inline asm: the
// compiler then tracks no VMEM->LDS event and inserts none of its own
// conservative vmcnt(0) drains; the scan loops' counted barrier waits are the
// only synchronisation (MI355X_MICROARCH.md, LDS-DMA section).
__device__ __forceinline__ void glds16_asm(const void* gsrc, uint32_t lds_uniform) {
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :
                 : "v"(gsrc), "{m0}"(__builtin_amdgcn_readfirstlane(lds_uniform))
                 : "memory");
}
// Eight ds_read_b128 of one ring half-stage with NO wait: the consumer MFMAs run
// only after the next counted barrier (s_waitcnt ... lgkmcnt(0); s_barrier).
template <int KB, typename T>
__device__ __forceinline__ void lds_read_half_nowait(uint32_t base, T (&a)[8]) {
#define FX_HR(o) "ds_read_b128 %0, %8 offset:" #o "\n\t"
    if (KB == 0)
        asm volatile("ds_read_b128 %0, %8\n\t"
                     "ds_read_b128 %1, %8 offset:2048\n\t"
                     "ds_read_b128 %2, %8 offset:4096\n\t"
                     "ds_read_b128 %3, %8 offset:6144\n\t"
                     "ds_read_b128 %4, %8 offset:8192\n\t"
                     "ds_read_b128 %5, %8 offset:10240\n\t"
                     "ds_read_b128 %6, %8 offset:12288\n\t"
                     "ds_read_b128 %7, %8 offset:14336"
                     : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), "=&v"(a[6]),
                       "=&v"(a[7])
                     : "v"(base)
                     : "memory");
    else
        asm volatile("ds_read_b128 %0, %8 offset:1024\n\t"
                     "ds_read_b128 %1, %8 offset:3072\n\t"
                     "ds_read_b128 %2, %8 offset:5120\n\t"
                     "ds_read_b128 %3, %8 offset:7168\n\t"
                     "ds_read_b128 %4, %8 offset:9216\n\t"
                     "ds_read_b128 %5, %8 offset:11264\n\t"
                     "ds_read_b128 %6, %8 offset:13312\n\t"
                     "ds_read_b128 %7, %8 offset:15360"
                     : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), "=&v"(a[6]),
                       "=&v"(a[7])
                     : "v"(base)
                     : "memory");
#undef FX_HR
}
__device__ __forceinline__ void lds_read_tau(const float* tau_base, const char* gt_base, float (&t)[2],
                                             unsigned (&gt)[2]) {
    asm volatile(
        "ds_read_b32 %0, %4\n\t"
        "ds_read_b32 %1, %4 offset:64\n\t"
        "ds_read_b32 %2, %5\n\t"
        "ds_read_b32 %3, %5 offset:64\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(t[0]), "=&v"(t[1]), "=&v"(gt[0]), "=&v"(gt[1])
        : "v"(lds_off(tau_base)), "v"(lds_off(gt_base))
        : "memory");
}

// key-in-accumulator versions of epi_push / epi_retry
template <int M, int N>
__device__ __forceinline__ bool epi3_push(const f32x4 (&acc)[M][N], const int (&qloc)[N], const float (&tn)[N],
                                          int rl0, int rlim, int trow0, unsigned (&pend)[N], float* lst_d,
                                          int* lst_i, int* cnt) {
    bool any = false;
#pragma unroll
    for (int n = 0; n < N; ++n) {
        float mn = acc[0][n][0];
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (m | i) mn = fminf(mn, acc[m][n][i]);
        any |= mn <= tn[n];
    }
    if (!__any(any)) return false;
    bool ovf = false;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v = acc[m][n][i];
                const int rl = rl0 + m * 16 + i;
                if (rl < rlim && v <= tn[n]) {
                    const int s = atomicAdd(&cnt[qloc[n]], 1);
                    if (s < CAP) {
                        lst_d[qloc[n] * CAP + s] = v;
                        lst_i[qloc[n] * CAP + s] = trow0 + rl;
                    } else {
                        pend[n] |= 1u << (m * 4 + i);
                        ovf = true;
                    }
                }
            }
    return ovf;
}

template <int M, int N>
__device__ __forceinline__ bool epi3_retry(const f32x4 (&acc)[M][N], const int (&qloc)[N], const float (&tn)[N],
                                           int rl0, int trow0, unsigned (&pend)[N], float* lst_d, int* lst_i,
                                           int* cnt) {
    bool ovf = false;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const unsigned bit = 1u << (m * 4 + i);
                if (pend[n] & bit) {
                    const float v = acc[m][n][i];
                    pend[n] &= ~bit;
                    if (v <= tn[n]) {
                        const int s = atomicAdd(&cnt[qloc[n]], 1);
                        if (s < CAP) {
                            lst_d[qloc[n] * CAP + s] = v;
                            lst_i[qloc[n] * CAP + s] = trow0 + rl0 + m * 16 + i;
                        } else {
                            pend[n] |= bit;
                            ovf = true;
                        }
                    }
                }
            }
    return ovf;
}

template <int DT, int METRIC, int KSTEPS>
__global__ __launch_bounds__(SCAN_THREADS, 1) void k_scan_q3(ScanParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename AsmMmaV<DT>::A frag_t;
    typedef typename AsmMmaV<DT>::B bfrag_t;
    constexpr int SPT = KSTEPS / 2;
    constexpr int NS = V2_NS;
    constexpr int M = TILE_R / 16;
    constexpr int N = 2;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int qtile, split;
    map_block(blockIdx.x, p, qtile, split);
    if (qtile >= p.n_qtiles) return;
    const int ct0 = (int)((int64_t)split * p.n_ctiles / p.splits);
    const int ct1 = (int)((int64_t)(split + 1) * p.n_ctiles / p.splits);
    const int ntiles = ct1 - ct0;
    const int64_t q0 = (int64_t)qtile * TILE_Q;
    constexpr int rb = KSTEPS * 64;

    float* lst_d = (float*)(smem + V2_LD_OFF);
    int* lst_i = (int*)(smem + V2_LI_OFF);
    int* cnt = (int*)(smem + V2_CNT_OFF);
    float* tau = (float*)(smem + V2_TAU_OFF);
    volatile int* flag = (volatile int*)(smem + V2_FLAG_OFF);
    for (int x = tid; x < TILE_Q; x += SCAN_THREADS) { cnt[x] = 0; tau[x] = FX_INF; }
    if (tid == 0) *flag = 0;

    bfrag_t b[KSTEPS][N];
    {
        const char* qb = p.qop + (q0 + wave * 32 + (lane & 15)) * rb + (lane >> 4) * 16;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
            for (int n = 0; n < N; ++n) b[ks][n] = *(const bfrag_t*)(qb + n * 16 * rb + ks * 64);
        // settle the operand loads here, once: otherwise the compiler re-waits
        // (vmcnt(0), draining the corpus DMA ring) at every tile's first MFMA
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
            for (int n = 0; n < N; ++n) AsmMmaV<DT>::settle(b[ks][n]);
    }
    int offs[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        const int bi = wave * 4 + jj, rblk = bi >> 1, kb = bi & 1;
        offs[jj] = (rblk * 16 + (lane & 15)) * rb + kb * 64 + (lane >> 4) * 16;
    }
    const unsigned* gtq = p.gtau + q0 + wave * 32;
    const uint32_t lds_base = lds_off(smem);
    // DMA piece `which` (0-3 corpus blocks, 4 norms + shared thresholds) of stage g
    auto issue_piece = [&](int g, int which) {
        int t = g / SPT;
        const int j = g - t * SPT;
        if (t >= ntiles) t = ntiles - 1;  // dummy stage: uniform vmcnt accounting
        const int64_t row0 = (int64_t)(ct0 + t) * TILE_R;
        if (which < 4) {
            glds16_asm(p.codes + row0 * rb + j * STAGE_B + offs[which],
                       lds_base + (g % NS) * V2_STAGE + (wave * 4 + which) * 1024);
        } else if (lane < 16) {
            const void* src = lane < 8 ? (const void*)(p.norms + row0 + wave * 32 + lane * 4)
                                       : (const void*)(gtq + (lane - 8) * 4);
            glds16_asm(src, lds_base + V2_NORM_OFF + (t & 3) * V2_SLOT_B + wave * 256);
        }
    };
    auto read_half = [&](int g, int kb, frag_t (&a)[M]) {
        const uint32_t slot = lds_base + (g % NS) * V2_STAGE + lane * 16;
        if (kb == 0) lds_read_half_nowait<0>(slot, a);
        else lds_read_half_nowait<1>(slot, a);
    };

#pragma unroll
    for (int st = 0; st < NS - 1; ++st)
#pragma unroll
        for (int w = 0; w < 5; ++w) issue_piece(st, w);

    f32x4 acc[M][N];
    const int rl0 = 4 * (lane >> 4);
    int qloc[N];
#pragma unroll
    for (int n = 0; n < N; ++n) qloc[n] = wave * 32 + n * 16 + (lane & 15);
    const bool qv0 = q0 + qloc[0] < p.nq, qv1 = q0 + qloc[1] < p.nq;
    unsigned pend[N] = {0u, 0u};

    auto overflow = [&](int tp) {
        const int trow0 = (ct0 + tp) * TILE_R;
        while (*flag) {
            __syncthreads();
            if (tid == 0) *flag = 0;
            compact_full(lst_d, lst_i, cnt, tau, wave, lane, p.gtau + q0);
            __syncthreads();
            float tn[N];
#pragma unroll
            for (int n = 0; n < N; ++n) tn[n] = tau[qloc[n]];
            if (epi3_retry<M, N>(acc, qloc, tn, rl0, trow0, pend, lst_d, lst_i, cnt)) *flag = 1;
            __syncthreads();
        }
    };

    frag_t s0[M], s1[M], s2[M];
    const int G = ntiles * SPT;
    asm volatile("s_waitcnt vmcnt(15)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (G > 0) {
        read_half(0, 0, s0);
        read_half(0, 1, s1);
    }

    for (int t = 0; t < ntiles; ++t) {
#pragma unroll
        for (int j = 0; j < SPT; ++j) {
            const int g = t * SPT + j;
            const int rx = (2 * j) % 3, ry = (2 * j + 1) % 3;  // sets of this stage's halves
            frag_t (&X)[M] = rx == 0 ? s0 : (rx == 1 ? s1 : s2);
            frag_t (&Y)[M] = ry == 0 ? s0 : (ry == 1 ? s1 : s2);
            frag_t (&Z)[M] = (3 - rx - ry) == 0 ? s0 : ((3 - rx - ry) == 1 ? s1 : s2);
            // stage g+1 landed for every wave; slot (g-1)%NS is free for the DMA
            asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            f32x4 yinit[M];
            if (j == 0) {
                if (METRIC == L2) {
                    lds_read_norms(smem + V2_NORM_OFF + (t & 3) * V2_SLOT_B + rl0 * 4, yinit);
                } else {
#pragma unroll
                    for (int m = 0; m < M; ++m) yinit[m] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
            if (j + 1 < SPT) read_half(g + 1, 0, Z);
            issue_piece(g + NS - 1, 0);
            issue_piece(g + NS - 1, 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
                for (int n = 0; n < N; ++n) {
                    if (j == 0) AsmMmaV<DT>::mmac(acc[m][n], X[m], b[0][n], yinit[m]);
                    else AsmMmaV<DT>::mma(acc[m][n], X[m], b[2 * j][n]);
                }
            __builtin_amdgcn_sched_barrier(0);
            issue_piece(g + NS - 1, 2);
            issue_piece(g + NS - 1, 3);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < M / 2; ++m)
#pragma unroll
                for (int n = 0; n < N; ++n) AsmMmaV<DT>::mma(acc[m][n], Y[m], b[2 * j + 1][n]);
            __builtin_amdgcn_sched_barrier(0);
            // X's last readers were issued >= 8 MFMAs ago: safe to overwrite
            if (j + 1 < SPT) read_half(g + 1, 1, X);
            issue_piece(g + NS - 1, 4);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = M / 2; m < M; ++m)
#pragma unroll
                for (int n = 0; n < N; ++n) AsmMmaV<DT>::mma(acc[m][n], Y[m], b[2 * j + 1][n]);
        }
        // epilogue: the accumulator holds the keys
        acc_fence_v(acc);
        {
            float tn[N];
            unsigned gt[N];
            const char* nb = smem + V2_NORM_OFF + (t & 3) * V2_SLOT_B;
            lds_read_tau(tau + qloc[0], nb + wave * 256 + 128 + (lane & 15) * 4, tn, gt);
            tn[0] = qv0 ? fminf(tn[0], ord2f(gt[0])) : -FX_INF;
            tn[1] = qv1 ? fminf(tn[1], ord2f(gt[1])) : -FX_INF;
            const int trow0 = (ct0 + t) * TILE_R;
            const int rlim = (int)(p.ntotal - (int64_t)trow0);
            if (epi3_push<M, N>(acc, qloc, tn, rl0, rlim, trow0, pend, lst_d, lst_i, cnt)) *flag = 1;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (lds_read_flag(flag)) overflow(t);
        if (t + 1 < ntiles) {
            read_half((t + 1) * SPT, 0, s0);
            read_half((t + 1) * SPT, 1, s1);
        }
    }

    // final flush: sorted top-KP per query of this (query tile, split)
    __syncthreads();
    const int64_t obase = ((int64_t)qtile * p.splits + split) * TILE_Q;
    for (int q = wave; q < TILE_Q; q += 4) {
        if (q0 + q >= p.nq) break;
        const int c = min(cnt[q], CAP);
        float d = lane < c ? lst_d[q * CAP + lane] : FX_INF;
        int i = lane < c ? lst_i[q * CAP + lane] : INT_MAX;
        sort64(d, i, lane);
        if (lane < KP) {
            p.cand_d[(obase + q) * KP + lane] = d;
            p.cand_i[(obase + q) * KP + lane] = i == INT_MAX ? -1 : i;
        }
    }
}

// ---------------------------------------------------------------------------
// merge + exact refine + certification: one wave per query
// ---------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ void load_chunk(const char* p, float* v) {  // 16 bytes -> E floats
    if (DT == F32) {
        float4 x = *(const float4*)p;
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    } else {
        uint4 x = *(const uint4*)p;
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint16_t lo = (uint16_t)(w[e] & 0xffffu), hi = (uint16_t)(w[e] >> 16);
            v[2 * e] = DT == BF16 ? bf2f(lo) : h2f(lo);
            v[2 * e + 1] = DT == BF16 ? bf2f(hi) : h2f(hi);
        }
    }
}

// exact metric value of (x, row) accumulated by `nl` lanes (lane sub of nl)
template <int DT, int METRIC>
__device__ __forceinline__ double exact_partial(const float* __restrict__ xq, const char* __restrict__ yrow,
                                                int row_bytes, int sub, int nl) {
    constexpr int E = DT == F32 ? 4 : 8;
    double acc = 0.0;
    for (int c = sub; c * 16 < row_bytes; c += nl) {
        float y[E];
        load_chunk<DT>(yrow + c * 16, y);
        const float* xc = xq + c * E;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (METRIC == L2) {
                const double df = (double)xc[e] - (double)y[e];
                acc = fma(df, df, acc);
            } else {
                acc = fma((double)xc[e], (double)y[e], acc);
            }
        }
    }
    return acc;
}

template <int DT, int METRIC>
__global__ __launch_bounds__(256) void k_refine(RefineParams p) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= p.nq) return;
    const int qtile = (int)(q / TILE_Q), qq = (int)(q % TILE_Q);
    const int ncand = p.splits * KP;

    // ---- phase 1: KP smallest approx keys over all splits (running best-64)
    float bd = FX_INF, td = FX_INF;
    int bi = INT_MAX, ti = INT_MAX;
    int nvalid = 0;
    for (int base = 0; base < ncand; base += 64) {
        const int c = base + lane;
        float d = FX_INF;
        int i = INT_MAX;
        if (c < ncand) {
            const int s = c / KP, j = c - s * KP;
            const int64_t off = (((int64_t)qtile * p.splits + s) * TILE_Q + qq) * KP + j;
            const int ii = p.cand_i[off];
            if (ii >= 0) { d = p.cand_d[off]; i = ii; }
        }
        nvalid += __popcll(__ballot(i != INT_MAX));
        const bool pass = i != INT_MAX && key_lt(d, i, td, ti);
        if (!__any(pass)) continue;
        if (!pass) { d = FX_INF; i = INT_MAX; }
        sort64(d, i, lane);
        merge_into(bd, bi, d, i, lane);
        td = __shfl(bd, KP - 1, 64);
        ti = __shfl(bi, KP - 1, 64);
    }

    // ---- phase 2: exact fp64 values of the KP selected rows (16 lanes / row)
    const float* xq = p.qf32 + q * (int64_t)p.kdim;
    const int grp = lane >> 4, sub = lane & 15;
    double ex = 0.0;
    for (int r = 0; r < KP / 4; ++r) {
        const int row = __shfl(bi, r * 4 + grp, 64);
        double a = 0.0;
        if (row != INT_MAX) a = exact_partial<DT, METRIC>(xq, p.codes + (int64_t)row * p.row_bytes, p.row_bytes, sub, 16);
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        const double v = __shfl(a, (lane & 3) * 16, 64);
        if ((lane >> 2) == r) ex = v;
    }
    double xn2 = 0.0;
    if (METRIC == L2) {
        for (int c = lane; c < p.kdim; c += 64) xn2 = fma((double)xq[c], (double)xq[c], xn2);
        xn2 = wave_sum_f64(xn2);
    }

    // ---- phase 3: order by (fp32 exact key, id), write top-k, certify
    float key = FX_INF;
    int id = INT_MAX;
    if (lane < KP && bi != INT_MAX) {
        key = METRIC == L2 ? (float)ex : -(float)ex;
        id = bi;
    }
    sort64(key, id, lane);
    if (lane < p.k) {
        const bool valid = id != INT_MAX;
        p.D[q * p.k + lane] = valid ? (METRIC == L2 ? key : -key) : (METRIC == L2 ? FLT_MAX : -FLT_MAX);
        p.I[q * p.k + lane] = valid ? (int64_t)id + p.id_offset : (int64_t)-1;
    }
    // Rows the selection dropped all have approx key >= td (DESIGN.md
    // "certification"); they cannot outrank the k-th result when
    // key_k < td (+|x|^2 for L2) - eps.
    if (nvalid >= KP) {
        const float kth = __shfl(key, p.k - 1, 64);
        const double bound = (METRIC == L2 ? (double)td + xn2 : (double)td) - (double)p.qeps[q];
        const double kup = (double)kth + fabs((double)kth) * 2.384185791015625e-7;  // + 2 ulp
        if (!(kup < bound) && lane == 0) {
            const int pos = atomicAdd(p.n_flag, 1);
            p.flag_list[pos] = (int)q;
        }
    }
}

// ---------------------------------------------------------------------------
// exact fallback: every row's exact key, (key, id) top-KP per wave
// ---------------------------------------------------------------------------
template <int DT, int METRIC>
__global__ __launch_bounds__(256) void k_exact_scan(const char* __restrict__ codes, int row_bytes, int kdim,
                                                    int64_t ntotal, const float* __restrict__ qf32,
                                                    const int* __restrict__ qlist, int fb_splits,
                                                    float* __restrict__ cand_d, int* __restrict__ cand_i) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int f = blockIdx.x / fb_splits, split = blockIdx.x % fb_splits;
    const int64_t q = qlist[f];
    const float* xq = qf32 + q * (int64_t)kdim;
    const int64_t r0 = ntotal * split / fb_splits, r1 = ntotal * (split + 1) / fb_splits;
    float bd = FX_INF, td = FX_INF;
    int bi = INT_MAX, ti = INT_MAX;
    for (int64_t base = r0 + (int64_t)wave * 64; base < r1; base += 256) {
        const int64_t row = base + lane;
        float key = FX_INF;
        int id = INT_MAX;
        if (row < r1) {
            const double v = exact_partial<DT, METRIC>(xq, codes + row * row_bytes, row_bytes, 0, 1);
            key = METRIC == L2 ? (float)v : -(float)v;
            id = (int)row;
        }
        const bool pass = id != INT_MAX && key_lt(key, id, td, ti);
        if (!__any(pass)) continue;
        if (!pass) { key = FX_INF; id = INT_MAX; }
        sort64(key, id, lane);
        merge_into(bd, bi, key, id, lane);
        td = __shfl(bd, KP - 1, 64);
        ti = __shfl(bi, KP - 1, 64);
    }
    if (lane < KP) {
        const int64_t o = (((int64_t)f * fb_splits + split) * 4 + wave) * KP + lane;
        cand_d[o] = bd;
        cand_i[o] = bi == INT_MAX ? -1 : bi;
    }
}

template <int METRIC>
__global__ __launch_bounds__(256) void k_merge_exact(const float* __restrict__ cand_d, const int* __restrict__ cand_i,
                                                     int per_query, const int* __restrict__ qlist, int nlist, int k,
                                                     int64_t id_offset, float* __restrict__ D, int64_t* __restrict__ I) {
    const int lane = threadIdx.x & 63;
    const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= nlist) return;
    float bd = FX_INF, td = FX_INF;
    int bi = INT_MAX, ti = INT_MAX;
    for (int base = 0; base < per_query; base += 64) {
        const int c = base + lane;
        float d = FX_INF;
        int i = INT_MAX;
        if (c < per_query) {
            const int ii = cand_i[(int64_t)f * per_query + c];
            if (ii >= 0) { d = cand_d[(int64_t)f * per_query + c]; i = ii; }
        }
        const bool pass = i != INT_MAX && key_lt(d, i, td, ti);
        if (!__any(pass)) continue;
        if (!pass) { d = FX_INF; i = INT_MAX; }
        sort64(d, i, lane);
        merge_into(bd, bi, d, i, lane);
        td = __shfl(bd, KP - 1, 64);
        ti = __shfl(bi, KP - 1, 64);
    }
    const int64_t q = qlist[f];
    if (lane < k) {
        const bool valid = bi != INT_MAX;
        D[q * k + lane] = valid ? (METRIC == L2 ? bd : -bd) : (METRIC == L2 ? FLT_MAX : -FLT_MAX);
        I[q * k + lane] = valid ? (int64_t)bi + id_offset : (int64_t)-1;
    }
}

// ---------------------------------------------------------------------------
// multi-GPU: merge [G][nq][k] gathered shard results
// ---------------------------------------------------------------------------
template <int METRIC>
__global__ __launch_bounds__(256) void k_merge_shards(int nshards, int64_t nq, int k, const float* __restrict__ Din,
                                                      const int64_t* __restrict__ Iin, float* __restrict__ Dout,
                                                      int64_t* __restrict__ Iout) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int total = nshards * k;
    float bd = FX_INF, td = FX_INF;
    long long bi = LLONG_MAX, ti = LLONG_MAX;
    for (int base = 0; base < total; base += 64) {
        const int c = base + lane;
        float d = FX_INF;
        long long i = LLONG_MAX;
        if (c < total) {
            const int s = c / k, j = c - s * k;
            const int64_t off = ((int64_t)s * nq + q) * k + j;
            const long long ii = Iin[off];
            if (ii >= 0) { d = METRIC == L2 ? Din[off] : -Din[off]; i = ii; }
        }
        const bool pass = i != LLONG_MAX && key_lt(d, i, td, ti);
        if (!__any(pass)) continue;
        if (!pass) { d = FX_INF; i = LLONG_MAX; }
        sort64(d, i, lane);
        merge_into(bd, bi, d, i, lane);
        const int kk = k < 64 ? k : 64;
        td = __shfl(bd, kk - 1, 64);
        ti = __shfl(bi, kk - 1, 64);
    }
    if (lane < k) {
        const bool valid = bi != LLONG_MAX;
        Dout[q * k + lane] = valid ? (METRIC == L2 ? bd : -bd) : (METRIC == L2 ? FLT_MAX : -FLT_MAX);
        Iout[q * k + lane] = valid ? (int64_t)bi : (int64_t)-1;
    }
}

// ---------------------------------------------------------------------------
// synthetic corpus and fp32 read-back
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_synth(void* __restrict__ out, int64_t row0, int64_t n, int d, int dt,
                                               uint64_t seed) {
    const int64_t total = n * d;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t r = e / d, c = e - r * d;
        uint64_t z = seed * 0x9E3779B97F4A7C15ull + (uint64_t)(row0 + r) * (uint64_t)d + (uint64_t)c;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const int b0 = (int)(z & 0xFF), b1 = (int)((z >> 8) & 0xFF);
        store_elem(out, e, dt, (float)(b0 + b1 - 255) / 64.0f);
    }
}

__global__ __launch_bounds__(256) void k_to_f32(const char* __restrict__ codes, int st_dt, int row_bytes, int64_t n,
                                                int d, float* __restrict__ out) {
    const int64_t total = n * d;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t r = e / d, c = e - r * d;
        out[e] = load_elem(codes + r * row_bytes, c, st_dt);
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline int grid_for(int64_t items, int per_block, int cap) {
    int64_t g = (items + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

hipError_t launch_convert_rows(const void* x, int x_dt, int64_t n, int d, void* codes_row0, int st_dt, int kdim,
                               float* norms_row0, unsigned* max_sq_bits, int normalize, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_convert_rows, dim3(grid_for(n, 4, 65536)), dim3(256), 0, s, x, x_dt, n, d, codes_row0,
                       st_dt, kdim, norms_row0, max_sq_bits, normalize);
    return hipGetLastError();
}

hipError_t launch_prep_queries(const void* q, int q_dt, int64_t nq, int64_t nq_pad, int d, int kdim, int st_dt,
                               int metric, float* qf32, void* qop, float* qeps, double max_norm, hipStream_t s) {
    const double u = 5.9604644775390625e-8;
    const double gamma = (double)kdim * u / (1.0 - (double)kdim * u);
    hipLaunchKernelGGL(k_prep_queries, dim3((unsigned)((nq_pad + 3) / 4)), dim3(256), 0, s, q, q_dt, nq, nq_pad, d,
                       kdim, st_dt, metric, qf32, qop, qeps, max_norm, gamma);
    return hipGetLastError();
}

template <int DT, int METRIC>
static hipError_t scan_t(const ScanParams& p, hipStream_t s) {
    // > 64 KiB of dynamic LDS must be opted into (per device; cheap to repeat)
    hipError_t e = hipFuncSetAttribute((const void*)k_scan_topk<DT, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_SCAN_BYTES);
    if (e != hipSuccess) return e;
    const int grid = p.qt_per_xcd > 0 ? 8 * p.qt_per_xcd * p.splits : p.n_qtiles * p.splits;
    hipLaunchKernelGGL((k_scan_topk<DT, METRIC>), dim3(grid), dim3(SCAN_THREADS), LDS_SCAN_BYTES, s, p);
    return hipGetLastError();
}

template <int DT, int METRIC, int KSTEPS>
static hipError_t scan_v2_t(const ScanParams& p, hipStream_t s) {
    const int grid = p.qt_per_xcd > 0 ? 8 * p.qt_per_xcd * p.splits : p.n_qtiles * p.splits;
    static const bool use_v2 = getenv("FX_SCAN_V2") != nullptr;
    if (use_v2) {
        hipError_t e = hipFuncSetAttribute((const void*)k_scan_qreg<DT, METRIC, KSTEPS>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, V2_LDS_BYTES);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_scan_qreg<DT, METRIC, KSTEPS>), dim3(grid), dim3(SCAN_THREADS), V2_LDS_BYTES, s, p);
        return hipGetLastError();
    }
    hipError_t e = hipFuncSetAttribute((const void*)k_scan_q3<DT, METRIC, KSTEPS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, V2_LDS_BYTES);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_scan_q3<DT, METRIC, KSTEPS>), dim3(grid), dim3(SCAN_THREADS), V2_LDS_BYTES, s, p);
    return hipGetLastError();
}

template <int DT, int METRIC, int KSTEPS, int ABL>
static hipError_t scan_abl_t(const ScanParams& p, hipStream_t s) {
    hipError_t e = hipFuncSetAttribute((const void*)k_scan_qreg<DT, METRIC, KSTEPS, ABL>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, V2_LDS_BYTES);
    if (e != hipSuccess) return e;
    const int grid = p.qt_per_xcd > 0 ? 8 * p.qt_per_xcd * p.splits : p.n_qtiles * p.splits;
    hipLaunchKernelGGL((k_scan_qreg<DT, METRIC, KSTEPS, ABL>), dim3(grid), dim3(SCAN_THREADS), V2_LDS_BYTES, s, p);
    return hipGetLastError();
}

template <int DT, int METRIC>
static hipError_t scan_v2_dispatch(const ScanParams& p, hipStream_t s, bool* handled) {
    *handled = true;
#ifdef FX_ABLATION
    if (DT == BF16 && METRIC == L2 && p.row_bytes == 1536 && p.dbg >= 2) {
        switch (p.dbg) {
            case 2: return scan_abl_t<DT, METRIC, 24, 2>(p, s);
            case 4: return scan_abl_t<DT, METRIC, 24, 4>(p, s);
            case 8: return scan_abl_t<DT, METRIC, 24, 8>(p, s);
            case 6: return scan_abl_t<DT, METRIC, 24, 6>(p, s);
            case 14: return scan_abl_t<DT, METRIC, 24, 14>(p, s);
            default: break;
        }
    }
#endif
    switch (p.row_bytes / 64) {
        case 8: return scan_v2_t<DT, METRIC, 8>(p, s);
        case 12: return scan_v2_t<DT, METRIC, 12>(p, s);
        case 16: return scan_v2_t<DT, METRIC, 16>(p, s);
        case 24: return scan_v2_t<DT, METRIC, 24>(p, s);
        default: *handled = false; return hipSuccess;
    }
}

bool scan_v2_supported(int row_bytes) {
    const int ks = row_bytes / 64;
    return ks == 8 || ks == 12 || ks == 16 || ks == 24;
}

hipError_t launch_scan(int st_dt, int metric, const ScanParams& p, hipStream_t s) {
    if (scan_v2_supported(p.row_bytes) && !getenv("FX_SCAN_V1")) {
        bool handled = false;
        hipError_t e;
        if (metric == L2) {
            if (st_dt == F32) e = scan_v2_dispatch<F32, L2>(p, s, &handled);
            else if (st_dt == BF16) e = scan_v2_dispatch<BF16, L2>(p, s, &handled);
            else e = scan_v2_dispatch<F16, L2>(p, s, &handled);
        } else {
            if (st_dt == F32) e = scan_v2_dispatch<F32, IP>(p, s, &handled);
            else if (st_dt == BF16) e = scan_v2_dispatch<BF16, IP>(p, s, &handled);
            else e = scan_v2_dispatch<F16, IP>(p, s, &handled);
        }
        if (handled) return e;
    }
    if (metric == L2) {
        if (st_dt == F32) return scan_t<F32, L2>(p, s);
        if (st_dt == BF16) return scan_t<BF16, L2>(p, s);
        return scan_t<F16, L2>(p, s);
    }
    if (st_dt == F32) return scan_t<F32, IP>(p, s);
    if (st_dt == BF16) return scan_t<BF16, IP>(p, s);
    return scan_t<F16, IP>(p, s);
}

template <int DT, int METRIC>
static hipError_t refine_t(const RefineParams& p, hipStream_t s) {
    hipLaunchKernelGGL((k_refine<DT, METRIC>), dim3((unsigned)((p.nq + 3) / 4)), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_refine(int st_dt, int metric, const RefineParams& p, hipStream_t s) {
    if (metric == L2) {
        if (st_dt == F32) return refine_t<F32, L2>(p, s);
        if (st_dt == BF16) return refine_t<BF16, L2>(p, s);
        return refine_t<F16, L2>(p, s);
    }
    if (st_dt == F32) return refine_t<F32, IP>(p, s);
    if (st_dt == BF16) return refine_t<BF16, IP>(p, s);
    return refine_t<F16, IP>(p, s);
}

template <int DT, int METRIC>
static void exact_scan_t(dim3 g, hipStream_t s, const char* codes, int row_bytes, int kdim, int64_t ntotal,
                         const float* qf32, const int* qlist, int fb_splits, float* cd, int* ci) {
    hipLaunchKernelGGL((k_exact_scan<DT, METRIC>), g, dim3(256), 0, s, codes, row_bytes, kdim, ntotal, qf32, qlist,
                       fb_splits, cd, ci);
}

hipError_t launch_exact_fallback(int st_dt, int metric, const char* codes, int row_bytes, int kdim, int64_t ntotal,
                                 const float* qf32, const int* qlist, int nlist, int k, int64_t id_offset,
                                 float* cand_d, int* cand_i, int fb_splits, float* D, int64_t* I, hipStream_t s) {
    if (nlist <= 0) return hipSuccess;
    const dim3 g((unsigned)(nlist * fb_splits));
    if (metric == L2) {
        if (st_dt == F32) exact_scan_t<F32, L2>(g, s, codes, row_bytes, kdim, ntotal, qf32, qlist, fb_splits, cand_d, cand_i);
        else if (st_dt == BF16) exact_scan_t<BF16, L2>(g, s, codes, row_bytes, kdim, ntotal, qf32, qlist, fb_splits, cand_d, cand_i);
        else exact_scan_t<F16, L2>(g, s, codes, row_bytes, kdim, ntotal, qf32, qlist, fb_splits, cand_d, cand_i);
    } else {
        if (st_dt == F32) exact_scan_t<F32, IP>(g, s, codes, row_bytes, kdim, ntotal, qf32, qlist, fb_splits, cand_d, cand_i);
        else if (st_dt == BF16) exact_scan_t<BF16, IP>(g, s, codes, row_bytes, kdim, ntotal, qf32, qlist, fb_splits, cand_d, cand_i);
        else exact_scan_t<F16, IP>(g, s, codes, row_bytes, kdim, ntotal, qf32, qlist, fb_splits, cand_d, cand_i);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int per_query = fb_splits * 4 * KP;
    const dim3 g2((unsigned)((nlist + 3) / 4));
    if (metric == L2)
        hipLaunchKernelGGL(k_merge_exact<L2>, g2, dim3(256), 0, s, cand_d, cand_i, per_query, qlist, nlist, k, id_offset, D, I);
    else
        hipLaunchKernelGGL(k_merge_exact<IP>, g2, dim3(256), 0, s, cand_d, cand_i, per_query, qlist, nlist, k, id_offset, D, I);
    return hipGetLastError();
}

hipError_t launch_merge_shards(int metric, int nshards, int64_t nq, int k, const float* D_in, const int64_t* I_in,
                               float* D_out, int64_t* I_out, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    const dim3 g((unsigned)((nq + 3) / 4));
    if (metric == L2)
        hipLaunchKernelGGL(k_merge_shards<L2>, g, dim3(256), 0, s, nshards, nq, k, D_in, I_in, D_out, I_out);
    else
        hipLaunchKernelGGL(k_merge_shards<IP>, g, dim3(256), 0, s, nshards, nq, k, D_in, I_in, D_out, I_out);
    return hipGetLastError();
}

hipError_t launch_synth(void* out, int64_t row0, int64_t n, int d, int dtype, uint64_t seed, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth, dim3(grid_for(n * d, 256, 16384)), dim3(256), 0, s, out, row0, n, d, dtype, seed);
    return hipGetLastError();
}

hipError_t launch_to_f32(const void* codes, int st_dt, int row_bytes, int64_t n, int d, float* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_to_f32, dim3(grid_for(n * d, 256, 16384)), dim3(256), 0, s, (const char*)codes, st_dt,
                       row_bytes, n, d, out);
    return hipGetLastError();
}

}  // namespace fx
