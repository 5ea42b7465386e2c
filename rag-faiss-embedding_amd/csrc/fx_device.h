// fx_device.h -- device-side helpers shared by the HIP translation units
// (fx_kernels.hip: add/refine/merge/synth + generic scan; fx_scan.hip: the
// MFMA scan).  Header-only, all inline.
#pragma once
#include "fx_internal.h"

#include <float.h>
#include <limits.h>

#include <utility>

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

// exact arithmetic of the refine, the exact fallback and the k > FX_BIG_K path
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

// ---------------------------------------------------------------------------
// wave-level (64-lane) bitonic helpers on (key, id) pairs, ascending,
// ties -> smaller id.  Used for LDS list compaction and every merge.
// ---------------------------------------------------------------------------
template <typename Id>
__device__ __forceinline__ bool key_lt(float d1, Id i1, float d2, Id i2) {
    return d1 < d2 || (d1 == d2 && i1 < i2);
}

template <int... Is, typename F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// x of lane ^ 16 / lane ^ 32 without the LDS crossbar: gfx950's
// v_permlane16_swap (odd 16-lane rows of the first operand <-> even rows of
// the second) and v_permlane32_swap (upper half of the first <-> lower half of
// the second) on two copies of x.  The s_nop covers a VALU write of the
// copies just before (inline asm is not padded by the compiler).
__device__ __forceinline__ int lane_xor16(int x, int lane) {
    int a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return (lane & 16) ? a : b;
}
__device__ __forceinline__ int lane_xor32(int x, int lane) {
    int a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return (lane & 32) ? a : b;
}
// x of lane ^ S for S = 1 .. 32, all on the VALU: DPP inside 16-lane rows
// (quad_perm for 1 and 2; row_ror for 4 and 8: ror:N reads lane - N mod 16),
// the permlane swaps across rows
template <int S>
__device__ __forceinline__ int lane_xor(int x, int lane) {
    if constexpr (S == 1) return __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    else if constexpr (S == 2) return __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
    else if constexpr (S == 4) {
        const int a = __builtin_amdgcn_update_dpp(0, x, 0x124, 0xF, 0xF, false);  // row_ror:4: lane - 4
        const int b = __builtin_amdgcn_update_dpp(0, x, 0x12C, 0xF, 0xF, false);  // row_ror:12: lane + 4
        return (lane & 4) ? a : b;
    } else if constexpr (S == 8) return __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);  // row_ror:8
    else if constexpr (S == 16) return lane_xor16(x, lane);
    else return lane_xor32(x, lane);
}
template <int S>
__device__ __forceinline__ float lane_xor(float x, int lane) {
    return __int_as_float(lane_xor<S>(__float_as_int(x), lane));
}
template <int S>
__device__ __forceinline__ long long lane_xor(long long x, int lane) {
    const int lo = lane_xor<S>((int)(x & 0xffffffffll), lane), hi = lane_xor<S>((int)(x >> 32), lane);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// ---------------------------------------------------------------------------
// wave-level (64-lane) bitonic helpers on (key, id) pairs, ascending,
// ties -> smaller id.  Used for LDS list compaction and every merge.  The
// partner exchange runs on the VALU (lane_xor), branch-free compares.
// ---------------------------------------------------------------------------
template <int S, typename Id>
__device__ __forceinline__ void cmpx_s(float& d, Id& i, int lane, bool asc) {
    const float od = lane_xor<S>(d, lane);
    const Id oi = lane_xor<S>(i, lane);
    const bool lower = (lane & S) == 0;
    const bool o_lt = (od < d) | ((od == d) & (oi < i));
    const bool m_lt = (d < od) | ((d == od) & (i < oi));
    const bool take = (lower == asc) ? o_lt : m_lt;
    d = take ? od : d;
    i = take ? oi : i;
}

template <typename Id>
__device__ __forceinline__ void sort64(float& d, Id& i, int lane) {
    static_for<6>([&](auto L) {  // size = 2 << L
        constexpr int size = 2 << decltype(L)::value;
        const bool asc = (lane & size) == 0;
        static_for<decltype(L)::value + 1>([&](auto T) {  // stride = size / 2 >> T
            constexpr int stride = (size >> 1) >> decltype(T)::value;
            cmpx_s<stride>(d, i, lane, asc);
        });
    });
}

template <typename Id>
__device__ __forceinline__ void merge64(float& d, Id& i, int lane) {  // bitonic -> ascending
    static_for<6>([&](auto T) { cmpx_s<(32 >> decltype(T)::value)>(d, i, lane, true); });
}

// best (ascending, one per lane) <- the 64 smallest of best U cand (cand sorted ascending)
template <typename Id>
__device__ __forceinline__ void merge_into(float& bd, Id& bi, float cd, Id ci, int lane) {
    float rd = __shfl(cd, 63 - lane, 64);
    Id ri = __shfl(ci, 63 - lane, 64);
    if (key_lt(rd, ri, bd, bi)) { bd = rd; bi = ri; }
    merge64(bd, bi, lane);
}

// butterfly sums with the partner exchange on the VALU (DPP / permlane:
// lane_xor) instead of ds_bpermute; the same addition order as a
// __shfl_xor loop over 32, 16, .., 1, so the same result bit for bit
__device__ __forceinline__ double wave_sum_f64(double v) {
    const int lane = __lane_id();
    static_for<6>([&](auto T) {
        constexpr int S = 32 >> decltype(T)::value;
        v += __longlong_as_double(lane_xor<S>((long long)__double_as_longlong(v), lane));
    });
    return v;
}
__device__ __forceinline__ float wave_sum_f32(float v) {
    const int lane = __lane_id();
    static_for<6>([&](auto T) {
        constexpr int S = 32 >> decltype(T)::value;
        v += lane_xor<S>(v, lane);
    });
    return v;
}


// LDS byte offset of a generic pointer into the extern LDS array
__device__ __forceinline__ uint32_t lds_off(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__device__ __forceinline__ void glds16(const void* gsrc, char* lds_uniform) {
    __builtin_amdgcn_global_load_lds(gsrc, (__attribute__((address_space(3))) void*)lds_uniform, 16, 0, 0);
}

// blockIdx -> (query tile, corpus split) over `ntl` query tiles of 128.
// Placement only changes speed, never results; both forms rely on the
// observed round-robin dispatch of blocks over the 8 XCDs (b, b + 8, ... share
// one XCD).
//   place 0: with >= 8 query tiles each XCD group owns a fixed set of query
//            tiles and all groups walk the corpus splits in the same order
//            (corpus rows re-read from L2 / the Infinity Cache);
//   place 1: corpus-partitioned -- XCD group x owns splits [x sx, (x+1) sx)
//            for every query tile and walks them query-tile-major, so the
//            ~32 blocks resident on an XCD stream the same split side by side
//            and the XCD's L2 serves one corpus fetch to all of them.
__device__ __forceinline__ void map_tile(int b, const ScanParams& p, int ntl, int& qtile, int& split) {
    if (p.place == 1) {
        const int xcd = b & 7, j = b >> 3;
        qtile = j % ntl;
        split = xcd * p.sx + j / ntl;
    } else if (p.qt_per_xcd > 0) {
        const int xcd = b & 7, j = b >> 3;
        qtile = xcd + 8 * (j % p.qt_per_xcd);
        split = j / p.qt_per_xcd;
    } else {
        qtile = b % ntl;
        split = b / ntl;
    }
}
__device__ __forceinline__ void map_block(int b, const ScanParams& p, int& qtile, int& split) {
    map_tile(b, p, p.n_qtiles, qtile, split);
}

// diagnostics (FX_SCAN_TRACE): where and when each block ran
__device__ __noinline__ void trace_block_start(const ScanParams& p, int qtile, int split) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned long long* t = p.trace + blockIdx.x * 4;
    t[0] = (unsigned long long)(xcc & 0xf) | ((unsigned long long)(hw & 0xffffff) << 8) |
           ((unsigned long long)qtile << 32);
    t[1] = (unsigned long long)split;
    t[2] = wall_clock64();
}

// order-preserving float <-> uint (atomicMin on floats of either sign)
__device__ __forceinline__ unsigned f2ord(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// ---------------------------------------------------------------------------
// block-wide (256 threads) top-K in LDS for any K <= FX_BIG_K: the paths that
// are not the fused scan's fixed KP = 32 lists (k > KP refine, the exact
// fallback, the k > 64 shard merge).  A candidate buffer of B = pow2 >= K +
// 256 (key, id) pairs; each round every thread offers at most one candidate
// that beats the running K-th (ties -> smaller id); before a round could
// overflow the buffer it is bitonic-sorted and cut to its K best.
// ---------------------------------------------------------------------------
constexpr int BT_THREADS = 256;
constexpr int BT_MAXK = 2 * FX_BIG_K;  // largest K of a block top-K (k_refine_big's K1)
constexpr int BT_MAXB = 4096;          // pow2 >= BT_MAXK + BT_THREADS

template <typename Id>
struct BtState {  // in LDS
    int cnt;
    int total;  // valid candidates offered so far
    float thr;
    Id thr_i;
};

template <typename Id> __device__ __forceinline__ Id bt_none();
template <> __device__ __forceinline__ int bt_none<int>() { return INT_MAX; }
template <> __device__ __forceinline__ long long bt_none<long long>() { return LLONG_MAX; }

__device__ __forceinline__ int bt_cap(int K) {
    int b = 256;
    while (b < K + BT_THREADS) b <<= 1;
    return b;
}

template <typename Id>
__device__ __forceinline__ void bt_init(BtState<Id>* st) {
    if (threadIdx.x == 0) {
        st->cnt = 0;
        st->total = 0;
        st->thr = FX_INF;
        st->thr_i = bt_none<Id>();
    }
    __syncthreads();
}

// ascending bitonic sort of (d, i)[0, n), n a power of two, all 256 threads
template <typename Id>
__device__ __forceinline__ void bt_sort(float* d, Id* i, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int t = threadIdx.x; t < n / 2; t += BT_THREADS) {
                const int lo = (t / stride) * 2 * stride + (t % stride), hi = lo + stride;
                const bool asc = (lo & size) == 0;
                const float dl = d[lo], dh = d[hi];
                const Id il = i[lo], ih = i[hi];
                if (asc ? key_lt(dh, ih, dl, il) : key_lt(dl, il, dh, ih)) {
                    d[lo] = dh;
                    d[hi] = dl;
                    i[lo] = ih;
                    i[hi] = il;
                }
            }
        }
    }
    __syncthreads();
}

// sort the buffer and keep its K best; afterwards d/i[0, cnt) is ascending
template <typename Id>
__device__ __forceinline__ void bt_flush(float* d, Id* i, BtState<Id>* st, int K, int B) {
    __syncthreads();
    const int c = st->cnt;
    for (int t = c + threadIdx.x; t < B; t += BT_THREADS) {
        d[t] = FX_INF;
        i[t] = bt_none<Id>();
    }
    bt_sort(d, i, B);
    if (threadIdx.x == 0) {
        st->cnt = c < K ? c : K;
        if (c >= K) {
            st->thr = d[K - 1];
            st->thr_i = i[K - 1];
        }
    }
    __syncthreads();
}

// one round: every thread offers (key, id) when `valid`; call with all 256
// threads; flushes first when the round could overflow
template <typename Id>
__device__ __forceinline__ void bt_round(float* d, Id* i, BtState<Id>* st, int K, int B, float key, Id id,
                                         bool valid) {
    __syncthreads();
    if (st->cnt > B - BT_THREADS) bt_flush(d, i, st, K, B);
    if (valid) {
        atomicAdd(&st->total, 1);
        if (key_lt(key, id, st->thr, st->thr_i)) {
            const int pos = atomicAdd(&st->cnt, 1);
            d[pos] = key;
            i[pos] = id;
        }
    }
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

// f32: a 64-B k-chunk is 4 k-steps of 16x16x4 (see Frag<F32>); B is kept as 4
// scalar AGPRs per chunk.
struct Bf32 { float x[4]; };

// MFMAs as inline asm (the B operand pinned in AGPRs: the builtin form left
// the stationary query fragments to the allocator, which spilled them).
// Accumulators are "+v" operands even where srcC is an initialiser, so they
// keep fixed registers across tiles.  mma2* issue the two query columns n = 0,
// 1 of one A fragment; INIT: 0 accumulate, 1 srcC = c_init (row norms), 2
// srcC = 0.  hipcc does not see the latency of these MFMAs: every register
// they read must stay unwritten until they have read it (the scan keeps its
// operand registers live and pinned, see fx_scan.hip) and acc_fence_v pads
// the XDL-write -> VALU-read wait states before an epilogue reads them.
template <int DT> struct AsmMmaV;
template <> struct AsmMmaV<BF16> {
    typedef bf16x8 A;
    typedef bf16x8 B;
    static __device__ __forceinline__ void settle(const B& b) { asm volatile("" ::"a"(b)); }
    template <int INIT>
    static __device__ __forceinline__ void mma2(f32x4& c0, f32x4& c1, const A& a, const B& b0, const B& b1,
                                                const f32x4& ci) {
        if constexpr (INIT == 0) {
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
                         "v_mfma_f32_16x16x32_bf16 %1, %2, %4, %1"
                         : "+v"(c0), "+v"(c1) : "v"(a), "a"(b0), "a"(b1));
        } else if constexpr (INIT == 1) {
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %3, %5\n\t"
                         "v_mfma_f32_16x16x32_bf16 %1, %2, %4, %5"
                         : "+v"(c0), "+v"(c1) : "v"(a), "a"(b0), "a"(b1), "v"(ci));
        } else {
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %3, 0\n\t"
                         "v_mfma_f32_16x16x32_bf16 %1, %2, %4, 0"
                         : "+v"(c0), "+v"(c1) : "v"(a), "a"(b0), "a"(b1));
        }
    }
};
template <> struct AsmMmaV<F16> {
    typedef f16x8 A;
    typedef f16x8 B;
    static __device__ __forceinline__ void settle(const B& b) { asm volatile("" ::"a"(b)); }
    template <int INIT>
    static __device__ __forceinline__ void mma2(f32x4& c0, f32x4& c1, const A& a, const B& b0, const B& b1,
                                                const f32x4& ci) {
        if constexpr (INIT == 0) {
            asm volatile("v_mfma_f32_16x16x32_f16 %0, %2, %3, %0\n\t"
                         "v_mfma_f32_16x16x32_f16 %1, %2, %4, %1"
                         : "+v"(c0), "+v"(c1) : "v"(a), "a"(b0), "a"(b1));
        } else if constexpr (INIT == 1) {
            asm volatile("v_mfma_f32_16x16x32_f16 %0, %2, %3, %5\n\t"
                         "v_mfma_f32_16x16x32_f16 %1, %2, %4, %5"
                         : "+v"(c0), "+v"(c1) : "v"(a), "a"(b0), "a"(b1), "v"(ci));
        } else {
            asm volatile("v_mfma_f32_16x16x32_f16 %0, %2, %3, 0\n\t"
                         "v_mfma_f32_16x16x32_f16 %1, %2, %4, 0"
                         : "+v"(c0), "+v"(c1) : "v"(a), "a"(b0), "a"(b1));
        }
    }
};
// F32S (split fp32) runs on the bf16 pipe; the scan issues the extra products
template <> struct AsmMmaV<F32S> : AsmMmaV<BF16> {};
// f32: a 64-B k-chunk is 4 k-steps of 16x16x4; the two columns' dependent
// chains are interleaved (40-cycle dependent latency vs 32-cycle issue)
template <> struct AsmMmaV<F32> {
    typedef f32x4 A;
    typedef Bf32 B;
    static __device__ __forceinline__ void settle(const B& b) {
        asm volatile("" ::"a"(b.x[0]), "a"(b.x[1]), "a"(b.x[2]), "a"(b.x[3]));
    }
    template <int INIT>
    static __device__ __forceinline__ void mma2(f32x4& c0, f32x4& c1, const A& a, const B& b0, const B& b1,
                                                const f32x4& ci) {
#define FX_F32_TAIL                                            \
    "v_mfma_f32_16x16x4_f32 %0, %3, %7, %0\n\t"                \
    "v_mfma_f32_16x16x4_f32 %1, %3, %11, %1\n\t"               \
    "v_mfma_f32_16x16x4_f32 %0, %4, %8, %0\n\t"                \
    "v_mfma_f32_16x16x4_f32 %1, %4, %12, %1\n\t"               \
    "v_mfma_f32_16x16x4_f32 %0, %5, %9, %0\n\t"                \
    "v_mfma_f32_16x16x4_f32 %1, %5, %13, %1"
#define FX_F32_OPS                                                                                      \
    : "+v"(c0), "+v"(c1)                                                                                \
    : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "a"(b0.x[0]), "a"(b0.x[1]), "a"(b0.x[2]), "a"(b0.x[3]), \
      "a"(b1.x[0]), "a"(b1.x[1]), "a"(b1.x[2]), "a"(b1.x[3]), "v"(ci)
        // operands: %2..%5 = a[0..3], %6..%9 = b0, %10..%13 = b1, %14 = ci
        if constexpr (INIT == 0) {
            asm volatile("v_mfma_f32_16x16x4_f32 %0, %2, %6, %0\n\t"
                         "v_mfma_f32_16x16x4_f32 %1, %2, %10, %1\n\t" FX_F32_TAIL FX_F32_OPS);
        } else if constexpr (INIT == 1) {
            asm volatile("v_mfma_f32_16x16x4_f32 %0, %2, %6, %14\n\t"
                         "v_mfma_f32_16x16x4_f32 %1, %2, %10, %14\n\t" FX_F32_TAIL FX_F32_OPS);
        } else {
            asm volatile("v_mfma_f32_16x16x4_f32 %0, %2, %6, 0\n\t"
                         "v_mfma_f32_16x16x4_f32 %1, %2, %10, 0\n\t" FX_F32_TAIL FX_F32_OPS);
        }
#undef FX_F32_TAIL
#undef FX_F32_OPS
    }
};

// 20 wait states before a VALU reads the accumulators: the XDL-write ->
// VALU-read requirement is (passes + 3) wait states, 19 for the longest
// (16-pass) MFMA; the scan's MFMAs have at most 8 passes, and the epilogue
// reads the last-written accumulators (acc[7][*]) only after 14 further VALU
// instructions.  (Was 48: each s_nop state costs a 4-cycle issue slot, so the
// pad cost ~190 cycles per tile.)
__device__ __forceinline__ void acc_fence_v(f32x4 (&acc)[8][2]) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
                 : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[1][0]), "+v"(acc[1][1]), "+v"(acc[2][0]),
                   "+v"(acc[2][1]), "+v"(acc[3][0]), "+v"(acc[3][1]), "+v"(acc[4][0]), "+v"(acc[4][1]),
                   "+v"(acc[5][0]), "+v"(acc[5][1]), "+v"(acc[6][0]), "+v"(acc[6][1]), "+v"(acc[7][0]),
                   "+v"(acc[7][1]));
}

}  // namespace fx
