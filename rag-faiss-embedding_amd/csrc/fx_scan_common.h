// fx_scan_common.h -- device helpers shared by the MFMA scan kernels
// (fx_scan.hip: k_scan_v4):
// LDS-DMA pieces with scalar bases, pinned LDS->operand reads, per-wave
// candidate lists.
#pragma once
#include "fx_device.h"

#include <utility>

namespace fx {

// Largest finite float: thresholds start here, so real keys always pass and
// padding rows (|y|^2 = +inf -> key +inf) never do.
constexpr float KEY_MAX = FLT_MAX;
// k_scan_v4's per-query LDS list capacity (KP < LCAP <= 64, one sort64 lane
// per entry); 64 in the product, 48 in the 6-slot-ring A/B build (FX_RING6:
// the lists then compact at 48 = capacity, entries past it wait in pend)
#ifndef FX_LCAP
#define FX_LCAP 64
#endif
constexpr int LCAP = FX_LCAP;
static_assert(LCAP > KP && LCAP <= 64, "list capacity");
// global-address-space float: loads through it are global_load (vmcnt only),
// not flat (which also counts against lgkmcnt as a possible LDS access)
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) unsigned guint;
// relaxed agent-scope atomicMin through a global pointer (global_atomic_umin:
// no lgkmcnt, so later LDS accesses do not wait for it)
__device__ __forceinline__ void gmin_u32(unsigned* p, unsigned v) {
    __hip_atomic_fetch_min((guint*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// one 1 KiB LDS-DMA piece: lane l moves 16 B from sbase + voff + OFF to
// LDS[lds + 16 l].  The instruction offset is added to the LDS address as
// well (LDS = M0 + OFF + 16 lane), so M0 is set to lds - OFF (>= 0: the ring
// starts at 4 KiB, OFF < 1.5 KiB).  The s_nop is the M0-write -> LDS-DMA wait
// state; NOP = 4 also covers a base SGPR the compiler has just written with
// v_readfirstlane (VALU-written SGPR -> VMEM: 5 wait states, which hipcc does
// not insert in front of inline asm).
template <int OFF, int NOP = 0>
__device__ __forceinline__ void dma_piece(uint32_t voff, const char* sbase, uint32_t lds) {
    static_assert(OFF >= 0 && OFF < 4096, "M0 = lds - OFF must not wrap (rings start at >= 4 KiB)");
    static_assert(NOP >= 0 && NOP <= 7, "s_nop range");
    asm volatile("s_nop %3\n\tglobal_load_lds_dwordx4 %0, %1 offset:%2" ::"v"(voff), "s"(sbase), "i"(OFF),
                 "i"(NOP), "{m0}"(lds - OFF)
                 : "memory");
}
// a wave-uniform pointer, asserted so (the "s" operand of dma_piece needs it in
// an SGPR pair; hipcc's divergence analysis does not always prove it)
__device__ __forceinline__ const char* sgpr_ptr(const char* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const char*)(((uint64_t)hi << 32) | lo);
}
// the per-stage row-norm / threshold piece: lanes 0-7 move 32 row norms,
// lanes 8-15 the wave's 32 shared thresholds; lanes 16-63 are masked off
__device__ __forceinline__ void dma_norm_piece(const char* vaddr, uint32_t m0) {
    uint64_t saved;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, 0xffff\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "v"(vaddr), "{m0}"(m0)
        : "memory");
}
// LDS -> MFMA operand registers.  "+v": the destination keeps its register
// for the whole kernel (no other value is ever placed there), so the only
// writes to an operand register are these reads, scheduled >= 8 MFMAs after
// the register's last MFMA reader
template <int OFF, typename T>
__device__ __forceinline__ void ds_rd128(T& d, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "+v"(d) : "v"(addr), "i"(OFF) : "memory");
}
template <int OFF, typename T>
__device__ __forceinline__ void ds_rd32(T& d, uint32_t addr) {
    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
}

// A bound on the rank-th smallest key of the union of up to 16 published
// lists (float keys, their first 16 entries: 4 per lane, as ordered uints in
// kv, 0xFFFFFFFF where absent): the smallest v found by 8 bisection steps
// over the ordered-uint range [lo, hi] such that at least `rank` entries are
// <= v (hi = the caller's own rank-th key, which already qualifies).  Counting
// entries is a valid lower bound on the rows below v (see compact_regs), so
// any v the bisection accepts bounds the global rank-th key.
__device__ __forceinline__ unsigned union_kth_v(const unsigned (&kv)[4], unsigned hi, int rank) {
    unsigned lo = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < 4; ++i) lo = kv[i] < lo ? kv[i] : lo;
    // wave minimum: the answer lies in [lo, hi]
    const int lane = __lane_id();
    static_for<6>([&](auto T) {
        const unsigned t = (unsigned)lane_xor<(32 >> decltype(T)::value)>((int)lo, lane);
        lo = t < lo ? t : lo;
    });
    for (int it = 0; it < 8 && lo < hi; ++it) {
        const unsigned mid = lo + (hi - lo) / 2;
        int c = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) c += __popcll(__builtin_amdgcn_ballot_w64(kv[i] <= mid));
        if (c >= rank) hi = mid;
        else lo = mid + 1;
    }
    return hi;
}

// Wave-level (64-lane) bitonic sort of (key, row) entries packed as one
// 64-bit value, hi = f2ord(key), lo = row: the packed order is (key asc, row
// asc) -- the lists' order, -0 before +0 aside (harmless: only which of two
// equal-keyed candidates is kept can differ).  Each step: the partner's two
// words by DPP / permlane, ONE 64-bit compare, and the per-lane direction
// folded into a compile-time lane mask (up_mask) applied on the SALU, so a
// step is ~8 instructions instead of ~25 for sort64's float + id compares.
constexpr uint64_t up_mask(int S, int size) {  // lanes that keep the smaller of (lane, lane ^ S)
    uint64_t m = 0;
    for (int l = 0; l < 64; ++l)
        if (((l & S) == 0) == ((l & size) == 0)) m |= 1ull << l;
    return m;
}
__device__ __forceinline__ uint32_t sel_mask(uint64_t m, uint32_t a, uint32_t b) {  // lane in m ? b : a
    uint32_t r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
template <int S, int SIZE>
__device__ __forceinline__ void cmpx_packed(uint32_t& hi, uint32_t& lo, int lane) {
    const uint32_t ohi = (uint32_t)lane_xor<S>((int)hi, lane), olo = (uint32_t)lane_xor<S>((int)lo, lane);
    const uint64_t o = ((uint64_t)ohi << 32) | olo, v = ((uint64_t)hi << 32) | lo;
    // take the partner's entry where (partner < mine) == (this lane keeps the smaller)
    const uint64_t take = ~(__builtin_amdgcn_ballot_w64(o < v) ^ up_mask(S, SIZE));
    hi = sel_mask(take, hi, ohi);
    lo = sel_mask(take, lo, olo);
}
// all 64 lanes active; ascending over the lanes afterwards
__device__ __forceinline__ void sort64_packed(uint32_t& hi, uint32_t& lo, int lane) {
    static_for<6>([&](auto L) {
        constexpr int size = 2 << decltype(L)::value;
        static_for<decltype(L)::value + 1>([&](auto T) {
            constexpr int stride = (size >> 1) >> decltype(T)::value;
            cmpx_packed<stride, size>(hi, lo, lane);
        });
    });
}
// a list slot -> its packed entry (lanes past the live count: (+inf, INT_MAX))
__device__ __forceinline__ void load_packed(const float* lst_d, const int* lst_i, int idx, bool live, uint32_t& hi,
                                            uint32_t& lo) {
    hi = live ? f2ord(lst_d[idx]) : f2ord(FX_INF);
    lo = live ? (uint32_t)lst_i[idx] : (uint32_t)INT_MAX;
}

// Per-wave candidate lists of k_scan_v4.  The wave owns 32 queries: query
// column c of accumulator half n (lanes with lane & 15 == c, n = 0, 1) is
// tile-local query qw0 + 16 n + c.  Each list lives in LDS ([query][LCAP keys |
// LCAP rows]); its entry count and its pruning threshold live in registers
// (cntv[n], tauv[n]), the same value in the 4 lanes that hold the query, so a
// push reserves its slots without an LDS atomic round trip.

// Exclusive prefix and total of `c` over the 4 lanes that hold one query
// (lane >> 4 = 0..3, the same lane & 15).
__device__ __forceinline__ void quad_prefix(int c, int lane, int& excl, int& total) {
    const int a = lane_xor16(c, lane);
    const int s2 = c + a;
    const int b = lane_xor32(s2, lane);
    excl = ((lane & 16) ? a : 0) + ((lane & 32) ? b : 0);
    total = s2 + b;
}

// A query's list in LDS: LCAP keys, then LCAP row ids (LSTRIDE words), so one
// ds_write2_b32 (offset1 = LCAP dwords) stores an entry's key and row.
constexpr int LSTRIDE = 2 * LCAP;
__device__ __forceinline__ void ds_wr_entry(uint32_t off, float key, int row) {
    asm volatile("ds_write2_b32 %0, %1, %2 offset1:%3" ::"v"(off), "v"(key), "v"(row), "i"(LCAP) : "memory");
}

// Push the 4 entries of one accumulator group (this lane's rows row0 .. row0+3
// of its query) that pass `tn` (and, RETRY, are selected by `elig`) into the
// query's list.  Entries that find the list full are returned as bits in
// `late` for a retry after compaction (the caller ORs them into pend at bit
// 4m+i).  Branch-free per lane: a lane stores all 4 entries, those that do not
// pass into the wave's trash slot (trash .. trash + 4 LCAP); the rare group
// that could overflow a list takes the per-entry slot check.  Rows of the
// index's padding never pass: the caller sets their keys to +inf (the edge
// tile), so no row bound is tested here.
template <bool RETRY>
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
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(s + c > LCAP) == 0, 1)) {
        uint32_t e = lq + (uint32_t)s * 4u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            ds_wr_entry(p[i] ? e : trash, a[i], row0 + i);
            e += p[i] ? 4u : 0u;
        }
    } else {
        int slot = s;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool ok = p[i] && slot < LCAP;
            ds_wr_entry(ok ? lq + (uint32_t)slot * 4u : trash, a[i], row0 + i);
            late |= (p[i] && !ok) ? (1u << i) : 0u;
            slot += (int)p[i];
        }
    }
    return late;
}

// Compact this wave's lists that hold `at` or more entries (KP < at <= LCAP)
// to their KP best; the list's threshold becomes its rank-th key (rank = KP
// unless the union bound is on), published to the shared per-query threshold.
// A list's threshold only improves here, so compacting before the list is
// full (at < LCAP) trades more compactions for fewer slow-path tiles.
//
// pub (k <= KP): the compacted list is also published to pub[query][split][KP],
// and the shared threshold becomes the rank-th smallest key of the union of
// the published lists of the uw splits of this one's window (their first
// 256 / uw keys each) -- a valid
// bound on the query's global rank-th key, because every published entry is
// the key of a distinct row of its split (a list read while its split
// rewrites it mixes two versions of the same improving list: entry i of
// either version still has i + 1 rows of that split at or below it, so
// counting entries never over-counts rows).  A split that starts late then
// prunes with what all earlier splits found.  rank (>= k): every dropped row
// lies above the final shared threshold, which k_refine folds into its
// certification bound (RefineParams.gtau).  The union reads of the full
// lists are issued together (one memory round trip per 4 lists, not one per
// list).
//
// defer (option union_defer): the window of up to two compacted lists is
// fetched by LDS-DMA into the wave's two union slots (1 KiB each: the
// window's 256 keys, 4 per lane) and bounded at the next tile's epilogue
// (union_finish) -- by then the DMA ring's counted stage waits have retired
// it (>= 12 younger pieces, SPT >= 4 stages) -- so the global round trip runs
// under the next tile's MFMAs instead of in the slow path.  upq[u]: the
// wave-local query of slot u, -1 free.  The window's LDS-DMA is a plain
// (non-coherent) global_load_lds, unlike the in-place path's agent-scope
// atomic loads, so it may see an older version of a published list from this
// XCD's L2.  That is safe by monotonicity: pub is reset to +inf before every
// search and a split only ever republishes a list whose entry i is <= the
// previous one's entry i (the KP best of a superset), so a stale entry is a
// larger key, i.e. a looser but still valid bound.  Windows still pending
// when a block's tile loop ends are not bounded (the bound only prunes; a
// skipped one costs speed, never a result).
struct ListRegs {
    int cnt[2];
    float tau[2];
};
// log2 of the published keys each split of a union window contributes
__device__ __forceinline__ int union_le(int uw) { return uw >= 64 ? 2 : uw >= 32 ? 3 : 4; }
__device__ __forceinline__ void union_finish(int (&upq)[2], const float* uslot, const ListRegs& r, unsigned* gtq,
                                             int splits, int split, int rank, int uw, int lane) {
    const int le = union_le(uw);
    const int w0 = split & ~(uw - 1);
    const int nsp = splits - w0 < uw ? splits - w0 : uw;
    const bool in_win = (lane >> (le - 2)) < nsp;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if (upq[u] < 0) continue;
        const int qi = upq[u];
        // a compiler-visible LDS load: its consumers wait for it (an asm
        // ds_read's result could be read before an asm lgkmcnt wait)
        const f32x4 raw = *(const f32x4*)(uslot + u * 256 + lane * 4);
        unsigned kv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) kv[j] = in_win ? f2ord(raw[j]) : 0xFFFFFFFFu;
        const unsigned own = f2ord(readlane_f(qi < 16 ? r.tau[0] : r.tau[1], qi & 15));
        const unsigned v = union_kth_v(kv, own, rank);
        if (lane == 0 && v < own) gmin_u32(gtq + qi, v);
        upq[u] = -1;
    }
}
__device__ __forceinline__ ListRegs compact_regs(float* lst, ListRegs r, unsigned* gtq, int qw0, int lane,
                                              float* pub, int splits, int split, int rank, int at, int uw,
                                              int (&upq)[2], float* uslot, int defer, int inplace_max) {
    float* lst_d = lst;                // keys of query q at q * LSTRIDE
    int* lst_i = (int*)(lst + LCAP);   // rows of query q at q * LSTRIDE
    int (&cntv)[2] = r.cnt;
    float (&tauv)[2] = r.tau;
    const uint64_t f0 = __builtin_amdgcn_ballot_w64(lane < 16 && cntv[0] >= at);
    const uint64_t f1 = __builtin_amdgcn_ballot_w64(lane < 16 && cntv[1] >= at);
    const uint64_t all = (f0 & 0xffffull) | ((f1 & 0xffffull) << 16);
    uint64_t full = all;
    while (full) {
        const int qi = __builtin_ctzll(full);
        full &= full - 1;
        const int q = qw0 + qi;
        // entries past the count are stale (rows of earlier rounds: kept or
        // dropped ones, so possibly duplicates) unless the list is full
        const int cq = __builtin_amdgcn_readlane(qi < 16 ? cntv[0] : cntv[1], qi & 15);
        // cq may exceed LCAP (overflowed pushes wait in `pend`): only the first
        // LCAP lanes hold entries of this list (lanes past it would read the
        // next query's row)
        const bool live = lane < cq && lane < LCAP;
        uint32_t hi, lo;
        load_packed(lst_d, lst_i, q * LSTRIDE + lane, live, hi, lo);
        sort64_packed(hi, lo, lane);
        const float d = ord2f(hi);
        const int i = (int)lo;
        if (lane < KP) {
            lst_d[q * LSTRIDE + lane] = d;
            lst_i[q * LSTRIDE + lane] = i;
        }
        const float dr = readlane_f(d, rank - 1);
        if ((lane & 15) == (qi & 15)) {
            if (qi < 16) { tauv[0] = dr; cntv[0] = KP; }
            else { tauv[1] = dr; cntv[1] = KP; }
        }
        // published to gtau too, so the final gtau stays below every split's
        // local threshold (k_refine); null gtq: no cross-split pruning (k > KP)
        if (gtq && lane == 0) gmin_u32(gtq + qi, f2ord(dr));
        if (pub && gtq && lane < KP)
            __hip_atomic_store((gfloat*)(pub + ((int64_t)qi * splits + split) * KP + lane), d, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!(pub && gtq)) return r;
    // union bounds: the window holds uw splits (16, 32 or 64) and their first
    // 256 / uw published keys (4 per lane)
    const int le = union_le(uw);  // log2(entries per list)
    const int w0 = split & ~(uw - 1);
    const int nsp = splits - w0 < uw ? splits - w0 : uw;
    uint64_t rest = all;
    // deferred: up to two windows fetched into the union slots (union_finish),
    // in the corpus pieces' form (scalar window base, per-lane byte offsets)
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
    // the rest now, up to 4 lists per memory round trip (at most inplace_max
    // lists: the others keep their own published bound until a later
    // compaction; the union only prunes)
    for (int done = 0; rest && done < inplace_max; done += 4) {
        int qs[4];
        unsigned kv[4][4];
        // (exactly inplace_max lists in all: a round takes at most what is left of it)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool take = rest != 0 && done + u < inplace_max;
            qs[u] = take ? __builtin_ctzll(rest) : -1;
            if (take) rest &= rest - 1;
        }
        // every lane loads unconditionally (absent lists read entry e of the
        // first list and are masked after the load): a load under a lane
        // condition becomes an exec-masked branch with its own vmcnt(0) wait,
        // which serialised the 16 round trips
        float raw[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const gfloat* lists = (const gfloat*)(pub + ((int64_t)(qs[u] < 0 ? 0 : qs[u]) * splits + w0) * KP);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int x = lane + 64 * j, l = x >> le, e = x & ((1 << le) - 1);  // list l, entry e
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
            const unsigned own = f2ord(readlane_f(qi < 16 ? tauv[0] : tauv[1], qi & 15));
            const unsigned v = union_kth_v(kv[u], own, rank);
            if (lane == 0 && v < own) gmin_u32(gtq + qi, v);
        }
    }
    return r;
}

// Re-bound the pruning threshold of this wave's list qi (wave-local query
// index) without compacting it (option tight_at): a bisection over the
// ordered-uint keys of its cq <= LCAP entries for the smallest v with at
// least `rank` entries <= v, starting from hi = the current threshold (which
// already qualifies: after a compaction it is the kept list's rank-th key,
// before one FLT_MAX).  Every entry is the key of a distinct row of this
// split, so v bounds the split's rank-th key: a valid threshold, published to
// the shared one too.  ~60 instructions per list against ~350 for a
// compaction, so thresholds can follow the pushes closely (fewer record tiles)
// while compactions happen only when a list is near full.
__device__ __forceinline__ void tighten_list(const float* lst_d, ListRegs& r, int qi, int q, int rank, unsigned* gtq,
                                             int lane) {
    const int cq = __builtin_amdgcn_readlane(qi < 16 ? r.cnt[0] : r.cnt[1], qi & 15);
    if (cq < rank) return;
    const unsigned kv = lane < cq ? f2ord(lst_d[q * LSTRIDE + lane]) : 0xFFFFFFFFu;
    unsigned hi = f2ord(readlane_f(qi < 16 ? r.tau[0] : r.tau[1], qi & 15));
    unsigned lo = kv;
    static_for<6>([&](auto T) {
        const unsigned t = (unsigned)lane_xor<(32 >> decltype(T)::value)>((int)lo, lane);
        lo = t < lo ? t : lo;
    });
    for (int it = 0; it < 8 && lo < hi; ++it) {
        const unsigned mid = lo + (hi - lo) / 2;
        if (__popcll(__builtin_amdgcn_ballot_w64(kv <= mid)) >= rank) hi = mid;
        else lo = mid + 1;
    }
    const float v = ord2f(hi);
    if ((lane & 15) == (qi & 15)) {
        if (qi < 16) r.tau[0] = fminf(r.tau[0], v);
        else r.tau[1] = fminf(r.tau[1], v);
    }
    if (gtq && lane == 0) gmin_u32(gtq + qi, hi);
}

// One MFMA of one query block with its B fragment in an AGPR (AG) or a VGPR:
// k_scan_v5's odd third block (72 B fragments at K = 768 do not fit the 256
// AGPRs) and k_scan_v4's one-live-block small batches.
template <int DT, int INIT, bool AG>
__device__ __forceinline__ void mma1(f32x4& c, const typename AsmMmaV<DT>::A& a, const typename AsmMmaV<DT>::B& b,
                                     const f32x4& ci) {
#define FX_M1(OP)                                                                                              \
    if constexpr (AG) {                                                                                        \
        if constexpr (INIT == 0) asm volatile(OP " %0, %1, %2, %0" : "+v"(c) : "v"(a), "a"(b));                \
        else if constexpr (INIT == 1) asm volatile(OP " %0, %1, %2, %3" : "+v"(c) : "v"(a), "a"(b), "v"(ci)); \
        else asm volatile(OP " %0, %1, %2, 0" : "+v"(c) : "v"(a), "a"(b));                                     \
    } else {                                                                                                   \
        if constexpr (INIT == 0) asm volatile(OP " %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));                \
        else if constexpr (INIT == 1) asm volatile(OP " %0, %1, %2, %3" : "+v"(c) : "v"(a), "v"(b), "v"(ci)); \
        else asm volatile(OP " %0, %1, %2, 0" : "+v"(c) : "v"(a), "v"(b));                                     \
    }
    if constexpr (DT == F16) {
        FX_M1("v_mfma_f32_16x16x32_f16")
    } else {
        FX_M1("v_mfma_f32_16x16x32_bf16")
    }
#undef FX_M1
}
// minima without fminf's operand canonicalisation (a v_max per operand: the
// compiler cannot see that asm results are canonical)
__device__ __forceinline__ float min_raw(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float min8_raw(const float (&g)[8]) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3\n\tv_min3_f32 %0, %0, %4, %5\n\t"
        "v_min3_f32 %0, %0, %6, %7\n\tv_min_f32 %0, %0, %8"
        : "=&v"(r)
        : "v"(g[0]), "v"(g[1]), "v"(g[2]), "v"(g[3]), "v"(g[4]), "v"(g[5]), "v"(g[6]), "v"(g[7]));
    return r;
}

// minimum of the 4 keys of an accumulator group: two VALU ops (fminf would
// canonicalise every operand first).  volatile: it stays where it is placed
// among the asm MFMAs (the caller keeps >= 2 MFMA pairs between the last XDL
// write of `a` and this read; hipcc does not see the asm MFMAs' hazards)
// One asm block: the compiler pads an s_nop between two inline-asm blocks
// where the second reads what the first wrote (it cannot see inside them).
__device__ __forceinline__ float min4(const f32x4& a) {
    float r;
    asm volatile("v_min3_f32 %0, %1, %2, %3\n\tv_min_f32 %0, %0, %4"
                 : "=&v"(r)
                 : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]));
    return r;
}

}  // namespace fx
