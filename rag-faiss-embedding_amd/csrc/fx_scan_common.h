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

template <int... Is, typename F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(std::make_integer_sequence<int, N>{}, f);
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

// A bound on the rank-th smallest key of the union of `nl` published lists
// (float keys, `stride` apart, the first 16 entries of each read: 4 per lane
// for up to 16 lists): the smallest v found by 8 bisection steps over the
// ordered-uint range [lo, hi] such that at least `rank` entries are <= v (hi
// = the caller's own rank-th key, which already qualifies).  Counting entries
// is a valid lower bound on the rows below v (see compact_wave), so any v the
// bisection accepts bounds the global rank-th key.
__device__ __forceinline__ unsigned union_kth(const float* lists, int nl, int stride, unsigned hi, int rank,
                                              int lane) {
    unsigned kv[4];
    unsigned lo = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int l = (lane >> 4) + 4 * i, e = lane & 15;  // list l, entry e
        kv[i] = l < nl ? f2ord(__hip_atomic_load(lists + l * stride + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                       : 0xFFFFFFFFu;
        lo = kv[i] < lo ? kv[i] : lo;
    }
    // wave minimum: the answer lies in [lo, hi]
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned t = __shfl_xor(lo, o, 64);
        lo = t < lo ? t : lo;
    }
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

// Compact this wave's full lists (cnt >= CAP) to their KP best; tau = KP-th,
// published to the shared per-query threshold.  Lists are owned by one wave.
// The 32 counts are read in one LDS access (lane i: query qw0 + i) and only
// the full lists are visited.
//
// pub (k_scan_v4, k <= KP): the compacted list is also published to
// pub[query][split][KP], and the shared threshold becomes the KP-th smallest
// key of the union of the published lists of up to 16 splits (this one's
// window of 16) -- a valid bound on the query's global KP-th key, because
// every published entry is the key of a distinct row of its split (a list
// read while its split rewrites it mixes two versions of the same
// improving list: entry i of either version still has i + 1 rows of that
// split at or below it, so counting entries never over-counts rows).  A
// split that starts late then prunes with what all earlier splits found,
// not only with the best single split's KP-th key.  rank (<= 16, >= k): the
// union bound is taken at this rank, below KP -- every dropped row then lies
// above the final shared threshold, which k_refine folds into its
// certification bound (RefineParams.gtau).
__device__ __noinline__ void compact_wave(float* lst_d, int* lst_i, int* cnt, float* tau, unsigned* gtq, int qw0,
                                          int lane, float* pub = nullptr, int splits = 0, int split = 0,
                                          int rank = KP) {
    uint64_t full = __builtin_amdgcn_ballot_w64(lane < 32 && cnt[qw0 + (lane & 31)] >= CAP);
    while (full) {
        const int qi = __builtin_ctzll(full);
        full &= full - 1;
        const int q = qw0 + qi;
        float d = lst_d[q * CAP + lane];
        int i = lst_i[q * CAP + lane];
        sort64(d, i, lane);
        if (lane < KP) {
            lst_d[q * CAP + lane] = d;
            lst_i[q * CAP + lane] = i;
        }
        // the list keeps KP entries; the threshold is its rank-th key (rank
        // = KP unless the union bound is on): published to gtau too, so the
        // final gtau stays below every split's local threshold (k_refine)
        if (lane == rank - 1) {
            tau[q] = d;
            if (gtq) atomicMin(gtq + qi, f2ord(d));  // null: no cross-split pruning (k > KP)
        }
        if (lane == 0) cnt[q] = KP;
        if (pub && gtq) {
            float* qp = pub + (int64_t)qi * splits * KP;  // pub: this wave's first query
            if (lane < KP) __hip_atomic_store(qp + split * KP + lane, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int w0 = split & ~15;
            const int nsp = splits - w0 < 16 ? splits - w0 : 16;
            const unsigned own = f2ord(__shfl(d, rank - 1, 64));
            const unsigned v = union_kth(qp + w0 * KP, nsp, KP, own, rank, lane);
            if (lane == 0 && v < own) atomicMin(gtq + qi, v);
        }
    }
}

// push the entries of accumulator group (m, n) selected by `elig` (4 bits)
// that pass `tn` into query q's list; entries that find the list full are
// recorded in `pend` (bit 4m+i) for a retry after compaction.  One LDS atomic
// per lane reserves all of its slots (the list belongs to this wave; the
// atomic only orders the four lanes that hold query q), so a push costs one
// LDS round trip however many of the lane's 4 rows pass.
template <int M, int N, int CAPL = CAP>
__device__ __forceinline__ bool push_group(const f32x4 (&acc)[M][N], int n, int m, unsigned elig, float tn, int q,
                                           int row0, int rlim, float* lst_d, int* lst_i, int* cnt, unsigned& pend) {
    unsigned msk = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (((elig >> i) & 1u) && acc[m][n][i] <= tn && row0 + i < rlim) msk |= 1u << i;
    bool ovf = false;
    if (msk) {
        int s = atomicAdd(&cnt[q], __popc(msk));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if ((msk >> i) & 1u) {
                if (s < CAPL) {
                    lst_d[q * CAPL + s] = acc[m][n][i];
                    lst_i[q * CAPL + s] = row0 + i;
                } else {
                    pend |= 1u << (m * 4 + i);
                    ovf = true;
                }
                ++s;
            }
        }
    }
    return ovf;
}

// LDS store through an explicit byte offset (the lean push below picks the
// offset per lane instead of branching)
__device__ __forceinline__ void ds_wr32(uint32_t off, float v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(off), "v"(v) : "memory");
}
__device__ __forceinline__ void ds_wr32(uint32_t off, int v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(off), "v"(v) : "memory");
}

// push_group without divergent branches (k_scan_v4's slow path): every lane
// takes one LDS atomic on cnt[q] (adding 0 when none of its 4 rows passes)
// and stores all 4 of its entries -- entries that do not pass, or find the
// list full, go to the wave's trash word `trash` instead of a list slot.  The
// group costs a fixed ~50 instructions and one LDS round trip, however the
// passing rows are spread over the lanes.  ld / li: LDS byte offsets of the
// key and row arrays ([query][CAP]).
template <int M, int N>
__device__ __forceinline__ bool push_lean(const f32x4 (&acc)[M][N], int n, int m, unsigned elig, float tn, int q,
                                          int row0, int rlim, uint32_t ld, uint32_t li, uint32_t trash, int* cnt,
                                          unsigned& pend) {
    unsigned msk = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) msk |= (acc[m][n][i] <= tn && row0 + i < rlim) ? (1u << i) : 0u;
    msk &= elig;
    const int s = atomicAdd(&cnt[q], (int)__popc(msk));
    unsigned late = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int slot = s + (int)__popc(msk & ((1u << i) - 1u));
        const bool take = (msk >> i) & 1u;
        const bool ok = take && slot < CAP;
        const uint32_t e = (uint32_t)(q * CAP + slot) * 4u;
        ds_wr32(ok ? ld + e : trash, acc[m][n][i]);
        ds_wr32(ok ? li + e : trash, row0 + i);
        late |= (take && !ok) ? (1u << i) : 0u;
    }
    pend |= late << (4 * m);
    return late != 0u;
}

// minimum of the 4 keys of an accumulator group: two VALU ops (fminf would
// canonicalise every operand first).  volatile: it stays where it is placed
// among the asm MFMAs (the caller keeps >= 2 MFMA pairs between the last XDL
// write of `a` and this read; hipcc does not see the asm MFMAs' hazards)
__device__ __forceinline__ float min4(const f32x4& a) {
    float t, r;
    asm volatile("v_min_f32 %0, %1, %2" : "=v"(t) : "v"(a[2]), "v"(a[3]));
    asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a[0]), "v"(a[1]), "v"(t));
    return r;
}

}  // namespace fx
