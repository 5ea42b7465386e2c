// fx_scan_common.h -- device helpers shared by the MFMA scan kernels
// (fx_scan.hip: k_scan_v4; fx_scan_q32.hip: k_scan_q32):
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

// Compact this wave's full lists (cnt >= CAP) to their KP best; tau = KP-th,
// published to the shared per-query threshold.  Lists are owned by one wave.
__device__ __noinline__ void compact_wave(float* lst_d, int* lst_i, int* cnt, float* tau, unsigned* gtq, int qw0,
                                          int lane) {
    for (int qi = 0; qi < 32; ++qi) {
        const int q = qw0 + qi;
        if (cnt[q] >= CAP) {
            float d = lst_d[q * CAP + lane];
            int i = lst_i[q * CAP + lane];
            sort64(d, i, lane);
            if (lane < KP) {
                lst_d[q * CAP + lane] = d;
                lst_i[q * CAP + lane] = i;
            }
            if (lane == KP - 1) {
                tau[q] = d;
                if (gtq) atomicMin(gtq + qi, f2ord(d));  // null: no cross-split pruning (k > KP)
            }
            if (lane == 0) cnt[q] = KP;
        }
    }
}

// push the entries of accumulator group (m, n) selected by `elig` (4 bits)
// that pass `tn` into query q's list; entries that find the list full are
// recorded in `pend` (bit 4m+i) for a retry after compaction
template <int M, int N>
__device__ __forceinline__ bool push_group(const f32x4 (&acc)[M][N], int n, int m, unsigned elig, float tn, int q,
                                           int row0, int rlim, float* lst_d, int* lst_i, int* cnt, unsigned& pend) {
    bool ovf = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float v = acc[m][n][i];
        const int rl = row0 + i;
        if (((elig >> i) & 1u) && v <= tn && rl < rlim) {
            const int s = atomicAdd(&cnt[q], 1);
            if (s < CAP) {
                lst_d[q * CAP + s] = v;
                lst_i[q * CAP + s] = rl;
            } else {
                pend |= 1u << (m * 4 + i);
                ovf = true;
            }
        }
    }
    return ovf;
}

}  // namespace fx
