// fx_kernels.hip -- HIP/CDNA4 (gfx950) kernels of the flat vector index.
//
// Replaces the arithmetic faiss-cpu performs behind IndexFlatL2.add/search
// (faiss_store.py:46,64; rag_datastore_manager.py:173,218):
//
//   k_convert_rows   add(): dtype conversion into the HBM-resident, 128-B
//                    row-aligned code matrix + |y|^2 per row (+ opt-in row
//                    L2 normalisation) -- R rows per wave, grid-stride over
//                    4,096 workgroups, nontemporal, HBM-bound.
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
//   k_refine_big     the same for k > KP (block top-K in LDS, scan without
//                    the shared threshold).
//   k_fb_scan /      fallback for uncertified queries, gated on the device
//   k_fb_merge       (exit at once when none): exact fp64 scan of every row,
//                    then (D, id) top-k.
//   k_merge_shards   multi-GPU: merge G gathered per-shard top-k lists.
//   k_synth          counter-based synthetic corpus (oracle/flat_l2.c twin).
#include "fx_device.h"

#include <float.h>
#include <limits.h>
#include <stdlib.h>

namespace fx {

thread_local bool g_graph_capture = false;

// ---------------------------------------------------------------------------
// add(): convert rows into the code matrix, compute |y|^2
// ---------------------------------------------------------------------------
// One wave per row; each lane converts 16-B output chunks (4 fp32 or 8
// bf16/fp16 values) read with 16-B / 8-B vector loads when the input rows
// are 16-B aligned (`vec`), else element by element.  Elements past d are the
// row's zero padding.  |y|^2 of the stored values in fp32; the largest |y|^2
// (certification margin) is reduced per workgroup in LDS and published with
// one global atomicMax per workgroup.
__device__ __forceinline__ void load_chunk_in(const void* __restrict__ x, int x_dt, int64_t base, int e0, int d,
                                              int E, bool vec, float* v) {
    if (vec && e0 + E <= d) {
        if (x_dt == F32) {
            const float4* p4 = (const float4*)((const float*)x + base + e0);
            const float4 a = p4[0];
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
            if (E == 8) {
                const float4 b = p4[1];
                v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
            }
        } else {
            const uint16_t* p = (const uint16_t*)x + base + e0;
            uint32_t w[4];
            if (E == 8) {
                const uint4 a = *(const uint4*)p;
                w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
            } else {
                const uint2 a = *(const uint2*)p;
                w[0] = a.x; w[1] = a.y;
            }
            for (int j = 0; j < E; ++j) {
                const uint16_t hv = (uint16_t)(w[j >> 1] >> (16 * (j & 1)));
                v[j] = x_dt == BF16 ? bf2f(hv) : h2f(hv);
            }
        }
        return;
    }
    for (int j = 0; j < E; ++j) v[j] = e0 + j < d ? load_elem(x, base + e0 + j, x_dt) : 0.0f;
}

__global__ __launch_bounds__(256) void k_convert_rows(const void* __restrict__ x, int x_dt, int64_t n, int d,
                                                      void* __restrict__ codes, int st_dt, int kdim,
                                                      float* __restrict__ norms, unsigned* __restrict__ max_sq_bits,
                                                      int normalize, int vec) {
    __shared__ unsigned bmax;
    if (threadIdx.x == 0) bmax = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    const int E = st_dt == F32 ? 4 : 8;  // values per 16-B output chunk
    const int nchunk = kdim / E;         // kdim * esize = row_bytes, a multiple of 128
    unsigned my_max = 0u;
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += nwaves) {
        const int64_t base = r * d;
        float scale = 1.0f;
        if (normalize) {
            double s = 0.0;
            for (int c = lane; c < nchunk; c += 64) {
                float v[8];
                load_chunk_in(x, x_dt, base, c * E, d, E, vec != 0, v);
                for (int j = 0; j < E; ++j) s = fma((double)v[j], (double)v[j], s);
            }
            s = wave_sum_f64(s);
            scale = s > 0.0 ? (float)(1.0 / sqrt(s)) : 1.0f;
        }
        float sq = 0.0f;
        char* out = (char*)codes + r * (int64_t)kdim * (st_dt == F32 ? 4 : 2);
        for (int c = lane; c < nchunk; c += 64) {
            float v[8];
            load_chunk_in(x, x_dt, base, c * E, d, E, vec != 0, v);
            if (st_dt == F32) {
                float4 o;
                o.x = v[0] * scale; o.y = v[1] * scale; o.z = v[2] * scale; o.w = v[3] * scale;
                sq = fmaf(o.x, o.x, sq); sq = fmaf(o.y, o.y, sq); sq = fmaf(o.z, o.z, sq); sq = fmaf(o.w, o.w, sq);
                *(float4*)(out + c * 16) = o;
            } else {
                uint32_t w[4];
                for (int j = 0; j < 8; j += 2) {
                    const uint16_t h0 = st_dt == BF16 ? f2bf(v[j] * scale) : f2h(v[j] * scale);
                    const uint16_t h1 = st_dt == BF16 ? f2bf(v[j + 1] * scale) : f2h(v[j + 1] * scale);
                    const float s0 = st_dt == BF16 ? bf2f(h0) : h2f(h0), s1 = st_dt == BF16 ? bf2f(h1) : h2f(h1);
                    sq = fmaf(s0, s0, sq);
                    sq = fmaf(s1, s1, sq);
                    w[j >> 1] = (uint32_t)h0 | ((uint32_t)h1 << 16);
                }
                *(uint4*)(out + c * 16) = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        sq = wave_sum_f32(sq);
        if (lane == 0) {
            norms[r] = sq;
            my_max = max(my_max, __float_as_uint(sq));  // non-negative floats order as uints
        }
    }
    if (lane == 0 && my_max) atomicMax(&bmax, my_max);
    __syncthreads();
    if (threadIdx.x == 0 && bmax) atomicMax(max_sq_bits, bmax);
}

// The same conversion specialised on (input dtype, storage dtype, normalise)
// for 16-B-aligned input rows: a wave takes R rows at a time (R * chunks per
// row a multiple of 64 lanes where possible: 2 rows of 768 bf16), issues every
// chunk load of those rows before converting any (up to CPL 16-B chunks in
// flight per lane), and reduces the R row norms together.  Chunks partly or
// wholly past d (row padding) take the element path.
// streamed-once operands of add(): NT = nontemporal loads / stores (the rows
// are read once and the codes are not re-read by this launch)
typedef unsigned cv_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned cv_u32x2 __attribute__((ext_vector_type(2)));
template <bool NT, typename V>
__device__ __forceinline__ V cv_load(const void* p) {
    if constexpr (NT) return __builtin_nontemporal_load((const V*)p);
    else return *(const V*)p;
}
template <bool NT>
__device__ __forceinline__ void cv_store16(void* p, cv_u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, (cv_u32x4*)p);
    else *(cv_u32x4*)p = v;
}

template <int XDT, int SDT, bool NORM, bool NT, int CPL>
__global__ __launch_bounds__(256) void k_convert_rows_t(const void* __restrict__ x, int64_t n, int d,
                                                        void* __restrict__ codes, int kdim, float* __restrict__ norms,
                                                        unsigned* __restrict__ max_sq_bits, int R) {
    constexpr int E = SDT == F32 ? 4 : 8;    // values per 16-B output chunk
    // CPL: chunks per lane per wave iteration (all loaded before any store)
    constexpr int RMAX = CPL;
    __shared__ unsigned bmax;
    if (threadIdx.x == 0) bmax = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int nchunk = kdim / E;
    const int tot = R * nchunk;  // <= 64 * CPL (host-checked)
    const int64_t ngroups = (n + R - 1) / R;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    unsigned my_max = 0u;
    for (int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g < ngroups; g += nwaves) {
        const int64_t r0 = g * R;
        float v[CPL][E];
        // all loads first
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const int c = lane + 64 * k;
            const int rr = c / nchunk, cc = c - rr * nchunk;
            const int64_t r = r0 + rr;
            const int e0 = cc * E;
            if (c < tot && r < n && e0 + E <= d) {
                const char* src = (const char*)x + ((r * d + e0) * (XDT == F32 ? 4 : 2));
                if constexpr (XDT == F32) {
                    const cv_u32x4 a = cv_load<NT, cv_u32x4>(src);
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[k][j] = __uint_as_float(a[j]);
                    if constexpr (E == 8) {
                        const cv_u32x4 b = cv_load<NT, cv_u32x4>(src + 16);
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[k][4 + j] = __uint_as_float(b[j]);
                    }
                } else if constexpr (E == 8) {
                    const cv_u32x4 a = cv_load<NT, cv_u32x4>(src);
                    const uint32_t w[4] = {a[0], a[1], a[2], a[3]};
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint16_t hv = (uint16_t)(w[j >> 1] >> (16 * (j & 1)));
                        v[k][j] = XDT == BF16 ? bf2f(hv) : h2f(hv);
                    }
                } else {
                    const cv_u32x2 a = cv_load<NT, cv_u32x2>(src);
                    const uint32_t w[2] = {a[0], a[1]};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint16_t hv = (uint16_t)(w[j >> 1] >> (16 * (j & 1)));
                        v[k][j] = XDT == BF16 ? bf2f(hv) : h2f(hv);
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < E; ++j)
                    v[k][j] = (c < tot && r < n && e0 + j < d) ? load_elem(x, r * d + e0 + j, XDT) : 0.0f;
            }
        }
        // per-row scale (opt-in normalisation: fp64 sum of the input squares)
        float scale[RMAX];
#pragma unroll
        for (int q = 0; q < RMAX; ++q) scale[q] = 1.0f;
        if constexpr (NORM) {
            double sr[RMAX] = {};
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const int rr = (lane + 64 * k) / nchunk;
                double t = 0.0;
#pragma unroll
                for (int j = 0; j < E; ++j) t = fma((double)v[k][j], (double)v[k][j], t);
#pragma unroll
                for (int q = 0; q < RMAX; ++q) sr[q] += rr == q ? t : 0.0;
            }
#pragma unroll
            for (int q = 0; q < RMAX; ++q) {
                if (q < R) {
                    const double s2 = wave_sum_f64(sr[q]);
                    scale[q] = s2 > 0.0 ? (float)(1.0 / sqrt(s2)) : 1.0f;
                }
            }
        }
        // convert, store, |y|^2 of the stored values
        float sq[RMAX] = {};
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const int c = lane + 64 * k;
            const int rr = c / nchunk, cc = c - rr * nchunk;
            const int64_t r = r0 + rr;
            if (c >= tot || r >= n) continue;
            float sc = scale[0];
#pragma unroll
            for (int q = 1; q < RMAX; ++q) sc = rr == q ? scale[q] : sc;
            float part = 0.0f;
            char* out = (char*)codes + r * (int64_t)kdim * (SDT == F32 ? 4 : 2) + cc * 16;
            if constexpr (SDT == F32) {
                float4 o;
                o.x = v[k][0] * sc; o.y = v[k][1] * sc; o.z = v[k][2] * sc; o.w = v[k][3] * sc;
                part = fmaf(o.x, o.x, part); part = fmaf(o.y, o.y, part);
                part = fmaf(o.z, o.z, part); part = fmaf(o.w, o.w, part);
                cv_store16<NT>(out, cv_u32x4{__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z),
                                             __float_as_uint(o.w)});
            } else {
                uint32_t w[4];
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    const uint16_t h0 = SDT == BF16 ? f2bf(v[k][j] * sc) : f2h(v[k][j] * sc);
                    const uint16_t h1 = SDT == BF16 ? f2bf(v[k][j + 1] * sc) : f2h(v[k][j + 1] * sc);
                    const float s0 = SDT == BF16 ? bf2f(h0) : h2f(h0), s1 = SDT == BF16 ? bf2f(h1) : h2f(h1);
                    part = fmaf(s0, s0, part);
                    part = fmaf(s1, s1, part);
                    w[j >> 1] = (uint32_t)h0 | ((uint32_t)h1 << 16);
                }
                cv_store16<NT>(out, cv_u32x4{w[0], w[1], w[2], w[3]});
            }
#pragma unroll
            for (int q = 0; q < RMAX; ++q) sq[q] += rr == q ? part : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < RMAX; ++q) {
            if (q < R && r0 + q < n) {
                const float t = wave_sum_f32(sq[q]);
                if (lane == 0) {
                    norms[r0 + q] = t;
                    my_max = max(my_max, __float_as_uint(t));
                }
            }
        }
    }
    if (lane == 0 && my_max) atomicMax(&bmax, my_max);
    __syncthreads();
    if (threadIdx.x == 0 && bmax) atomicMax(max_sq_bits, bmax);
}

// Centre of an L2 scan image: mu = mean of a strided sample of up to
// MU_SAMPLE stored rows.  Any mu gives correct results (distances are
// translation invariant and the certification terms are computed for the
// centred operands); a centre inside the data shrinks the operands' norms,
// and with them the bound, by the spread-to-norm ratio of clustered
// embeddings.  Pass 1: block (column group of 64, row group g) sums its sample
// rows and their squares in fp64; pass 2 (one block) sums the row groups in a
// fixed order (deterministic) and, when min_ratio > 0, drops a centre whose
// norm is small next to the rows' (mu = 0: no common direction to remove).
__global__ __launch_bounds__(256) void k_mu_partial(const char* __restrict__ codes, int dt, int row_bytes, int kdim,
                                                    int64_t n, int64_t ns, double* __restrict__ part) {
    __shared__ double red[2][4][64];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), sub = threadIdx.x >> 6, g = blockIdx.y;
    double acc = 0.0, acc2 = 0.0;
    if (c < kdim)
        for (int64_t i = (int64_t)g * 4 + sub; i < ns; i += MU_GROUPS * 4) {
            const double v = (double)load_elem(codes + (i * n / ns) * (int64_t)row_bytes, c, dt);
            acc += v;
            acc2 += v * v;
        }
    red[0][sub][threadIdx.x & 63] = acc;
    red[1][sub][threadIdx.x & 63] = acc2;
    __syncthreads();
    if (sub == 0 && c < kdim) {
        const int l = threadIdx.x;
        part[(int64_t)g * kdim + c] = red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l];
        part[(int64_t)(MU_GROUPS + g) * kdim + c] = red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l];
    }
}
__global__ __launch_bounds__(256) void k_mu_finish(const double* __restrict__ part, int kdim, int d, int64_t ns,
                                                   float min_ratio, float* __restrict__ mu) {
    __shared__ double red[2][256];
    double m2 = 0.0, y2 = 0.0;
    for (int c = threadIdx.x; c < kdim; c += 256) {
        double s = 0.0, s2 = 0.0;
        for (int g = 0; g < MU_GROUPS; ++g) {
            s += part[(int64_t)g * kdim + c];
            s2 += part[(int64_t)(MU_GROUPS + g) * kdim + c];
        }
        const float m = c < d ? (float)(s / (double)ns) : 0.0f;  // padding columns stay 0
        mu[c] = m;
        m2 += (double)m * m;
        y2 += s2 / (double)ns;
    }
    red[0][threadIdx.x] = m2;
    red[1][threadIdx.x] = y2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (min_ratio > 0.0f && red[0][0] < (double)min_ratio * red[1][0])
        for (int c = threadIdx.x; c < kdim; c += 256) mu[c] = 0.0f;
}

// 16-bit L2 scan image (IMG_C16): per stored row, S = |y - mu|^2 (fp64 sum
// of the exact differences, one rounding to fp32) -- the scan's srcC, whose
// query operand is then x - mu -- and its maximum -> cmax_bits.  One wave per
// row, 16-B chunks per lane, grid-stride.
template <int DT>
__global__ __launch_bounds__(256) void k_centre_norms(const char* __restrict__ codes, int row_bytes, int64_t r0,
                                                      int64_t r1, const float* __restrict__ mu,
                                                      float* __restrict__ cnorms, unsigned* __restrict__ cmax_bits) {
    __shared__ unsigned bmax;
    if (threadIdx.x == 0) bmax = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int nchunk = row_bytes / 16;
    unsigned my_max = 0u;
    for (int64_t row = r0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < r1; row += (int64_t)gridDim.x * 4) {
        const char* src = codes + row * (int64_t)row_bytes;
        double acc = 0.0;
        for (int c = lane; c < nchunk; c += 64) {
            const cv_u32x4 w4 = __builtin_nontemporal_load((const cv_u32x4*)(src + c * 16));
            const uint32_t w[4] = {w4[0], w4[1], w4[2], w4[3]};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint16_t hv = (uint16_t)(w[j >> 1] >> (16 * (j & 1)));
                const double y = (double)(DT == BF16 ? bf2f(hv) : h2f(hv));
                const double t = y - (mu ? (double)mu[c * 8 + j] : 0.0);
                acc = fma(t, t, acc);
            }
        }
        acc = wave_sum_f64(acc);
        if (lane == 0) {
            const float sq = (float)acc;
            cnorms[row] = sq;
            my_max = max(my_max, __float_as_uint(sq));
        }
    }
    if (lane == 0 && my_max) atomicMax(&bmax, my_max);
    __syncthreads();
    if (threadIdx.x == 0 && bmax) atomicMax(cmax_bits, bmax);
}

// fp32 rows -> F32S scan image: row r, v = fl(y - mu) (mu = 0 when null),
// = [rn_bf16(v) for v in row | rn_bf16(v - hi)] in the same row_bytes (kdim
// fp32 = 2 planes of kdim bf16); cnorms[r] = |v|^2 (fp32 fma chain per lane +
// wave sum: the scan's srcC) and its maximum -> cmax_bits.  One wave per row.
__global__ __launch_bounds__(256) void k_split_rows(const float* __restrict__ codes, int kdim, int64_t r0,
                                                    int64_t r1, const float* __restrict__ mu,
                                                    uint16_t* __restrict__ split, float* __restrict__ cnorms,
                                                    unsigned* __restrict__ cmax_bits) {
    __shared__ unsigned bmax;
    if (threadIdx.x == 0) bmax = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    unsigned my_max = 0u;
    for (int64_t row = r0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < r1; row += (int64_t)gridDim.x * 4) {
        const float* src = codes + row * kdim;
        uint16_t* out = split + row * (int64_t)(2 * kdim);
        float sq = 0.0f;
        for (int c = lane * 4; c < kdim; c += 256) {
            const float4 v = *(const float4*)(src + c);
            float vv[4] = {v.x, v.y, v.z, v.w};
            if (mu) {
                const float4 m = *(const float4*)(mu + c);
                vv[0] -= m.x; vv[1] -= m.y; vv[2] -= m.z; vv[3] -= m.w;
            }
            uint16_t hi[4], lo[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                hi[j] = f2bf(vv[j]);
                lo[j] = f2bf(vv[j] - bf2f(hi[j]));
                sq = fmaf(vv[j], vv[j], sq);
            }
            *(uint2*)(out + c) = make_uint2(hi[0] | ((uint32_t)hi[1] << 16), hi[2] | ((uint32_t)hi[3] << 16));
            *(uint2*)(out + kdim + c) = make_uint2(lo[0] | ((uint32_t)lo[1] << 16), lo[2] | ((uint32_t)lo[3] << 16));
        }
        sq = wave_sum_f32(sq);
        if (lane == 0) {
            cnorms[row] = sq;
            my_max = max(my_max, __float_as_uint(sq));
        }
    }
    if (lane == 0 && my_max) atomicMax(&bmax, my_max);
    __syncthreads();
    if (threadIdx.x == 0 && bmax) atomicMax(cmax_bits, bmax);
}

// ---------------------------------------------------------------------------
// search(): query preparation
// ---------------------------------------------------------------------------
// One wave per query row.  Scan operand and certification terms by mode:
//   F32S (fp32 index, split image): [hi | lo] bf16 planes of -2 (x - mu) (IP:
//     -x); E from the split scan's dropped terms, shift =
//     |x - mu|^2, rho = 0;
//   L2, scan dtype F32 / BF16 / F16: operand -2 op with op = rn_dt(fl(x - mu))
//     (mu = 0 without a centred image); with r = (x - mu) - op (exact in fp64)
//     the scan key of row y is  a(y) = srcC - 2 op.y  (srcC = |y - mu|^2, or
//     |y|^2 without a centre), and  a(y) + s_q = D(y) + 2 r.(y - x) + err,
//     s_q = |x|^2 - |mu|^2 - 2 r.x,  |2 r.(y - x)| <= 2 rho sqrt(D(y)),
//     rho = |r|,  |err| <= E = u Smax + gamma_{K+1} (Smax + 2 M |op|)
//     (fp32 fma-chain accumulation of K exact products onto srcC: Smax = max
//     srcC, M = max |y|);
//   IP: operand -op, op = rn_dt(x): a(y) = -x.y + r.y, E = (gamma + u) |op| M
//     + rho M, shift 0, rho 0.
// A non-finite operand (fp16 overflow of -2 op) sets E = +inf: the query is
// never certified and goes to the exact fallback.
__global__ __launch_bounds__(256) void k_prep_queries(PrepParams p, double gamma) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p.pub) {  // the published lists of the scan's union bound -> +inf (grid-stride)
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.npub; i += stride) p.pub[i] = FX_INF;
    }
    if (r >= p.nq_pad) return;
    if (lane == 0) {
        if (p.gtau) p.gtau[r] = 0xff800000u;  // f2ord(+inf)
        if (r == 0)
            for (int i = 0; i < 3; ++i)
                if (p.zero[i]) *p.zero[i] = 0;
    }
    const int64_t nq = p.nq_dev ? min((int64_t)*p.nq_dev, p.nq) : p.nq;
    const bool live = r < nq;
    const int64_t src = live && p.qidx ? (int64_t)p.qidx[r] : r;  // source row of q
    // the index-wide bound terms, fetched before the row's loop (one memory
    // round trip less on the one-query path)
    const unsigned mbits = *p.mbits, img_bits = *p.img_bits;
    const int kdim = p.kdim;
    const float scale = p.metric == L2 ? -2.0f : -1.0f;
    // xn2 |x|^2, sc |x - mu|^2 (F32S), on2 |op|^2, rr |r|^2, rx r.x, mn2 |mu|^2
    double xn2 = 0.0, sc = 0.0, on2 = 0.0, rr = 0.0, rx = 0.0, mn2 = 0.0;
    bool bad = false;
    for (int c = lane; c < kdim; c += 64) {
        const float v = (live && c < p.d) ? load_elem(p.q, src * p.d + c, p.q_dt) : 0.0f;
        p.qf32[r * (int64_t)kdim + c] = v;
        const float m = p.mu ? p.mu[c] : 0.0f;
        xn2 += (double)v * (double)v;
        mn2 += (double)m * (double)m;
        if (p.st_dt == F32S) {
            // split operand of the pre-scaled (centred) query (x' - hi is exact
            // in fp32: hi is within 2^-8 |x'| of x')
            const float vc = v - m;
            const double xm = (double)v - (double)m;
            sc += xm * xm;
            on2 += (double)vc * (double)vc;
            const float xs = vc * scale;
            const uint16_t hi = f2bf(xs);
            uint16_t* row = (uint16_t*)p.qop + r * (int64_t)(2 * kdim);
            row[c] = hi;
            row[kdim + c] = f2bf(xs - bf2f(hi));
        } else {
            const float op = round_to(v - m, p.st_dt);
            const float sop = op * scale;  // exact (power of two) unless it overflows fp16
            bad |= !__builtin_isfinite(round_to(sop, p.st_dt));
            store_elem(p.qop, r * (int64_t)kdim + c, p.st_dt, sop);
            const double rc = ((double)v - (double)m) - (double)op;
            rr += rc * rc;
            rx += rc * (double)v;
            on2 += (double)op * (double)op;
        }
    }
    xn2 = wave_sum_f64(xn2);
    sc = wave_sum_f64(sc);
    on2 = wave_sum_f64(on2);
    rr = wave_sum_f64(rr);
    rx = wave_sum_f64(rx);
    mn2 = wave_sum_f64(mn2);
    bad = __any(bad);
    if (!live || lane != 0) return;
    const double u = 5.9604644775390625e-8;  // 2^-24
    // M: the largest stored-row norm; Smax: the largest srcC of the scan image
    // (both read on the device: add() never waits for the host to learn them)
    const double M = sqrt((double)__uint_as_float(mbits));
    const double Smax = (double)__uint_as_float(img_bits);
    const double on = sqrt(on2);
    double eps, shift = 0.0, rho = 0.0;
    if (p.st_dt == F32S) {
        // the split scan drops lo*lo and both residuals v - hi - lo: per
        // product <= 3 * 2^-16 (1 + 2^-7) |x_k||y_k| (delta); centring: the
        // operands are fl(y - mu), fl(x - mu): each product and square carries
        // <= 2u + u^2 more (3u); gamma covers its 3 K + 1 accumulated terms
        const double Mc = sqrt(Smax), delta = 4.73e-5, cu = p.mu ? 3.0 * u : 0.0;
        if (p.metric == L2) {
            eps = (2.0 * gamma + u + cu) * (Mc * Mc + 2.0 * on * Mc) + 2.0 * delta * on * Mc;
            shift = sc;
        } else {
            eps = (gamma + u) * on * Mc + delta * on * Mc;
        }
    } else if (p.metric == L2) {
        eps = u * Smax * 1.01 + gamma * (Smax * 1.01 + 2.0 * M * on);
        shift = xn2 - mn2 - 2.0 * rx;
        eps += 1e-12 * (xn2 + mn2 + 2.0 * fabs(rx));  // fp64 rounding of shift
        rho = sqrt(rr);
    } else {
        eps = (gamma + u) * on * M + sqrt(rr) * M;
    }
    p.qeps[r] = bad ? FX_INF : (float)(eps * 1.0625 + 1e-30);
    p.qrho[r] = (float)(rho * 1.0000002);
    p.qshift[r] = shift;
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

template <int DT, int METRIC>
__global__ __launch_bounds__(SCAN_THREADS, 1) void k_scan_topk(ScanParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef typename Frag<DT>::T frag_t;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    int qtile, split;
    map_block(blockIdx.x, p, qtile, split);
    const int64_t nq = p.nq_dev ? min((int64_t)*p.nq_dev, p.nq) : p.nq;
    if (qtile >= p.n_qtiles || (int64_t)qtile * TILE_Q >= nq) return;
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
                qv[n] = q0 + qloc[n] < nq;
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
        if (q0 + q >= nq) break;
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
// merge one chunk of 64 candidates (one per lane) into the running best-64
// Candidate-list integrity (RefineParams.n_drop): an entry's row id is -1
// (an empty slot) or a row of the index.  Anything else means a corrupted
// list; it is never gathered (a fault would follow) but counted, so the
// search reports it instead of returning a silently thinner candidate set.
__device__ __forceinline__ int cand_id_corrupt(int ii, int64_t ntotal) { return ii != -1 && (ii < 0 || ii >= ntotal); }
// per-lane counts -> the device word (one wave-uniform branch in the common case: none)
__device__ __forceinline__ void count_dropped(int bad, int* n_drop, int lane) {
    (void)lane;
    if (__builtin_amdgcn_ballot_w64(bad != 0) != 0 && bad != 0 && n_drop) atomicAdd(n_drop, bad);
}

__device__ __forceinline__ void refine_take(float d, int i, float& bd, int& bi, float& td, int& ti, int& nvalid,
                                            int lane) {
    nvalid += __popcll(__ballot(i != INT_MAX));
    const bool pass = i != INT_MAX && key_lt(d, i, td, ti);
    if (!__any(pass)) return;
    if (!pass) { d = FX_INF; i = INT_MAX; }
    sort64(d, i, lane);
    merge_into(bd, bi, d, i, lane);
    td = __shfl(bd, KP - 1, 64);
    ti = __shfl(bi, KP - 1, 64);
}

// Small batches scan with many corpus splits (1,024 at nq = 1 on 10M rows),
// which leaves one refine wave per query walking splits * KP candidates.
// This pre-pass merges every G splits' lists of a query into their top KP
// (one wave per (query, group of G splits), all loads issued first), written
// in the same [qtile][group][128][KP] layout; the refine then reads
// ceil(splits / G) lists.  The union of the groups' top KP holds the global
// top KP under the (key, id) order, so the refine's selection, its KP-th key
// and its "at least KP valid candidates" test are unchanged.
template <int G>
__global__ __launch_bounds__(256) void k_reduce_cand(const float* __restrict__ cd, const int* __restrict__ ci,
                                                     int splits, int64_t nq, int ngroups, float* __restrict__ od,
                                                     int* __restrict__ oi, int64_t ntotal, int* __restrict__ n_drop,
                                                     int qt) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t q = w / ngroups;
    const int g = (int)(w - q * ngroups);
    if (q >= nq) return;
    const int qtile = (int)(q / qt), qq = (int)(q % qt);
    const int s0 = g * G, ns = min(G, splits - s0);
    constexpr int NL = G * KP / 64;  // loads per lane
    float dv[NL];
    int iv[NL];
    int bad = 0;
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int c = u * 64 + lane, s = c / KP, j = c - s * KP;
        dv[u] = FX_INF;
        iv[u] = INT_MAX;
        if (s < ns) {
            const int64_t off = (((int64_t)qtile * splits + s0 + s) * qt + qq) * KP + j;
            const int ii = ci[off];
            const float dd = cd[off];
            if (ii >= 0 && ii < ntotal) { dv[u] = dd; iv[u] = ii; }
            else bad += cand_id_corrupt(ii, ntotal);
        }
    }
    count_dropped(bad, n_drop, lane);
    float bd = FX_INF, td = FX_INF;
    int bi = INT_MAX, ti = INT_MAX, nvalid = 0;
#pragma unroll
    for (int u = 0; u < NL; ++u) refine_take(dv[u], iv[u], bd, bi, td, ti, nvalid, lane);
    if (lane < KP) {
        const int64_t o = (((int64_t)qtile * ngroups + g) * qt + qq) * KP + lane;
        od[o] = bd;
        oi[o] = bi == INT_MAX ? -1 : bi;
    }
}

// flagged queries past the re-scan's capacity go straight to the exact scan
__global__ __launch_bounds__(256) void k_rescan_chunks(const int* __restrict__ n_flag, int cap, int nchunks,
                                                       int* __restrict__ counts) {
    const int nf = n_flag[0];
    for (int c = (int)threadIdx.x; c < nchunks; c += (int)blockDim.x) {
        const int left = nf - c * cap;
        counts[c] = left <= 0 ? 0 : (left < cap ? left : cap);
    }
}

hipError_t launch_rescan_chunks(const int* n_flag, int cap, int nchunks, int* counts, hipStream_t s) {
    hipLaunchKernelGGL(k_rescan_chunks, dim3(1), dim3(256), 0, s, n_flag, cap, nchunks, counts);
    return hipGetLastError();
}

hipError_t launch_reduce_cand(const float* cd, const int* ci, int splits, int64_t nq, int qt, float* od,
                              int* oi, int* ngroups, int64_t ntotal, int* n_drop, hipStream_t s) {
    constexpr int G = 16;
    *ngroups = (splits + G - 1) / G;
    const int64_t waves = nq * (int64_t)*ngroups;
    hipLaunchKernelGGL((k_reduce_cand<G>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, cd, ci, splits, nq,
                       *ngroups, od, oi, ntotal, n_drop, qt);
    return hipGetLastError();
}

// Certification of a query's top-k: every row the selection
// dropped has approx key >= tb, so (k_prep_queries) its exact distance D
// satisfies D + 2 rho sqrt(D) >= T = tb + shift - E, i.e.
// sqrt(D) >= sqrt(rho^2 + T) - rho = T / (sqrt(rho^2 + T) + rho) (rho = 0:
// D >= T, which is also the IP form).  The top-k is exact when the k-th
// exact key, plus 2 ulp for its own fp32 rounding, lies below that.
__device__ __forceinline__ bool certified_v(float kth, float tb, double shift, float eps, float rho_f) {
    const double T = (double)tb + shift - (double)eps;
    const double rho = (double)rho_f;
    double dmin = T;
    if (rho > 0.0) {
        const double t = T > 0.0 ? T : 0.0;
        const double sd = t / (sqrt(rho * rho + t) + rho);
        dmin = sd * sd * (1.0 - 1e-12);
    }
    const double kup = (double)kth + fabs((double)kth) * 2.384185791015625e-7;  // + 2 ulp
    return kup < dmin;
}
__device__ __forceinline__ bool certified(float kth, float tb, const RefineParams& p, int64_t q) {
    return certified_v(kth, tb, p.qshift[q], p.qeps[q], p.qrho[q]);
}

// PF = chunks of 64 candidates whose loads are issued together in phase 1
// (PF = 4 for the small-batch scan's many splits: one wave per query is
// latency-bound on one dependent load per chunk otherwise)
template <int DT, int METRIC, int PF = 1>
__global__ __launch_bounds__(256) void k_refine(RefineParams p) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= p.nq) return;
    const int qtile = (int)(q / p.qt), qq = (int)(q % p.qt);
    const int ncand = p.splits * KP;

    // ---- phase 1: KP smallest approx keys over all splits (running best-64)
    float bd = FX_INF, td = FX_INF;
    int bi = INT_MAX, ti = INT_MAX;
    int nvalid = 0, bad = 0;
    if constexpr (PF > 1) {
        for (int base = 0; base < ncand; base += 64 * PF) {
            float dv[PF];
            int iv[PF];
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int c = base + u * 64 + lane;
                dv[u] = FX_INF;
                iv[u] = INT_MAX;
                if (c < ncand) {
                    const int s = c / KP, j = c - s * KP;
                    const int64_t off = (((int64_t)qtile * p.splits + s) * p.qt + qq) * KP + j;
                    const float dd = p.cand_d[off];  // both loads in flight together
                    const int ii = p.cand_i[off];
                    if (ii >= 0 && ii < p.ntotal) { dv[u] = dd; iv[u] = ii; }
                    else bad += cand_id_corrupt(ii, p.ntotal);
                }
            }
#pragma unroll
            for (int u = 0; u < PF; ++u) refine_take(dv[u], iv[u], bd, bi, td, ti, nvalid, lane);
        }
    } else {
        for (int base = 0; base < ncand; base += 64) {
            const int c = base + lane;
            float d = FX_INF;
            int i = INT_MAX;
            if (c < ncand) {
                const int s = c / KP, j = c - s * KP;
                const int64_t off = (((int64_t)qtile * p.splits + s) * p.qt + qq) * KP + j;
                const int ii = p.cand_i[off];
                if (ii >= 0 && ii < p.ntotal) { d = p.cand_d[off]; i = ii; }
                else bad += cand_id_corrupt(ii, p.ntotal);
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
    }

    count_dropped(bad, p.n_drop, lane);

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
    // Fewer than KP candidates in all: nothing was dropped unless some split
    // pruned with a threshold, and every pruning threshold of the scan is
    // published to the shared one (compactions, the cold-start bound), so a
    // finite gtau means "certify" 
    const unsigned gq = p.gtau ? p.gtau[q] : 0xff800000u;
    if (nvalid >= KP || gq < 0xff800000u) {
        const float kth = __shfl(key, p.k - 1, 64);
        // a split may also have pruned with the shared threshold (a bound on
        // a rank below KP, compact_wave): dropped rows lie above min(td, it)
        const float tb = p.gtau ? fminf(td, ord2f(gq)) : td;
        if (!certified(kth, tb, p, q) && lane == 0 && !p.force_fb) {
            const int pos = atomicAdd(p.n_flag, 1);
            p.flag_list[pos] = (int)q;
        }
    }
    if (p.force_fb && lane == 0) {
        const int pos = atomicAdd(p.n_flag, 1);
        p.flag_list[pos] = (int)q;
    }
}

// refine_take for a chunk that is two ascending runs of KP = 32 (lanes 0-31,
// 32-63): two consecutive splits' lists as the scan flushed them (sorted by
// (key, row)).  Reversing the lower run makes the chunk bitonic, and a 6-step
// merge sorts it DEscending -- ready to meet the ascending running best
// lane by lane (the 64 smallest of the union, bitonic) without the reversal
// merge_into does; the 21-step sort is only for a chunk that is not two
// sorted runs (a corrupted id masked to INT_MAX, -0 against +0 keys).
__device__ __forceinline__ void merge64_desc(float& d, int& i, int lane) {  // bitonic -> descending
    static_for<6>([&](auto T) { cmpx_s<(32 >> decltype(T)::value)>(d, i, lane, false); });
}
__device__ __forceinline__ void refine_take2(float d, int i, float& bd, int& bi, float& td, int& ti, int& nvalid,
                                             int lane) {
    nvalid += __popcll(__ballot(i != INT_MAX));
    const bool pass = i != INT_MAX && key_lt(d, i, td, ti);
    if (!__any(pass)) return;
    if (!pass) { d = FX_INF; i = INT_MAX; }  // (a suffix of each sorted run)
    const float pd = __shfl(d, lane - 1, 64);
    const int pi = __shfl(i, lane - 1, 64);
    const bool sorted = !__any((lane & 31) != 0 && key_lt(d, i, pd, pi));
    if (sorted) {  // [lower run reversed | upper run]: bitonic
        const int src = lane < 32 ? 31 - lane : lane;
        d = __shfl(d, src, 64);
        i = __shfl(i, src, 64);
        merge64_desc(d, i, lane);
    } else {
        sort64(d, i, lane);
        d = __shfl(d, 63 - lane, 64);
        i = __shfl(i, 63 - lane, 64);
    }
    if (key_lt(d, i, bd, bi)) { bd = d; bi = i; }  // ascending best vs descending chunk: bitonic
    merge64(bd, bi, lane);
    td = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bd), KP - 1));
    ti = __builtin_amdgcn_readlane(bi, KP - 1);
}

// Small batches over many corpus splits (the reference's one-query call: 192
// splits on a 100k-row index, 1,024 on 10M rows): one workgroup of
// REFINE_WG_WAVES waves per query instead of k_reduce_cand + k_refine (one
// launch less on the latency-bound path, and the candidate walk in
// parallel).  Each wave walks every NW-th chunk of the query's splits * KP
// candidates into its own top KP (refine_take2: chunks are pairs of sorted
// split lists); the NW lists are merged pairwise in LDS (log2 NW bitonic
// merges) into the query's top KP -- the union of the waves' top KP holds
// the global top KP under the (key, id) order, so the selection, its KP-th
// key td and the candidate count are k_refine's; the exact re-rank of the KP
// rows is spread over the waves, and wave 0 orders, writes and certifies
// exactly as k_refine does.
constexpr int RWG_XQ_MAX = 4096;  // k_refine_wg keeps queries of up to this many dims in LDS
template <int DT, int METRIC, int NW>
__global__ __launch_bounds__(64 * NW) void k_refine_wg(RefineParams p) {
    static_assert((NW & (NW - 1)) == 0 && NW >= 2, "pairwise merge tree");
    constexpr int PF = 8;  // chunks of 64 whose loads are in flight together (one round at 256 splits)
    __shared__ float s_d[NW * KP];
    __shared__ int s_i[NW * KP];
    __shared__ int s_nv[NW];
    __shared__ double s_ex[KP];
    __shared__ float s_xq[RWG_XQ_MAX];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t q = blockIdx.x;
    if (q >= p.nq) return;  // (block-uniform)
    const int qtile = (int)(q / p.qt), qq = (int)(q % p.qt);
    const int ncand = p.splits * KP;
    // everything that does not depend on the selection is fetched now, beside
    // phase 1's loads (the kernel is a chain of memory round trips): the fp32
    // query into LDS for phase 2, the certification terms for phase 3
    const bool xq_lds = p.kdim <= RWG_XQ_MAX;
    if (xq_lds)
        for (int c = threadIdx.x; c < p.kdim; c += 64 * NW) s_xq[c] = p.qf32[q * (int64_t)p.kdim + c];
    const unsigned gq = p.gtau ? p.gtau[q] : 0xff800000u;
    const double c_shift = p.qshift[q];
    const float c_eps = p.qeps[q], c_rho = p.qrho[q];

    // ---- phase 1: this wave's KP best approx keys over its chunks
    float bd = FX_INF, td = FX_INF;
    int bi = INT_MAX, ti = INT_MAX;
    int nvalid = 0, bad = 0;
    for (int base = w * 64 * PF; base < ncand; base += NW * 64 * PF) {
        float dv[PF];
        int iv[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int c = base + u * 64 + lane;
            dv[u] = FX_INF;
            iv[u] = INT_MAX;
            if (c < ncand) {
                const int s = c / KP, j = c - s * KP;
                const int64_t off = (((int64_t)qtile * p.splits + s) * p.qt + qq) * KP + j;
                const float dd = p.cand_d[off];
                const int ii = p.cand_i[off];
                if (ii >= 0 && ii < p.ntotal) { dv[u] = dd; iv[u] = ii; }
                else bad += cand_id_corrupt(ii, p.ntotal);
            }
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) refine_take2(dv[u], iv[u], bd, bi, td, ti, nvalid, lane);
    }
    count_dropped(bad, p.n_drop, lane);
    if (lane < KP) {
        s_d[w * KP + lane] = bd;
        s_i[w * KP + lane] = bi;
    }
    if (lane == 0) s_nv[w] = nvalid;
    __syncthreads();

    // ---- the query's top KP: pairwise bitonic merges of the waves' ascending lists
#pragma unroll
    for (int st = 1; st < NW; st <<= 1) {
        if ((w & (2 * st - 1)) == 0) {
            const int src = lane < KP ? w * KP + lane : (w + st) * KP + (63 - lane);
            float d = s_d[src];
            int i = s_i[src];
            merge64(d, i, lane);
            if (lane < KP) {
                s_d[w * KP + lane] = d;
                s_i[w * KP + lane] = i;
            }
        }
        __syncthreads();
    }
    bd = lane < KP ? s_d[lane] : FX_INF;
    bi = lane < KP ? s_i[lane] : INT_MAX;
    td = s_d[KP - 1];
    nvalid = 0;
#pragma unroll
    for (int v = 0; v < NW; ++v) nvalid += s_nv[v];

    // ---- phase 2: exact fp64 values of the KP selected rows (16 lanes / row,
    // 4 rows per wave-step; step r on wave r % NW)
    const float* xq = xq_lds ? (const float*)s_xq : p.qf32 + q * (int64_t)p.kdim;
    const int grp = lane >> 4, sub = lane & 15;
    for (int r = w; r < KP / 4; r += NW) {
        const int row = __shfl(bi, r * 4 + grp, 64);
        double a = 0.0;
        if (row != INT_MAX) a = exact_partial<DT, METRIC>(xq, p.codes + (int64_t)row * p.row_bytes, p.row_bytes, sub, 16);
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (sub == 0) s_ex[r * 4 + grp] = a;
    }
    __syncthreads();
    if (w != 0) return;

    // ---- phase 3 (wave 0): order by (fp32 exact key, id), write top-k, certify
    float key = FX_INF;
    int id = INT_MAX;
    if (lane < KP && bi != INT_MAX) {
        const double ex = s_ex[lane];
        key = METRIC == L2 ? (float)ex : -(float)ex;
        id = bi;
    }
    sort64(key, id, lane);
    if (lane < p.k) {
        const bool valid = id != INT_MAX;
        p.D[q * p.k + lane] = valid ? (METRIC == L2 ? key : -key) : (METRIC == L2 ? FLT_MAX : -FLT_MAX);
        p.I[q * p.k + lane] = valid ? (int64_t)id + p.id_offset : (int64_t)-1;
    }
    if (nvalid >= KP || gq < 0xff800000u) {  // (k_refine: certify when anything pruned)
        const float kth = __shfl(key, p.k - 1, 64);
        const float tb = p.gtau ? fminf(td, ord2f(gq)) : td;
        if (!certified_v(kth, tb, c_shift, c_eps, c_rho) && lane == 0 && !p.force_fb) {
            const int pos = atomicAdd(p.n_flag, 1);
            p.flag_list[pos] = (int)q;
        }
    }
    if (p.force_fb && lane == 0) {
        const int pos = atomicAdd(p.n_flag, 1);
        p.flag_list[pos] = (int)q;
    }
}

// ---------------------------------------------------------------------------
// k > KP: refine without the fixed 64-lane lists (one workgroup per query)
// ---------------------------------------------------------------------------
// The scan ran with share = 0 (no cross-split threshold), so a split drops a
// row only when its own list is full, and then every dropped row has approx
// key >= that split's KP-th output entry.  Phase 1 selects the K1 best approx
// keys over all splits (block top-K in LDS) and the bound tb below which no
// unselected row can lie: min(KP-th entry of every full split, K1-th kept
// entry when candidates were cut).  Phase 2 computes the selected rows'
// exact distances (fp64, one rounding), phase 3 orders them by (D, id),
// writes the top-k and certifies it against tb like k_refine.
template <int DT, int METRIC>
__global__ __launch_bounds__(BT_THREADS) void k_refine_big(RefineParams p) {
    __shared__ float sd[BT_MAXB];
    __shared__ int si[BT_MAXB];
    __shared__ float ed[BT_MAXB];
    __shared__ int ei[BT_MAXB];
    __shared__ BtState<int> st;
    __shared__ unsigned t_split;
    const int64_t q = blockIdx.x;
    if (q >= (p.nq_dev ? min((int64_t)*p.nq_dev, p.nq) : p.nq)) return;
    const int64_t oq = p.out_idx ? (int64_t)p.out_idx[q] : q;  // output row (the re-scan scatters)
    const int tid = threadIdx.x;
    const int qtile = (int)(q / p.qt), qq = (int)(q % p.qt);
    const int K1 = p.k1, B = bt_cap(K1);
    if (tid == 0) t_split = f2ord(FX_INF);
    bt_init(&st);
    const int ncand = p.splits * KP;
    for (int c0 = 0; c0 < ncand; c0 += BT_THREADS) {
        const int c = c0 + tid;
        float d = FX_INF;
        int i = INT_MAX;
        bool valid = false;
        if (c < ncand) {
            const int s = c / KP, j = c - s * KP;
            const int64_t off = (((int64_t)qtile * p.splits + s) * p.qt + qq) * KP + j;
            const int ii = p.cand_i[off];
            if (ii >= 0 && ii < p.ntotal) {
                d = p.cand_d[off];
                i = ii;
                valid = true;
                if (j == KP - 1) atomicMin(&t_split, f2ord(d));  // a full split's KP-th key
            } else if (cand_id_corrupt(ii, p.ntotal) && p.n_drop) {
                atomicAdd(p.n_drop, 1);
            }
        }
        bt_round(sd, si, &st, K1, B, d, i, valid);
    }
    bt_flush(sd, si, &st, K1, B);
    const int n1 = st.cnt;
    float tb = ord2f(t_split);
    if (st.total > n1) tb = fminf(tb, sd[n1 - 1]);

    // phase 2: exact keys of the n1 selected rows, 16 lanes per row
    const float* xq = p.qf32 + q * (int64_t)p.kdim;
    const int grp = tid >> 4, sub = tid & 15;
    for (int r0 = 0; r0 < n1; r0 += BT_THREADS / 16) {
        const int r = r0 + grp;
        double a = 0.0;
        if (r < n1) a = exact_partial<DT, METRIC>(xq, p.codes + (int64_t)si[r] * p.row_bytes, p.row_bytes, sub, 16);
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (sub == 0 && r < n1) {
            ed[r] = METRIC == L2 ? (float)a : -(float)a;
            ei[r] = si[r];
        }
    }
    int n2 = 2;
    while (n2 < n1) n2 <<= 1;
    for (int t = n1 + tid; t < n2; t += BT_THREADS) {
        ed[t] = FX_INF;
        ei[t] = INT_MAX;
    }
    bt_sort(ed, ei, n2);  // (syncs: ed/ei complete)

    // phase 3: top-k out (faiss padding past the candidates), certification
    for (int t = tid; t < p.k; t += BT_THREADS) {
        const bool valid = t < n1;
        p.D[oq * p.k + t] = valid ? (METRIC == L2 ? ed[t] : -ed[t]) : (METRIC == L2 ? FLT_MAX : -FLT_MAX);
        p.I[oq * p.k + t] = valid ? (int64_t)ei[t] + p.id_offset : (int64_t)-1;
    }
    if (tid == 0) {
        bool ok;
        if (!(tb < FX_INF)) ok = true;  // no row was dropped anywhere: the candidates are every row
        else if (n1 < p.k) ok = false;
        else {
            ok = certified(ed[p.k - 1], tb, p, q);
        }
        if (!ok || p.force_fb) {
            const int pos = atomicAdd(p.n_flag, 1);
            p.flag_list[pos] = (int)oq;
        }
    }
}

// ---------------------------------------------------------------------------
// exact fallback for uncertified queries, decided on the device: the host
// always enqueues these two launches after the refine; they read the
// uncertified count n_flag[0] (list at n_flag + 1) and exit at once when it
// is 0, so a device-resident search never waits for the host.
// k_fb_scan: work item = (flagged query f, corpus split); exact fp64 key of
// every row of the split, block top-k -> cd/ci[item][k].
// k_fb_merge: per flagged query, top-k of its splits' lists -> D / I.
// ---------------------------------------------------------------------------
template <int DT, int METRIC>
__global__ __launch_bounds__(BT_THREADS) void k_fb_scan(const char* __restrict__ codes, int row_bytes, int kdim,
                                                        int64_t ntotal, const float* __restrict__ qf32,
                                                        const int* __restrict__ n_flag, int k,
                                                        float* __restrict__ cd, int* __restrict__ ci) {
    __shared__ float sd[BT_MAXB];
    __shared__ int si[BT_MAXB];
    __shared__ BtState<int> st;
    const int nf = n_flag[0];
    if (nf <= 0) return;
    const int* qlist = n_flag + 1;
    const int fbs = fb_splits_for(nf, ntotal), B = bt_cap(k);
    const int64_t items = (int64_t)nf * fbs;
    for (int64_t w = blockIdx.x; w < items; w += gridDim.x) {
        const int f = (int)(w / fbs), split = (int)(w % fbs);
        const float* xq = qf32 + (int64_t)qlist[f] * kdim;
        const int64_t r0 = ntotal * split / fbs, r1 = ntotal * (split + 1) / fbs;
        bt_init(&st);
        for (int64_t base = r0; base < r1; base += BT_THREADS) {
            const int64_t row = base + threadIdx.x;
            const bool valid = row < r1;
            float key = FX_INF;
            if (valid) {
                const double v = exact_partial<DT, METRIC>(xq, codes + row * row_bytes, row_bytes, 0, 1);
                key = METRIC == L2 ? (float)v : -(float)v;
            }
            bt_round(sd, si, &st, k, B, key, valid ? (int)row : INT_MAX, valid);
        }
        bt_flush(sd, si, &st, k, B);
        const int c = st.cnt;
        for (int t = threadIdx.x; t < k; t += BT_THREADS) {
            cd[w * k + t] = t < c ? sd[t] : FX_INF;
            ci[w * k + t] = t < c ? si[t] : -1;
        }
        __syncthreads();
    }
}

template <int METRIC>
__global__ __launch_bounds__(BT_THREADS) void k_fb_merge(const int* __restrict__ n_flag, int64_t ntotal, int k,
                                                         const float* __restrict__ cd, const int* __restrict__ ci,
                                                         int64_t id_offset, float* __restrict__ D,
                                                         int64_t* __restrict__ I) {
    __shared__ float sd[BT_MAXB];
    __shared__ int si[BT_MAXB];
    __shared__ BtState<int> st;
    const int nf = n_flag[0];
    if (nf <= 0) return;
    const int* qlist = n_flag + 1;
    const int fbs = fb_splits_for(nf, ntotal), B = bt_cap(k);
    const int64_t per = (int64_t)fbs * k;
    for (int f = blockIdx.x; f < nf; f += gridDim.x) {
        bt_init(&st);
        for (int64_t c0 = 0; c0 < per; c0 += BT_THREADS) {
            const int64_t c = (int64_t)f * per + c0 + threadIdx.x;
            const bool in = c0 + threadIdx.x < per;
            const int ii = in ? ci[c] : -1;
            bt_round(sd, si, &st, k, B, ii >= 0 ? cd[c] : FX_INF, ii >= 0 ? ii : INT_MAX, ii >= 0);
        }
        bt_flush(sd, si, &st, k, B);
        const int64_t q = qlist[f];
        const int c = st.cnt;
        for (int t = threadIdx.x; t < k; t += BT_THREADS) {
            const bool valid = t < c;
            D[q * k + t] = valid ? (METRIC == L2 ? sd[t] : -sd[t]) : (METRIC == L2 ? FLT_MAX : -FLT_MAX);
            I[q * k + t] = valid ? (int64_t)si[t] + id_offset : (int64_t)-1;
        }
        __syncthreads();
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

// k > 64: one workgroup per query, block top-k over the G*k gathered entries
template <int METRIC>
__global__ __launch_bounds__(BT_THREADS) void k_merge_shards_big(int nshards, int64_t nq, int k,
                                                                 const float* __restrict__ Din,
                                                                 const int64_t* __restrict__ Iin,
                                                                 float* __restrict__ Dout,
                                                                 int64_t* __restrict__ Iout) {
    __shared__ float sd[BT_MAXB];
    __shared__ long long si[BT_MAXB];
    __shared__ BtState<long long> st;
    const int64_t q = blockIdx.x;
    if (q >= nq) return;
    const int B = bt_cap(k), total = nshards * k;
    bt_init(&st);
    for (int c0 = 0; c0 < total; c0 += BT_THREADS) {
        const int c = c0 + threadIdx.x;
        long long ii = -1;
        float d = FX_INF;
        if (c < total) {
            const int sh = c / k, j = c - sh * k;
            const int64_t off = ((int64_t)sh * nq + q) * k + j;
            ii = Iin[off];
            if (ii >= 0) d = METRIC == L2 ? Din[off] : -Din[off];
        }
        bt_round(sd, si, &st, k, B, d, ii >= 0 ? ii : LLONG_MAX, ii >= 0);
    }
    bt_flush(sd, si, &st, k, B);
    const int c = st.cnt;
    for (int t = threadIdx.x; t < k; t += BT_THREADS) {
        const bool valid = t < c;
        Dout[q * k + t] = valid ? (METRIC == L2 ? sd[t] : -sd[t]) : (METRIC == L2 ? FLT_MAX : -FLT_MAX);
        Iout[q * k + t] = valid ? (int64_t)si[t] : (int64_t)-1;
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
// Row kernels (add() conversion, split image) end each workgroup with one
// atomicMax on a single word (the max row norm): at 65,536 workgroups those
// serialised and set the kernel time (1M x 768 bf16: 0.86 ms whatever the
// bytes); a grid-stride launch of 4,096 workgroups (16 per CU) moves the same
// chunk in 0.574 ms = 5.36 TB/s, above a torch device copy on the same box
// (profiles/r2/add_grid_ab.txt)
constexpr int ROWS_GRID_CAP = 4096;

static inline int grid_for(int64_t items, int per_block, int cap) {
    int64_t g = (items + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

hipError_t launch_convert_rows(const void* x, int x_dt, int64_t n, int d, void* codes_row0, int st_dt, int kdim,
                               float* norms_row0, unsigned* max_sq_bits, int normalize, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int vec = ((int64_t)d * (x_dt == F32 ? 4 : 2)) % 16 == 0 && ((uintptr_t)x & 15) == 0;
    // rows per wave iteration: the fewest that fill whole 64-lane passes
    const int nchunk = kdim / (st_dt == F32 ? 4 : 8);
    int R = 1;
    while (R < 4 && (R * nchunk) % 64 != 0) R *= 2;
    if (vec && R * nchunk <= 64 * 4) {
        // grid-stride over row groups with a bounded grid (ROWS_GRID_CAP);
        // nontemporal loads / stores (1M x 768 bf16: 0.900 -> 0.882 ms, same box)
        const unsigned grid = grid_for((n + R - 1) / R, 4, ROWS_GRID_CAP);
#define FX_CONV(XD, SD)                                                                                           \
        if (x_dt == XD && st_dt == SD) {                                                                         \
            if (normalize)                                                                                       \
                hipLaunchKernelGGL((k_convert_rows_t<XD, SD, true, true, 4>), dim3(grid), dim3(256), 0, s, x, n, \
                                   d, codes_row0, kdim, norms_row0, max_sq_bits, R);                            \
            else                                                                                                 \
                hipLaunchKernelGGL((k_convert_rows_t<XD, SD, false, true, 4>), dim3(grid), dim3(256), 0, s, x,   \
                                   n, d, codes_row0, kdim, norms_row0, max_sq_bits, R);                         \
            return hipGetLastError();                                                                            \
        }
        FX_CONV(F32, F32) FX_CONV(F32, BF16) FX_CONV(F32, F16)
        FX_CONV(BF16, F32) FX_CONV(BF16, BF16) FX_CONV(BF16, F16)
        FX_CONV(F16, F32) FX_CONV(F16, BF16) FX_CONV(F16, F16)
#undef FX_CONV
    }
    hipLaunchKernelGGL(k_convert_rows, dim3(grid_for(n, 4, ROWS_GRID_CAP)), dim3(256), 0, s, x, x_dt, n, d, codes_row0,
                       st_dt, kdim, norms_row0, max_sq_bits, normalize, vec);
    return hipGetLastError();
}

hipError_t launch_split_rows(const float* codes, int kdim, int64_t r0, int64_t r1, const float* mu, void* split,
                             float* cnorms, unsigned* cmax_bits, hipStream_t s) {
    if (r1 <= r0) return hipSuccess;
    hipLaunchKernelGGL(k_split_rows, dim3(grid_for(r1 - r0, 4, ROWS_GRID_CAP)), dim3(256), 0, s, codes, kdim, r0, r1, mu,
                       (uint16_t*)split, cnorms, cmax_bits);
    return hipGetLastError();
}

hipError_t launch_mu(const char* codes, int dt, int row_bytes, int d, int64_t n, double* part, float* mu,
                     float min_ratio, hipStream_t s) {
    if (n <= 0) return hipErrorInvalidValue;
    const int kdim = row_bytes / dtype_size(dt);
    const int64_t ns = n < MU_SAMPLE ? n : MU_SAMPLE;
    hipLaunchKernelGGL(k_mu_partial, dim3((unsigned)((kdim + 63) / 64), MU_GROUPS), dim3(256), 0, s, codes, dt,
                       row_bytes, kdim, n, ns, part);
    hipLaunchKernelGGL(k_mu_finish, dim3(1), dim3(256), 0, s, part, kdim, d, ns, min_ratio, mu);
    return hipGetLastError();
}

hipError_t launch_centre_norms(const char* codes, int dt, int row_bytes, int64_t r0, int64_t r1, const float* mu,
                               float* cnorms, unsigned* cmax_bits, hipStream_t s) {
    if (r1 <= r0) return hipSuccess;
    const dim3 g(grid_for(r1 - r0, 4, ROWS_GRID_CAP));
    if (dt == BF16)
        hipLaunchKernelGGL(k_centre_norms<BF16>, g, dim3(256), 0, s, codes, row_bytes, r0, r1, mu, cnorms, cmax_bits);
    else if (dt == F16)
        hipLaunchKernelGGL(k_centre_norms<F16>, g, dim3(256), 0, s, codes, row_bytes, r0, r1, mu, cnorms, cmax_bits);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_prep_queries(const PrepParams& p, hipStream_t s) {
    const double u = 5.9604644775390625e-8;
    // terms accumulated by the scan's fp32 MFMA chain: K products (3 K for F32S) + srcC
    const double nt = p.st_dt == F32S ? 3.0 * p.kdim + 1.0 : (double)p.kdim + 1.0;
    const double gamma = nt * u / (1.0 - nt * u);
    hipLaunchKernelGGL(k_prep_queries, dim3((unsigned)((p.nq_pad + 3) / 4)), dim3(256), 0, s, p, gamma);
    return hipGetLastError();
}

template <int DT, int METRIC>
static hipError_t scan_t(const ScanParams& p, hipStream_t s) {
    // > 64 KiB of dynamic LDS must be opted into (per device; cheap to repeat)
    hipError_t e = g_graph_capture ? hipSuccess : hipFuncSetAttribute((const void*)k_scan_topk<DT, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_SCAN_BYTES);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_scan_topk<DT, METRIC>), dim3(p.grid), dim3(SCAN_THREADS), LDS_SCAN_BYTES, s, p);
    return hipGetLastError();
}

hipError_t launch_scan(int st_dt, int metric, const ScanParams& p, hipStream_t s) {
    if (p.tr == V5_TR) return launch_scan_v5(st_dt, metric, p, s);  // (the plan chose k_scan_v5)
    if (p.qt != TILE_Q || p.tr != TILE_R) return hipErrorInvalidValue;
    // the MFMA scan (fx_scan.hip) covers every row width it has a register
    // layout for; other widths take the generic kernel above
    if (st_dt == F32S) {  // the split-fp32 operand exists only for the MFMA scans
        bool handled = false;
        hipError_t e = launch_scan_mfma(st_dt, metric, p, s, &handled);
        return handled ? e : hipErrorInvalidValue;
    }
    {
        bool handled = false;
        hipError_t e = launch_scan_mfma(st_dt, metric, p, s, &handled);
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
    if (p.k > KP || p.k1 > 0)  // (k1 > 0 with k <= KP: the re-scan's wide candidate set)
        hipLaunchKernelGGL((k_refine_big<DT, METRIC>), dim3((unsigned)p.nq), dim3(BT_THREADS), 0, s, p);
    else if (p.wg == 4)
        hipLaunchKernelGGL((k_refine_wg<DT, METRIC, 4>), dim3((unsigned)p.nq), dim3(64 * 4), 0, s, p);
    else if (p.wg == 8)
        hipLaunchKernelGGL((k_refine_wg<DT, METRIC, 8>), dim3((unsigned)p.nq), dim3(64 * 8), 0, s, p);
    else if (p.wg)
        hipLaunchKernelGGL((k_refine_wg<DT, METRIC, 16>), dim3((unsigned)p.nq), dim3(64 * 16), 0, s, p);
    else if (p.prefetch > 1)
        hipLaunchKernelGGL((k_refine<DT, METRIC, 4>), dim3((unsigned)((p.nq + 3) / 4)), dim3(256), 0, s, p);
    else
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
static void fb_t(hipStream_t s, const char* codes, int row_bytes, int kdim, int64_t ntotal, const float* qf32,
                 const int* n_flag, int k, float* cd, int* ci) {
    hipLaunchKernelGGL((k_fb_scan<DT, METRIC>), dim3(FB_SCAN_GRID), dim3(BT_THREADS), 0, s, codes, row_bytes, kdim,
                       ntotal, qf32, n_flag, k, cd, ci);
}

hipError_t launch_exact_fallback(int st_dt, int metric, const char* codes, int row_bytes, int kdim, int64_t ntotal,
                                 const float* qf32, const int* n_flag, int k, int64_t id_offset, float* cand_d,
                                 int* cand_i, float* D, int64_t* I, hipStream_t s) {
    if (metric == L2) {
        if (st_dt == F32) fb_t<F32, L2>(s, codes, row_bytes, kdim, ntotal, qf32, n_flag, k, cand_d, cand_i);
        else if (st_dt == BF16) fb_t<BF16, L2>(s, codes, row_bytes, kdim, ntotal, qf32, n_flag, k, cand_d, cand_i);
        else fb_t<F16, L2>(s, codes, row_bytes, kdim, ntotal, qf32, n_flag, k, cand_d, cand_i);
    } else {
        if (st_dt == F32) fb_t<F32, IP>(s, codes, row_bytes, kdim, ntotal, qf32, n_flag, k, cand_d, cand_i);
        else if (st_dt == BF16) fb_t<BF16, IP>(s, codes, row_bytes, kdim, ntotal, qf32, n_flag, k, cand_d, cand_i);
        else fb_t<F16, IP>(s, codes, row_bytes, kdim, ntotal, qf32, n_flag, k, cand_d, cand_i);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (metric == L2)
        hipLaunchKernelGGL(k_fb_merge<L2>, dim3(FB_MERGE_GRID), dim3(BT_THREADS), 0, s, n_flag, ntotal, k, cand_d,
                           cand_i, id_offset, D, I);
    else
        hipLaunchKernelGGL(k_fb_merge<IP>, dim3(FB_MERGE_GRID), dim3(BT_THREADS), 0, s, n_flag, ntotal, k, cand_d,
                           cand_i, id_offset, D, I);
    return hipGetLastError();
}

hipError_t launch_merge_shards(int metric, int nshards, int64_t nq, int k, const float* D_in, const int64_t* I_in,
                               float* D_out, int64_t* I_out, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    if (k > 64) {
        if (metric == L2)
            hipLaunchKernelGGL(k_merge_shards_big<L2>, dim3((unsigned)nq), dim3(BT_THREADS), 0, s, nshards, nq, k,
                               D_in, I_in, D_out, I_out);
        else
            hipLaunchKernelGGL(k_merge_shards_big<IP>, dim3((unsigned)nq), dim3(BT_THREADS), 0, s, nshards, nq, k,
                               D_in, I_in, D_out, I_out);
        return hipGetLastError();
    }
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
