// fx_hugek.hip -- search() and the shard merge for k > FX_BIG_K.
//
// faiss IndexFlatL2::search takes any k (faiss_store.py:49,64 and
// rag_datastore_manager.py:218 pass the caller's k straight through); the
// fused scan keeps at most FX_BIG_K candidates per query, so larger k takes
// this path instead: the exact distance of every (query, row) pair of a batch
// (fp64 sum, one rounding to fp32 -- the refine's and the oracle's
// definition), packed with the row id into one 64-bit sort key
//
//     key = ord(D') << idbits | row      (D' = D for L2, -D for IP)
//
// (ord: the order-preserving bits of a float, so unsigned key order is
// (D, id) order, faiss's), a radix sort of each query's keys (rocPRIM via
// hipCUB: one device-wide sort per query for large corpora, one segmented
// sort per batch for small ones), and the first k keys unpacked into D / I,
// padded with I = -1 / D = +-FLT_MAX past ntotal as faiss does.  HBM-bound:
// the corpus is read once per batch of HK_QB queries (the key kernel keeps
// HK_QB fp64 accumulators per row), the keys are written once and sorted.
//
// The shard merge (fx_merge_shards with k > FX_BIG_K) is a G-way merge of
// each query's gathered lists (each already in the index order).
#include "fx_device.h"

#include <hipcub/hipcub.hpp>

namespace fx {

constexpr int HK_QB = 8;               // queries per pass of the key kernel over a row
constexpr int HK_THREADS = 256;
constexpr int64_t HK_SEG_SORT_MAX = 1 << 16;  // corpora up to this many rows: segmented sort per batch

// order-preserving bits of a float key, -0 folded into +0 (equal as floats)
__device__ __forceinline__ unsigned hk_ord(float f) { return f2ord(f + 0.0f); }

// queries [n][d] (dtype q_dt) -> fp32 [n][kdim], zero padded (exact_partial
// walks the whole padded row)
__global__ __launch_bounds__(HK_THREADS) void k_hk_queries(const void* __restrict__ q, int q_dt, int64_t n, int d,
                                                           int kdim, float* __restrict__ out) {
    const int64_t total = n * kdim;
    for (int64_t i = (int64_t)blockIdx.x * HK_THREADS + threadIdx.x; i < total; i += (int64_t)gridDim.x * HK_THREADS) {
        const int64_t r = i / kdim;
        const int c = (int)(i - r * kdim);
        out[i] = c < d ? load_elem(q, r * d + c, q_dt) : 0.0f;
    }
}

// key of every (query, row) pair of the batch: work item = (row, group of
// HK_QB queries); the row's 16-B chunks are loaded once per group
template <int DT, int METRIC>
__global__ __launch_bounds__(HK_THREADS) void k_hk_keys(const char* __restrict__ codes, int row_bytes, int kdim,
                                                        int64_t ntotal, const float* __restrict__ qf32, int qb,
                                                        int idbits, uint64_t* __restrict__ keys) {
    constexpr int E = DT == F32 ? 4 : 8;
    const int ngrp = (qb + HK_QB - 1) / HK_QB;
    const int64_t items = ntotal * ngrp;
    for (int64_t w = (int64_t)blockIdx.x * HK_THREADS + threadIdx.x; w < items; w += (int64_t)gridDim.x * HK_THREADS) {
        const int g = (int)(w / ntotal);
        const int64_t row = w - (int64_t)g * ntotal;
        const int q0 = g * HK_QB;
        const int nqg = min(HK_QB, qb - q0);
        const char* yrow = codes + row * row_bytes;
        double acc[HK_QB];
#pragma unroll
        for (int j = 0; j < HK_QB; ++j) acc[j] = 0.0;
        for (int c = 0; c * 16 < row_bytes; ++c) {
            float y[E];
            load_chunk<DT>(yrow + c * 16, y);
#pragma unroll
            for (int j = 0; j < HK_QB; ++j) {
                if (j < nqg) {
                    const float* xc = qf32 + (int64_t)(q0 + j) * kdim + c * E;
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        if (METRIC == L2) {
                            const double df = (double)xc[e] - (double)y[e];
                            acc[j] = fma(df, df, acc[j]);
                        } else {
                            acc[j] = fma((double)xc[e], (double)y[e], acc[j]);
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < HK_QB; ++j) {
            if (j < nqg) {
                const float f = METRIC == L2 ? (float)acc[j] : -(float)acc[j];
                keys[(int64_t)(q0 + j) * ntotal + row] = ((uint64_t)hk_ord(f) << idbits) | (uint64_t)row;
            }
        }
    }
}

__global__ void k_hk_offsets(int* __restrict__ offs, int nseg, int seglen) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i <= nseg; i += gridDim.x * blockDim.x) offs[i] = i * seglen;
}

// first k keys of each sorted segment -> D / I (rows q0 .. q0 + nseg of the output)
__global__ __launch_bounds__(HK_THREADS) void k_hk_out(const uint64_t* __restrict__ sorted, int64_t seglen, int nseg,
                                                       int k, int idbits, int metric, int64_t id_offset,
                                                       float* __restrict__ D, int64_t* __restrict__ I) {
    const int64_t total = (int64_t)nseg * k;
    const uint64_t idmask = (idbits >= 64) ? ~0ull : ((1ull << idbits) - 1);
    for (int64_t i = (int64_t)blockIdx.x * HK_THREADS + threadIdx.x; i < total; i += (int64_t)gridDim.x * HK_THREADS) {
        const int64_t q = i / k, t = i - q * k;
        if (t < seglen) {
            const uint64_t key = sorted[q * seglen + t];
            const float f = ord2f((unsigned)(key >> idbits));
            D[i] = metric == L2 ? f : -f;
            I[i] = (int64_t)(key & idmask) + id_offset;
        } else {
            D[i] = metric == L2 ? FLT_MAX : -FLT_MAX;
            I[i] = -1;
        }
    }
}

namespace {

int id_bits(int64_t ntotal) {
    int b = 1;
    while (b < 32 && ((int64_t)1 << b) < ntotal) ++b;
    return b;
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

unsigned grid_for(int64_t items) {
    const int64_t g = (items + HK_THREADS - 1) / HK_THREADS;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 8192));
}

// rocPRIM temporary bytes of one batch's sort
hipError_t sort_temp_bytes(int64_t ntotal, int qb, int end_bit, size_t* bytes) {
    *bytes = 0;
    if (ntotal > HK_SEG_SORT_MAX)
        return hipcub::DeviceRadixSort::SortKeys(nullptr, *bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                 (int)ntotal, 0, end_bit, (hipStream_t)0);
    return hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, *bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                      (int)(ntotal * qb), qb, (const int*)nullptr,
                                                      (const int*)nullptr, 0, end_bit, (hipStream_t)0);
}

struct HkCarve {
    size_t qf32 = 0, keys = 0, sorted = 0, offs = 0, temp = 0, temp_bytes = 0, total = 0;
};

hipError_t carve(int64_t ntotal, int kdim, int qb, HkCarve* c) {
    const int end_bit = 32 + id_bits(ntotal);
    hipError_t e = sort_temp_bytes(ntotal, qb, end_bit, &c->temp_bytes);
    if (e != hipSuccess) return e;
    size_t o = 0;
    c->qf32 = o;
    o = align_up(o + (size_t)qb * kdim * 4);
    c->keys = o;
    o = align_up(o + (size_t)qb * ntotal * 8);
    c->sorted = o;
    o = align_up(o + (size_t)qb * ntotal * 8);
    c->offs = o;
    o = align_up(o + (size_t)(qb + 1) * 4);
    c->temp = o;
    o = align_up(o + c->temp_bytes);
    c->total = o;
    return hipSuccess;
}

template <int DT, int METRIC>
void launch_keys_t(const HugeKParams& p, const float* qf32, int qb, int idbits, uint64_t* keys, hipStream_t s) {
    const int64_t items = p.ntotal * ((qb + HK_QB - 1) / HK_QB);
    hipLaunchKernelGGL((k_hk_keys<DT, METRIC>), dim3(grid_for(items)), dim3(HK_THREADS), 0, s, p.codes, p.row_bytes,
                       p.kdim, p.ntotal, qf32, qb, idbits, keys);
}

void launch_keys(const HugeKParams& p, const float* qf32, int qb, int idbits, uint64_t* keys, hipStream_t s) {
    if (p.metric == L2) {
        if (p.st_dt == F32) launch_keys_t<F32, L2>(p, qf32, qb, idbits, keys, s);
        else if (p.st_dt == BF16) launch_keys_t<BF16, L2>(p, qf32, qb, idbits, keys, s);
        else launch_keys_t<F16, L2>(p, qf32, qb, idbits, keys, s);
    } else {
        if (p.st_dt == F32) launch_keys_t<F32, IP>(p, qf32, qb, idbits, keys, s);
        else if (p.st_dt == BF16) launch_keys_t<BF16, IP>(p, qf32, qb, idbits, keys, s);
        else launch_keys_t<F16, IP>(p, qf32, qb, idbits, keys, s);
    }
}

}  // namespace

int hugek_batch(int64_t ntotal, int64_t nq) {
    // keys of a batch <= 2^27 (1 GiB per key buffer), at least one query
    const int64_t qb = std::max<int64_t>(1, ((int64_t)1 << 27) / std::max<int64_t>(ntotal, 1));
    return (int)std::min<int64_t>(qb, std::max<int64_t>(nq, 1));
}

hipError_t hugek_workspace(int64_t ntotal, int kdim, int qb, size_t* bytes) {
    HkCarve c;
    hipError_t e = carve(ntotal, kdim, qb, &c);
    *bytes = c.total;
    return e;
}

hipError_t launch_hugek_search(const HugeKParams& p, void* ws, size_t ws_bytes, int qb, hipStream_t s) {
    HkCarve c;
    hipError_t e = carve(p.ntotal, p.kdim, qb, &c);
    if (e != hipSuccess) return e;
    if (c.total > ws_bytes || p.ntotal <= 0 || p.ntotal > INT_MAX) return hipErrorInvalidValue;
    char* base = (char*)ws;
    float* qf32 = (float*)(base + c.qf32);
    uint64_t* keys = (uint64_t*)(base + c.keys);
    uint64_t* sorted = (uint64_t*)(base + c.sorted);
    int* offs = (int*)(base + c.offs);
    void* temp = base + c.temp;
    const int idbits = id_bits(p.ntotal);
    const int end_bit = 32 + idbits;
    const int esz = p.q_dt == F32 ? 4 : 2;
    for (int64_t b0 = 0; b0 < p.nq; b0 += qb) {
        const int nb = (int)std::min<int64_t>(qb, p.nq - b0);
        hipLaunchKernelGGL(k_hk_queries, dim3(grid_for((int64_t)nb * p.kdim)), dim3(HK_THREADS), 0, s,
                           (const char*)p.q + b0 * p.d * esz, p.q_dt, (int64_t)nb, p.d, p.kdim, qf32);
        launch_keys(p, qf32, nb, idbits, keys, s);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        size_t tb = c.temp_bytes;
        if (p.ntotal > HK_SEG_SORT_MAX) {
            for (int j = 0; j < nb; ++j) {
                e = hipcub::DeviceRadixSort::SortKeys(temp, tb, keys + (int64_t)j * p.ntotal,
                                                      sorted + (int64_t)j * p.ntotal, (int)p.ntotal, 0, end_bit, s);
                if (e != hipSuccess) return e;
            }
        } else {
            hipLaunchKernelGGL(k_hk_offsets, dim3(1), dim3(256), 0, s, offs, nb, (int)p.ntotal);
            e = hipcub::DeviceSegmentedRadixSort::SortKeys(temp, tb, keys, sorted, (int)(p.ntotal * nb), nb, offs,
                                                           offs + 1, 0, end_bit, s);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_hk_out, dim3(grid_for((int64_t)nb * p.k)), dim3(HK_THREADS), 0, s, sorted, p.ntotal, nb,
                           p.k, idbits, p.metric, p.id_offset, p.D + b0 * p.k, p.I + b0 * p.k);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// shard merge for k > FX_BIG_K: a G-way merge of each query's gathered lists
// ---------------------------------------------------------------------------
// Every per-shard list is already in the index order ((D, id) ascending for L2,
// (-D, id) for IP; missing entries I = -1 last), so the merged top k is a
// G-way merge: one thread per query keeps the G list heads and emits the
// smallest k times (O(k G) per query; the rare large-k path).
constexpr int HKM_MAXG = FX_HUGEK_MAX_SHARDS;

__global__ __launch_bounds__(64) void k_hkm_merge(int nshards, int64_t nq, int k, int metric,
                                                  const float* __restrict__ D_in, const int64_t* __restrict__ I_in,
                                                  float* __restrict__ D_out, int64_t* __restrict__ I_out) {
    const int64_t q = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (q >= nq) return;
    int pos[HKM_MAXG];
    float hk[HKM_MAXG];
    int64_t hid[HKM_MAXG];
    auto load = [&](int g) {
        const int64_t src = ((int64_t)g * nq + q) * k + pos[g];
        const int64_t id = pos[g] < k ? I_in[src] : -1;
        hid[g] = id < 0 ? INT64_MAX : id;
        hk[g] = id < 0 ? FX_INF : (metric == L2 ? D_in[src] : -D_in[src]);
    };
    for (int g = 0; g < nshards; ++g) {
        pos[g] = 0;
        load(g);
    }
    for (int t = 0; t < k; ++t) {
        int best = 0;
        for (int g = 1; g < nshards; ++g)
            if (hk[g] < hk[best] || (hk[g] == hk[best] && hid[g] < hid[best])) best = g;
        const int64_t o = q * k + t;
        if (hid[best] == INT64_MAX) {
            D_out[o] = metric == L2 ? FLT_MAX : -FLT_MAX;
            I_out[o] = -1;
            continue;
        }
        D_out[o] = metric == L2 ? hk[best] : -hk[best];
        I_out[o] = hid[best];
        ++pos[best];
        load(best);
    }
}

hipError_t launch_merge_shards_sort(int metric, int nshards, int64_t nq, int k, const float* D_in, const int64_t* I_in,
                                    float* D_out, int64_t* I_out, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    if (nshards > HKM_MAXG) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_hkm_merge, dim3((unsigned)((nq + 63) / 64)), dim3(64), 0, s, nshards, nq, k, metric, D_in,
                       I_in, D_out, I_out);
    return hipGetLastError();
}

}  // namespace fx
