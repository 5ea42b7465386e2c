// fx_index.cpp -- host implementation of the C ABI declared in
// include/fx_index.h.  Owns HBM (code matrix, row norms, search workspace),
// sequences the kernels of fx_kernels.hip on one HIP stream per index, and
// reproduces faiss's IndexFlatL2 API contract (faiss_store.py:29-128,
// rag_datastore_manager.py:138-218) at the C level.
#include "../../include/fx_index.h"

#include <float.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "fx_internal.h"

using namespace fx;

namespace {

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                             \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess)                                                                     \
            return set_err(FX_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                           __LINE__);                                                             \
    } while (0)

// Restores the caller's current device on scope exit (torch keeps its own
// notion of the current device per thread).
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t want) {
        if (want <= bytes) return hipSuccess;
        const size_t grow = std::max(want, bytes + bytes / 2);
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, grow);
        if (e == hipSuccess) bytes = grow;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

}  // namespace

struct FxIndex {
    int d = 0, dtype = F32, metric = L2, device = 0, normalize = 0;
    int row_bytes = 0, kdim = 0;
    int64_t ntotal = 0, cap_rows = 0, id_offset = 0;
    char* codes = nullptr;
    float* norms = nullptr;
    unsigned* max_sq_bits = nullptr;  // device
    hipStream_t own_stream = nullptr;
    hipStream_t user_stream = nullptr;
    // search workspace
    DevBuf qin, qf32, qop, qeps, cand_d, cand_i, cand2_d, cand2_i, dws, iws, flag, fbc_d, fbc_i, stage, gtau, trace,
        dbgbuf, stamps, pub;
    // F32S scan image of an fp32 index (default; FX_F32_SPLIT=0 scans the fp32
    // rows with fp32 MFMA instead): rows [0, split_rows) are current.  L2
    // indexes centre it (FX_CENTER=0: off): image rows fl(y - mu), their
    // |.|^2 in cnorms (the scan's srcC), max in max_sq_bits[1]; mu = mean of a
    // row sample, recomputed (and the image rebuilt) whenever ntotal has
    // doubled since (mu_rows), so the centre follows the data at O(1)
    // amortised cost per added row
    DevBuf split, cnorms, centre, mu_part, qxn2;
    int64_t split_rows = 0, mu_rows = 0;
    bool centred = false;
    // FX_SEARCH_GRAPH=1: the search of a small host batch (the reference's
    // one-query call form) replayed as one hipGraph per shape, over pinned
    // host staging; `gkey` = the shape and every buffer the graph captured
    hipGraphExec_t gexec = nullptr;
    std::vector<uint64_t> gkey;
    bool gfailed = false;
    void* ghq = nullptr;
    float* ghD = nullptr;
    int64_t* ghI = nullptr;
    int* ghnf = nullptr;
    size_t ghq_bytes = 0, ghd_n = 0;
    int64_t last_fallbacks = 0;
    // uncertified count of the last search, copied stream-ordered into pinned
    // memory; read (after a stream sync) only when asked for (fb_pending)
    int* pin_nf = nullptr;
    bool fb_pending = false;
    // profiling
    bool profile = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_scan, ev_merge;
    std::mutex mu;

    hipStream_t stream() const { return user_stream ? user_stream : own_stream; }
};

namespace {

int check_dtype(int dt) { return dt == FX_F32 || dt == FX_BF16 || dt == FX_F16; }

hipError_t grow(FxIndex* h, int64_t need_rows) {
    if (need_rows <= h->cap_rows) return hipSuccess;
    int64_t cap = round_up(std::max<int64_t>(need_rows, h->cap_rows + h->cap_rows / 2), TILE_R);
    char* codes = nullptr;
    float* norms = nullptr;
    hipError_t e = hipMalloc(&codes, (size_t)cap * h->row_bytes);
    if (e != hipSuccess) return e;
    e = hipMalloc(&norms, (size_t)cap * sizeof(float));
    if (e != hipSuccess) {
        (void)hipFree(codes);
        return e;
    }
    hipStream_t s = h->stream();
    // zero-fill: padding rows of the last tile must be finite
    e = hipMemsetAsync(codes + (size_t)h->ntotal * h->row_bytes, 0, (size_t)(cap - h->ntotal) * h->row_bytes, s);
    // padding rows: |y|^2 = +inf keeps them out of the scan's candidate lists
    if (e == hipSuccess) e = hipMemsetD32Async((hipDeviceptr_t)(norms + h->ntotal), 0x7f800000u, (size_t)(cap - h->ntotal), s);
    if (e == hipSuccess && h->ntotal > 0) {
        e = hipMemcpyAsync(codes, h->codes, (size_t)h->ntotal * h->row_bytes, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(norms, h->norms, (size_t)h->ntotal * sizeof(float), hipMemcpyDeviceToDevice, s);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        (void)hipFree(codes);
        (void)hipFree(norms);
        return e;
    }
    if (h->codes) (void)hipFree(h->codes);
    if (h->norms) (void)hipFree(h->norms);
    h->codes = codes;
    h->norms = norms;
    h->cap_rows = cap;
    return hipSuccess;
}

// choose corpus splits per query tile: enough workgroups to fill 256 CUs
// several times over (1 workgroup per CU resident: 129 KiB LDS)
// k > KP: no cross-split pruning (ScanParams.share = 0) and at least k/4
// splits, so that a split's KP-list rarely holds fewer than all of its top-k
// rows and the certification bound (the smallest full split's KP-th key)
// lies far beyond the k-th distance
// split count whose live workgroups (one per CU: the scans' LDS) fill whole
// rounds of 256 CUs best, with >= ~4 rounds and >= min_tiles tiles per split
int fill_splits(int live_tiles, int eff_tiles, int n_ctiles, int min_tiles) {
    const int max_splits = std::max(1, n_ctiles / min_tiles);
    const int s0 = std::max(1, std::min(max_splits, (1024 + eff_tiles - 1) / eff_tiles));
    int best = s0;
    double best_eff = 0.0;
    for (int s = s0; s <= std::min(max_splits, 4 * s0); ++s) {
        const double live = (double)live_tiles * s;
        const double rounds = std::ceil(live / 256.0);
        const double eff = live / (rounds * 256.0);
        if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
        if (eff > 0.985) break;
    }
    return best;
}

// choose the scan kernel and its corpus splits per query tile
// k > KP: no cross-split pruning (ScanParams.share = 0) and at least k/4
// splits, so that a split's KP-list rarely holds fewer than all of its top-k
// rows and the certification bound (the smallest full split's KP-th key)
// lies far beyond the k-th distance
void plan_scan(const FxIndex* h, int64_t nq, int k, int scan_dt, ScanParams& p) {
    p.n_qtiles = (int)((nq + TILE_Q - 1) / TILE_Q);
    p.n_ctiles = (int)((h->ntotal + TILE_R - 1) / TILE_R);
    p.q32_tiles = 0;
    p.n_wtiles = 0;
    p.place = 0;
    p.sx = 0;
    p.pub = nullptr;
    p.prune_rank = KP;
    p.share = k <= KP ? 1 : 0;
    const int rb64 = h->row_bytes / 64;
    const char* q32_env = getenv("FX_SCAN_Q32");
    if (q32_env && atoi(q32_env) == 1 && nq <= 32 && k <= KP && h->row_bytes % 64 == 0 &&
        (rb64 == 8 || rb64 == 12 || rb64 == 16 || rb64 == 24)) {
        // small batch (k_scan_q32): one 32-query tile; one round of one
        // workgroup per CU, each split >= 4 tiles; every corpus byte read once
        p.q32_tiles = (int)((nq + 31) / 32);
        p.qt_per_xcd = 0;
        p.splits = std::max(1, std::min(p.n_ctiles / 4, 256 / p.q32_tiles));
        p.grid = p.q32_tiles * p.splits;
        return;
    }
    // large batches: the wide-tile scan (192 queries per workgroup; FX_SCAN_W
    // = 0 / 1 forces it off / on where it has a kernel for the row width)
    const char* w_env = getenv("FX_SCAN_W");
    const bool want_w = w_env ? atoi(w_env) == 1 : false;
    const bool wide = want_w && scan_w_supported(scan_dt, h->row_bytes);
    if (wide) p.n_wtiles = (int)((nq + scan_w_queries() - 1) / scan_w_queries());
    const int ntl = wide ? p.n_wtiles : p.n_qtiles;              // query tiles of the chosen scan
    const int nct = wide ? (int)((h->ntotal + 63) / 64) : p.n_ctiles;  // its corpus tiles
    const int min_tiles = wide ? 8 : 4;
    // placement (map_tile): FX_SCAN_PLACE = 0 / 1 forces query-tile groups /
    // the corpus-partitioned form
    // default: corpus-partitioned for k_scan_v4 (fewer corpus fetches past L2:
    // 257 vs 742 GB per config (d) launch, and ~2 % faster)
    const char* pl_env = getenv("FX_SCAN_PLACE");
    const int place = pl_env ? atoi(pl_env) : (wide ? 0 : 1);
    if (place == 1 && ntl >= 8 && nct >= 8 * min_tiles) {
        // XCD x owns 1/8 of the corpus for every query tile; sx splits per
        // XCD so that its ntl * sx blocks fill whole rounds of its 32 CUs
        p.place = 1;
        p.qt_per_xcd = 0;
        const int max_sx = std::max(1, nct / (8 * min_tiles));
        int best = 1;
        double best_eff = 0.0;
        for (int sx = 1; sx <= std::min(max_sx, 16); ++sx) {
            const double live = (double)ntl * sx;
            const double eff = live / (std::ceil(live / 32.0) * 32.0);
            if (eff > best_eff + 1e-9) { best_eff = eff; best = sx; }
            if (eff > 0.985 && live >= 128) break;
        }
        // FX_SCAN_SX: splits per XCD, for placement A/B runs only
        if (const char* sx_env = getenv("FX_SCAN_SX"); sx_env && *sx_env) best = std::max(1, std::min(max_sx, atoi(sx_env)));
        if (k > KP) best = std::max(best, std::min(max_sx, ((k + 3) / 4 + 7) / 8));
        p.sx = best;
        p.splits = 8 * best;
        p.grid = 8 * ntl * best;
        return;
    }
    p.qt_per_xcd = ntl >= 8 ? (ntl + 7) / 8 : 0;
    const int eff_q = p.qt_per_xcd > 0 ? 8 * p.qt_per_xcd : ntl;
    p.splits = fill_splits(ntl, eff_q, nct, min_tiles);
    if (k > KP) p.splits = std::max(p.splits, std::min(std::max(1, nct / min_tiles), (k + 3) / 4));
    p.grid = eff_q * p.splits;
}

// k > KP: approx candidates the refine re-ranks exactly (k_refine_big)
int big_k1(int k) { return k > KP ? std::max(2 * k, 64) : 0; }

// small batches over many splits: merge the candidate lists 16 splits at a
// time before the refine (k_reduce_cand; FX_REDUCE_CAND=0 turns it off)
bool use_reduce(int k, int64_t nq, int splits) {
    const char* e = getenv("FX_REDUCE_CAND");
    return k <= KP && nq <= 256 && splits >= 64 && !(e && atoi(e) == 0);
}

hipError_t ensure_pinned_count(FxIndex* h) {
    if (h->pin_nf) return hipSuccess;
    hipError_t e = hipHostMalloc((void**)&h->pin_nf, sizeof(int), hipHostMallocDefault);
    if (e == hipSuccess) *h->pin_nf = 0;
    return e;
}

// fp32 index (unless FX_F32_SPLIT=0): bring its F32S scan image up to date
// (rows appended since the last search); *split says whether the scan uses it
hipError_t update_scan_image(FxIndex* h, bool* split) {
    const int rb64 = h->row_bytes / 64;
    const char* split_env = getenv("FX_F32_SPLIT");
    *split = !(split_env && atoi(split_env) == 0) && h->dtype == F32 && h->row_bytes % 64 == 0 &&
             (rb64 == 8 || rb64 == 12 || rb64 == 16 || rb64 == 24);
    if (!*split) return hipSuccess;
    hipStream_t s = h->stream();
    const void* old = h->split.p;
    const void* old_n = h->cnorms.p;
    hipError_t e = h->split.ensure((size_t)h->cap_rows * h->row_bytes);
    if (e == hipSuccess) e = h->cnorms.ensure((size_t)h->cap_rows * 4);
    if (e != hipSuccess) return e;
    bool rebuild = h->split.p != old || h->cnorms.p != old_n || h->split_rows > h->ntotal;
    const char* ce = getenv("FX_CENTER");
    const bool centre = h->metric == L2 && !(ce && atoi(ce) == 0);
    if (centre != h->centred) rebuild = true;
    if (centre && (h->mu_rows == 0 || h->ntotal >= 2 * h->mu_rows)) {
        // (re)centre on the current rows
        if ((e = h->centre.ensure((size_t)h->kdim * 4)) != hipSuccess) return e;
        if ((e = h->mu_part.ensure((size_t)MU_GROUPS * h->kdim * 8)) != hipSuccess) return e;
        if ((e = launch_mu((const float*)h->codes, h->kdim, h->d, h->ntotal, (double*)h->mu_part.p, (float*)h->centre.p,
                           s)) != hipSuccess)
            return e;
        h->mu_rows = h->ntotal;
        rebuild = true;
    }
    h->centred = centre;
    if (rebuild) {  // zero image (finite padding rows), +inf padding norms
        if ((e = hipMemsetAsync(h->split.p, 0, h->split.bytes, s)) != hipSuccess) return e;
        if ((e = hipMemsetD32Async((hipDeviceptr_t)h->cnorms.p, 0x7f800000u, h->cnorms.bytes / 4, s)) != hipSuccess)
            return e;
        if ((e = hipMemsetAsync(h->max_sq_bits + 1, 0, 4, s)) != hipSuccess) return e;
        h->split_rows = 0;
    }
    e = launch_split_rows((const float*)h->codes, h->kdim, h->split_rows, h->ntotal,
                          centre ? (const float*)h->centre.p : nullptr, h->split.p, (float*)h->cnorms.p,
                          h->max_sq_bits + 1, s);
    if (e == hipSuccess) h->split_rows = h->ntotal;
    return e;
}

int do_search(FxIndex* h, int64_t nq, const void* q, int q_dtype, int q_mem, int k, float* D, int64_t* I,
              int out_mem) {
    hipStream_t s = h->stream();
    const int64_t nq_pad = round_up(nq, QPAD);
    const int qes = dtype_size(q_dtype);
    // queries -> device
    const void* qdev = q;
    if (q_mem == FX_MEM_HOST) {
        HIP_TRY(h->qin.ensure((size_t)nq * h->d * qes));
        HIP_TRY(hipMemcpyAsync(h->qin.p, q, (size_t)nq * h->d * qes, hipMemcpyHostToDevice, s));
        qdev = h->qin.p;
    }
    HIP_TRY(h->qf32.ensure((size_t)nq_pad * h->kdim * 4));
    HIP_TRY(h->qop.ensure((size_t)nq_pad * h->row_bytes));
    void* qop = h->qop.p;
    HIP_TRY(h->qeps.ensure((size_t)nq * 4));
    // fp32 index: scan it through its split-bf16 image (F32S:
    // 3 bf16 products per term on the bf16 MFMA pipe instead of fp32 MFMA);
    // the refine and the certification still use the fp32 rows
    bool split = false;
    HIP_TRY(update_scan_image(h, &split));
    const int scan_dt = split ? (int)F32S : h->dtype;
    HIP_TRY(h->qxn2.ensure((size_t)nq * 8));
    HIP_TRY(launch_prep_queries(qdev, q_dtype, nq, nq_pad, h->d, h->kdim, scan_dt, h->metric, (float*)h->qf32.p,
                                qop, (float*)h->qeps.p, h->max_sq_bits + (split ? 1 : 0),
                                split && h->centred ? (const float*)h->centre.p : nullptr, (double*)h->qxn2.p, s));

    ScanParams sp;
    plan_scan(h, nq, k, scan_dt, sp);
    sp.codes = split ? (const char*)h->split.p : h->codes;
    sp.norms = split ? (const float*)h->cnorms.p : h->norms;
    sp.ntotal = h->ntotal;
    sp.row_bytes = h->row_bytes;
    sp.qop = (const char*)qop;
    sp.nq = nq;
    sp.dbg = getenv("FX_SCAN_DBG") ? atoi(getenv("FX_SCAN_DBG")) : 0;
    HIP_TRY(h->gtau.ensure((size_t)nq_pad * 4));
    sp.gtau = (unsigned*)h->gtau.p;
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)sp.gtau, 0xff800000u, (size_t)nq_pad, s));  // ord(+inf)
    // k_scan_v4's published per-split lists (the union threshold, see
    // compact_wave): slow-path tiles 25.7 -> 16.5 %, config (d) -3 %;
    // FX_SCAN_PUB=0 turns them off
    const char* pub_env = getenv("FX_SCAN_PUB");
    if (sp.share && sp.q32_tiles == 0 && sp.n_wtiles == 0 && sp.splits > 1 && !(pub_env && atoi(pub_env) == 0)) {
        const size_t npub = (size_t)sp.n_qtiles * TILE_Q * sp.splits * KP;
        HIP_TRY(h->pub.ensure(npub * 4));
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)h->pub.p, 0x7f800000u, npub, s));  // +inf: no entry
        sp.pub = (float*)h->pub.p;
        // union bound taken at rank max(2k, 16) (<= KP): tighter pruning; the
        // refine's certification bound is capped by the final threshold
        const char* rk_env = getenv("FX_PRUNE_RANK");
        sp.prune_rank = rk_env ? atoi(rk_env) : std::max(2 * k, 16);
        sp.prune_rank = std::max(k, std::min(KP, sp.prune_rank));
    }
    const int cand_splits = sp.splits;  // one candidate list per (query, split)
    const size_t ncand = (size_t)sp.n_qtiles * cand_splits * TILE_Q * KP;
    HIP_TRY(h->cand_d.ensure(ncand * 4));
    HIP_TRY(h->cand_i.ensure(ncand * 4));
    sp.cand_d = (float*)h->cand_d.p;
    sp.cand_i = (int*)h->cand_i.p;
    // diagnostics: per-block placement/timing of the scan -> binary file
    const char* trace_path = getenv("FX_SCAN_TRACE");
    const size_t grid = (size_t)sp.grid;
    sp.trace = nullptr;
    sp.dbgbuf = nullptr;
    sp.stamps = nullptr;
    const char* stamp_path = getenv("FX_SCAN_STAMPS");
    if (stamp_path) {
        HIP_TRY(h->stamps.ensure(grid * 4 * 128));
        HIP_TRY(hipMemsetAsync(h->stamps.p, 0, grid * 4 * 128, s));
        sp.stamps = (unsigned long long*)h->stamps.p;
    }
    const size_t nkeys = (size_t)sp.n_qtiles * TILE_Q * sp.n_ctiles * TILE_R;
    if ((sp.dbg & 32) && nkeys <= (size_t)1 << 26) {
        HIP_TRY(h->dbgbuf.ensure(nkeys * 4));
        HIP_TRY(hipMemsetAsync(h->dbgbuf.p, 0xff, nkeys * 4, s));
        sp.dbgbuf = (unsigned*)h->dbgbuf.p;
    }
    if (trace_path) {
        HIP_TRY(h->trace.ensure(grid * 32));
        HIP_TRY(hipMemsetAsync(h->trace.p, 0, grid * 32, s));
        sp.trace = (unsigned long long*)h->trace.p;
    }

    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    if (h->profile) {
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        HIP_TRY(hipEventCreate(&e2));
        HIP_TRY(hipEventRecord(e0, s));
    }
    HIP_TRY(launch_scan(scan_dt, h->metric, sp, s));
    if (h->profile) HIP_TRY(hipEventRecord(e1, s));

    float* Dd = D;
    int64_t* Id = I;
    if (out_mem == FX_MEM_HOST) {
        HIP_TRY(h->dws.ensure((size_t)nq * k * 4));
        HIP_TRY(h->iws.ensure((size_t)nq * k * 8));
        Dd = (float*)h->dws.p;
        Id = (int64_t*)h->iws.p;
    }
    HIP_TRY(h->flag.ensure((size_t)(nq + 1) * 4));
    int* n_flag = (int*)h->flag.p;
    HIP_TRY(hipMemsetAsync(n_flag, 0, 4, s));

    RefineParams rp;
    rp.cand_d = sp.cand_d;
    rp.cand_i = sp.cand_i;
    rp.splits = cand_splits;
    rp.nq = nq;
    rp.k = k;
    rp.codes = h->codes;
    rp.row_bytes = h->row_bytes;
    rp.kdim = h->kdim;
    rp.qf32 = (const float*)h->qf32.p;
    rp.qeps = (const float*)h->qeps.p;
    rp.qxn2 = (const double*)h->qxn2.p;
    rp.id_offset = h->id_offset;
    rp.D = Dd;
    rp.I = Id;
    rp.n_flag = n_flag;
    rp.flag_list = n_flag + 1;
    // small batches: one wave per query walks splits * KP candidates (256 splits
    // at nq = 1); issue 4 chunks of loads at a time (nq = 1: 0.84 -> ~0.3 ms)
    rp.prefetch = (sp.q32_tiles > 0 || nq <= 256) ? 4 : 1;
    rp.k1 = big_k1(k);
    rp.force_fb = getenv("FX_FORCE_FALLBACK") ? atoi(getenv("FX_FORCE_FALLBACK")) : 0;
    rp.gtau = sp.share ? sp.gtau : nullptr;
    if (use_reduce(k, nq, cand_splits)) {
        const size_t nred = (size_t)sp.n_qtiles * ((cand_splits + 15) / 16) * TILE_Q * KP;
        HIP_TRY(h->cand2_d.ensure(nred * 4));
        HIP_TRY(h->cand2_i.ensure(nred * 4));
        int ng = 0;
        HIP_TRY(launch_reduce_cand(sp.cand_d, sp.cand_i, cand_splits, nq, sp.n_qtiles, (float*)h->cand2_d.p,
                                   (int*)h->cand2_i.p, &ng, s));
        rp.cand_d = (const float*)h->cand2_d.p;
        rp.cand_i = (const int*)h->cand2_i.p;
        rp.splits = ng;
    }
    HIP_TRY(launch_refine(h->dtype, h->metric, rp, s));
    if (h->profile) {
        HIP_TRY(hipEventRecord(e2, s));
        h->ev_scan.emplace_back(e0, e1);
        h->ev_merge.emplace_back(e1, e2);
    }

    // Certification result: uncertified queries (rare: only when the
    // candidate margin is inside the scan's worst-case rounding bound) are
    // re-ranked by the exact fp64 scan.  Decided on the device: both
    // fallback kernels are always enqueued and exit at once when the refine
    // flagged nothing, so no host round trip sits inside the search.
    if (sp.dbg == 0) {
        const size_t nfb = (size_t)std::max<int64_t>(4096, nq) * k;
        HIP_TRY(h->fbc_d.ensure(nfb * 4));
        HIP_TRY(h->fbc_i.ensure(nfb * 4));
        HIP_TRY(launch_exact_fallback(h->dtype, h->metric, h->codes, h->row_bytes, h->kdim, h->ntotal,
                                      (const float*)h->qf32.p, n_flag, k, h->id_offset, (float*)h->fbc_d.p,
                                      (int*)h->fbc_i.p, Dd, Id, s));
    }
    HIP_TRY(ensure_pinned_count(h));
    HIP_TRY(hipMemcpyAsync(h->pin_nf, n_flag, 4, hipMemcpyDeviceToHost, s));
    h->fb_pending = true;
    if (const char* cpath = getenv("FX_SCAN_CAND")) {  // diagnostics: raw scan candidate lists
        std::vector<float> cd(ncand);
        std::vector<int> ci(ncand);
        HIP_TRY(hipMemcpy(cd.data(), sp.cand_d, ncand * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(ci.data(), sp.cand_i, ncand * 4, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(cpath, "wb")) {
            fwrite(cd.data(), 4, ncand, f);
            fwrite(ci.data(), 4, ncand, f);
            fclose(f);
        }
    }
    if (sp.dbgbuf) {  // diagnostics: the scan's key matrix [n_qtiles*128][n_ctiles*128] -> file
        std::vector<float> kv(nkeys);
        HIP_TRY(hipMemcpy(kv.data(), sp.dbgbuf, nkeys * 4, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("FX_SCAN_KEYS") ? getenv("FX_SCAN_KEYS") : "/tmp/fx_keys.bin", "wb")) {
            fwrite(kv.data(), 4, kv.size(), f);
            fclose(f);
        }
    }
    if (sp.stamps) {
        std::vector<unsigned long long> st(grid * 4 * 16);
        HIP_TRY(hipMemcpy(st.data(), sp.stamps, grid * 4 * 128, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(stamp_path, "wb")) {
            fwrite(st.data(), 8, st.size(), f);
            fclose(f);
        }
    }
    if (sp.trace) {
        std::vector<unsigned long long> tr(grid * 4);
        HIP_TRY(hipMemcpy(tr.data(), sp.trace, grid * 32, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(trace_path, "wb")) {
            fwrite(tr.data(), 8, tr.size(), f);
            fclose(f);
        }
    }
    if (out_mem == FX_MEM_HOST) {
        HIP_TRY(hipMemcpyAsync(D, Dd, (size_t)nq * k * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(I, Id, (size_t)nq * k * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        h->last_fallbacks = *h->pin_nf;
        h->fb_pending = false;
    }
    return FX_OK;
}

// Shape + every device buffer a captured search touches: the graph is valid
// while all of them are unchanged
std::vector<uint64_t> graph_key(const FxIndex* h, int64_t nq, int q_dtype, int k, int scan_dt) {
    ScanParams sp;
    plan_scan(h, nq, k, scan_dt, sp);
    const char* se = getenv("FX_F32_SPLIT");  // (part of the key: unset and "1" both mean on)
    return {(uint64_t)nq, (uint64_t)q_dtype, (uint64_t)k, (uint64_t)h->ntotal, (uint64_t)h->id_offset,
            (uint64_t)(se ? atoi(se) : 1),
            (uint64_t)(getenv("FX_FORCE_FALLBACK") ? atoi(getenv("FX_FORCE_FALLBACK")) : 0),
            (uint64_t)sp.splits, (uint64_t)sp.q32_tiles, (uint64_t)sp.qt_per_xcd, (uint64_t)sp.n_wtiles,
            (uint64_t)sp.place, (uint64_t)sp.sx, (uint64_t)sp.grid,
            (uint64_t)(uintptr_t)h->codes, (uint64_t)(uintptr_t)h->norms, (uint64_t)(uintptr_t)h->split.p,
            (uint64_t)(uintptr_t)h->cnorms.p, (uint64_t)(uintptr_t)h->centre.p, (uint64_t)(uintptr_t)h->qxn2.p,
            (uint64_t)h->centred,
            (uint64_t)(uintptr_t)h->qin.p, (uint64_t)(uintptr_t)h->qf32.p, (uint64_t)(uintptr_t)h->qop.p,
            (uint64_t)(uintptr_t)h->qeps.p, (uint64_t)(uintptr_t)h->gtau.p, (uint64_t)(uintptr_t)h->cand_d.p,
            (uint64_t)(uintptr_t)h->cand_i.p, (uint64_t)(uintptr_t)h->cand2_d.p, (uint64_t)(uintptr_t)h->cand2_i.p,
            (uint64_t)(uintptr_t)h->dws.p, (uint64_t)(uintptr_t)h->iws.p,
            (uint64_t)(uintptr_t)h->flag.p, (uint64_t)(uintptr_t)h->fbc_d.p, (uint64_t)(uintptr_t)h->fbc_i.p};
}

void graph_release(FxIndex* h) {
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    h->gexec = nullptr;
    h->gkey.clear();
}

// Record the stream-ordered search of do_search (host queries, host results,
// no diagnostics) into h->gexec.  Runs right after a do_search of the same
// shape, so every workspace is sized and every kernel attribute set.
hipError_t graph_build(FxIndex* h, int64_t nq, int q_dtype, int k, bool split) {
    graph_release(h);
    hipStream_t s = h->stream();
    const size_t qb = (size_t)nq * h->d * dtype_size(q_dtype), nd = (size_t)nq * k;
    hipError_t e = hipSuccess;
    if (qb > h->ghq_bytes) {
        if (h->ghq) (void)hipHostFree(h->ghq);
        h->ghq = nullptr;
        h->ghq_bytes = 0;
        if ((e = hipHostMalloc(&h->ghq, qb, hipHostMallocDefault)) != hipSuccess) return e;
        h->ghq_bytes = qb;
    }
    if (nd > h->ghd_n) {
        if (h->ghD) (void)hipHostFree(h->ghD);
        if (h->ghI) (void)hipHostFree(h->ghI);
        h->ghD = nullptr;
        h->ghI = nullptr;
        h->ghd_n = 0;
        if ((e = hipHostMalloc((void**)&h->ghD, nd * 4, hipHostMallocDefault)) != hipSuccess) return e;
        if ((e = hipHostMalloc((void**)&h->ghI, nd * 8, hipHostMallocDefault)) != hipSuccess) return e;
        h->ghd_n = nd;
    }
    if (!h->ghnf && (e = hipHostMalloc((void**)&h->ghnf, 4, hipHostMallocDefault)) != hipSuccess) return e;

    const int scan_dt = split ? (int)F32S : h->dtype;
    const int64_t nq_pad = round_up(nq, QPAD);
    ScanParams sp;
    plan_scan(h, nq, k, scan_dt, sp);
    sp.codes = split ? (const char*)h->split.p : h->codes;
    sp.norms = split ? (const float*)h->cnorms.p : h->norms;
    sp.ntotal = h->ntotal;
    sp.row_bytes = h->row_bytes;
    sp.qop = (const char*)h->qop.p;
    sp.nq = nq;
    sp.dbg = 0;
    sp.gtau = (unsigned*)h->gtau.p;
    sp.cand_d = (float*)h->cand_d.p;
    sp.cand_i = (int*)h->cand_i.p;
    sp.trace = nullptr;
    sp.dbgbuf = nullptr;
    sp.stamps = nullptr;
    int* n_flag = (int*)h->flag.p;
    RefineParams rp;
    rp.cand_d = sp.cand_d;
    rp.cand_i = sp.cand_i;
    rp.splits = sp.splits;
    rp.nq = nq;
    rp.k = k;
    rp.codes = h->codes;
    rp.row_bytes = h->row_bytes;
    rp.kdim = h->kdim;
    rp.qf32 = (const float*)h->qf32.p;
    rp.qeps = (const float*)h->qeps.p;
    rp.qxn2 = (const double*)h->qxn2.p;
    rp.id_offset = h->id_offset;
    rp.D = (float*)h->dws.p;
    rp.I = (int64_t*)h->iws.p;
    rp.n_flag = n_flag;
    rp.flag_list = n_flag + 1;
    // small batches: one wave per query walks splits * KP candidates (256 splits
    // at nq = 1); issue 4 chunks of loads at a time (nq = 1: 0.84 -> ~0.3 ms)
    rp.prefetch = (sp.q32_tiles > 0 || nq <= 256) ? 4 : 1;
    rp.k1 = big_k1(k);
    rp.force_fb = getenv("FX_FORCE_FALLBACK") ? atoi(getenv("FX_FORCE_FALLBACK")) : 0;
    rp.gtau = sp.share ? sp.gtau : nullptr;

    if ((e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal)) != hipSuccess) return e;
    g_graph_capture = true;
    hipError_t ce = hipMemcpyAsync(h->qin.p, h->ghq, qb, hipMemcpyHostToDevice, s);
    if (ce == hipSuccess)
        ce = launch_prep_queries(h->qin.p, q_dtype, nq, nq_pad, h->d, h->kdim, scan_dt, h->metric, (float*)h->qf32.p,
                                 h->qop.p, (float*)h->qeps.p, h->max_sq_bits + (split ? 1 : 0),
                                 split && h->centred ? (const float*)h->centre.p : nullptr, (double*)h->qxn2.p, s);
    if (ce == hipSuccess)
        ce = hipMemsetD32Async((hipDeviceptr_t)sp.gtau, 0xff800000u, (size_t)nq_pad, s);
    if (ce == hipSuccess) ce = launch_scan(scan_dt, h->metric, sp, s);
    if (ce == hipSuccess) ce = hipMemsetAsync(n_flag, 0, 4, s);
    if (ce == hipSuccess && use_reduce(k, nq, sp.splits)) {  // sized by the preceding do_search
        int ng = 0;
        ce = launch_reduce_cand(sp.cand_d, sp.cand_i, sp.splits, nq, sp.n_qtiles, (float*)h->cand2_d.p,
                                (int*)h->cand2_i.p, &ng, s);
        rp.cand_d = (const float*)h->cand2_d.p;
        rp.cand_i = (const int*)h->cand2_i.p;
        rp.splits = ng;
    }
    if (ce == hipSuccess) ce = launch_refine(h->dtype, h->metric, rp, s);
    if (ce == hipSuccess)
        ce = launch_exact_fallback(h->dtype, h->metric, h->codes, h->row_bytes, h->kdim, h->ntotal,
                                   (const float*)h->qf32.p, n_flag, k, h->id_offset, (float*)h->fbc_d.p,
                                   (int*)h->fbc_i.p, rp.D, rp.I, s);
    if (ce == hipSuccess) ce = hipMemcpyAsync(h->ghD, rp.D, nd * 4, hipMemcpyDeviceToHost, s);
    if (ce == hipSuccess) ce = hipMemcpyAsync(h->ghI, rp.I, nd * 8, hipMemcpyDeviceToHost, s);
    if (ce == hipSuccess) ce = hipMemcpyAsync(h->ghnf, n_flag, 4, hipMemcpyDeviceToHost, s);
    g_graph_capture = false;
    hipGraph_t graph = nullptr;
    e = hipStreamEndCapture(s, &graph);  // always end the capture: the stream must leave capture mode
    if (ce != hipSuccess) e = ce;
    if (e == hipSuccess) e = hipGraphInstantiate(&h->gexec, graph, nullptr, nullptr, 0);
    if (graph) (void)hipGraphDestroy(graph);
    if (e != hipSuccess) {
        h->gexec = nullptr;
        (void)hipGetLastError();
        return e;
    }
    h->gkey = graph_key(h, nq, q_dtype, k, scan_dt);
    return hipSuccess;
}

// Small host batches under FX_SEARCH_GRAPH=1: replay the captured search
// (the exact fallback included: it is device-gated); on a shape / buffer
// change run do_search and re-capture.
int graph_search(FxIndex* h, int64_t nq, const void* q, int q_dtype, int k, float* D, int64_t* I) {
    bool split = false;
    HIP_TRY(update_scan_image(h, &split));
    if (h->gexec && graph_key(h, nq, q_dtype, k, split ? (int)F32S : h->dtype) == h->gkey) {
        hipStream_t s = h->stream();
        memcpy(h->ghq, q, (size_t)nq * h->d * dtype_size(q_dtype));
        HIP_TRY(hipGraphLaunch(h->gexec, s));
        HIP_TRY(hipStreamSynchronize(s));
        memcpy(D, h->ghD, (size_t)nq * k * 4);
        memcpy(I, h->ghI, (size_t)nq * k * 8);
        h->last_fallbacks = *h->ghnf;
        h->fb_pending = false;
        return FX_OK;
    }
    const int rc = do_search(h, nq, q, q_dtype, FX_MEM_HOST, k, D, I, FX_MEM_HOST);
    if (rc == FX_OK && !h->gfailed) {
        const hipError_t e = graph_build(h, nq, q_dtype, k, split);
        if (e != hipSuccess) {  // stay on do_search for this index
            h->gfailed = true;
            if (getenv("FX_SEARCH_GRAPH_VERBOSE")) fprintf(stderr, "fx: search graph capture failed: %s\n", hipGetErrorString(e));
        } else if (getenv("FX_SEARCH_GRAPH_VERBOSE")) {
            fprintf(stderr, "fx: search graph captured (nq=%lld k=%d)\n", (long long)nq, k);
        }
    }
    return rc;
}

}  // namespace

extern "C" {

const char* fx_last_error(void) { return g_err.c_str(); }

int fx_device_count(int* out) {
    if (!out) return set_err(FX_E_ARG, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *out = 0;
        return set_err(FX_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *out = n;
    return FX_OK;
}

int fx_index_create(int d, int storage_dtype, int metric, int device, FxIndex** out) {
    if (!out) return set_err(FX_E_ARG, "null out");
    *out = nullptr;
    if (d <= 0) return set_err(FX_E_ARG, "dimension must be positive (got %d)", d);
    if (!check_dtype(storage_dtype)) return set_err(FX_E_ARG, "bad storage dtype %d", storage_dtype);
    if (metric != FX_METRIC_L2 && metric != FX_METRIC_INNER_PRODUCT)
        return set_err(FX_E_ARG, "bad metric %d", metric);
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return set_err(FX_E_HIP, "device %d not available (%d devices)", device, n);
    DeviceGuard g(device);
    if (!g.ok) return set_err(FX_E_HIP, "hipSetDevice(%d) failed", device);
    FxIndex* h = new FxIndex();
    h->d = d;
    h->dtype = storage_dtype;
    h->metric = metric;
    h->device = device;
    h->row_bytes = (int)round_up((int64_t)d * dtype_size(storage_dtype), ROW_ALIGN);
    h->kdim = h->row_bytes / dtype_size(storage_dtype);
    // A BLOCKING stream: work on the legacy null stream (torch's default
    // stream, cuda_stream == 0) is ordered before and after it, so a caller
    // that binds "stream 0" (fx_index_set_stream(h, NULL)) stays ordered.
    hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamDefault);
    if (e == hipSuccess) e = hipMalloc(&h->max_sq_bits, 16);
    if (e == hipSuccess) e = hipMemset(h->max_sq_bits, 0, 16);
    if (e != hipSuccess) {
        fx_index_free(h);
        return set_err(FX_E_HIP, "index init: %s", hipGetErrorString(e));
    }
    *out = h;
    return FX_OK;
}

void fx_index_free(FxIndex* h) {
    if (!h) return;
    {
        DeviceGuard g(h->device);
        if (h->own_stream) (void)hipStreamSynchronize(h->own_stream);
        if (h->user_stream) (void)hipStreamSynchronize(h->user_stream);
        if (h->codes) (void)hipFree(h->codes);
        if (h->norms) (void)hipFree(h->norms);
        if (h->max_sq_bits) (void)hipFree(h->max_sq_bits);
        for (DevBuf* b : {&h->qin, &h->qf32, &h->qop, &h->qeps, &h->cand_d, &h->cand_i, &h->dws, &h->iws, &h->flag,
                          &h->fbc_d, &h->fbc_i, &h->stage, &h->gtau, &h->trace, &h->dbgbuf, &h->split, &h->cnorms,
                          &h->centre, &h->mu_part, &h->qxn2, &h->stamps, &h->pub, &h->cand2_d, &h->cand2_i})
            b->release();
        graph_release(h);
        if (h->ghq) (void)hipHostFree(h->ghq);
        if (h->ghD) (void)hipHostFree(h->ghD);
        if (h->ghI) (void)hipHostFree(h->ghI);
        if (h->ghnf) (void)hipHostFree(h->ghnf);
        if (h->pin_nf) (void)hipHostFree(h->pin_nf);
        for (auto& pr : h->ev_scan) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
        for (auto& pr : h->ev_merge) (void)hipEventDestroy(pr.second);
        if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    }
    delete h;
}

int fx_index_set_normalize(FxIndex* h, int on) {
    if (!h) return set_err(FX_E_ARG, "null index");
    std::lock_guard<std::mutex> lk(h->mu);
    h->normalize = on ? 1 : 0;
    return FX_OK;
}

int fx_index_set_stream(FxIndex* h, void* stream) {
    if (!h) return set_err(FX_E_ARG, "null index");
    std::lock_guard<std::mutex> lk(h->mu);
    h->user_stream = (hipStream_t)stream;
    return FX_OK;
}

int fx_index_set_id_offset(FxIndex* h, int64_t off) {
    if (!h || off < 0) return set_err(FX_E_ARG, "bad index/offset");
    std::lock_guard<std::mutex> lk(h->mu);
    h->id_offset = off;
    return FX_OK;
}

int fx_index_dim(const FxIndex* h, int* out) {
    if (!h || !out) return set_err(FX_E_ARG, "null argument");
    *out = h->d;
    return FX_OK;
}
int fx_index_ntotal(const FxIndex* h, int64_t* out) {
    if (!h || !out) return set_err(FX_E_ARG, "null argument");
    *out = h->ntotal;
    return FX_OK;
}
int fx_index_storage_dtype(const FxIndex* h, int* out) {
    if (!h || !out) return set_err(FX_E_ARG, "null argument");
    *out = h->dtype;
    return FX_OK;
}
int fx_index_metric(const FxIndex* h, int* out) {
    if (!h || !out) return set_err(FX_E_ARG, "null argument");
    *out = h->metric;
    return FX_OK;
}

int fx_index_reserve(FxIndex* h, int64_t n) {
    if (!h || n < 0) return set_err(FX_E_ARG, "bad reserve");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    HIP_TRY(grow(h, n));
    return FX_OK;
}

int fx_index_add(FxIndex* h, int64_t n, const void* x, int x_dtype, int x_mem) {
    if (!h) return set_err(FX_E_ARG, "null index");
    if (n < 0) return set_err(FX_E_ARG, "negative n");
    if (n == 0) return FX_OK;
    if (!x) return set_err(FX_E_ARG, "null x");
    if (!check_dtype(x_dtype)) return set_err(FX_E_ARG, "bad x dtype %d", x_dtype);
    if ((int64_t)h->ntotal + n >= (int64_t)INT32_MAX) return set_err(FX_E_UNSUPPORTED, "more than 2^31-1 rows per shard");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    hipStream_t s = h->stream();
    HIP_TRY(grow(h, h->ntotal + n));
    const size_t xes = dtype_size(x_dtype);
    if (x_mem == FX_MEM_DEVICE) {
        HIP_TRY(launch_convert_rows(x, x_dtype, n, h->d, h->codes + (size_t)h->ntotal * h->row_bytes, h->dtype,
                                    h->kdim, h->norms + h->ntotal, h->max_sq_bits, h->normalize, s));
    } else {
        // stream host rows through a bounded staging buffer (<= 256 MiB)
        const int64_t chunk = std::max<int64_t>(1, (256ll << 20) / ((int64_t)h->d * xes));
        for (int64_t r0 = 0; r0 < n; r0 += chunk) {
            const int64_t nr = std::min(chunk, n - r0);
            HIP_TRY(h->stage.ensure((size_t)nr * h->d * xes));
            HIP_TRY(hipMemcpyAsync(h->stage.p, (const char*)x + (size_t)r0 * h->d * xes, (size_t)nr * h->d * xes,
                                   hipMemcpyHostToDevice, s));
            HIP_TRY(launch_convert_rows(h->stage.p, x_dtype, nr, h->d,
                                        h->codes + (size_t)(h->ntotal + r0) * h->row_bytes, h->dtype, h->kdim,
                                        h->norms + h->ntotal + r0, h->max_sq_bits, h->normalize, s));
            HIP_TRY(hipStreamSynchronize(s));  // staging buffer reuse
        }
    }
    h->ntotal += n;
    return FX_OK;
}

int fx_index_search(FxIndex* h, int64_t nq, const void* q, int q_dtype, int q_mem, int k, float* D, int64_t* I,
                    int out_mem) {
    if (!h) return set_err(FX_E_ARG, "null index");
    if (nq < 0) return set_err(FX_E_ARG, "negative nq");
    if (k <= 0) return set_err(FX_E_ARG, "k must be positive (got %d)", k);
    if (k > FX_MAX_K) return set_err(FX_E_UNSUPPORTED, "k=%d exceeds FX_MAX_K=%d", k, FX_MAX_K);
    static_assert(FX_MAX_K == FX_BIG_K, "ABI k limit = the big-k refine's");
    if (!check_dtype(q_dtype)) return set_err(FX_E_ARG, "bad query dtype %d", q_dtype);
    if (nq == 0) return FX_OK;
    if (!q || !D || !I) return set_err(FX_E_ARG, "null buffer");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    if (h->ntotal == 0) {
        // faiss: empty index -> every slot missing (I = -1, D = FLT_MAX)
        const float dfill = h->metric == L2 ? FLT_MAX : -FLT_MAX;
        if (out_mem == FX_MEM_HOST) {
            std::fill(D, D + (size_t)nq * k, dfill);
            std::fill(I, I + (size_t)nq * k, (int64_t)-1);
        } else {  // stream-ordered fills: -1 is all ones in two's complement
            uint32_t bits;
            memcpy(&bits, &dfill, 4);
            HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)D, bits, (size_t)nq * k, h->stream()));
            HIP_TRY(hipMemsetAsync(I, 0xff, (size_t)nq * k * 8, h->stream()));
        }
        h->last_fallbacks = 0;
        h->fb_pending = false;
        return FX_OK;
    }
    const char* ge = getenv("FX_SEARCH_GRAPH");
    if (ge && atoi(ge) == 1 && q_mem == FX_MEM_HOST && out_mem == FX_MEM_HOST && nq <= 64 && !h->profile &&
        !getenv("FX_SCAN_DBG") && !getenv("FX_SCAN_TRACE") && !getenv("FX_SCAN_CAND") && h->user_stream == nullptr)
        return graph_search(h, nq, q, q_dtype, k, D, I);
    return do_search(h, nq, q, q_dtype, q_mem, k, D, I, out_mem);
}

int fx_index_last_fallbacks(FxIndex* h, int64_t* out) {
    if (!h || !out) return set_err(FX_E_ARG, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->fb_pending) {  // a device-resident search left its count in flight
        DeviceGuard g(h->device);
        HIP_TRY(hipStreamSynchronize(h->stream()));
        h->last_fallbacks = *h->pin_nf;
        h->fb_pending = false;
    }
    *out = h->last_fallbacks;
    return FX_OK;
}

int fx_index_reset(FxIndex* h) {
    if (!h) return set_err(FX_E_ARG, "null index");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    HIP_TRY(hipStreamSynchronize(h->stream()));
    HIP_TRY(hipMemset(h->max_sq_bits, 0, 8));
    if (h->codes && h->cap_rows > 0) {
        HIP_TRY(hipMemset(h->codes, 0, (size_t)h->cap_rows * h->row_bytes));
        HIP_TRY(hipMemsetD32((hipDeviceptr_t)h->norms, 0x7f800000u, (size_t)h->cap_rows));
    }
    h->ntotal = 0;
    h->split_rows = 0;
    h->mu_rows = 0;
    return FX_OK;
}

int fx_index_reconstruct_n(FxIndex* h, int64_t i0, int64_t n, float* out) {
    if (!h || !out || i0 < 0 || n < 0 || i0 + n > h->ntotal) return set_err(FX_E_ARG, "bad reconstruct range");
    if (n == 0) return FX_OK;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    hipStream_t s = h->stream();
    const int64_t chunk = std::max<int64_t>(1, (128ll << 20) / ((int64_t)h->d * 4));
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
        const int64_t nr = std::min(chunk, n - r0);
        HIP_TRY(h->stage.ensure((size_t)nr * h->d * 4));
        HIP_TRY(launch_to_f32(h->codes + (size_t)(i0 + r0) * h->row_bytes, h->dtype, h->row_bytes, nr, h->d,
                              (float*)h->stage.p, s));
        HIP_TRY(hipMemcpyAsync(out + (size_t)r0 * h->d, h->stage.p, (size_t)nr * h->d * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return FX_OK;
}

int fx_index_write(FxIndex* h, const char* path) {
    if (!h || !path) return set_err(FX_E_ARG, "null argument");
    if (h->metric != FX_METRIC_L2) return set_err(FX_E_UNSUPPORTED, "IxF2 writer supports METRIC_L2 only");
    FILE* f = fopen(path, "wb");
    if (!f) return set_err(FX_E_IO, "cannot open %s for writing", path);
    const int32_t d = h->d, metric = FX_METRIC_L2;
    const int64_t nt = h->ntotal, dummy = 1 << 20, count = h->ntotal * (int64_t)h->d;
    const uint8_t trained = 1;
    bool ok = fwrite("IxF2", 1, 4, f) == 4 && fwrite(&d, 4, 1, f) == 1 && fwrite(&nt, 8, 1, f) == 1 &&
              fwrite(&dummy, 8, 1, f) == 1 && fwrite(&dummy, 8, 1, f) == 1 && fwrite(&trained, 1, 1, f) == 1 &&
              fwrite(&metric, 4, 1, f) == 1 && fwrite(&count, 8, 1, f) == 1;
    const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / ((int64_t)h->d * 4));
    std::vector<float> buf;
    for (int64_t r0 = 0; ok && r0 < nt; r0 += chunk) {
        const int64_t nr = std::min(chunk, nt - r0);
        buf.resize((size_t)nr * h->d);
        int rc = fx_index_reconstruct_n(h, r0, nr, buf.data());
        if (rc != FX_OK) {
            fclose(f);
            return rc;
        }
        ok = fwrite(buf.data(), 4, buf.size(), f) == buf.size();
    }
    if (fclose(f) != 0) ok = false;
    if (!ok) return set_err(FX_E_IO, "short write to %s", path);
    return FX_OK;
}

int fx_index_read(const char* path, int storage_dtype, int device, FxIndex** out) {
    if (!path || !out) return set_err(FX_E_ARG, "null argument");
    *out = nullptr;
    FILE* f = fopen(path, "rb");
    if (!f) return set_err(FX_E_IO, "could not open %s for reading", path);
    char fourcc[4];
    int32_t d = 0, metric = 0;
    int64_t nt = 0, d1 = 0, d2 = 0, count = 0;
    uint8_t trained = 0;
    bool ok = fread(fourcc, 1, 4, f) == 4 && fread(&d, 4, 1, f) == 1 && fread(&nt, 8, 1, f) == 1 &&
              fread(&d1, 8, 1, f) == 1 && fread(&d2, 8, 1, f) == 1 && fread(&trained, 1, 1, f) == 1 &&
              fread(&metric, 4, 1, f) == 1 && fread(&count, 8, 1, f) == 1;
    if (!ok) {
        fclose(f);
        return set_err(FX_E_IO, "%s: truncated IxF2 header", path);
    }
    if (memcmp(fourcc, "IxF2", 4) != 0) {
        fclose(f);
        return set_err(FX_E_IO, "%s: unsupported index fourcc (only IxF2 / IndexFlatL2)", path);
    }
    if (d <= 0 || nt < 0 || metric != FX_METRIC_L2 || count != nt * (int64_t)d) {
        fclose(f);
        return set_err(FX_E_IO, "%s: inconsistent IxF2 header", path);
    }
    FxIndex* h = nullptr;
    int rc = fx_index_create(d, storage_dtype, FX_METRIC_L2, device, &h);
    if (rc != FX_OK) {
        fclose(f);
        return rc;
    }
    rc = fx_index_reserve(h, nt);
    const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / ((int64_t)d * 4));
    std::vector<float> buf;
    for (int64_t r0 = 0; rc == FX_OK && r0 < nt; r0 += chunk) {
        const int64_t nr = std::min(chunk, nt - r0);
        buf.resize((size_t)nr * d);
        if (fread(buf.data(), 4, buf.size(), f) != buf.size()) {
            rc = set_err(FX_E_IO, "%s: truncated IxF2 codes", path);
            break;
        }
        rc = fx_index_add(h, nr, buf.data(), FX_F32, FX_MEM_HOST);
    }
    fclose(f);
    if (rc != FX_OK) {
        fx_index_free(h);
        return rc;
    }
    *out = h;
    return FX_OK;
}

int fx_merge_shards(int metric, int nshards, int64_t nq, int k, const float* D_in, const int64_t* I_in, float* D_out,
                    int64_t* I_out, int device, void* stream) {
    if (nshards <= 0 || nq < 0 || k <= 0 || k > FX_MAX_K) return set_err(FX_E_ARG, "bad merge shape");
    if (!D_in || !I_in || !D_out || !I_out) return set_err(FX_E_ARG, "null buffer");
    if (metric != FX_METRIC_L2 && metric != FX_METRIC_INNER_PRODUCT) return set_err(FX_E_ARG, "bad metric");
    DeviceGuard g(device);
    if (!g.ok) return set_err(FX_E_HIP, "hipSetDevice(%d) failed", device);
    HIP_TRY(launch_merge_shards(metric, nshards, nq, k, D_in, I_in, D_out, I_out, (hipStream_t)stream));
    return FX_OK;
}

int fx_synth_fill(void* out, int64_t row0, int64_t n, int d, int dtype, uint64_t seed, int device, void* stream) {
    if (!out || n < 0 || d <= 0 || row0 < 0 || !check_dtype(dtype)) return set_err(FX_E_ARG, "bad synth args");
    DeviceGuard g(device);
    if (!g.ok) return set_err(FX_E_HIP, "hipSetDevice(%d) failed", device);
    HIP_TRY(launch_synth(out, row0, n, d, dtype, seed, (hipStream_t)stream));
    return FX_OK;
}

int fx_index_profile(FxIndex* h, int enable) {
    if (!h) return set_err(FX_E_ARG, "null index");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    HIP_TRY(hipStreamSynchronize(h->stream()));
    for (auto& pr : h->ev_scan) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (auto& pr : h->ev_merge) (void)hipEventDestroy(pr.second);
    h->ev_scan.clear();
    h->ev_merge.clear();
    h->profile = enable != 0;
    return FX_OK;
}

int fx_index_profile_read(FxIndex* h, double* scan_ms, double* merge_ms, int64_t* launches) {
    if (!h || !scan_ms || !merge_ms || !launches) return set_err(FX_E_ARG, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    HIP_TRY(hipStreamSynchronize(h->stream()));
    double a = 0, b = 0;
    for (size_t i = 0; i < h->ev_scan.size(); ++i) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, h->ev_scan[i].first, h->ev_scan[i].second));
        a += ms;
        HIP_TRY(hipEventElapsedTime(&ms, h->ev_merge[i].first, h->ev_merge[i].second));
        b += ms;
    }
    *scan_ms = a;
    *merge_ms = b;
    *launches = (int64_t)h->ev_scan.size();
    return FX_OK;
}

}  // extern "C"
