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

// Per-index tuning options.  Initial values come from the FX_* environment
// variables, read ONCE when the index is created (never on the search path);
// fx_index_set_option changes them afterwards (range-checked: opt_range).
// Test hooks and diagnostic dumps exist only in the diagnostic build
// (-DFX_DIAG: libfx_index_diag.so, make diag / abl), never in libfx_index.so.
struct Options {
    int search_graph = 0;    // FX_SEARCH_GRAPH: replay small host searches as one hipGraph (round 5: -7 %
                             // per one-query call, r5r; off since round 6: with the call down to three
                             // kernels and one packed copy, the eager enqueue is 3-7 % faster: 97-101 vs
                             // 104 us on a 100k x 384 fp32 index, profiles/r6/latency_graph_r6f.jsonl)
    int place = -1;          // FX_SCAN_PLACE: scan block placement (-1 automatic, 0, 1)
    int sx = 0;              // FX_SCAN_SX: corpus splits per XCD under placement 1 (0 automatic)
    int reduce_cand = 1;     // FX_REDUCE_CAND: small nq over many splits: 1 one 16-wave workgroup refine per
                             // query (k_refine_wg), 2 merge 16 splits' lists first (k_reduce_cand, round 3),
                             // 0 the one-wave-per-query refine
    int f32_split = 1;       // FX_F32_SPLIT: fp32 indexes scan their split-bf16 image
    int centre = 1;          // FX_CENTER: L2 scan images are centred on a row sample's mean
    int pub = 1;             // FX_SCAN_PUB: union threshold over published per-split lists
    int prune_rank = 0;      // FX_PRUNE_RANK: rank of the shared threshold (0: max(6k/5, 12))
    int compact_at = 0;      // FX_COMPACT_AT: list fill that triggers a compaction (0: default 48, KP < v <= CAP)
    int union_w = 0;         // FX_UNION_W: splits per union-bound window (16, 32, 64; 0: by split count)
    int union_defer = 1;     // FX_UNION_DEFER: union bounds fetched by LDS-DMA, bounded a tile later (0: in place)
    int union_inplace = -1;  // FX_UNION_INPLACE: most lists per compaction call bounded in place beyond the
                             // deferred ones (-1: 0 with union_defer, all without; r5v: 0 is -1.4 % on the
                             // N = 8 shard and (b), (d) unchanged)
    int tight_at = -1;       // FX_TIGHT_AT: a list that took entries and holds >= this many gets its threshold
                             // re-bounded without a compaction (-1 default, 0 off, KP < v <= CAP)
    int cold_bound = -1;     // FX_COLD_BOUND: an empty list's first record tile bounds its threshold by the
                             // rank-th of the tile's group minima before pushing (0 off, 1 on, -1: on for
                             // splits of <= 256 tiles).  tight_at measured slower and off
                             // (profiles/r5/ab/r5h_tight_cold.txt); cold_bound -1.8 % on (b), -1 % on (d)
                             // at nq = 256 (short splits), +0.5-0.9 % on the long splits of (d) and the
                             // N = 8 shard (r5h, r5i, r5k)
    int graph_verbose = 0;   // FX_SEARCH_GRAPH_VERBOSE
    int refine_waves = REFINE_WG_WAVES;  // FX_REFINE_WAVES: waves of k_refine_wg's workgroup (4, 8, 16)
    int scan_v5 = 1;         // FX_SCAN_V5: 16-bit rows of 512 / 768 / 1,536 B scan with k_scan_v5 (64-row
                             // tiles, 256 / 192 queries per workgroup; fx_scan5.hip) where it adds no
                             // padding work; 2: wherever it has the shape (tests); 0: k_scan_v4
    int convoy = 1;          // FX_CONVOY: k_scan_v5 blocks start where the other blocks of their split
                             // are (ScanParams.conv); 0: at the split's first tile
    int convoy_every = 4;    // FX_CONVOY_EVERY: a block publishes its tile every this many tiles (1/2/4/8;
                             // 1: (d) 1.8x slower -- every block of a split writing one line each tile)
    int host_spin = 1;       // FX_HOST_SPIN: a host-output search waits for its results by polling the
                             // stream (1) instead of a blocking hipStreamSynchronize (0)
#ifdef FX_DIAG
    int force_fallback = 0;  // FX_FORCE_FALLBACK: flag every query (1: -> re-scan, 2: -> exact scan)
    int scan_dbg = 0;        // FX_SCAN_DBG: ablation switches of -DFX_ABLATION builds / key dump (32)
    std::string trace, stamps, cand, keys;  // FX_SCAN_TRACE / _STAMPS / _CAND / _KEYS dump paths
#else
    static constexpr int force_fallback = 0, scan_dbg = 0;
#endif

    void from_env() {
        auto num = [](const char* name, int& v) {
            if (const char* e = getenv(name); e && *e) v = atoi(e);
        };
        auto str = [](const char* name, std::string& v) {
            if (const char* e = getenv(name); e && *e) v = e;
        };
        num("FX_SEARCH_GRAPH", search_graph);
        num("FX_SCAN_PLACE", place);
        num("FX_SCAN_SX", sx);
        num("FX_REDUCE_CAND", reduce_cand);
        num("FX_F32_SPLIT", f32_split);
        num("FX_CENTER", centre);
        num("FX_SCAN_PUB", pub);
        num("FX_PRUNE_RANK", prune_rank);
        num("FX_COMPACT_AT", compact_at);
        num("FX_UNION_W", union_w);
        num("FX_UNION_DEFER", union_defer);
        num("FX_UNION_INPLACE", union_inplace);
        num("FX_TIGHT_AT", tight_at);
        num("FX_COLD_BOUND", cold_bound);
        num("FX_SEARCH_GRAPH_VERBOSE", graph_verbose);
        num("FX_HOST_SPIN", host_spin);
        num("FX_SCAN_V5", scan_v5);
        num("FX_CONVOY", convoy);
        num("FX_CONVOY_EVERY", convoy_every);
        num("FX_REFINE_WAVES", refine_waves);
        if (refine_waves != 4 && refine_waves != 8 && refine_waves != 16) refine_waves = REFINE_WG_WAVES;
        (void)str;
#ifdef FX_DIAG
        num("FX_FORCE_FALLBACK", force_fallback);
        num("FX_SCAN_DBG", scan_dbg);
        str("FX_SCAN_TRACE", trace);
        str("FX_SCAN_STAMPS", stamps);
        str("FX_SCAN_CAND", cand);
        str("FX_SCAN_KEYS", keys);
#endif
    }
    // option name -> its slot and accepted range [lo, hi] (allowed: a value
    // list when `set` is non-null)
    struct Slot {
        const char* name;
        int* v;
        int lo, hi;
        const int* set;
        int nset;
    };
    int* find(const char* name, int64_t value, const char** why) {
        static const int kWindows[] = {0, 16, 32, 64};
        static const int kWaves[] = {4, 8, 16};
        const Slot slots[] = {
            {"search_graph", &search_graph, 0, 1, nullptr, 0},
            {"scan_place", &place, -1, 1, nullptr, 0},
            {"scan_sx", &sx, 0, 1 << 16, nullptr, 0},
            {"reduce_cand", &reduce_cand, 0, 2, nullptr, 0},
            {"f32_split", &f32_split, 0, 1, nullptr, 0},
            {"centre", &centre, 0, 1, nullptr, 0},
            {"scan_pub", &pub, 0, 1, nullptr, 0},
            {"prune_rank", &prune_rank, 0, KP, nullptr, 0},
            {"compact_at", &compact_at, 0, CAP, nullptr, 0},
            {"union_w", &union_w, 0, 64, kWindows, 4},
            {"union_defer", &union_defer, 0, 1, nullptr, 0},
            {"union_inplace", &union_inplace, -1, 64, nullptr, 0},
            {"tight_at", &tight_at, -1, CAP, nullptr, 0},
            {"cold_bound", &cold_bound, -1, 1, nullptr, 0},
            {"host_spin", &host_spin, 0, 1, nullptr, 0},
            {"scan_v5", &scan_v5, 0, 2, nullptr, 0},
            {"convoy", &convoy, 0, 1, nullptr, 0},
            {"convoy_every", &convoy_every, 1, 8, nullptr, 0},
            {"refine_waves", &refine_waves, 4, 16, kWaves, 3},
#ifdef FX_DIAG
            {"force_fallback", &force_fallback, 0, 2, nullptr, 0},
            {"scan_dbg", &scan_dbg, 0, 1 << 20, nullptr, 0},
#endif
        };
        for (const Slot& sl : slots) {
            if (strcmp(name, sl.name) != 0) continue;
            bool ok = value >= sl.lo && value <= sl.hi;
            if (ok && sl.set) {
                ok = false;
                for (int i = 0; i < sl.nset; ++i) ok |= value == sl.set[i];
            }
            // compact_at: 0 (default) or a fill in (KP, CAP]
            if (ok && sl.v == &compact_at) ok = value == 0 || value > KP;
            // tight_at: -1 (default), 0 (off) or a fill in (KP, CAP]
            if (ok && sl.v == &tight_at) ok = value <= 0 || value > KP;
            *why = ok ? nullptr : "value out of range";
            return sl.v;
        }
        *why = "unknown option";
        return nullptr;
    }
};

// scan image of the index (what the MFMA scan streams, and its row constants)
enum ImageKind {
    IMG_NONE = 0,  // the stored rows with srcC = |y|^2 (IP: no row constant)
    IMG_F32S = 1,  // fp32 index: [hi | lo] bf16 planes of fl(y - mu), srcC = |y - mu|^2
    IMG_C16 = 2,   // bf16 / fp16 L2 index: the stored rows, srcC = |y - mu|^2 (the query operand is x - mu)
};

}  // namespace

namespace {

// The device-side plan of one search: scan, refine and fallback parameters
// over the index's workspace.  Sizes the workspace (a no-op when it is large
// enough already, as it is for a graph capture right after do_search).
struct SearchPlan {
    int64_t nq = 0, nq_pad = 0;
    int k = 0, q_dtype = F32, scan_dt = F32;
    ScanParams sp{};
    RefineParams rp{};
    PrepParams pp{};
    bool reduce = false;
    size_t ncand = 0;
    // the re-scan of the queries pass 1 left uncertified (plan_rescan)
    ScanParams sp2{};
    RefineParams rp2{};
    PrepParams pp2{};
    int* n_exact = nullptr;  // queries the re-scan left uncertified too (-> exact scan)
    int nchunks = 0;         // re-scan chunks of <= RESCAN_MAX flagged queries each
    int* chunk_cnt = nullptr;  // [nchunks] live queries of each chunk (k_rescan_chunks, on the device)
};

}  // namespace

struct FxIndex {
    int d = 0, dtype = F32, metric = L2, device = 0, normalize = 0;
    int row_bytes = 0, kdim = 0;
    int64_t ntotal = 0, cap_rows = 0, id_offset = 0;
    char* codes = nullptr;
    float* norms = nullptr;
    // device words: [0] max |y|^2 of the stored rows, [1] max srcC of the scan
    // image (F32S / C16), as float bits (non-negative floats order as uints)
    unsigned* max_sq_bits = nullptr;
    hipStream_t own_stream = nullptr;
    hipStream_t user_stream = nullptr;
    hipEvent_t switch_ev = nullptr;  // orders the work of a stream the index leaves before the next one's
    Options opt;
    // search workspace
    DevBuf qin, qf32, qop, qeps, qrho, cand_d, cand_i, cand2_d, cand2_i, dws, iws, flag, fbc_d, fbc_i, stage, gtau,
        trace, dbgbuf, stamps, pub;
    // the re-scan of uncertified queries (plan_rescan): its own query
    // operands, thresholds, candidate lists and flagged list
    DevBuf rq_f32, rq_op, rq_eps, rq_rho, rq_shift, rq_gtau, rq_cand_d, rq_cand_i, rq_flag;
    // k > FX_BIG_K (fx_hugek.hip): query batch, sort keys, rocPRIM temporaries
    DevBuf hk_ws;
    // scan image (ImageKind; rows [0, img_rows) current).  L2 images are
    // centred (Options.centre): mu = mean of a row sample, recomputed (and the
    // image rebuilt) whenever ntotal has doubled since (mu_rows), so the
    // centre follows the data at O(1) amortised cost per added row.
    //   F32S: split = [hi | lo] bf16 planes of fl(y - mu), cnorms = |y - mu|^2
    //   C16:  cnorms = |y - mu|^2 of the stored bf16 / fp16 rows (no copy of
    //         the codes; a 16-bit centre whose norm is small next to the rows'
    //         is set to 0 on the device: k_mu_finish)
    DevBuf split, cnorms, centre, mu_part, qshift;
    int64_t img_rows = 0, mu_rows = 0;
    int img_kind = IMG_NONE;
    bool centred = false;
    // search_graph: the search of a small host batch (the reference's one-query
    // call form) replayed as one hipGraph per shape, over pinned host staging;
    // `gkey` = the shape and every buffer the graph captured
    hipGraphExec_t gexec = nullptr;
    std::vector<uint64_t> gkey;
    bool gfailed = false;
    void* ghq = nullptr;
    char* ghout = nullptr;  // pinned mirror of hout for the graph's one D2H copy
    size_t ghq_bytes = 0, ghout_bytes = 0;
    SearchPlan gplan;       // the captured search's plan (its fallback chain runs eagerly when needed)
    // host-output searches: ONE packed device buffer [D | I | n_drop | n_flag |
    // flag list] (host_out_layout) and its pinned mirror, so the common case
    // returns through one D2H copy
    DevBuf hout;
    char* hpin = nullptr;
    size_t hpin_bytes = 0;
    char* qpin = nullptr;   // pinned staging of a host-output search's host queries (<= QPIN_MAX)
    size_t qpin_bytes = 0;
    int64_t last_fallbacks = 0;
    // uncertified count of the last search, copied stream-ordered into pinned
    // memory; read (after a stream sync) only when asked for (fb_pending)
    int* pin_nf = nullptr;  // [0] queries re-scanned, [1] queries sent to the exact scan, [2] dropped ids
    bool fb_pending = false;
    int64_t last_exact = 0;
    // candidate entries the refine dropped for a row id outside [0, ntotal)
    // (a corrupted candidate list; 0 unless something is broken)
    int64_t last_dropped = 0;
    int* dev_drop = nullptr;  // its device word, zeroed at the start of every search
    DevBuf conv;  // k_scan_v5 convoy words (CONV_WORDS; zeroed once, then only hints)
    int last_plan[3] = {0, 0, 0};  // the last search's scan plan: tile rows (128 k_scan_v4, 64 k_scan_v5), qt, splits
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

// split count whose live workgroups (one per CU: the scan's LDS) fill whole
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

// the scan's grid: corpus splits per query tile and block placement.
// k > KP: no cross-split pruning (ScanParams.share = 0) and at least k/4
// splits, so that a split's KP-list rarely holds fewer than all of its top-k
// rows and the certification bound (the smallest full split's KP-th key)
// lies far beyond the k-th distance
void plan_scan(const FxIndex* h, int64_t nq, int k, ScanParams& p) {
    // the scan's shape: k_scan_v5 (64-row tiles x 256 queries) for the 16-bit
    // rows it has (not with the key-matrix dump, whose layout is k_scan_v4's)
    const int sdt = h->img_kind == IMG_F32S ? (int)F32S : h->dtype;
    // ... when its wider query tiles add no padding work: v5 query slots within
    // 5 % of k_scan_v4's (nq = 256 on 1,536-B rows would scan 384 slots for
    // 256 queries: 5.59 against 3.61 ms, profiles/r6/ab_v5_d_r6e.txt; one-query
    // calls keep k_scan_v4's 128-query tile)
    const int v5qt = h->opt.scan_v5 != 0 && !(h->opt.scan_dbg & 32) ? scan_v5_qt(sdt, h->row_bytes) : 0;
    const int64_t slots4 = (nq + TILE_Q - 1) / TILE_Q * TILE_Q;
    const bool v5 = v5qt > 0 && (h->opt.scan_v5 == 2 || (nq + v5qt - 1) / v5qt * v5qt * 20 <= slots4 * 21);
    p.qt = v5 ? v5qt : TILE_Q;
    p.tr = v5 ? V5_TR : TILE_R;
    p.n_qtiles = (int)((nq + p.qt - 1) / p.qt);
    p.n_ctiles = (int)((h->ntotal + p.tr - 1) / p.tr);
    p.place = 0;
    p.sx = 0;
    p.pub = nullptr;
    p.prune_rank = KP;
    // default 48: with the union bound deferred a compaction is cheap enough
    // that tightening the threshold 16 entries earlier pays (same-box sweep,
    // profiles/r4/ab/compact_r4c.txt: (d) -1.1 %, (b) and the N = 8 shard -0.2 %)
    p.compact_at = h->opt.compact_at > KP && h->opt.compact_at <= CAP ? h->opt.compact_at : 48;
    p.share = k <= KP ? 1 : 0;
    p.union_w = 16;
    p.union_defer = h->opt.union_defer;
    p.union_inplace = h->opt.union_inplace >= 0 ? h->opt.union_inplace : p.union_defer ? 0 : (1 << 30);
    // list re-bounding between compactions (k <= KP only; -1: the default)
    p.tight_at = p.share && h->opt.tight_at > KP ? h->opt.tight_at : 0;
    p.cold_bound = 0;  // below, once the split count is known
    const int ntl = p.n_qtiles, nct = p.n_ctiles;
    // >= 3 tiles per split: a 100k-row index (782 tiles) then fills all 256
    // CUs with one query tile (256 splits; 192 at 4 tiles)
    constexpr int min_tiles = 3;
    // placement (map_tile): corpus-partitioned by default (config (d): 257 vs
    // 742 GB fetched past L2 per launch, ~2 % faster); scan_place = 0 forces
    // the query-tile groups of round 1.  Also for fewer than 8 query tiles:
    // the ntl blocks of one split then run side by side on one XCD, so the
    // split is fetched past L2 once for all of them (nq = 256: once instead
    // of twice)
    const int place = h->opt.place >= 0 ? h->opt.place : 1;
    if (place == 1 && nct >= 8 * min_tiles) {
        // XCD x owns 1/8 of the corpus for every query tile; sx splits per
        // XCD so that its ntl * sx blocks fill whole rounds of its 32 CUs
        p.place = 1;
        p.qt_per_xcd = 0;
        const int max_sx = std::max(1, nct / (8 * min_tiles));
        int best = 1;
        double best_eff = 0.0;
        for (int sx = 1; sx <= std::min(max_sx, std::max(16, 128 / ntl)); ++sx) {
            const double live = (double)ntl * sx;
            const double eff = live / (std::ceil(live / 32.0) * 32.0);
            if (eff > best_eff + 1e-9) { best_eff = eff; best = sx; }
            if (eff > 0.985 && live >= 128) break;
        }
        if (h->opt.sx > 0) best = std::max(1, std::min(max_sx, h->opt.sx));  // placement A/B runs only
        if (k > KP) best = std::max(best, std::min(max_sx, ((k + 3) / 4 + 7) / 8));
        p.sx = best;
        p.splits = 8 * best;
        p.grid = 8 * ntl * best;
    } else {
        p.qt_per_xcd = ntl >= 8 ? (ntl + 7) / 8 : 0;
        const int eff_q = p.qt_per_xcd > 0 ? 8 * p.qt_per_xcd : ntl;
        p.splits = fill_splits(ntl, eff_q, nct, min_tiles);
        if (k > KP) p.splits = std::max(p.splits, std::min(std::max(1, nct / min_tiles), (k + 3) / 4));
        p.grid = eff_q * p.splits;
    }
    // union-bound window (compact_regs): as many splits as there are, up to
    // 64, each contributing its first 256 / window published keys
    const int uw = h->opt.union_w;
    p.union_w = uw == 16 || uw == 32 || uw == 64 ? uw : p.splits <= 16 ? 16 : p.splits <= 32 ? 32 : 64;
    // cold-start bound: pays on short splits, where a block's first record
    // tiles are a large share of its work
    const int cb = h->opt.cold_bound;
    p.cold_bound = !p.share ? 0 : cb >= 0 ? cb : ((int64_t)(nct + p.splits - 1) / p.splits) * p.tr <= 256 * TILE_R ? 1 : 0;
    if (v5) p.tight_at = 0;  // (k_scan_v5 has no between-compaction re-bound)
}

// k > KP: approx candidates the refine re-ranks exactly (k_refine_big)
int big_k1(int k) { return k > KP ? std::max(2 * k, 64) : 0; }

// small batches over many splits (k <= KP, nq <= 256, >= 64 splits): the
// candidate walk is shared by the waves of one workgroup per query
// (reduce_cand 1, k_refine_wg) or by a separate merge of 16 splits' lists at a
// time before the refine (reduce_cand 2, k_reduce_cand)
bool small_many(int k, int64_t nq, int splits) { return k <= KP && nq <= 256 && splits >= 64; }

hipError_t ensure_pinned_count(FxIndex* h) {
    if (h->pin_nf) return hipSuccess;
    hipError_t e = hipHostMalloc((void**)&h->pin_nf, 3 * sizeof(int), hipHostMallocDefault);
    if (e == hipSuccess) h->pin_nf[0] = h->pin_nf[1] = h->pin_nf[2] = 0;
    return e;
}

// which scan image the index's current options call for
int image_kind(const FxIndex* h) {
    const int rb64 = h->row_bytes / 64;
    if (h->dtype == F32)
        return h->opt.f32_split != 0 && h->row_bytes % 64 == 0 && (rb64 == 8 || rb64 == 12 || rb64 == 16 || rb64 == 24)
                   ? IMG_F32S
                   : IMG_NONE;
    return h->metric == L2 && h->opt.centre != 0 ? IMG_C16 : IMG_NONE;
}

// bring the scan image up to date (rows appended since the last search)
hipError_t update_scan_image(FxIndex* h) {
    const int kind = image_kind(h);
    hipStream_t s = h->stream();
    hipError_t e = hipSuccess;
    if (kind == IMG_NONE) {
        h->img_kind = IMG_NONE;
        return hipSuccess;
    }
    const void* old = h->split.p;
    const void* old_n = h->cnorms.p;
    if (kind == IMG_F32S && (e = h->split.ensure((size_t)h->cap_rows * h->row_bytes)) != hipSuccess) return e;
    if ((e = h->cnorms.ensure((size_t)h->cap_rows * 4)) != hipSuccess) return e;
    bool rebuild = h->split.p != old || h->cnorms.p != old_n || h->img_rows > h->ntotal || kind != h->img_kind;
    const bool centre = h->metric == L2 && h->opt.centre != 0;
    if (centre != h->centred) rebuild = true;
    if (centre && (h->mu_rows == 0 || h->ntotal >= 2 * h->mu_rows || kind != h->img_kind)) {
        // (re)centre on the current rows
        if ((e = h->centre.ensure((size_t)h->kdim * 4)) != hipSuccess) return e;
        if ((e = h->mu_part.ensure((size_t)2 * MU_GROUPS * h->kdim * 8)) != hipSuccess) return e;
        // 16-bit rows: a centre whose norm is below 0.1 of the rows' mean
        // square norm (no common direction) is dropped (mu = 0), which keeps
        // 16-bit-exact queries exact in the scan operand
        if ((e = launch_mu(h->codes, h->dtype, h->row_bytes, h->d, h->ntotal, (double*)h->mu_part.p,
                           (float*)h->centre.p, kind == IMG_C16 ? 0.1f : 0.0f, s)) != hipSuccess)
            return e;
        h->mu_rows = h->ntotal;
        rebuild = true;
    }
    h->centred = centre;
    h->img_kind = kind;
    if (rebuild) {  // zero image (finite padding rows), +inf padding norms
        if (kind == IMG_F32S && (e = hipMemsetAsync(h->split.p, 0, h->split.bytes, s)) != hipSuccess) return e;
        if ((e = hipMemsetD32Async((hipDeviceptr_t)h->cnorms.p, 0x7f800000u, h->cnorms.bytes / 4, s)) != hipSuccess)
            return e;
        if ((e = hipMemsetAsync(h->max_sq_bits + 1, 0, 4, s)) != hipSuccess) return e;
        h->img_rows = 0;
    }
    const float* mu = centre ? (const float*)h->centre.p : nullptr;
    if (kind == IMG_F32S)
        e = launch_split_rows((const float*)h->codes, h->kdim, h->img_rows, h->ntotal, mu, h->split.p,
                              (float*)h->cnorms.p, h->max_sq_bits + 1, s);
    else
        e = launch_centre_norms(h->codes, h->dtype, h->row_bytes, h->img_rows, h->ntotal, mu, (float*)h->cnorms.p,
                                h->max_sq_bits + 1, s);
    if (e == hipSuccess) h->img_rows = h->ntotal;
    return e;
}


// The re-scan of the queries pass 1 could not certify (rows flag_list[0 ..
// n_flag) of the batch, gathered on the device): the same MFMA scan over
// them without cross-split pruning and with ~k1/4 corpus splits, then
// k_refine_big re-ranking k1 = max(512, 4k) approx candidates exactly, so the
// certification bound sits near the k1-th key instead of the ~2k-th.  Its
// uncertified queries go to the exact scan.  Launched always; every kernel
// reads the flagged count and exits at once when it is 0.
// The re-scan's workspace is sized for RESCAN_MAX flagged queries whatever
// the batch (its lists are k1/4 splits wide); a batch that could flag more
// runs it in ceil(nq / RESCAN_MAX) chunks over the flagged list, each chunk's
// live count decided on the device (k_rescan_chunks: empty chunks exit at
// once), so a large batch never pays for a workspace it almost never uses
// and never sends re-scannable queries to the exact scan.
hipError_t plan_rescan(FxIndex* h, SearchPlan& P) {
    hipError_t e;
    const int64_t nq = std::min<int64_t>(P.nq, RESCAN_MAX);
    const int k1 = std::min(2 * FX_BIG_K, std::max(512, 4 * P.k));
    int* n_flag = P.rp.n_flag;
    ScanParams& sp = P.sp2;
    sp = P.sp;
    sp.nq = nq;
    plan_scan(h, nq, k1, sp);  // k1 > KP: share = 0, >= k1/4 splits
    const int64_t nq_pad = round_up(nq, std::max<int64_t>(QPAD, sp.qt));
    if ((e = h->rq_f32.ensure((size_t)nq_pad * h->kdim * 4)) != hipSuccess) return e;
    if ((e = h->rq_op.ensure((size_t)nq_pad * h->row_bytes)) != hipSuccess) return e;
    if ((e = h->rq_eps.ensure((size_t)nq * 4)) != hipSuccess) return e;
    if ((e = h->rq_rho.ensure((size_t)nq * 4)) != hipSuccess) return e;
    if ((e = h->rq_shift.ensure((size_t)nq * 8)) != hipSuccess) return e;
    if ((e = h->rq_gtau.ensure((size_t)nq_pad * 4)) != hipSuccess) return e;
    P.nchunks = (int)((P.nq + RESCAN_MAX - 1) / RESCAN_MAX);
    // [count | every query may go exact | the chunks' live counts]
    if ((e = h->rq_flag.ensure((size_t)(P.nq + 1 + P.nchunks) * 4)) != hipSuccess) return e;
    PrepParams& pp = P.pp2;
    pp = P.pp;
    pp.nq = nq;
    pp.nq_pad = nq_pad;
    pp.q = h->qf32.p;  // pass 1's fp32 copy of the batch, rows padded to kdim
    pp.q_dt = F32;
    pp.d = h->kdim;
    pp.qidx = P.rp.flag_list;
    pp.nq_dev = n_flag;
    pp.qf32 = (float*)h->rq_f32.p;
    pp.qop = h->rq_op.p;
    pp.qeps = (float*)h->rq_eps.p;
    pp.qrho = (float*)h->rq_rho.p;
    pp.qshift = (double*)h->rq_shift.p;
    sp.qop = (const char*)h->rq_op.p;
    sp.gtau = (unsigned*)h->rq_gtau.p;
    sp.pub = nullptr;
    sp.prune_rank = KP;
    sp.dbg = 0;
    sp.trace = nullptr;
    sp.dbgbuf = nullptr;
    sp.stamps = nullptr;
    sp.nq_dev = n_flag;
    const size_t ncand = (size_t)sp.n_qtiles * sp.splits * sp.qt * KP;
    if ((e = h->rq_cand_d.ensure(ncand * 4)) != hipSuccess) return e;
    if ((e = h->rq_cand_i.ensure(ncand * 4)) != hipSuccess) return e;
    sp.cand_d = (float*)h->rq_cand_d.p;
    sp.cand_i = (int*)h->rq_cand_i.p;
    RefineParams& rp = P.rp2;
    rp = P.rp;
    rp.nq = nq;
    rp.cand_d = sp.cand_d;
    rp.cand_i = sp.cand_i;
    rp.splits = sp.splits;
    rp.qt = sp.qt;
    rp.qf32 = pp.qf32;
    rp.qeps = pp.qeps;
    rp.qrho = pp.qrho;
    rp.qshift = pp.qshift;
    rp.k1 = k1;
    rp.gtau = nullptr;
    rp.nq_dev = n_flag;
    rp.out_idx = P.rp.flag_list;
    P.n_exact = (int*)h->rq_flag.p;
    P.chunk_cnt = P.n_exact + 1 + P.nq;
    rp.n_flag = P.n_exact;
    rp.flag_list = P.n_exact + 1;
    rp.force_fb = h->opt.force_fallback == 2;
    rp.wg = 0;
    return hipSuccess;
}

// words (non-null: a host-output search): [n_drop | n_flag | flag list[nq]]
// inside the packed output buffer; otherwise the index's own counter words
hipError_t plan_search(FxIndex* h, int64_t nq, const void* qdev, int q_dtype, int k, float* Dd, int64_t* Id,
                       int* words, SearchPlan& P) {
    hipError_t e;
    P.nq = nq;
    P.k = k;
    P.q_dtype = q_dtype;
    P.scan_dt = h->img_kind == IMG_F32S ? (int)F32S : h->dtype;
    ScanParams& sp = P.sp;
    plan_scan(h, nq, k, sp);
    h->last_plan[0] = sp.tr;
    h->last_plan[1] = sp.qt;
    h->last_plan[2] = sp.splits;
    P.nq_pad = round_up(nq, std::max<int64_t>(QPAD, sp.qt));  // whole scan tiles of (zero) queries
    const bool img = h->img_kind != IMG_NONE;
    if ((e = h->qf32.ensure((size_t)P.nq_pad * h->kdim * 4)) != hipSuccess) return e;
    if ((e = h->qop.ensure((size_t)P.nq_pad * h->row_bytes)) != hipSuccess) return e;
    if ((e = h->qeps.ensure((size_t)nq * 4)) != hipSuccess) return e;
    if ((e = h->qrho.ensure((size_t)nq * 4)) != hipSuccess) return e;
    if ((e = h->qshift.ensure((size_t)nq * 8)) != hipSuccess) return e;

    PrepParams& pp = P.pp;
    pp.q = qdev;
    pp.q_dt = q_dtype;
    pp.nq = nq;
    pp.nq_pad = P.nq_pad;
    pp.d = h->d;
    pp.kdim = h->kdim;
    pp.st_dt = P.scan_dt;
    pp.metric = h->metric;
    pp.qf32 = (float*)h->qf32.p;
    pp.qop = h->qop.p;
    pp.qeps = (float*)h->qeps.p;
    pp.qrho = (float*)h->qrho.p;
    pp.qshift = (double*)h->qshift.p;
    pp.mbits = h->max_sq_bits;
    pp.img_bits = img ? h->max_sq_bits + 1 : h->max_sq_bits;
    pp.mu = img && h->centred ? (const float*)h->centre.p : nullptr;
    pp.qidx = nullptr;
    pp.nq_dev = nullptr;

    sp.codes = h->img_kind == IMG_F32S ? (const char*)h->split.p : h->codes;
    sp.norms = img ? (const float*)h->cnorms.p : h->norms;
    sp.ntotal = h->ntotal;
    sp.row_bytes = h->row_bytes;
    sp.qop = (const char*)h->qop.p;
    sp.nq = nq;
    sp.dbg = h->opt.scan_dbg;
    if ((e = h->gtau.ensure((size_t)P.nq_pad * 4)) != hipSuccess) return e;
    sp.gtau = (unsigned*)h->gtau.p;
    sp.conv = nullptr;
    // (only grids of more than one dispatch round: a single round's blocks
    // start together, and the word's read would only add a round trip to
    // the one-query call)
    if (h->opt.convoy != 0 && sp.grid > 256 && sp.splits <= CONV_MAX) {
        if (!h->conv.p) {
            if ((e = h->conv.ensure((size_t)CONV_WORDS * 4)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(h->conv.p, 0, (size_t)CONV_WORDS * 4, h->stream())) != hipSuccess) return e;
        }
        sp.conv = (unsigned*)h->conv.p;
    }
    {
        const int ce = h->opt.convoy_every;
        sp.conv_every = ce >= 8 ? 8 : ce >= 4 ? 4 : ce >= 2 ? 2 : 1;
    }
    // k_scan_v4's published per-split lists (the union threshold, see
    // compact_wave): slow-path tiles 25.7 -> 16.5 %, config (d) -3 %
    if (sp.share && sp.splits > 1 && h->opt.pub != 0) {
        const size_t npub = (size_t)sp.n_qtiles * sp.qt * sp.splits * KP;
        if ((e = h->pub.ensure(npub * 4)) != hipSuccess) return e;
        sp.pub = (float*)h->pub.p;
        // union bound taken at rank max(6k/5, 12) (<= KP): tighter pruning;
        // the refine's certification bound is capped by the final threshold.
        // (k = 10: 12, was 20 -- config (b) -4.5 %, (d) -1 %, 0 fallbacks in
        // every certification stress case; profiles/r3/ab/prune_rank*)
        sp.prune_rank = h->opt.prune_rank > 0 ? h->opt.prune_rank : std::max(6 * k / 5, 12);
        sp.prune_rank = std::max(k, std::min(KP, sp.prune_rank));
    }
    P.ncand = (size_t)sp.n_qtiles * sp.splits * sp.qt * KP;
    if ((e = h->cand_d.ensure(P.ncand * 4)) != hipSuccess) return e;
    if ((e = h->cand_i.ensure(P.ncand * 4)) != hipSuccess) return e;
    sp.cand_d = (float*)h->cand_d.p;
    sp.cand_i = (int*)h->cand_i.p;
    sp.trace = nullptr;
    sp.dbgbuf = nullptr;
    sp.stamps = nullptr;
    sp.nq_dev = nullptr;

    if ((e = h->flag.ensure((size_t)(nq + 1) * 4)) != hipSuccess) return e;
    RefineParams& rp = P.rp;
    rp.cand_d = sp.cand_d;
    rp.cand_i = sp.cand_i;
    rp.splits = sp.splits;
    rp.qt = sp.qt;
    rp.nq = nq;
    rp.ntotal = h->ntotal;
    rp.k = k;
    rp.codes = h->codes;
    rp.row_bytes = h->row_bytes;
    rp.kdim = h->kdim;
    rp.qf32 = pp.qf32;
    rp.qeps = pp.qeps;
    rp.qrho = pp.qrho;
    rp.qshift = pp.qshift;
    rp.id_offset = h->id_offset;
    rp.D = Dd;
    rp.I = Id;
    rp.n_flag = words ? words + 1 : (int*)h->flag.p;
    rp.flag_list = rp.n_flag + 1;
    rp.n_drop = words ? words : h->dev_drop;
    // small batches: one wave per query walks splits * KP candidates (256 splits
    // at nq = 1); issue 4 chunks of loads at a time (nq = 1: 0.84 -> ~0.3 ms)
    rp.prefetch = nq <= 256 ? 4 : 1;
    rp.k1 = big_k1(k);
    rp.force_fb = h->opt.force_fallback != 0;
    rp.gtau = sp.share ? sp.gtau : nullptr;
    rp.nq_dev = nullptr;
    rp.out_idx = nullptr;
    P.reduce = small_many(k, nq, sp.splits) && h->opt.reduce_cand == 2;
    rp.wg = small_many(k, nq, sp.splits) && h->opt.reduce_cand == 1 ? h->opt.refine_waves : 0;
    if (P.reduce) {
        const size_t nred = (size_t)sp.n_qtiles * ((sp.splits + 15) / 16) * sp.qt * KP;
        if ((e = h->cand2_d.ensure(nred * 4)) != hipSuccess) return e;
        if ((e = h->cand2_i.ensure(nred * 4)) != hipSuccess) return e;
    }
    const size_t nfb = (size_t)std::max<int64_t>(4096, nq) * k;
    if ((e = h->fbc_d.ensure(nfb * 4)) != hipSuccess) return e;
    if ((e = h->fbc_i.ensure(nfb * 4)) != hipSuccess) return e;
    return plan_rescan(h, P);
}

// Enqueue the planned search on s up to its certification: query preparation
// (which also resets the shared thresholds, the published lists and the
// search's counters: one kernel instead of memsets), scan, refine +
// certification (small batches over many splits: one workgroup per query,
// or the separate candidate reduction when asked for).  No host sync: the
// same sequence is what a search graph captures.
hipError_t enqueue_main(FxIndex* h, SearchPlan& P, hipStream_t s, bool timed, hipEvent_t* ev) {
    hipError_t e;
    PrepParams pp1 = P.pp;
    pp1.gtau = P.sp.gtau;
    pp1.zero[0] = P.rp.n_drop;
    pp1.zero[1] = P.rp.n_flag;
    pp1.zero[2] = P.n_exact;
    pp1.pub = P.sp.pub;  // only live queries publish: nq rows of [splits][KP]
    pp1.npub = P.sp.pub ? P.nq * P.sp.splits * KP : 0;
    if ((e = launch_prep_queries(pp1, s)) != hipSuccess) return e;
    if (timed && (e = hipEventRecord(ev[0], s)) != hipSuccess) return e;
    if ((e = launch_scan(P.scan_dt, h->metric, P.sp, s)) != hipSuccess) return e;
    if (timed && (e = hipEventRecord(ev[1], s)) != hipSuccess) return e;
    RefineParams rp = P.rp;
    if (P.reduce) {
        int ng = 0;
        if ((e = launch_reduce_cand(P.sp.cand_d, P.sp.cand_i, P.sp.splits, P.nq, P.sp.qt, (float*)h->cand2_d.p,
                                    (int*)h->cand2_i.p, &ng, P.rp.ntotal, P.rp.n_drop, s)) != hipSuccess)
            return e;
        rp.cand_d = (const float*)h->cand2_d.p;
        rp.cand_i = (const int*)h->cand2_i.p;
        rp.splits = ng;
    }
    if ((e = launch_refine(h->dtype, h->metric, rp, s)) != hipSuccess) return e;
    if (timed && (e = hipEventRecord(ev[2], s)) != hipSuccess) return e;
    return hipSuccess;
}

// The chain for the queries the refine could not certify (rare: only when the
// candidate margin is inside the scan's rounding bound): a re-scan with a
// wide candidate set (plan_rescan), then the exact scan for what that still
// cannot certify.  Device-gated: every kernel reads the flagged count and
// exits at once when it is 0.  A device-resident search enqueues it always
// (no host round trip inside the search); a host-output search enqueues it
// only when its packed result says some query was flagged (finish_host_out).
hipError_t enqueue_fallback(FxIndex* h, SearchPlan& P, hipStream_t s) {
    hipError_t e;
#ifdef FX_ABLATION
    if ((P.sp.dbg & ~32) != 0) return hipSuccess;  // ablated scans: results invalid, no fallback chain
#endif
    if ((e = launch_rescan_chunks(P.rp.n_flag, (int)RESCAN_MAX, P.nchunks, P.chunk_cnt, s)) != hipSuccess) return e;
    for (int c = 0; c < P.nchunks; ++c) {  // chunk c: flagged queries [c RESCAN_MAX, ...)
        const int* list = P.rp.flag_list + (size_t)c * RESCAN_MAX;
        PrepParams pp = P.pp2;
        pp.qidx = list;
        pp.nq_dev = P.chunk_cnt + c;
        pp.zero[0] = pp.zero[1] = pp.zero[2] = nullptr;
        pp.pub = nullptr;
        pp.npub = 0;
        ScanParams sp = P.sp2;
        pp.gtau = sp.gtau;  // reset by the chunk's query preparation
        sp.nq_dev = P.chunk_cnt + c;
        RefineParams rp2 = P.rp2;
        rp2.nq_dev = P.chunk_cnt + c;
        rp2.out_idx = list;
        if ((e = launch_prep_queries(pp, s)) != hipSuccess) return e;
        if ((e = launch_scan(P.scan_dt, h->metric, sp, s)) != hipSuccess) return e;
        if ((e = launch_refine(h->dtype, h->metric, rp2, s)) != hipSuccess) return e;
    }
    return launch_exact_fallback(h->dtype, h->metric, h->codes, h->row_bytes, h->kdim, h->ntotal, P.rp.qf32,
                                 P.n_exact, P.k, h->id_offset, (float*)h->fbc_d.p, (int*)h->fbc_i.p, P.rp.D, P.rp.I,
                                 s);
}

// Host-output searches (the reference's call form) return through ONE packed
// device buffer, copied back with one D2H:
//   [D: nq k f32 | I: nq k i64 | n_drop | n_flag | flag list: nq i32]
// (the copy covers D .. n_flag; the flag list stays on the device for the
// fallback chain)
struct HostOut {
    size_t offI = 0, offW = 0, copy_bytes = 0, bytes = 0;
};
HostOut host_out_layout(int64_t nq, int k) {
    HostOut L;
    L.offI = (size_t)round_up(nq * k * 4, 8);
    L.offW = L.offI + (size_t)nq * k * 8;
    L.copy_bytes = L.offW + 8;
    L.bytes = L.offW + (size_t)(2 + nq) * 4;
    return L;
}

hipError_t ensure_pinned(char*& p, size_t& have, size_t want) {
    if (want <= have) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    have = 0;
    const size_t grow = std::max(want, have + have / 2);
    hipError_t e = hipHostMalloc((void**)&p, grow, hipHostMallocDefault);
    if (e == hipSuccess) have = grow;
    return e;
}

#ifdef FX_DIAG
template <typename T>
hipError_t dump_device(const std::string& path, const void* dev, size_t n) {
    std::vector<T> v(n);
    hipError_t e = hipMemcpy(v.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    if (FILE* f = fopen(path.c_str(), "ab")) {
        fwrite(v.data(), sizeof(T), n, f);
        fclose(f);
    }
    return hipSuccess;
}
#endif

// a host-output search whose refine dropped candidate ids outside [0, ntotal)
// (a corrupted scan list): the top-k may be missing rows, so it is an error
// (include/fx_index.h, fx_index_last_dropped_candidates)
int integrity_error(const FxIndex* h) {
    return set_err(FX_E_INTEGRITY, "search: %lld candidate row ids outside [0, %lld) were dropped (corrupted scan list)",
                   (long long)h->last_dropped, (long long)h->ntotal);
}

// Wait for a host-output search's results.  The one-query call is latency
// bound: polling the stream (host_spin) returns as soon as the D2H copy is
// done, where a blocking synchronise adds the runtime's wake-up latency.
hipError_t wait_results(const FxIndex* h, hipStream_t s) {
    if (!h->opt.host_spin) return hipStreamSynchronize(s);
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipErrorNotReady) return e;
    }
}

// A host-output search after its packed copy landed in `pin` (the stream is
// synchronised): when the refine flagged queries, run their fallback chain
// now and copy the results again (rare); then hand D / I to the caller.
int finish_host_out(FxIndex* h, SearchPlan& P, const HostOut& L, char* pin, float* D, int64_t* I) {
    hipStream_t s = h->stream();
    const int nflag = ((const int*)(pin + L.offW))[1];
    h->last_exact = 0;
    if (nflag > 0) {
        HIP_TRY(ensure_pinned_count(h));
        HIP_TRY(enqueue_fallback(h, P, s));
        HIP_TRY(hipMemcpyAsync(pin, P.rp.D, L.copy_bytes, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(h->pin_nf + 1, P.n_exact, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        h->last_exact = h->pin_nf[1];
    }
    const int* w = (const int*)(pin + L.offW);
    memcpy(D, pin, (size_t)P.nq * P.k * 4);
    memcpy(I, pin + L.offI, (size_t)P.nq * P.k * 8);
    h->last_fallbacks = nflag;
    h->last_dropped = w[0];
    h->fb_pending = false;
    return h->last_dropped > 0 ? integrity_error(h) : FX_OK;
}

// host queries of a host-output search up to this size go through pinned
// staging (a memcpy and an async DMA instead of the runtime's pageable path:
// the one-query call is latency bound); the call waits for its results, so
// the staging buffer is free again when it returns
constexpr size_t QPIN_MAX = (size_t)4 << 20;

int do_search(FxIndex* h, int64_t nq, const void* q, int q_dtype, int q_mem, int k, float* D, int64_t* I,
              int out_mem) {
    hipStream_t s = h->stream();
    const int qes = dtype_size(q_dtype);
    // queries -> device
    const void* qdev = q;
    if (q_mem == FX_MEM_HOST) {
        const size_t qb = (size_t)nq * h->d * qes;
        HIP_TRY(h->qin.ensure(qb));
        if (out_mem == FX_MEM_HOST && qb <= QPIN_MAX && ensure_pinned(h->qpin, h->qpin_bytes, qb) == hipSuccess) {
            memcpy(h->qpin, q, qb);
            HIP_TRY(hipMemcpyAsync(h->qin.p, h->qpin, qb, hipMemcpyHostToDevice, s));
        } else {
            HIP_TRY(hipMemcpyAsync(h->qin.p, q, qb, hipMemcpyHostToDevice, s));
        }
        qdev = h->qin.p;
    }
    // host results: the packed output buffer (host_out_layout)
    const bool host_out = out_mem == FX_MEM_HOST;
    HostOut L;
    float* Dd = D;
    int64_t* Id = I;
    int* words = nullptr;
    if (host_out) {
        L = host_out_layout(nq, k);
        HIP_TRY(h->hout.ensure(L.bytes));
        HIP_TRY(ensure_pinned(h->hpin, h->hpin_bytes, L.copy_bytes));
        Dd = (float*)h->hout.p;
        Id = (int64_t*)((char*)h->hout.p + L.offI);
        words = (int*)((char*)h->hout.p + L.offW);
    }
    HIP_TRY(update_scan_image(h));
    SearchPlan P;
    HIP_TRY(plan_search(h, nq, qdev, q_dtype, k, Dd, Id, words, P));
#ifdef FX_DIAG
    // diagnostics (Options): per-block placement/timing, phase stamps, the
    // scan's key matrix, raw candidate lists -> binary files
    const size_t grid = (size_t)P.sp.grid;
    if (!h->opt.stamps.empty()) {
        HIP_TRY(h->stamps.ensure(grid * 4 * 128));
        HIP_TRY(hipMemsetAsync(h->stamps.p, 0, grid * 4 * 128, s));
        P.sp.stamps = (unsigned long long*)h->stamps.p;
    }
    const size_t nkeys = (size_t)P.sp.n_qtiles * P.sp.qt * P.sp.n_ctiles * P.sp.tr;
    if ((P.sp.dbg & 32) && nkeys <= (size_t)1 << 26) {
        HIP_TRY(h->dbgbuf.ensure(nkeys * 4));
        HIP_TRY(hipMemsetAsync(h->dbgbuf.p, 0xff, nkeys * 4, s));
        P.sp.dbgbuf = (unsigned*)h->dbgbuf.p;
    }
    if (!h->opt.trace.empty()) {
        HIP_TRY(h->trace.ensure(grid * 32));
        HIP_TRY(hipMemsetAsync(h->trace.p, 0, grid * 32, s));
        P.sp.trace = (unsigned long long*)h->trace.p;
    }
#endif
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    if (h->profile)
        for (auto& x : ev) HIP_TRY(hipEventCreate(&x));
    HIP_TRY(enqueue_main(h, P, s, h->profile, ev));
    if (h->profile) {
        h->ev_scan.emplace_back(ev[0], ev[1]);
        h->ev_merge.emplace_back(ev[1], ev[2]);
    }
    if (!host_out) {
        // device results: the uncertified queries' chain is enqueued always and
        // decided on the device; the counts follow stream-ordered into pinned
        // memory, read only when asked for (read_counts)
        HIP_TRY(enqueue_fallback(h, P, s));
        HIP_TRY(ensure_pinned_count(h));
        HIP_TRY(hipMemcpyAsync(h->pin_nf, P.rp.n_flag, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(h->pin_nf + 1, P.n_exact, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(h->pin_nf + 2, P.rp.n_drop, 4, hipMemcpyDeviceToHost, s));
        h->fb_pending = true;
    }
#ifdef FX_DIAG
    if (!h->opt.cand.empty()) {
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(dump_device<float>(h->opt.cand, P.sp.cand_d, P.ncand));
        HIP_TRY(dump_device<int>(h->opt.cand, P.sp.cand_i, P.ncand));
    }
    if (P.sp.dbgbuf) {  // the scan's key matrix [n_qtiles*128][n_ctiles*128]
        HIP_TRY(hipStreamSynchronize(s));
        const std::string path = h->opt.keys.empty() ? std::string("/tmp/fx_keys.bin") : h->opt.keys;
        if (FILE* f = fopen(path.c_str(), "wb")) fclose(f);  // truncate: one dump per search
        HIP_TRY(dump_device<float>(path, P.sp.dbgbuf, nkeys));
    }
    if (P.sp.stamps) {
        HIP_TRY(hipStreamSynchronize(s));
        if (FILE* f = fopen(h->opt.stamps.c_str(), "wb")) fclose(f);
        HIP_TRY(dump_device<unsigned long long>(h->opt.stamps, P.sp.stamps, grid * 4 * 16));
    }
    if (P.sp.trace) {
        HIP_TRY(hipStreamSynchronize(s));
        if (FILE* f = fopen(h->opt.trace.c_str(), "wb")) fclose(f);
        HIP_TRY(dump_device<unsigned long long>(h->opt.trace, P.sp.trace, grid * 4));
    }
#endif
    if (!host_out) return FX_OK;
    // host results: ONE packed D2H copy [D | I | n_drop | n_flag]
    HIP_TRY(hipMemcpyAsync(h->hpin, h->hout.p, L.copy_bytes, hipMemcpyDeviceToHost, s));
    HIP_TRY(wait_results(h, s));
    return finish_host_out(h, P, L, h->hpin, D, I);
}

// k > FX_BIG_K: exact keys of every (query, row) pair and a radix sort per
// query (fx_hugek.hip).  Every result is exact, so no query is "uncertified".
constexpr size_t HK_KEEP_BYTES = (size_t)512 << 20;
int do_search_hugek(FxIndex* h, int64_t nq, const void* q, int q_dtype, int q_mem, int k, float* D, int64_t* I,
                    int out_mem) {
    hipStream_t s = h->stream();
    const void* qdev = q;
    if (q_mem == FX_MEM_HOST) {
        HIP_TRY(h->qin.ensure((size_t)nq * h->d * dtype_size(q_dtype)));
        HIP_TRY(hipMemcpyAsync(h->qin.p, q, (size_t)nq * h->d * dtype_size(q_dtype), hipMemcpyHostToDevice, s));
        qdev = h->qin.p;
    }
    float* Dd = D;
    int64_t* Id = I;
    if (out_mem == FX_MEM_HOST) {
        HIP_TRY(h->dws.ensure((size_t)nq * k * 4));
        HIP_TRY(h->iws.ensure((size_t)nq * k * 8));
        Dd = (float*)h->dws.p;
        Id = (int64_t*)h->iws.p;
    }
    const int qb = hugek_batch(h->ntotal, nq);
    size_t ws = 0;
    HIP_TRY(hugek_workspace(h->ntotal, h->kdim, qb, &ws));
    HIP_TRY(h->hk_ws.ensure(ws));
    HugeKParams p{};
    p.codes = h->codes;
    p.row_bytes = h->row_bytes;
    p.kdim = h->kdim;
    p.d = h->d;
    p.st_dt = h->dtype;
    p.metric = h->metric;
    p.ntotal = h->ntotal;
    p.q = qdev;
    p.q_dt = q_dtype;
    p.nq = nq;
    p.k = k;
    p.id_offset = h->id_offset;
    p.D = Dd;
    p.I = Id;
    HIP_TRY(launch_hugek_search(p, h->hk_ws.p, h->hk_ws.bytes, qb, s));
    // the sort keys + rocPRIM temporaries stay cached for the next call up to
    // HK_KEEP_BYTES; a larger workspace (up to 2 GiB of keys) is released
    // after the call, which waits for the stream (hipFree would anyway)
    if (h->hk_ws.bytes > HK_KEEP_BYTES) {
        HIP_TRY(hipStreamSynchronize(s));
        h->hk_ws.release();
    }
    h->last_fallbacks = 0;
    h->last_exact = 0;
    h->last_dropped = 0;
    h->fb_pending = false;
    if (out_mem == FX_MEM_HOST) {
        HIP_TRY(hipMemcpyAsync(D, Dd, (size_t)nq * k * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(I, Id, (size_t)nq * k * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return FX_OK;
}

// Shape + options + every device buffer a captured search touches: the graph
// is valid while all of them are unchanged
std::vector<uint64_t> graph_key(const FxIndex* h, int64_t nq, int q_dtype, int k) {
    const Options& o = h->opt;
    return {(uint64_t)nq, (uint64_t)q_dtype, (uint64_t)k, (uint64_t)h->ntotal, (uint64_t)h->id_offset,
            (uint64_t)h->img_kind, (uint64_t)h->centred, (uint64_t)h->img_rows,
            (uint64_t)o.force_fallback, (uint64_t)o.place, (uint64_t)o.sx, (uint64_t)o.reduce_cand,
            (uint64_t)o.pub, (uint64_t)o.prune_rank, (uint64_t)o.compact_at, (uint64_t)o.union_w,
            (uint64_t)o.union_defer, (uint64_t)(int64_t)o.union_inplace, (uint64_t)(int64_t)o.tight_at, (uint64_t)o.cold_bound,
            (uint64_t)o.reduce_cand, (uint64_t)o.scan_v5, (uint64_t)o.refine_waves, (uint64_t)o.convoy, (uint64_t)o.convoy_every,
            (uint64_t)(uintptr_t)h->codes, (uint64_t)(uintptr_t)h->norms, (uint64_t)(uintptr_t)h->split.p,
            (uint64_t)(uintptr_t)h->cnorms.p, (uint64_t)(uintptr_t)h->centre.p, (uint64_t)(uintptr_t)h->qshift.p,
            (uint64_t)(uintptr_t)h->qin.p, (uint64_t)(uintptr_t)h->qf32.p, (uint64_t)(uintptr_t)h->qop.p,
            (uint64_t)(uintptr_t)h->qeps.p, (uint64_t)(uintptr_t)h->qrho.p, (uint64_t)(uintptr_t)h->gtau.p,
            (uint64_t)(uintptr_t)h->pub.p, (uint64_t)(uintptr_t)h->cand_d.p, (uint64_t)(uintptr_t)h->cand_i.p,
            (uint64_t)(uintptr_t)h->cand2_d.p, (uint64_t)(uintptr_t)h->cand2_i.p,
            (uint64_t)(uintptr_t)h->hout.p, (uint64_t)(uintptr_t)h->conv.p,
            (uint64_t)(uintptr_t)h->flag.p, (uint64_t)(uintptr_t)h->fbc_d.p, (uint64_t)(uintptr_t)h->fbc_i.p,
            (uint64_t)(uintptr_t)h->rq_f32.p, (uint64_t)(uintptr_t)h->rq_op.p, (uint64_t)(uintptr_t)h->rq_eps.p,
            (uint64_t)(uintptr_t)h->rq_rho.p, (uint64_t)(uintptr_t)h->rq_shift.p, (uint64_t)(uintptr_t)h->rq_gtau.p,
            (uint64_t)(uintptr_t)h->rq_cand_d.p, (uint64_t)(uintptr_t)h->rq_cand_i.p,
            (uint64_t)(uintptr_t)h->rq_flag.p};
}

void graph_release(FxIndex* h) {
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    h->gexec = nullptr;
    h->gkey.clear();
}

// Record the stream-ordered search of do_search (host queries, host results,
// no diagnostics) into h->gexec: the query's H2D copy, enqueue_main (prep,
// scan, refine: no fallback chain) and the packed result's one D2H copy.
// Runs right after a do_search of the same shape, so every workspace is
// sized and every kernel attribute set.
hipError_t graph_build(FxIndex* h, int64_t nq, int q_dtype, int k) {
    graph_release(h);
    hipStream_t s = h->stream();
    const size_t qb = (size_t)nq * h->d * dtype_size(q_dtype);
    const HostOut L = host_out_layout(nq, k);
    hipError_t e = hipSuccess;
    if (qb > h->ghq_bytes) {
        if (h->ghq) (void)hipHostFree(h->ghq);
        h->ghq = nullptr;
        h->ghq_bytes = 0;
        if ((e = hipHostMalloc(&h->ghq, qb, hipHostMallocDefault)) != hipSuccess) return e;
        h->ghq_bytes = qb;
    }
    if ((e = ensure_pinned(h->ghout, h->ghout_bytes, L.copy_bytes)) != hipSuccess) return e;
    if ((e = h->hout.ensure(L.bytes)) != hipSuccess) return e;  // (sized by the do_search before)
    char* hb = (char*)h->hout.p;
    SearchPlan& P = h->gplan;
    P = SearchPlan{};
    if ((e = plan_search(h, nq, h->qin.p, q_dtype, k, (float*)hb, (int64_t*)(hb + L.offI), (int*)(hb + L.offW),
                         P)) != hipSuccess)
        return e;
    P.sp.dbg = 0;

    if ((e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal)) != hipSuccess) return e;
    g_graph_capture = true;
    hipError_t ce = hipMemcpyAsync(h->qin.p, h->ghq, qb, hipMemcpyHostToDevice, s);
    if (ce == hipSuccess) ce = enqueue_main(h, P, s, false, nullptr);
    if (ce == hipSuccess) ce = hipMemcpyAsync(h->ghout, hb, L.copy_bytes, hipMemcpyDeviceToHost, s);
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
    h->gkey = graph_key(h, nq, q_dtype, k);
    return hipSuccess;
}

// Small host batches under search_graph: replay the captured search; its
// fallback chain runs eagerly only when the packed result flags a query
// (finish_host_out).  On a shape / buffer / option change run do_search and
// re-capture.
int graph_search(FxIndex* h, int64_t nq, const void* q, int q_dtype, int k, float* D, int64_t* I) {
    HIP_TRY(update_scan_image(h));
    if (h->gexec && graph_key(h, nq, q_dtype, k) == h->gkey) {
        hipStream_t s = h->stream();
        memcpy(h->ghq, q, (size_t)nq * h->d * dtype_size(q_dtype));
        HIP_TRY(hipGraphLaunch(h->gexec, s));
        HIP_TRY(wait_results(h, s));
        return finish_host_out(h, h->gplan, host_out_layout(nq, k), h->ghout, D, I);
    }
    const int rc = do_search(h, nq, q, q_dtype, FX_MEM_HOST, k, D, I, FX_MEM_HOST);
    if (rc == FX_OK && !h->gfailed) {
        const hipError_t e = graph_build(h, nq, q_dtype, k);
        if (e != hipSuccess) {  // stay on do_search for this index
            h->gfailed = true;
            if (h->opt.graph_verbose) fprintf(stderr, "fx: search graph capture failed: %s\n", hipGetErrorString(e));
        } else if (h->opt.graph_verbose) {
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
    h->opt.from_env();
    // A BLOCKING stream: work on the legacy null stream (torch's default
    // stream, cuda_stream == 0) is ordered before and after it, so a caller
    // that binds "stream 0" (fx_index_set_stream(h, NULL)) stays ordered.
    hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->switch_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc(&h->max_sq_bits, 16);
    if (e == hipSuccess) e = hipMemset(h->max_sq_bits, 0, 16);
    if (e == hipSuccess) e = hipMalloc(&h->dev_drop, 16);
    if (e == hipSuccess) e = hipMemset(h->dev_drop, 0, 16);
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
        if (h->dev_drop) (void)hipFree(h->dev_drop);
        for (DevBuf* b : {&h->qin, &h->qf32, &h->qop, &h->qeps, &h->cand_d, &h->cand_i, &h->dws, &h->iws, &h->flag,
                          &h->fbc_d, &h->fbc_i, &h->stage, &h->gtau, &h->trace, &h->dbgbuf, &h->split, &h->cnorms,
                          &h->centre, &h->mu_part, &h->qshift, &h->qrho, &h->stamps, &h->pub, &h->cand2_d,
                          &h->cand2_i, &h->rq_f32, &h->rq_op, &h->rq_eps, &h->rq_rho, &h->rq_shift, &h->rq_gtau,
                          &h->rq_cand_d, &h->rq_cand_i, &h->rq_flag, &h->hk_ws, &h->hout, &h->conv})
            b->release();
        graph_release(h);
        if (h->ghq) (void)hipHostFree(h->ghq);
        if (h->ghout) (void)hipHostFree(h->ghout);
        if (h->hpin) (void)hipHostFree(h->hpin);
        if (h->qpin) (void)hipHostFree(h->qpin);
        if (h->pin_nf) (void)hipHostFree(h->pin_nf);
        for (auto& pr : h->ev_scan) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
        for (auto& pr : h->ev_merge) (void)hipEventDestroy(pr.second);
        if (h->switch_ev) (void)hipEventDestroy(h->switch_ev);
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
    const hipStream_t prev = h->stream();
    h->user_stream = (hipStream_t)stream;
    const hipStream_t next = h->stream();
    if (next != prev) {
        // the index's work stays in call order across a stream switch: the new
        // stream waits (on the device) for everything enqueued on the old one
        DeviceGuard g(h->device);
        HIP_TRY(hipEventRecord(h->switch_ev, prev));
        HIP_TRY(hipStreamWaitEvent(next, h->switch_ev, 0));
    }
    return FX_OK;
}

int fx_index_set_option(FxIndex* h, const char* name, int64_t value) {
    if (!h || !name) return set_err(FX_E_ARG, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    const char* why = nullptr;
    int* slot = h->opt.find(name, value, &why);
    if (!slot) return set_err(FX_E_ARG, "unknown option '%s'", name);
    if (why) return set_err(FX_E_ARG, "option '%s': %s (%lld)", name, why, (long long)value);
    *slot = (int)value;
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
    static_assert(FX_MAX_K == FX_BIG_K, "ABI k limit of the scan path = the big-k refine's");
    if (!check_dtype(q_dtype)) return set_err(FX_E_ARG, "bad query dtype %d", q_dtype);
    if (nq == 0) return FX_OK;
    if (!q || !D || !I) return set_err(FX_E_ARG, "null buffer");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    if (h->ntotal > 0 && k > FX_MAX_K) return do_search_hugek(h, nq, q, q_dtype, q_mem, k, D, I, out_mem);
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
        h->last_exact = 0;
        h->last_dropped = 0;
        h->fb_pending = false;
        return FX_OK;
    }
    const Options& o = h->opt;
#ifdef FX_DIAG
    const bool diag = o.scan_dbg != 0 || !o.trace.empty() || !o.cand.empty() || !o.stamps.empty();
#else
    constexpr bool diag = false;
#endif
    if (o.search_graph == 1 && q_mem == FX_MEM_HOST && out_mem == FX_MEM_HOST && nq <= 64 && !h->profile && !diag &&
        h->user_stream == nullptr)
        return graph_search(h, nq, q, q_dtype, k, D, I);
    return do_search(h, nq, q, q_dtype, q_mem, k, D, I, out_mem);
}

// the counts of the last search (after a device-resident one: synchronises the
// index stream, which is ordered after every stream the index used before)
static int read_counts(FxIndex* h) {
    if (h->fb_pending) {
        DeviceGuard g(h->device);
        HIP_TRY(hipStreamSynchronize(h->stream()));
        h->last_fallbacks = h->pin_nf[0];
        h->last_exact = h->pin_nf[1];
        h->last_dropped = h->pin_nf[2];
        h->fb_pending = false;
        if (h->last_dropped > 0) return integrity_error(h);
    }
    return FX_OK;
}

int fx_index_last_dropped_candidates(FxIndex* h, int64_t* out) {
    if (!h || !out) return set_err(FX_E_ARG, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    const int rc = read_counts(h);
    if (rc != FX_OK) return rc;
    *out = h->last_dropped;
    return FX_OK;
}

int fx_index_last_fallbacks(FxIndex* h, int64_t* out) {
    if (!h || !out) return set_err(FX_E_ARG, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    const int rc = read_counts(h);
    if (rc != FX_OK) return rc;
    *out = h->last_fallbacks;
    return FX_OK;
}

int fx_index_last_scan_plan(FxIndex* h, int* tile_rows, int* query_tile, int* splits) {
    if (!h || !tile_rows || !query_tile || !splits) return set_err(FX_E_ARG, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    *tile_rows = h->last_plan[0];
    *query_tile = h->last_plan[1];
    *splits = h->last_plan[2];
    return FX_OK;
}

int fx_index_last_exact_fallbacks(FxIndex* h, int64_t* out) {
    if (!h || !out) return set_err(FX_E_ARG, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    const int rc = read_counts(h);
    if (rc != FX_OK) return rc;
    *out = h->last_exact;
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
    h->img_rows = 0;
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
    if (nshards <= 0 || nq < 0 || k <= 0) return set_err(FX_E_ARG, "bad merge shape");
    if (!D_in || !I_in || !D_out || !I_out) return set_err(FX_E_ARG, "null buffer");
    if (metric != FX_METRIC_L2 && metric != FX_METRIC_INNER_PRODUCT) return set_err(FX_E_ARG, "bad metric");
    DeviceGuard g(device);
    if (!g.ok) return set_err(FX_E_HIP, "hipSetDevice(%d) failed", device);
    if (k > FX_MAX_K && nshards > FX_HUGEK_MAX_SHARDS)
        return set_err(FX_E_UNSUPPORTED, "merge of k = %d > %d lists supports at most %d shards (got %d)", k, FX_MAX_K,
                       FX_HUGEK_MAX_SHARDS, nshards);
    if (k > FX_MAX_K)  // stream-ordered sort merge (fx_hugek.hip)
        HIP_TRY(launch_merge_shards_sort(metric, nshards, nq, k, D_in, I_in, D_out, I_out, (hipStream_t)stream));
    else
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
