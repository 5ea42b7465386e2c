// fx_internal.h -- shared between the HIP kernels (fx_kernels.hip) and the
// host C ABI (fx_index.cpp).  Not part of the public ABI (include/fx_index.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fx {

// ---- tiling of the fused scan kernel (see DESIGN.md "scan kernel") --------
constexpr int TILE_R = 128;   // corpus rows per tile (MFMA M side)
constexpr int TILE_Q = 128;   // queries per tile      (MFMA N side)
constexpr int STAGE_B = 128;  // bytes of each row's K staged per pipeline stage
constexpr int KP = 32;        // candidates kept per (query, corpus split)
constexpr int FX_BIG_K = 1024;  // largest k of the scan path (k > KP: k_refine_big; == FX_MAX_K of the
                                // ABI); larger k: fx_hugek.hip
constexpr int CAP = 64;       // LDS candidate-list capacity per query (2*KP)
constexpr int ROW_ALIGN = 128;  // row stride alignment in bytes (== STAGE_B)
constexpr int SCAN_THREADS = 256;

// dynamic LDS carve of the scan kernel (all in ONE extern array: see
// cdna_hip_programming.md 5.4 item 4(a))
constexpr int LDS_STAGE = 2 * (TILE_R + TILE_Q) * STAGE_B;   // 64 KiB double buffer
constexpr int LDS_NORM_OFF = LDS_STAGE;                       // 2 x 512 B row norms
constexpr int LDS_LD_OFF = LDS_NORM_OFF + 2 * TILE_R * 4;    // lst_d [TILE_Q][CAP] f32
constexpr int LDS_LI_OFF = LDS_LD_OFF + TILE_Q * CAP * 4;    // lst_i [TILE_Q][CAP] i32
constexpr int LDS_CNT_OFF = LDS_LI_OFF + TILE_Q * CAP * 4;   // cnt   [TILE_Q] i32
constexpr int LDS_TAU_OFF = LDS_CNT_OFF + TILE_Q * 4;        // tau   [TILE_Q] f32
constexpr int LDS_FLAG_OFF = LDS_TAU_OFF + TILE_Q * 4;       // overflow flag (16 B)
constexpr int LDS_SCAN_BYTES = LDS_FLAG_OFF + 16;

enum Dtype { F32 = 0, BF16 = 1, F16 = 2,
             // scan-only operand format of an fp32 index (FX_F32_SPLIT=1): every
             // value v as bf16 hi = rn(v) and lo = rn(v - hi), rows laid out
             // [hi plane | lo plane] in the fp32 row's bytes; the scan sums
             // hi*hi + hi*lo + lo*hi with bf16 MFMAs (never a storage dtype)
             F32S = 3 };
enum Metric { IP = 0, L2 = 1 };

inline int dtype_size(int dt) { return dt == F32 ? 4 : 2; }

struct ScanParams {
    const char* codes;     // [cap_rows][row_bytes] storage dtype, zero padded
    const float* norms;    // [cap_rows] |y|^2 (fp32, of stored values)
    int64_t ntotal;
    int row_bytes;
    const char* qop;       // [nq_pad][row_bytes] queries in storage dtype
    int64_t nq;
    int n_qtiles;
    int n_ctiles;          // corpus tiles (ceil(ntotal / TILE_R))
    int splits;            // corpus splits per query tile
    int qt_per_xcd;        // query tiles assigned per XCD group
    float* cand_d;         // [n_qtiles][splits][TILE_Q][KP]
    int* cand_i;
    int dbg;               // ablation switches (FX_SCAN_DBG; 0 in production)
    unsigned* gtau;        // [n_qtiles * TILE_Q] order-preserving bits of the best
                           // known KP-th key per query across splits (atomicMin)
    unsigned long long* trace;  // diagnostics only (FX_SCAN_TRACE): per block
                                // {xcc | hw_id << 8 | qtile << 32, split, t_start, t_end}
    unsigned* dbgbuf;           // diagnostics only (FX_SCAN_DBG & 32): operand self-check
    int share;                  // 1: splits publish their KP-th key to gtau and prune with it
                                // (k <= KP); 0: no cross-split pruning (k > KP, k_refine_big)
    int place;                  // block placement (map_tile): 0 query-tile groups per XCD, 1
                                // corpus-partitioned (XCD x owns splits [x sx, (x+1) sx))
    int sx;                     // place 1: corpus splits per XCD (splits = 8 sx)
    int grid;                   // workgroups of the scan launch
    int prune_rank;             // rank of the union bound published to gtau (compact_wave)
    int union_w;                // union bound window: 16, 32 or 64 splits (their first 256 / union_w keys)
    int compact_at;             // a list is compacted once it holds this many entries (KP < v <= CAP;
                                // the threshold only improves at a compaction)
    float* pub;                 // k_scan_v4 with share: [n_qtiles * TILE_Q][splits][KP] each split's
                                // last compacted top-KP keys per query (null: not used)
    unsigned long long* stamps; // diagnostics only (FX_SCAN_STAMPS, -DFX_ABLATION builds):
                                // [grid][4 waves][16] per-wave cycle sums of the scan's phases
    const int* nq_dev;          // non-null (the re-scan of uncertified queries): the live query
                                // count is min(*nq_dev, nq), known only on the device
    int union_defer;            // 1: a compaction's union bound is fetched by LDS-DMA and bounded at
                                // the next tile's epilogue (compact_regs); 0: waited for in place
    int tight_at;               // > 0: a list that took entries in a tile and holds >= tight_at (below
                                // the compaction trigger) gets its threshold re-bounded (tighten_list)
    int union_inplace;          // most lists per compaction call bounded in place by the union (those
                                // past the deferred slots); the rest publish only their own bound
    int cold_bound;             // 1: a still-empty list's first record tile bounds its threshold by the
                                // prune_rank-th of the tile's group minima before pushing
    int qt;                     // queries per scan tile (the candidate layout's [qtile][split][qt][KP]):
                                // TILE_Q (k_scan_v4 / k_scan_topk) or 256 (k_scan_v5)
    int tr;                     // corpus rows per scan tile: TILE_R, or 64 (k_scan_v5)
    unsigned* conv;             // convoy words of k_scan_v4 / v5, one line per split (null: every block starts at its
                                // split's first tile): blocks publish the split-relative tile they scan,
                                // and a starting block begins there (circularly), so blocks of one split
                                // read the same rows at the same time whenever they started
    int conv_every;             // publish every conv_every tiles (power of 2)
};
// convoy splits per index (splits above this scan without them); one 64-B
// line (16 words) per split
constexpr int CONV_MAX = 4096;
constexpr int CONV_WORDS = CONV_MAX * 16;

// queries are zero-padded to a multiple of QPAD (the scan's query tile)
constexpr int QPAD = TILE_Q;

struct RefineParams {
    const float* cand_d;   // scan output (approx keys)
    const int* cand_i;
    int splits;
    int64_t nq;
    int k;
    const char* codes;
    int row_bytes;
    int kdim;
    const float* qf32;     // [nq_pad][kdim] fp32 queries, zero padded
    const float* qeps;     // [nq] E: query-wide bound on |approx key + shift - exact|
    const float* qrho;     // [nq] rho = |x - mu - x_op| (the scan operand's rounding): the bound adds
                           // 2 rho sqrt(D) for a row at exact distance D (L2, 16-bit / fp32 rows)
    const double* qshift;  // [nq] s_q: approx key + s_q estimates the exact distance
    int64_t id_offset;
    float* D;              // [nq][k]
    int64_t* I;
    int* n_flag;           // uncertified counter
    int* flag_list;        // [nq] uncertified query ids
    int prefetch;          // > 1: phase-1 loads issued 4 chunks at a time (small-batch scan)
    int k1;                // k > KP: approx candidates re-ranked exactly (2k, <= 2 FX_BIG_K)
    int force_fb;          // test hook (FX_FORCE_FALLBACK=1): flag every query -> exact fallback
    const unsigned* gtau;  // k <= KP: the scan's final shared thresholds (ordered bits): every row a split
                           // dropped lies above it, so it caps the certification bound; null: unused
    const int* nq_dev;     // non-null: live query count min(*nq_dev, nq) (the re-scan)
    const int* out_idx;    // non-null: query q's results go to row out_idx[q] of D / I, and an
                           // uncertified q is flagged as out_idx[q] (the re-scan's gathered queries)
    int64_t ntotal;        // rows of the index: a candidate row id outside [0, ntotal) is never gathered
    int* n_drop;           // ... and counted here (ids other than -1 outside [0, ntotal): a corrupted
                           // candidate list), read back by fx_index_last_dropped_candidates
    int qt;                // queries per scan tile of the candidate layout (ScanParams.qt)
    int wg;                // > 0: small batches over many splits (k <= KP): one workgroup of wg (4, 8, 16) waves per query
                           // (k_refine_wg: the waves share the walk over splits * KP candidates); 0: k_refine
};
// waves of k_refine_wg's workgroup (one query per workgroup) unless the
// index's option refine_waves says otherwise (4, 8 or 16)
constexpr int REFINE_WG_WAVES = 16;

// exact fallback (k_fb_scan / k_fb_merge): corpus splits per flagged query,
// decided on the device from the flagged count nf; items nf * fbs <=
// max(4096, nf), so the candidate buffer is max(4096, nq) * k entries
constexpr int FB_SCAN_GRID = 1024, FB_MERGE_GRID = 256;
__host__ __device__ inline int fb_splits_for(int nf, int64_t ntotal) {
    int s = nf >= 4096 ? 1 : 4096 / (nf > 0 ? nf : 1);
    if (s > 256) s = 256;
    const int64_t by_rows = ntotal / 1024 > 0 ? ntotal / 1024 : 1;
    if (s > by_rows) s = (int)by_rows;
    return s < 1 ? 1 : s;
}

// the re-scan of uncertified queries takes them in chunks of at most this
// many (its workspace is sized for one chunk)
constexpr int64_t RESCAN_MAX = 2048;
// counts[c] = live queries of re-scan chunk c: the flagged queries
// [c cap, min(n_flag[0], (c+1) cap)); device-gated like the fallbacks
hipError_t launch_rescan_chunks(const int* n_flag, int cap, int nchunks, int* counts, hipStream_t s);

// True on a thread that is capturing a search into a hipGraph (fx_index.cpp
// graph_build): the scan launchers then skip hipFuncSetAttribute, which the
// do_search right before the capture has already applied for the same kernel.
extern thread_local bool g_graph_capture;

// launchers (stream-ordered, no host sync) -- fx_kernels.hip
hipError_t launch_convert_rows(const void* x, int x_dt, int64_t n, int d, void* codes_row0, int st_dt,
                               int kdim, float* norms_row0, unsigned* max_sq_bits, int normalize,
                               hipStream_t s);
// search(): query preparation (k_prep_queries): fp32 copy for the exact
// refine, the scan operand, and the per-query certification terms
struct PrepParams {
    const void* q;          // [nq][d] caller queries, dtype q_dt, on the device
    int q_dt;
    int64_t nq, nq_pad;
    int d, kdim;
    int st_dt;              // scan dtype (F32, BF16, F16, F32S)
    int metric;
    float* qf32;            // [nq_pad][kdim] fp32 queries, zero padded
    void* qop;              // [nq_pad][row_bytes] scan operand (x - mu in the scan dtype, pre-scaled)
    float* qeps;            // [nq] E
    float* qrho;            // [nq] rho
    double* qshift;         // [nq] s_q
    const unsigned* mbits;     // max |y|^2 of the stored rows (float bits)
    const unsigned* img_bits;  // max srcC of the scan image (= mbits without an image)
    const float* mu;        // centre of the scan image (null: none)
    const int* qidx;        // non-null: row r of the batch is row qidx[r] of q (the re-scan's gather)
    const int* nq_dev;      // non-null: live query count min(*nq_dev, nq); later rows are padding
    // the search's resets, folded into this first kernel instead of memsets:
    unsigned* gtau;         // non-null: [nq_pad] the scan's shared thresholds, set to ord(+inf)
    int* zero[3];           // non-null entries: counters set to 0 (dropped ids, flagged, exact)
    float* pub;             // non-null: the scan's published lists, npub floats set to +inf
    int64_t npub;
};
hipError_t launch_prep_queries(const PrepParams& p, hipStream_t s);
hipError_t launch_scan(int st_dt, int metric, const ScanParams& p, hipStream_t s);
// fx_scan.hip: the MFMA scan; *handled = false when it has no kernel for p.row_bytes
hipError_t launch_scan_mfma(int st_dt, int metric, const ScanParams& p, hipStream_t s, bool* handled);
hipError_t launch_refine(int st_dt, int metric, const RefineParams& p, hipStream_t s);
// small batches: merge each 16 splits' candidate lists of a query into their
// top KP (k_reduce_cand); *ngroups = ceil(splits / 16) lists per query after
hipError_t launch_reduce_cand(const float* cd, const int* ci, int splits, int64_t nq, int qt, float* od,
                              int* oi, int* ngroups, int64_t ntotal, int* n_drop, hipStream_t s);
// fx_scan5.hip: the 64-row-tile, 256-query scan (k_scan_v5) and the shapes it has
int scan_v5_qt(int st_dt, int row_bytes);  // its queries per workgroup for these rows (0: no shape)
hipError_t launch_scan_v5(int st_dt, int metric, const ScanParams& p, hipStream_t s);
constexpr int V5_TR = 64;
// both fallback launches, always enqueued; they read the flagged count at
// n_flag[0] (list at n_flag + 1) and do nothing when it is 0
hipError_t launch_exact_fallback(int st_dt, int metric, const char* codes, int row_bytes, int kdim,
                                 int64_t ntotal, const float* qf32, const int* n_flag, int k,
                                 int64_t id_offset, float* cand_d, int* cand_i, float* D, int64_t* I,
                                 hipStream_t s);
hipError_t launch_merge_shards(int metric, int nshards, int64_t nq, int k, const float* D_in,
                               const int64_t* I_in, float* D_out, int64_t* I_out, hipStream_t s);
// k > FX_BIG_K (fx_hugek.hip): exact key of every (query, row) pair, a radix
// sort per query, the first k -> D / I (faiss padding past ntotal)
struct HugeKParams {
    const char* codes;     // [ntotal][row_bytes] stored rows (storage dtype st_dt)
    int row_bytes, kdim, d, st_dt, metric;
    int64_t ntotal;
    const void* q;         // [nq][d] queries on the device, dtype q_dt
    int q_dt;
    int64_t nq;
    int k;
    int64_t id_offset;
    float* D;              // [nq][k] on the device
    int64_t* I;
};
// queries per batch, and the workspace bytes a batch of qb queries needs
int hugek_batch(int64_t ntotal, int64_t nq);
hipError_t hugek_workspace(int64_t ntotal, int kdim, int qb, size_t* bytes);
hipError_t launch_hugek_search(const HugeKParams& p, void* ws, size_t ws_bytes, int qb, hipStream_t s);
// fx_merge_shards for k > FX_BIG_K: per query, a G-way merge of the gathered
// lists (each in the index order); at most FX_HUGEK_MAX_SHARDS shards
constexpr int FX_HUGEK_MAX_SHARDS = 64;
hipError_t launch_merge_shards_sort(int metric, int nshards, int64_t nq, int k, const float* D_in,
                                    const int64_t* I_in, float* D_out, int64_t* I_out, hipStream_t s);
// fp32 code rows [r0, r1) -> their F32S scan image (same row stride)
// (centred by mu when non-null), with the image rows' |v|^2 -> cnorms and their
// maximum -> cmax_bits (atomicMax)
hipError_t launch_split_rows(const float* codes, int kdim, int64_t r0, int64_t r1, const float* mu, void* split,
                             float* cnorms, unsigned* cmax_bits, hipStream_t s);
// mu[kdim] <- mean of a strided sample of <= MU_SAMPLE of the n stored rows
// (dtype dt, row stride row_bytes; part: 2 * MU_GROUPS * kdim doubles of
// scratch).  min_ratio > 0: mu is set to 0 when |mu|^2 < min_ratio * the
// sample's mean |y|^2 (no common direction to remove)
constexpr int64_t MU_SAMPLE = 1 << 20;
constexpr int MU_GROUPS = 64;
hipError_t launch_mu(const char* codes, int dt, int row_bytes, int d, int64_t n, double* part, float* mu,
                     float min_ratio, hipStream_t s);
// 16-bit rows [r0, r1) -> cnorms = |y - mu|^2 (fp64 sum, one rounding; mu null:
// |y|^2), their maximum -> cmax_bits (atomicMax)
hipError_t launch_centre_norms(const char* codes, int dt, int row_bytes, int64_t r0, int64_t r1, const float* mu,
                               float* cnorms, unsigned* cmax_bits, hipStream_t s);
hipError_t launch_synth(void* out, int64_t row0, int64_t n, int d, int dtype, uint64_t seed,
                        hipStream_t s);
hipError_t launch_to_f32(const void* codes, int st_dt, int row_bytes, int64_t n, int d, float* out,
                         hipStream_t s);

}  // namespace fx
