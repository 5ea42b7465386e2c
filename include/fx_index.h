/*
 * fx_index.h -- C ABI of the MI355X-native flat (brute-force) vector index.
 *
 * Drop-in boundary for the reference's dense-retrieval hot path.  The
 * reference binds faiss-cpu through SWIG; every call it makes maps to one
 * entry point below (the faiss C-API name of the same operation is given
 * for maintainers who bind through C instead of SWIG):
 *
 *   reference call site                              faiss C API                  this ABI
 *   faiss.IndexFlatL2(d)  faiss_store.py:29,126,     faiss_IndexFlatL2_new_with   fx_index_create
 *                         rag_datastore_manager.py:138
 *   index.add(x)          faiss_store.py:46,         faiss_Index_add              fx_index_add
 *                         rag_datastore_manager.py:173
 *   index.search(x, k)    faiss_store.py:64,         faiss_Index_search           fx_index_search
 *                         rag_datastore_manager.py:218
 *   index.ntotal          faiss_store.py:53          faiss_Index_ntotal           fx_index_ntotal
 *   (re)IndexFlatL2(d)    faiss_store.py:126         faiss_Index_reset            fx_index_reset
 *   faiss.write_index     faiss_store.py:91,         faiss_write_index_fname      fx_index_write
 *                         rag_datastore_manager.py:186
 *   faiss.read_index      faiss_store.py:106,        faiss_read_index_fname       fx_index_read
 *                         rag_datastore_manager.py:205
 *   (GC of the index)     --                         faiss_Index_free             fx_index_free
 *   (exceptions)          faiss_store.py:79-81,120   faiss_get_last_error         fx_last_error
 *
 * Semantics follow IndexFlatL2 (squared L2, no sqrt, no normalisation,
 * results ascending, ties -> smaller id, missing slots I = -1 and
 * D = FLT_MAX).  Returned ids are bit-exact with the CPU oracle; distances
 * are recomputed exactly (fp64 sum, one rounding to fp32).
 *
 * Conventions: every function returns 0 on success and a negative FX_E*
 * code on failure, with a thread-local message in fx_last_error().  Pointers
 * are plain host or device pointers as flagged by the *_mem arguments; no
 * torch or HIP types appear in the signatures (streams are passed as void*).
 */
#ifndef FX_INDEX_H
#define FX_INDEX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct FxIndex FxIndex;

/* element types (storage dtype of the index, or dtype of caller buffers) */
enum { FX_F32 = 0, FX_BF16 = 1, FX_F16 = 2 };
/* metrics, numbered as faiss MetricType */
enum { FX_METRIC_INNER_PRODUCT = 0, FX_METRIC_L2 = 1 };
/* where a caller buffer lives */
enum { FX_MEM_HOST = 0, FX_MEM_DEVICE = 1 };

/* error codes */
enum {
    FX_OK = 0,
    FX_E_ARG = -1,      /* invalid argument (faiss: AssertionError in the SWIG wrapper) */
    FX_E_HIP = -2,      /* HIP runtime failure / no device                            */
    FX_E_IO = -3,       /* file open / read / write / format error                     */
    FX_E_UNSUPPORTED = -4,
    FX_E_OOM = -5,
    FX_E_INTEGRITY = -6 /* a host-output search whose candidate lists held row ids outside
                           [0, ntotal): its top-k may be missing rows (never in a correct build) */
};

/* Largest k served by the fused scan path (per query).  fx_index_search
 * itself has no k cap, as faiss's IndexFlatL2::search (faiss_store.py:49,64
 * pass the caller's k): k <= 32 takes the fused scan's fixed candidate lists,
 * 32 < k <= FX_MAX_K a block top-K refine without cross-split pruning, and
 * k > FX_MAX_K the exact sort path (every (query, row) distance exactly,
 * one radix sort per query; HBM-bound, for the rare caller that asks).
 * fx_merge_shards takes any k the same way. */
#define FX_MAX_K 1024

const char* fx_last_error(void);
int fx_device_count(int* out);

/* faiss.IndexFlatL2(d) (faiss_store.py:29).  storage_dtype FX_F32 keeps the
 * reference's fp32 codes; FX_BF16 / FX_F16 halve HBM bytes per row.
 * device: HIP device ordinal the corpus is resident on. */
int fx_index_create(int d, int storage_dtype, int metric, int device, FxIndex** out);
void fx_index_free(FxIndex* index);

/* Opt-in row L2 normalisation applied at add time (cosine / IP mode; the
 * reference default is off: SURVEY.md section 8a a8). */
int fx_index_set_normalize(FxIndex* index, int on);
/* Run the index's kernels on `stream` (a hipStream_t; NULL = the index's own
 * stream, which is a blocking stream and therefore ordered with work on the
 * legacy null stream).  Lets a caller order index work after its own
 * producers.  Switching streams keeps the index's calls in order: the new
 * stream waits (on the device, no host sync) for the work already enqueued on
 * the previous one. */
int fx_index_set_stream(FxIndex* index, void* stream);
/* Per-index tuning option (name -> integer value).  Initial
 * values come from the FX_* environment variables, read once at index
 * creation; nothing on the search path reads the environment.  Names and
 * accepted values: "search_graph" 0/1 (default 0; 1: replay small host searches
 * as one hipGraph), "scan_place" -1/0/1, "scan_sx" >= 0, "reduce_cand" 0/1/2 (small
 * batches over many splits: 1, the default, one 16-wave workgroup refine per
 * query; 2 a separate merge of 16 splits' lists first; 0 neither),
 * "f32_split" 0/1, "centre" 0/1, "scan_pub" 0/1, "prune_rank" 0..32,
 * "compact_at" 0 (= 48) or 33..64 (list fill that triggers a compaction), "union_w"
 * 0/16/32/64 (splits per union-bound window), "union_defer" 0/1 (default 1:
 * a compaction's union bound fetched by LDS-DMA and bounded a tile later
 * instead of waited for), "union_inplace" -1..64 (at most this many lists
 * per compaction bounded by the union in place beyond the deferred ones; -1,
 * the default: 0 with union_defer, all without), "tight_at" -1/0 (off) or 33..64 (a list that took
 * entries and holds at least this many gets its threshold re-bounded between
 * compactions), "cold_bound" -1/0/1 (an empty list's first record tile bounds its
 * threshold from the per-lane group minima; -1, the default: on for corpus
 * splits of <= 256 tiles), "scan_v5" 0/1/2 (default 1: the 64-row-tile scan
 * for 16-bit rows of 512 / 768 / 1536 B where it adds no padding work; 2
 * wherever it has the shape), "refine_waves" 4/8/16,
 * "convoy" 0/1 (k_scan_v5 blocks start their split where its running blocks
 * are), "convoy_every" 1/2/4/8,
 * "host_spin" 0/1.  None changes results, only
 * speed.  Unknown name or out-of-range value: FX_E_ARG.  (The diagnostic
 * build libfx_index_diag.so adds test hooks -- "force_fallback",
 * "scan_dbg" -- that the product library does not have.) */
int fx_index_set_option(FxIndex* index, const char* name, int64_t value);
/* Global id of local row 0 (row-sharded multi-GPU: shard offset). */
int fx_index_set_id_offset(FxIndex* index, int64_t offset);

int fx_index_dim(const FxIndex* index, int* out);
int fx_index_ntotal(const FxIndex* index, int64_t* out);
int fx_index_storage_dtype(const FxIndex* index, int* out);
int fx_index_metric(const FxIndex* index, int* out);

/* Pre-size HBM for n rows (optional; add grows geometrically). */
int fx_index_reserve(FxIndex* index, int64_t n);

/* index.add(x) (faiss_store.py:46): append n rows of x[n][d] (row-major,
 * dtype x_dtype, host or device); rows get ids ntotal .. ntotal+n-1.
 * With FX_MEM_DEVICE it is stream-ordered (returns without waiting for the
 * device, unless the code matrix has to grow). */
int fx_index_add(FxIndex* index, int64_t n, const void* x, int x_dtype, int x_mem);

/* index.search(x, k) (faiss_store.py:64): q[nq][d] -> D[nq][k] (f32),
 * I[nq][k] (int64), out buffers caller-allocated on out_mem.  k >= 1 (any
 * k; past ntotal I = -1, D = +-FLT_MAX as faiss pads).  Blocks until results are in host memory when out_mem is
 * FX_MEM_HOST; with FX_MEM_DEVICE (queries and results on the device) it
 * is stream-ordered: it enqueues its work and returns without waiting for
 * the device (the re-scan and exact fallback for uncertified queries are
 * enqueued always and decided on the device).  A host-output search returns
 * through one packed device-to-host copy [D | I | counters] and enqueues
 * that chain only when the copy says a query was uncertified (then copies
 * again).  Workspace growth (first search of a larger shape) may
 * synchronise through hipMalloc / hipFree; so does a k > FX_MAX_K search
 * whose sort workspace exceeds 512 MiB (it is released after the call, a
 * smaller one is kept for the next). */
int fx_index_search(FxIndex* index, int64_t nq, const void* q, int q_dtype, int q_mem,
                    int k, float* D, int64_t* I, int out_mem);

/* Number of queries of the last search whose top-k could not be certified
 * from the scan's candidate margin and were re-scanned with a wide candidate
 * set (after an FX_MEM_DEVICE search this synchronises the index stream). */
int fx_index_last_fallbacks(FxIndex* index, int64_t* out);
/* Of those, the queries the re-scan could not certify either, re-ranked by
 * the exact fp64 scan of every row. */
int fx_index_last_exact_fallbacks(FxIndex* index, int64_t* out);
/* Candidate-list integrity of the last search: entries the exact re-rank
 * dropped because their row id (other than the empty-slot -1) lay outside
 * [0, ntotal).  Always 0 unless a scan list was corrupted; the dropped
 * entries are never gathered, so a non-zero count means the top-k may be
 * missing rows (faiss itself cannot return such a result: faiss_store.py:64).
 * A host-output search (FX_MEM_HOST) checks it itself and returns
 * FX_E_INTEGRITY; after a device-resident search the caller must read it
 * (this call synchronises the index stream). */
int fx_index_last_dropped_candidates(FxIndex* index, int64_t* out);

/* The scan plan of the last search (no faiss counterpart: which scan kernel
 * ran, for benchmarks and profiles): tile_rows 128 = k_scan_v4, 64 =
 * k_scan_v5; query_tile = queries per workgroup; splits = corpus splits per
 * query tile.  All 0 before the first search. */
int fx_index_last_scan_plan(FxIndex* index, int* tile_rows, int* query_tile, int* splits);

/* IndexFlatL2 reset (faiss_store.py:124-128). Keeps the HBM allocation. */
int fx_index_reset(FxIndex* index);

/* Copy rows [i0, i0+n) back as fp32 (host).  Used by write_index. */
int fx_index_reconstruct_n(FxIndex* index, int64_t i0, int64_t n, float* out);

/* faiss.write_index / faiss.read_index on the IxF2 format (faiss_store.py:
 * 91,106): fourcc "IxF2", i32 d, i64 ntotal, i64 1<<20, i64 1<<20,
 * u8 is_trained, i32 metric, i64 ntotal*d, f32 codes. */
int fx_index_write(FxIndex* index, const char* path);
int fx_index_read(const char* path, int storage_dtype, int device, FxIndex** out);

/* ---- row-sharded multi-GPU support (one process per GPU) --------------- */

/* Merge G per-shard result lists (device pointers, layout [G][nq][k], global
 * ids, each list ordered) into D_out/I_out [nq][k] under the index order
 * (L2: ascending; IP: descending; ties -> smaller id).  `stream` may be NULL.
 * k > FX_MAX_K merges at most 64 shards (FX_E_UNSUPPORTED beyond). */
int fx_merge_shards(int metric, int nshards, int64_t nq, int k, const float* D_in,
                    const int64_t* I_in, float* D_out, int64_t* I_out, int device, void* stream);

/* ---- synthetic corpora (bench / tests) -------------------------------- */

/* out[r][c] for rows [row0, row0+n) of the counter-based generator shared
 * with oracle/flat_l2.c (exact in fp32/bf16/fp16).  Device memory. */
int fx_synth_fill(void* out, int64_t row0, int64_t n, int d, int dtype, uint64_t seed,
                  int device, void* stream);

/* ---- kernel timing for the roofline report ---------------------------- */

/* When enabled, every search records HIP events around its scan kernel
 * (on the stream it is launched on).  _read synchronises and returns the
 * summed scan-kernel milliseconds and the number of launches since reset. */
int fx_index_profile(FxIndex* index, int enable);
int fx_index_profile_read(FxIndex* index, double* scan_ms, double* merge_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* FX_INDEX_H */
