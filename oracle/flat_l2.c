/*
 * oracle/flat_l2.c -- CPU restatement of FAISS IndexFlatL2 search.
 * TEST INFRASTRUCTURE ONLY: linked by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, always as the checker / the timed CPU
 * baseline, never by the product path (rag-faiss-embedding_amd/).
 *
 * The reference calls faiss.IndexFlatL2.search (faiss_store.py:64,
 * rag_datastore_manager.py:218); faiss-cpu (requirements.txt:13, unpinned) is
 * not vendored and not installed here, so this file restates its published
 * algorithm (faiss/utils/distances.cpp::knn_L2sqr):
 *
 *   fxo_knn_exact*   exact sum_t (x_t - y_t)^2 in fp64, rounded once to fp32,
 *                    per-query max-heap of size k, ties -> smaller id,
 *                    missing slots I=-1 / D=FLT_MAX.  The parity key.
 *   fxo_knn_blas     the FAISS BLAS path for nq >= 20: |y|^2 once, blocks of
 *                    4096 queries x 1024 rows, fp32 ip = x.y, D = |x|^2 +
 *                    |y|^2 - 2 ip clamped at 0, same heap.  The timed
 *                    "CPU FAISS" baseline (a port, not faiss itself).
 *   fxo_synth_fill   the counter-based synthetic corpus (oracle/flat_l2.py
 *                    synth(); identical integer definition on the GPU).
 *
 * Build: oracle/Makefile -> oracle/_build/libfx_oracle.so (OpenMP).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define GOLDEN 0x9E3779B97F4A7C15ULL

static inline float synth_val(uint64_t seed, uint64_t row, uint64_t d, uint64_t col) {
    uint64_t z = seed * GOLDEN + row * d + col;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    int b0 = (int)(z & 0xFF), b1 = (int)((z >> 8) & 0xFF);
    return (float)(b0 + b1 - 255) / 64.0f;
}

void fxo_synth_fill(uint64_t seed, int64_t row0, int64_t nrows, int d, float* out, int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nrows; ++r)
        for (int c = 0; c < d; ++c)
            out[r * (int64_t)d + c] = synth_val(seed, (uint64_t)(row0 + r), (uint64_t)d, (uint64_t)c);
}

/* ---- max-heap of (dist, id) with FAISS CMax order: larger dist on top,
 *      among equal dists the larger id is "larger" (so it is evicted first). */
static inline int heap_gt(float d1, int64_t i1, float d2, int64_t i2) {
    return d1 > d2 || (d1 == d2 && i1 > i2);
}

static void heap_push_replace(float* hd, int64_t* hi, int k, float d, int64_t id) {
    /* replace the top (largest) then sift down */
    int i = 0;
    for (;;) {
        int l = 2 * i + 1, r = l + 1, m = i;
        float md = d; int64_t mi = id;
        if (l < k && heap_gt(hd[l], hi[l], md, mi)) { m = l; md = hd[l]; mi = hi[l]; }
        if (r < k && heap_gt(hd[r], hi[r], md, mi)) { m = r; }
        if (m == i) break;
        hd[i] = hd[m]; hi[i] = hi[m];
        i = m;
    }
    hd[i] = d; hi[i] = id;
}

static inline void heap_offer(float* hd, int64_t* hi, int k, float d, int64_t id) {
    if (heap_gt(hd[0], hi[0], d, id)) heap_push_replace(hd, hi, k, d, id);
}

static void heap_init(float* hd, int64_t* hi, int k) {
    for (int j = 0; j < k; ++j) { hd[j] = FLT_MAX; hi[j] = -1; }
}

/* Sort the heap ascending by (d, id); empty slots (-1, FLT_MAX) go last. */
static void heap_finish(float* hd, int64_t* hi, int k) {
    for (int a = 1; a < k; ++a) {
        float d = hd[a]; int64_t id = hi[a]; int b = a - 1;
        while (b >= 0) {
            int gt;
            if (hi[b] < 0) gt = (id >= 0);
            else if (id < 0) gt = 0;
            else gt = heap_gt(hd[b], hi[b], d, id);
            if (!gt) break;
            hd[b + 1] = hd[b]; hi[b + 1] = hi[b]; --b;
        }
        hd[b + 1] = d; hi[b + 1] = id;
    }
}

static inline double l2_exact64(const float* x, const float* y, int d) {
    double s = 0.0;
    for (int t = 0; t < d; ++t) { double e = (double)x[t] - (double)y[t]; s += e * e; }
    return s;
}

/* Exact k-NN of xq[nq][d] against xb[nb][d]. */
void fxo_knn_exact(const float* xq, int64_t nq, const float* xb, int64_t nb, int d, int k,
                   float* D, int64_t* I, int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t q = 0; q < nq; ++q) {
        float* hd = D + q * k; int64_t* hi = I + q * k;
        heap_init(hd, hi, k);
        for (int64_t j = 0; j < nb; ++j) {
            float dist = (float)l2_exact64(xq + q * d, xb + j * d, d);
            heap_offer(hd, hi, k, dist, j);
        }
        heap_finish(hd, hi, k);
    }
}

/* Streaming exact k-NN against the synthetic corpus rows [0, nb) of seed
 * `cseed` (generated on the fly, never materialised): used to check GPU
 * results at full BASELINE sizes (1e7..1e8 rows) on a query subset.
 *
 * The generator's values are v = n / 64 with n = b0 + b1 - 255 an integer in
 * [-255, 255].  When every query value is on that grid too (the synthetic
 * queries of the tests and the bench), 4096 * sum_t (x_t - y_t)^2 is the
 * integer |nx|^2 + |ny|^2 - 2 nx.ny (< 2^31 for d <= 8192), so the exact sum
 * -- which the fp64 restatement below also computes exactly, every partial
 * sum of such terms being representable -- is obtained in integer arithmetic
 * (16-bit products, 32-bit sums: vectorised) and rounded to fp32 once, the
 * same value bit for bit (tests/test_oracle.py checks the two paths agree).
 * Queries off the grid take the fp64 path. */
static int on_grid(const float* xq, int64_t n, int16_t* out) {
    for (int64_t i = 0; i < n; ++i) {
        const float v = xq[i] * 64.0f;
        if (!(v == floorf(v)) || v < -255.0f || v > 255.0f) return 0;
        out[i] = (int16_t)v;
    }
    return 1;
}

static inline int32_t dot_i16(const int16_t* x, const int16_t* y, int d) {
    int32_t s = 0;
    for (int t = 0; t < d; ++t) s += (int32_t)x[t] * (int32_t)y[t];
    return s;
}

/* dots of 4 queries x 4 rows (d a multiple of 16 on the AVX2 path: the
 * callers pad rows and queries with zeros to d16) */
#if defined(__AVX2__)
#include <immintrin.h>
static inline int32_t hsum8(__m256i v) {
    __m128i s = _mm_add_epi32(_mm256_castsi256_si128(v), _mm256_extracti128_si256(v, 1));
    s = _mm_add_epi32(s, _mm_shuffle_epi32(s, 0x4E));
    s = _mm_add_epi32(s, _mm_shuffle_epi32(s, 0xB1));
    return _mm_cvtsi128_si32(s);
}
static inline void dot_i16_2x4(const int16_t* x0, const int16_t* x1, const int16_t* y0, int d16, int32_t out[2][4]) {
    __m256i a[2][4];
    for (int u = 0; u < 2; ++u)
        for (int v = 0; v < 4; ++v) a[u][v] = _mm256_setzero_si256();
    for (int t = 0; t < d16; t += 16) {
        const __m256i q0 = _mm256_loadu_si256((const __m256i*)(x0 + t));
        const __m256i q1 = _mm256_loadu_si256((const __m256i*)(x1 + t));
        for (int v = 0; v < 4; ++v) {
            const __m256i r = _mm256_loadu_si256((const __m256i*)(y0 + (size_t)v * d16 + t));
            a[0][v] = _mm256_add_epi32(a[0][v], _mm256_madd_epi16(q0, r));
            a[1][v] = _mm256_add_epi32(a[1][v], _mm256_madd_epi16(q1, r));
        }
    }
    for (int u = 0; u < 2; ++u)
        for (int v = 0; v < 4; ++v) out[u][v] = hsum8(a[u][v]);
}
#else
static inline void dot_i16_2x4(const int16_t* x0, const int16_t* x1, const int16_t* y0, int d16, int32_t out[2][4]) {
    for (int v = 0; v < 4; ++v) {
        out[0][v] = dot_i16(x0, y0 + (size_t)v * d16, d16);
        out[1][v] = dot_i16(x1, y0 + (size_t)v * d16, d16);
    }
}
#endif

void fxo_knn_exact_synth(uint64_t cseed, int64_t nb, int d, const float* xq, int64_t nq, int k,
                         float* D, int64_t* I, int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
    int nt = 1;
#pragma omp parallel
    {
#pragma omp single
        nt = omp_get_num_threads();
    }
    const int d16 = (d + 15) / 16 * 16;  /* zero-padded stride of the integer rows */
    int16_t* qraw = (int16_t*)malloc(sizeof(int16_t) * (size_t)(nq > 0 ? nq : 1) * d);
    int16_t* qi = (int16_t*)calloc((size_t)(nq > 0 ? nq : 1) * d16, sizeof(int16_t));
    int64_t* qn = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nq > 0 ? nq : 1));
    const int grid = d <= 8192 && on_grid(xq, nq * (int64_t)d, qraw);
    if (grid)
        for (int64_t q = 0; q < nq; ++q) {
            memcpy(qi + q * d16, qraw + q * d, sizeof(int16_t) * d);
            qn[q] = dot_i16(qi + q * d16, qi + q * d16, d16);
        }
    free(qraw);
    /* per-thread heaps over a row partition, merged at the end */
    float* hdall = (float*)malloc(sizeof(float) * (size_t)nt * nq * k);
    int64_t* hiall = (int64_t*)malloc(sizeof(int64_t) * (size_t)nt * nq * k);
#pragma omp parallel
    {
        int t = omp_get_thread_num();
        float* hd = hdall + (size_t)t * nq * k;
        int64_t* hi = hiall + (size_t)t * nq * k;
        for (int64_t q = 0; q < nq; ++q) heap_init(hd + q * k, hi + q * k, k);
        float* row = (float*)malloc(sizeof(float) * d);
        /* grid path: blocks of RB rows (generated once) x 4 queries x 4 rows */
        enum { RB = 64 };
        int16_t* rowi = (int16_t*)calloc((size_t)RB * d16, sizeof(int16_t));
        int64_t yn[RB];
        int64_t r0 = nb * t / nt, r1 = nb * (t + 1) / nt;
        for (int64_t j0 = r0; grid && j0 < r1; j0 += RB) {
            const int nr = (int)(r1 - j0 < RB ? r1 - j0 : RB);
            for (int r = 0; r < RB; ++r) {  /* rows past the block's end: zero (never offered) */
                int16_t* y = rowi + (size_t)r * d16;
                for (int c = 0; c < d; ++c)
                    y[c] = r < nr ? (int16_t)(synth_val(cseed, (uint64_t)(j0 + r), (uint64_t)d, (uint64_t)c) * 64.0f)
                                  : 0;
                yn[r] = dot_i16(y, y, d16);
            }
            for (int64_t q = 0; q < nq; q += 2) {
                const int16_t* x0 = qi + (size_t)q * d16;
                const int16_t* x1 = qi + (size_t)(q + 1 < nq ? q + 1 : q) * d16;
                for (int r = 0; r < nr; r += 4) {
                    int32_t dots[2][4];
                    dot_i16_2x4(x0, x1, rowi + (size_t)r * d16, d16, dots);
                    for (int u = 0; u < 2 && q + u < nq; ++u)
                        for (int v = 0; v < 4 && r + v < nr; ++v) {
                            const int64_t e = qn[q + u] + yn[r + v] - 2 * (int64_t)dots[u][v];
                            heap_offer(hd + (q + u) * k, hi + (q + u) * k, k, (float)((double)e / 4096.0),
                                       j0 + r + v);
                        }
                }
            }
        }
        for (int64_t j = r0; !grid && j < r1; ++j) {
            for (int c = 0; c < d; ++c) row[c] = synth_val(cseed, (uint64_t)j, (uint64_t)d, (uint64_t)c);
            {
                for (int64_t q = 0; q < nq; ++q) {
                    float dist = (float)l2_exact64(xq + q * d, row, d);
                    heap_offer(hd + q * k, hi + q * k, k, dist, j);
                }
            }
        }
        free(row);
        free(rowi);
    }
    for (int64_t q = 0; q < nq; ++q) {
        float* od = D + q * k; int64_t* oi = I + q * k;
        heap_init(od, oi, k);
        for (int t = 0; t < nt; ++t)
            for (int j = 0; j < k; ++j) {
                int64_t id = hiall[((size_t)t * nq + q) * k + j];
                if (id >= 0) heap_offer(od, oi, k, hdall[((size_t)t * nq + q) * k + j], id);
            }
        heap_finish(od, oi, k);
    }
    free(hdall); free(hiall); free(qi); free(qn);
}

/* The same search on the fp64 path only (the grid shortcut off): the check of
 * fxo_knn_exact_synth's integer path (tests/test_oracle.py). */
void fxo_knn_exact_synth_f64(uint64_t cseed, int64_t nb, int d, const float* xq, int64_t nq, int k,
                             float* D, int64_t* I, int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t q = 0; q < nq; ++q) {
        float* hd = D + q * k; int64_t* hi = I + q * k;
        float* row = (float*)malloc(sizeof(float) * d);
        heap_init(hd, hi, k);
        for (int64_t j = 0; j < nb; ++j) {
            for (int c = 0; c < d; ++c) row[c] = synth_val(cseed, (uint64_t)j, (uint64_t)d, (uint64_t)c);
            heap_offer(hd, hi, k, (float)l2_exact64(xq + q * d, row, d), j);
        }
        heap_finish(hd, hi, k);
        free(row);
    }
}

/* ---- FAISS BLAS-path restatement (the timed CPU baseline) ---------------- */

#define QB 4096   /* faiss distance_compute_blas_query_bs */
#define DB 1024   /* faiss distance_compute_blas_database_bs */

/* ip[i][j] = x_i . y_j for a block, register-blocked 4 queries x 4 rows so the
 * compiler emits FMA vector code (the inner t-loop is contiguous in both). */
static void ip_block(const float* x, int nx, const float* y, int ny, int d, float* ip) {
    int i = 0;
    for (; i + 4 <= nx; i += 4) {
        const float* x0 = x + (size_t)i * d; const float* x1 = x0 + d;
        const float* x2 = x1 + d; const float* x3 = x2 + d;
        int j = 0;
        for (; j + 4 <= ny; j += 4) {
            const float* y0 = y + (size_t)j * d; const float* y1 = y0 + d;
            const float* y2 = y1 + d; const float* y3 = y2 + d;
            float s[16];
            float a00 = 0, a01 = 0, a02 = 0, a03 = 0, a10 = 0, a11 = 0, a12 = 0, a13 = 0;
            float a20 = 0, a21 = 0, a22 = 0, a23 = 0, a30 = 0, a31 = 0, a32 = 0, a33 = 0;
#pragma omp simd reduction(+:a00,a01,a02,a03,a10,a11,a12,a13,a20,a21,a22,a23,a30,a31,a32,a33)
            for (int t = 0; t < d; ++t) {
                float q0 = x0[t], q1 = x1[t], q2 = x2[t], q3 = x3[t];
                float b0 = y0[t], b1 = y1[t], b2 = y2[t], b3 = y3[t];
                a00 += q0 * b0; a01 += q0 * b1; a02 += q0 * b2; a03 += q0 * b3;
                a10 += q1 * b0; a11 += q1 * b1; a12 += q1 * b2; a13 += q1 * b3;
                a20 += q2 * b0; a21 += q2 * b1; a22 += q2 * b2; a23 += q2 * b3;
                a30 += q3 * b0; a31 += q3 * b1; a32 += q3 * b2; a33 += q3 * b3;
            }
            s[0] = a00; s[1] = a01; s[2] = a02; s[3] = a03; s[4] = a10; s[5] = a11; s[6] = a12; s[7] = a13;
            s[8] = a20; s[9] = a21; s[10] = a22; s[11] = a23; s[12] = a30; s[13] = a31; s[14] = a32; s[15] = a33;
            for (int a = 0; a < 4; ++a)
                for (int b = 0; b < 4; ++b) ip[(size_t)(i + a) * ny + j + b] = s[a * 4 + b];
        }
        for (; j < ny; ++j)
            for (int a = 0; a < 4; ++a) {
                float acc = 0; const float* xa = x + (size_t)(i + a) * d; const float* yj = y + (size_t)j * d;
                for (int t = 0; t < d; ++t) acc += xa[t] * yj[t];
                ip[(size_t)(i + a) * ny + j] = acc;
            }
    }
    for (; i < nx; ++i)
        for (int j = 0; j < ny; ++j) {
            float acc = 0; const float* xa = x + (size_t)i * d; const float* yj = y + (size_t)j * d;
            for (int t = 0; t < d; ++t) acc += xa[t] * yj[t];
            ip[(size_t)i * ny + j] = acc;
        }
}

void fxo_knn_blas(const float* xq, int64_t nq, const float* xb, int64_t nb, int d, int k,
                  float* D, int64_t* I, int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
    float* xn = (float*)malloc(sizeof(float) * (size_t)nq);
    float* yn = (float*)malloc(sizeof(float) * (size_t)nb);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nq; ++i) {
        float s = 0; for (int t = 0; t < d; ++t) s += xq[i * d + t] * xq[i * d + t]; xn[i] = s;
    }
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < nb; ++j) {
        float s = 0; for (int t = 0; t < d; ++t) s += xb[j * d + t] * xb[j * d + t]; yn[j] = s;
    }
    for (int64_t q = 0; q < nq; ++q) heap_init(D + q * k, I + q * k, k);
    for (int64_t i0 = 0; i0 < nq; i0 += QB) {
        int64_t i1 = i0 + QB < nq ? i0 + QB : nq;
        int nx = (int)(i1 - i0);
        /* parallelise over query sub-blocks of 16 so each thread owns its heaps */
#pragma omp parallel
        {
            float* ip = (float*)malloc(sizeof(float) * 16 * DB);
#pragma omp for schedule(dynamic, 1)
            for (int qs = 0; qs < nx; qs += 16) {
                int nqs = nx - qs < 16 ? nx - qs : 16;
                const float* xs = xq + (size_t)(i0 + qs) * d;
                for (int64_t j0 = 0; j0 < nb; j0 += DB) {
                    int ny = (int)((j0 + DB < nb ? j0 + DB : nb) - j0);
                    ip_block(xs, nqs, xb + (size_t)j0 * d, ny, d, ip);
                    for (int a = 0; a < nqs; ++a) {
                        int64_t q = i0 + qs + a;
                        float* hd = D + q * k; int64_t* hi = I + q * k;
                        float xa = xn[q];
                        for (int b = 0; b < ny; ++b) {
                            float dist = xa + yn[j0 + b] - 2.0f * ip[(size_t)a * ny + b];
                            if (dist < 0) dist = 0;
                            if (dist < hd[0] || (dist == hd[0] && j0 + b < hi[0]))
                                heap_push_replace(hd, hi, k, dist, j0 + b);
                        }
                    }
                }
            }
            free(ip);
        }
    }
    for (int64_t q = 0; q < nq; ++q) heap_finish(D + q * k, I + q * k, k);
    free(xn); free(yn);
}

int fxo_max_threads(void) { return omp_get_max_threads(); }
