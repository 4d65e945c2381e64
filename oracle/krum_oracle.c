/*
 * oracle/krum_oracle.c -- CPU restatement of Biscotti's Multi-Krum arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in biscotti_amd/ links, loads or calls
 * this file.  It is used by tests/ (as the parity checker), by
 * __graft_entry__.smoke() (as the checker) and by bench.py's cpu_baseline leg
 * (timed as the "port" CPU baseline).  The product path is the HIP library
 * biscotti_amd/libbk.so and fails loudly when that library is missing.
 *
 * What it restates (reference @ /root/reference, DistributedML/Biscotti v1):
 *   krum(deltas, clip)            ML/code/logistic_validator.py:36-49
 *                                 (== ML/Pytorch/client_obj.py:114-127)
 *   get_krum_scores(X, groupsize) ML/code/logistic_validator.py:54-65
 *                                 (== ML/Pytorch/client_obj.py:132-143)
 *   masked mean (commented out)   ML/code/logistic_validator.py:51
 *   clip = int(0.5 * n)           DistSys/krum.go:110 (NumAdversaries, main.go:783)
 *
 * Semantics kept exactly:
 *   sq[i]      = np.sum(X**2, axis=1)   -> numpy pairwise summation (restated
 *                                          in np_pairwise_sum below, bit-exact)
 *   D[i][j]    = (sq[i] + sq[j]) - 2*dot(x_i, x_j)   (numpy evaluation order)
 *   score[i]   = np.sum(np.sort(D[i])[1:groupsize-1])  (full ascending sort with
 *                NaN last, drop rank 0, numpy pairwise sum of ranks 1..k,
 *                k = groupsize-2 = n-f-2, empty slice -> 0.0)
 *   selection  = the m = n-f smallest scores (np.argpartition(scores, m)[:m]);
 *                NaN scores order last; ties at the boundary -> lower index
 *                first (numpy's introselect is implementation-defined there;
 *                documented in DESIGN.md).  Returned ascending (a set).
 *   mean       = sum of the selected rows (ascending index order) / m
 *   f < 1 or f >= n -> error (numpy raises ValueError for f = 0 at :45).
 *
 * The only deliberate difference from the reference is the dot product:
 * numpy calls BLAS dsyrk/dgemm whose blocking/rounding is library-specific;
 * here it is a plain fp64 FMA dot over k-blocks.  Scores therefore agree with
 * the reference to rounding, and the selected set is pinned against golden
 * vectors produced by the reference itself (tests/golden/gen_goldens.py).
 *
 * The synthetic-input generator (oracle_synth_*) is an independent restatement
 * of the spec in DESIGN.md "Synthetic inputs" and must agree bit-for-bit with
 * the GPU generator in biscotti_amd/csrc/bk_synth.h and with the numpy
 * generator in tests/golden/synth_np.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_OK 0
#define OR_EINVAL (-1)
#define OR_ENOMEM (-2)

/* ------------------------------------------------------------------------ */
/* numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src,        */
/* pairwise_sum_DOUBLE): <8 sequential, <=128 eight accumulators, else split */
/* ------------------------------------------------------------------------ */
static double np_pairwise_sum(const double *a, int64_t n, int64_t stride)
{
    if (n < 8) {
        double res = -0.0;
        for (int64_t i = 0; i < n; i++) res += a[i * stride];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j * stride];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[(i + j) * stride];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i * stride];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise_sum(a, n2, stride) + np_pairwise_sum(a + n2 * stride, n - n2, stride);
    }
}

/* numpy sort order for float64: ascending, NaN last. */
static int cmp_np_double(const void *pa, const void *pb)
{
    double a = *(const double *)pa, b = *(const double *)pb;
    int na = isnan(a), nb = isnan(b);
    if (na || nb) return na - nb;
    return (a < b) ? -1 : (a > b) ? 1 : 0;
}

/* Selection order: score ascending, NaN last, ties by index. */
typedef struct { double s; int64_t i; } scored_t;
static int cmp_scored(const void *pa, const void *pb)
{
    const scored_t *a = (const scored_t *)pa, *b = (const scored_t *)pb;
    int na = isnan(a->s), nb = isnan(b->s);
    if (na != nb) return na - nb;
    if (!na) {
        if (a->s < b->s) return -1;
        if (a->s > b->s) return 1;
    }
    return (a->i < b->i) ? -1 : (a->i > b->i) ? 1 : 0;
}

static int cmp_i64(const void *pa, const void *pb)
{
    int64_t a = *(const int64_t *)pa, b = *(const int64_t *)pb;
    return (a < b) ? -1 : (a > b) ? 1 : 0;
}

int oracle_check_args(int64_t n, int64_t d, int64_t f)
{
    if (n < 1 || d < 1 || f < 1 || f >= n) return OR_EINVAL;
    return OR_OK;
}

/* ------------------------------------------------------------------------ */
/* Gram / distance matrix.  X is row-major n x ld, fp64 or fp32 (widened).   */
/* ------------------------------------------------------------------------ */
#define KB 512

static inline double ld_elem(const void *X, int is_f32, int64_t ld, int64_t i, int64_t k)
{
    return is_f32 ? (double)((const float *)X)[i * ld + k] : ((const double *)X)[i * ld + k];
}

/* G (upper triangle incl. diagonal, row-major n x n) += X[:,k0:k1] X[:,k0:k1]^T */
static void gram_block(const double *Xb, int64_t n, int64_t kw, double *G)
{
    /* Xb: n x kw contiguous copy of the column block. 4x4 register tiles. */
    int64_t nt = (n + 3) / 4;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t ti = 0; ti < nt; ti++) {
        int64_t i0 = ti * 4;
        for (int64_t j0 = i0; j0 < n; j0 += 4) {
            double acc[4][4] = {{0}};
            const double *a[4], *b[4];
            for (int p = 0; p < 4; p++) {
                a[p] = Xb + (i0 + p < n ? i0 + p : n - 1) * kw;
                b[p] = Xb + (j0 + p < n ? j0 + p : n - 1) * kw;
            }
            for (int64_t k = 0; k < kw; k++) {
                double av0 = a[0][k], av1 = a[1][k], av2 = a[2][k], av3 = a[3][k];
                double bv0 = b[0][k], bv1 = b[1][k], bv2 = b[2][k], bv3 = b[3][k];
                acc[0][0] = fma(av0, bv0, acc[0][0]); acc[0][1] = fma(av0, bv1, acc[0][1]);
                acc[0][2] = fma(av0, bv2, acc[0][2]); acc[0][3] = fma(av0, bv3, acc[0][3]);
                acc[1][0] = fma(av1, bv0, acc[1][0]); acc[1][1] = fma(av1, bv1, acc[1][1]);
                acc[1][2] = fma(av1, bv2, acc[1][2]); acc[1][3] = fma(av1, bv3, acc[1][3]);
                acc[2][0] = fma(av2, bv0, acc[2][0]); acc[2][1] = fma(av2, bv1, acc[2][1]);
                acc[2][2] = fma(av2, bv2, acc[2][2]); acc[2][3] = fma(av2, bv3, acc[2][3]);
                acc[3][0] = fma(av3, bv0, acc[3][0]); acc[3][1] = fma(av3, bv1, acc[3][1]);
                acc[3][2] = fma(av3, bv2, acc[3][2]); acc[3][3] = fma(av3, bv3, acc[3][3]);
            }
            for (int p = 0; p < 4; p++)
                for (int q = 0; q < 4; q++) {
                    int64_t i = i0 + p, j = j0 + q;
                    if (i < n && j < n && i <= j) G[i * n + j] += acc[p][q];
                }
        }
    }
}

/* Full symmetric Gram X X^T (fp64 result). Returns 0 or OR_ENOMEM. */
int oracle_gram(const void *X, int is_f32, int64_t n, int64_t d, int64_t ld, double *G)
{
    memset(G, 0, sizeof(double) * n * n);
    double *Xb = (double *)malloc(sizeof(double) * n * KB);
    if (!Xb) return OR_ENOMEM;
    for (int64_t k0 = 0; k0 < d; k0 += KB) {
        int64_t kw = (d - k0 < KB) ? d - k0 : KB;
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; i++)
            for (int64_t k = 0; k < kw; k++) Xb[i * kw + k] = ld_elem(X, is_f32, ld, i, k0 + k);
        gram_block(Xb, n, kw, G);
    }
    free(Xb);
    for (int64_t i = 0; i < n; i++)
        for (int64_t j = 0; j < i; j++) G[i * n + j] = G[j * n + i];
    return OR_OK;
}

/* np.sum(X**2, axis=1): square elementwise (rounded), then pairwise sum. */
int oracle_sqnorms(const void *X, int is_f32, int64_t n, int64_t d, int64_t ld, double *sq)
{
    int err = OR_OK;
#pragma omp parallel
    {
        double *row = (double *)malloc(sizeof(double) * d);
        if (!row) {
#pragma omp atomic write
            err = OR_ENOMEM;
        } else {
#pragma omp for schedule(static)
            for (int64_t i = 0; i < n; i++) {
                for (int64_t k = 0; k < d; k++) {
                    double v = ld_elem(X, is_f32, ld, i, k);
                    row[k] = v * v;
                }
                sq[i] = np_pairwise_sum(row, d, 1);
            }
            free(row);
        }
    }
    return err;
}

/* scores from a precomputed distance row source: D[i][j] = (sq_i+sq_j) - 2G_ij */
static void scores_from_gram(const double *G, const double *sq, int64_t n, int64_t groupsize,
                             double *scores, double *Dout)
{
    /* slice [1:groupsize-1] with python semantics (negative stop wraps) */
    int64_t start = 1, stop = groupsize - 1;
    if (stop < 0) stop += n;
    if (stop < 0) stop = 0;
    if (stop > n) stop = n;
    if (start > n) start = n;
    int64_t cnt = stop > start ? stop - start : 0;
#pragma omp parallel
    {
        double *row = (double *)malloc(sizeof(double) * n);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; i++) {
            for (int64_t j = 0; j < n; j++) {
                double t = sq[i] + sq[j];
                double g2 = 2.0 * G[i * n + j];
                row[j] = t - g2;
            }
            if (Dout) memcpy(Dout + i * n, row, sizeof(double) * n);
            qsort(row, (size_t)n, sizeof(double), cmp_np_double);
            scores[i] = cnt > 0 ? np_pairwise_sum(row + start, cnt, 1) : 0.0;
        }
        free(row);
    }
}

/* get_krum_scores(X, groupsize) restated.  D (n x n) optional output. */
int oracle_krum_scores(const void *X, int is_f32, int64_t n, int64_t d, int64_t ld,
                       int64_t groupsize, double *scores, double *Dout)
{
    double *G = (double *)malloc(sizeof(double) * n * n);
    double *sq = (double *)malloc(sizeof(double) * n);
    if (!G || !sq) { free(G); free(sq); return OR_ENOMEM; }
    int e = oracle_gram(X, is_f32, n, d, ld, G);
    if (!e) e = oracle_sqnorms(X, is_f32, n, d, ld, sq);
    if (!e) scores_from_gram(G, sq, n, groupsize, scores, Dout);
    free(G); free(sq);
    return e;
}

/* Selection of the m smallest scores; sel_out ascending. Returns m. */
int64_t oracle_select(const double *scores, int64_t n, int64_t m, int64_t *sel_out)
{
    scored_t *v = (scored_t *)malloc(sizeof(scored_t) * n);
    if (!v) return OR_ENOMEM;
    for (int64_t i = 0; i < n; i++) { v[i].s = scores[i]; v[i].i = i; }
    qsort(v, (size_t)n, sizeof(scored_t), cmp_scored);
    for (int64_t r = 0; r < m; r++) sel_out[r] = v[r].i;
    free(v);
    qsort(sel_out, (size_t)m, sizeof(int64_t), cmp_i64);
    return m;
}

/* mean of selected rows, ascending index order, sequential per column, / m */
void oracle_mean(const void *X, int is_f32, int64_t d, int64_t ld, const int64_t *sel, int64_t m,
                 double *mean)
{
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < d; k++) {
        double s = 0.0;
        for (int64_t r = 0; r < m; r++) s += ld_elem(X, is_f32, ld, sel[r], k);
        mean[k] = s / (double)m;
    }
}

/* krum(deltas, clip) + masked mean.  sel_out: m entries ascending.
 * scores (n) and mean (d) may be NULL. Returns m (>0) or error (<0). */
int64_t oracle_krum(const void *X, int is_f32, int64_t n, int64_t d, int64_t ld, int64_t f,
                    int64_t *sel_out, double *scores, double *mean)
{
    if (oracle_check_args(n, d, f)) return OR_EINVAL;
    int64_t m = n - f;
    double *sc = scores ? scores : (double *)malloc(sizeof(double) * n);
    if (!sc) return OR_ENOMEM;
    int e = oracle_krum_scores(X, is_f32, n, d, ld, m, sc, NULL);
    if (e) { if (!scores) free(sc); return e; }
    int64_t r = oracle_select(sc, n, m, sel_out);
    if (!scores) free(sc);
    if (r < 0) return r;
    if (mean) oracle_mean(X, is_f32, d, ld, sel_out, m, mean);
    return m;
}

int oracle_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void oracle_set_threads(int t)
{
#ifdef _OPENMP
    if (t > 0) omp_set_num_threads(t);
#else
    (void)t;
#endif
}

/* ------------------------------------------------------------------------ */
/* Synthetic inputs (spec: DESIGN.md "Synthetic inputs").                    */
/* ------------------------------------------------------------------------ */
static inline uint64_t sm64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
static inline uint64_t stream_base(uint64_t seed, uint64_t stream)
{
    return sm64(sm64(seed) ^ (stream * 0xD1B54A32D192ED03ULL));
}
static inline double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }
static inline double gauss(uint64_t base, uint64_t idx)
{
    uint64_t c = base + 4ULL * idx;
    double u0 = u01(sm64(c)), u1 = u01(sm64(c + 1)), u2 = u01(sm64(c + 2)), u3 = u01(sm64(c + 3));
    double s01 = u0 + u1;
    double s23 = u2 + u3;
    double s = s01 + s23;
    double t = s - 2.0;
    return t * 1.7320508075688772;
}

/* Fisher-Yates: position p holds original row perm[p]. */
void oracle_synth_perm(uint64_t seed, int64_t n, int64_t *perm)
{
    uint64_t b = stream_base(seed, 3);
    for (int64_t i = 0; i < n; i++) perm[i] = i;
    for (int64_t i = n - 1; i >= 1; i--) {
        int64_t j = (int64_t)(sm64(b + (uint64_t)i) % (uint64_t)(i + 1));
        int64_t t = perm[i]; perm[i] = perm[j]; perm[j] = t;
    }
}

#define SYNTH_FP32ROUND 1

/* Fill rows [0,n) x columns [c0, c0+dl) of the n x d_total synthetic matrix
 * into X (row-major, leading dimension ld, fp64 or fp32). */
void oracle_synth_fill(void *X, int is_f32, int64_t n, int64_t dl, int64_t ld, int64_t c0,
                       int64_t d_total, uint64_t seed, int64_t nbyz, double mu_scale,
                       double byz_scale, double sigma, int flags)
{
    int64_t *perm = (int64_t *)malloc(sizeof(int64_t) * n);
    oracle_synth_perm(seed, n, perm);
    uint64_t b0 = stream_base(seed, 0), b1 = stream_base(seed, 1), b2 = stream_base(seed, 2),
             b4 = stream_base(seed, 4);
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < n; p++) {
        int64_t r = perm[p];
        int byz = r >= n - nbyz;
        for (int64_t k = 0; k < dl; k++) {
            int64_t c = c0 + k;
            double mu = mu_scale * gauss(b0, (uint64_t)c);
            double base = mu;
            if (byz) {
                double sh = byz_scale * gauss(b1, (uint64_t)c);
                base = mu + sh;
            }
            uint64_t e = (uint64_t)r * (uint64_t)d_total + (uint64_t)c;
            double nz = sigma * gauss(b2, e);
            double x = base + nz;
            if (flags & SYNTH_FP32ROUND) {
                double w = (double)(float)x;
                double nz2 = 1e-6 * gauss(b4, e);
                x = w + nz2;
            }
            if (is_f32) ((float *)X)[p * ld + k] = (float)x;
            else ((double *)X)[p * ld + k] = x;
        }
    }
    free(perm);
}
