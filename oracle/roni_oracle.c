/*
 * oracle/roni_oracle.c -- CPU restatement of Biscotti's RONI verifier
 * (SURVEY.md §8(f) row 4).  TEST INFRASTRUCTURE ONLY (see krum_oracle.c).
 *
 *   roni(ww, delta)   ML/code/logistic_validator.py:22-33
 *       yhat  = np.sign(np.dot(Xvalid, ww))
 *       yhat2 = np.sign(np.dot(Xvalid, ww + delta))       (ww + delta rounded first)
 *       g_err   = np.sum(yhat  != yvalid) / float(yvalid.size)
 *       new_err = np.sum(yhat2 != yvalid) / float(yvalid.size)
 *       return new_err - g_err
 *   np.sign: +1 / -1 / 0 (for +-0) / NaN; NaN != label is True.
 *
 * Pinned against the reference itself: tests/golden/gen_roni_goldens.py runs
 * the reference roni on repo inputs (tests/test_roni_oracle.py).  The dot is a
 * sequential fp64 FMA chain; numpy's BLAS order is library-specific, so only
 * dots within rounding of zero could flip a sign (none in the goldens).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

static int64_t roni_errors(const double *Xv, int64_t nv, int64_t d, int64_t ldv, const double *yv,
                           const double *w)
{
    int64_t e = 0;
    for (int64_t v = 0; v < nv; ++v) {
        double s = 0.0;
        for (int64_t k = 0; k < d; ++k) s = fma(Xv[v * ldv + k], w[k], s);
        const double yh = s > 0.0 ? 1.0 : (s < 0.0 ? -1.0 : (s == 0.0 ? 0.0 : s));
        e += !(yh == yv[v]);
    }
    return e;
}

int oracle_roni(const double *Xv, int64_t nv, int64_t d, int64_t ldv, const double *yv,
                const double *ww, const double *deltas, int64_t n, int64_t ld, double *scores)
{
    double *w = (double *)malloc(sizeof(double) * (size_t)d);
    if (!w) return -2;
    const double dn = (double)nv;
    const double g_err = (double)roni_errors(Xv, nv, d, ldv, yv, ww) / dn;
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t k = 0; k < d; ++k) w[k] = ww[k] + deltas[i * ld + k];
        const double new_err = (double)roni_errors(Xv, nv, d, ldv, yv, w) / dn;
        scores[i] = new_err - g_err;
    }
    free(w);
    return 0;
}
