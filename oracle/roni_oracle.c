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

/*
 * The torch-path RONI verifier (the mnist / lfw softmax models):
 *
 *   roni(ww, delta)   ML/Pytorch/client_obj.py:100-112
 *       myclient.updateModel(weights);          original = myclient.getTrainErr()
 *       myclient.updateModel(weights + update); after    = myclient.getTrainErr()
 *       return after - original
 *   updateModel       ML/Pytorch/client.py:114-121 via SoftmaxModel.reshape
 *                     (ML/Pytorch/softmax_model.py:20-24): the flat fp64 vector
 *                     [W (C x D_in, row-major), b (C)] -> torch.FloatTensor, i.e.
 *                     every parameter rounded to fp32 (after the fp64 add)
 *   getTrainErr       client.py:136-144: for every mini-batch of the SHUFFLED
 *                     trainloader (client.py:20, shuffle=True) out = model(x)
 *                     (nn.Linear: x W^T + b), pred = np.argmax(out, 1); the loop
 *                     overwrites pred / labels, so the return value is
 *                     1 - accuracy_score of the LAST mini-batch only.  `original`
 *                     and `after` are therefore measured on two different
 *                     random batches (two shuffles).
 *
 * Two restatements:
 *   oracle_roni_softmax          every update scored on the same sample set
 *                                (the reference with batch_size >= the set:
 *                                one batch holding every sample)
 *   oracle_roni_softmax_batches  the last-batch semantics: per update j the
 *                                caller passes the two last batches its
 *                                shuffles drew, idx[(2j) nb ..] (original, model
 *                                ww) and idx[(2j+1) nb ..] (after, ww + delta_j)
 * Logit of class c: fp32( (sum_k x_k W_ck, k ascending, in fp64) + b_c ): every
 * product of two fp32 values is exact in fp64, so this is the fp64-accumulated
 * logit rounded once.  torch's CPU sgemm rounds in fp32 in its own order, so
 * the argmax can differ only where the top two logits lie within its rounding:
 * a sample is a NEAR TIE when
 *     !( l1 - l2 - u (|l1| + |l2|)  >  E_a + max_c E_c ),  E_c = g (|x| |w_c| + |b_c|),
 * (l1 = the winning logit of class a, l2 the best other, u = 2^-24,
 * g = gamma_{D_in + 1}(u) (1 + 2^-10): the standard bound on any fp32 summation
 * order of the D_in products and the bias, with the Cauchy-Schwarz bound
 * sum_k |x_k w_ck| <= |x| |w_c|), or any logit is not finite.  The counts of
 * near ties per evaluation are returned (a score that differs
 * from the reference's must come with a near tie).
 * np.argmax: the first maximum, and a NaN counts as the maximum (its first
 * occurrence wins).  accuracy_score = correct / nb (fp64), so
 *   score = (1 - c_after / nb) - (1 - c_orig / nb).
 * Pinned against the reference itself: tests/golden/gen_roni_softmax_goldens.py
 * runs the reference Client.updateModel / getTrainErr with SoftmaxModel on repo
 * inputs (tests/test_roni_oracle.py).
 */
static double softmax_g(int64_t din)
{
    const double u = 0x1p-24, nn = (double)(din + 1);
    return nn * u / (1.0 - nn * u) * (1.0 + 0x1p-10);
}

/* one evaluation: correct predictions and near ties of model (W, b) over the
 * samples rows[0 .. cnt) (rows == NULL: 0 .. cnt) */
static void softmax_eval(const float *Xv, int64_t din, int64_t ldv, const int32_t *yv, int64_t C,
                         const float *W, const float *b, const double *wn, const int64_t *rows,
                         int64_t cnt, int64_t *good, int64_t *near)
{
    const double g = softmax_g(din), u = 0x1p-24;
    double wmax = 0.0, bmax = 0.0;
    for (int64_t c = 0; c < C; ++c) {
        wmax = wn[c] > wmax ? wn[c] : wmax;
        bmax = fabs((double)b[c]) > bmax ? fabs((double)b[c]) : bmax;
    }
    float lg[16];
    for (int64_t i = 0; i < cnt; ++i) {
        const int64_t v = rows ? rows[i] : i;
        const float *x = Xv + v * ldv;
        double xx = 0.0;
        for (int64_t k = 0; k < din; ++k) xx += (double)x[k] * (double)x[k];
        const double xn = sqrt(xx);
        int best = 0;
        for (int64_t c = 0; c < C; ++c) {
            double s = 0.0;
            for (int64_t k = 0; k < din; ++k) s += (double)x[k] * (double)W[c * din + k];
            lg[c] = (float)(s + (double)b[c]);
            if (c > 0 && !(lg[best] != lg[best]) && (lg[c] != lg[c] || lg[c] > lg[best])) best = (int)c;
        }
        *good += best == yv[v];
        int fin = 1;
        double l2 = -INFINITY;
        for (int64_t c = 0; c < C; ++c) {
            fin = fin && isfinite(lg[c]);
            if (c != best && (double)lg[c] > l2) l2 = lg[c];
        }
        const double l1 = lg[best];
        const double ea = g * (xn * wn[best] + fabs((double)b[best]));
        const double emax = g * (xn * wmax + bmax);
        *near += !fin || !(l1 - l2 - u * (fabs(l1) + fabs(l2)) > ea + emax);
    }
}

/* the model of update j (j < 0: ww) as torch holds it: fp32 weights, fp32
 * bias, and the fp64 norms of the C weight rows */
static void softmax_model(const double *ww, const double *delta, int64_t C, int64_t din, float *w,
                          double *wn)
{
    const int64_t d = C * din + C;
    for (int64_t k = 0; k < d; ++k) w[k] = (float)(delta ? ww[k] + delta[k] : ww[k]);
    for (int64_t c = 0; c < C; ++c) {
        double s = 0.0;
        for (int64_t k = 0; k < din; ++k) s += (double)w[c * din + k] * (double)w[c * din + k];
        wn[c] = sqrt(s);
    }
}

int oracle_roni_softmax(const float *Xv, int64_t nv, int64_t din, int64_t ldv, const int32_t *yv,
                        int64_t C, const double *ww, const double *deltas, int64_t n, int64_t ld,
                        double *scores, int32_t *near_ties)
{
    if (C > 16) return -1;
    const int64_t d = C * din + C;
    float *w = (float *)malloc(sizeof(float) * (size_t)d);
    if (!w) return -2;
    double wn[16];
    const double dn = (double)nv;
    int64_t good = 0, near = 0;
    softmax_model(ww, NULL, C, din, w, wn);
    softmax_eval(Xv, din, ldv, yv, C, w, w + C * din, wn, NULL, nv, &good, &near);
    const double orig = 1.0 - (double)good / dn;
    if (near_ties) near_ties[0] = (int32_t)near;
    for (int64_t i = 0; i < n; ++i) {
        softmax_model(ww, deltas + i * ld, C, din, w, wn);
        good = near = 0;
        softmax_eval(Xv, din, ldv, yv, C, w, w + C * din, wn, NULL, nv, &good, &near);
        const double after = 1.0 - (double)good / dn;
        scores[i] = after - orig;
        if (near_ties) near_ties[1 + i] = (int32_t)near;
    }
    free(w);
    return 0;
}

int oracle_roni_softmax_batches(const float *Xv, int64_t nv, int64_t din, int64_t ldv,
                                const int32_t *yv, int64_t C, const double *ww,
                                const double *deltas, int64_t n, int64_t ld, const int64_t *idx,
                                int64_t nb, double *scores, int32_t *near_ties)
{
    if (C > 16) return -1;
    for (int64_t i = 0; i < 2 * n * nb; ++i)
        if (idx[i] < 0 || idx[i] >= nv) return -3;
    const int64_t d = C * din + C;
    float *w0 = (float *)malloc(sizeof(float) * (size_t)d), *w = (float *)malloc(sizeof(float) * (size_t)d);
    if (!w0 || !w) {
        free(w0);
        free(w);
        return -2;
    }
    double wn0[16], wn[16];
    const double dn = (double)nb;
    softmax_model(ww, NULL, C, din, w0, wn0);
    for (int64_t j = 0; j < n; ++j) {
        int64_t g0 = 0, n0 = 0, g1 = 0, n1 = 0;
        softmax_eval(Xv, din, ldv, yv, C, w0, w0 + C * din, wn0, idx + 2 * j * nb, nb, &g0, &n0);
        softmax_model(ww, deltas + j * ld, C, din, w, wn);
        softmax_eval(Xv, din, ldv, yv, C, w, w + C * din, wn, idx + (2 * j + 1) * nb, nb, &g1, &n1);
        const double orig = 1.0 - (double)g0 / dn, after = 1.0 - (double)g1 / dn;
        scores[j] = after - orig;
        if (near_ties) {
            near_ties[2 * j] = (int32_t)n0;
            near_ties[2 * j + 1] = (int32_t)n1;
        }
    }
    free(w0);
    free(w);
    return 0;
}
