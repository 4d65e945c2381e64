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
 *   updateModel       ML/Pytorch/client.py:108-115 via SoftmaxModel.reshape
 *                     (ML/Pytorch/softmax_model.py:19-24): the flat fp64 vector
 *                     [W (C x D_in, row-major), b (C)] -> torch.FloatTensor, i.e.
 *                     every parameter rounded to fp32 (after the fp64 add)
 *   getTrainErr       client.py:131-139: out = model(inputs.float()) (nn.Linear:
 *                     x W^T + b), pred = np.argmax(out, 1), 1 - accuracy_score
 *
 * Restated with the logit of class c as fp32( (sum_k x_k W_ck, k ascending, in
 * fp64) + b_c ): every product of two fp32 values is exact in fp64, so this is
 * the fp64-accumulated logit rounded once (torch's sgemm rounds in its own
 * order; the two can differ only on fp32 near-ties of the top two logits).
 * np.argmax: the first maximum, and a NaN counts as the maximum (its first
 * occurrence wins).  accuracy_score = correct / nv (fp64), so
 *   score = (1 - c_after / nv) - (1 - c_orig / nv).
 * PARITY UNPINNED by the reference itself: ML/Pytorch/client_obj.py is
 * Python 2 and its client / dataset modules (torchvision, the mnist files)
 * are absent; the GPU kernel is checked bit for bit against
 * this restatement (tests/test_gpu_roni_softmax.py).
 */
static int64_t softmax_correct(const float *Xv, int64_t nv, int64_t din, int64_t ldv,
                               const int32_t *yv, int64_t C, const float *W, const float *b)
{
    int64_t good = 0;
    for (int64_t v = 0; v < nv; ++v) {
        const float *x = Xv + v * ldv;
        int best = 0;
        float bl = 0.0f;
        for (int64_t c = 0; c < C; ++c) {
            double s = 0.0;
            for (int64_t k = 0; k < din; ++k) s += (double)x[k] * (double)W[c * din + k];
            const float lg = (float)(s + (double)b[c]);
            if (c == 0) {
                bl = lg;
            } else if (!(bl != bl) && (lg != lg || lg > bl)) {
                best = (int)c;
                bl = lg;
            }
        }
        good += best == yv[v];
    }
    return good;
}

int oracle_roni_softmax(const float *Xv, int64_t nv, int64_t din, int64_t ldv, const int32_t *yv,
                        int64_t C, const double *ww, const double *deltas, int64_t n, int64_t ld,
                        double *scores)
{
    const int64_t d = C * din + C;
    float *w = (float *)malloc(sizeof(float) * (size_t)d);
    if (!w) return -2;
    for (int64_t k = 0; k < d; ++k) w[k] = (float)ww[k];
    const double dn = (double)nv;
    const double orig = 1.0 - (double)softmax_correct(Xv, nv, din, ldv, yv, C, w, w + C * din) / dn;
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t k = 0; k < d; ++k) w[k] = (float)(ww[k] + deltas[i * ld + k]);
        const double after =
            1.0 - (double)softmax_correct(Xv, nv, din, ldv, yv, C, w, w + C * din) / dn;
        scores[i] = after - orig;
    }
    free(w);
    return 0;
}
