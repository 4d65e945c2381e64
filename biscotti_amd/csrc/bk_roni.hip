// bk_roni.hip -- the RONI verifier, gfx950.
//
// roni(ww, delta), ML/code/logistic_validator.py:22-33 (bound as pyRoniFunc,
// DistSys/honest.go:235-243; called per update by verifyUpdate,
// honest.go:598-629; the verdict roniScore > 0.02 rejects, main.go:213-226):
//     yhat   = sign(Xvalid . ww)            g_err   = mean(yhat  != yvalid)
//     yhat2  = sign(Xvalid . (ww + delta))  new_err = mean(yhat2 != yvalid)
//     score  = new_err - g_err
// batched over n updates: model 0 is ww, model j >= 1 is ww + delta_{j-1}
// (added elementwise in fp64 first, as numpy does).
//
//   K7  k_roni_count   grid (row chunks, groups of 16 models): the block
//                      builds its 16 models in LDS ([d][16], broadcast reads),
//                      each thread takes validation rows and runs 16 fp64 dots
//                      per row from one pass over the row, np.sign semantics
//                      (0 -> 0, NaN -> NaN), per-model wave sums of the
//                      mismatches, one integer atomic per wave and model
//                      (counts are exact and order-free)
//   K7b k_roni_score   score[i] = cnt[i+1]/nv - cnt[0]/nv in fp64
//
// Bound: the validation set is re-read once per 16 models (from L2 / Infinity
// Cache for creditcard-sized sets: 85,000 x 25 fp64 = 17 MB); the dots are
// fp64 VALU work, 16 independent FMA chains per row.  Built with
// -ffp-contract=off: ww + delta rounds exactly like numpy; the dot itself is a
// plain fp64 FMA chain (BLAS order is library-specific: only the sign matters,
// and it differs from numpy's only for dots within rounding of 0).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bk_internal.h"

namespace bk {

constexpr int RONI_ROWS = 1024;  // validation rows per block (4 per thread)
constexpr int RONI_MPB = 16;     // models per block: each x element loaded feeds 16 FMAs

// grid (row chunks, model groups); models m0 .. m0+15 of the n+1 (0 = ww)
__global__ __launch_bounds__(256) void k_roni_count(const double *__restrict__ Xv, int64_t nv,
                                                    int64_t d, int64_t ldv,
                                                    const double *__restrict__ yv,
                                                    const double *__restrict__ ww,
                                                    const double *__restrict__ deltas, int64_t ld,
                                                    int64_t nmod, unsigned int *__restrict__ cnt) {
    extern __shared__ __attribute__((aligned(16))) double w[];  // [d][RONI_MPB]
    const int64_t m0 = (int64_t)blockIdx.y * RONI_MPB;
    for (int64_t e = threadIdx.x; e < d * RONI_MPB; e += 256) {
        const int64_t k = e / RONI_MPB, j = m0 + e % RONI_MPB;
        double v = 0.0;  // models past the end: never counted
        if (j < nmod) v = j == 0 ? ww[k] : ww[k] + deltas[(j - 1) * ld + k];
        w[e] = v;
    }
    __syncthreads();
    unsigned int mine[RONI_MPB];
#pragma unroll
    for (int j = 0; j < RONI_MPB; ++j) mine[j] = 0;
    const int64_t r0 = (int64_t)blockIdx.x * RONI_ROWS;
    for (int64_t v = r0 + threadIdx.x; v < r0 + RONI_ROWS && v < nv; v += 256) {
        const double *x = Xv + v * ldv;
        double s[RONI_MPB];
#pragma unroll
        for (int j = 0; j < RONI_MPB; ++j) s[j] = 0.0;
        for (int64_t k = 0; k < d; ++k) {
            const double xk = x[k];
            const double *wk = w + k * RONI_MPB;
#pragma unroll
            for (int j = 0; j < RONI_MPB; ++j) s[j] = __builtin_fma(xk, wk[j], s[j]);
        }
        const double y = yv[v];
#pragma unroll
        for (int j = 0; j < RONI_MPB; ++j) {
            const double yh = s[j] > 0.0 ? 1.0 : (s[j] < 0.0 ? -1.0 : (s[j] == 0.0 ? 0.0 : s[j]));
            mine[j] += !(yh == y);  // NaN never equals: an error, as in numpy
        }
    }
    // per model: wave total, then one atomic per wave
#pragma unroll
    for (int j = 0; j < RONI_MPB; ++j) {
        unsigned int tot = mine[j];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        if ((threadIdx.x & 63) == 0 && tot && m0 + j < nmod) atomicAdd(&cnt[m0 + j], tot);
    }
}

__global__ void k_roni_score(const unsigned int *__restrict__ cnt, int64_t n, int64_t nv,
                             double *__restrict__ scores) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double dn = (double)nv;
    const double g_err = (double)cnt[0] / dn;
    const double new_err = (double)cnt[i + 1] / dn;
    scores[i] = new_err - g_err;
}

hipError_t launch_roni(const double *Xv, int64_t nv, int64_t d, int64_t ldv, const double *yv,
                       const double *ww, const double *deltas, int64_t n, int64_t ld,
                       unsigned int *cnt, double *scores, hipStream_t st) {
    hipError_t e = hipMemsetAsync(cnt, 0, (size_t)(n + 1) * sizeof(unsigned int), st);
    if (e != hipSuccess) return e;
    const dim3 grid((unsigned)((nv + RONI_ROWS - 1) / RONI_ROWS),
                    (unsigned)((n + 1 + RONI_MPB - 1) / RONI_MPB));
    hipLaunchKernelGGL(k_roni_count, grid, dim3(256), (size_t)d * RONI_MPB * sizeof(double), st,
                       Xv, nv, d, ldv, yv, ww, deltas, ld, n + 1, cnt);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_score, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cnt, n,
                       nv, scores);
    return hipGetLastError();
}

}  // namespace bk
