// bk_internal.h -- shared declarations between the C ABI (bk_api.hip) and the
// kernels (bk_kernels.hip).  Not installed; the public surface is include/bk.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bk_synth.h"

namespace bk {

// Split-K plan of K1 for one (n, d): T = ceil(n/64) sub-tile rows, ntile =
// T(T+1)/2 upper sub-tiles, S k-pieces of kc columns (multiple of 8), one wave
// per (sub-tile, piece) task, four tasks per 256-thread workgroup.
struct Plan {
    int n = 0, T = 0, ntile = 0, S = 0, nwg = 0;
    int64_t d = 0, kc = 0;
};

hipError_t configure_kernels();
hipError_t launch_gram(const void *X, int dtype, int64_t ld, int n, int64_t d, const Plan &pl,
                       double *part, hipStream_t st);
hipError_t launch_reduce(const double *part, const Plan &pl, double *U, hipStream_t st);
hipError_t launch_sum_ranks(const double *Ug, int R, int64_t stride, double *U, hipStream_t st);
hipError_t launch_expand(const double *U, int n, int T, int ntile, double *G, double *diag,
                         hipStream_t st);
hipError_t launch_scores(const double *G, const double *diag, int n, int64_t k, double *scores,
                         hipStream_t st);
hipError_t launch_rank(const double *scores, int n, int m, int *mask, hipStream_t st);
hipError_t launch_compact(const int *mask, int n, int64_t *sel, hipStream_t st);
hipError_t launch_mean(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *sel, int m,
                       double *mean, int num_cu, hipStream_t st);
hipError_t launch_synth(void *X, int dtype, int64_t ld, int64_t n, int64_t dl, int64_t c0,
                        const int64_t *perm, const SynthParams &P, hipStream_t st);

}  // namespace bk
