// bk_aggregate.hip -- the two HBM-bound steps either side of Multi-Krum
// (SURVEY.md §8(f) rows 2 and 3), gfx950.
//
//   K5  k_qsum    secure-aggregation quantised sum of the accepted updates:
//                 sum[c] = sum_r int64(X[idx[r]][c] * 10^p)   (wrapping int64)
//                 [+ float64(sum[c]) / 10^p]
//                 updateFloatToInt / updateIntToFloat, DistSys/kyber.go:698-710,
//                 745-757, as summed by the miners before recovery
//                 (honest.go:401-409, 442-502).
//   K6  k_noise   NoisedDelta = Delta + (0 + noise_0 + ... + noise_{k-1}) / k,
//                 the client-side DP step of DistSys/main.go:1606-1653 (sum in
//                 arrival order, divide by the float count) and :1524-1537.
//
// The plain block aggregation (GlobalW += sum of accepted Delta, in update
// order, honest.go:361-375) is K4's ACCUM variant in bk_kernels.hip.
//
// All three are one pass over HBM: 16 bytes per lane, columns across lanes,
// rows (or noise vectors) as the sequential inner loop with 8 loads in flight.
// Built with -ffp-contract=off: every add/mul/div rounds exactly as Go's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bk_internal.h"

namespace bk {

typedef double d2v __attribute__((ext_vector_type(2)));

// Go (amd64) int64(float64): CVTTSD2SQ truncates toward zero; NaN and values
// outside [-2^63, 2^63) give the "integer indefinite" 0x8000000000000000.
__host__ __device__ __forceinline__ int64_t go_f64_to_i64(double y) {
    if (y >= -9223372036854775808.0 && y < 9223372036854775808.0) return (int64_t)y;
    return INT64_MIN;
}

// used-once streaming reads: non-temporal (see ld2s in bk_kernels.hip)
template <typename T>
__device__ __forceinline__ double ldv(const T *p) {
#ifndef BK_NO_NT
    return (double)__builtin_nontemporal_load(p);
#else
    return (double)*p;
#endif
}
__device__ __forceinline__ d2v ldnt(const double *p) {
#ifndef BK_NO_NT
    return __builtin_nontemporal_load(reinterpret_cast<const d2v *>(p));
#else
    return *reinterpret_cast<const d2v *>(p);
#endif
}

template <typename T, bool FLT>
__global__ __launch_bounds__(256) void k_qsum(const T *__restrict__ X, int64_t ld, int64_t d,
                                              const int64_t *__restrict__ idx, int m, double scale,
                                              int64_t *__restrict__ sum, double *__restrict__ sumf) {
    extern __shared__ __attribute__((aligned(16))) int64_t srow[];
    for (int r = threadIdx.x; r < m; r += 256) srow[r] = idx[r] * ld;
    __syncthreads();
    for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < d;
         c += (int64_t)gridDim.x * 256) {
        uint64_t acc = 0;  // int64 wraps in Go; unsigned arithmetic is the same bits
        int r = 0;
        for (; r + 8 <= m; r += 8) {
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = ldv(X + srow[r + q] + c);
#pragma unroll
            for (int q = 0; q < 8; ++q) acc += (uint64_t)go_f64_to_i64(v[q] * scale);
        }
        for (; r < m; ++r) acc += (uint64_t)go_f64_to_i64(ldv(X + srow[r] + c) * scale);
        sum[c] = (int64_t)acc;
        if constexpr (FLT) sumf[c] = (double)(int64_t)acc / scale;
    }
}

// out[i][c] = delta[i][c] + ((0 + noise[i][0][c]) + ... + noise[i][k-1][c]) / k
// noise vector j of update i at noise + (i*k + j)*nld; out may alias delta.
template <bool VEC>
__global__ __launch_bounds__(256) void k_noise(const double *delta, int64_t ld, int64_t n,
                                               int64_t d, const double *__restrict__ noise,
                                               int64_t k, int64_t nld, double *out, int64_t old) {
    const double dk = (double)k;
    const int64_t npair = (d + 1) >> 1;
    for (int64_t i = blockIdx.y; i < n; i += gridDim.y) {
        const double *nz = noise + i * k * nld;
        for (int64_t cp = (int64_t)blockIdx.x * 256 + threadIdx.x; cp < npair;
             cp += (int64_t)gridDim.x * 256) {
            const int64_t c = cp * 2;
            if (VEC && c + 1 < d) {
                d2v s = {0.0, 0.0};
                int64_t j = 0;
                for (; j + 8 <= k; j += 8) {
                    d2v v[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        v[q] = ldnt(nz + (j + q) * nld + c);
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        s.x += v[q].x;
                        s.y += v[q].y;
                    }
                }
                for (; j < k; ++j) {
                    const d2v v = ldnt(nz + j * nld + c);
                    s.x += v.x;
                    s.y += v.y;
                }
                const d2v a = ldnt(delta + i * ld + c);
                d2v o;
                o.x = a.x + s.x / dk;
                o.y = a.y + s.y / dk;
                // written once, not re-read by this kernel: a non-temporal store
                // (0.839 -> 0.744 ms for 128 x 2^20 with k = 2, tools/ab_noise.py)
#ifndef BK_NO_NT
                __builtin_nontemporal_store(o, reinterpret_cast<d2v *>(out + i * old + c));
#else
                *reinterpret_cast<d2v *>(out + i * old + c) = o;
#endif
            } else {
                for (int64_t cc = c; cc < c + 2 && cc < d; ++cc) {
                    double s = 0.0;
                    for (int64_t j = 0; j < k; ++j) s += nz[j * nld + cc];
                    out[i * old + cc] = delta[i * ld + cc] + s / dk;
                }
            }
        }
    }
}

hipError_t launch_qsum(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *idx, int m,
                       double scale, int64_t *sum, double *sumf, int num_cu, hipStream_t st) {
    int64_t blocks = (d + 255) / 256;
    const int64_t cap = (int64_t)num_cu * 16;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const size_t lds = (size_t)m * sizeof(int64_t);
    dim3 grid((unsigned)blocks), block(256);
    if (dtype == 0) {
        if (sumf)
            hipLaunchKernelGGL((k_qsum<double, true>), grid, block, lds, st, (const double *)X, ld,
                               d, idx, m, scale, sum, sumf);
        else
            hipLaunchKernelGGL((k_qsum<double, false>), grid, block, lds, st, (const double *)X, ld,
                               d, idx, m, scale, sum, sumf);
    } else {
        if (sumf)
            hipLaunchKernelGGL((k_qsum<float, true>), grid, block, lds, st, (const float *)X, ld, d,
                               idx, m, scale, sum, sumf);
        else
            hipLaunchKernelGGL((k_qsum<float, false>), grid, block, lds, st, (const float *)X, ld,
                               d, idx, m, scale, sum, sumf);
    }
    return hipGetLastError();
}

hipError_t launch_noise(const double *delta, int64_t ld, int64_t n, int64_t d, const double *noise,
                        int64_t k, int64_t nld, double *out, int64_t old, int num_cu,
                        hipStream_t st) {
    const int64_t npair = (d + 1) / 2;
    int64_t bx = (npair + 255) / 256;
    if (bx > 4096) bx = 4096;
    if (bx < 1) bx = 1;
    // enough blocks in y to fill the chip (>= 16 per CU), rows grid-strided
    int64_t by = ((int64_t)num_cu * 16 + bx - 1) / bx;
    if (by > n) by = n;
    if (by > 65535) by = 65535;
    if (by < 1) by = 1;
    const bool vec = (ld % 2) == 0 && (nld % 2) == 0 && (old % 2) == 0 &&
                     ((uintptr_t)delta % 16) == 0 && ((uintptr_t)noise % 16) == 0 &&
                     ((uintptr_t)out % 16) == 0;
    dim3 grid((unsigned)bx, (unsigned)by), block(256);
    if (vec)
        hipLaunchKernelGGL(k_noise<true>, grid, block, 0, st, delta, ld, n, d, noise, k, nld, out,
                           old);
    else
        hipLaunchKernelGGL(k_noise<false>, grid, block, 0, st, delta, ld, n, d, noise, k, nld, out,
                           old);
    return hipGetLastError();
}

hipError_t configure_aggregate_kernels() {
    for (const void *k : {(const void *)k_qsum<double, true>, (const void *)k_qsum<double, false>,
                          (const void *)k_qsum<float, true>, (const void *)k_qsum<float, false>}) {
        hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace bk
