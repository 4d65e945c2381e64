// bk_device.h -- device helpers shared by the kernels of libbk (bk_kernels.hip,
// bk_small.hip): the total order of the row sort, the packed upper-tile
// addressing, the register bitonic building blocks and the selection margin.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bk_internal.h"

namespace bk {

typedef double d2v __attribute__((ext_vector_type(2)));

// total order on doubles for sorting / selection: ascending, +0 == -0, NaN last
__device__ __forceinline__ uint64_t dkey(double v) {
    if (v != v) return 0xFFF8000000000000ULL;
    if (v == 0.0) v = 0.0;
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
__device__ __forceinline__ double dkey_inv(uint64_t k) {
    const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k;
    return __longlong_as_double((long long)b);
}

// G_ij straight from the packed upper 64x64 tiles (K1b's output): tiles below
// the diagonal and the lower half of diagonal tiles read the transposed
// element -- the same values the former K1c expansion copied, so bit-identical
__device__ __forceinline__ int64_t upper_tile(int T, int a, int b) {
    return (int64_t)(a * T - a * (a - 1) / 2 + (b - a)) * 4096;
}
__device__ __forceinline__ double u_at(const double *__restrict__ U, int T, int r, int c) {
    const int br = r >> 6, bc = c >> 6, ir = r & 63, ic = c & 63;
    if (br < bc || (br == bc && ir <= ic)) return U[upper_tile(T, br, bc) + ir * 64 + ic];
    return U[upper_tile(T, bc, br) + ic * 64 + ir];
}

template <typename K>
struct K2Ord;
template <>
struct K2Ord<uint64_t> {
    static __device__ __forceinline__ uint64_t lo(uint64_t a, uint64_t b) { return a < b ? a : b; }
    static __device__ __forceinline__ uint64_t hi(uint64_t a, uint64_t b) { return a < b ? b : a; }
    static __device__ __forceinline__ uint64_t bits(uint64_t a) { return a; }
    static __device__ __forceinline__ uint64_t from(uint64_t b) { return b; }
    static __device__ __forceinline__ double val(uint64_t a) { return dkey_inv(a); }
    static __device__ __forceinline__ uint64_t neg(uint64_t a) { return ~a; }  // order-reversing
};
template <>
struct K2Ord<double> {  // no NaN in the row: IEEE min / max
    static __device__ __forceinline__ double lo(double a, double b) { return __builtin_fmin(a, b); }
    static __device__ __forceinline__ double hi(double a, double b) { return __builtin_fmax(a, b); }
    static __device__ __forceinline__ uint64_t bits(double a) { return (uint64_t)__double_as_longlong(a); }
    static __device__ __forceinline__ double from(uint64_t b) { return __longlong_as_double((long long)b); }
    static __device__ __forceinline__ double val(double a) { return a; }
    static __device__ __forceinline__ double neg(double a) { return -a; }  // order-reversing
};

template <typename K>
__device__ __forceinline__ void k2_cas(K &a, K &b) {  // ascending: a gets the min
    const K l = K2Ord<K>::lo(a, b), h = K2Ord<K>::hi(a, b);
    a = l;
    b = h;
}

// the 64-bit value of lane (lane ^ M), 0 < M <= 63
template <int M>
__device__ __forceinline__ uint64_t k2_xchg(uint64_t v) {
    const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
    int a, b;
    if constexpr (M <= 3) {  // DPP quad_perm: lane ^ M within each quad
        constexpr int P = (0 ^ M) | ((1 ^ M) << 2) | ((2 ^ M) << 4) | ((3 ^ M) << 6);
        a = __builtin_amdgcn_mov_dpp(lo, P, 0xF, 0xF, false);
        b = __builtin_amdgcn_mov_dpp(hi, P, 0xF, 0xF, false);
    } else if constexpr (M <= 31) {  // ds_swizzle bit-mask mode: and 0x1F, xor M
        a = __builtin_amdgcn_ds_swizzle(lo, 0x1F | (M << 10));
        b = __builtin_amdgcn_ds_swizzle(hi, 0x1F | (M << 10));
    } else {
        a = __shfl_xor(lo, M);
        b = __shfl_xor(hi, M);
    }
    return (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)b << 32);
}

// a stage whose partner is lane ^ M, register q ^ XL (XL = 0: xor stage;
// XL = KPT - 1: the mirror stage opening a merge); `lower`: this lane holds
// the lower index of every pair, so it keeps the minima
template <typename K, int KPT, int M, int XL>
__device__ __forceinline__ void k2_lane_stage(K (&v)[KPT], bool lower) {
    K o[KPT];
#pragma unroll
    for (int q = 0; q < KPT; ++q) o[q] = K2Ord<K>::from(k2_xchg<M>(K2Ord<K>::bits(v[q])));
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
        const K w = o[q ^ XL];
        const K l = K2Ord<K>::lo(v[q], w), h = K2Ord<K>::hi(v[q], w);
        v[q] = lower ? l : h;
    }
}

template <typename K, int KPT, int XL>
__device__ __forceinline__ void k2_lane_dispatch(K (&v)[KPT], int m, bool lower) {
    switch (m) {
    case 1: k2_lane_stage<K, KPT, 1, XL>(v, lower); break;
    case 2: k2_lane_stage<K, KPT, 2, XL>(v, lower); break;
    case 3: k2_lane_stage<K, KPT, 3, XL>(v, lower); break;
    case 4: k2_lane_stage<K, KPT, 4, XL>(v, lower); break;
    case 7: k2_lane_stage<K, KPT, 7, XL>(v, lower); break;
    case 8: k2_lane_stage<K, KPT, 8, XL>(v, lower); break;
    case 15: k2_lane_stage<K, KPT, 15, XL>(v, lower); break;
    case 16: k2_lane_stage<K, KPT, 16, XL>(v, lower); break;
    case 31: k2_lane_stage<K, KPT, 31, XL>(v, lower); break;
    case 32: k2_lane_stage<K, KPT, 32, XL>(v, lower); break;
    default: k2_lane_stage<K, KPT, 63, XL>(v, lower); break;
    }
}

// gamma_n = n u / (1 - n u) (Higham's bound for a length-n dot product or sum
// in any order, every step one rounding); +inf once n u >= 1
__device__ __forceinline__ double gamma_n(double nn, double u) {
    const double t = nn * u;
    return t < 1.0 ? t / (1.0 - t) : __builtin_inf();
}

// The selection margin record (include/bk.h bk_selection_margin; k_compact):
// from the boundary scores lo (rank m-1) and hi (rank m), M = max finite
// G_ii, the Gram's column count d and unit roundoff u_gram, an absolute bound
// eg on every Gram element's error beyond that (the int8-sliced Gram, K1i8;
// 0 otherwise), and k.  A score sums k distances G_ii + G_jj - 2 G_ij, so a
// Gram error of eg moves each by <= 4 eg:
//   e = 4 k (M' (gamma_{d+2}(u_G) + 2 u + gamma_k(u)) + eg (1 + gamma_k(u))),
//   M' = (M + eg) (1 + 2 gamma_{d+2}(u_G))
//   margin[0..7] = {gap, err_bound, near_tie, M, s_lo, s_hi, d, k}, margin[8] = u_G
// (u_G is what the certified re-run reads: an int8 record reports 2^-30, so
// any Gram that is not exact fp64 re-runs on a near tie)
__device__ __forceinline__ void write_margin(double *margin, double lo, double hi, double M,
                                             double dg, int64_t k, double u_gram, double eg = 0.0) {
    const double u = 0x1p-53, kk = (double)k;
    const double gG = gamma_n(dg + 2.0, u_gram), gR = gamma_n(dg + 2.0, u);
    const double gk = gamma_n(kk, u);
    const double Mt = (M + eg) * (1.0 + 2.0 * gG);
    const double e_here = 4.0 * kk * (Mt * (gG + 2.0 * u + gk) + eg * (1.0 + gk));
    const double e_ref = 4.0 * kk * Mt * (gR + 2.0 * u + gk);
    const double bound = 2.0 * (e_here + e_ref) * (1.0 + 0x1p-40);
    // NaN scores rank last here and in numpy: a finite-to-NaN boundary is certain
    const double gap = (hi != hi && lo == lo) ? __builtin_inf() : hi - lo;
    margin[0] = gap;
    margin[1] = bound;
    margin[2] = (gap > bound) ? 0.0 : 1.0;  // NaN gap -> near tie
    margin[3] = M;
    margin[4] = lo;
    margin[5] = hi;
    margin[6] = dg;
    margin[7] = kk;
    margin[8] = eg != 0.0 && u_gram < 0x1p-30 ? 0x1p-30 : u_gram;  // internal: the re-run decision
}


// The margin from a packed record's trailing record {dg, d32, eg}: dg = the
// Gram's column count, d32 = how many of them were accumulated on the fp32
// MFMA, eg = the int8-sliced columns' absolute error bound (all summed by every
// exchange).  u_G = 2^-24 as soon as one column was on the fp32 MFMA.
//   dg NaN (a rank poisoned its partial: bk_multikrum_sharded_device) -> the
//          record is invalid (MARGIN_POISONED)
//   dg < 1 (a caller's record without a column count, e.g. pack_upper(G, 0))
//          -> the bound is unknown: err_bound = +inf, near_tie = 1
//   eg +inf (a non-finite input on the int8 path) -> near_tie = 1
__device__ __forceinline__ void write_margin_rec(double *margin, double lo, double hi, double M,
                                                 double dg, double d32, double eg, int64_t k) {
    if (dg != dg || d32 != d32) {
        write_margin(margin, lo, hi, M, 0.0, k, 0x1p-53);
        margin[1] = __builtin_nan("");
        margin[2] = MARGIN_POISONED;
        margin[6] = __builtin_nan("");
        return;
    }
    const double u_gram = d32 > 0.0 ? 0x1p-24 : 0x1p-53;
    write_margin(margin, lo, hi, M, dg, k, u_gram, eg == eg ? eg : __builtin_inf());
    if (!(dg >= 1.0)) {
        margin[1] = __builtin_inf();
        margin[2] = 1.0;
    }
}

}  // namespace bk
