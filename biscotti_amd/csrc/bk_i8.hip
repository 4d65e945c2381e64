// bk_i8.hip -- K1i8: the Gram of fp32 rows from exact int8 slices (Ozaki
// scheme), on v_mfma_i32_32x32x32_i8 (bk_set_f32_mode(ctx, BK_F32_I8);
// BASELINE config E, 4096 x 262,144 fp32).
//
// The reference's Gram is np.dot(X, X.T) in fp64 (ML/code/logistic_validator.py:
// 59-60).  Here the columns are cut into R ranges (one per XCD); within range r
// row i is scaled by a power of two s_ir >= max_k |x_ik| and split into three
// signed 7-bit digits,
//     x_ik / s_ir = a0/64 + a1/2^13 + a2/2^20 + rho,   |a_t| <= 64, |rho| <= 2^-21,
// all exact in fp64 (fp32 inputs, power-of-two scaling, integer subtractions).
// The range's Gram is then
//     P_r = s_i s_j 2^-26 (2^14 L0 + 2^7 L1 + L2),
//     L0 = A0 A0^T,  L1 = A0 A1^T + A1 A0^T,  L2 = A0 A2^T + A1 A1^T + A2 A0^T,
// six int8 GEMMs accumulated EXACTLY in int32 (|a a'| <= 2^12 per column,
// <= 2^15 columns per range in practice, < 2^31), combined exactly in fp64
// (< 2^53), so every range partial is exact for the truncated digits and the
// whole Gram deterministic.  The dropped terms (a1 a2, a2 a1, a2 a2 and rho)
// bound the error of every element absolutely (DESIGN.md §4 "K1i8"):
//     |G_ij - G~_ij| <= sum_r 2^-21 (2 S_r L1_r + 2.03 d_r S_r^2) (1 + 2^-20),
//     S_r = max_i s_ir,  L1_r = max_i ||x_i,r||_1,  d_r = the range's columns,
// which k_i8_bound writes into the packed record's trailing element [2]; the
// selection margin adds it to every distance (bk_device.h write_margin), so the
// near-tie contract holds: a set that differs from the reference's comes with
// near_tie = 1.  A non-finite input makes that bound +inf (always a near tie;
// BK_F32_I8_CERTIFIED re-runs it exact).
//
//   k_i8_slice   one workgroup per (row, range): the range's row slice read
//                once into registers, its max |x| and ||x||_1, then the three
//                digit planes: HBM-bound, 4 (8) + 3 bytes per element
//   k_i8_bound   the absolute error bound (one workgroup, a wave per range)
//   k_gram_i8    128 x 128 output tiles of one range per workgroup, 4 waves of
//                64 x 64 (2 x 2 MFMA blocks x 3 levels: 192 int32 accumulators
//                per lane), digit planes staged through LDS in chunks of 64
//                columns (48 KiB per stage, 2 stages), 16-B granules
//                XOR-swizzled so every ds_read_b128 fragment read is
//                conflict-free; every XCD sweeps the column ranges in the same
//                order over a compact piece of the tile order (i8_layout), so
//                an XCD's concurrent tiles share row-blocks in its L2 and the
//                XCDs share the range's digit lines in the Infinity Cache
//   k_i8_reduce  U = sum over ranges (fixed order) of the exact range partials,
//                + the trailing record {d, 0, bound, 0}
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <vector>

#include "bk_internal.h"

namespace bk {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int I8_TILE = 128, I8_KC = 64, I8_S = 3;
constexpr int I8_PLANE = I8_TILE * I8_KC;          // one digit plane of one operand per stage: 8 KiB
constexpr int I8_OPND = I8_S * I8_PLANE;           // 24 KiB
constexpr int I8_STAGE = 2 * I8_OPND;              // 48 KiB
// digit-plane layout (A/B builds): 0 = row-major (row i's range at i * dp),
// 1 = blocked per (row-block of 128, 64-column chunk): 8 KiB contiguous, so a
// chunk fetch of a row-block is one 8-KiB run instead of 128 64-B pieces
#ifndef BK_I8_BLOCKED
#define BK_I8_BLOCKED 1
#endif
// byte offset of (row, column) in one digit plane (column a multiple of 16
// for the 16-B stores and loads; dp = padded columns)
__host__ __device__ __forceinline__ int64_t i8_off(int64_t row, int64_t col, int64_t dp) {
#if BK_I8_BLOCKED
    return (((row >> 7) * (dp >> 6) + (col >> 6)) << 13) + ((row & 127) << 6) + (col & 63);
#else
    return row * dp + col;
#endif
}
// bytes between consecutive 64-column chunks of one row
constexpr int64_t I8_CHUNK_STRIDE = BK_I8_BLOCKED ? 8192 : I8_KC;
// K1i8's workgroup -> (tile, range) map (A/B builds): 0 = range b mod R, 1 =
// every XCD on the same range at a time (i8_layout)
#ifndef BK_I8_MAP
#define BK_I8_MAP 1
#endif
constexpr int I8_LDS = 2 * I8_STAGE;               // 96 KiB: two stages
#ifndef BK_I8_ABL
#define BK_I8_ABL 0
#endif
// waves per workgroup of the two- and three-digit Gram kernels (4: one per
// SIMD, 64 x 128 / 64 x 64 per wave; 8: two per SIMD, 64 x 64 / 64 x 32)
#ifndef BK_I8_W2
#define BK_I8_W2 4
#endif
#ifndef BK_I8_W3
#define BK_I8_W3 4
#endif
constexpr int I8_NBJ2 = BK_I8_W2 == 8 ? 2 : 4, I8_NBJ3 = BK_I8_W3 == 8 ? 1 : 2;
// the super-block of the tile order (i8_layout): BK_I8_SBI row blocks of 128
// by BK_I8_SBC columns (in units of 128) -- an XCD's ~32 concurrent tiles
// share these row blocks in its L2
#ifndef BK_I8_SBI
#define BK_I8_SBI 4
#endif
#ifndef BK_I8_SBC
#define BK_I8_SBC 4
#endif
constexpr int I8_RANGE_BYTES = 131072;             // a row's slice of one column range (i8_layout)
// the exponent of a (row, range) slice holding a NaN or an infinity: its
// digits are zero, k_gram_i8 writes NaN into every Gram element of that row
// (so K2 scores it NaN and ranks it last, as the reference's NaN distances
// do), and k_i8_bound's scale 2^e becomes +inf (the bound, a near tie)
constexpr int I8_NONFINITE = 1 << 20;

// ---------------------------------------------------------------------------
// slicing: grid (npad rows, R ranges), 512 threads.  The range's row slice
// (<= 128 KiB: R is chosen for it, i8_layout) is read ONCE from HBM straight
// into registers -- thread t holds 16 consecutive columns of each 8,192-column
// block, every load issued before the first is used -- while its max |x| and
// ||x||_1 accumulate; then the digits are cut from the registers, three 16-B
// stores per 16 columns.  (r4a staged the slice through 128 KiB of LDS: one
// workgroup per CU, its loads in dependent rounds: 4.4 ms at config E.)
// T = float (config E) or double (fp64 rows: the same digits, every step
// exact in fp64 too; only the remainder past the third digit is dropped)
// ---------------------------------------------------------------------------
// NT threads, MAXU blocks of 16 NT columns: <512, full> for the ranges of a
// whole batch; <256, 1> for ranges of <= 4,096 columns (a column shard's
// ranges: config E's 8-rank shard has 4,096 per range), where 512 threads
// would leave half idle and every register block but one unused
constexpr int I8_SLICE_NT = 512;
// NS: digit planes written (3, or 2 for BK_F32_I8X2: x / s = a0/64 + a1/2^13 + rho,
// |rho| <= 2^-14)
template <typename T, int NS, int NT = I8_SLICE_NT,
          int MAXU = I8_RANGE_BYTES / (int)(sizeof(T) * 16 * I8_SLICE_NT)>
__global__ __launch_bounds__(NT) void k_i8_slice(const T *__restrict__ X, int64_t ld, int n,
                                                 int64_t d, const int64_t *__restrict__ rb, int R,
                                                 int8_t *__restrict__ S, int64_t dp, int64_t plane,
                                                 int *__restrict__ es, double *__restrict__ l1o) {
    constexpr int EPG = 16 / sizeof(T);  // elements per 16-B load
    constexpr int BLK = 16 * NT;         // columns per block
    static_assert(MAXU >= 1 && MAXU * BLK * (int)sizeof(T) <= I8_RANGE_BYTES, "range blocks");
    typedef T gvec __attribute__((ext_vector_type(EPG)));
    __shared__ double smx[NT / 64], sl1[NT / 64];
    __shared__ int sfin[NT / 64];
#if BK_I8_BLOCKED
    // rows 2k and 2k + 1 (the two 64-B halves of every 128-B line the blocked
    // layout writes) on the same XCD, 8 blocks apart in dispatch order, so its
    // L2 merges the halves before they go to memory
    const int bx = blockIdx.x;
    const int i = (bx & ~15) | ((bx & 7) << 1) | ((bx >> 3) & 1);
#else
    const int i = blockIdx.x;
#endif
    const int r = blockIdx.y, tid = threadIdx.x;
    const int64_t c0 = rb[r], c1 = rb[r + 1];
    const int64_t ce = c1 < d ? c1 : d;  // columns past d are zero
    const int len = (int)(c1 - c0);      // a multiple of 64, <= MAXU * BLK
    const T *xr = X + (int64_t)(i < n ? i : 0) * ld + c0;
    T v[MAXU][16];
#pragma unroll
    for (int u = 0; u < MAXU; ++u) {
        const int c = u * BLK + 16 * tid;
        if (i < n && c0 + c + 16 <= ce) {
#pragma unroll
            for (int q = 0; q < 16 / EPG; ++q) {
                const gvec g = *reinterpret_cast<const gvec *>(xr + c + EPG * q);
#pragma unroll
                for (int e = 0; e < EPG; ++e) v[u][EPG * q + e] = g[e];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) v[u][e] = (i < n && c < len && c0 + c + e < ce) ? xr[c + e] : (T)0;
        }
    }
    double mx = 0.0, l1 = 0.0;
    int fin = 1;
#pragma unroll
    for (int u = 0; u < MAXU; ++u)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const double a = __builtin_fabs((double)v[u][e]);
            fin &= a <= 1.7976931348623157e308;  // NaN and +-inf fail
            mx = a > mx ? a : mx;
            l1 += a;
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double m2 = __shfl_xor(mx, o);
        mx = m2 > mx ? m2 : mx;
        l1 += __shfl_xor(l1, o);
        fin &= __shfl_xor(fin, o);
    }
    if ((tid & 63) == 0) {
        smx[tid >> 6] = mx;
        sl1[tid >> 6] = l1;
        sfin[tid >> 6] = fin;
    }
    __syncthreads();
    mx = smx[0];
    l1 = sl1[0];
    fin = sfin[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) {
        mx = smx[w] > mx ? smx[w] : mx;
        l1 += sl1[w];
        fin &= sfin[w];
    }
    // s = 2^e > max |x| (frexp: mx = m 2^e, m in [0.5, 1)); all-zero rows: e = 0
    int e = 0;
    if (fin && mx > 0.0) (void)frexp(mx, &e);
    if (tid == 0) {
        es[(int64_t)i * R + r] = fin ? e : I8_NONFINITE;
        l1o[(int64_t)i * R + r] = fin ? l1 : __builtin_inf();
    }
    int8_t *s0 = S, *s1 = s0 + plane, *s2 = s1 + plane;  // (s2: three digits only)
#pragma unroll
    for (int u = 0; u < MAXU; ++u) {
        const int c = u * BLK + 16 * tid;
        if (c >= len) continue;
        int dig[3][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int p0 = 0, p1 = 0, p2 = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const double x = fin ? (double)v[u][4 * q + w] : 0.0;
                const double y = ldexp(x, 6 - e);  // 64 x / s, exact
                const double a0 = __builtin_rint(y);
                const double y1 = (y - a0) * 128.0;  // exact
                const double a1 = __builtin_rint(y1);
                p0 |= ((int)a0 & 0xff) << (8 * w);
                p1 |= ((int)a1 & 0xff) << (8 * w);
                if constexpr (NS == 3) {
                    const double a2 = __builtin_rint((y1 - a1) * 128.0);
                    p2 |= ((int)a2 & 0xff) << (8 * w);
                }
            }
            dig[0][q] = p0;
            dig[1][q] = p1;
            dig[2][q] = p2;
        }
        const int64_t o = i8_off(i, c0 + c, dp);
        *reinterpret_cast<v4i *>(s0 + o) = v4i{dig[0][0], dig[0][1], dig[0][2], dig[0][3]};
        *reinterpret_cast<v4i *>(s1 + o) = v4i{dig[1][0], dig[1][1], dig[1][2], dig[1][3]};
        if constexpr (NS == 3)
            *reinterpret_cast<v4i *>(s2 + o) = v4i{dig[2][0], dig[2][1], dig[2][2], dig[2][3]};
    }
}

// the absolute error bound of the sliced Gram (header), into out[0]
// one workgroup of 16 waves: wave w takes ranges w, w + 16, ... (its lanes
// over the rows: the max scale and the max norm of the range, exact whatever
// the order; a NaN / inf norm is sticky), the range's term goes to LDS, and
// thread 0 adds the terms in range order -- the same sum as one thread looping
// over the ranges (r4c's form: 71 us at config D's 128 ranges, on the path)
constexpr int I8_BOUND_NT = 1024, I8_BOUND_BATCH = 1024;
__global__ __launch_bounds__(I8_BOUND_NT) void k_i8_bound(const int *__restrict__ es,
                                                          const double *__restrict__ l1,
                                                          const int64_t *__restrict__ rb, int R, int n,
                                                          int64_t d, int ns, double *__restrict__ out) {
    __shared__ double term[I8_BOUND_BATCH];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double tot = 0.0;
    for (int r0 = 0; r0 < R; r0 += I8_BOUND_BATCH) {
        const int r1 = R - r0 < I8_BOUND_BATCH ? R : r0 + I8_BOUND_BATCH;
        for (int r = r0 + wave; r < r1; r += I8_BOUND_NT / 64) {
            double smax = 0.0, lmax = 0.0;
            for (int i = lane; i < n; i += 64) {
                const double sv = ldexp(1.0, es[(int64_t)i * R + r]);
                const double v = l1[(int64_t)i * R + r];
                smax = sv > smax ? sv : smax;
                lmax = (v > lmax || v != v) ? v : lmax;  // a NaN / inf norm poisons the bound
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double x = __shfl_xor(smax, o), y = __shfl_xor(lmax, o);
                smax = x > smax ? x : smax;
                lmax = (y > lmax || y != y) ? y : lmax;
            }
            if (lane == 0) {
                const int64_t c1 = rb[r + 1] < d ? rb[r + 1] : d;
                const double dr = (double)(c1 > rb[r] ? c1 - rb[r] : 0);
                // scaled before the product: smax^2 alone overflows for rows near
                // 2^512 whose Gram (and this bound) are finite.  Three digits:
                // 2^-21 (2 S L1 + 2.03 d S^2); two digits (three products):
                // 2^-14 (2 S L1 + 1.0001 d S^2) -- the dropped a1 b1 2^-26 term
                // and the remainders rho (|rho| <= 2^-14), DESIGN.md §4 K1i8
                term[r - r0] = ns == 3 ? (0x1p-21 * smax) * (2.0 * lmax + 2.03 * dr * smax)
                                       : (0x1p-14 * smax) * (2.0 * lmax + 1.0001 * dr * smax);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int r = r0; r < r1; ++r) tot += term[r - r0];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = (tot == tot && tot < __builtin_inf()) ? tot * (1.0 + 0x1p-20)
                                                                         : __builtin_inf();
}

// ---------------------------------------------------------------------------
// the int8 Gram: one 128 x TJ tile of one range per workgroup
// ---------------------------------------------------------------------------
__device__ __forceinline__ int i8_swz(int row, int g) { return g ^ ((row >> 2) & 3); }

// NS digit planes, NBJ 32-column blocks per wave along the tile's columns:
//   <3, 2>  128 x 128 tiles, the six products of weight >= 2^-26 (three
//           accumulator levels, 192 int32 per lane)
//   <2, 4>  128 x 256 tiles, the three products of weight >= 2^-19
//           (BK_F32_I8X2: L0 = A0 A0^T, L1 = A0 A1^T + A1 A0^T; two levels,
//           256 int32 per lane)
// Both stage 48 KiB per 64-column chunk (NS (128 + TJ) rows of 64 B) and run
// 24 MFMAs against 12 fragment reads per 32-column k-step and wave, so the
// two-digit tile does the same instruction stream per chunk for twice the
// output elements and half the products each.
// NW: waves per workgroup, 4 (one per SIMD) or 8 (two per SIMD: while one
// wave waits on its LDS fragment reads or the barrier, the other issues
// MFMAs); the waves tile the output 2 x NW/2, each 64 x 32 NBJ.
template <int NS, int NBJ, int NW = 4>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4)))
void k_gram_i8(const int8_t *__restrict__ S, int64_t dp, int64_t plane,
               const int64_t *__restrict__ rb, int R, const int2 *__restrict__ order,
               const int *__restrict__ es, int n, int T64, double *__restrict__ part,
               int64_t ntile64, PieceMarks pm) {
    constexpr int NT = 64 * NW;                        // threads
    constexpr int TJ = (NW / 2) * 32 * NBJ;            // the tile's columns (rows of operand B)
    constexpr int NGR = I8_STAGE / 16 / NT;            // 16-B granules each thread stages per chunk
    constexpr int NMF = (NS == 3 ? 6 : 3) * 2 * NBJ;   // MFMAs per k-step and wave
    constexpr int NRD = NS * (2 + NBJ);                // fragment reads per k-step and wave
    constexpr int NL = NS;                             // accumulator levels
    constexpr int NP = NS == 3 ? 6 : 3;                // digit products
    constexpr int A_BYTES = NS * I8_TILE * I8_KC;      // operand A (the tile's rows) per stage
    constexpr int B_PLANE = TJ * I8_KC;
    static_assert(A_BYTES + NS * B_PLANE == I8_STAGE, "48 KiB stages");
    static_assert(NW == 4 ? (NMF == 24 && NRD == 12 && NGR == 12) : (NW == 8 && NGR == 6),
                  "4 waves: 24 MFMAs per 12 reads, 12 granules; 8 waves: 6 granules");
    extern __shared__ __attribute__((aligned(16))) int8_t lds[];  // two stages of I8_STAGE bytes
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // this workgroup's item: its tile (row block I of 128, column block J of
    // TJ: I | J << 16) and column range (i8_layout; r < 0: a padding workgroup
    // of a short XCD list)
    const bool wt = piece_handed(pm) && !pm.nowt;  // the partials go to the communication stream
    const int2 item = order[blockIdx.x];
    if (item.y < 0) {
        piece_done(pm);
        return;
    }
    const int r = item.y, I = item.x & 0xffff, J = item.x >> 16;
    const int64_t k0 = rb[r], k1 = rb[r + 1];
    const int nch = (int)((k1 - k0) / I8_KC);
    // staging: granule q = tid + NT u (u < NGR) of the chunk: q < 512 NS is
    // operand A (digit q >> 9, row (q >> 2) & 127), the rest operand B (digit
    // q' / (4 TJ), row (q' >> 2) % TJ); g = q & 3 the 16-B granule of the row
    const int8_t *src[NGR];
    int dst[NGR];
#pragma unroll
    for (int u = 0; u < NGR; ++u) {
        const int q = tid + NT * u;
        const int g = q & 3;
        int t, row, grow, off;
        if (q < 512 * NS) {
            t = q >> 9;
            row = (q >> 2) & 127;
            grow = I * I8_TILE + row;
            off = t * I8_TILE * I8_KC;
        } else {
            const int qb = q - 512 * NS;
            t = qb / (4 * TJ);
            row = (qb >> 2) % TJ;
            grow = J * TJ + row;
            off = A_BYTES + t * B_PLANE;
        }
        src[u] = S + (int64_t)t * plane + i8_off(grow, k0 + 16 * g, dp);
        dst[u] = off + row * I8_KC + 16 * i8_swz(row, g);
    }
    v4i pf[NGR];
    // BK_I8_ABL (timing-only ablations, tools/ builds; the product is 0): 1 =
    // every chunk fetch from the range's first 4 chunks (L2-resident: no HBM /
    // Infinity Cache latency), 2 = no LDS stores, 3 = no fragment reads, 4 = no MFMAs
    auto fetch = [&](int ch) {
        if constexpr (BK_I8_ABL == 1) ch &= 3;
#pragma unroll
        for (int u = 0; u < NGR; ++u) pf[u] = *reinterpret_cast<const v4i *>(src[u] + (int64_t)ch * I8_CHUNK_STRIDE);
    };
    auto put = [&](int8_t *b) {
        if constexpr (BK_I8_ABL == 2) {
            if (nch > 1000000) b[dst[0]] = (int8_t)pf[0][0];  // keep the loads
            return;
        }
#pragma unroll
        for (int u = 0; u < NGR; ++u) *reinterpret_cast<v4i *>(b + dst[u]) = pf[u];
    };
    v16i acc[NL][2][NBJ];
#pragma unroll
    for (int l = 0; l < NL; ++l)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < NBJ; ++b) acc[l][a][b] = v16i{};
    const int wr = (wave & 1) * 64, wc = (wave >> 1) * (32 * NBJ);  // this wave's 64 x 32 NBJ
    const int fr = lane & 31, fh = lane >> 5;
    // the fragments of k-step ks (32 columns: granules 2 ks + fh) of stage b
    auto frags = [&](const int8_t *b, int ks, v4i (&fa)[NS][2], v4i (&fb)[NS][NBJ]) {
        if constexpr (BK_I8_ABL == 3) {
            if (ks == 0 && b == nullptr) fa[0][0] = v4i{1, 1, 1, 1};  // (never) the registers as they are
            return;
        }
        const int g = 2 * ks + fh;
#pragma unroll
        for (int t = 0; t < NS; ++t) {
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int ra = wr + 32 * a + fr;
                fa[t][a] = *reinterpret_cast<const v4i *>(b + t * I8_TILE * I8_KC + ra * I8_KC +
                                                          16 * i8_swz(ra, g));
            }
#pragma unroll
            for (int bb = 0; bb < NBJ; ++bb) {
                const int rbw = wc + 32 * bb + fr;
                fb[t][bb] = *reinterpret_cast<const v4i *>(b + A_BYTES + t * B_PLANE + rbw * I8_KC +
                                                           16 * i8_swz(rbw, g));
            }
        }
    };
    // the digit products of one k-step {level, A digit, B digit}, product-major
    // over the blocks: consecutive MFMAs never accumulate into the same
    // registers.  (Measured neutral against block-major chains at config E.)
    auto mma = [&](const v4i (&fa)[NS][2], const v4i (&fb)[NS][NBJ]) {
        if constexpr (BK_I8_ABL == 4) {
            acc[0][0][0][0] += fa[0][0][0] ^ fb[0][0][1];  // keep the reads
            return;
        }
        constexpr int PT[6][3] = {{0, 0, 0}, {1, 0, 1}, {1, 1, 0}, {2, 0, 2}, {2, 1, 1}, {2, 2, 0}};
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int bb = 0; bb < NBJ; ++bb)
                    acc[PT[p][0]][a][bb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
                        fa[PT[p][1]][a], fb[PT[p][2]][bb], acc[PT[p][0]][a][bb], 0, 0, 0);
    };
    // Software pipeline at k-step granularity, one wave per SIMD: the MFMAs
    // always run from registers while the same instruction stream moves the
    // next operands, one memory instruction per MFMA gap (sched_group_barrier),
    // so the matrix pipe does not wait on LDS.  Per chunk ch:
    //   phase A: MFMAs of k-step 0 (F0)  | LDS reads of k-step 1 -> F1
    //   barrier: every wave has read all of chunk ch and stored chunk ch + 1
    //   phase B: MFMAs of k-step 1 (F1)  | LDS reads of chunk ch + 1's k-step 0
    //            -> F0, chunk ch + 2 (fetched one chunk earlier) stored into
    //            chunk ch's stage, chunk ch + 3 fetched
    // Chunk indices past the range are clamped (a stage nobody reads again
    // gets a stale copy; the last chunk is fetched again): no branch.
    if (nch > 0) {
        v4i F0a[NS][2], F0b[NS][NBJ], F1a[NS][2], F1b[NS][NBJ];
        const auto cl = [&](int c) { return c < nch ? c : nch - 1; };
        fetch(0);
        put(lds);
        fetch(cl(1));
        put(lds + I8_STAGE);
        fetch(cl(2));
        __syncthreads();
        frags(lds, 0, F0a, F0b);
        // chunk ch from stage C; chunk ch + 1 is in stage N, chunk ch + 2 goes
        // to C.  __restrict__: the stages never overlap, so the compiler may
        // interleave C's stores with N's reads (and both with the MFMAs)
        auto body = [&](int ch, int8_t *__restrict__ C, const int8_t *__restrict__ N) {
            mma(F0a, F0b);
            frags(C, 1, F1a, F1b);
            if constexpr (NW == 4) {
#pragma unroll
                for (int q = 0; q < 12; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                }
            } else {  // the reads first (the other wave of the SIMD covers their latency)
#pragma unroll
                for (int q = 0; q < NMF; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (q < NRD) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // no motion across the phases
            __syncthreads();
            mma(F1a, F1b);
            frags(N, 0, F0a, F0b);
            put(C);
            fetch(cl(ch + 3));
            if constexpr (NW == 4) {
#pragma unroll
                for (int q = 0; q < 12; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
                    __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
                }
            } else {
#pragma unroll
                for (int q = 0; q < NMF; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (q < NGR) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                    if (q < NRD) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    if (q < NGR) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        for (int ch = 0; ch < nch; ++ch)
            body(ch, lds + (ch & 1) * I8_STAGE, lds + ((ch + 1) & 1) * I8_STAGE);
    }
    // epilogue: C/D lane l, reg e of a 32 x 32 block: row (e & 3) + 8 (e >> 2) + 4 (l >> 5), col l & 31.
    // Three digits: G = s_i s_j 2^-26 (2^14 L0 + 2^7 L1 + L2); two: s_i s_j 2^-19 (2^7 L0 + L1)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < NBJ; ++bb) {
            const int gj = J * TJ + wc + 32 * bb + fr;
            const int bj = gj >> 6;
            const int ej = gj < n ? es[(int64_t)gj * R + r] : 0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int gi = I * I8_TILE + wr + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * fh;
                const int bi = gi >> 6;
                if (bi > bj || bj >= T64) continue;  // the lower half of a diagonal tile; padding
                const int ei = gi < n ? es[(int64_t)gi * R + r] : 0;
                double v;
                int sh;
                if constexpr (NS == 3) {
                    v = (double)acc[0][a][bb][e] * 16384.0 + (double)acc[1][a][bb][e] * 128.0 +
                        (double)acc[2][a][bb][e];
                    sh = -26;
                } else {
                    v = (double)acc[0][a][bb][e] * 128.0 + (double)acc[1][a][bb][e];
                    sh = -19;
                }
                const int64_t u = (int64_t)bi * T64 - (int64_t)bi * (bi - 1) / 2 + (bj - bi);
                st_part(&part[((int64_t)r * ntile64 + u) * 4096 + (gi & 63) * 64 + (gj & 63)],
                        (ei == I8_NONFINITE || ej == I8_NONFINITE) ? __builtin_nan("") : ldexp(v, ei + ej + sh),
                        wt);
            }
        }
    piece_done(pm);
}

// U = sum over the R ranges, in order; the trailing record {d, 0, bound, 0}
// (e0 / e1 / rec: one piece of the packed upper when the exchange overlaps
// the Gram -- the same sums, the record only with the last piece)
__global__ __launch_bounds__(256) void k_i8_reduce(const double *__restrict__ part, int R,
                                                   int64_t usz, double *__restrict__ U, double d,
                                                   const double *__restrict__ bound, int64_t e0,
                                                   int64_t e1, int rec) {
    const int64_t e = e0 + ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (e < e1) {
        // ranges in order, 8 loads in flight per thread (R is a multiple of 8)
        d2v acc = *reinterpret_cast<const d2v *>(part + e);
        for (int r0 = 1; r0 < R; r0 += 8) {
            d2v v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                v[u] = r0 + u < R ? __builtin_nontemporal_load(reinterpret_cast<const d2v *>(
                                        part + (int64_t)(r0 + u) * usz + e))
                                  : d2v{0.0, 0.0};
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (r0 + u < R) {
                    acc.x += v[u].x;
                    acc.y += v[u].y;
                }
        }
        *reinterpret_cast<d2v *>(U + e) = acc;
    }
    if (rec && blockIdx.x == 0 && threadIdx.x == 0) {
        U[usz] = d;
        U[usz + 1] = 0.0;
        U[usz + 2] = bound[0];
        U[usz + 3] = 0.0;
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// R column ranges: at least one per XCD, and as many more (in eights) as keep
// a row's slice of a range within 128 KiB, so k_i8_slice holds it in
// registers (config E, fp32: 8 ranges of 32,768 columns; config D, fp64: 64 of
// 16,384); <= 32,768 columns per range keeps every int32 sum exact.  Then, if
// the (tile, range) items leave the last round of workgroups on an XCD well
// short of full, R is raised (in eights, up to 4x, ranges >= 16 chunks) to the
// count that fills the rounds (config D: 10 tiles x 64 ranges = 2.5 rounds of
// 32 CUs per XCD -> 128 ranges, 5 rounds; config E stays at 8: 16.5 of 17)
#ifndef BK_I8_RQ
#define BK_I8_RQ 8  // column ranges come in multiples of this (A/B builds)
#endif
// The workgroup order of a tile list over R ranges.  Workgroup b runs on XCD
// b mod 8 (dispatch order; speed only).  Every XCD sweeps the ranges in the
// same order, taking a contiguous piece of the tile order per range (ceil or
// floor of NT / 8 tiles, the extra tiles rotating over the XCDs so the totals
// balance): at any time the whole chip works on one column range, so the
// digit lines one XCD fetches are found in the Infinity Cache by the others,
// while each XCD's concurrent tiles stay compact (few row-blocks per chunk in
// its L2)
static std::vector<int> i8_sweep_order(const std::vector<int> &tiles, int R) {
    std::vector<int> order;
    const int NT = (int)tiles.size();
#if BK_I8_MAP == 0
    // r3/r4a: workgroup b runs range b mod R (= its XCD when R = 8) and tile b / R
    for (int b = 0; b < NT * R; ++b) {
        order.push_back(tiles[b / R]);
        order.push_back(b % R);
    }
#else
    std::vector<std::vector<int>> per(8);
    for (int r = 0; r < R; ++r) {
        const int q = NT / 8, rem = NT % 8;
        int j = 0;
        for (int x = 0; x < 8; ++x) {
            const int cnt = q + (((x - r) % 8 + 8) % 8 < rem ? 1 : 0);
            for (int k = 0; k < cnt; ++k, ++j) {
                per[x].push_back(tiles[j]);
                per[x].push_back(r);
            }
        }
    }
    size_t mx = 0;
    for (auto &v : per) mx = std::max(mx, v.size() / 2);
    for (size_t sidx = 0; sidx < mx; ++sidx)
        for (int x = 0; x < 8; ++x) {
            const bool on = sidx < per[x].size() / 2;
            order.push_back(on ? per[x][2 * sidx] : 0);
            order.push_back(on ? per[x][2 * sidx + 1] : -1);
        }
#endif
    return order;
}

I8Layout i8_layout(int n, int64_t d, int es, int num_cu, int ns) {
    I8Layout L;
    L.ns = ns == 2 ? 2 : 3;
    L.tj = L.ns == 2 ? 256 : I8_TILE;  // k_gram_i8<2, 4>: 128 x 256 tiles
    L.npad = (n + L.tj - 1) / L.tj * L.tj;
    L.dp = (d + I8_KC - 1) / I8_KC * I8_KC;
    const int64_t nk = L.dp / I8_KC;
    const int64_t cmax = I8_RANGE_BYTES / es;  // columns per range
    // the output tiles: row block I of 128, column block J of tj, every tile
    // holding some element of the upper triangle (128 I <= tj J + tj - 1) and
    // no tile past the last row; super-blocked (4 row blocks x 512 columns,
    // row by row) so consecutive tiles share row blocks
    const int TI = (n + I8_TILE - 1) / I8_TILE, TJn = (n + L.tj - 1) / L.tj, rj = L.tj / I8_TILE;
    const int SBI = BK_I8_SBI, SBJ = BK_I8_SBC / rj > 0 ? BK_I8_SBC / rj : 1;
    std::vector<int> tiles;  // I | J << 16
    for (int BI = 0; BI < (TI + SBI - 1) / SBI; ++BI)
        for (int BJ = 0; BJ < (TJn + SBJ - 1) / SBJ; ++BJ)
            for (int I = BI * SBI; I < BI * SBI + SBI && I < TI; ++I)
                for (int J = BJ * SBJ; J < BJ * SBJ + SBJ && J < TJn; ++J)
                    if (I <= rj * J + rj - 1) tiles.push_back(I | J << 16);
    const int NT = (int)tiles.size();
    const int64_t R0 = (L.dp + cmax - 1) / cmax;  // the fewest ranges the slice width allows
    int64_t R = (R0 + BK_I8_RQ - 1) / BK_I8_RQ * BK_I8_RQ;
    R = nk < R ? nk : R;
    const int ncu = num_cu > 0 ? num_cu : 256;
    if (R0 < BK_I8_RQ) {
        // short rows (one rank's shard of a d-sharded call, e.g. E at 8 GPUs:
        // 32,768 columns): every range of a tile is one workgroup that pays a
        // fixed cost (pipeline fill, the 128 x tj partial it writes, its share
        // of k_i8_reduce), so fewer, longer ranges win until the grid gets
        // short of workgroups.  cost(R) = workgroup rounds x (columns per
        // range + C0) + C1 R, in columns, C1 growing as the n^2 partials each
        // range adds to k_i8_reduce; C0 = 2048 and C1 = 3072 at n = 4096
        // fitted over E's 8- and 4-rank shards, two and three digits
        // (profiles/r05/ab_i8_ranges.log: within 2 % of the best R measured,
        // 1.1-1.5x faster than the 8 ranges of before)
        const double c1 = 3072.0 * ((double)n / 4096.0) * ((double)n / 4096.0);
        auto cost = [&](int64_t r) {
            const double rounds = std::ceil((double)NT * r / ncu);
            return rounds * ((double)L.dp / r + 2048.0) + c1 * r;
        };
        int64_t best = R0;
        for (int64_t r = R0 + 1; r <= BK_I8_RQ && r <= nk; ++r)
            if (cost(r) < cost(best)) best = r;
        R = best;
    } else {
        const double cx = num_cu > 0 ? num_cu / 8.0 : 32.0;  // CUs per XCD
        auto eff = [&](int64_t r) {
            const double rounds = (double)((NT * r + 7) / 8) / cx;
            return rounds / std::ceil(rounds);
        };
        int64_t best = R;
        for (int64_t r = R + BK_I8_RQ; r <= 4 * R && nk / r >= 16; r += BK_I8_RQ)
            if (eff(r) > eff(best) + 0.05) best = r;
        R = best;
    }
#ifdef BK_I8_RFIX
    R = BK_I8_RFIX < nk ? BK_I8_RFIX : nk;  // A/B builds: a fixed range count
#endif
    L.R = (int)R;
    L.es = es;
    L.rb.resize(L.R + 1);
    for (int r = 0; r <= L.R; ++r) L.rb[r] = nk * r / L.R * I8_KC;
    L.plane = (int64_t)L.npad * L.dp;
    L.T128 = L.npad / I8_TILE;
    L.T64 = (n + 63) / 64;
    L.ntile64 = (int64_t)L.T64 * (L.T64 + 1) / 2;
    L.tiles = tiles;
    L.order = i8_sweep_order(tiles, L.R);
    return L;
}

bool i8_pieces(const I8Layout &L, int k, std::vector<int> &tile_end,
               std::vector<std::vector<int>> &orders) {
    // 128-row blocks: weight = the tiles of the block row; every cut is valid
    const int TI = (L.T64 + 1) / 2;  // 128-row blocks holding rows
    std::vector<double> w((size_t)TI, 0.0);
    for (int t : L.tiles) w[(size_t)(t & 0xffff)] += 1.0;
    std::vector<char> valid((size_t)TI, 1);
    const std::vector<int> cut = piece_cuts(w, valid, k);
    if ((int)cut.size() != k - 1) return false;
    tile_end.clear();
    orders.clear();
    int I0 = 0;
    for (int p = 0; p < k; ++p) {
        const int I1 = p + 1 < k ? cut[(size_t)p] : TI;
        std::vector<int> sub;
        for (int t : L.tiles)
            if ((t & 0xffff) >= I0 && (t & 0xffff) < I1) sub.push_back(t);
        orders.push_back(i8_sweep_order(sub, L.R));
        // the packed upper's 64 x 64 sub-tiles of rows [0, 128 I1): rows of
        // 64-row blocks b < 2 I1 (clipped to the last block)
        const int64_t b1 = std::min<int64_t>(2 * (int64_t)I1, L.T64);
        tile_end.push_back((int)(b1 * L.T64 - b1 * (b1 - 1) / 2));
        I0 = I1;
    }
    return true;
}

size_t i8_workspace(const I8Layout &L) {
    // digit planes, rb, order, exponents, norms, bound, range partials
    return (size_t)L.ns * L.plane + 256 + (size_t)(L.R + 1) * 8 + L.order.size() * 4 + 256 +
           (size_t)L.npad * L.R * (4 + 8) + 256 + 256 +
           (size_t)L.R * L.ntile64 * 4096 * 8 + 256;
}

hipError_t configure_i8_kernels() {
    hipError_t e = hipFuncSetAttribute((const void *)k_gram_i8<3, I8_NBJ3, BK_I8_W3>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, I8_LDS);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute((const void *)k_gram_i8<2, I8_NBJ2, BK_I8_W2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               I8_LDS);
}

static char *align256(char *p) { return (char *)(((uintptr_t)p + 255) & ~(uintptr_t)255); }

// the workspace's pieces (i8_workspace)
struct I8Ws {
    int8_t *S;
    int *es;
    double *l1, *bound, *part;
};
static I8Ws i8_ws(const I8Layout &L, void *ws) {
    I8Ws w;
    char *p = align256((char *)ws);
    w.S = (int8_t *)p;
    p = align256(p + (size_t)L.ns * L.plane);
    w.es = (int *)p;
    p = align256(p + (size_t)L.npad * L.R * 4);
    w.l1 = (double *)p;
    p = align256(p + (size_t)L.npad * L.R * 8);
    w.bound = (double *)p;
    p = align256(p + 256);
    w.part = (double *)p;
    return w;
}

hipError_t launch_i8_slice(const void *X, int dtype, int64_t ld, int n, int64_t d,
                           const I8Layout &L, void *ws, const void *tables, hipStream_t st) {
    const I8Ws w = i8_ws(L, ws);
    const int64_t *rb = (const int64_t *)tables;
    int64_t lmax = 0;  // the longest range: its row slice must fit the kernel's registers
    for (int r = 0; r < L.R; ++r) lmax = std::max<int64_t>(lmax, L.rb[r + 1] - L.rb[r]);
    if (lmax * L.es > I8_RANGE_BYTES) return hipErrorInvalidValue;
    const dim3 grid((unsigned)L.npad, (unsigned)L.R);
    const bool shortr = lmax <= 16 * 256;  // every range fits <256, 1>
    auto go = [&](auto tag, auto ns) {
        using T = decltype(tag);
        constexpr int NS = decltype(ns)::value;
        if (shortr)
            hipLaunchKernelGGL((k_i8_slice<T, NS, 256, 1>), grid, dim3(256), 0, st, (const T *)X, ld, n,
                               d, rb, L.R, w.S, L.dp, L.plane, w.es, w.l1);
        else
            hipLaunchKernelGGL((k_i8_slice<T, NS>), grid, dim3(I8_SLICE_NT), 0, st, (const T *)X, ld, n,
                               d, rb, L.R, w.S, L.dp, L.plane, w.es, w.l1);
    };
    using N2 = std::integral_constant<int, 2>;
    using N3 = std::integral_constant<int, 3>;
    if (dtype == 0 && L.ns == 2)
        go(double{}, N2{});
    else if (dtype == 0)
        go(double{}, N3{});
    else if (L.ns == 2)
        go(float{}, N2{});
    else
        go(float{}, N3{});
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_i8_bound, dim3(1), dim3(I8_BOUND_NT), 0, st, w.es, w.l1, rb, L.R, n, d, L.ns,
                       w.bound);
    return hipGetLastError();
}

hipError_t launch_i8_gemm(int n, const I8Layout &L, void *ws, const void *tables, hipStream_t st,
                          const void *order_p, int64_t items, const PieceMarks &pm) {
    const I8Ws w = i8_ws(L, ws);
    const int64_t *rb = (const int64_t *)tables;  // {rb (R + 1 int64), order (int pairs)}
    const int2 *order = order_p ? (const int2 *)order_p
                                : (const int2 *)((const char *)tables + (size_t)(L.R + 1) * 8);
    if (!order_p) items = (int64_t)L.order.size() / 2;  // one workgroup each
    if (items < 1) return hipSuccess;
    if (L.ns == 2)
        hipLaunchKernelGGL((k_gram_i8<2, I8_NBJ2, BK_I8_W2>), dim3((unsigned)items), dim3(64 * BK_I8_W2), I8_LDS, st, w.S, L.dp,
                           L.plane, rb, L.R, order, w.es, n, L.T64, w.part, L.ntile64, pm);
    else
        hipLaunchKernelGGL((k_gram_i8<3, I8_NBJ3, BK_I8_W3>), dim3((unsigned)items), dim3(64 * BK_I8_W3), I8_LDS, st, w.S, L.dp,
                           L.plane, rb, L.R, order, w.es, n, L.T64, w.part, L.ntile64, pm);
    return hipGetLastError();
}

hipError_t launch_i8_reduce(int64_t d, const I8Layout &L, void *ws, double *U, hipStream_t st,
                            int64_t e0, int64_t e1, bool rec) {
    const I8Ws w = i8_ws(L, ws);
    const int64_t usz = L.ntile64 * 4096;
    if (e1 < 0) e1 = usz;
    if (e1 <= e0) return hipSuccess;
    hipLaunchKernelGGL(k_i8_reduce, dim3((unsigned)(((e1 - e0) / 2 + 255) / 256)), dim3(256), 0, st,
                       w.part, L.R, usz, U, (double)d, w.bound, e0, e1, rec ? 1 : 0);
    return hipGetLastError();
}

}  // namespace bk
