// bk_kernels.hip -- CDNA4 (gfx950) kernels of the Multi-Krum engine.
//
// Pipeline for one Multi-Krum call (DESIGN.md "Kernels"):
//   K1  k_gram      split-K, upper-triangle fp64 Gram partials on
//                   v_mfma_f64_16x16x4_f64 (the -2XX^T term of
//                   logistic_validator.py:59-60; norms come from its diagonal)
//   K1b k_reduce    fixed-order sum of the split-K partials -> packed upper
//   K2  k_scores    per row: D_ij = (G_ii + G_jj) - 2 G_ij read straight from the
//                   packed upper tiles (no n x n expansion), bitonic sort in LDS
//                   (NaN last), sum of ranks 1..k      (logistic_validator.py:62-63)
//   K3  k_rank      rank of each score (ties -> lower index, NaN last), mask
//   K3b k_compact   mask -> ascending selected indices (argpartition set, :45)
//   K4  k_mean      masked mean of the selected rows, fp64, ascending order (:51)
//                   (ACCUM: the block aggregation GlobalW += sum, honest.go:361-375)
//
// Built with -ffp-contract=off: every non-MFMA add/mul rounds exactly as the
// numpy reference evaluates it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>

#include "bk_device.h"
#include "bk_internal.h"
#include "bk_synth.h"

namespace bk {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef double d4v __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------

// Bijective XCD remap (cdna_hip_programming.md T1): blocks b and b+8 share an
// XCD, so give each XCD a contiguous range of logical workgroups.  Speed only.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// upper-triangle sub-tile u -> (bi, bj), bi <= bj, T blocks per side
__device__ __forceinline__ void tri_decode(int u, int T, int &bi, int &bj) {
    int i = 0, off = 0;
    while (u >= off + (T - i)) { off += T - i; ++i; }
    bi = i;
    bj = i + (u - off);
}

template <typename T, bool VEC>
__device__ __forceinline__ d2v ld2(const T *p) {
    d2v r;
    if constexpr (std::is_same<T, double>::value) {
        if constexpr (VEC) {
            r = *reinterpret_cast<const d2v *>(p);
        } else {
            r.x = p[0];
            r.y = p[1];
        }
    } else {
        if constexpr (VEC) {
            const f2v v = *reinterpret_cast<const f2v *>(p);
            r.x = (double)v.x;
            r.y = (double)v.y;
        } else {
            r.x = (double)p[0];
            r.y = (double)p[1];
        }
    }
    return r;
}

// Streaming read of data used once (K4 and its aggregation variant): a
// non-temporal load.  K4 at config D: 0.549 -> 0.495 ms (5.5 -> 6.1 TB/s,
// profiles/r01/ab_mean_nt.log).  -DBK_NO_NT restores plain loads for A/B.
template <typename T, bool VEC>
__device__ __forceinline__ d2v ld2s(const T *p) {
#ifndef BK_NO_NT
    if constexpr (VEC && std::is_same<T, double>::value) {
        return __builtin_nontemporal_load(reinterpret_cast<const d2v *>(p));
    } else if constexpr (VEC) {
        const f2v v = __builtin_nontemporal_load(reinterpret_cast<const f2v *>(p));
        return d2v{(double)v.x, (double)v.y};
    }
#endif
    return ld2<T, VEC>(p);
}

// ---------------------------------------------------------------------------
// K1: split-K upper-triangle Gram on fp64 MFMA.
//
// One WAVE owns one task = (64x64 upper sub-tile u, k-piece s).  No LDS, no
// barriers: fp64 MFMA is 64 cycles per 16x16x4 on gfx950, so a wave's 16
// accumulators hide everything if operands arrive from a register ring P
// k-blocks deep.  The contraction index is permuted inside each 8-column
// k-block so that every lane loads 16 contiguous bytes per row:
//   lane l (rr = l&15, g = l>>4) holds X[row rr][kb*8 + 2g + s] for MFMA
//   sub-step s in {0,1}; A and B use the same permutation, so the product is
//   exactly X X^T (the order of the k-sum is a free choice, as in any BLAS).
// Output: acc[a][b] is the 16x16 block (a,b) of the sub-tile; element
// (row g + 4r, col rr) sits in register r (f64 MFMA C/D map,
// cdna_hip_programming.md §3).
// ---------------------------------------------------------------------------

template <typename T, bool VEC, bool DIAG>
__device__ __forceinline__ void gram_load(const T *(&pa)[4], const T *(&pb)[4],
                                          int64_t off, d2v (&a)[4], d2v (&b)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = ld2<T, VEC>(pa[i] + off);
    if constexpr (!DIAG) {
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = ld2<T, VEC>(pb[j] + off);
    }
}

template <bool DIAG>
__device__ __forceinline__ void gram_mma(d4v (&acc)[4][4], const d2v (&a)[4], const d2v (&b)[4]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (DIAG && j < i) continue;
                const double bv = DIAG ? a[j][s] : b[j][s];
                acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i][s], bv, acc[i][j], 0, 0, 0);
            }
        }
    }
}

template <typename T, bool VEC, bool DIAG, int P>
__device__ __forceinline__ void gram_task(const T *__restrict__ X, int64_t ld, int n, int rowA,
                                          int rowB, int64_t k0, int64_t k1, d4v (&acc)[4][4]) {
    const int lane = threadIdx.x & 63, rr = lane & 15, g = lane >> 4;
    const T *pa[4];
    const T *pb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int ra = min(rowA + i * 16 + rr, n - 1);
        pa[i] = X + (int64_t)ra * ld + k0 + 2 * g;
        const int rb = min(rowB + i * 16 + rr, n - 1);
        pb[i] = X + (int64_t)rb * ld + k0 + 2 * g;
    }
    const int64_t len = k1 - k0;
    const int64_t nb = len >> 3;
    const int64_t rem = nb % P;

    // (1) the first nb % P blocks, unpipelined, so the ring runs a multiple of P
    for (int64_t kb = 0; kb < rem; ++kb) {
        d2v a[4], b[4];
        gram_load<T, VEC, DIAG>(pa, pb, kb * 8, a, b);
        gram_mma<DIAG>(acc, a, b);
    }
    // (2) register ring, P k-blocks in flight
    if (nb > rem) {
        d2v ra[P][4], rb[P][4];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            gram_load<T, VEC, DIAG>(pa, pb, (rem + p) * 8, ra[p], rb[p]);
            __builtin_amdgcn_sched_barrier(0);  // issue stages in ring order
        }
        for (int64_t kb = rem; kb < nb; kb += P) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                gram_mma<DIAG>(acc, ra[p], rb[p]);
                int64_t nk = kb + P + p;
                nk = nk < nb ? nk : nb - 1;  // clamped re-load past the end keeps waits static
                gram_load<T, VEC, DIAG>(pa, pb, nk * 8, ra[p], rb[p]);
                // keep the prefetch here: without the fence the scheduler sinks it to
                // the top of the next trip and the ring degenerates to load-then-wait
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    // (3) ragged tail: len % 8 columns, guarded scalar loads
    if (len & 7) {
        const int64_t kt = nb * 8;
        d2v a[4], b[4];
        const bool v0 = kt + 2 * g < len, v1 = kt + 2 * g + 1 < len;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a[i].x = v0 ? (double)pa[i][kt] : 0.0;
            a[i].y = v1 ? (double)pa[i][kt + 1] : 0.0;
            b[i].x = v0 ? (double)pb[i][kt] : 0.0;
            b[i].y = v1 ? (double)pb[i][kt + 1] : 0.0;
        }
        gram_mma<DIAG>(acc, a, b);
    }
}

template <typename T, bool VEC, int P>
__global__ __launch_bounds__(256, 1) void k_gram(const T *__restrict__ X, int64_t ld, int n,
                                                 int64_t d, int T_, int ntile, int S, int64_t kc,
                                                 int nwg, double *__restrict__ part) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lwg = xcd_remap(blockIdx.x, nwg);
    const int task = lwg * 4 + wave;  // tasks are piece-major: task = s*ntile + u
    if (task >= ntile * S) return;    // wave-uniform
    const int s = task / ntile, u = task - s * ntile;
    int bi, bj;
    tri_decode(u, T_, bi, bj);
    const int64_t k0 = (int64_t)s * kc;
    const int64_t k1 = min(d, k0 + kc);

    d4v acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = d4v{0.0, 0.0, 0.0, 0.0};

    if (k1 > k0) {
        if (bi == bj)
            gram_task<T, VEC, true, P>(X, ld, n, bi * 64, bj * 64, k0, k1, acc);
        else
            gram_task<T, VEC, false, P>(X, ld, n, bi * 64, bj * 64, k0, k1, acc);
    }

    double *out = part + (int64_t)task * 4096;
    const int rr = lane & 15, g = lane >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) out[(i * 16 + g + 4 * r) * 64 + j * 16 + rr] = acc[i][j][r];
}

// ---------------------------------------------------------------------------
// K1 v3: LDS-shared split-K Gram (aligned fp64 input; the headline path).
//
// Workgroup = 8 waves (2 per SIMD), owns one (group, piece) of the host plan
// (bk_plan.hip): each wave runs one wave-task -- an off-diagonal 64x64
// sub-tile (128 accumulator registers), or the two diagonal sub-tiles of a
// 128-row super-block (upper 16x16 blocks only, 2 x 10 x 8 registers).  The
// group's <= 8 row-blocks are staged ONCE per workgroup through a 4-deep LDS
// ring filled by global_load_lds (16 B per lane, 1 KiB = 16 rows x 64 B per
// instruction, no VGPR staging, 3 k-blocks in flight).  Operands come back by
// ds_read_b128: lane (rr, g) of row-group q reads row 16q+rr, 16-byte granule
// g of the 8-column k-block = columns 2g, 2g+1 = MFMA sub-steps s = 0, 1 (the
// same k permutation for A and B, so the product is X X^T).  Granules are
// XOR-swizzled by (row >> 1) & 3 on the global SOURCE address (glds writes
// lane-linearly) and on the read: conflict-free for ds_read_b128.
// One s_barrier per 8-column k-block (64 MFMAs per SIMD in between).
// ---------------------------------------------------------------------------
typedef float f4v __attribute__((ext_vector_type(4)));
// One 16-byte LDS granule in the input type: 2 doubles or 4 floats.  A k-block
// is 8 granules (128 B) per row: 16 fp64 columns or 32 fp32 columns, so the
// LDS image, swizzle and glds shape are the same for both input types.
template <typename T>
struct G3T;
// op / acc: MFMA operand and accumulator types; F32C: the fp32 MFMA, whose
// C/D map is row = 4*(lane>>4) + reg (the f64 one is (lane>>4) + 4*reg)
template <>
struct G3T<double> {
    typedef d2v gran;
    typedef double op;
    typedef d4v acc;
    static constexpr int SUB = 2;   // MFMA sub-steps (k=4 each) per granule
    static constexpr bool F32C = false;
    static __device__ __forceinline__ double at(const d2v &v, int s) { return v[s]; }
    static __device__ __forceinline__ d4v mma(double a, double b, d4v c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
};
template <>
struct G3T<float> {
    typedef f4v gran;
    typedef double op;
    typedef d4v acc;
    static constexpr int SUB = 4;
    static constexpr bool F32C = false;
    // fp32 -> fp64 is exact, and so is every fp32 x fp32 product in fp64
    static __device__ __forceinline__ double at(const f4v &v, int s) { return (double)v[s]; }
    static __device__ __forceinline__ d4v mma(double a, double b, d4v c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
};
// fp32 rows on the fp32 MFMA (bk_set_f32_mode(ctx, BK_F32_MFMA), config E's
// "fp32 MFMA path"): products rounded to fp32 and summed in fp32 within one
// workgroup segment; the segments' partial slabs are summed in fp64 (K1b)
template <>
struct G3T<f32m> {
    typedef f4v gran;
    typedef float op;
    typedef f4v acc;
    static constexpr int SUB = 4;
    static constexpr bool F32C = true;
    static __device__ __forceinline__ float at(const f4v &v, int s) { return v[s]; }
    static __device__ __forceinline__ f4v mma(float a, float b, f4v c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
};
// output row of accumulator register r of lane group g in a 16x16 block
template <typename T>
__device__ __forceinline__ constexpr int g3_crow(int g, int r) {
    return G3T<T>::F32C ? 4 * g + r : g + 4 * r;
}

template <typename T>
__device__ __forceinline__ typename G3T<T>::gran g3_frag(const char *lds_blk, int q, int h, int rr,
                                                         int g) {
    const int row = q * 16 + rr;
    return *reinterpret_cast<const typename G3T<T>::gran *>(lds_blk + row * 128 +
                                                            16 * ((4 * h + g) ^ (row & 7)));
}

__device__ __forceinline__ void g3_wait(int vm) {
    switch (vm) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    }
}

// the same with the count known at compile time: one instruction, no branch tree
template <int N>
__device__ __forceinline__ void g3_waitc() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void g3_barrier() {
    // every wave's glds for the stage have landed (each waited for its own)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// diagonal sub-tile: upper 16x16 blocks (i <= j) in a flat array of 10
__device__ __forceinline__ constexpr int dix(int i, int j) { return i * 4 - i * (i - 1) / 2 + (j - i); }

template <int KIND, typename V>
struct G3Acc;
template <typename V>
struct G3Acc<T_OFF, V> {
    V a[4][4];
};
template <typename V>
struct G3Acc<T_PAIR, V> {
    V a[10], b[10];
};
template <typename V>
struct G3Acc<T_DIAG1, V> {
    V a[10];
};

// SKIP: leave block (0,3) to the OFF wave that took it (balanced band quads)
template <typename T, bool SKIP = false>
__device__ __forceinline__ void diag_mma(typename G3T<T>::acc (&acc)[10], const d2v (&a)[4]) {
    typedef typename G3T<T>::op O;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i; j < 4; ++j) {
                if (SKIP && i == 0 && j == 3) continue;
                acc[dix(i, j)] = G3T<T>::mma((O)a[i][s], (O)a[j][s], acc[dix(i, j)]);
            }
}
// the ragged-tail OFF product from direct loads (values exact in op)
template <typename T>
__device__ __forceinline__ void off_mma_tail(typename G3T<T>::acc (&acc)[4][4], const d2v (&a)[4],
                                             const d2v (&b)[4]) {
    typedef typename G3T<T>::op O;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = G3T<T>::mma((O)a[i][s], (O)b[j][s], acc[i][j]);
}
// the same over one granule of either input type
template <typename T, bool SKIP = false>
__device__ __forceinline__ void diag_mma_g(typename G3T<T>::acc (&acc)[10],
                                           const typename G3T<T>::gran (&a)[4]) {
#pragma unroll
    for (int s = 0; s < G3T<T>::SUB; ++s) {
        typename G3T<T>::op v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = G3T<T>::at(a[i], s);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i; j < 4; ++j) {
                if (SKIP && i == 0 && j == 3) continue;
                acc[dix(i, j)] = G3T<T>::mma(v[i], v[j], acc[dix(i, j)]);
            }
    }
}

template <typename T>
__device__ __forceinline__ void g3_load_rows(d2v (&a)[4], const T *__restrict__ X, int64_t ld,
                                             int n, int b, int64_t c, int64_t d, int rr) {
    // guarded direct loads for the ragged tail (c = first column of this lane)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const T *pr = X + (int64_t)min(b * 64 + q * 16 + rr, n - 1) * ld;
        a[q].x = c < d ? (double)pr[c] : 0.0;
        a[q].y = c + 1 < d ? (double)pr[c + 1] : 0.0;
    }
}

// (wt: write-through stores, a piece handed to the communication stream --
// bk_internal.h piece_done)
template <typename T = double>
__device__ __forceinline__ void store_tile(double *out, const typename G3T<T>::acc (&acc)[4][4],
                                           int rr, int g, bool wt = false) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                st_part(&out[(i * 16 + g3_crow<T>(g, r)) * 64 + j * 16 + rr], (double)acc[i][j][r], wt);
}

template <typename T, bool SKIP = false>
__device__ __forceinline__ void store_diag(double *out, const typename G3T<T>::acc (&acc)[10],
                                           int rr, int g, bool wt = false) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (SKIP && i == 0 && j == 3) continue;  // written by the OFF wave that took it
#pragma unroll
            for (int r = 0; r < 4; ++r)
                st_part(&out[(i * 16 + g3_crow<T>(g, r)) * 64 + j * 16 + rr],
                        j >= i ? (double)acc[dix(i, j)][r] : 0.0, wt);
        }
}

// one MFMA sub-step S (element S of each lane's granule) of an off-diagonal
// tile; XT = 1 / 2: also block (0,3) of the diagonal tile of the A / B row-block
// (operands already in registers: fragments 0 and 3 of that side)
template <typename T, int S, int XT = 0>
__device__ __forceinline__ void off_mma(typename G3T<T>::acc (&acc)[4][4],
                                        const typename G3T<T>::gran (&a)[4],
                                        const typename G3T<T>::gran (&b)[4],
                                        typename G3T<T>::acc &x) {
    typename G3T<T>::op va[4], vb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        va[i] = G3T<T>::at(a[i], S);
        vb[i] = G3T<T>::at(b[i], S);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[i][j] = G3T<T>::mma(va[i], vb[j], acc[i][j]);
    if constexpr (XT == 1) x = G3T<T>::mma(va[0], va[3], x);
    if constexpr (XT == 2) x = G3T<T>::mma(vb[0], vb[3], x);
}
// all SUB sub-steps of one granule
template <typename T, int XT = 0>
__device__ __forceinline__ void off_mma_gran(typename G3T<T>::acc (&acc)[4][4],
                                             const typename G3T<T>::gran (&a)[4],
                                             const typename G3T<T>::gran (&b)[4],
                                             typename G3T<T>::acc &x) {
    off_mma<T, 0, XT>(acc, a, b, x);
    off_mma<T, 1, XT>(acc, a, b, x);
    if constexpr (G3T<T>::SUB == 4) {
        off_mma<T, 2, XT>(acc, a, b, x);
        off_mma<T, 3, XT>(acc, a, b, x);
    }
}
// STAG: waves 4-7 (the SIMD partners of waves 0-3) run their OFF tile half a
// k-block behind -- the second 8-column half of block t-1 is issued after the
// barrier of block t, from registers -- so that after every barrier one wave
// of each SIMD has MFMAs ready while its partner waits for its LDS reads.  The
// accumulation order (block by block, column by column) is unchanged, so the
// result is bitwise identical to the unstaggered schedule.
// BK_K1_PROBE (debug builds only): shader cycles spent in the vmcnt wait and
// in the barrier, per wave, reported through the BK_TRACE_FILE timeline
#ifdef BK_K1_PROBE
#define G3_PROBE(v) const long long v = (long long)__builtin_readcyclecounter()
#else
#define G3_PROBE(v) const long long v = 0
#endif
// NB > 0: the group stages exactly NB row-blocks (compile time: a single
// s_waitcnt and straight-line glds); NB = 0: read G.nb at run time.
// XT (balanced band quads, GroupDesc::xt): OFF 1 / 2 = also block (0,3) of the
// A / B row-block's diagonal tile, stored into xout (the PAIR wave's slab);
// PAIR 1 = skip that block in both diagonal tiles
template <typename T, int KIND, int MODE, bool STAG, int NB, int XT = 0>
__device__ __forceinline__ void g3_wave(const T *__restrict__ X, int64_t ld, int n, int nfull,
                                        int64_t d, const GroupDesc &G, const int *wd, char *lds,
                                        int wave, int lane, double *out, long long (&probe)[2],
                                        double *xout = nullptr, bool wt = false) {
    constexpr int XO = KIND == T_OFF ? XT : 0;     // OFF: extra block side
    constexpr bool XP = KIND == T_PAIR && XT != 0;  // PAIR: skip block (0,3)
    typedef typename G3T<T>::gran gran;
    constexpr int EPG = 16 / (int)sizeof(T);  // elements per 16-B granule
    constexpr int BKE = 8 * EPG;               // columns per k-block (16 fp64, 32 fp32)
    const int rr = lane & 15, g = lane >> 4;
    int blk[G3_MAXB];
#pragma unroll
    for (int b = 0; b < G3_MAXB; ++b) blk[b] = G.blk[b];
    const int c = NB > 0 ? NB : G.nb;  // glds per wave per k-block (8 per row-block, 8 waves)
    const int sA = G.task[wave][1], sB = G.task[wave][2];
    const int kst = wd[1], kstr = wd[2], kend = wd[3];
    const int nk = kst < kend ? (kend - 1 - kst) / kstr + 1 : 0;

    // this wave's c (<= 6) glds per k-block: fixed per-lane row pointers and LDS
    // offsets; a stage only adds the k-block's column.  Instruction i of a stage
    // moves rows 8ii..8ii+7 (128 B each) of slot b = i/8; lane L takes row
    // 8ii + L/8, granule (L&7) of the LDS row <- global granule (L&7)^(row&7).
    // ESPL: waves 0-3 issue NB + ESPL of the stage's 8 NB glds and waves 4-7
    // NB - ESPL.  The timeline probe shows waves 0-3 waiting ~2,400-2,600
    // cycles per k-block at the barrier and the staggered waves 4-7 ~100: the
    // latter are the critical path, and each glds costs its wave ~100-185
    // cycles of issue.  Super pairs 6 -> 8 / 4, quads 4 -> 6 / 2: K1 at D
    // 4.07 -> 4.00 ms, the 8-GPU shard and C unchanged (profiles/r01/ab_gldssplit.log);
    // -DBK_GLDS_E6=0 -DBK_GLDS_E4=0 restores the even split.
#ifndef BK_GLDS_E6
#define BK_GLDS_E6 2
#endif
#ifndef BK_GLDS_E4
#define BK_GLDS_E4 2
#endif
    // the fp32-MFMA kernel runs unstaggered, so its waves split evenly (the
    // uneven split put the band quads' loop at 0.65 there, even 0.905)
    constexpr int ESPL = G3T<T>::F32C ? 0 : NB == 6 ? BK_GLDS_E6 : NB == 4 ? BK_GLDS_E4 : 0;
    constexpr int CLO = NB + ESPL, CHI = NB - ESPL;
    constexpr int GMAX = G3_MAXB + 2;
    static_assert(CLO <= GMAX && CHI >= 0, "glds split exceeds the per-wave pointer table");
    const bool hi = wave >= 4;
    const T *gsrc[GMAX];
    int gdst[GMAX];
    {
        const int rq = lane >> 3, j = lane & 7;
#pragma unroll
        for (int m = 0; m < GMAX; ++m) {
            int i = wave + 8 * m;
            if constexpr (ESPL != 0) {
                i = hi ? 4 * CLO + (wave - 4) + 4 * m : wave + 4 * m;
                if (i >= 8 * NB) i = 0;  // beyond this wave's count: never issued
            }
            const int b = i >> 3, ii = i & 7;
            const int rl = ii * 8 + rq;
#ifdef BK_K1_SAMEROWS  // timing-only ablation: every slot reads row-block 0 (all L2 hits)
            const int grow = min(rl, n - 1);
#else
            const int grow = min(blk[b] * 64 + rl, n - 1);
#endif
            gsrc[m] = X + (int64_t)grow * ld + EPG * (j ^ (rl & 7));
            gdst[m] = b * G3_BLK + ii * 1024;
        }
    }
    auto issue = [&](int64_t kb, int stage) {
#ifdef BK_K1_L2WINDOW  // timing-only ablation: every k-block read from the first W (L2-resident)
        const int64_t col = (kb % BK_K1_L2WINDOW) * BKE;
#else
        const int64_t col = kb * BKE;
#endif
        char *base = lds + stage * G3_STAGE;
#ifndef BK_K1_GLDS_LIMIT  // timing-only ablation: issue at most this many glds per wave
#define BK_K1_GLDS_LIMIT G3_MAXB
#endif
        if constexpr (ESPL != 0) {
            if (hi) {
#pragma unroll
                for (int m = 0; m < CHI; ++m)
                    __builtin_amdgcn_global_load_lds((const void *)(gsrc[m] + col),
                                                     (void *)(base + gdst[m]), 16, 0, 0);
            } else {
#pragma unroll
                for (int m = 0; m < CLO; ++m)
                    __builtin_amdgcn_global_load_lds((const void *)(gsrc[m] + col),
                                                     (void *)(base + gdst[m]), 16, 0, 0);
            }
            return;
        }
#pragma unroll
        for (int m = 0; m < (NB > 0 ? NB : G3_MAXB); ++m)
            if ((NB > 0 || m < c) && m < BK_K1_GLDS_LIMIT)
                __builtin_amdgcn_global_load_lds((const void *)(gsrc[m] + col),
                                                 (void *)(base + gdst[m]), 16, 0, 0);
    };

    typedef typename G3T<T>::acc AV;
    G3Acc<KIND == T_NONE ? T_DIAG1 : KIND, AV> acc;
    if constexpr (KIND == T_OFF) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc.a[i][j] = AV{0, 0, 0, 0};
    } else if constexpr (KIND == T_PAIR) {
#pragma unroll
        for (int i = 0; i < 10; ++i) acc.a[i] = acc.b[i] = AV{0, 0, 0, 0};
    } else if constexpr (KIND == T_DIAG1) {
#pragma unroll
        for (int i = 0; i < 10; ++i) acc.a[i] = AV{0, 0, 0, 0};
    }
    AV xacc = AV{0, 0, 0, 0};  // XO: the extra diagonal block
    gran ha[4], hb[4];  // STAG: the held second granule of the previous k-block
#pragma unroll
    for (int q = 0; q < 4; ++q) ha[q] = hb[q] = gran{};

#pragma unroll
    for (int s = 0; s < G3_STAGES - 1; ++s)
        if (s < nk && MODE != 2) issue(kst + (int64_t)s * kstr, s);
    int buf = 0;
    for (int t = 0; t < nk; ++t) {
        const int ahead = min(nk - t - 1, G3_STAGES - 2);  // stages issued after t
        G3_PROBE(p0);
        if constexpr (NB > 0 && MODE != 2 && ESPL != 0) {
            if (ahead > 0) {
                if (hi)
                    g3_waitc<CHI>();
                else
                    g3_waitc<CLO>();
            } else {
                g3_waitc<0>();
            }
        } else if constexpr (NB > 0 && MODE != 2) {
            if (ahead > 0)
                g3_waitc<(NB < BK_K1_GLDS_LIMIT ? NB : BK_K1_GLDS_LIMIT)>();
            else
                g3_waitc<0>();
        } else {
            g3_wait(MODE == 2 ? 0 : ahead * c);
        }
        G3_PROBE(p1);
        g3_barrier();
        G3_PROBE(p2);
        probe[0] += p1 - p0;
        probe[1] += p2 - p1;
        const char *ls = lds + buf * G3_STAGE;
        const int nbuf = buf == 0 ? G3_STAGES - 1 : buf - 1;  // (t + STAGES - 1) % STAGES
        const bool more = t + G3_STAGES - 1 < nk && MODE != 2;
        const int64_t nkb = kst + (int64_t)(t + G3_STAGES - 1) * kstr;
        buf = buf == G3_STAGES - 1 ? 0 : buf + 1;
        if constexpr (MODE == 1) {
            if (more) issue(nkb, nbuf);
            continue;
        }
        if constexpr (KIND == T_OFF) {
            gran a0[4], b0[4], a1[4], b1[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) a0[q] = g3_frag<T>(ls + sA * G3_BLK, q, 0, rr, g);
#pragma unroll
            for (int q = 0; q < 4; ++q) b0[q] = g3_frag<T>(ls + sB * G3_BLK, q, 0, rr, g);
            if constexpr (STAG) {
                if (t > 0) off_mma_gran<T, XO>(acc.a, ha, hb, xacc);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) a1[q] = g3_frag<T>(ls + sA * G3_BLK, q, 1, rr, g);
#pragma unroll
            for (int q = 0; q < 4; ++q) b1[q] = g3_frag<T>(ls + sB * G3_BLK, q, 1, rr, g);
            if (more) issue(nkb, nbuf);
            off_mma_gran<T, XO>(acc.a, a0, b0, xacc);
            if constexpr (STAG) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    ha[q] = a1[q];
                    hb[q] = b1[q];
                }
            } else {
                off_mma_gran<T, XO>(acc.a, a1, b1, xacc);
            }
        } else if constexpr (KIND == T_PAIR) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                gran a[4], b[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = g3_frag<T>(ls + sA * G3_BLK, q, h, rr, g);
#pragma unroll
                for (int q = 0; q < 4; ++q) b[q] = g3_frag<T>(ls + sB * G3_BLK, q, h, rr, g);
                if (h == 0 && more) issue(nkb, nbuf);
                diag_mma_g<T, XP>(acc.a, a);
                diag_mma_g<T, XP>(acc.b, b);
            }
        } else if constexpr (KIND == T_DIAG1) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                gran a[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = g3_frag<T>(ls + sA * G3_BLK, q, h, rr, g);
                if (h == 0 && more) issue(nkb, nbuf);
                diag_mma_g<T>(acc.a, a);
            }
        } else {
            if (more) issue(nkb, nbuf);
        }
    }
    if constexpr (KIND == T_OFF && STAG && MODE != 1)
        if (nk > 0) off_mma_gran<T, XO>(acc.a, ha, hb, xacc);
    if constexpr (KIND != T_NONE) {
        // ragged tail columns [nfull*BKE, d): one workgroup per group, direct loads
        const int64_t c0 = (int64_t)nfull * BKE;
        if (wd[4] && c0 < d) {
#pragma unroll
            for (int h = 0; h < BKE / 8; ++h) {
                const int64_t cc = c0 + 8 * h + 2 * g;
                d2v a[4], b[4];
                g3_load_rows<T>(a, X, ld, n, blk[sA], cc, d, rr);
                g3_load_rows<T>(b, X, ld, n, blk[sB], cc, d, rr);
                if constexpr (KIND == T_OFF) {
                    typedef typename G3T<T>::op O;
                    off_mma_tail<T>(acc.a, a, b);
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        if constexpr (XO == 1) xacc = G3T<T>::mma((O)a[0][s2], (O)a[3][s2], xacc);
                        if constexpr (XO == 2) xacc = G3T<T>::mma((O)b[0][s2], (O)b[3][s2], xacc);
                    }
                } else if constexpr (KIND == T_PAIR) {
                    diag_mma<T, XP>(acc.a, a);
                    diag_mma<T, XP>(acc.b, b);
                } else {
                    diag_mma<T>(acc.a, a);
                }
            }
        }
        if constexpr (KIND == T_OFF) {
            store_tile<T>(out, acc.a, rr, g, wt);
            if constexpr (XO != 0) {  // block (0,3) of the PAIR wave's diagonal tile
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st_part(&xout[g3_crow<T>(g, r) * 64 + 48 + rr], (double)xacc[r], wt);
            }
        } else if constexpr (KIND == T_PAIR) {
            store_diag<T, XP>(out, acc.a, rr, g, wt);
            store_diag<T, XP>(out + 4096, acc.b, rr, g, wt);
        } else {
            store_diag<T>(out, acc.a, rr, g, wt);
        }
    }
}

#ifndef G3_STAGGER
#define G3_STAGGER 1
#endif
template <typename T, int MODE, int NB>
__device__ __forceinline__ void g3_dispatch(const T *__restrict__ X, int64_t ld, int n,
                                            int nfull, int64_t d, const GroupDesc &G,
                                            const int *wd, char *lds, int wave, int lane,
                                            double *out, long long (&probe)[2], bool wt) {
    // the balanced quads always stage 4 row-blocks: only NB = 4 (and the
    // run-time NB = 0 of the ablation modes) carries the XT variants
    const int xt = (NB == 4 || NB == 0) ? G.xt[wave] : 0;
    double *xout = out - (int64_t)wave * 2 * 4096 + (int64_t)G.xslot[wave] * 4096;
    switch (G.task[wave][0]) {
    case T_OFF:
        // the stagger covers the fp64 MFMA's 64-cycle issue; on the fp32 MFMA
        // (32 cycles) it costs more than it hides: E's loop efficiency 0.776
        // staggered, 0.845 not (tools/trace_gram.py)
#ifndef BK_F32_STAGGER  // probe knob: 1 staggers the fp32-MFMA kernel too
#define BK_F32_STAGGER 0
#endif
        if (wave >= 4 && G3_STAGGER && (!G3T<T>::F32C || BK_F32_STAGGER)) {
            if (xt == 1)
                g3_wave<T, T_OFF, MODE, true, NB, (NB == 4 || NB == 0) ? 1 : 0>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, xout, wt);
            else if (xt == 2)
                g3_wave<T, T_OFF, MODE, true, NB, (NB == 4 || NB == 0) ? 2 : 0>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, xout, wt);
            else
                g3_wave<T, T_OFF, MODE, true, NB>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, nullptr, wt);
        } else {
            if (xt == 1)
                g3_wave<T, T_OFF, MODE, false, NB, (NB == 4 || NB == 0) ? 1 : 0>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, xout, wt);
            else if (xt == 2)
                g3_wave<T, T_OFF, MODE, false, NB, (NB == 4 || NB == 0) ? 2 : 0>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, xout, wt);
            else
                g3_wave<T, T_OFF, MODE, false, NB>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, nullptr, wt);
        }
        break;
    case T_PAIR:
        if (xt)
            g3_wave<T, T_PAIR, MODE, false, NB, (NB == 4 || NB == 0) ? 1 : 0>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, nullptr, wt);
        else
            g3_wave<T, T_PAIR, MODE, false, NB>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, nullptr, wt);
        break;
    case T_DIAG1:
        g3_wave<T, T_DIAG1, MODE, false, NB>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, nullptr, wt);
        break;
    default:
        g3_wave<T, T_NONE, MODE, false, NB>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, nullptr, wt);
        break;
    }
}
template <int MODE, typename T = double>
__global__ __launch_bounds__(512, 2) void k_gram3(const T *__restrict__ X, int64_t ld, int n,
                                                  int nfull, int64_t d,
                                                  const GroupDesc *__restrict__ groups,
                                                  const int *__restrict__ segtab,
                                                  const int *__restrict__ wgtab,
                                                  double *__restrict__ part,
                                                  long long *__restrict__ trace, PieceMarks pm) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // debug timeline (BK_TRACE_FILE): per workgroup 100 MHz start/end, shader
    // clock start/end, HW_ID, XCC_ID
    long long t_rt0 = 0, t_mt0 = 0;
    if (trace && threadIdx.x == 0) {
        t_rt0 = (long long)__builtin_amdgcn_s_memrealtime();
        t_mt0 = (long long)__builtin_amdgcn_s_memtime();
    }
    long long probe[2] = {0, 0};
    const bool wt = piece_handed(pm) && !pm.nowt;  // this workgroup's slabs go to the communication stream
    const int v0 = segtab[2 * blockIdx.x], nseg = segtab[2 * blockIdx.x + 1];
    long long ideal = 0;  // sum of nk * cost over the segments (trace only)
    for (int sg = 0; sg < nseg; ++sg) {
        const int v = v0 + sg;
        const int *wd = wgtab + 5 * v;
        const GroupDesc &G = groups[wd[0]];
        double *out = part + ((int64_t)v * 16 + wave * 2) * 4096;
        if (sg > 0) __syncthreads();  // the previous segment's waves are done with the LDS ring
        if constexpr (MODE == 0) {
            switch (G.nb) {
            case 1: g3_dispatch<T, MODE, 1>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, wt); break;
            case 2: g3_dispatch<T, MODE, 2>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, wt); break;
            case 3: g3_dispatch<T, MODE, 3>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, wt); break;
            case 4: g3_dispatch<T, MODE, 4>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, wt); break;
            case 5: g3_dispatch<T, MODE, 5>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, wt); break;
            default: g3_dispatch<T, MODE, 6>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, wt); break;
            }
        } else {
            g3_dispatch<T, MODE, 0>(X, ld, n, nfull, d, G, wd, lds, wave, lane, out, probe, wt);
        }
        if (trace) ideal += (long long)(wd[1] < wd[3] ? (wd[3] - 1 - wd[1]) / wd[2] + 1 : 0) * G.cost;
    }
    piece_done(pm);
    if (trace) {
#ifdef BK_K1_PROBE
        if (lane == 0) {
            trace[24 * blockIdx.x + 8 + wave] = probe[0];
            trace[24 * blockIdx.x + 16 + wave] = probe[1];
        }
#endif
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            long long *tr = trace + 24 * blockIdx.x;
            tr[0] = t_rt0;
            tr[1] = (long long)__builtin_amdgcn_s_memrealtime();
            tr[2] = t_mt0;
            tr[3] = (long long)__builtin_amdgcn_s_memtime();
            tr[4] = hw;
            tr[5] = xcc;
            // first segment's group and cost; k-blocks scaled so nk * cost = the ideal
            const int g0 = nseg > 0 ? wgtab[5 * v0] : 0;
            const int c0 = groups[g0].cost > 0 ? groups[g0].cost : 1;
            tr[6] = g0 | ((long long)c0 << 32);
            tr[7] = (ideal + c0 / 2) / c0;
        }
    }
}

// K1b v3: U[u] = sum over the owning group's workgroups (fixed order) of its slab
// block = 32 elements of one sub-tile x 8 interleaved sub-lists of its
// workgroups' slabs (sub-list q sums slabs q, q+8, q+16, ... in order), then
// the 8 sub-sums in order: a fixed order (deterministic), with 8x the loads in
// flight of one serial chain -- small-n plans have ~256 slabs per sub-tile
__global__ __launch_bounds__(256) void k_reduce3(const double *__restrict__ part,
                                                 const int *__restrict__ red,
                                                 const int *__restrict__ wglist,
                                                 double *__restrict__ U, int64_t usz,
                                                 double dcols, double dcols32, int u0, int rec) {
    // the packed upper's two trailing elements: the Gram's column count, and
    // how many of those columns were accumulated at fp32 unit roundoff (the
    // fp32 MFMA); both are summed with the tiles by every exchange, so after
    // one they are totals (K3b's margin: the total d, and u_G = 2^-24 as soon
    // as any shard ran on the fp32 MFMA)
    // (u0 / rec: one piece of the packed upper -- sub-tiles from u0 on, the
    // record only with the last piece -- when the exchange overlaps the Gram)
    if (rec && blockIdx.x == 0 && threadIdx.x == 0) {
        U[usz] = dcols;
        U[usz + 1] = dcols32;
        U[usz + 2] = 0.0;  // no int8-sliced columns
        U[usz + 3] = 0.0;
    }
#ifndef BK_REDUCE_V1
    // 64 elements per block, 2 per lane (16-B loads), 8 slabs in flight per
    // sub-list; the same order of adds as below (bitwise the same U)
    __shared__ d2v sub[8][32];
    const int u = u0 + (blockIdx.x >> 6), el = threadIdx.x & 31, q = threadIdx.x >> 5;
    const int e = (blockIdx.x & 63) * 64 + el * 2;
    const int off = red[3 * u], np = red[3 * u + 1], slot = red[3 * u + 2];
    const int *wl = wglist + off;
    d2v acc = {0.0, 0.0};
    int s = q;
    for (; s + 56 < np; s += 64) {
        d2v v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            v[k] = *reinterpret_cast<const d2v *>(part + ((int64_t)wl[s + 8 * k] * 16 + slot) * 4096 + e);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc.x += v[k].x;
            acc.y += v[k].y;
        }
    }
    for (; s < np; s += 8) {
        const d2v v = *reinterpret_cast<const d2v *>(part + ((int64_t)wl[s] * 16 + slot) * 4096 + e);
        acc.x += v.x;
        acc.y += v.y;
    }
    sub[q][el] = acc;
    __syncthreads();
    if (q == 0) {
        d2v t = sub[0][el];
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            t.x += sub[k][el].x;
            t.y += sub[k][el].y;
        }
        *reinterpret_cast<d2v *>(U + (int64_t)u * 4096 + e) = t;
    }
#else
    __shared__ double sub[8][32];
    const int u = u0 + (blockIdx.x >> 7), el = threadIdx.x & 31, q = threadIdx.x >> 5;
    const int e = (blockIdx.x & 127) * 32 + el;
    const int off = red[3 * u], np = red[3 * u + 1], slot = red[3 * u + 2];
    const int *wl = wglist + off;
    double acc = 0.0;
    int s = q;
    for (; s + 24 < np; s += 32) {
        const double v0 = part[((int64_t)wl[s + 0] * 16 + slot) * 4096 + e];
        const double v1 = part[((int64_t)wl[s + 8] * 16 + slot) * 4096 + e];
        const double v2 = part[((int64_t)wl[s + 16] * 16 + slot) * 4096 + e];
        const double v3 = part[((int64_t)wl[s + 24] * 16 + slot) * 4096 + e];
        acc += v0;
        acc += v1;
        acc += v2;
        acc += v3;
    }
    for (; s < np; s += 8) acc += part[((int64_t)wl[s] * 16 + slot) * 4096 + e];
    sub[q][el] = acc;
    __syncthreads();
    if (q == 0) {
        double t = sub[0][el];
#pragma unroll
        for (int k = 1; k < 8; ++k) t += sub[k][el];
        U[(int64_t)u * 4096 + e] = t;
    }
#endif
}

// ---------------------------------------------------------------------------
// K1b: packed upper U[u][64][64] = sum_{s=0..S-1} part[s*ntile+u] (fixed order)
// grid: ntile*16 blocks of 256 threads (4 rows x 64 cols each)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_reduce(const double *__restrict__ part, int ntile, int S,
                                                double *__restrict__ U, double dcols) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // as k_reduce3 (v1 never runs the fp32 MFMA)
        U[(int64_t)ntile * 4096] = dcols;
        U[(int64_t)ntile * 4096 + 1] = 0.0;
        U[(int64_t)ntile * 4096 + 2] = 0.0;
        U[(int64_t)ntile * 4096 + 3] = 0.0;
    }
    const int u = blockIdx.x >> 4, chunk = blockIdx.x & 15;
    const int e = chunk * 256 + threadIdx.x;
    const double *p = part + (int64_t)u * 4096 + e;
    const int64_t stride = (int64_t)ntile * 4096;
    double acc = 0.0;
    int s = 0;
    for (; s + 4 <= S; s += 4) {
        const double v0 = p[(s + 0) * stride], v1 = p[(s + 1) * stride];
        const double v2 = p[(s + 2) * stride], v3 = p[(s + 3) * stride];
        acc += v0;
        acc += v1;
        acc += v2;
        acc += v3;
    }
    for (; s < S; ++s) acc += p[s * stride];
    U[(int64_t)u * 4096 + e] = acc;
}

// Fixed-order sum of R packed partials (deterministic multi-GPU mode):
// U[e] = sum_{r=0..R-1} Ug[r*stride + e]
__global__ __launch_bounds__(256) void k_sum_ranks(const double *__restrict__ Ug, int R,
                                                   int64_t stride, double *__restrict__ U) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= stride) return;
    double acc = 0.0;
    for (int r = 0; r < R; ++r) acc += Ug[(int64_t)r * stride + e];
    U[e] = acc;
}

// ---------------------------------------------------------------------------
// K2: score[i] = sum of ranks 1..k of sort(D[i])   (logistic_validator.py:62-63)
// One workgroup per row; the row lives in LDS as order-preserving u64 keys.
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void k_scores(const double *__restrict__ U, int T_, int n,
                                               int npow2, int64_t k, double *__restrict__ scores,
                                               double *__restrict__ diag) {
    extern __shared__ __attribute__((aligned(16))) uint64_t keys[];
    __shared__ double red[NT / 64];
    const int i = blockIdx.x, tid = threadIdx.x;
    const double di = u_at(U, T_, i, i);
    if (tid == 0) diag[i] = di;  // ||x_i||^2 for the selection margin (K3b)
    for (int j = tid; j < npow2; j += NT) {
        uint64_t key = ~0ULL;  // padding sorts after every real value (NaN included)
        if (j < n) {
            const double t = di + u_at(U, T_, j, j);
            const double g2 = 2.0 * u_at(U, T_, i, j);
            key = dkey(t - g2);
        }
        keys[j] = key;
    }
    __syncthreads();
    for (int size = 2; size <= npow2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < (npow2 >> 1); t += NT) {
                const int lo = 2 * t - (t & (stride - 1));
                const int hi = lo + stride;
                const bool asc = (lo & size) == 0;
                const uint64_t a = keys[lo], b = keys[hi];
                if ((a > b) == asc) {
                    keys[lo] = b;
                    keys[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    double acc = 0.0;
    for (int64_t r = 1 + tid; r <= k; r += NT) acc += dkey_inv(keys[r]);
    // fixed-shape reduction: wave butterfly, then waves in order
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((tid & 63) == 0) red[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += red[w];
        scores[i] = (k > 0) ? s : 0.0;
    }
}

// K2 v2: the same scores, bitwise, with the row's keys in REGISTERS.  Thread
// t holds keys t*KPT .. t*KPT+KPT-1 (blocked).  Bitonic stages with a stride
// below KPT are compare-exchanges inside a thread; strides up to the wave's
// span (64 KPT keys) exchange across lanes -- DPP quad permutes for lane xor
// 1 / 2, ds_swizzle (bit-mask mode, no LDS banks) for 4 / 8 / 16, ds_bpermute
// for 32 -- with no barriers; only strides beyond a wave go through LDS.
// Keys are the distances as fp64 (-0 -> +0), ordered by v_min/v_max_f64 (two
// instructions per compare-exchange); a row holding a NaN (rare: NaN / Inf
// updates) is sorted as v1's order-preserving u64 keys instead (NaN last).
// The sorted row is written to LDS once and summed in v1's exact shape: v1's
// NT_SUM threads (256, or 1024 above 2048 keys), each summing ranks 1+t,
// 1+t+NT_SUM, ..., the wave butterfly, then the waves in order -- emulated
// with H = NT_SUM / NT accumulators per thread.  Any correct sort of the same
// keys gives the same array, so the scores are bitwise v1's.
// Row loads: from the packed upper tiles (u_at), or -- for large n, after
// k_transpose -- from Ut (the off-diagonal tiles transposed) and a contiguous
// diagonal, so a row is read in 512-B runs instead of 8-B strided elements.
// bitonic sort of N = NT * KPT keys, blocked (thread t holds keys t KPT ..),
// in the all-ascending form: each merge of size s opens with the mirror stage
// (partner e ^ (s - 1)) and continues with xor stages (e ^ s/4, ..., e ^ 1);
// the lower index of every pair takes the minimum, so no stage needs a
// direction.  The sorted keys end in keys_lds.
template <typename K, int NT, int KPT>
__device__ __forceinline__ void k2_sort(K (&v)[KPT], K *keys_lds, int N, int tid) {
    constexpr int LK = KPT == 1 ? 0 : KPT == 2 ? 1 : KPT == 4 ? 2 : KPT == 8 ? 3 : 4;
    constexpr int WSPAN = 64 * KPT;  // keys per wave
    const int lane = tid & 63, e0 = tid * KPT;
    for (int size = 2; size <= N; size <<= 1) {
        // (1) the mirror stage
        if (size <= KPT) {
#pragma unroll
            for (int q = 0; q < KPT; ++q) {
                const int p = q ^ (size - 1);
                if (q < p && ((q ^ p) & (size >> 1))) k2_cas(v[q], v[p]);
            }
        } else if (size <= WSPAN) {
            const int m = (size - 1) >> LK;
            k2_lane_dispatch<K, KPT, KPT - 1>(v, m, (lane & ((size >> 1) >> LK)) == 0);
        } else {
            __syncthreads();  // earlier readers of keys_lds are done
#pragma unroll
            for (int q = 0; q < KPT; ++q) keys_lds[e0 + q] = v[q];
            __syncthreads();
            const int half = size >> 1;
            for (int p = tid; p < (N >> 1); p += NT) {
                const int lo = (p / half) * size + (p & (half - 1));
                const int hi = lo ^ (size - 1);
                K a = keys_lds[lo], b = keys_lds[hi];
                k2_cas(a, b);
                keys_lds[lo] = a;
                keys_lds[hi] = b;
            }
            __syncthreads();
            // (2a) xor stages beyond the wave, still in LDS
            int stride = size >> 2;
            for (; stride >= WSPAN; stride >>= 1) {
                for (int p = tid; p < (N >> 1); p += NT) {
                    const int lo = 2 * p - (p & (stride - 1));
                    const int hi = lo + stride;
                    K a = keys_lds[lo], b = keys_lds[hi];
                    k2_cas(a, b);
                    keys_lds[lo] = a;
                    keys_lds[hi] = b;
                }
                __syncthreads();
            }
#pragma unroll
            for (int q = 0; q < KPT; ++q) v[q] = keys_lds[e0 + q];
        }
        // (2b) xor stages across lanes, then (2c) inside the thread
        for (int stride = min(size >> 2, WSPAN >> 1); stride >= KPT; stride >>= 1) {
            const int m = stride >> LK;
            k2_lane_dispatch<K, KPT, 0>(v, m, (lane & m) == 0);
        }
#pragma unroll
        for (int st = KPT / 2; st >= 1; st >>= 1) {
            if (st > (size >> 2)) continue;
#pragma unroll
            for (int q = 0; q < KPT; ++q)
                if ((q & st) == 0) k2_cas(v[q], v[q + st]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KPT; ++q) keys_lds[e0 + q] = v[q];
    __syncthreads();
}

// K2 v3 sort, 16 keys per thread (N >= 4096): every compare-exchange inside a
// thread.  A stage on index bit b is register-local when b is one of the 4
// bits the current layout keeps in the register index; layout L_j keeps bits
// j .. j+3 there (thread t, register q hold key e = (t mod 2^j) | q 2^j |
// (t >> j) 2^(j+4)), and a merge of 2^B keys walks its bits B-1 .. 0 in
// chunks of 4, moving the keys to L_(hi-3) .. L_0 through LDS before each
// chunk (3 moves per merge at N = 4096, 20 in all) instead of lane exchanges
// (v2: 33 DPP / swizzle / bpermute stages of ~6 instructions per key).  The
// merges use the classic alternating directions, folded into the keys:
// before merge B the keys of blocks with bit B set are negated (order
// reversed: -x for fp64, ~x for the u64 keys), so every stage keeps the
// minimum at the lower index and the sequence entering each merge is bitonic;
// at B = log2 N nothing is negated.  LDS words are padded by one per 16 keys
// (word e + e/16), which keeps every layout's 16-lane write groups and 32-lane
// read groups on distinct banks.  Any correct sort gives the same array.
__device__ __forceinline__ int k2_pad(int e) { return e + (e >> 4); }
template <int J>
__device__ __forceinline__ int k2_lbase(int t) {
    const int e = (t & ((1 << J) - 1)) | ((t >> J) << (J + 4));
    return e + (e >> 4);
}
template <int J>
__device__ __forceinline__ constexpr int k2_loff(int q) {  // padded word of (t, q) - of (t, 0)
    if constexpr (J >= 4)
        return (q << J) + (q << (J - 4));
    else
        return (q << J) + (q >> (4 - J));
}
template <typename K, int J>
__device__ __forceinline__ void k2_put(const K (&v)[16], K *lds, int t) {
    K *p = lds + k2_lbase<J>(t);
#pragma unroll
    for (int q = 0; q < 16; ++q) p[k2_loff<J>(q)] = v[q];
}
template <typename K, int J>
__device__ __forceinline__ void k2_get(K (&v)[16], const K *lds, int t) {
    const K *p = lds + k2_lbase<J>(t);
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = p[k2_loff<J>(q)];
}
// the ordering point of a move: a workgroup barrier, or -- when every key
// stays inside its wave -- only a compiler fence (a wave's LDS operations
// execute in order, so its reads see its own lanes' writes)
__device__ __forceinline__ void k2_sync(bool local) {
    if (local) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}
// L_from -> L_to.  Thread bits 6.. (the wave index) are key bits 10.. in every
// layout L_j with j <= 6, so a move between two such layouts keeps each key in
// its wave, in the wave's own LDS words: no workgroup barrier (16 of the 20
// moves at N = 4096)
template <typename K>
__device__ __forceinline__ void k2_move(K (&v)[16], K *lds, int t, int from, int to) {
    const bool local = from <= 6 && to <= 6;
    k2_sync(local);  // earlier readers of these words are done
    switch (from) {
    case 0: k2_put<K, 0>(v, lds, t); break;
    case 1: k2_put<K, 1>(v, lds, t); break;
    case 2: k2_put<K, 2>(v, lds, t); break;
    case 3: k2_put<K, 3>(v, lds, t); break;
    case 4: k2_put<K, 4>(v, lds, t); break;
    case 5: k2_put<K, 5>(v, lds, t); break;
    case 6: k2_put<K, 6>(v, lds, t); break;
    case 7: k2_put<K, 7>(v, lds, t); break;
    case 8: k2_put<K, 8>(v, lds, t); break;
    case 9: k2_put<K, 9>(v, lds, t); break;
    default: k2_put<K, 10>(v, lds, t); break;
    }
    k2_sync(local);
    switch (to) {
    case 0: k2_get<K, 0>(v, lds, t); break;
    case 1: k2_get<K, 1>(v, lds, t); break;
    case 2: k2_get<K, 2>(v, lds, t); break;
    case 3: k2_get<K, 3>(v, lds, t); break;
    case 4: k2_get<K, 4>(v, lds, t); break;
    case 5: k2_get<K, 5>(v, lds, t); break;
    case 6: k2_get<K, 6>(v, lds, t); break;
    case 7: k2_get<K, 7>(v, lds, t); break;
    case 8: k2_get<K, 8>(v, lds, t); break;
    case 9: k2_get<K, 9>(v, lds, t); break;
    default: k2_get<K, 10>(v, lds, t); break;
    }
}
// an ascending stage on register bit R (pairs q, q + 2^R)
template <typename K, int R>
__device__ __forceinline__ void k2_rstage(K (&v)[16]) {
#pragma unroll
    for (int q = 0; q < 16; ++q)
        if (!(q & (1 << R))) k2_cas(v[q], v[q | (1 << R)]);
}
template <typename K>
__device__ __forceinline__ void k2_rstages(K (&v)[16], int top) {  // register bits top .. 0
    switch (top) {
    case 3: k2_rstage<K, 3>(v); [[fallthrough]];
    case 2: k2_rstage<K, 2>(v); [[fallthrough]];
    case 1: k2_rstage<K, 1>(v); [[fallthrough]];
    default: k2_rstage<K, 0>(v);
    }
}
template <typename K>
__device__ __forceinline__ void k2_negate(K (&v)[16]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = K2Ord<K>::neg(v[q]);
}
// v: thread t's keys t*16 .. t*16+15 (L_0); on return the whole row sorted
// ascending sits in lds at the padded words k2_pad(e)
template <typename K>
__device__ __forceinline__ void k2_sort16(K (&v)[16], K *lds, int N, int tid) {
    if (tid & 1) k2_negate(v);  // blocks of 16 with bit 4 set sort descending
    // merges of 2 .. 16 keys inside the thread (all-ascending mirror form)
#pragma unroll
    for (int size = 2; size <= 16; size <<= 1) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int p = q ^ (size - 1);
            if (q < p && ((q ^ p) & (size >> 1))) k2_cas(v[q], v[p]);
        }
#pragma unroll
        for (int st = size >> 2; st >= 1; st >>= 1)
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if ((q & st) == 0) k2_cas(v[q], v[q + st]);
    }
    for (int B = 5; (1 << B) <= N; ++B) {
        if (((tid >> (B - 4)) ^ (tid >> (B - 5))) & 1) k2_negate(v);  // direction of merge B
        int cur = 0;
        for (int hi = B - 1; hi >= 0;) {
            const int j = hi > 3 ? hi - 3 : 0;
            k2_move(v, lds, tid, cur, j);
            cur = j;
            k2_rstages(v, hi - j);
            hi = j - 1;
        }
    }
    __syncthreads();
    k2_put<K, 0>(v, lds, tid);
    __syncthreads();
}

// v1's summation shape over the sorted keys (virtual thread t' = tid + NT h)
// ranks >= nfin hold NaN (v1's keys sort NaN after +inf; v2/v3 sort the NaN
// distances as +inf and put the NaN back here, at the same ranks)
template <typename K, int NT, int NT_SUM, bool PAD = false>
__device__ __forceinline__ double k2_sum(const K *keys_lds, int64_t k, int tid, double *red,
                                         int64_t nfin = INT64_MAX) {
    constexpr int H = NT_SUM / NT;
    const int lane = tid & 63;
#pragma unroll
    for (int h = 0; h < H; ++h) {
        double acc = 0.0;
        for (int64_t r = 1 + tid + NT * h; r <= k; r += NT_SUM)
            acc += r < nfin ? K2Ord<K>::val(keys_lds[PAD ? k2_pad((int)r) : r]) : __builtin_nan("");
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) red[(tid >> 6) + (NT / 64) * h] = acc;
    }
    __syncthreads();
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < NT_SUM / 64; ++w) sum += red[w];
    return sum;
}

// row i of G, element e: packed upper tiles, or (TR) Ut + contiguous diagonal
template <bool TR>
__device__ __forceinline__ double k2_g(const double *__restrict__ U, const double *__restrict__ Ut,
                                       int T_, int i, int e) {
    if constexpr (!TR) {
        return u_at(U, T_, i, e);
    } else {
        const int br = i >> 6, bc = e >> 6, ir = i & 63, ic = e & 63;
        if (br < bc || (br == bc && ir <= ic)) return U[upper_tile(T_, br, bc) + ir * 64 + ic];
        if (br == bc) return U[upper_tile(T_, br, br) + ic * 64 + ir];
        return Ut[upper_tile(T_, bc, br) + ir * 64 + ic];  // (Ut tile) = (U tile)^T
    }
}

// MODE (timing-only ablations, tools/k2_modes.py): 1 = loads and keys, no
// sort; 2 = sort of synthetic keys, no loads
template <int NT, int KPT, int NT_SUM, bool TR, int MODE = 0>
__global__ __launch_bounds__(NT) void k_scores2(const double *__restrict__ U,
                                                const double *__restrict__ Ut,
                                                const double *__restrict__ dg_in, int T_, int n,
                                                int N, int64_t k, double *__restrict__ scores,
                                                double *__restrict__ diag, int r0) {
    static_assert(NT_SUM % NT == 0 && NT % 64 == 0, "summation shape");
    extern __shared__ __attribute__((aligned(16))) uint64_t keys[];  // N
    __shared__ double red[NT_SUM / 64];
    // row i: workgroup b scores row r0 + b (a rank's share of the rows when the
    // scoring is split over the ranks of a sharded call; r0 = 0 otherwise)
    const int i = r0 + (int)blockIdx.x, tid = threadIdx.x;
    const double di = TR ? dg_in[i] : u_at(U, T_, i, i);
    if (tid == 0) diag[i] = di;
    // distances, element e = tid + NT q (consecutive lanes, consecutive
    // columns: coalesced row reads), through LDS into the blocked layout.  A
    // NaN distance sorts as +inf and is counted: v1's order puts the row's
    // NaNs right after every +inf and before the padding, i.e. at ranks
    // n - nan .. n - 1, and k2_sum adds NaN there -- the same scores, bitwise,
    // without a second (u64-key) sort in the kernel (its registers held K2 at
    // 3 waves per SIMD)
    constexpr bool V3 = KPT == 16;  // the register-local sort (k2_sort16)
    __shared__ int s_nan;
    if (tid == 0) s_nan = 0;
    __syncthreads();
    double *kd = reinterpret_cast<double *>(keys);
    int nanc = 0;
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
        const int e = tid + NT * q;
        double x = __builtin_inf();  // padding sorts after every real value
        if (MODE == 2) {
            x = (double)((e * 2654435761u + i) & 0xFFFFF);
        } else if (e < n) {
            const double t = di + (TR ? dg_in[e] : u_at(U, T_, e, e));
            const double g2 = 2.0 * k2_g<TR>(U, Ut, T_, i, e);
            x = t - g2;
            x = x == 0.0 ? 0.0 : x;  // -0 == +0 (v1's dkey)
            if (x != x) {
                ++nanc;
                x = __builtin_inf();
            }
        }
        kd[V3 ? k2_pad(e) : e] = x;
    }
    if (MODE == 1) {
        if (kd[tid] == 1.2345) scores[i] = kd[tid];  // keep the loads
        return;
    }
    if (nanc) atomicAdd(&s_nan, nanc);
    __syncthreads();
    double dv[KPT];
    if constexpr (V3) {
        k2_get<double, 0>(dv, kd, tid);
    } else {
#pragma unroll
        for (int q = 0; q < KPT; ++q) dv[q] = kd[tid * KPT + q];
    }
    const int64_t nfin = n - s_nan;
    __syncthreads();  // kd[] reads before the sort's writes
    double sum;
    if constexpr (V3) {
        k2_sort16<double>(dv, kd, N, tid);
        sum = k2_sum<double, NT, NT_SUM, true>(kd, k, tid, red, nfin);
    } else {
        k2_sort<double, NT, KPT>(dv, kd, N, tid);
        sum = k2_sum<double, NT, NT_SUM>(kd, k, tid, red, nfin);
    }
    if (tid == 0) scores[i] = (k > 0) ? sum : 0.0;
}

// Ut (the off-diagonal upper tiles transposed) and the contiguous diagonal,
// for K2's coalesced row reads at large n; one 64x64 tile per block through LDS
// [bj0, bj1]: the off-diagonal tiles transposed are those of block-columns
// bj0..bj1 only -- the rows [64 bj0, 64 bj1 + 64) a rank scores under split
// scoring read no others; the diagonal (every row's G_jj) always
__global__ __launch_bounds__(256) void k_transpose(const double *__restrict__ U, int T_,
                                                   double *__restrict__ Ut,
                                                   double *__restrict__ dg, int bj0, int bj1) {
    __shared__ double t[64][65];
    int bi, bj;
    tri_decode(blockIdx.x, T_, bi, bj);
    const double *src = U + (int64_t)blockIdx.x * 4096;
    if (bi == bj) {
        if (threadIdx.x < 64) dg[bi * 64 + threadIdx.x] = src[threadIdx.x * 65];
        return;
    }
    if (bj < bj0 || bj > bj1) return;  // block-uniform
    for (int e = threadIdx.x; e < 4096; e += 256) t[e >> 6][e & 63] = src[e];
    __syncthreads();
    double *dst = Ut + (int64_t)blockIdx.x * 4096;
    for (int e = threadIdx.x; e < 4096; e += 256) dst[e] = t[e & 63][e >> 6];
}

// ---------------------------------------------------------------------------
// K3: rank_i = #{j : key_j < key_i} + #{j < i : key_j == key_i}; mask = rank < m
// ---------------------------------------------------------------------------
// one wave per row: lanes sweep j, a ballot counts the keys ranked before i.
// The ranks are a permutation of 0..n-1, so exactly one row writes each of
// bnd[0] = the highest selected score (rank m-1) and bnd[1] = the lowest
// rejected one (rank m): the selection boundary, for K3b's margin.
__global__ __launch_bounds__(256) void k_rank(const double *__restrict__ scores, int n, int m,
                                              int *__restrict__ mask, double *__restrict__ bnd) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= n) return;  // wave-uniform
    const double si = scores[i];
    const uint64_t ki = dkey(si);
    int cnt = 0;
    for (int j0 = 0; j0 < n; j0 += 64) {
        const int j = j0 + lane;
        bool before = false;
        if (j < n) {
            const uint64_t kj = dkey(scores[j]);
            before = (kj < ki) || (kj == ki && j < i);
        }
        cnt += __popcll(__ballot(before));
    }
    if (lane == 0) {
        mask[i] = cnt < m ? 1 : 0;
        if (cnt == m - 1) bnd[0] = si;
        if (cnt == m) bnd[1] = si;
    }
}

// K3b: ascending compaction of mask (single workgroup of 1024 threads), then
// the selection margin (SURVEY.md §7 "Hard parts", §8(d)):
//   gap       = s[rank m] - s[rank m-1]  (lowest rejected - highest selected)
//   err_bound = 2 (e_here + e_ref),  e = 4 k M' (gamma_{d+2}(u_G) + 2 u + gamma_k(u))
// where M' = max finite G_ii (1 + 2 gamma_{d+2}(u_G)) bounds max ||x_i||^2, u =
// 2^-53 (the distance and score arithmetic, and numpy's BLAS Gram), u_G the
// Gram's unit roundoff here (2^-53; 2^-24 on the fp32 MFMA), d = the Gram's
// column count (carried in the packed upper's trailing element, so it is the
// TOTAL d after a multi-GPU exchange).  Every computed score lies within e of
// the exact one, so whenever gap > err_bound the reference selects exactly this
// set; otherwise near_tie = 1 (also for exact ties, e.g. k = 0).
// margin[0..7] = {gap, err_bound, near_tie, M, s_lo, s_hi, d, k}
__global__ __launch_bounds__(1024) void k_compact(const int *__restrict__ mask, int n,
                                                  int64_t *__restrict__ sel,
                                                  const double *__restrict__ diag,
                                                  const double *__restrict__ bnd,
                                                  const double *__restrict__ dcols, int64_t k,
                                                  double *__restrict__ margin) {
    __shared__ int pre[1024];
    __shared__ double mx[16];
    const int tid = threadIdx.x;
    const int chunk = (n + 1023) / 1024;
    const int c0 = min(n, tid * chunk), c1 = min(n, c0 + chunk);
    int cnt = 0;
    for (int j = c0; j < c1; ++j) cnt += mask[j];
    pre[tid] = cnt;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
        const int v = tid >= o ? pre[tid - o] : 0;
        __syncthreads();
        pre[tid] += v;
        __syncthreads();
    }
    int pos = pre[tid] - cnt;
    for (int j = c0; j < c1; ++j)
        if (mask[j]) sel[pos++] = j;
    if (!margin) return;  // block-uniform
    // M = max finite G_ii (NaN / Inf rows have NaN / Inf scores in the
    // reference too: they order last, deterministically)
    double m = 0.0;
    for (int j = tid; j < n; j += 1024) {
        const double v = diag[j];
        if (v == v && v < __builtin_inf() && v > m) m = v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
    if ((tid & 63) == 0) mx[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) {
        double M = 0.0;
        for (int w = 0; w < 16; ++w) M = fmax(M, mx[w]);
        // the packed record's trailing record: the Gram's column count, the
        // part of it accumulated on the fp32 MFMA and the int8-sliced columns'
        // absolute error bound (after an exchange: totals)
        write_margin_rec(margin, bnd[0], bnd[1], M, dcols[0], dcols[1], dcols[2], k);
    }
}

// ---------------------------------------------------------------------------
// K4: mean[c] = (sum over selected rows, ascending) / m      (:51, fp64)
// ---------------------------------------------------------------------------
// ACCUM = false: mean[c] = (sum over r in sel order of X[sel[r]][c]) / m   (K4)
// ACCUM = true:  mean[c] = mean[c] + X[sel[0]][c] + X[sel[1]][c] + ...       (in sel
//                order, sequential: the GlobalW update of honest.go:361-375)
// SEG (a large selection, m >= MEAN_SEG_MIN): block row y sums the selected
// rows [y L, y L + L) into part[y][c] (no divide), k_mean_comb adds the
// segments in order -- a fixed order that depends on m only, so every shard
// and device of one call adds alike
#ifndef BK_MEAN_DEPTH
#define BK_MEAN_DEPTH 8  // rows' loads in flight per thread (same adds in the same order at any depth)
#endif
template <typename T, bool VEC, bool ACCUM = false, bool SEG = false>
__global__ __launch_bounds__(256) void k_mean(const T *__restrict__ X, int64_t ld, int64_t d,
                                              const int64_t *__restrict__ sel, int m,
                                              double *__restrict__ mean) {
    extern __shared__ __attribute__((aligned(16))) int64_t srow[];  // row offsets (elements)
    if constexpr (SEG) {
        const int r0 = (int)blockIdx.y * MEAN_SEG_ROWS;
        sel += r0;
        m = m - r0 < MEAN_SEG_ROWS ? m - r0 : MEAN_SEG_ROWS;
        mean += (int64_t)blockIdx.y * d;
    }
    for (int r = threadIdx.x; r < m; r += 256) srow[r] = sel[r] * ld;
    __syncthreads();
    const double dm = SEG ? 1.0 : (double)m;
    const int64_t npair = (d + 1) >> 1;
    for (int64_t cp = (int64_t)blockIdx.x * 256 + threadIdx.x; cp < npair;
         cp += (int64_t)gridDim.x * 256) {
        const int64_t c = cp * 2;
        if (c + 1 < d) {
            d2v acc = {0.0, 0.0};
            if constexpr (ACCUM) acc = d2v{mean[c], mean[c + 1]};
            int r = 0;
            for (; r + BK_MEAN_DEPTH <= m; r += BK_MEAN_DEPTH) {
                d2v v[BK_MEAN_DEPTH];
#pragma unroll
                for (int q = 0; q < BK_MEAN_DEPTH; ++q) v[q] = ld2s<T, VEC>(X + srow[r + q] + c);
#pragma unroll
                for (int q = 0; q < BK_MEAN_DEPTH; ++q) {
                    acc.x += v[q].x;
                    acc.y += v[q].y;
                }
            }
            for (; r < m; ++r) {
                const d2v v = ld2s<T, VEC>(X + srow[r] + c);
                acc.x += v.x;
                acc.y += v.y;
            }
            if constexpr (ACCUM || SEG) {
                mean[c] = acc.x;
                mean[c + 1] = acc.y;
            } else {
                mean[c] = acc.x / dm;
                mean[c + 1] = acc.y / dm;
            }
        } else {
            double acc = ACCUM ? mean[c] : 0.0;
            for (int r = 0; r < m; ++r) acc += (double)X[srow[r] + c];
            mean[c] = (ACCUM || SEG) ? acc : acc / dm;
        }
    }
}

// fp32 rows with 16-B aligned starts: 4 columns per thread from one 16-B load
// (the f2v form above moves 8 B per load: config E's K4 ran at 3.9 TB/s).  The
// same per-column order of adds as k_mean, so the same bits.
template <bool ACCUM, bool SEG = false>
__global__ __launch_bounds__(256) void k_mean_f4(const float *__restrict__ X, int64_t ld, int64_t d,
                                                 const int64_t *__restrict__ sel, int m,
                                                 double *__restrict__ mean) {
    extern __shared__ __attribute__((aligned(16))) int64_t srow[];
    if constexpr (SEG) {  // as k_mean's SEG
        const int r0 = (int)blockIdx.y * MEAN_SEG_ROWS;
        sel += r0;
        m = m - r0 < MEAN_SEG_ROWS ? m - r0 : MEAN_SEG_ROWS;
        mean += (int64_t)blockIdx.y * d;
    }
    for (int r = threadIdx.x; r < m; r += 256) srow[r] = sel[r] * ld;
    __syncthreads();
    const double dm = SEG ? 1.0 : (double)m;
    const int64_t nq = (d + 3) >> 2;
    for (int64_t cq = (int64_t)blockIdx.x * 256 + threadIdx.x; cq < nq;
         cq += (int64_t)gridDim.x * 256) {
        const int64_t c = cq * 4;
        if (c + 3 < d) {
            double acc[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] = ACCUM ? mean[c + e] : 0.0;
            int r = 0;
            for (; r + 8 <= m; r += 8) {
                f4v v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    v[q] = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(X + srow[r + q] + c));
#pragma unroll
                for (int q = 0; q < 8; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[e] += (double)v[q][e];
            }
            for (; r < m; ++r) {
                const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(X + srow[r] + c));
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] += (double)v[e];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) mean[c + e] = (ACCUM || SEG) ? acc[e] : acc[e] / dm;
        } else {
            for (int64_t cc = c; cc < d; ++cc) {
                double acc = ACCUM ? mean[cc] : 0.0;
                for (int r = 0; r < m; ++r) acc += (double)X[srow[r] + cc];
                mean[cc] = (ACCUM || SEG) ? acc : acc / dm;
            }
        }
    }
}

// the segments of a large selection's K4, in segment order, then / m
__global__ __launch_bounds__(256) void k_mean_comb(const double *__restrict__ part, int S, int64_t d,
                                                   int m, double *__restrict__ mean) {
    const double dm = (double)m;
    for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < d; c += (int64_t)gridDim.x * 256) {
        double acc = 0.0;
        for (int y = 0; y < S; ++y) acc += __builtin_nontemporal_load(part + (int64_t)y * d + c);
        mean[c] = acc / dm;
    }
}

// ---------------------------------------------------------------------------
// synthetic batch: grid (column blocks, rows)
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_synth(T *__restrict__ X, int64_t ld, int64_t dl,
                                               int64_t c0, const int64_t *__restrict__ perm,
                                               SynthParams P) {
    const int64_t p = blockIdx.y;
    const int64_t r = perm[p];
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < dl; k += (int64_t)gridDim.x * 256)
        X[p * ld + k] = (T)synth_elem(P, r, c0 + k);
}

// ===========================================================================
// launchers
// ===========================================================================

static constexpr int GRAM_P = 4;

hipError_t launch_gram(const void *X, int dtype, int64_t ld, int n, int64_t d, const Plan &pl,
                       double *part, hipStream_t st) {
    const bool vec = dtype == 0 ? ((ld % 2) == 0 && ((uintptr_t)X % 16) == 0)
                                : ((ld % 2) == 0 && ((uintptr_t)X % 8) == 0);
    dim3 grid((unsigned)pl.nwg), block(256);
    if (dtype == 0) {
        if (vec)
            hipLaunchKernelGGL((k_gram<double, true, GRAM_P>), grid, block, 0, st,
                               (const double *)X, ld, n, d, pl.T, pl.ntile, pl.S, pl.kc, pl.nwg, part);
        else
            hipLaunchKernelGGL((k_gram<double, false, GRAM_P>), grid, block, 0, st,
                               (const double *)X, ld, n, d, pl.T, pl.ntile, pl.S, pl.kc, pl.nwg, part);
    } else {
        if (vec)
            hipLaunchKernelGGL((k_gram<float, true, GRAM_P>), grid, block, 0, st, (const float *)X,
                               ld, n, d, pl.T, pl.ntile, pl.S, pl.kc, pl.nwg, part);
        else
            hipLaunchKernelGGL((k_gram<float, false, GRAM_P>), grid, block, 0, st, (const float *)X,
                               ld, n, d, pl.T, pl.ntile, pl.S, pl.kc, pl.nwg, part);
    }
    return hipGetLastError();
}

hipError_t launch_reduce(const double *part, const Plan &pl, double *U, hipStream_t st) {
    hipLaunchKernelGGL(k_reduce, dim3((unsigned)pl.ntile * 16), dim3(256), 0, st, part, pl.ntile,
                       pl.S, U, (double)pl.d);
    return hipGetLastError();
}

// U[e] += P[e]: the host entries' running sum of column-chunk Gram partials
// (chunk order, so deterministic)
__global__ __launch_bounds__(256) void k_add_upper(double *__restrict__ U,
                                                   const double *__restrict__ P, int64_t count) {
    const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (e + 1 < count) {
        d2v u = *reinterpret_cast<const d2v *>(U + e), p = *reinterpret_cast<const d2v *>(P + e);
        *reinterpret_cast<d2v *>(U + e) = u + p;
    } else if (e < count) {
        U[e] += P[e];
    }
}

hipError_t launch_add_upper(double *U, const double *P, int64_t count, hipStream_t st) {
    hipLaunchKernelGGL(k_add_upper, dim3((unsigned)((count + 511) / 512)), dim3(256), 0, st, U, P,
                       count);
    return hipGetLastError();
}

hipError_t launch_sum_ranks(const double *Ug, int R, int64_t stride, double *U, hipStream_t st) {
    hipLaunchKernelGGL(k_sum_ranks, dim3((unsigned)((stride + 255) / 256)), dim3(256), 0, st, Ug, R,
                       stride, U);
    return hipGetLastError();
}

static int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

template <int NT, int KPT, int NT_SUM, bool TR>
static void launch_scores2(const double *U, const double *Ut, const double *dg, int T, int n, int N,
                           int64_t k, double *scores, double *diag, hipStream_t st, int r0,
                           int rows) {
    const size_t lds = (size_t)(KPT == 16 ? N + N / 16 : N) * sizeof(uint64_t);  // v3: padded
    if constexpr (kProbes) {  // timing-only ablations (tools/k2_modes.py): probe builds only
        static const int mode = [] {
            const char *e = probe_env("BK_K2_MODE");
            return e ? atoi(e) : 0;
        }();
        if (mode == 1) {
            hipLaunchKernelGGL((k_scores2<NT, KPT, NT_SUM, TR, 1>), dim3(rows), dim3(NT), lds, st,
                               U, Ut, dg, T, n, N, k, scores, diag, r0);
            return;
        }
        if (mode == 2) {
            hipLaunchKernelGGL((k_scores2<NT, KPT, NT_SUM, TR, 2>), dim3(rows), dim3(NT), lds, st,
                               U, Ut, dg, T, n, N, k, scores, diag, r0);
            return;
        }
    }
    hipLaunchKernelGGL((k_scores2<NT, KPT, NT_SUM, TR>), dim3(rows), dim3(NT), lds, st, U, Ut, dg,
                       T, n, N, k, scores, diag, r0);
}

bool scores_transposed(int n) {
    static const int tmin = [] {
        const char *e = probe_env("BK_K2_TRANSPOSE_MIN_N");  // probe knob
        return e ? atoi(e) : 2049;
    }();
    return n >= tmin;
}

hipError_t launch_transpose(const double *U, int T, double *Ut, double *dg, hipStream_t st,
                            int bj0, int bj1) {
    if (bj1 < 0) bj1 = T - 1;
    hipLaunchKernelGGL(k_transpose, dim3((unsigned)(T * (T + 1) / 2)), dim3(256), 0, st, U, T, Ut,
                       dg, bj0, bj1);
    return hipGetLastError();
}

hipError_t launch_scores(const double *U, const double *Ut, const double *dg, int T, int n,
                         int64_t k, double *scores, double *diag, hipStream_t st, int r0,
                         int rows) {
    if (rows < 0) rows = n - r0;
    if (r0 < 0 || rows < 0 || r0 + rows > n) return hipErrorInvalidValue;
    if (rows == 0) return hipSuccess;
    const int np2 = next_pow2(n < 2 ? 2 : n);
    const size_t lds = (size_t)np2 * sizeof(uint64_t);
    static const bool v1 = [] {
        const char *e = probe_env("BK_SCORES");
        return e && strcmp(e, "v1") == 0;
    }();
    static const int kpt_big = [] {  // probe knob: keys per thread above 2048 keys
        const char *e = probe_env("BK_K2_KPT");
        return e ? atoi(e) : 16;
    }();
    if (!v1) {
        // v2: 256 threads up to 2048 keys (KPT = N / 256), then KPT = 16 (or
        // 4); the v1 summation shape (256 / 1024 threads) is emulated
        const int N = np2 < 256 ? 256 : np2;
#define BK_K2(NT, KPT, NS, TR) \
    launch_scores2<NT, KPT, NS, TR>(U, Ut, dg, T, n, N, k, scores, diag, st, r0, rows)
        if (Ut) {
            switch (N) {
            case 4096:
                if (kpt_big == 4)
                    BK_K2(1024, 4, 1024, true);
                else
                    BK_K2(256, 16, 1024, true);
                break;
            case 8192: BK_K2(512, 16, 1024, true); break;
            default: BK_K2(1024, 16, 1024, true); break;
            }
        } else {
            switch (N) {
            case 256: BK_K2(256, 1, 256, false); break;
            case 512: BK_K2(256, 2, 256, false); break;
            case 1024: BK_K2(256, 4, 256, false); break;
            case 2048: BK_K2(256, 8, 256, false); break;
            case 4096:
                if (kpt_big == 4)
                    BK_K2(1024, 4, 1024, false);
                else
                    BK_K2(256, 16, 1024, false);
                break;
            case 8192: BK_K2(512, 16, 1024, false); break;
            default: BK_K2(1024, 16, 1024, false); break;
            }
        }
#undef BK_K2
        return hipGetLastError();
    }
    if (r0 != 0 || rows != n) return hipErrorInvalidValue;  // v1 (probe builds): whole calls only
    if (np2 <= 2048) {
        hipLaunchKernelGGL(k_scores<256>, dim3(n), dim3(256), lds, st, U, T, n, np2, k, scores,
                           diag);
    } else {
        hipLaunchKernelGGL(k_scores<1024>, dim3(n), dim3(1024), lds, st, U, T, n, np2, k, scores,
                           diag);
    }
    return hipGetLastError();
}

hipError_t launch_rank(const double *scores, int n, int m, int *mask, double *bnd,
                       hipStream_t st) {
    hipLaunchKernelGGL(k_rank, dim3((n + 3) / 4), dim3(256), 0, st, scores, n, m, mask, bnd);
    return hipGetLastError();
}

// split scoring (bk_api.hip stage_finish): the gathered slices {ch scores,
// status} of `parts` ranks -> the n scores, contiguous; rec = the Gram's
// trailing record dcols[0..2], or NaN words when any rank's status is not 0
__global__ __launch_bounds__(256) void k_split_unpack(const double *__restrict__ sg, int64_t ch,
                                                      int parts, int n,
                                                      const double *__restrict__ dcols,
                                                      double *__restrict__ scores,
                                                      double *__restrict__ rec) {
    const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (i < n) scores[i] = sg[i + i / ch];
    if (blockIdx.x != 0) return;
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    for (int p = (int)threadIdx.x; p < parts; p += 256)
        if (sg[(int64_t)p * (ch + 1) + ch] != 0.0) bad = 1;  // NaN compares unequal too
    __syncthreads();
    if (threadIdx.x < 3) rec[threadIdx.x] = bad ? __builtin_nan("") : dcols[threadIdx.x];
}

hipError_t launch_split_unpack(const double *sg, int64_t ch, int parts, int n, const double *dcols,
                               double *scores, double *rec, hipStream_t st) {
    hipLaunchKernelGGL(k_split_unpack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sg, ch,
                       parts, n, dcols, scores, rec);
    return hipGetLastError();
}

hipError_t launch_compact(const int *mask, int n, int64_t *sel, const double *diag,
                          const double *bnd, const double *dcols, int64_t k, double *margin,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, st, mask, n, sel, diag, bnd, dcols, k,
                       margin);
    return hipGetLastError();
}

template <bool ACCUM>
static hipError_t launch_colsum(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *sel,
                                int m, double *mean, int num_cu, hipStream_t st);

template <bool SEG>
static hipError_t launch_mean_seg(const void *X, int dtype, int64_t ld, int64_t d,
                                  const int64_t *sel, int m, double *out, int num_cu, hipStream_t st);

hipError_t launch_mean(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *sel, int m,
                       double *mean, int num_cu, hipStream_t st, double *seg_part) {
    const int S = mean_segments(m);
    if (S <= 1 || !seg_part) return launch_colsum<false>(X, dtype, ld, d, sel, m, mean, num_cu, st);
    // a large selection: the rows in segments of MEAN_SEG_ROWS (grid y), then
    // the segments in order.  A shard's few columns (config E on 8 GPUs: 32,768
    // fp32 columns, 8,192 column threads) left most CUs idle with one thread
    // walking all m rows: 0.25 ms at 1.5 TB/s
    hipError_t e = launch_mean_seg<true>(X, dtype, ld, d, sel, m, seg_part, num_cu, st);
    if (e != hipSuccess) return e;
    int64_t b = (d + 255) / 256;
    if (b > (int64_t)num_cu * 8) b = (int64_t)num_cu * 8;
    if (b < 1) b = 1;
    hipLaunchKernelGGL(k_mean_comb, dim3((unsigned)b), dim3(256), 0, st, seg_part, S, d, m, mean);
    return hipGetLastError();
}

template <bool SEG>
static hipError_t launch_mean_seg(const void *X, int dtype, int64_t ld, int64_t d,
                                  const int64_t *sel, int m, double *out, int num_cu, hipStream_t st) {
    const int S = mean_segments(m);
    const size_t lds = (size_t)MEAN_SEG_ROWS * sizeof(int64_t);
    const int64_t cap = ((int64_t)num_cu * 16 + S - 1) / S;  // ~16 blocks per CU in all
    const dim3 block(256);
    if (dtype != 0 && (ld % 4) == 0 && ((uintptr_t)X % 16) == 0) {
        int64_t b4 = ((d + 3) / 4 + 255) / 256;
        b4 = b4 > cap ? cap : b4 < 1 ? 1 : b4;
        hipLaunchKernelGGL((k_mean_f4<false, true>), dim3((unsigned)b4, (unsigned)S), block, lds, st,
                           (const float *)X, ld, d, sel, m, out);
        return hipGetLastError();
    }
    int64_t b = ((d + 1) / 2 + 255) / 256;
    b = b > cap ? cap : b < 1 ? 1 : b;
    const dim3 grid((unsigned)b, (unsigned)S);
    const bool vec = dtype == 0 ? ((ld % 2) == 0 && ((uintptr_t)X % 16) == 0)
                                : ((ld % 2) == 0 && ((uintptr_t)X % 8) == 0);
    if (dtype == 0) {
        if (vec)
            hipLaunchKernelGGL((k_mean<double, true, false, true>), grid, block, lds, st, (const double *)X,
                               ld, d, sel, m, out);
        else
            hipLaunchKernelGGL((k_mean<double, false, false, true>), grid, block, lds, st, (const double *)X,
                               ld, d, sel, m, out);
    } else {
        if (vec)
            hipLaunchKernelGGL((k_mean<float, true, false, true>), grid, block, lds, st, (const float *)X, ld,
                               d, sel, m, out);
        else
            hipLaunchKernelGGL((k_mean<float, false, false, true>), grid, block, lds, st, (const float *)X, ld,
                               d, sel, m, out);
    }
    return hipGetLastError();
}

hipError_t launch_accumulate(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *idx,
                             int m, double *global, int num_cu, hipStream_t st) {
    return launch_colsum<true>(X, dtype, ld, d, idx, m, global, num_cu, st);
}

template <bool ACCUM>
static hipError_t launch_colsum(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *sel,
                                int m, double *mean, int num_cu, hipStream_t st) {
    const int64_t npair = (d + 1) / 2;
    int64_t blocks = (npair + 255) / 256;
    const int64_t cap = (int64_t)num_cu * 16;  // 1, 2, 4, 8 per CU: no faster (v13 probe)
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const size_t lds = (size_t)m * sizeof(int64_t);
    const bool vec = dtype == 0 ? ((ld % 2) == 0 && ((uintptr_t)X % 16) == 0)
                                : ((ld % 2) == 0 && ((uintptr_t)X % 8) == 0);
    dim3 grid((unsigned)blocks), block(256);
    if (dtype != 0 && (ld % 4) == 0 && ((uintptr_t)X % 16) == 0) {
        int64_t b4 = ((d + 3) / 4 + 255) / 256;
        if (b4 > (int64_t)num_cu * 16) b4 = (int64_t)num_cu * 16;
        if (b4 < 1) b4 = 1;
        hipLaunchKernelGGL((k_mean_f4<ACCUM>), dim3((unsigned)b4), block, lds, st, (const float *)X, ld,
                           d, sel, m, mean);
        return hipGetLastError();
    }
    if (dtype == 0) {
        if (vec)
            hipLaunchKernelGGL((k_mean<double, true, ACCUM>), grid, block, lds, st, (const double *)X, ld, d,
                               sel, m, mean);
        else
            hipLaunchKernelGGL((k_mean<double, false, ACCUM>), grid, block, lds, st, (const double *)X, ld,
                               d, sel, m, mean);
    } else {
        if (vec)
            hipLaunchKernelGGL((k_mean<float, true, ACCUM>), grid, block, lds, st, (const float *)X, ld, d,
                               sel, m, mean);
        else
            hipLaunchKernelGGL((k_mean<float, false, ACCUM>), grid, block, lds, st, (const float *)X, ld, d,
                               sel, m, mean);
    }
    return hipGetLastError();
}

hipError_t launch_synth(void *X, int dtype, int64_t ld, int64_t n, int64_t dl, int64_t c0,
                        const int64_t *perm, const SynthParams &P, hipStream_t st) {
    int64_t bx = (dl + 255) / 256;
    if (bx > 4096) bx = 4096;
    if (bx < 1) bx = 1;
    dim3 grid((unsigned)bx, (unsigned)n), block(256);
    if (dtype == 0)
        hipLaunchKernelGGL(k_synth<double>, grid, block, 0, st, (double *)X, ld, dl, c0, perm, P);
    else
        hipLaunchKernelGGL(k_synth<float>, grid, block, 0, st, (float *)X, ld, dl, c0, perm, P);
    return hipGetLastError();
}

hipError_t launch_gram3(const void *X, int dtype, int64_t ld, int n, int64_t d, const Plan3 &pl0,
                        double *part, hipStream_t st, int mode, long long *trace, bool f32_mfma,
                        const int *seg, int nwg, const PieceMarks &pm) {
    // mode != 0: timing-only ablations (1: no MFMA, 2: no global loads) -- wrong
    // results, so they exist only in probe builds (-DBK_PROBES); the product ignores mode
    (void)mode;
    // seg / nwg: one piece's launch table (the exchange overlapping the Gram):
    // the same segments and slabs, a subset of the launched workgroups
    Plan3 pl = pl0;
    if (seg) {
        pl.d_seg = const_cast<int *>(seg);
        pl.nwg = nwg;
    }
    if (pl.nwg < 1) return hipSuccess;
    const dim3 grid((unsigned)pl.nwg), block(512);
    if (dtype != 0 && f32_mfma)  // fp32 input on the fp32 MFMA
        hipLaunchKernelGGL((k_gram3<0, f32m>), grid, block, G3_LDS, st, (const f32m *)X, ld, n,
                           pl.nfull, d, pl.d_groups, pl.d_seg, pl.d_wg, part, trace, pm);
    else if (dtype != 0)  // fp32 input, exact (widened onto the fp64 MFMA): production mode only
        hipLaunchKernelGGL((k_gram3<0, float>), grid, block, G3_LDS, st, (const float *)X, ld, n,
                           pl.nfull, d, pl.d_groups, pl.d_seg, pl.d_wg, part, trace, pm);
#ifdef BK_PROBES
    else if (mode == 1)
        hipLaunchKernelGGL(k_gram3<1>, grid, block, G3_LDS, st, (const double *)X, ld, n, pl.nfull,
                           d, pl.d_groups, pl.d_seg, pl.d_wg, part, trace, pm);
    else if (mode == 2)
        hipLaunchKernelGGL(k_gram3<2>, grid, block, G3_LDS, st, (const double *)X, ld, n, pl.nfull,
                           d, pl.d_groups, pl.d_seg, pl.d_wg, part, trace, pm);
#endif
    else
        hipLaunchKernelGGL(k_gram3<0>, grid, block, G3_LDS, st, (const double *)X, ld, n, pl.nfull,
                           d, pl.d_groups, pl.d_seg, pl.d_wg, part, trace, pm);
    return hipGetLastError();
}

hipError_t launch_reduce3(const double *part, const Plan3 &pl, double *U, hipStream_t st,
                          bool f32_mfma, int u0, int u1, bool rec) {
    const int64_t usz = (int64_t)pl.ntile * 4096;
    const double d32 = f32_mfma ? (double)pl.d : 0.0;
    if (u1 < 0) u1 = pl.ntile;
    if (u1 <= u0) return hipSuccess;
#ifndef BK_REDUCE_V1
    hipLaunchKernelGGL(k_reduce3, dim3((unsigned)(u1 - u0) * 64), dim3(256), 0, st, part, pl.d_red,
                       pl.d_wglist, U, usz, (double)pl.d, d32, u0, rec ? 1 : 0);
#else
    hipLaunchKernelGGL(k_reduce3, dim3((unsigned)(u1 - u0) * 128), dim3(256), 0, st, part, pl.d_red,
                       pl.d_wglist, U, usz, (double)pl.d, d32, u0, rec ? 1 : 0);
#endif
    return hipGetLastError();
}

hipError_t configure_kernels() {
    for (const void *k : {(const void *)k_gram3<0>, (const void *)k_gram3<0, float>,
                          (const void *)k_gram3<0, f32m>}) {
        hipError_t e0 = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS);
        if (e0 != hipSuccess) return e0;
    }
#ifdef BK_PROBES
    for (const void *k : {(const void *)k_gram3<1>, (const void *)k_gram3<2>}) {
        hipError_t e0 = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS);
        if (e0 != hipSuccess) return e0;
    }
#endif
    // the row sort may need up to BK_MAX_N * 8 = 128 KiB of dynamic LDS
    hipError_t e = hipFuncSetAttribute((const void *)k_scores<1024>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void *)k_scores<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            131072);
    if (e != hipSuccess) return e;
    for (const void *kk : {(const void *)k_scores2<256, 16, 1024, false>,
                           (const void *)k_scores2<512, 16, 1024, false>,
                           (const void *)k_scores2<1024, 16, 1024, false>,
                           (const void *)k_scores2<1024, 4, 1024, false>,
                           (const void *)k_scores2<256, 16, 1024, true>,
                           (const void *)k_scores2<512, 16, 1024, true>,
                           (const void *)k_scores2<1024, 16, 1024, true>,
                           (const void *)k_scores2<1024, 4, 1024, true>,
#ifdef BK_PROBES  // the timing-only K2 ablations (BK_K2_MODE)
                           (const void *)k_scores2<256, 16, 1024, false, 1>,
                           (const void *)k_scores2<512, 16, 1024, false, 1>,
                           (const void *)k_scores2<1024, 16, 1024, false, 1>,
                           (const void *)k_scores2<1024, 4, 1024, false, 1>,
                           (const void *)k_scores2<256, 16, 1024, false, 2>,
                           (const void *)k_scores2<512, 16, 1024, false, 2>,
                           (const void *)k_scores2<1024, 16, 1024, false, 2>,
                           (const void *)k_scores2<1024, 4, 1024, false, 2>,
                           (const void *)k_scores2<256, 16, 1024, true, 1>,
                           (const void *)k_scores2<512, 16, 1024, true, 1>,
                           (const void *)k_scores2<1024, 16, 1024, true, 1>,
                           (const void *)k_scores2<1024, 4, 1024, true, 1>,
                           (const void *)k_scores2<256, 16, 1024, true, 2>,
                           (const void *)k_scores2<512, 16, 1024, true, 2>,
                           (const void *)k_scores2<1024, 16, 1024, true, 2>,
                           (const void *)k_scores2<1024, 4, 1024, true, 2>,
#endif
                       }) {
        e = hipFuncSetAttribute(kk, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024);  // v3 at N = 16384: 136 KiB
        if (e != hipSuccess) return e;
    }
    // the masked column sums keep up to BK_MAX_N row offsets in LDS
    for (const void *k : {(const void *)k_mean<double, true, false>,
                          (const void *)k_mean<double, false, false>,
                          (const void *)k_mean<float, true, false>,
                          (const void *)k_mean<float, false, false>,
                          (const void *)k_mean<double, true, true>,
                          (const void *)k_mean<double, false, true>,
                          (const void *)k_mean<float, true, true>,
                          (const void *)k_mean<float, false, true>,
                          (const void *)k_mean_f4<false>, (const void *)k_mean_f4<true>}) {
        e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace bk
