// bk_small.hip -- the whole Multi-Krum of a SMALL batch in ONE launch.
//
// Biscotti's verifiers run n <= 100 (config B, mnist: 100 x 7,850; config A,
// creditcard: n <= 10, d = 25; usenix-eval runs n = 28..70).  There the six
// dependent launches of the general path (K1, K1b, K2, K3, K3b, K4) ARE the
// cost: each takes 4-9 us however little it computes (rocprof of config B:
// 58 us per step, profiles/r02).  k_small does the same work in one
// persistent launch whose workgroups pull ITEMS from a queue (one returning
// atomic per item) in dependency order:
//
//   G items  (4 per 128    split-K Gram partial of 128 columns: a quarter of
//             columns)     the upper 16x16 blocks of the (n <= 128) Gram
//                          each, fp64 MFMA
//   S items  (one per row) the row's Gram entries and the diagonal summed
//                          over the P partials in a fixed order (no separate
//                          reduce phase), distances, sort by counting, sum of
//                          ranks 1..k in K2's exact shape
//   M items  (64 columns)  stage the item's columns of every row in LDS while
//                          the scores are computed; then rank the n scores
//                          (each item itself: no serial selection step),
//                          compact the selection, mean of the selected rows
//                          ascending from LDS (K4's order); item 0 writes sel
//                          and the margin
//
// The first G items go to workgroups 0.. by blockIdx, the rest are dequeued
// in order.  An item only waits (a relaxed sc1 poll of a counter) for items
// before it: dequeued ones run on running workgroups, and the statically held
// G items wait for nothing, so their workgroups finish once dispatched.  No
// co-residency is assumed, only that every workgroup of the grid (<= one per
// CU) is eventually dispatched (MI355X_MICROARCH.md, "Workgroup dispatch").  Hand-offs are the guide's write-through form ("Valid forms",
// table row 1): EVERY store of handed-off bytes is an sc1 store (agent-scope
// relaxed atomic store), every storing wave drains vmcnt(0), a workgroup
// barrier, then one lane's agent-scope atomic add; EVERY load of them is an
// sc1 load.  No release / acquire fences: a buffer_wbl2 writes back the XCD's
// dirty L2 (~6.5 us with fresh data), which cost the first version 85 us.
// The last workgroup to exit resets the counters for the next launch.  A wait
// gives up after ~1 s and raises an error word instead of hanging the GPU.
// Results are deterministic: every sum has a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "bk_device.h"
#include "bk_internal.h"

namespace bk {

// queue words, each on a 128-B line of its own: the item head, the top
// arrival counters of the G and S phases (C_R, F_R, R_GRP: the lines of the
// former reduce phase, unused since S items sum the partials themselves), a
// spare line, the error word; then the "phase done" flags F_G, F_S, each
// replicated once per XCD (a waiting workgroup polls its own XCD's copy: 1/8
// of the pollers on any line); then the arrival counters of groups of 32
// items (G_GRP: up to 1024 G items, S_GRP: 128 S items).  Same-address atomics
// serialize at ~11 ns each, so 246 G items arriving together on one counter
// took ~2.7 us; a group's last arriver (told by its add's return value) adds
// once to the phase's top counter instead.
enum { C_HEAD = 0, C_G = 1, C_R = 2, C_S = 3, C_SPARE = 4, C_ERR = 5, F_G = 6, F_R = 14, F_S = 22,
       G_GRP = 30, R_GRP = 62, S_GRP = 67, C_LINES = 71 };
static_assert(C_LINES * 32 == SMALL_CTR_WORDS, "bk_internal.h SMALL_CTR_WORDS");
#ifndef BK_SMALL_KC
#define BK_SMALL_KC 128
#endif
constexpr int SMALL_KC = BK_SMALL_KC;  // columns per chunk (groups of 8)
constexpr int SMALL_GR = SMALL_KC / 2;  // 16-B granules per staged row
constexpr int SMALL_SPLIT = SMALL_SPLIT_ITEMS;  // G items per chunk (each: a quarter of the blocks)
#ifndef BK_SMALL_NT
#define BK_SMALL_NT 512
#endif
// threads per k_small workgroup: 256 (one wave per SIMD) or 512 (two: the
// MFMA pipe issues back to back only from two waves, tools/ubench_fp64_data:
// 71 vs 77 TF/s, and the rank loops split over four threads per key)
constexpr int SMALL_NT = BK_SMALL_NT;
constexpr int SMALL_NW = SMALL_NT / 64;  // waves per workgroup
static_assert(SMALL_NT == 256 || SMALL_NT == 512, "k_small runs 4 or 8 waves");

// G item it -> (chunk c, part h).  The SPLIT parts of a chunk are items 8
// apart, so under the static first assignment (workgroup b runs item b;
// blocks b, b + 8 share an XCD) they stage the same columns through one L2
__device__ __forceinline__ void g_item(int it, int P, int &c, int &h) {
    const int full = (P >> 3) * (8 * SMALL_SPLIT);
    if (it < full) {
        h = (it >> 3) % SMALL_SPLIT;
        c = 8 * (it / (8 * SMALL_SPLIT)) + (it & 7);
    } else {
        const int t = it - full, r = P & 7;
        h = t / r;
        c = (P & ~7) + t % r;
    }
}

struct SmallArgs {
    const void *X;
    int64_t ld, d;
    int n, f, kc, P, Q, nS, C, nblk, T;
    // the launch's share (bk_multikrum's pipelined host entry, config B): the G
    // items of chunks [g0, g0 + gn) and, with sm, the S and M items.  The
    // one-launch call: g0 = 0, gn = P, sm = 1.  A G-only launch (sm = 0) hands
    // its partials to the next launch on the stream by the kernel boundary; an
    // S+M-only launch (gn = 0) finds every partial written
    int g0, gn, sm;
    double *part, *U, *scores, *diag, *mean, *margin;
    double *scores_out;  // optional second copy of the scores (the host entry's mapped block)
    int64_t *sel;
    unsigned *ctr;
    uint64_t spin_max;  // polls before a wait gives up (~1 s; a test knob lowers it)
    int check_lines;    // debug: the last workgroup out checks every queue word
    long long *trace;  // debug (BK_SMALL_TRACE): per item {start, waited, end, hw id,
                       // shader clock at start, at end, two in-item stamps}
};

__device__ __forceinline__ unsigned ctr_load(const unsigned *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the handed-off bytes: sc1 (write-through) stores and sc1 loads
template <typename V>
__device__ __forceinline__ void st1(V *p, V v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename V>
__device__ __forceinline__ V ld1(const V *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-B sc1 load at byte offset off of a wave-uniform base (buffer_load_dwordx4
// ... sc1: bypasses L1, served from L2 / memory)
__device__ __forceinline__ d2v ld1_16(const double *base, unsigned nbytes, unsigned off) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base), 0, nbytes, 0x00020000);
    return __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

// 16-B write-through (sc1) store at byte offset off of a wave-uniform base
// (MI355X_MICROARCH.md: narrow sc1 stores cost ~2.7x per byte)
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st1_16(double *base, unsigned nbytes, unsigned off, d2v v) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(base, 0, nbytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), r, off, 0, 16);
}

// G_ij from the packed upper tiles (u_at) with sc1 loads
__device__ __forceinline__ double u_at1(const double *U, int T, int r, int c) {
    const int br = r >> 6, bc = c >> 6, ir = r & 63, ic = c & 63;
    if (br < bc || (br == bc && ir <= ic)) return ld1(U + upper_tile(T, br, bc) + ir * 64 + ic);
    return ld1(U + upper_tile(T, bc, br) + ic * 64 + ir);
}

__device__ __forceinline__ unsigned *cline(unsigned *ctr, int line) { return ctr + 32 * line; }

// debug trace: in-item stamp q (0, 1) of the current item (tr = its record)
__device__ __forceinline__ void stamp(long long *tr, int q) {
    if (tr && threadIdx.x == 0) tr[6 + q] = (long long)__builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ int xcc_id() {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return (int)(x & 7);
}

// wait for a phase's flag (lane 0 polls this XCD's copy), then the workgroup
// goes on: its loads of the handed-off bytes are sc1 loads, after this barrier
__device__ __forceinline__ void wg_wait_flag(unsigned *ctr, int flag, uint64_t spin_max) {
    if (threadIdx.x == 0) {
        const unsigned *p = cline(ctr, flag + xcc_id());
        uint64_t spins = 0;
        while (ctr_load(p) == 0u) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > spin_max) {  // ~1 s: never hang the GPU on a broken hand-off
                __hip_atomic_fetch_or(cline(ctr, C_ERR), 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

// every wave drains its sc1 stores, then one lane counts the arrival of item
// idx (of count) on its group's counter; the group's last arriver counts the
// group on the phase's top counter, and the workgroup whose top add returns
// ngroups - 1 sees every other producer's bytes (the guide's row 1: the last
// adder, told by the value its add returned; each group's last adder saw its
// members' adds, which followed their drained sc1 stores)
__device__ __forceinline__ bool wg_arrive(unsigned *ctr, int top, int grp, int idx, int count,
                                          unsigned *s_last) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int g = idx >> 5, gs = count - 32 * g < 32 ? count - 32 * g : 32;
        const unsigned ng = (unsigned)((count + 31) >> 5);
        unsigned last = 0;
        if (__hip_atomic_fetch_add(cline(ctr, grp + g), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) == (unsigned)gs - 1u)
            last = __hip_atomic_fetch_add(cline(ctr, top), 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) == ng - 1u;
        *s_last = last;
    }
    __syncthreads();
    return *s_last != 0;
}

// the last arriver raises a phase flag on every XCD's copy (one wave
// instruction, 8 lanes, sc1 stores), after its own stores have drained
__device__ __forceinline__ void wg_raise(unsigned *ctr, int flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 8) st1(cline(ctr, flag + (int)threadIdx.x), 1u);
}

// upper 16x16 block b (row-major over bi <= bj) of an NB x NB block grid
__host__ __device__ constexpr int blk_bi(int b, int NB) {
    int bi = 0;
    while (b >= NB - bi) {
        b -= NB - bi;
        ++bi;
    }
    return bi;
}
__host__ __device__ constexpr int blk_bj(int b, int NB) {
    int bi = 0;
    while (b >= NB - bi) {
        b -= NB - bi;
        ++bi;
    }
    return bi + b;
}

typedef double d4 __attribute__((ext_vector_type(4)));

// sub-step S (0: columns 2g, 1: 2g+1) of this wave's blocks J.. per 8-column
// group; block positions are compile-time, so the fragments stay in registers
template <int NB, int W, int S, int J, int NJ, int NW>
__device__ __forceinline__ void small_mma_s(d4 *acc, const d2v (&fr)[NB]) {
    if constexpr (J < NJ) {
        constexpr int b = W + NW * J;
        constexpr int bi = blk_bi(b, NB), bj = blk_bj(b, NB);
        acc[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[bi][S], fr[bj][S], acc[J], 0, 0, 0);
        small_mma_s<NB, W, S, J + 1, NJ, NW>(acc, fr);
    }
}
// both sub-steps, blocks interleaved: consecutive MFMAs never share an
// accumulator; wave W of NW owns blocks W, W + NW, ...
template <int NB, int W, int J, int NJ, int NW>
__device__ __forceinline__ void small_mma(d4 *acc, const d2v (&fr)[NB]) {
    small_mma_s<NB, W, 0, J, NJ, NW>(acc, fr);
    small_mma_s<NB, W, 1, J, NJ, NW>(acc, fr);
}

// 2 consecutive elements as fp64; VEC: one 16-B (fp64) / 8-B (fp32) load,
// else two scalar loads (rows not aligned for it: odd ld, e.g. config A's d = 25)
template <typename T, bool VEC>
__device__ __forceinline__ d2v sm_ld2(const T *p) {
    if constexpr (!VEC) {
        return d2v{(double)p[0], (double)p[1]};
    } else if constexpr (sizeof(T) == 8) {
        return *reinterpret_cast<const d2v *>(p);
    } else {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 v = *reinterpret_cast<const f2 *>(p);
        return d2v{(double)v.x, (double)v.y};
    }
}

// G item s, wave W: the blocks b = W, W + 4, ... of the NB x NB upper grid over
// columns [c0, c1).  Lane (rr, g) holds columns 2g, 2g+1 of each 8-column group
// (the same k permutation for A and B, so the product is exactly X X^T); the
// output element (row g + 4r, col rr) of a 16x16 block sits in register r.
// G item s: the item's rows x 64 columns are staged in LDS once (every load
// in flight, coalesced 512-B rows; a per-wave re-load of every row-block took
// 11 us per item), granules XOR-swizzled by (row & 31) so the fragment reads
// (16 rows x 16 B per lane group) hit distinct banks
__device__ __forceinline__ int sg_off(int row, int gran) {
    return row * (SMALL_GR * 16) + ((gran ^ (row & (SMALL_GR - 1))) << 4);
}

template <typename T, bool VEC, int NB, int NT = SMALL_NT>
struct SmallStage {
    static constexpr int ROWS = 16 * NB;
    static constexpr int PER = (ROWS * SMALL_GR + NT - 1) / NT;  // 16-B granules per thread
    d2v v[PER];
    // every load of the item in flight at once (coalesced rows)
    __device__ __forceinline__ void load(const SmallArgs &a, int s, int tid) {
        const T *X = (const T *)a.X;
        const int64_t c0 = (int64_t)s * SMALL_KC;
        const int len = (int)(c0 + SMALL_KC < a.d ? SMALL_KC : a.d - c0);
        static_assert(PER * NT == ROWS * SMALL_GR, "every thread stages PER whole granules");
        const int len2 = len & ~1;  // whole column pairs of this chunk (KC but for the last)
        if (VEC && len2 >= 2) {
            // ONE code path for full chunks and the ragged last one: 16-B loads
            // at clamped pairs, columns past the chunk zeroed by a select, no
            // branch per load.  A separate path for the ragged chunk ran its
            // items ~3-5 us behind the others (its code ran cold from the
            // instruction cache on the few CUs that took it), and the phase
            // waits for the last item
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int gidx = tid + NT * q;
                const int row = gidx / SMALL_GR, col = 2 * (gidx % SMALL_GR);
                const T *p = X + (int64_t)min(row, a.n - 1) * a.ld + c0;
                const d2v pr = sm_ld2<T, true>(p + (col < len2 ? col : len2 - 2));
                v[q] = d2v{col < len2 ? pr.x : 0.0, col + 1 < len2 ? pr.y : 0.0};
            }
            if (len & 1) {  // an odd ragged chunk: its last column (rare)
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    const int gidx = tid + NT * q;
                    const int row = gidx / SMALL_GR, col = 2 * (gidx % SMALL_GR);
                    if (col == len - 1) v[q].x = (double)X[(int64_t)min(row, a.n - 1) * a.ld + c0 + col];
                }
            }
            return;
        }
        // unaligned rows (or a 1-column chunk): element loads at clamped
        // columns, out-of-range ones zeroed by a select
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int gidx = tid + NT * q;
            const int row = gidx / SMALL_GR, col = 2 * (gidx % SMALL_GR);
            const T *p = X + (int64_t)min(row, a.n - 1) * a.ld + c0;
            const double x0 = (double)p[col < len ? col : len - 1];
            const double x1 = (double)p[col + 1 < len ? col + 1 : len - 1];
            v[q] = d2v{col < len ? x0 : 0.0, col + 1 < len ? x1 : 0.0};
        }
    }
    // granules [g0, g1) of every row into LDS
    __device__ __forceinline__ void store(char *tile, int g0, int g1, int tid) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int gidx = tid + NT * q;
            const int row = gidx / SMALL_GR, gr = gidx % SMALL_GR;
            if (gr >= g0 && gr < g1) *reinterpret_cast<d2v *>(tile + sg_off(row, gr)) = v[q];
        }
    }
};

// the MFMAs of 8-column groups [t0, t1) of the staged tile, blocks J0 .. J1-1
// of this wave's list
template <int NB, int W, int J0, int J1, int NW = SMALL_NW>
__device__ __forceinline__ void small_gram_groups(d4 *acc, const char *tile, int lane, int t0,
                                                  int t1) {
    const int rr = lane & 15, g = lane >> 4;
    if constexpr (J1 > J0) {
#pragma unroll
        for (int t = 0; t < SMALL_KC / 8; ++t) {
            if (t < t0 || t >= t1) continue;
            d2v fr[NB];
#pragma unroll
            for (int rb = 0; rb < NB; ++rb)
                fr[rb] = *reinterpret_cast<const d2v *>(tile + sg_off(16 * rb + rr, 4 * t + g));
            small_mma<NB, W, J0, J1, NW>(acc, fr);
        }
    }
}

// G item (chunk c, part PART): columns [KC c, KC c + KC) staged once, then
// wave W runs part PART of its blocks b = W + 4 j (the j range cut in SPLIT
// pieces), so the Gram's MFMAs spread over SPLIT times as many CUs while a
// chunk's partial (one per KC columns, the same bytes whatever KC is) is
// written once per KC columns; the partials written sc1.  (Staging half the columns and computing it while the other half
// landed was 1.3 us slower per item: one more barrier.)
template <typename T, bool VEC, int NB, int W, int PART>
__device__ __forceinline__ void small_gram_wave(const SmallArgs &a, int c, long long *tr, int lane,
                                                char *tile, SmallStage<T, VEC, NB> &st, double *wb) {
    constexpr int NBLK = NB * (NB + 1) / 2;
    constexpr int NJ = (NBLK - W + SMALL_NW - 1) / SMALL_NW;  // this wave's blocks
    constexpr int J0 = PART * NJ / SMALL_SPLIT, J1 = (PART + 1) * NJ / SMALL_SPLIT;
    constexpr int NG = SMALL_KC / 8;
    const int rr = lane & 15, g = lane >> 4;
    d4 acc[NJ > 0 ? NJ : 1];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = d4{0.0, 0.0, 0.0, 0.0};
    st.store(tile, 0, SMALL_GR, lane + 64 * W);
    __syncthreads();
    stamp(tr, 0);
    small_gram_groups<NB, W, J0, J1>(acc, tile, lane, 0, NG);
    if (W == 0) {  // wave 0's MFMAs done (debug trace only)
        if (tr && J1 > J0) asm volatile("s_nop 0" ::"v"(acc[J0][0]));
        stamp(tr, 1);
    }
    // the chunk's partial Gram in full-square layout (row-major NP x NP, NP =
    // 16 NB) plus its diagonal as a contiguous vector, so that an S item reads
    // its row and every G_jj in coalesced runs.  Each block goes through this
    // wave's 16 x 17 LDS scratch and out as 16-B sc1 stores: as it is and
    // transposed for an off-diagonal block; a diagonal block is first made
    // symmetric from its upper elements (as the packed upper U held them), so
    // the square is exactly symmetric
    constexpr int NP = 16 * NB;
    constexpr unsigned NBYTES = (NP * NP + NP) * 8;
    double *sq = a.part + (int64_t)__builtin_amdgcn_readfirstlane(c) * (NP * NP + NP);
#pragma unroll
    for (int j = J0; j < J1; ++j) {
        const int b = W + SMALL_NW * j;
        const int bi = blk_bi(b, NB), bj = blk_bj(b, NB);
#pragma unroll
        for (int r = 0; r < 4; ++r) wb[(g + 4 * r) * 17 + rr] = (double)acc[j][r];
        if (bi == bj) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (g + 4 * r > rr) wb[(g + 4 * r) * 17 + rr] = wb[rr * 17 + g + 4 * r];
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int gi = lane + 64 * q, row = gi >> 3, gc = gi & 7;
            st1_16(sq, NBYTES, ((16 * bi + row) * NP + 16 * bj + 2 * gc) * 8,
                   d2v{wb[row * 17 + 2 * gc], wb[row * 17 + 2 * gc + 1]});
            if (bi != bj)
                st1_16(sq, NBYTES, ((16 * bj + row) * NP + 16 * bi + 2 * gc) * 8,
                       d2v{wb[(2 * gc) * 17 + row], wb[(2 * gc + 1) * 17 + row]});
        }
        if (bi == bj && lane < 8)
            st1_16(sq, NBYTES, (NP * NP + 16 * bi + 2 * lane) * 8,
                   d2v{wb[(2 * lane) * 17 + 2 * lane], wb[(2 * lane + 1) * 17 + 2 * lane + 1]});
    }
}

template <typename T, bool VEC, int NB, int W>
__device__ __forceinline__ void small_gram_w(const SmallArgs &a, int c, int h, long long *tr,
                                             int lane, char *tile, SmallStage<T, VEC, NB> &st,
                                             double *wb) {
    static_assert(SMALL_SPLIT == 4, "parts");
    switch (h) {
    case 0: small_gram_wave<T, VEC, NB, W, 0>(a, c, tr, lane, tile, st, wb); break;
    case 1: small_gram_wave<T, VEC, NB, W, 1>(a, c, tr, lane, tile, st, wb); break;
    case 2: small_gram_wave<T, VEC, NB, W, 2>(a, c, tr, lane, tile, st, wb); break;
    default: small_gram_wave<T, VEC, NB, W, 3>(a, c, tr, lane, tile, st, wb); break;
    }
}

template <typename T, bool VEC, int NB>
__device__ __forceinline__ void small_gram(const SmallArgs &a, int it, int wave, int lane,
                                           char *tile, double *wb) {
    int c, h;
    g_item(it, a.gn, c, h);
    c += a.g0;
    long long *tr = a.trace ? a.trace + 8 * (int64_t)it : nullptr;
    SmallStage<T, VEC, NB> st;
    st.load(a, c, lane + 64 * wave);
    switch (wave) {
    case 0: small_gram_w<T, VEC, NB, 0>(a, c, h, tr, lane, tile, st, wb); break;
    case 1: small_gram_w<T, VEC, NB, 1>(a, c, h, tr, lane, tile, st, wb); break;
    case 2: small_gram_w<T, VEC, NB, 2>(a, c, h, tr, lane, tile, st, wb); break;
#if BK_SMALL_NT == 512
    case 3: small_gram_w<T, VEC, NB, 3>(a, c, h, tr, lane, tile, st, wb); break;
    case 4: small_gram_w<T, VEC, NB, 4>(a, c, h, tr, lane, tile, st, wb); break;
    case 5: small_gram_w<T, VEC, NB, 5>(a, c, h, tr, lane, tile, st, wb); break;
    case 6: small_gram_w<T, VEC, NB, 6>(a, c, h, tr, lane, tile, st, wb); break;
    default: small_gram_w<T, VEC, NB, 7>(a, c, h, tr, lane, tile, st, wb); break;
#else
    default: small_gram_w<T, VEC, NB, 3>(a, c, h, tr, lane, tile, st, wb); break;
#endif
    }
}

// upper 16x16 block index of block (bi <= bj) in an NB x NB grid (row-major)
__device__ __forceinline__ int blk_idx(int bi, int bj, int NB) {
    return bi * NB - bi * (bi - 1) / 2 + (bj - bi);
}

// S item i: row i with the whole workgroup, straight from the G items'
// full-square partials (no separate reduce phase): G_ij (the upper element
// (min, max), as the packed upper U held it) and every G_jj, each summed over
// the P chunk partials in chunk order.  Then the distances, a sort by
// counting (thread t ranks key t & 127 against half of the row, t >> 7; key e
// goes to position #{keys before it in the (value, index) total order}), and
// K2's summation with its own 256 threads: thread t sums rank 1 + t, the wave
// butterfly, the 4 waves in order -- the same sorted array and the same
// shape, so the score is K2's bitwise for the same Gram.
template <int NB>
__device__ __forceinline__ void small_scores(const SmallArgs &a, int i, int tid, uint64_t *kbuf,
                                             double *sbuf, int *rk, double *gv, d2v *gv2,
                                             double *red, long long *tr) {
    const int n = a.n, lane = tid & 63, wave = tid >> 6;
    const int64_t k = n - a.f - 2 > 0 ? n - a.f - 2 : 0;
    // 16-B element pairs of the row (NP/2) and of the diagonal vector (NP/2),
    // each summed over the P chunk partials in two fixed chains (chunks
    // [0, P/2) and [P/2, P), each in order), then chain 0 + chain 1; a
    // wave's lanes read consecutive 16-B granules (sc1 16-B loads move ~1.5x
    // the bytes per second of 8-B ones)
    const int NP = 16 * NB;
    const int64_t stride = (int64_t)NP * NP + NP;
    const int pr = tid % NP, ch = tid / NP;  // pair pr < NP (row: pr < NP/2), chain ch < 256/NP
    const int half = (a.P + 1) >> 1;
    if (ch < 2) {
        const unsigned e0 = pr < NP / 2 ? (unsigned)(i * NP + 2 * pr) : (unsigned)(NP * NP + 2 * pr - NP);
        const unsigned nbytes = (unsigned)(a.P * stride * 8);
        const int sb = ch ? half : 0, se = ch ? a.P : half;
        d2v acc = {0.0, 0.0};
        for (int s0 = sb; s0 < se; s0 += 32) {  // P <= 256: 4 rounds at most
            d2v v[32];
            // every load unconditional (past the chain's end: its last chunk
            // again, dropped below), so no branch per load; acc starts at
            // +0.0 and is never -0.0, so adding +0.0 leaves it bit for bit
#pragma unroll
            for (int u = 0; u < 32; ++u)
                v[u] = ld1_16(a.part, nbytes, (unsigned)((e0 + (s0 + u < se ? s0 + u : se - 1) * stride) * 8));
#pragma unroll
            for (int u = 0; u < 32; ++u) {
                const bool on = s0 + u < se;
                acc.x += on ? v[u].x : 0.0;
                acc.y += on ? v[u].y : 0.0;
            }
        }
        gv2[ch * NP + pr] = acc;
    }
    __syncthreads();
    // gv[j] = G_ij (j < NP), gv[NP + j] = G_jj
    if (tid < NP) {
        const d2v c0 = gv2[tid], c1 = gv2[NP + tid];
        gv[2 * tid] = c0.x + c1.x;
        gv[2 * tid + 1] = c0.y + c1.y;
    }
    __syncthreads();
    stamp(tr, 0);
    const int e = tid & 127, h = tid >> 7;
    const double di = gv[NP + i];
    if (h == 0) {
        uint64_t key = ~0ULL;  // padding sorts last
        if (e < n) key = dkey((di + gv[NP + e]) - 2.0 * gv[e]);
        kbuf[e] = key;
    }
    __syncthreads();
    const uint64_t key = kbuf[e];
    // the P2 = NT / 128 threads of key e each compare it against NP / P2
    // keys: the keys past NP (padding) never precede a real one, so the real
    // keys' positions are unchanged
    constexpr int P2 = SMALL_NT / 128, HK = 16 * NB / P2, U = HK % 8 == 0 ? 8 : 4;
    int cnt = 0;
#pragma unroll
    for (int j0 = 0; j0 < HK; j0 += U) {
        uint64_t o[U];
#pragma unroll
        for (int u = 0; u < U; ++u) o[u] = kbuf[HK * h + j0 + u];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = HK * h + j0 + u;
            cnt += (o[u] < key) || (o[u] == key && j < e);
        }
    }
    if (h >= 1) rk[(h - 1) * 128 + e] = cnt;
    __syncthreads();
    if (h == 0 && e < 16 * NB) {
#pragma unroll
        for (int q = 1; q < P2; ++q) cnt += rk[(q - 1) * 128 + e];
        sbuf[cnt] = dkey_inv(key);
    }
    __syncthreads();
    stamp(tr, 1);
    double acc = 0.0;
    if (1 + tid <= k && 1 + tid < 128) acc += sbuf[1 + tid];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0 && wave < 4) red[wave] = acc;  // K2's shape: 4 waves (any more hold +0.0)
    __syncthreads();
    if (tid == 0) {
        double sum = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w) sum += red[w];
        st1(a.scores + i, k > 0 ? sum : 0.0);
        st1(a.diag + i, di);
    }
}

// M item c, part 1 (before the scores exist): columns [64 c, 64 c + 64) of
// every row into LDS as fp64 (exact for fp32 rows), every load in flight --
// so after the scores only LDS work is left.  Thread t: column t & 63, rows
// t >> 6, + 4, ...
template <typename T, int NB>
__device__ __forceinline__ void small_mean_stage(const SmallArgs &a, int c, int tid, double *cols) {
    if (!a.mean) return;
    const int cl = tid & 63, r0 = tid >> 6;
    const int64_t col = (int64_t)c * 64 + cl;
    const T *X = (const T *)a.X + (col < a.d ? col : a.d - 1);
    // rows r0, r0 + NW, ... < 16 NB (rows past n repeat row n - 1: loads
    // without a guard, and the mean's mask never selects them)
    constexpr int RU = 16 * NB / SMALL_NW;
    double v[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
        const int r = r0 + SMALL_NW * u;
        v[u] = (double)X[(int64_t)(r < a.n ? r : a.n - 1) * a.ld];
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) cols[(r0 + SMALL_NW * u) * 64 + cl] = v[u];
}

// M item c, part 2: every M item ranks the n published scores itself (n <=
// 128: one LDS pass, no separate selection hand-off), compacts the selection
// with ballots, and sums its 64 staged columns of the m selected rows in
// ascending order from LDS (K4's order: the same bits).  Item 0 also writes
// sel and the margin.
template <int NB>
__device__ __forceinline__ void small_mean(const SmallArgs &a, int c, int tid, int wave, int lane,
                                           uint64_t *keys, int *srow, double *dg, double *bnd,
                                           uint64_t *balw, int *rkm, const double *cols,
                                           long long *tr) {
    const int n = a.n, m = n - a.f;
    double si = 0.0;
    if (tid < n) {
        si = ld1(a.scores + tid);
        keys[tid] = dkey(si);
    } else if (tid < 128) {
        keys[tid] = ~0ULL;  // padding: after every real key (NaN included)
    } else if (c == 0 && tid - 128 < n) {
        dg[tid - 128] = ld1(a.diag + tid - 128);
    }
    __syncthreads();
    stamp(tr, 0);
    // rank of row e in the (score, index) total order: threads e and 128 + e
    // count over the two halves of the NP = 16 NB (padded) keys -- a fixed
    // trip count, every LDS read issued ahead, no branch
    const int e = tid & 127, h = tid >> 7;
    const uint64_t ki = keys[e];
    // P2 parts of the NP = 16 NB keys (n <= NP: no real key past them)
    constexpr int P2 = SMALL_NT / 128, HK = 16 * NB / P2, U = HK % 8 == 0 ? 8 : 4;
    int cnt = 0;
#pragma unroll
    for (int j0 = 0; j0 < HK; j0 += U) {
        uint64_t o[U];
#pragma unroll
        for (int u = 0; u < U; ++u) o[u] = keys[HK * h + j0 + u];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = HK * h + j0 + u;
            cnt += (o[u] < ki) || (o[u] == ki && j < e);
        }
    }
    if (h >= 1 && e < n) rkm[(h - 1) * 128 + e] = cnt;
    __syncthreads();
    bool on = false;
    if (h == 0 && e < n) {
#pragma unroll
        for (int q = 1; q < P2; ++q) cnt += rkm[(q - 1) * 128 + e];
        on = cnt < m;
        if (c == 0 && cnt == m - 1) bnd[0] = si;
        if (c == 0 && cnt == m) bnd[1] = si;
        if (c == 0 && a.scores_out) a.scores_out[e] = si;
    }
    // compaction: rows 0..63 in wave 0, 64..127 in wave 1
    const uint64_t bal = __ballot(on);
    if (wave < 2 && lane == 0) balw[wave] = bal;
    __syncthreads();
    if (on) {
        const int pos = (wave ? __popcll(balw[0]) : 0) + __popcll(bal & ((1ull << lane) - 1));
        srow[pos] = tid;
        if (c == 0 && a.sel) a.sel[pos] = (int64_t)tid;
    }
    if (c == 0 && wave == 3) {
        double M = 0.0;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = lane + 64 * q;
            if (j < n) {
                const double v = dg[j];
                if (v == v && v < __builtin_inf() && v > M) M = v;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) M = fmax(M, __shfl_xor(M, o));
        if (lane == 0) {
            const int64_t k = n - a.f - 2 > 0 ? n - a.f - 2 : 0;
            write_margin(a.margin, bnd[0], bnd[1], M, (double)a.d, k, 0x1p-53);
        }
    }
    __syncthreads();
    stamp(tr, 1);
    if (!a.mean || wave != 0) return;
    // one column per lane of wave 0: the 16 NB staged rows in ascending order
    // from LDS (immediate-offset reads, no index chain, no branch), each
    // row's value or +0.0 by the selection mask.  acc starts at +0.0 and a round-to-nearest sum is
    // -0.0 only if both addends are, so acc is never -0.0 and acc + 0.0 == acc
    // bit for bit (NaN and inf included): the adds of the selected rows in
    // ascending order, K4's sum, bit for bit
    const int64_t col = (int64_t)c * 64 + lane;
    // the selection masks in SGPRs (bit r: row r, resp. 64 + r, selected;
    // zero past n), so each row's select is a scalar test
    const uint64_t s0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(balw[0] >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)balw[0]);
    const uint64_t s1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(balw[1] >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)balw[1]);
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < (NB < 4 ? 16 * NB : 64); ++r) {
        const double v = cols[r * 64 + lane];
        acc += ((s0 >> r) & 1) ? v : 0.0;
    }
#pragma unroll
    for (int r = 0; r < 16 * NB - 64; ++r) {
        const double v = cols[(64 + r) * 64 + lane];
        acc += ((s1 >> r) & 1) ? v : 0.0;
    }
    if (col < a.d) a.mean[col] = acc / (double)m;
}

template <typename T, bool VEC, int NB>
__global__ __launch_bounds__(SMALL_NT) void k_small(SmallArgs a) {
    __shared__ int s_item;
    __shared__ unsigned s_old;
    __shared__ __attribute__((aligned(16))) char tile[16 * NB * SMALL_GR * 16];  // G: rows x KC columns
    __shared__ uint64_t kbuf[128];                                      // S / selection keys
    __shared__ __attribute__((aligned(16))) double sbuf[128];          // S: the sorted row
    __shared__ int rk[(SMALL_NT / 128 - 1) * 128];                      // partial ranks
    __shared__ double red[4];                                           // S waves
    __shared__ double bnd[2];
    __shared__ double dgl[128];
    __shared__ int srow[128];
    __shared__ uint64_t balw[2];
    __shared__ double wbuf[SMALL_NW][16 * 17];  // G: each wave's block on its way out
    static_assert(16 * NB * SMALL_GR * 16 >= 6 * 16 * NB * 8, "S items keep their sums in the tile");
    const int tid = threadIdx.x, wave = tid >> 6;
    const int NGI = SMALL_SPLIT * a.gn;  // G items: SPLIT per chunk of this launch
    const int total = NGI + (a.sm ? a.n + a.C : 0);
    unsigned *ctr = a.ctr;
    // the first S0 items (G items) go to workgroups by blockIdx, the rest in
    // queue order (one returning atomic each): 256 dequeues on one counter
    // take ~3 us, which delayed the last G item's start by that much
    const int S0 = NGI < (int)gridDim.x ? NGI : (int)gridDim.x;
    bool last_out = false;
    // debug trace: per workgroup {entry, exit} after the item records
    if (a.trace && tid == 0) a.trace[8 * total + 2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
    for (bool first = true;; first = false) {
        if (first && (int)blockIdx.x < S0) {
            if (tid == 0) s_item = (int)blockIdx.x;
        } else if (tid == 0) {
            s_item = S0 + (int)__hip_atomic_fetch_add(cline(ctr, C_HEAD), 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        const int it = s_item;
        // the item's view of the arguments, opaque to the optimizer: without
        // this, every predicate and constant the items derive from n, f, P, d
        // (row masks, chunk masks, the margin's gamma divisions) was hoisted
        // out of the item loop into a ~2,300-instruction prologue, spilled to
        // VGPR lanes and run cold from the instruction cache: 4.4 us before
        // the first item started
        SmallArgs b = a;
        asm volatile("" : "+s"(b.n), "+s"(b.f), "+s"(b.P), "+s"(b.C), "+s"(b.d), "+s"(b.ld));
        int ot = tid;  // the thread index, opaque likewise (per-thread LDS / row offsets)
        asm volatile("" : "+v"(ot));
        const int olane = ot & 63;
        __syncthreads();
        if (it >= total) {
            // every workgroup ends on exactly one failed dequeue; the last of
            // them (its add returned total - S0 + grid - 1) is the last one out
            last_out = it == total + (int)gridDim.x - 1;
            break;
        }
        long long t0 = 0, m0 = 0;
        if (a.trace && tid == 0) {
            t0 = (long long)__builtin_amdgcn_s_memrealtime();
            m0 = (long long)__builtin_amdgcn_s_memtime();
        }
        if (it < NGI) {
            small_gram<T, VEC, NB>(b, it, wave, olane, tile, &wbuf[wave][0]);
            // (a G-only launch: the kernel boundary is the hand-off)
            if (a.sm && wg_arrive(ctr, C_G, G_GRP, it, NGI, &s_old)) wg_raise(ctr, F_G);
        } else if (it < NGI + a.n) {
            if (NGI > 0) wg_wait_flag(ctr, F_G, a.spin_max);
            if (a.trace && tid == 0) a.trace[8 * it + 1] = (long long)__builtin_amdgcn_s_memrealtime();
            // the S item's chain sums and Gram row live in the (idle) G tile
            d2v *gv2 = reinterpret_cast<d2v *>(tile);
            double *gv = reinterpret_cast<double *>(tile) + 4 * 16 * NB;
            small_scores<NB>(b, it - NGI, ot, kbuf, sbuf, rk, gv, gv2, red,
                         a.trace ? a.trace + 8 * it : nullptr);
            if (wg_arrive(ctr, C_S, S_GRP, it - NGI, a.n, &s_old)) wg_raise(ctr, F_S);
        } else {
            // while the scores are computed: this item's 64 columns of every
            // row into LDS, so after the scores only LDS work is left
            double *cols = reinterpret_cast<double *>(tile);
            small_mean_stage<T, NB>(b, it - NGI - a.n, ot, cols);
            wg_wait_flag(ctr, F_S, a.spin_max);
            if (a.trace && tid == 0) a.trace[8 * it + 1] = (long long)__builtin_amdgcn_s_memrealtime();
            small_mean<NB>(b, it - NGI - a.n, ot, wave, olane, kbuf, srow, dgl, bnd, balw, rk, cols,
                       a.trace ? a.trace + 8 * it : nullptr);
        }
        if (a.trace && tid == 0) {
            unsigned hw;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            a.trace[8 * it] = t0;
            a.trace[8 * it + 2] = (long long)__builtin_amdgcn_s_memrealtime();
            a.trace[8 * it + 3] = (long long)hw | ((long long)blockIdx.x << 32);
            a.trace[8 * it + 4] = m0;
            a.trace[8 * it + 5] = (long long)__builtin_amdgcn_s_memtime();
        }
    }
    // the last workgroup out resets the queue for the next launch (stream
    // order: the next launch starts after this one has completed)
    if (last_out) {
        __shared__ unsigned s_err;
        if (tid == 0) s_err = ctr_load(cline(ctr, C_ERR));
        __syncthreads();
        if (s_err) {
            // a wait gave up: the outputs are invalid.  The margin says so
            // (read_margin: BK_EHIP, from bk_synchronize, the synchronous
            // entries and bk_selection_margin*), and so does the data path:
            // every selected index becomes -1
            if (tid == 0) {
                a.margin[0] = __builtin_nan("");
                a.margin[2] = MARGIN_HANDOFF_TIMEOUT;
            }
            if (a.sel && tid < a.n - a.f) a.sel[tid] = -1;
        }
        if (a.check_lines) {
            // debug (BK_SMALL_CHECK_LINES): the reset below clears word 0 of
            // each line only, because no other word is ever written; check
            // that invariant over every word of every line, clear any word
            // that breaks it and report the launch (MARGIN_QUEUE_DIRTY)
            __shared__ unsigned s_dirty;
            if (tid == 0) s_dirty = 0;
            __syncthreads();
            for (int w = tid; w < C_LINES * 32; w += SMALL_NT) {
                if ((w & 31) == 0) continue;
                if (ctr_load(ctr + w) != 0u) {
                    __hip_atomic_store(ctr + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s_dirty = 1;  // benign race: every writer stores 1
                }
            }
            __syncthreads();
            if (tid == 0 && s_dirty) a.margin[2] = MARGIN_QUEUE_DIRTY;
        }
        __syncthreads();
        // only word 0 of each line is ever written (checked under check_lines)
        if (tid < C_LINES) __hip_atomic_store(ctr + 32 * tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (a.trace && tid == 0) a.trace[8 * total + 2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
}

// k_tiny: the whole call in ONE workgroup for n <= 16, d <= 128 (config A,
// creditcard: 10 x 25; a real localTest verifier sees n <= 4).  Three
// hand-offs between CUs (~1 us each) were most of k_small's 15 us there; one
// workgroup needs none.  Same arithmetic as k_small for a one-chunk batch, so
// the same bits: the chunk staged alike, the 16 x 16 Gram block by the same
// MFMA sequence (small_gram_groups), made symmetric from its upper elements,
// each row's distances in numpy's order, a sort by counting, K2's summation
// shape (lane t adds rank 1 + t, the wave butterfly, then the four waves'
// sums in order -- here waves 1-3 hold +0.0), the (score, index) rank, and
// the mean of the selected rows in ascending order (K4's adds).
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void k_tiny(SmallArgs a) {
    __shared__ __attribute__((aligned(16))) char tile[16 * SMALL_GR * 16];  // 16 rows x 128 columns
    __shared__ double gm[16 * 17];          // the Gram block (symmetric)
    __shared__ uint64_t keys[4][16];        // each wave's row keys
    __shared__ double srt[4][16];           // each wave's sorted row
    __shared__ double scs[16];
    __shared__ uint64_t skey[16];
    __shared__ double bnd[2];
    __shared__ uint64_t balw;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int n = a.n, m = n - a.f;
    const int64_t k = n - a.f - 2 > 0 ? n - a.f - 2 : 0;
    {
        SmallStage<T, VEC, 1, 256> st;
        st.load(a, 0, tid);
        st.store(tile, 0, SMALL_GR, tid);
    }
    __syncthreads();
    if (wave == 0) {
        d4 acc[1] = {d4{0.0, 0.0, 0.0, 0.0}};
        small_gram_groups<1, 0, 0, 1, 4>(acc, tile, lane, 0, SMALL_KC / 8);
        const int rr = lane & 15, g = lane >> 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) gm[(g + 4 * r) * 17 + rr] = acc[0][r];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (g + 4 * r > rr) gm[(g + 4 * r) * 17 + rr] = gm[rr * 17 + g + 4 * r];
    }
    __syncthreads();
    // scores: wave w takes rows w, w + 4, ...
    for (int i = wave; i < n; i += 4) {
        const double di = gm[i * 17 + i];
        uint64_t key = ~0ULL;  // padding sorts last
        if (lane < n) key = dkey((di + gm[lane * 17 + lane]) - 2.0 * gm[i * 17 + lane]);
        if (lane < 16) keys[wave][lane] = key;
        __builtin_amdgcn_wave_barrier();
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint64_t o = keys[wave][j];
            cnt += (o < key) || (o == key && j < lane);
        }
        if (lane < 16) srt[wave][cnt] = dkey_inv(key);
        __builtin_amdgcn_wave_barrier();
        double acc = 0.0;
        if (1 + lane <= k) acc += srt[wave][1 + lane];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) {
            double sum = 0.0;  // the four waves' sums in order (waves 1-3: +0.0)
            sum += acc;
            sum += 0.0;
            sum += 0.0;
            sum += 0.0;
            const double sv = k > 0 ? sum : 0.0;
            scs[i] = sv;
            a.scores[i] = sv;
            a.diag[i] = di;
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    if (tid < 16) skey[tid] = tid < n ? dkey(scs[tid]) : ~0ULL;
    __syncthreads();
    if (wave == 0) {
        bool on = false;
        if (lane < n) {
            const uint64_t ki = skey[lane];
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint64_t o = skey[j];
                cnt += (o < ki) || (o == ki && j < lane);
            }
            on = cnt < m;
            if (cnt == m - 1) bnd[0] = scs[lane];
            if (cnt == m) bnd[1] = scs[lane];
        }
        const uint64_t bal = __ballot(on);
        if (on && a.sel) a.sel[__popcll(bal & ((1ull << lane) - 1))] = (int64_t)lane;
        if (lane == 0) balw = bal;
    }
    __syncthreads();
    if (tid == 0) {
        double M = 0.0;
        for (int j = 0; j < n; ++j) {
            const double v = gm[j * 17 + j];
            if (v == v && v < __builtin_inf() && v > M) M = v;
        }
        write_margin(a.margin, bnd[0], bnd[1], M, (double)a.d, k, 0x1p-53);
    }
    if (a.mean && tid < a.d) {
        // column tid, the 16 staged rows in ascending order, each row's value
        // or +0.0 by the selection mask (acc is never -0.0: k_small's M items)
        const uint64_t sb = balw;
        double acc = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const double v = reinterpret_cast<const d2v *>(tile + sg_off(r, tid >> 1))[0][tid & 1];
            acc += ((sb >> r) & 1) ? v : 0.0;
        }
        a.mean[tid] = acc / (double)m;
    }
}

template <typename T, bool VEC>
static void launch_small_t(const SmallArgs &a, int NBv, int grid, hipStream_t st) {
    switch (NBv) {
    case 1: hipLaunchKernelGGL((k_small<T, VEC, 1>), dim3(grid), dim3(SMALL_NT), 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_small<T, VEC, 2>), dim3(grid), dim3(SMALL_NT), 0, st, a); break;
    case 3: hipLaunchKernelGGL((k_small<T, VEC, 3>), dim3(grid), dim3(SMALL_NT), 0, st, a); break;
    case 4: hipLaunchKernelGGL((k_small<T, VEC, 4>), dim3(grid), dim3(SMALL_NT), 0, st, a); break;
    case 5: hipLaunchKernelGGL((k_small<T, VEC, 5>), dim3(grid), dim3(SMALL_NT), 0, st, a); break;
    case 6: hipLaunchKernelGGL((k_small<T, VEC, 6>), dim3(grid), dim3(SMALL_NT), 0, st, a); break;
    case 7: hipLaunchKernelGGL((k_small<T, VEC, 7>), dim3(grid), dim3(SMALL_NT), 0, st, a); break;
    default: hipLaunchKernelGGL((k_small<T, VEC, 8>), dim3(grid), dim3(SMALL_NT), 0, st, a); break;
    }
}

bool tiny_ok(int n, int64_t d) {
    static const bool on = [] {
        const char *e = getenv("BK_TINY");  // 0: k_small for every n <= 128 (A/B)
        return !(e && atoi(e) == 0);
    }();
    return on && n <= 16 && d <= SMALL_KC;
}

SmallPlan small_plan(int n, int64_t d, int num_cu) {
    SmallPlan p;
    p.nb16 = (n + 15) / 16;
    p.nblk = p.nb16 * (p.nb16 + 1) / 2;
    (void)num_cu;
    const int64_t kc = SMALL_KC;
    p.kc = (int)kc;
    p.P = (int)((d + kc - 1) / kc);
    p.ng = SMALL_SPLIT * p.P;
    p.Q = 0;   // no reduce items: every S item sums its own row of the partials
    p.nS = n;  // one S item per row
    p.C = (int)((d + 63) / 64);  // M items: 64 columns each
    return p;
}

hipError_t launch_small(const void *X, int dtype, int64_t ld, int n, int64_t d, int f,
                        const SmallPlan &p, double *part, double *U, double *scores, double *diag,
                        int64_t *sel, double *mean, double *margin, unsigned *ctr, int num_cu,
                        hipStream_t st, long long *trace, uint64_t spin_max, int check_lines,
                        double *scores_out, int g0, int gn, bool sm) {
    SmallArgs a;
    a.g0 = g0;
    a.gn = gn < 0 ? p.P : gn;
    a.sm = sm ? 1 : 0;
    a.scores_out = scores_out;
    a.trace = trace;
    a.spin_max = spin_max;
    a.check_lines = check_lines;
    a.X = X;
    a.ld = ld;
    a.d = d;
    a.n = n;
    a.f = f;
    a.kc = p.kc;
    a.P = p.P;
    a.Q = p.Q;
    a.nS = p.nS;
    a.C = mean ? p.C : 1;  // item 0 writes sel and the margin even without a mean
    a.nblk = p.nblk;
    a.T = (n + 63) / 64;
    a.part = part;
    a.U = U;
    a.scores = scores;
    a.diag = diag;
    a.mean = mean;
    a.margin = margin;
    a.sel = sel;
    a.ctr = ctr;
    const int total = SMALL_SPLIT * a.gn + (a.sm ? a.n + a.C : 0);
    const int grid = total < num_cu ? total : num_cu;
    const bool vec = (ld % 2) == 0 && ((uintptr_t)X % (dtype == 0 ? 16 : 8)) == 0;
    if (tiny_ok(n, d) && !trace && g0 == 0 && a.gn == p.P && sm) {  // one workgroup (k_tiny)
        if (scores_out) a.scores = scores_out;  // k_tiny never reads its scores back
        if (dtype == 0 && vec)
            hipLaunchKernelGGL((k_tiny<double, true>), dim3(1), dim3(256), 0, st, a);
        else if (dtype == 0)
            hipLaunchKernelGGL((k_tiny<double, false>), dim3(1), dim3(256), 0, st, a);
        else if (vec)
            hipLaunchKernelGGL((k_tiny<float, true>), dim3(1), dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL((k_tiny<float, false>), dim3(1), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    if (dtype == 0 && vec)
        launch_small_t<double, true>(a, p.nb16, grid, st);
    else if (dtype == 0)
        launch_small_t<double, false>(a, p.nb16, grid, st);
    else if (vec)
        launch_small_t<float, true>(a, p.nb16, grid, st);
    else
        launch_small_t<float, false>(a, p.nb16, grid, st);
    return hipGetLastError();
}

}  // namespace bk
