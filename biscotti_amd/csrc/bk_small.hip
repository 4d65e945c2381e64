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
//   R items  (4 per block) fixed-order sum of the P partials -> packed upper U
//   S items  (one per row) distances, sort by counting, sum of ranks 1..k in
//                          K2's exact shape
//   M items  (128 columns) rank the n scores (each item itself: no serial
//                          selection step), compact the selection, mean of
//                          the selected rows ascending (K4's order); item 0
//                          writes sel and the margin
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
// arrival counters of the G, R and S phases, a spare line, the error word;
// then the "phase done" flags F_G, F_R, F_S, each replicated once per XCD (a
// waiting workgroup polls its own XCD's copy: 1/8 of the pollers on any
// line); then the arrival counters of groups of 32 items (G_GRP: up to 1024 G
// items, R_GRP: 144 R items, S_GRP: 128 S items).  Same-address atomics
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
constexpr int SMALL_SPLIT = 4;          // G items per chunk (each: a quarter of the blocks)

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
    double *part, *U, *scores, *diag, *mean, *margin;
    int64_t *sel;
    unsigned *ctr;
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
__device__ __forceinline__ void wg_wait_flag(unsigned *ctr, int flag) {
    if (threadIdx.x == 0) {
        const unsigned *p = cline(ctr, flag + xcc_id());
        uint64_t spins = 0;
        while (ctr_load(p) == 0u) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1ull << 24)) {  // ~1 s: never hang the GPU on a broken hand-off
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
template <int NB, int W, int S, int J, int NJ>
__device__ __forceinline__ void small_mma_s(d4 *acc, const d2v (&fr)[NB]) {
    if constexpr (J < NJ) {
        constexpr int b = W + 4 * J;
        constexpr int bi = blk_bi(b, NB), bj = blk_bj(b, NB);
        acc[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[bi][S], fr[bj][S], acc[J], 0, 0, 0);
        small_mma_s<NB, W, S, J + 1, NJ>(acc, fr);
    }
}
// both sub-steps, blocks interleaved: consecutive MFMAs never share an accumulator
template <int NB, int W, int J, int NJ>
__device__ __forceinline__ void small_mma(d4 *acc, const d2v (&fr)[NB]) {
    small_mma_s<NB, W, 0, J, NJ>(acc, fr);
    small_mma_s<NB, W, 1, J, NJ>(acc, fr);
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

template <typename T, bool VEC, int NB>
struct SmallStage {
    static constexpr int ROWS = 16 * NB;
    static constexpr int PER = (ROWS * SMALL_GR + 255) / 256;  // 16-B granules per thread
    d2v v[PER];
    // every load of the item in flight at once (coalesced rows)
    __device__ __forceinline__ void load(const SmallArgs &a, int s) {
        const T *X = (const T *)a.X;
        const int64_t c0 = (int64_t)s * SMALL_KC;
        const int len = (int)(c0 + SMALL_KC < a.d ? SMALL_KC : a.d - c0);
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int gidx = threadIdx.x + 256 * q;
            const int row = gidx / SMALL_GR, gr = gidx % SMALL_GR, col = 2 * gr;
            d2v x = {0.0, 0.0};
            if (row < ROWS) {
                const T *p = X + (int64_t)min(row, a.n - 1) * a.ld + c0 + col;
                if (VEC && col + 1 < len) {
                    x = sm_ld2<T, true>(p);
                } else {
                    x.x = col < len ? (double)p[0] : 0.0;
                    x.y = col + 1 < len ? (double)p[1] : 0.0;
                }
            }
            v[q] = x;
        }
    }
    // granules [g0, g1) of every row into LDS
    __device__ __forceinline__ void store(char *tile, int g0, int g1) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int gidx = threadIdx.x + 256 * q;
            const int row = gidx / SMALL_GR, gr = gidx % SMALL_GR;
            if (row < ROWS && gr >= g0 && gr < g1) *reinterpret_cast<d2v *>(tile + sg_off(row, gr)) = v[q];
        }
    }
};

// the MFMAs of 8-column groups [t0, t1) of the staged tile, blocks J0 .. J1-1
// of this wave's list
template <int NB, int W, int J0, int J1>
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
            small_mma<NB, W, J0, J1>(acc, fr);
        }
    }
}

// G item (chunk c, part PART): columns [KC c, KC c + KC) staged once, then
// wave W runs part PART of its blocks b = W + 4 j (the j range cut in SPLIT
// pieces), so the Gram's MFMAs spread over SPLIT times as many CUs while a
// chunk's partial (one per KC columns: ~NBLK * 2 KiB written sc1, the same
// bytes whatever KC is) is written once per KC columns; the partials written
// sc1.  (Staging half the columns and computing it while the other half
// landed was 1.3 us slower per item: one more barrier.)
template <typename T, bool VEC, int NB, int W, int PART>
__device__ __forceinline__ void small_gram_wave(const SmallArgs &a, int c, long long *tr, int lane,
                                                char *tile, SmallStage<T, VEC, NB> &st) {
    constexpr int NBLK = NB * (NB + 1) / 2;
    constexpr int NJ = (NBLK - W + 3) / 4;  // this wave's blocks
    constexpr int J0 = PART * NJ / SMALL_SPLIT, J1 = (PART + 1) * NJ / SMALL_SPLIT;
    constexpr int NG = SMALL_KC / 8;
    const int rr = lane & 15, g = lane >> 4;
    d4 acc[NJ > 0 ? NJ : 1];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = d4{0.0, 0.0, 0.0, 0.0};
    st.store(tile, 0, SMALL_GR);
    __syncthreads();
    stamp(tr, 0);
    small_gram_groups<NB, W, J0, J1>(acc, tile, lane, 0, NG);
    if (W == 0) {  // wave 0's MFMAs done (debug trace only)
        if (tr && J1 > J0) asm volatile("s_nop 0" ::"v"(acc[J0][0]));
        stamp(tr, 1);
    }
#pragma unroll
    for (int j = J0; j < J1; ++j) {
        double *out = a.part + ((int64_t)c * NBLK + W + 4 * j) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) st1(out + (g + 4 * r) * 16 + rr, (double)acc[j][r]);
    }
}

template <typename T, bool VEC, int NB, int W>
__device__ __forceinline__ void small_gram_w(const SmallArgs &a, int c, int h, long long *tr,
                                             int lane, char *tile, SmallStage<T, VEC, NB> &st) {
    static_assert(SMALL_SPLIT == 4, "parts");
    switch (h) {
    case 0: small_gram_wave<T, VEC, NB, W, 0>(a, c, tr, lane, tile, st); break;
    case 1: small_gram_wave<T, VEC, NB, W, 1>(a, c, tr, lane, tile, st); break;
    case 2: small_gram_wave<T, VEC, NB, W, 2>(a, c, tr, lane, tile, st); break;
    default: small_gram_wave<T, VEC, NB, W, 3>(a, c, tr, lane, tile, st); break;
    }
}

template <typename T, bool VEC, int NB>
__device__ __forceinline__ void small_gram(const SmallArgs &a, int it, int wave, int lane,
                                           char *tile) {
    int c, h;
    g_item(it, a.P, c, h);
    long long *tr = a.trace ? a.trace + 8 * (int64_t)it : nullptr;
    SmallStage<T, VEC, NB> st;
    st.load(a, c);
    switch (wave) {
    case 0: small_gram_w<T, VEC, NB, 0>(a, c, h, tr, lane, tile, st); break;
    case 1: small_gram_w<T, VEC, NB, 1>(a, c, h, tr, lane, tile, st); break;
    case 2: small_gram_w<T, VEC, NB, 2>(a, c, h, tr, lane, tile, st); break;
    default: small_gram_w<T, VEC, NB, 3>(a, c, h, tr, lane, tile, st); break;
    }
}

// R item q: 64 elements (quarter q & 3) of block q >> 2, summed over the P
// partials in a fixed order (4 interleaved chains, then the chains in order)
__device__ __forceinline__ void small_reduce(const SmallArgs &a, int q, int tid, int NB,
                                             double (*red)[64]) {
    const int b = q >> 2, h = q & 3, el = tid & 63, ch = tid >> 6;
    const int e = 64 * h + el;
    const double *p = a.part + (int64_t)b * 256 + e;
    const int64_t stride = (int64_t)a.nblk * 256;
    double acc = 0.0;
    int s = ch;
    for (; s < a.P; s += 4 * 32) {  // 32 loads in flight per thread (P <= 512: 4 rounds at most)
        double v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) v[u] = s + 4 * u < a.P ? ld1(p + (int64_t)(s + 4 * u) * stride) : 0.0;
#pragma unroll
        for (int u = 0; u < 32; ++u)
            if (s + 4 * u < a.P) acc += v[u];
    }
    red[ch][el] = acc;
    __syncthreads();
    if (ch == 0) {
        const double t = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
        const int bi = blk_bi(b, NB), bj = blk_bj(b, NB);
        const int r = 16 * bi + (e >> 4), c = 16 * bj + (e & 15);
        st1(a.U + upper_tile(a.T, r >> 6, c >> 6) + (r & 63) * 64 + (c & 63), t);
        if (q == 0 && el == 0) st1(a.U + (int64_t)a.T * (a.T + 1) / 2 * 4096, (double)a.d);
    }
}

// S item i: row i with the whole workgroup.  Distances, then a sort by
// counting (thread t ranks key t & 127 against half of the row, t >> 7; key e
// goes to position #{keys before it in the (value, index) total order}), then
// K2's summation with its own 256 threads: thread t sums rank 1 + t, the wave
// butterfly, the 4 waves in order -- the same sorted array and the same shape,
// so the score is K2's bitwise (for the same U).
__device__ __forceinline__ void small_scores(const SmallArgs &a, int i, int tid, uint64_t *kbuf,
                                             double *sbuf, int *rk, double *red, long long *tr) {
    const int n = a.n, lane = tid & 63, wave = tid >> 6;
    const int64_t k = n - a.f - 2 > 0 ? n - a.f - 2 : 0;
    const int e = tid & 127, h = tid >> 7;
    const double di = u_at1(a.U, a.T, i, i);
    if (h == 0) {
        uint64_t key = ~0ULL;  // padding sorts last
        if (e < n) key = dkey((di + u_at1(a.U, a.T, e, e)) - 2.0 * u_at1(a.U, a.T, i, e));
        kbuf[e] = key;
    }
    __syncthreads();
    stamp(tr, 0);
    const uint64_t key = kbuf[e];
    int cnt = 0;
#pragma unroll
    for (int j0 = 0; j0 < 64; j0 += 8) {
        uint64_t o[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = kbuf[64 * h + j0 + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = 64 * h + j0 + u;
            cnt += (o[u] < key) || (o[u] == key && j < e);
        }
    }
    if (h == 1) rk[e] = cnt;
    __syncthreads();
    if (h == 0) sbuf[cnt + rk[e]] = dkey_inv(key);
    __syncthreads();
    stamp(tr, 1);
    double acc = 0.0;
    if (1 + tid <= k && 1 + tid < 128) acc += sbuf[1 + tid];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) red[wave] = acc;
    __syncthreads();
    if (tid == 0) {
        double sum = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w) sum += red[w];
        st1(a.scores + i, k > 0 ? sum : 0.0);
        st1(a.diag + i, di);
    }
}

// M item c: every M item ranks the n published scores itself (n <= 128: one
// LDS pass, no separate selection hand-off), compacts the selection with
// ballots, and sums columns [128 c, 128 c + 128) of the m selected rows in
// ascending order (K4's order: the same bits), every load in flight at once.
// Item 0 also writes sel and the margin.
template <typename T>
__device__ __forceinline__ void small_mean(const SmallArgs &a, int c, int wave, int lane,
                                           uint64_t *keys, int64_t *soff, double *dg, double *bnd,
                                           uint64_t *balw, int *rkm, char *tile, long long *tr) {
    const int n = a.n, m = n - a.f, tid = threadIdx.x;
    double si = 0.0;
    if (tid < n) {
        si = ld1(a.scores + tid);
        keys[tid] = dkey(si);
    } else if (c == 0 && tid >= 128 && tid - 128 < n) {
        dg[tid - 128] = ld1(a.diag + tid - 128);
    }
    __syncthreads();
    stamp(tr, 0);
    // rank of row e in the (score, index) total order: threads e and 128 + e
    // count over the two halves of the keys
    const int e = tid & 127, h = tid >> 7;
    int cnt = 0;
    uint64_t ki = 0;
    if (e < n) {
        ki = keys[e];
        const int j1 = n < 64 * h + 64 ? n : 64 * h + 64;
        int j = 64 * h;
        for (; j + 8 <= j1; j += 8) {
            uint64_t o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) o[u] = keys[j + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) cnt += (o[u] < ki) || (o[u] == ki && j + u < e);
        }
        for (; j < j1; ++j) {
            const uint64_t o = keys[j];
            cnt += (o < ki) || (o == ki && j < e);
        }
    }
    if (h == 1 && e < n) rkm[e] = cnt;
    __syncthreads();
    bool on = false;
    if (h == 0 && e < n) {
        cnt += rkm[e];
        on = cnt < m;
        if (c == 0 && cnt == m - 1) bnd[0] = si;
        if (c == 0 && cnt == m) bnd[1] = si;
    }
    // compaction: rows 0..63 in wave 0, 64..127 in wave 1
    const uint64_t bal = __ballot(on);
    if (wave < 2 && lane == 0) balw[wave] = bal;
    __syncthreads();
    if (on) {
        const int pos = (wave ? __popcll(balw[0]) : 0) + __popcll(bal & ((1ull << lane) - 1));
        soff[pos] = (int64_t)tid * a.ld;
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
    if (!a.mean) return;
    // the selected rows' offsets in registers (lane u: selected row u, or
    // 64 + u in waves 2-3; lanes past m repeat row m - 1, so every load is
    // valid), read with v_readlane per load instead of a broadcast LDS read +
    // wait per load.  v_readlane ignores EXEC, so no lane may skip the offset
    // loads: every lane runs the loads (columns past d clamped to the last one)
    // and only the store is conditional.  mm (= m) is re-derived from LDS so
    // the per-row tests stay inside the item (hoisted out of the item loop,
    // 64 loop-invariant masks were spilled and cost ~4 us per item).
    // Waves 0-1 load rows 0..63 of the item's 128 columns, waves 2-3 rows
    // 64..m-1 at the same time into LDS (the G tile: (m - 64) KiB <= 8 NB KiB);
    // waves 0-1 then add them in order: K4's ascending sum, bit for bit
    const int mm = __popcll(balw[0]) + __popcll(balw[1]);
    const int cl = e;  // (e = tid & 127, h = tid >> 7 as in the rank)
    const int64_t col = (int64_t)c * 128 + cl;
    const T *X = (const T *)a.X + (col < a.d ? col : a.d - 1);
    double *spill = reinterpret_cast<double *>(tile);  // [row - 64][128]
    const int64_t o = soff[64 * h + lane < mm ? 64 * h + lane : mm - 1];
    double acc = 0.0;
    if (h == 0) {
        double v[64];
#pragma unroll
        for (int u = 0; u < 64; ++u) v[u] = (double)X[__builtin_amdgcn_readlane((long long)o, u)];
#pragma unroll
        for (int u = 0; u < 64; ++u) acc = u < mm ? acc + v[u] : acc;
    } else if (mm > 64) {
        double v[64];
#pragma unroll
        for (int u = 0; u < 64; ++u) v[u] = (double)X[__builtin_amdgcn_readlane((long long)o, u)];
#pragma unroll
        for (int u = 0; u < 64; ++u)
            if (64 + u < mm) spill[u * 128 + cl] = v[u];
    }
    __syncthreads();
    if (h == 0) {
        for (int u = 64; u < mm; ++u) acc += spill[(u - 64) * 128 + cl];
        if (col < a.d) a.mean[col] = acc / (double)m;
    }
}

template <typename T>
__device__ __forceinline__ void small_prefetch(const SmallArgs &a, int c, int tid) {
    const int64_t col = (int64_t)c * 128 + (tid & 127);
    if (!a.mean || col >= a.d) return;
    const T *X = (const T *)a.X;
    T acc = 0;
    for (int r = tid >> 7; r < a.n; r += 32) {
        T v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = r + 2 * u < a.n ? X[(int64_t)(r + 2 * u) * a.ld + col] : (T)0;
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u];
    }
    asm volatile("" ::"v"(acc));  // keep the loads
}

template <typename T, bool VEC, int NB>
__global__ __launch_bounds__(256) void k_small(SmallArgs a) {
    __shared__ int s_item;
    __shared__ unsigned s_old;
    __shared__ __attribute__((aligned(16))) char tile[16 * NB * SMALL_GR * 16];  // G: rows x KC columns
    __shared__ uint64_t kbuf[128];                                      // S / selection keys
    __shared__ __attribute__((aligned(16))) double sbuf[128];          // S: the sorted row
    __shared__ int rk[128];
    __shared__ double red[4][64];                                       // R chains, S waves
    __shared__ double bnd[2];
    __shared__ double dgl[128];
    __shared__ int64_t soff[128];
    __shared__ uint64_t balw[2];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int NGI = SMALL_SPLIT * a.P;  // G items: SPLIT per chunk
    const int total = NGI + a.Q + a.n + a.C;
    unsigned *ctr = a.ctr;
    // the first S0 items (G items) go to workgroups by blockIdx, the rest in
    // queue order (one returning atomic each): 256 dequeues on one counter
    // take ~3 us, which delayed the last G item's start by that much
    const int S0 = NGI < (int)gridDim.x ? NGI : (int)gridDim.x;
    bool last_out = false;
    for (bool first = true;; first = false) {
        if (first && (int)blockIdx.x < S0) {
            if (tid == 0) s_item = (int)blockIdx.x;
        } else if (tid == 0) {
            s_item = S0 + (int)__hip_atomic_fetch_add(cline(ctr, C_HEAD), 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        const int it = s_item;
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
            small_gram<T, VEC, NB>(a, it, wave, lane, tile);
            if (wg_arrive(ctr, C_G, G_GRP, it, NGI, &s_old)) wg_raise(ctr, F_G);
        } else if (it < NGI + a.Q) {
            wg_wait_flag(ctr, F_G);
            if (a.trace && tid == 0) a.trace[8 * it + 1] = (long long)__builtin_amdgcn_s_memrealtime();
            small_reduce(a, it - NGI, tid, NB, red);
            if (wg_arrive(ctr, C_R, R_GRP, it - NGI, a.Q, &s_old)) wg_raise(ctr, F_R);
        } else if (it < NGI + a.Q + a.n) {
            wg_wait_flag(ctr, F_R);
            if (a.trace && tid == 0) a.trace[8 * it + 1] = (long long)__builtin_amdgcn_s_memrealtime();
            small_scores(a, it - NGI - a.Q, tid, kbuf, sbuf, rk, &red[0][0],
                         a.trace ? a.trace + 8 * it : nullptr);
            if (wg_arrive(ctr, C_S, S_GRP, it - NGI - a.Q, a.n, &s_old)) wg_raise(ctr, F_S);
        } else {
            // while the scores are computed: pull this item's columns of
            // every row toward this XCD's L2, so the mean's loads hit it
            small_prefetch<T>(a, it - NGI - a.Q - a.n, tid);
            wg_wait_flag(ctr, F_S);
            if (a.trace && tid == 0) a.trace[8 * it + 1] = (long long)__builtin_amdgcn_s_memrealtime();
            small_mean<T>(a, it - NGI - a.Q - a.n, wave, lane, kbuf, soff, dgl, bnd, balw, rk, tile,
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
    // order: the next launch starts after this one has completed) -- every
    // word of every line
    if (last_out) {
        if (tid == 0 && ctr_load(cline(ctr, C_ERR))) {  // a wait gave up: outputs invalid
            a.margin[0] = __builtin_nan("");
            a.margin[2] = 2.0;  // read_margin reports BK_EHIP
        }
        __syncthreads();
        for (int w = tid; w < C_LINES * 32; w += 256)
            __hip_atomic_store(ctr + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <typename T, bool VEC>
static void launch_small_t(const SmallArgs &a, int NBv, int grid, hipStream_t st) {
    switch (NBv) {
    case 1: hipLaunchKernelGGL((k_small<T, VEC, 1>), dim3(grid), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_small<T, VEC, 2>), dim3(grid), dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((k_small<T, VEC, 3>), dim3(grid), dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((k_small<T, VEC, 4>), dim3(grid), dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL((k_small<T, VEC, 5>), dim3(grid), dim3(256), 0, st, a); break;
    case 6: hipLaunchKernelGGL((k_small<T, VEC, 6>), dim3(grid), dim3(256), 0, st, a); break;
    case 7: hipLaunchKernelGGL((k_small<T, VEC, 7>), dim3(grid), dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((k_small<T, VEC, 8>), dim3(grid), dim3(256), 0, st, a); break;
    }
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
    p.Q = 4 * p.nblk;
    p.nS = n;  // one S item per row
    p.C = (int)((d + 127) / 128);
    return p;
}

hipError_t launch_small(const void *X, int dtype, int64_t ld, int n, int64_t d, int f,
                        const SmallPlan &p, double *part, double *U, double *scores, double *diag,
                        int64_t *sel, double *mean, double *margin, unsigned *ctr, int num_cu,
                        hipStream_t st, long long *trace) {
    SmallArgs a;
    a.trace = trace;
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
    const int total = SMALL_SPLIT * a.P + a.Q + a.n + a.C;
    const int grid = total < num_cu ? total : num_cu;
    const bool vec = (ld % 2) == 0 && ((uintptr_t)X % (dtype == 0 ? 16 : 8)) == 0;
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
