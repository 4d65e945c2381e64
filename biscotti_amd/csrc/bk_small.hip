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
//   G items  (P of them)  split-K Gram partial of d/P columns: every upper
//                          16x16 block of the (n <= 128) Gram, fp64 MFMA
//   R items  (4 per block) fixed-order sum of the P partials -> packed upper U
//   S items  (4 rows each) one wave per row: distances, register bitonic sort
//                          (k2_*), sum of ranks 1..k in K2's exact shape; the
//                          last S item to finish (arrival counter) ranks the
//                          scores, compacts the selection, writes the margin
//   M items  (256 columns) mean of the selected rows, ascending (K4's order)
//
// An item only waits (a relaxed poll, then an agent-scope acquire) for items
// dequeued BEFORE it, and a dequeued item's workgroup is running, so the queue
// always drains: no co-residency is assumed (MI355X_MICROARCH.md, "Workgroup
// dispatch").  Producers publish with every wave's vmcnt(0), a barrier, an
// agent release fence and a relaxed atomic add (the guide's "Valid forms").
// The last workgroup to exit resets the counters for the next launch.  A wait
// gives up after ~1 s and raises an error word instead of hanging the GPU.
// Results are deterministic: every sum has a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "bk_device.h"
#include "bk_internal.h"

namespace bk {

enum { C_HEAD = 0, C_G = 1, C_R = 2, C_S = 3, C_SEL = 4, C_EXIT = 5, C_ERR = 6 };

struct SmallArgs {
    const void *X;
    int64_t ld, d;
    int n, f, kc, P, Q, nS, C, nblk, T;
    double *part, *U, *scores, *diag, *mean, *margin;
    int64_t *sel;
    unsigned *ctr;
};

__device__ __forceinline__ unsigned ctr_load(const unsigned *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wait until *p >= target (lane 0 polls), then acquire for the whole workgroup
__device__ __forceinline__ void wg_wait(unsigned *p, unsigned target, unsigned *err) {
    if (threadIdx.x == 0) {
        uint64_t spins = 0;
        while (ctr_load(p) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1ull << 23)) {  // ~1 s: never hang the GPU on a broken hand-off
                __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// publish this workgroup's stores, then count; returns the counter's old value
__device__ __forceinline__ unsigned wg_signal(unsigned *p, unsigned *s_old) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *s_old = __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return *s_old;
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

// the 2 MFMAs of this wave's J-th block per 8-column group; block positions are
// compile-time, so the fragment array stays in registers
template <int NB, int W, int J, int NJ>
__device__ __forceinline__ void small_mma(d4 *acc, const d2v (&fr)[NB]) {
    if constexpr (J < NJ) {
        constexpr int b = W + 4 * J;
        constexpr int bi = blk_bi(b, NB), bj = blk_bj(b, NB);
        acc[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[bi].x, fr[bj].x, acc[J], 0, 0, 0);
        acc[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[bi].y, fr[bj].y, acc[J], 0, 0, 0);
        small_mma<NB, W, J + 1, NJ>(acc, fr);
    }
}

template <typename T>
__device__ __forceinline__ d2v sm_ld2(const T *p) {  // 2 consecutive elements as fp64
    if constexpr (sizeof(T) == 8) {
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
template <typename T, int NB, int W>
__device__ __forceinline__ void small_gram_wave(const SmallArgs &a, int s, int lane) {
    constexpr int NBLK = NB * (NB + 1) / 2;
    constexpr int NJ = (NBLK - W + 3) / 4;  // this wave's blocks
    const T *X = (const T *)a.X;
    const int rr = lane & 15, g = lane >> 4;
    const int64_t c0 = (int64_t)s * a.kc, c1 = c0 + a.kc < a.d ? c0 + a.kc : a.d;
    const T *rows[NB];
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        const int r = min(16 * rb + rr, a.n - 1);  // rows past n: duplicates, never read back
        rows[rb] = X + (int64_t)r * a.ld + c0 + 2 * g;
    }
    d4 acc[NJ > 0 ? NJ : 1];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = d4{0.0, 0.0, 0.0, 0.0};
    const int64_t len = c1 - c0, nfull = len >> 3;
    d2v fr[NB], nx[NB];
    if (nfull > 0) {
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) fr[rb] = sm_ld2<T>(rows[rb]);
    }
    for (int64_t t = 0; t < nfull; ++t) {
        const int64_t tn = t + 1 < nfull ? t + 1 : t;  // clamped prefetch keeps the loop simple
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) nx[rb] = sm_ld2<T>(rows[rb] + tn * 8);
        small_mma<NB, W, 0, NJ>(acc, fr);
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) fr[rb] = nx[rb];
    }
    if (len & 7) {  // ragged tail: guarded scalar loads
        const int64_t k0 = nfull * 8 + 2 * g;
        const bool v0 = k0 < len, v1 = k0 + 1 < len;
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            fr[rb].x = v0 ? (double)rows[rb][nfull * 8] : 0.0;
            fr[rb].y = v1 ? (double)rows[rb][nfull * 8 + 1] : 0.0;
        }
        small_mma<NB, W, 0, NJ>(acc, fr);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        double *out = a.part + ((int64_t)s * NBLK + W + 4 * j) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(g + 4 * r) * 16 + rr] = acc[j][r];
    }
}

template <typename T, int NB>
__device__ __forceinline__ void small_gram(const SmallArgs &a, int s, int wave, int lane) {
    switch (wave) {
    case 0: small_gram_wave<T, NB, 0>(a, s, lane); break;
    case 1: small_gram_wave<T, NB, 1>(a, s, lane); break;
    case 2: small_gram_wave<T, NB, 2>(a, s, lane); break;
    default: small_gram_wave<T, NB, 3>(a, s, lane); break;
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
    for (; s + 28 < a.P; s += 32) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(s + 4 * u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; s < a.P; s += 4) acc += p[(int64_t)s * stride];
    red[ch][el] = acc;
    __syncthreads();
    if (ch == 0) {
        const double t = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
        const int bi = blk_bi(b, NB), bj = blk_bj(b, NB);
        const int r = 16 * bi + (e >> 4), c = 16 * bj + (e & 15);
        a.U[upper_tile(a.T, r >> 6, c >> 6) + (r & 63) * 64 + (c & 63)] = t;
        if (q == 0 && el == 0) a.U[(int64_t)a.T * (a.T + 1) / 2 * 4096] = (double)a.d;
    }
}

// S item j: rows 4j + wave, one wave each: K2's distances, sort and sum shape
// (v1's 256-thread summation emulated: ranks 1 + t', t' = lane + 64 h)
__device__ __forceinline__ void small_scores(const SmallArgs &a, int j, int wave, int lane,
                                             double *kbuf) {
    const int i = 4 * j + wave;
    if (i >= a.n) return;  // wave-uniform; no barrier below
    const int n = a.n;
    const int64_t k = n - a.f - 2 > 0 ? n - a.f - 2 : 0;
    const double di = u_at(a.U, a.T, i, i);
    bool nan = false;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = lane + 64 * q;
        double x = __builtin_inf();
        if (e < n) {
            x = (di + u_at(a.U, a.T, e, e)) - 2.0 * u_at(a.U, a.T, i, e);
            x = x == 0.0 ? 0.0 : x;
            nan |= x != x;
        }
        kbuf[e] = x;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    double v[2] = {kbuf[2 * lane], kbuf[2 * lane + 1]};
    const bool any_nan = __ballot(nan) != 0;
    double sorted0, sorted1;  // this lane's two sorted keys, as values
    if (!any_nan) {
        for (int size = 2; size <= 128; size <<= 1) {  // the all-ascending bitonic of k2_sort
            if (size == 2) {
                k2_cas(v[0], v[1]);
            } else {
                k2_lane_dispatch<double, 2, 1>(v, (size - 1) >> 1, (lane & ((size >> 1) >> 1)) == 0);
                for (int st = size >> 2; st >= 2; st >>= 1)
                    k2_lane_dispatch<double, 2, 0>(v, st >> 1, (lane & (st >> 1)) == 0);
                k2_cas(v[0], v[1]);
            }
        }
        sorted0 = v[0];
        sorted1 = v[1];
    } else {  // a NaN in the row: order-preserving u64 keys, NaN last
        uint64_t u[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) u[q] = 2 * lane + q < n ? dkey(v[q]) : ~0ULL;
        for (int size = 2; size <= 128; size <<= 1) {
            if (size == 2) {
                k2_cas(u[0], u[1]);
            } else {
                k2_lane_dispatch<uint64_t, 2, 1>(u, (size - 1) >> 1, (lane & ((size >> 1) >> 1)) == 0);
                for (int st = size >> 2; st >= 2; st >>= 1)
                    k2_lane_dispatch<uint64_t, 2, 0>(u, st >> 1, (lane & (st >> 1)) == 0);
                k2_cas(u[0], u[1]);
            }
        }
        sorted0 = dkey_inv(u[0]);
        sorted1 = dkey_inv(u[1]);
    }
    __builtin_amdgcn_wave_barrier();
    kbuf[2 * lane] = sorted0;
    kbuf[2 * lane + 1] = sorted1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    double sum = 0.0;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int r = 1 + lane + 64 * h;
        double acc = 0.0;
        if (r <= k) acc += kbuf[r];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        sum += acc;  // (0 + red_0) + red_1 + ... : K2's order over the 4 virtual waves
    }
    if (lane == 0) {
        a.scores[i] = k > 0 ? sum : 0.0;
        a.diag[i] = di;
    }
}

// the last S item: rank, compact, margin (n <= 128, one workgroup)
__device__ __forceinline__ void small_select(const SmallArgs &a, int wave, int lane, int *msk,
                                             double *bnd) {
    const int n = a.n, m = n - a.f;
    for (int i = wave; i < n; i += 4) {
        const double si = a.scores[i];
        const uint64_t ki = dkey(si);
        int cnt = 0;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = lane + 64 * q;
            bool before = false;
            if (j < n) {
                const uint64_t kj = dkey(a.scores[j]);
                before = (kj < ki) || (kj == ki && j < i);
            }
            cnt += __popcll(__ballot(before));
        }
        if (lane == 0) {
            msk[i] = cnt < m ? 1 : 0;
            if (cnt == m - 1) bnd[0] = si;
            if (cnt == m) bnd[1] = si;
        }
    }
    __syncthreads();
    if (wave == 0) {
        int base = 0;
        double M = 0.0;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = lane + 64 * q;
            const bool on = j < n && msk[j];
            const uint64_t bal = __ballot(on);
            const int pos = base + __popcll(bal & ((1ull << lane) - 1));
            if (on) a.sel[pos] = j;
            base += __popcll(bal);
            if (j < n) {
                const double v = a.diag[j];
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
}

// M item c: mean of columns [256 c, 256 c + 256): each thread one column, the
// m selected rows in ascending order (K4's order: the same bits)
template <typename T>
__device__ __forceinline__ void small_mean(const SmallArgs &a, int c, int tid, int64_t *soff) {
    const int m = a.n - a.f;
    for (int r = tid; r < m; r += 256) soff[r] = a.sel[r] * a.ld;
    __syncthreads();
    const int64_t col = (int64_t)c * 256 + tid;
    if (col < a.d) {
        const T *X = (const T *)a.X;
        double acc = 0.0;
        int r = 0;
        for (; r + 16 <= m; r += 16) {
            double v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = (double)X[soff[r + u] + col];
#pragma unroll
            for (int u = 0; u < 16; ++u) acc += v[u];
        }
        for (; r < m; ++r) acc += (double)X[soff[r] + col];
        a.mean[col] = acc / (double)m;
    }
}

template <typename T, int NB>
__global__ __launch_bounds__(256) void k_small(SmallArgs a) {
    __shared__ int s_item;
    __shared__ unsigned s_old;
    __shared__ __attribute__((aligned(16))) double kbuf[4][128];  // S: one row per wave
    __shared__ double red[4][64];                                 // R: the 4 chains
    __shared__ int msk[128];
    __shared__ double bnd[2];
    __shared__ int64_t soff[128];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int total = a.P + a.Q + a.nS + a.C;
    unsigned *ctr = a.ctr;
    for (;;) {
        if (tid == 0)
            s_item = (int)__hip_atomic_fetch_add(&ctr[C_HEAD], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int it = s_item;
        __syncthreads();
        if (it >= total) break;
        if (it < a.P) {
            small_gram<T, NB>(a, it, wave, lane);
            wg_signal(&ctr[C_G], &s_old);
        } else if (it < a.P + a.Q) {
            wg_wait(&ctr[C_G], (unsigned)a.P, &ctr[C_ERR]);
            small_reduce(a, it - a.P, tid, NB, red);
            wg_signal(&ctr[C_R], &s_old);
        } else if (it < a.P + a.Q + a.nS) {
            wg_wait(&ctr[C_R], (unsigned)a.Q, &ctr[C_ERR]);
            small_scores(a, it - a.P - a.Q, wave, lane, kbuf[wave]);
            if (wg_signal(&ctr[C_S], &s_old) == (unsigned)a.nS - 1) {
                // the last S item: every score and diagonal is published
                if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                small_select(a, wave, lane, msk, bnd);
                wg_signal(&ctr[C_SEL], &s_old);
            }
        } else {
            wg_wait(&ctr[C_SEL], 1u, &ctr[C_ERR]);
            small_mean<T>(a, it - a.P - a.Q - a.nS, tid, soff);
        }
    }
    // the last workgroup out resets the queue for the next launch (stream
    // order: the next launch starts after this one has completed)
    if (tid == 0) {
        const unsigned e = __hip_atomic_fetch_add(&ctr[C_EXIT], 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        if (e == gridDim.x - 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (ctr_load(&ctr[C_ERR])) {  // a wait gave up: the outputs are invalid
                a.margin[0] = __builtin_nan("");
                a.margin[2] = 2.0;  // read_margin reports BK_EHIP
            }
            for (int c = C_HEAD; c <= C_ERR; ++c)
                __hip_atomic_store(&ctr[c], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <typename T>
static void launch_small_t(const SmallArgs &a, int NBv, int grid, hipStream_t st) {
    switch (NBv) {
    case 1: hipLaunchKernelGGL((k_small<T, 1>), dim3(grid), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_small<T, 2>), dim3(grid), dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((k_small<T, 3>), dim3(grid), dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((k_small<T, 4>), dim3(grid), dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL((k_small<T, 5>), dim3(grid), dim3(256), 0, st, a); break;
    case 6: hipLaunchKernelGGL((k_small<T, 6>), dim3(grid), dim3(256), 0, st, a); break;
    case 7: hipLaunchKernelGGL((k_small<T, 7>), dim3(grid), dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((k_small<T, 8>), dim3(grid), dim3(256), 0, st, a); break;
    }
}

SmallPlan small_plan(int n, int64_t d, int num_cu) {
    SmallPlan p;
    p.nb16 = (n + 15) / 16;
    p.nblk = p.nb16 * (p.nb16 + 1) / 2;
    int64_t kc = 64;
    if (const char *e = getenv("BK_SMALL_KC")) kc = atoll(e) > 0 ? atoll(e) : kc;
    kc = (kc + 7) / 8 * 8;
    // at most 2 partial rounds per CU: the R items read P partials each
    const int64_t pmax = 2 * (int64_t)num_cu;
    if ((d + kc - 1) / kc > pmax) kc = ((d + pmax - 1) / pmax + 7) / 8 * 8;
    p.kc = (int)kc;
    p.P = (int)((d + kc - 1) / kc);
    p.Q = 4 * p.nblk;
    p.nS = (n + 3) / 4;
    p.C = (int)((d + 255) / 256);
    return p;
}

hipError_t launch_small(const void *X, int dtype, int64_t ld, int n, int64_t d, int f,
                        const SmallPlan &p, double *part, double *U, double *scores, double *diag,
                        int64_t *sel, double *mean, double *margin, unsigned *ctr, int num_cu,
                        hipStream_t st) {
    SmallArgs a;
    a.X = X;
    a.ld = ld;
    a.d = d;
    a.n = n;
    a.f = f;
    a.kc = p.kc;
    a.P = p.P;
    a.Q = p.Q;
    a.nS = p.nS;
    a.C = mean ? p.C : 0;
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
    const int total = a.P + a.Q + a.nS + a.C;
    const int grid = total < num_cu ? total : num_cu;
    if (dtype == 0)
        launch_small_t<double>(a, p.nb16, grid, st);
    else
        launch_small_t<float>(a, p.nb16, grid, st);
    return hipGetLastError();
}

}  // namespace bk
