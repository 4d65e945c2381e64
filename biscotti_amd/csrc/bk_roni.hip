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
//   K7  k_roni_mm_prep<false> + k_roni_sign   the logistic verifier as one
//                      fp64-MFMA GEMM (samples x models) with np.sign and the
//                      mismatch count fused into its epilogue
//   K7b k_roni_score   score[i] = cnt[i+1]/nv - cnt[0]/nv in fp64
//   K8  the torch-path (softmax) verifier: k_roni_mm_prep<true> +
//       k_roni_logits over a whole sample set, or k_roni_batch over the last
//       mini-batches the reference actually scores (below)
//
// Built with -ffp-contract=off: ww + delta rounds exactly like numpy; every dot
// is a plain fp64 FMA chain over k ascending (the MFMA chains round alike,
// tools/probe_mfma_order.hip).  BLAS order is library-specific: only the sign
// (K7) or the argmax (K8) matters, and they differ from the reference's only
// within rounding (K8 counts those samples: "near ties").
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "bk_internal.h"

namespace bk {

__global__ void k_roni_score(const unsigned int *__restrict__ cnt, int64_t n, int64_t nv,
                             double *__restrict__ scores) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double dn = (double)nv;
    const double g_err = (double)cnt[0] / dn;
    const double new_err = (double)cnt[i + 1] / dn;
    scores[i] = new_err - g_err;
}

__global__ void k_roni_mc_score(const unsigned int *__restrict__ good, int64_t n, int64_t nv,
                                double *__restrict__ scores) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double dn = (double)nv;
    const double orig = 1.0 - (double)good[0] / dn;  // 1 - accuracy_score
    const double after = 1.0 - (double)good[i + 1] / dn;
    scores[i] = after - orig;
}

// ---------------------------------------------------------------------------
// K8 on the matrix pipe (r3b).  The n + 1 models' logits are one GEMM,
// sum_k x[s][k] W_j[c][k] for M = nv samples, N = (n + 1) C model-class
// columns, K = d_in.  v_mfma_f64_16x16x4_f64 rounds like four fp64 FMAs in k
// order (tools/probe_mfma_order.hip), so a chain of them over k
// ascending from +0.0 is the same fp64 sum, bit for bit, as K8's per-lane FMA
// chain -- and as the oracle's.
//
// Columns: a 128-column tile holds P = 128 / C whole models (tile y: models
// P y .. P y + P - 1, column (j - P y) C + c), the rest zero padding (at most
// C - 1 columns: 8 of 128 for mnist's 10 classes), so the argmax never crosses
// a tile.  K7 uses the same layout with C = 1.
//
//   K8a' k_roni_mm_prep   Wt[k][col] = fp32(ww + delta_j) widened (K7: the
//                         fp64 sum), rows padded to a multiple of 32; bt[col]
//                         the biases.  32 k x 64 columns per workgroup through
//                         LDS: reads run along k (the flat weights' order),
//                         writes along the columns
//   K8b' k_roni_logits    the logits GEMM with the argmax and the count fused
//                         into its epilogue (below)
// Bound: fp64 MFMA (nv x (n+1) C x d_in MACs).
constexpr int RMM_NT = 128;  // columns per tile (= RG_NT below)
typedef double d4 __attribute__((ext_vector_type(4)));

static inline int64_t rmm_ldl(int64_t n, int C) {
    const int64_t P = RMM_NT / C;
    return (n + 1 + P - 1) / P * RMM_NT;
}
static inline int64_t rmm_rows(int64_t din) { return (din + 31) / 32 * 32; }  // whole K7 chunks

// softmax (K8): fp32(ww + delta_j) widened, plus the biases; logistic (K7):
// ww + delta_j in fp64 (numpy's add), no bias.  Grid (ldl / 64, rows / 32).
template <bool SOFTMAX>
__global__ __launch_bounds__(256) void k_roni_mm_prep(const double *__restrict__ ww,
                                                      const double *__restrict__ deltas, int64_t ld,
                                                      int64_t din, int C, int64_t nmod, int64_t ldl,
                                                      int64_t rows, double *__restrict__ Wt,
                                                      double *__restrict__ bt) {
    __shared__ double tile[32][65];
    const int tid = threadIdx.x;
    const int P = RMM_NT / C;
    const int64_t col0 = (int64_t)blockIdx.x * 64, k0 = (int64_t)blockIdx.y * 32;
    {  // read: thread t -> column t >> 2, features (t & 3) * 8 .. + 7 (contiguous in the source)
        const int lc = tid >> 2, kk = (tid & 3) * 8;
        const int64_t col = col0 + lc;
        const int64_t y = col / RMM_NT;
        const int w = (int)(col - y * RMM_NT), p = w / C, c = w - p * C;
        const int64_t j = y * P + p;
        const bool live = p < P && j < nmod;
        const double *src0 = ww + (int64_t)c * din;
        const double *src1 = deltas + (j > 0 ? (j - 1) * ld : 0) + (int64_t)c * din;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = k0 + kk + u;
            double v = 0.0;  // padding: zero weights (x * 0 adds +0 to a chain that is never -0)
            if (live && k < din) {
                v = j == 0 ? src0[k] : src0[k] + src1[k];
                if (SOFTMAX) v = (double)(float)v;
            }
            tile[kk + u][lc] = v;
        }
        if (SOFTMAX && blockIdx.y == 0 && (tid & 3) == 0) {
            double v = 0.0;
            if (live) {
                const int64_t idx = (int64_t)C * din + c;
                v = (double)(float)(j == 0 ? ww[idx] : ww[idx] + deltas[(j - 1) * ld + idx]);
            }
            bt[col] = v;
        }
    }
    __syncthreads();
    // write: 64 consecutive columns of 4 rows per pass
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int kk = u * 4 + (tid >> 6), lc = tid & 63;
        if (k0 + kk < rows) Wt[(k0 + kk) * ldl + col0 + lc] = tile[kk][lc];
    }
}

// K8b' k_roni_logits: 64-sample x 128-column tiles, 4 waves of 32 samples x
// 64 columns (2 x 4 MFMA blocks), three waves per SIMD: 768 workgroup slots
// for the mnist bench shape's 846 tiles (94 sample tiles x 9 column tiles of
// 12 models; a split of k would break the FMA chain's order, so the tiles
// carry all of k).
// The samples go through LDS in chunks of 64 features ([sample][k], row
// stride 68 floats: the A fragment's 16 rows x 4 k and a staging write's 64
// lanes along k hit distinct banks; the next chunk's loads are in flight
// under this chunk's MFMAs); the B fragments come from L2 one k-step ahead,
// into alternating register sets.  Epilogue: logit = fp32(acc + b) into an
// LDS tile, then wave w takes models w, w + 4, ... of the tile, lane l sample
// l: np.argmax over the C logits, one ballot count and one atomic per model
// and workgroup.
// K8's near-tie test (oracle/roni_oracle.c softmax_eval, the same fp64
// expression): the winning logit l1 (class a) and the best other l2 can swap
// under torch's fp32 sgemm rounding only if
//     !( l1 - l2 - u (|l1| + |l2|)  >  E_a + max_c E_c ),  E_c = g (|x| |w_c| + |b_c|)
// (g = gamma_{d_in + 1}(2^-24) (1 + 2^-10), host-computed), or a logit is not
// finite.  xn = |x| of the sample, wn / b the model's C weight-row norms and
// biases (fp32 values), all fp64.
__device__ inline bool softmax_near_tie(const float *lg, int C, int best, double xn,
                                        const double *wn, const double *b, double g) {
    double wmax = 0.0, bmax = 0.0, l2 = -__builtin_inf();
    bool fin = true;
    for (int c = 0; c < C; ++c) {
        const double w = wn[c], ab = __builtin_fabs(b[c]), v = (double)lg[c];
        wmax = w > wmax ? w : wmax;
        bmax = ab > bmax ? ab : bmax;
        fin = fin && __builtin_isfinite(v);
        if (c != best && v > l2) l2 = v;
    }
    const double u = 0x1p-24, l1 = (double)lg[best];
    const double ea = g * (xn * wn[best] + __builtin_fabs(b[best]));
    const double emax = g * (xn * wmax + bmax);
    return !fin || !(l1 - l2 - u * (__builtin_fabs(l1) + __builtin_fabs(l2)) > ea + emax);
}

// |x_s| for every sample, bit for bit the oracle's sequential sum of squares
// in k order (every fp32 square is exact in fp64).  The sum is one dependent
// fp64 add per feature, so the kernel's floor is that chain plus one load
// round trip: a workgroup takes 16 samples (375 workgroups for 6,000), all 256
// threads stage a 16 x 512 chunk through LDS with every load in flight (the
// next chunk's issued before this one is summed), thread s < 16 adds its
// sample's squares in k order.  (r4f: 64 samples per workgroup and 64-feature
// chunks loaded one after another: 94 workgroups, 47 us at 6,000 x 784.)
constexpr int XN_S = 16, XN_KC = 512, XN_PT = XN_S * XN_KC / 256;
__global__ __launch_bounds__(256) void k_roni_xnorm(const float *__restrict__ Xv, int64_t nv,
                                                    int64_t din, int64_t ldv,
                                                    double *__restrict__ xn) {
    __shared__ float t[XN_S][XN_KC + 1];
    const int tid = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * XN_S;
    float v[XN_PT];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int u = 0; u < XN_PT; ++u) {
            const int i = tid + 256 * u, r = i / XN_KC, kk = i % XN_KC;
            const int64_t sr = s0 + r < nv ? s0 + r : nv - 1;
            v[u] = k0 + kk < din ? Xv[sr * ldv + k0 + kk] : 0.0f;
        }
    };
    double acc = 0.0;
    load(0);
    for (int64_t k0 = 0; k0 < din; k0 += XN_KC) {
        __syncthreads();  // the previous chunk has been summed
#pragma unroll
        for (int u = 0; u < XN_PT; ++u) {
            const int i = tid + 256 * u;
            t[i / XN_KC][i % XN_KC] = v[u];
        }
        __syncthreads();
        if (k0 + XN_KC < din) load(k0 + XN_KC);
        if (tid < XN_S) {
            const int kn = (int)(din - k0 < XN_KC ? din - k0 : XN_KC);
            int kk = 0;
            for (; kk + 16 <= kn; kk += 16) {
                float q[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) q[u] = t[tid][kk + u];
#pragma unroll
                for (int u = 0; u < 16; ++u) acc += (double)q[u] * (double)q[u];
            }
            for (; kk < kn; ++kk) {
                const double q = (double)t[tid][kk];
                acc += q * q;
            }
        }
    }
    if (tid < XN_S && s0 + tid < nv) xn[s0 + tid] = __builtin_sqrt(acc);
}

// |w_col| of every model-class column of Wt (the fp32 weights widened), k in
// order: the oracle's sequential sum.  A workgroup takes 16 columns (one
// 128-B run of each row): all 256 threads load a 256-row chunk of them with
// every load in flight (the next chunk's issued before this one is summed),
// thread c < 16 adds its column's values in k order from LDS.  (r4f: 64
// columns per workgroup, 16 workgroups for 1,024 columns: 19 us at d = 784.)
constexpr int WN_C = 16, WN_KC = 256, WN_PT = WN_C * WN_KC / 256;
__global__ __launch_bounds__(256) void k_roni_wnorm(const double *__restrict__ Wt, int64_t ldl,
                                                    int64_t din, double *__restrict__ wn) {
    __shared__ double t[WN_KC][WN_C + 1];
    const int tid = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * WN_C;
    const int cc = tid % WN_C, r0 = tid / WN_C;  // 16 rows per pass of the workgroup
    const int64_t col = c0 + cc < ldl ? c0 + cc : ldl - 1;
    double v[WN_PT];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int u = 0; u < WN_PT; ++u) {
            const int64_t k = k0 + r0 + (256 / WN_C) * u;
            v[u] = k < din ? Wt[k * ldl + col] : 0.0;
        }
    };
    double acc = 0.0;
    load(0);
    for (int64_t k0 = 0; k0 < din; k0 += WN_KC) {
        __syncthreads();  // the previous chunk has been summed
#pragma unroll
        for (int u = 0; u < WN_PT; ++u) t[r0 + (256 / WN_C) * u][cc] = v[u];
        __syncthreads();
        if (k0 + WN_KC < din) load(k0 + WN_KC);
        if (tid < WN_C) {
            const int kn = (int)(din - k0 < WN_KC ? din - k0 : WN_KC);
            int kk = 0;
            for (; kk + 16 <= kn; kk += 16) {
                double q[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) q[u] = t[kk + u][tid];
#pragma unroll
                for (int u = 0; u < 16; ++u) acc += q[u] * q[u];
            }
            for (; kk < kn; ++kk) acc += t[kk][tid] * t[kk][tid];
        }
    }
    if (tid < WN_C && c0 + tid < ldl) wn[c0 + tid] = __builtin_sqrt(acc);
}

constexpr int RG_MT = 64, RG_NT = 128, RG_LT = RG_NT + 1;
constexpr int RL_KC = 64, RL_XS = 68;

__global__ __launch_bounds__(256) void k_roni_logits(const float *__restrict__ Xv, int64_t nv,
                                                     int64_t din, int64_t ldv,
                                                     const int32_t *__restrict__ yv, int C,
                                                     const double *__restrict__ Wt,
                                                     const double *__restrict__ bt, int64_t ldl,
                                                     int64_t nmod, int nx, int xcd_cols,
                                                     unsigned int *__restrict__ good,
                                                     const double *__restrict__ xn,
                                                     const double *__restrict__ wnrm, double g,
                                                     unsigned int *__restrict__ near) {
    __shared__ float xs[RG_MT][RL_XS];
    __shared__ float lt[RG_MT][RG_LT];
    const int tid = threadIdx.x, l = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    // tile (x, y): with xcd_cols, column tile y lives on XCD y mod 8 (block
    // numbers = y mod 8), so an XCD's L2 holds only its eighth of Wt
    const int blk = blockIdx.x;
    int tx, ty;
    if (xcd_cols) {
        const int q = blk >> 3;
        tx = q % nx;
        ty = (blk & 7) + 8 * (q / nx);
    } else {
        tx = blk % nx;
        ty = blk / nx;
    }
    const int64_t s0 = (int64_t)tx * RG_MT;
    const int64_t cb = (int64_t)ty * RG_NT, c0 = cb + 64 * wn;
    // a wave whose 64 columns are all padding (the last tile's) skips its
    // MFMAs: only the staging and the barriers are shared
    const int P = RG_NT / C;
    const int64_t live_models = nmod - (int64_t)ty * P < P ? nmod - (int64_t)ty * P : P;
    const bool live = 64 * wn < live_models * C;
    d4 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) acc[a][bb] = d4{0.0, 0.0, 0.0, 0.0};
    // staging: thread t moves feature t & 63 of samples (t >> 6) + 4 u
    const int xk = tid & 63, xsr = tid >> 6;
    const double *wcol = Wt + c0 + (l & 15) + (int64_t)(l >> 4) * ldl;
    const int arow = 32 * wm + (l & 15), ak = l >> 4;
    float xv[16];  // clamped addresses, every load in flight
    auto load_x = [&](int64_t k0) {
        int64_t k = k0 + xk;
        k = k < din ? k : din - 1;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            int64_t s = s0 + xsr + 4 * u;
            s = s < nv ? s : nv - 1;
            xv[u] = Xv[s * ldv + k];
        }
    };
    load_x(0);
    for (int64_t k0 = 0; k0 < din; k0 += RL_KC) {
        __syncthreads();  // the previous chunk has been consumed
        const bool kin = k0 + xk < din;
#pragma unroll
        for (int u = 0; u < 16; ++u) xs[xsr + 4 * u][xk] = kin ? xv[u] : 0.0f;
        __syncthreads();
        if (k0 + RL_KC < din) load_x(k0 + RL_KC);
        const int kn = (int)(din - k0 < RL_KC ? din - k0 : RL_KC);
        // k-steps in pairs (rows past d_in are zero in LDS and in Wt), the B
        // fragments of the next step loaded before this step's MFMAs, into the
        // other register set: their L2 latency runs under the MFMAs
        const int steps = live ? ((kn + 7) >> 3) << 1 : 0;
        const double *wk = wcol + k0 * ldl;
        double b0[4], b1[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) b0[b] = live ? wk[16 * b] : 0.0;
        for (int st = 0; st < steps; st += 2) {
            const int64_t o1 = (int64_t)(st + 1) * 4 * ldl;
            const int64_t o2 = (int64_t)(st + 2 < steps ? st + 2 : st + 1) * 4 * ldl;
#pragma unroll
            for (int b = 0; b < 4; ++b) b1[b] = wk[o1 + 16 * b];
            double a0 = (double)xs[arow][4 * st + ak];
            double a1 = (double)xs[arow + 16][4 * st + ak];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                acc[0][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0[b], acc[0][b], 0, 0, 0);
                acc[1][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0[b], acc[1][b], 0, 0, 0);
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) b0[b] = wk[o2 + 16 * b];
            a0 = (double)xs[arow][4 * st + 4 + ak];
            a1 = (double)xs[arow + 16][4 * st + 4 + ak];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                acc[0][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1[b], acc[0][b], 0, 0, 0);
                acc[1][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1[b], acc[1][b], 0, 0, 0);
            }
        }
    }
    // D reg r of lane l: sample row (l >> 4) + 4 r of the block, column l & 15
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int lc = 64 * wn + 16 * b + (l & 15);
        const double bias = bt[cb + lc];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                lt[32 * wm + 16 * a + (l >> 4) + 4 * r][lc] = (float)(acc[a][b][r] + bias);
    }
    __syncthreads();
    // np.argmax: the first maximum, a NaN wins at its first place
    const int64_t s = s0 + l;
    const int64_t sc = s < nv ? s : nv - 1;
    const int ysl = yv[sc];
    const double xnl = xn[sc];
    for (int p = wave; p < P; p += 4) {
        const int64_t j = (int64_t)ty * P + p;
        if (j >= nmod) break;  // wave-uniform
        const float *lg = &lt[l][p * C];
        const int64_t col0 = cb + (int64_t)p * C;
        int best = 0;
        float bl = lg[0];
        for (int c = 1; c < C; ++c) {
            const float v = lg[c];
            if (!(bl != bl) && (v != v || v > bl)) {
                best = c;
                bl = v;
            }
        }
        const bool nt = softmax_near_tie(lg, C, best, xnl, wnrm + col0, bt + col0, g);
        const unsigned int ok = (unsigned int)__popcll(__ballot(s < nv && best == ysl));
        const unsigned int nn = (unsigned int)__popcll(__ballot(s < nv && nt));
        if (l == 0 && ok) atomicAdd(&good[j], ok);
        if (l == 0 && nn) atomicAdd(&near[j], nn);
    }
}

// K7' k_roni_sign: the logistic verifier's GEMM (fp64 samples, one model per
// column) with the sign test fused into its epilogue.  Same 64 x 128 tiles
// and waves; both operands through LDS in chunks of 32 k ([sample][k] row
// stride 34 doubles, [k][column] row stride 144 doubles: every fragment read
// and staging write on distinct banks), the next chunk's loads in registers
// under this chunk's MFMAs (and the tile's labels with its first chunk).  A
// workgroup walks tiles_per_wg (8) sample tiles; with d <= 32 (creditcard:
// 25) the weights are staged once.  Counts stay in
// registers; two lane butterflies and one atomic per model and wave at the end.
constexpr int RS_KC = 32, RS_XS = 34, RS_BS = 144;

__global__ __launch_bounds__(256) void k_roni_sign(const double *__restrict__ Xv, int64_t nv,
                                                   int64_t din, int64_t ldv,
                                                   const double *__restrict__ yv,
                                                   const double *__restrict__ Wt, int64_t ldl,
                                                   int64_t nmod, int nx, int tiles_per_wg,
                                                   unsigned int *__restrict__ cnt) {
    __shared__ double xs[RG_MT][RS_XS];
    __shared__ double bs[RS_KC][RS_BS];
    const int tid = threadIdx.x, l = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const int tx = blockIdx.x % nx, ty = blockIdx.x / nx;
    const int64_t tiles = (nv + RG_MT - 1) / RG_MT;
    const int64_t t0 = (int64_t)tx * tiles_per_wg;
    const int nt = (int)(tiles - t0 < tiles_per_wg ? tiles - t0 : tiles_per_wg);
    const int nch = (int)((din + RS_KC - 1) / RS_KC);
    const int ni = nt * nch;
    const bool restage_b = nch > 1;
    const int64_t cb = (int64_t)ty * RG_NT;  // the tile's first column
    // staging maps (global loads coalesced, LDS writes conflict-free): sample
    // (t >> 5) + 8 u, feature t & 31; weights row 2 u + (t >> 7), column t & 127
    const int xs_s = tid >> 5, xs_k = tid & 31;
    const int bs_k = tid >> 7, bs_c = tid & 127;
    double xv[8], bv[16], yn[8], yc[8];
    // y of this lane's 8 epilogue rows (a, r), loaded with the tile's first chunk
    auto load_y = [&](int tt) {
        const int64_t s0 = (t0 + tt) * RG_MT + 32 * wm + (l >> 4);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t s = s0 + 16 * a + 4 * r;
                yn[4 * a + r] = yv[s < nv ? s : nv - 1];
            }
    };
    auto prefetch = [&](int it, bool with_b) {
        const int tt = it / nch, ch = it - tt * nch;
        if (ch == 0) load_y(tt);
        int64_t k = (int64_t)ch * RS_KC + xs_k;
        k = k < din ? k : din - 1;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            int64_t s = (t0 + tt) * RG_MT + xs_s + 8 * u;
            s = s < nv ? s : nv - 1;
            xv[u] = Xv[s * ldv + k];
        }
        if (with_b) {
            const double *br = Wt + ((int64_t)ch * RS_KC + bs_k) * ldl + cb + bs_c;
#pragma unroll
            for (int u = 0; u < 16; ++u) bv[u] = br[2 * u * ldl];
        }
    };
    d4 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) acc[a][bb] = d4{0.0, 0.0, 0.0, 0.0};
    unsigned int mis[4] = {0, 0, 0, 0};
    const int arow = 32 * wm + (l & 15), ak = l >> 4;
    const int bcol = 64 * wn + (l & 15);
    prefetch(0, true);
    for (int it = 0; it < ni; ++it) {
        const int tt = it / nch, ch = it - tt * nch;
        __syncthreads();  // the previous chunk has been consumed
        const bool kin = (int64_t)ch * RS_KC + xs_k < din;
#pragma unroll
        for (int u = 0; u < 8; ++u) xs[xs_s + 8 * u][xs_k] = kin ? xv[u] : 0.0;
        if (restage_b || it == 0) {
#pragma unroll
            for (int u = 0; u < 16; ++u) bs[bs_k + 2 * u][bs_c] = bv[u];
        }
        __syncthreads();
        if (ch == 0) {
#pragma unroll
            for (int q = 0; q < 8; ++q) yc[q] = yn[q];
        }
        if (it + 1 < ni) prefetch(it + 1, restage_b);
        const int64_t kr = din - (int64_t)ch * RS_KC;
        const int steps = ((int)(kr < RS_KC ? kr : RS_KC) + 3) >> 2;  // rows past d are zero
        for (int st = 0; st < steps; ++st) {
            const double a0 = xs[arow][4 * st + ak], a1 = xs[arow + 16][4 * st + ak];
            double bf[4];
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) bf[bb] = bs[4 * st + ak][bcol + 16 * bb];
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) {
                acc[0][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bf[bb], acc[0][bb], 0, 0, 0);
                acc[1][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bf[bb], acc[1][bb], 0, 0, 0);
            }
        }
        if (ch != nch - 1) continue;
        // D reg r of lane l: sample row (l >> 4) + 4 r of the block, model column l & 15
        const int64_t s0 = (t0 + tt) * RG_MT;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t s = s0 + 32 * wm + 16 * a + (l >> 4) + 4 * r;
                const double y = yc[4 * a + r];
#pragma unroll
                for (int bb = 0; bb < 4; ++bb) {
                    const double v = acc[a][bb][r];  // np.sign: 0 -> 0, NaN -> NaN
                    const double yh = v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : (v == 0.0 ? 0.0 : v));
                    mis[bb] += (s < nv && !(yh == y)) ? 1u : 0u;
                    acc[a][bb][r] = 0.0;
                }
            }
    }
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
        unsigned int tot = mis[bb];
        tot += __shfl_xor(tot, 16);
        tot += __shfl_xor(tot, 32);
        const int64_t j = cb + 64 * wn + 16 * bb + l;
        if (l < 16 && tot && j < nmod) atomicAdd(&cnt[j], tot);
    }
}

// K7' for d <= 32 (the creditcard verifier: d = 25), r6: every wave works
// alone -- no LDS, no barriers.  A wave owns 64 model columns and walks `per`
// blocks of 32 samples: its B fragments (all <= 8 k-steps x 4 column blocks)
// are loaded once into registers, each sample block's A fragments and labels
// straight from global memory into registers, issued as soon as the previous
// block's MFMAs have read theirs.
// The same fragments, the same v_mfma_f64_16x16x4_f64 chain over k ascending
// from +0.0 and the same epilogue as k_roni_sign: bitwise the same counts.
// (k_roni_sign at creditcard shape: 113 us, MFMA busy 34 %, two workgroups per
// CU by LDS, a barrier pair per tile; profiles/r06/pmc_roni_r06.md.)
constexpr int RSR_S = 8;  // k-steps of 4: d <= 32
template <int NA>  // 16-sample row blocks per wave block: 2 (2 waves / SIMD) or 1 (3)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NA == 1 ? 3 : 2))) void k_roni_sign_reg(const double *__restrict__ Xv, int64_t nv,
                                                       int64_t din, int64_t ldv,
                                                       const double *__restrict__ yv,
                                                       const double *__restrict__ Wt, int64_t ldl,
                                                       int64_t nmod, int64_t sblocks, int per,
                                                       unsigned int *__restrict__ cnt, int abl) {
    const int l = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t cblocks = ldl / 64;
    const int64_t cb = (w % cblocks) * 64;  // neighbouring waves: the same samples
    const int64_t sb0 = (w / cblocks) * per;
    if (sb0 >= sblocks) return;  // whole waves only; nothing below synchronises
    const int nsb = (int)(sblocks - sb0 < per ? sblocks - sb0 : per);
    const int S = (int)((din + 3) / 4);
    const int kq = l >> 4, c16 = l & 15;
    double bf[RSR_S][4];
#pragma unroll
    for (int st = 0; st < RSR_S; ++st)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {  // rows past d are zero in Wt (rmm_rows >= 32)
            const double w = Wt[(int64_t)(4 * st + kq) * ldl + cb + 16 * bb + c16];
            bf[st][bb] = st < S ? w : 0.0;
        }
    double an[NA][RSR_S], yn[4 * NA];
    auto load = [&](int64_t sb) {
        const int64_t r0 = sb * 16 * NA;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            int64_t s = r0 + 16 * a + c16;
            s = s < nv ? s : nv - 1;
#pragma unroll
            for (int st = 0; st < RSR_S; ++st) {  // unconditional loads, then a select
                const int64_t k = 4 * st + kq;
                const double x = Xv[s * ldv + (k < din ? k : din - 1)];
                an[a][st] = k < din ? x : 0.0;
            }
        }
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t s = r0 + 16 * a + kq + 4 * r;
                yn[4 * a + r] = yv[s < nv ? s : nv - 1];
            }
    };
    unsigned int mis[4] = {0, 0, 0, 0};
    load(sb0);
    for (int i = 0; i < nsb; ++i) {
        d4 acc[NA][4];
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) acc[a][bb] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < RSR_S; ++st) {
            if (st < S) {
#pragma unroll
                for (int bb = 0; bb < 4; ++bb) {
#pragma unroll
                    for (int a = 0; a < NA; ++a)
                        acc[a][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(an[a][st], bf[st][bb], acc[a][bb], 0, 0, 0);
                }
            }
        }
        // the next block's fragments land in the same registers once these
        // MFMAs have read them: their latency runs under the MFMAs in flight
        // and this block's epilogue (a second buffer would take the wave past
        // 256 registers, one wave per SIMD)
        double yc[4 * NA];
#pragma unroll
        for (int q = 0; q < 4 * NA; ++q) yc[q] = yn[q];
        if (i + 1 < nsb && !(abl & 2)) load(sb0 + i + 1);  // abl & 2: timing-only, no reloads
        // D reg r of lane l: sample row (l >> 4) + 4 r of the block, column l & 15
        const int64_t s0 = (sb0 + i) * 16 * NA;
        if (abl & 1) {  // timing-only: one compare per accumulator instead of the epilogue
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) mis[bb] += (unsigned int)(acc[0][bb][0] == 1234.5 || acc[NA - 1][bb][3] == 1234.5);
            continue;
        }
        // !(np.sign(v) == y) by the label's class: sign(v) is 1, -1, +-0 or
        // NaN, so it equals y only for y = 1 and v > 0, y = -1 and v < 0, or
        // y = +-0 and v = +-0 (any other y, NaN included, never matches).
        // Three compares per output and lane-mask logic, no selects.
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double y = yc[4 * a + r];
                const bool ok = s0 + 16 * a + kq + 4 * r < nv;
                const bool yp = y == 1.0, yn = y == -1.0, yz = y == 0.0;
#pragma unroll
                for (int bb = 0; bb < 4; ++bb) {
                    const double v = acc[a][bb][r];
                    const bool match = (yp & (v > 0.0)) | (yn & (v < 0.0)) | (yz & (v == 0.0));
                    mis[bb] += (unsigned int)(ok & !match);
                }
            }
    }
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
        unsigned int tot = mis[bb];
        tot += __shfl_xor(tot, 16);
        tot += __shfl_xor(tot, 32);
        const int64_t j = cb + 16 * bb + l;
        if (l < 16 && tot && j < nmod) atomicAdd(&cnt[j], tot);
    }
}

double roni_softmax_g(int64_t din) {
    const double u = 0x1p-24, nn = (double)(din + 1);
    return nn * u / (1.0 - nn * u) * (1.0 + 0x1p-10);
}

// Wt ((rows + 1) x ldl: the weights, then the biases), wn (ldl), xn (nv)
size_t roni_softmax_ws(int64_t n, int64_t din, int64_t nv, int C) {
    const int64_t ldl = rmm_ldl(n, C);
    return ((size_t)(rmm_rows(din) + 1) * ldl + (size_t)ldl + (size_t)nv) * sizeof(double);
}

hipError_t launch_roni_xnorm(const float *Xv, int64_t nv, int64_t din, int64_t ldv, double *xn,
                             hipStream_t st) {
    hipLaunchKernelGGL(k_roni_xnorm, dim3((unsigned)((nv + XN_S - 1) / XN_S)), dim3(256), 0, st, Xv, nv, din,
                       ldv, xn);
    return hipGetLastError();
}

// xn: the samples' norms (nullable: computed here into the workspace);
// good / near: 2 (n + 1) counters (correct predictions, then near ties)
hipError_t launch_roni_softmax(const float *Xv, int64_t nv, int64_t din, int64_t ldv,
                               const int32_t *yv, int C, const double *ww, const double *deltas,
                               int64_t n, int64_t ld, double *ws, const double *xn,
                               unsigned int *good, double *scores, int32_t *near_out,
                               hipStream_t st) {
    const int64_t nmod = n + 1, ldl = rmm_ldl(n, C), rows = rmm_rows(din);
    double *Wt = ws, *bt = ws + rows * ldl, *wn = bt + ldl, *xw = wn + ldl;
    unsigned int *near = good + nmod;
    hipError_t e = hipMemsetAsync(good, 0, (size_t)2 * nmod * sizeof(unsigned int), st);
    if (e != hipSuccess) return e;
    if (!xn) {
        if ((e = launch_roni_xnorm(Xv, nv, din, ldv, xw, st)) != hipSuccess) return e;
        xn = xw;
    }
    hipLaunchKernelGGL(k_roni_mm_prep<true>, dim3((unsigned)(ldl / 64), (unsigned)((rows + 31) / 32)),
                       dim3(256), 0, st, ww, deltas, ld, din, C, nmod, ldl, rows, Wt, bt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_wnorm, dim3((unsigned)((ldl + WN_C - 1) / WN_C)), dim3(256), 0, st, Wt, ldl,
                       din, wn);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int64_t nx64 = (nv + RG_MT - 1) / RG_MT, ny64 = ldl / RG_NT;
    if (nx64 * ny64 > 0x7fffffff) return hipErrorInvalidConfiguration;  // grid limit
    const int nx = (int)nx64, ny = (int)ny64;
    hipLaunchKernelGGL(k_roni_logits, dim3((unsigned)(nx * ny)), dim3(256), 0, st, Xv, nv, din, ldv,
                       yv, C, Wt, bt, ldl, nmod, nx, ny % 8 == 0 ? 1 : 0, good, xn, wn,
                       roni_softmax_g(din), near);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_mc_score, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, good,
                       n, nv, scores);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (near_out)
        e = hipMemcpyAsync(near_out, near, (size_t)nmod * sizeof(int32_t), hipMemcpyDeviceToDevice,
                           st);
    return e;
}

// ---------------------------------------------------------------------------
// K8 with the reference's batch semantics.  getTrainErr
// (ML/Pytorch/client.py:136-144) walks the SHUFFLED trainloader (client.py:20)
// and returns the error of its LAST mini-batch only (the loop overwrites pred
// and labels): client_obj.roni (client_obj.py:100-112) measures `original`
// (model ww) and `after` (model ww + delta) on two different random batches of
// batch_size samples (10 in Biscotti, honest.go:47).  The caller draws them and
// passes per update j the sample indices idx[(2 j) nb ..] and idx[(2 j + 1) nb ..].
//
//   k_roni_batch   one workgroup per update, both evaluations: the two models'
//                  fp32 weights (ww, and ww + delta_j rounded after the fp64 add)
//                  and the two batches' samples staged through LDS in chunks of
//                  RB_KC features; thread (e, s, c) runs logit c of sample s of
//                  evaluation e as the fp64 FMA chain over k ascending (the
//                  oracle's, bit for bit), rounds fp32(acc + b); then np.argmax,
//                  the correct count, the near-tie count (the same test as the
//                  full-set kernel) and the score, written by the workgroup.
// Bound: HBM -- each update's delta (C (d_in + 1) fp64) and its 2 nb gathered
// samples are read once; the FMA work is 2 nb C d_in per update.
// r4d: 512 threads and 16 samples per tile (Biscotti's batch of 10 is one
// tile: one pass of the k-chains instead of two), the tile's sample indices
// read once into LDS, and every staging load of a chunk issued before the
// first LDS store (r4c staged one element per loop trip with the index load
// and the sample load dependent in each: 160 us for 100 updates, 0.01 of HBM)
constexpr int RB_NT = 512, RB_ST = 16, RB_KC = 128, RB_KP = RB_KC + 4;
constexpr int RB_WPT = 2 * 16 * RB_KC / RB_NT;       // weight elements per thread (C <= 16)
constexpr int RB_XPT = 2 * RB_ST * RB_KC / RB_NT;    // sample elements per thread

__global__ __launch_bounds__(RB_NT) void k_roni_batch(const float *__restrict__ Xv, int64_t nv,
                                                      int64_t din, int64_t ldv,
                                                      const int32_t *__restrict__ yv, int C,
                                                      const double *__restrict__ ww,
                                                      const double *__restrict__ deltas, int64_t ld,
                                                      const int64_t *__restrict__ idx, int64_t nb,
                                                      double g, double *__restrict__ scores,
                                                      int32_t *__restrict__ near_out) {
    // read through 16-B (f4) casts: aligned explicitly, not by the LDS layout's luck
    __shared__ __attribute__((aligned(16))) float xs[2][RB_ST][RB_KP];
    __shared__ __attribute__((aligned(16))) float wsm[2][16][RB_KP];
    __shared__ float lgs[2][RB_ST][16];
    __shared__ double xnl[2][RB_ST], wnl[2][16], bl[2][16];
    __shared__ int64_t srow[2][RB_ST];
    __shared__ unsigned int cnt[5];  // good0, good1, near0, near1, bad index
    const int tid = threadIdx.x;
    const int64_t j = blockIdx.x;
    const double *dj = deltas + j * ld;
    const int64_t *ix = idx + 2 * j * nb;
    const int nlog = 2 * RB_ST * C;
    const bool lt = tid < nlog;
    const int le = tid / (RB_ST * C), lr = tid - le * (RB_ST * C), ls = lr / C, lc = lr - ls * C;
    if (tid < 5) cnt[tid] = 0;
    if (tid < 2 * C) {  // the two models' fp32 biases
        const int e = tid / C, c = tid - e * C;
        const int64_t bi = (int64_t)C * din + c;
        bl[e][c] = (double)(float)(e == 0 ? ww[bi] : ww[bi] + dj[bi]);
    }
    double wnacc = 0.0;  // thread (e, s = 0, c): |w_c| of model e (first tile)
    unsigned int good[2] = {0, 0}, near[2] = {0, 0};
    for (int64_t st0 = 0; st0 < nb; st0 += RB_ST) {
        const int ns = (int)(nb - st0 < RB_ST ? nb - st0 : RB_ST);
        __syncthreads();  // the previous tile's rows and logits have been used
        if (tid < 2 * RB_ST) {  // the tile's sample rows (padding repeats sample 0, never counted)
            const int e = tid / RB_ST, s = tid - e * RB_ST;
            int64_t row = ix[e * nb + st0 + (s < ns ? s : 0)];
            if (row < 0 || row >= nv) {
                cnt[4] = 1;  // reported as score NaN, near ties -1; never read out of range
                row = 0;
            }
            srow[e][s] = row;
        }
        double acc = 0.0, xacc = 0.0;  // logit (le, ls, lc); thread c == 0: |x_s|
        double wa[RB_WPT], wb[RB_WPT];
        float xv[RB_XPT];
        // chunk k0's loads into registers (every load issued before any use)
        auto load = [&](int64_t k0) {
            const int kn = (int)(din - k0 < RB_KC ? din - k0 : RB_KC);
#pragma unroll
            for (int q = 0; q < RB_WPT; ++q) {
                const int i = tid + RB_NT * q;
                const int e = i / (16 * RB_KC), r = i - e * (16 * RB_KC), c = r / RB_KC,
                          kk = r - c * RB_KC;
                const bool on = c < C && kk < kn;
                const int64_t wi = on ? (int64_t)c * din + k0 + kk : 0;
                wa[q] = on ? ww[wi] : 0.0;
                wb[q] = on && e == 1 ? dj[wi] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < RB_XPT; ++q) {
                const int i = tid + RB_NT * q;
                const int e = i / (RB_ST * RB_KC), r = i - e * (RB_ST * RB_KC), s = r / RB_KC,
                          kk = r - s * RB_KC;
                xv[q] = kk < kn ? Xv[srow[e][s] * ldv + k0 + kk] : 0.0f;
            }
        };
        __syncthreads();  // srow is written
        load(0);
        for (int64_t k0 = 0; k0 < din; k0 += RB_KC) {
            const int kn = (int)(din - k0 < RB_KC ? din - k0 : RB_KC);
            __syncthreads();  // the previous chunk has been consumed
#pragma unroll
            for (int q = 0; q < RB_WPT; ++q) {
                const int i = tid + RB_NT * q;
                const int e = i / (16 * RB_KC), r = i - e * (16 * RB_KC), c = r / RB_KC,
                          kk = r - c * RB_KC;
                if (c < C) wsm[e][c][kk] = kk < kn ? (float)(e == 0 ? wa[q] : wa[q] + wb[q]) : 0.0f;
            }
#pragma unroll
            for (int q = 0; q < RB_XPT; ++q) {
                const int i = tid + RB_NT * q;
                const int e = i / (RB_ST * RB_KC), r = i - e * (RB_ST * RB_KC), s = r / RB_KC,
                          kk = r - s * RB_KC;
                xs[e][s][kk] = xv[q];
            }
            __syncthreads();
            // the next chunk's loads fly under this chunk's FMA chains
            if (k0 + RB_KC < din) load(k0 + RB_KC);
            if (lt) {
                const float *xr = xs[le][ls], *wr = wsm[le][lc];
                const bool xn = lc == 0, wn = ls == 0 && st0 == 0;
                // 16 columns at a time: their 8 LDS reads issued together, then
                // the 16 FMAs of the chain in k order (r4c read 2 floats and
                // waited for them before every FMA: ~100 cycles per step)
                int kk = 0;
                for (; kk + 16 <= kn; kk += 16) {
                    typedef float f4 __attribute__((ext_vector_type(4)));
                    f4 xq[4], wq[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        xq[q] = *reinterpret_cast<const f4 *>(xr + kk + 4 * q);
                        wq[q] = *reinterpret_cast<const f4 *>(wr + kk + 4 * q);
                    }
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        const double x = (double)xq[u >> 2][u & 3], w = (double)wq[u >> 2][u & 3];
                        acc = __builtin_fma(x, w, acc);
                        if (xn) xacc += x * x;
                        if (wn) wnacc += w * w;
                    }
                }
                for (; kk < kn; ++kk) {
                    const double x = (double)xr[kk];
                    acc = __builtin_fma(x, (double)wr[kk], acc);
                    if (xn) xacc += x * x;
                    if (wn) wnacc += (double)wr[kk] * (double)wr[kk];
                }
            }
        }
        if (lt) {
            lgs[le][ls][lc] = (float)(acc + bl[le][lc]);
            if (lc == 0) xnl[le][ls] = __builtin_sqrt(xacc);
            if (ls == 0 && st0 == 0) wnl[le][lc] = __builtin_sqrt(wnacc);
        }
        __syncthreads();
        if (tid < 2 * RB_ST) {
            const int e = tid / RB_ST, s = tid - e * RB_ST;
            if (s < ns) {
                const float *lg = lgs[e][s];
                int best = 0;
                float b0 = lg[0];
                for (int c = 1; c < C; ++c)
                    if (!(b0 != b0) && (lg[c] != lg[c] || lg[c] > b0)) {
                        best = c;
                        b0 = lg[c];
                    }
                good[e] += best == yv[srow[e][s]];
                near[e] += softmax_near_tie(lg, C, best, xnl[e][s], wnl[e], bl[e], g);
            }
        }
    }
    if (tid < 2 * RB_ST) {
        atomicAdd(&cnt[0], good[0]);
        atomicAdd(&cnt[1], good[1]);
        atomicAdd(&cnt[2], near[0]);
        atomicAdd(&cnt[3], near[1]);
    }
    __syncthreads();
    if (tid == 0) {
        const double dn = (double)nb;
        const double orig = 1.0 - (double)cnt[0] / dn, after = 1.0 - (double)cnt[1] / dn;
        const bool bad = cnt[4] != 0;
        scores[j] = bad ? __builtin_nan("") : after - orig;
        if (near_out) {
            near_out[2 * j] = bad ? -1 : (int32_t)cnt[2];
            near_out[2 * j + 1] = bad ? -1 : (int32_t)cnt[3];
        }
    }
}

hipError_t launch_roni_softmax_batches(const float *Xv, int64_t nv, int64_t din, int64_t ldv,
                                       const int32_t *yv, int C, const double *ww,
                                       const double *deltas, int64_t n, int64_t ld,
                                       const int64_t *idx, int64_t nb, double *scores,
                                       int32_t *near_out, hipStream_t st) {
    hipLaunchKernelGGL(k_roni_batch, dim3((unsigned)n), dim3(RB_NT), 0, st, Xv, nv, din, ldv, yv, C,
                       ww, deltas, ld, idx, nb, roni_softmax_g(din), scores, near_out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K7 on the matrix pipe (r3b): S[s][j] = x_s . w_j as one GEMM (M = nv
// samples, N = n + 1 models, K = d) on k_roni_sign: a chain of
// v_mfma_f64_16x16x4_f64 over k ascending from +0.0 -- the same fp64 FMA
// chain as K7's VALU kernel and the oracle, bit for bit -- and the sign test
// fused into the epilogue.  No cap on d (K7's LDS model held d <= 1024).

size_t roni_ws(int64_t n, int64_t d) {
    return (size_t)rmm_rows(d) * ((n + 1 + RMM_NT - 1) / RMM_NT * RMM_NT) * sizeof(double);
}

hipError_t launch_roni(const double *Xv, int64_t nv, int64_t d, int64_t ldv, const double *yv,
                       const double *ww, const double *deltas, int64_t n, int64_t ld,
                       double *ws, unsigned int *cnt, double *scores, hipStream_t st) {
    const int64_t nmod = n + 1, ldl = (nmod + RMM_NT - 1) / RMM_NT * RMM_NT, rows = rmm_rows(d);
    hipError_t e = hipMemsetAsync(cnt, 0, (size_t)nmod * sizeof(unsigned int), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_mm_prep<false>, dim3((unsigned)(ldl / 64), (unsigned)((rows + 31) / 32)),
                       dim3(256), 0, st, ww, deltas, ld, d, 1, nmod, ldl, rows, ws, (double *)nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // sample tiles per workgroup (8; BK_RONI_TILES for A/B): more, shorter
    // workgroups hide each tile's barrier and LDS latency behind the others
    static const int per_env = [] {
        const char *e = probe_env("BK_RONI_TILES");
        const int v = e ? atoi(e) : 0;
        return v >= 1 && v <= 256 ? v : 8;
    }();
    if (d <= 4 * RSR_S && !probe_env("BK_RONI_LDS")) {
        // one round of resident waves (2 per SIMD at 256 registers): each
        // wave walks `per` 32-sample blocks, and the grid never spills into a
        // second round (2,050 waves for 2,048 slots would double the time)
        static const int64_t slots = [] {
            int dev = 0, cus = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
                cus <= 0)
                cus = 256;
            return (int64_t)cus * 4 * 2;
        }();
        const char *na_env = probe_env("BK_RONI_NA");
        const int na = na_env && atoi(na_env) == 2 ? 2 : 1;
        const int64_t sblocks = (nv + 16 * na - 1) / (16 * na), cblocks = ldl / 64;
        int64_t groups = slots * (na == 1 ? 3 : 2) / 2 / cblocks;
        if (groups < 1) groups = 1;
        if (const char *g = probe_env("BK_RONI_GROUPS")) groups = atoi(g) > 0 ? atoi(g) : groups;
        const int64_t per = (sblocks + groups - 1) / groups;
        const char *ab = probe_env("BK_RONI_ABL");  // timing-only ablations (probe build)
        const int abl = ab ? atoi(ab) : 0;
        const int64_t waves = cblocks * ((sblocks + per - 1) / per);
        if ((waves + 3) / 4 > 0x7fffffff) return hipErrorInvalidConfiguration;
        if (na == 1)
            hipLaunchKernelGGL(k_roni_sign_reg<1>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, Xv,
                               nv, d, ldv, yv, ws, ldl, nmod, sblocks, (int)per, cnt, abl);
        else
            hipLaunchKernelGGL(k_roni_sign_reg<2>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, Xv,
                               nv, d, ldv, yv, ws, ldl, nmod, sblocks, (int)per, cnt, abl);
    } else {
    const int64_t tiles = (nv + RG_MT - 1) / RG_MT, ny = ldl / RG_NT;
    const int64_t per = per_env;
    const int64_t nx64 = (tiles + per - 1) / per;
    if (nx64 * ny > 0x7fffffff) return hipErrorInvalidConfiguration;  // grid limit
    const int nx = (int)nx64;
    hipLaunchKernelGGL(k_roni_sign, dim3((unsigned)(nx * ny)), dim3(256), 0, st, Xv, nv, d, ldv, yv,
                       ws, ldl, nmod, nx, (int)per, cnt);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_score, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cnt, n,
                       nv, scores);
    return hipGetLastError();
}

}  // namespace bk
