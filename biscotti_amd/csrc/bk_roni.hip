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
#include <stdlib.h>

#include "bk_internal.h"

namespace bk {

// A/B knob: BK_RONI_VALU=1 runs the r3a VALU kernels (K7 for d <= 1024, K8)
static bool roni_valu() {
    static const bool v = [] {
        const char *e = getenv("BK_RONI_VALU");
        return e && atoi(e) != 0;
    }();
    return v;
}

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

static hipError_t launch_roni_valu(const double *Xv, int64_t nv, int64_t d, int64_t ldv,
                                   const double *yv, const double *ww, const double *deltas,
                                   int64_t n, int64_t ld, unsigned int *cnt, double *scores,
                                   hipStream_t st) {
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


// ---------------------------------------------------------------------------
// K8: the torch-path RONI (the mnist / lfw softmax verifiers) --
// client_obj.roni(ww, delta), ML/Pytorch/client_obj.py:100-112: the flat
// weights [W (C x D_in, row-major), b (C)] rounded to fp32 after the fp64
// add (SoftmaxModel.reshape -> torch.FloatTensor, softmax_model.py:19-24), the
// training error 1 - accuracy of argmax(x W^T + b) (client.py:131-139), and
// score = err(ww + delta) - err(ww).  d = 7,850 for mnist: the model no longer
// fits K7's LDS layout, and the error is a 10-way argmax, not a sign.
//
//   K8a k_roni_mc_prep   Wm[j][k][c] = fp32(ww + delta_j) widened to fp64,
//                        classes padded to 16 (one 128-B row per feature, so
//                        a wave's model row is read with wave-uniform scalar
//                        loads), bm[j][c] the biases
//   K8b k_roni_mc_count  grid (64-sample chunks, groups of 4 models): wave w
//                        runs model 4 y + w, lane l sample 64 x + l.  The
//                        chunk's samples are staged 64 features at a time in
//                        LDS, transposed ([k][sample]: a lane's reads are
//                        consecutive words); each lane runs C fp64 FMA chains
//                        over k ascending (every fp32 x fp32 product is exact
//                        in fp64), adds the bias, rounds the logits to fp32,
//                        takes np.argmax (first maximum; a NaN is the maximum)
//                        and the wave counts correct predictions (ballot).
//   K8c k_roni_mc_score  score[i] = (1 - good[i+1]/nv) - (1 - good[0]/nv)
//
// Bound: fp64 VALU (nv x (n+1) x C x D_in FMAs); the samples are re-read
// once per 4 models (L2), the models once per 64 samples (scalar cache).
constexpr int RMC_S = 64, RMC_M = 4, RMC_KC = 64, RMC_CP = 16;

__global__ __launch_bounds__(256) void k_roni_mc_prep(const double *__restrict__ ww,
                                                      const double *__restrict__ deltas, int64_t ld,
                                                      int64_t din, int C, double *__restrict__ Wm,
                                                      double *__restrict__ bm) {
    const int64_t j = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;  // k * 16 + c
    const int64_t k = e >> 4;
    const int c = (int)(e & 15);
    if (k < din) {
        double v = 0.0;  // padding classes: zero weights, never compared
        if (c < C) {
            const int64_t idx = (int64_t)c * din + k;
            v = (double)(float)(j == 0 ? ww[idx] : ww[idx] + deltas[(j - 1) * ld + idx]);
        }
        Wm[(j * din + k) * RMC_CP + c] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x < RMC_CP) {
        const int cc = (int)threadIdx.x;
        double v = 0.0;
        if (cc < C) {
            const int64_t idx = (int64_t)C * din + cc;
            v = (double)(float)(j == 0 ? ww[idx] : ww[idx] + deltas[(j - 1) * ld + idx]);
        }
        bm[j * RMC_CP + cc] = v;
    }
}

// NC: classes computed (compile time); C: classes compared (C <= NC)
template <int NC>
__global__ __launch_bounds__(256) void k_roni_mc_count(const float *__restrict__ Xv, int64_t nv,
                                                       int64_t din, int64_t ldv,
                                                       const int32_t *__restrict__ yv, int C,
                                                       const double *__restrict__ Wm,
                                                       const double *__restrict__ bm, int64_t nmod,
                                                       unsigned int *__restrict__ good) {
    __shared__ float xs[RMC_KC][RMC_S + 1];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t j = (int64_t)blockIdx.y * RMC_M + wave;
    const int64_t jj = j < nmod ? j : nmod - 1;  // an idle wave reads a real model, never counts
    const int64_t s0 = (int64_t)blockIdx.x * RMC_S;
    const double *wj = Wm + jj * din * RMC_CP;
    double acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0;
    // staging: thread t moves features (t & 3) * 16 .. + 15 of sample t >> 2
    const int ts = tid >> 2, tk = (tid & 3) * 16;
    const int64_t srow = s0 + ts < nv ? s0 + ts : nv - 1;
    const float *xrow = Xv + srow * ldv;
    for (int64_t k0 = 0; k0 < din; k0 += RMC_KC) {
        __syncthreads();  // the previous chunk has been consumed
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int64_t k = k0 + tk + u;
            xs[tk + u][ts] = k < din ? xrow[k] : 0.0f;
        }
        __syncthreads();
        const int kn = (int)(din - k0 < RMC_KC ? din - k0 : RMC_KC);
        const double *wk = wj + k0 * RMC_CP;
        for (int kk = 0; kk < kn; ++kk) {
            const double x = (double)xs[kk][lane];
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c] = __builtin_fma(x, wk[kk * RMC_CP + c], acc[c]);
        }
    }
    // logits in fp32, np.argmax: the first maximum, a NaN wins at its first place
    int best = 0;
    float bl = 0.0f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (c >= C) break;
        const float lg = (float)(acc[c] + bm[jj * RMC_CP + c]);
        if (c == 0) {
            bl = lg;
        } else if (!(bl != bl) && (lg != lg || lg > bl)) {
            best = c;
            bl = lg;
        }
    }
    const int64_t s = s0 + lane;
    const bool ok = s < nv && best == yv[s < nv ? s : nv - 1];
    const unsigned int cnt = (unsigned int)__popcll(__ballot(ok));
    if (lane == 0 && j < nmod && cnt) atomicAdd(&good[j], cnt);
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
// K8 on the matrix pipe (r3b).  The n + 1 models' logits are one GEMM:
// L[s][j C + c] = sum_k x[s][k] W_j[c][k], M = nv samples, N = (n + 1) C
// model-class columns, K = d_in.  v_mfma_f64_16x16x4_f64 rounds like four
// fp64 FMAs in k order (tools/probe_mfma_order.hip), so a chain of
// them over k ascending from +0.0 is the same fp64 sum, bit for bit, as K8's
// per-lane FMA chain -- and as the oracle's.
//
//   K8a' k_roni_mm_prep   Wt[k][j C + c] = fp32(ww + delta_j) widened, the
//                         columns padded to RMM_NT, rows to a multiple of 8;
//                         bt[col] the biases
//   K8b' k_roni_mm_logits grid (64-sample tiles, 128-column tiles), 4 waves,
//                         each 32 samples x 64 columns (2 x 4 MFMA blocks):
//                         the tile's samples staged 64 features at a time in
//                         LDS ([k][sample], row stride 80 floats: the A
//                         fragment reads hit distinct banks), the B fragments
//                         from L2 (every sample tile reads the same Wt);
//                         logit = fp32(acc + b) stored to L
//   K8c' k_roni_mm_count  wave w: model 4 y + w, lane l: sample 64 x + l: the
//                         argmax of the C logits, one ballot count per wave
// Bound: fp64 MFMA (nv x (n+1) C x d_in MACs); L is nv x ldL fp32 (24.6 MB at
// the mnist bench shape), written and read once.
constexpr int RMM_MT = 64, RMM_NT = 128, RMM_KC = 64, RMM_XS = 80;
typedef double d4 __attribute__((ext_vector_type(4)));

static inline int64_t rmm_ldl(int64_t n, int C) {
    return ((n + 1) * C + RMM_NT - 1) / RMM_NT * RMM_NT;
}
static inline int64_t rmm_rows(int64_t din) { return (din + 7) / 8 * 8; }

// softmax (K8): fp32(ww + delta_j) widened, plus the bias row `rows`;
// logistic (K7): ww + delta_j in fp64 (numpy's add), no bias
template <bool SOFTMAX>
__global__ __launch_bounds__(256) void k_roni_mm_prep(const double *__restrict__ ww,
                                                      const double *__restrict__ deltas, int64_t ld,
                                                      int64_t din, int C, int64_t nmod, int64_t rows,
                                                      int64_t ldl, double *__restrict__ Wt,
                                                      double *__restrict__ bt) {
    for (int64_t k = blockIdx.y; k < rows + (SOFTMAX ? 1 : 0); k += gridDim.y)
        for (int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x; col < ldl;
             col += (int64_t)gridDim.x * 256) {
            const int64_t j = col / C;
            const int c = (int)(col - j * C);
            const bool bias = SOFTMAX && k == rows;
            double v = 0.0;  // padding: zero weights (x * 0 adds +0 to a chain that is never -0)
            if (j < nmod && (bias || k < din)) {
                const int64_t idx = bias ? (int64_t)C * din + c : (int64_t)c * din + k;
                v = j == 0 ? ww[idx] : ww[idx] + deltas[(j - 1) * ld + idx];
                if (SOFTMAX) v = (double)(float)v;
            }
            if (bias)
                bt[col] = v;
            else
                Wt[k * ldl + col] = v;
        }
}

__global__ __launch_bounds__(256) void k_roni_mm_logits(const float *__restrict__ Xv, int64_t nv,
                                                        int64_t din, int64_t ldv,
                                                        const double *__restrict__ Wt,
                                                        const double *__restrict__ bt, int64_t ldl,
                                                        int nx, int xcd_cols, float *__restrict__ L) {
    __shared__ float xs[RMM_KC][RMM_XS];
    const int tid = threadIdx.x, l = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    // tile (x, y): with xcd_cols, column tile y lives on XCD y mod 8 (blocks
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
    const int64_t s0 = (int64_t)tx * RMM_MT;
    const int64_t c0 = (int64_t)ty * RMM_NT + 64 * wn;
    d4 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) acc[a][bb] = d4{0.0, 0.0, 0.0, 0.0};
    // staging: thread t moves features (t & 3) * 16 .. + 15 of sample t >> 2;
    // the next chunk's loads are in flight during this chunk's MFMAs
    const int ts = tid >> 2, tk = (tid & 3) * 16;
    const int64_t srow = s0 + ts < nv ? s0 + ts : nv - 1;
    const float *xrow = Xv + srow * ldv;
    const double *wcol = Wt + c0 + (l & 15) + (int64_t)(l >> 4) * ldl;
    const int arow = 32 * wm + (l & 15), ak = l >> 4;
    float xv[16];  // clamped addresses, every load in flight
#pragma unroll
    for (int u = 0; u < 16; ++u) xv[u] = xrow[tk + u < din ? tk + u : din - 1];
    for (int64_t k0 = 0; k0 < din; k0 += RMM_KC) {
        __syncthreads();  // the previous chunk has been consumed
#pragma unroll
        for (int u = 0; u < 16; ++u) xs[tk + u][ts] = k0 + tk + u < din ? xv[u] : 0.0f;
        __syncthreads();
        if (k0 + RMM_KC < din) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int64_t k = k0 + RMM_KC + tk + u;
                xv[u] = xrow[k < din ? k : din - 1];
            }
        }
        const int kn = (int)(din - k0 < RMM_KC ? din - k0 : RMM_KC);
        // k-steps in pairs (rows past d_in are zero in LDS and in Wt), the B
        // fragments of the next step loaded before this step's MFMAs, into the
        // other register set: their L2 latency runs under the MFMAs
        const int steps = ((kn + 7) >> 3) << 1;
        const double *wk = wcol + k0 * ldl;
        double b0[4], b1[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) b0[b] = wk[16 * b];
        for (int st = 0; st < steps; st += 2) {
            const int64_t o1 = (int64_t)(st + 1) * 4 * ldl;
            const int64_t o2 = (int64_t)(st + 2 < steps ? st + 2 : st + 1) * 4 * ldl;
#pragma unroll
            for (int b = 0; b < 4; ++b) b1[b] = wk[o1 + 16 * b];
            double a0 = (double)xs[4 * st + ak][arow];
            double a1 = (double)xs[4 * st + ak][arow + 16];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                acc[0][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0[b], acc[0][b], 0, 0, 0);
                acc[1][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0[b], acc[1][b], 0, 0, 0);
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) b0[b] = wk[o2 + 16 * b];
            a0 = (double)xs[4 * st + 4 + ak][arow];
            a1 = (double)xs[4 * st + 4 + ak][arow + 16];
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
        const int64_t col = c0 + 16 * b + (l & 15);
        const double bias = bt[col];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t s = s0 + 32 * wm + 16 * a + (l >> 4) + 4 * r;
                if (s < nv) L[s * ldl + col] = (float)(acc[a][b][r] + bias);
            }
    }
}

__global__ __launch_bounds__(256) void k_roni_mm_count(const float *__restrict__ L, int64_t nv,
                                                       int64_t ldl, const int32_t *__restrict__ yv,
                                                       int C, int64_t nmod,
                                                       unsigned int *__restrict__ good) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t j = (int64_t)blockIdx.y * 4 + (tid >> 6);
    const int64_t s = (int64_t)blockIdx.x * 64 + lane;
    if (j >= nmod) return;  // wave-uniform
    const int64_t sr = s < nv ? s : nv - 1;
    const float *lg = L + sr * ldl + j * C;
    // np.argmax: the first maximum, a NaN wins at its first place
    int best = 0;
    float bl = lg[0];
    for (int c = 1; c < C; ++c) {
        const float v = lg[c];
        if (!(bl != bl) && (v != v || v > bl)) {
            best = c;
            bl = v;
        }
    }
    const bool ok = s < nv && best == yv[sr];
    const unsigned int cnt = (unsigned int)__popcll(__ballot(ok));
    if (lane == 0 && cnt) atomicAdd(&good[j], cnt);
}

size_t roni_softmax_ws(int64_t n, int64_t din, int64_t nv, int C) {
    const int64_t ldl = rmm_ldl(n, C);
    const size_t mm = (size_t)(rmm_rows(din) + 1) * ldl * sizeof(double) +
                      (size_t)nv * ldl * sizeof(float);
    const size_t mc = (size_t)(n + 1) * ((size_t)din * RMC_CP + RMC_CP) * sizeof(double);
    return mm > mc ? mm : mc;
}

static hipError_t launch_roni_softmax_mm(const float *Xv, int64_t nv, int64_t din, int64_t ldv,
                                         const int32_t *yv, int C, const double *ww,
                                         const double *deltas, int64_t n, int64_t ld, double *ws,
                                         unsigned int *good, double *scores, hipStream_t st) {
    const int64_t nmod = n + 1, ldl = rmm_ldl(n, C), rows = rmm_rows(din);
    double *Wt = ws, *bt = ws + rows * ldl;
    float *L = (float *)(bt + ldl);
    hipError_t e = hipMemsetAsync(good, 0, (size_t)nmod * sizeof(unsigned int), st);
    if (e != hipSuccess) return e;
    const unsigned gx = (unsigned)((ldl + 255) / 256 < 64 ? (ldl + 255) / 256 : 64);
    const unsigned gy = (unsigned)(rows + 1 < 8192 ? rows + 1 : 8192);
    hipLaunchKernelGGL(k_roni_mm_prep<true>, dim3(gx, gy), dim3(256), 0, st, ww, deltas, ld, din, C, nmod,
                       rows, ldl, Wt, bt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int nx = (int)((nv + RMM_MT - 1) / RMM_MT), ny = (int)(ldl / RMM_NT);
    hipLaunchKernelGGL(k_roni_mm_logits, dim3((unsigned)(nx * ny)), dim3(256), 0, st, Xv, nv, din,
                       ldv, Wt, bt, ldl, nx, ny % 8 == 0 ? 1 : 0, L);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_mm_count, dim3((unsigned)((nv + 63) / 64), (unsigned)((nmod + 3) / 4)),
                       dim3(256), 0, st, L, nv, ldl, yv, C, nmod, good);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_mc_score, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, good,
                       n, nv, scores);
    return hipGetLastError();
}

hipError_t launch_roni_softmax(const float *Xv, int64_t nv, int64_t din, int64_t ldv,
                               const int32_t *yv, int C, const double *ww, const double *deltas,
                               int64_t n, int64_t ld, double *ws, unsigned int *good,
                               double *scores, hipStream_t st) {
    if (!roni_valu())
        return launch_roni_softmax_mm(Xv, nv, din, ldv, yv, C, ww, deltas, n, ld, ws, good, scores,
                                      st);
    const int64_t nmod = n + 1;
    double *Wm = ws, *bm = ws + (size_t)nmod * din * RMC_CP;
    hipError_t e = hipMemsetAsync(good, 0, (size_t)nmod * sizeof(unsigned int), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_mc_prep, dim3((unsigned)((din * RMC_CP + 255) / 256), (unsigned)nmod),
                       dim3(256), 0, st, ww, deltas, ld, din, C, Wm, bm);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const dim3 grid((unsigned)((nv + RMC_S - 1) / RMC_S), (unsigned)((nmod + RMC_M - 1) / RMC_M));
    if (C == 2)
        hipLaunchKernelGGL(k_roni_mc_count<2>, grid, dim3(256), 0, st, Xv, nv, din, ldv, yv, C, Wm, bm, nmod, good);
    else if (C == 10)
        hipLaunchKernelGGL(k_roni_mc_count<10>, grid, dim3(256), 0, st, Xv, nv, din, ldv, yv, C, Wm, bm, nmod, good);
    else if (C == 12)
        hipLaunchKernelGGL(k_roni_mc_count<12>, grid, dim3(256), 0, st, Xv, nv, din, ldv, yv, C, Wm, bm, nmod, good);
    else
        hipLaunchKernelGGL(k_roni_mc_count<RMC_CP>, grid, dim3(256), 0, st, Xv, nv, din, ldv, yv, C, Wm, bm, nmod, good);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_mc_score, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, good,
                       n, nv, scores);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K7 on the matrix pipe (r3b): S[s][j] = x_s . w_j as one GEMM (M = nv
// samples, N = n + 1 models, K = d), a chain of v_mfma_f64_16x16x4_f64 over k
// ascending from +0.0 -- the same fp64 FMA chain as K7's VALU kernel and the
// oracle, bit for bit -- and the sign test fused into the epilogue: each lane
// counts the mismatches of its column over its rows, two lane butterflies sum
// a column's 16 lanes, one atomic per model and wave.  A workgroup walks
// RSG_T sample tiles of 64 (the counts stay in registers), 4 waves of 32
// samples x 64 models.  The validation rows are staged 32 features at a time
// in LDS ([k][sample] fp64, row stride 80: the A fragment reads hit distinct
// banks), the models come from L2.  No cap on d (K7's LDS model held d <= 1024).
constexpr int RSG_T = 8, RSG_KC = 32, RSG_XS = 80;

__global__ __launch_bounds__(256) void k_roni_mm_sign(const double *__restrict__ Xv, int64_t nv,
                                                      int64_t d, int64_t ldv,
                                                      const double *__restrict__ yv,
                                                      const double *__restrict__ Wt, int64_t ldl,
                                                      int64_t nmod, unsigned int *__restrict__ cnt) {
    __shared__ double xs[RSG_KC][RSG_XS];
    const int tid = threadIdx.x, l = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const int64_t c0 = (int64_t)blockIdx.y * RMM_NT + 64 * wn;
    const double *wcol = Wt + c0 + (l & 15) + (int64_t)(l >> 4) * ldl;
    const int arow = 32 * wm + (l & 15), ak = l >> 4;
    const int ts = tid >> 2, tk = (tid & 3) * 8;  // staging: 8 features of one sample
    unsigned int mis[4] = {0, 0, 0, 0};
    for (int t = 0; t < RSG_T; ++t) {
        const int64_t s0 = ((int64_t)blockIdx.x * RSG_T + t) * 64;
        if (s0 >= nv) break;  // uniform
        d4 acc[2][4];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
        const int64_t srow = s0 + ts < nv ? s0 + ts : nv - 1;
        const double *xrow = Xv + srow * ldv;
        for (int64_t k0 = 0; k0 < d; k0 += RSG_KC) {
            __syncthreads();  // the previous chunk (or tile) has been consumed
            double xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t k = k0 + tk + u;
                xv[u] = xrow[k < d ? k : d - 1];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) xs[tk + u][ts] = k0 + tk + u < d ? xv[u] : 0.0;
            __syncthreads();
            const int kn = (int)(d - k0 < RSG_KC ? d - k0 : RSG_KC);
            const int steps = ((kn + 7) >> 3) << 1;
            const double *wk = wcol + k0 * ldl;
            double b0[4], b1[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) b0[b] = wk[16 * b];
            for (int st = 0; st < steps; st += 2) {
                const int64_t o1 = (int64_t)(st + 1) * 4 * ldl;
                const int64_t o2 = (int64_t)(st + 2 < steps ? st + 2 : st + 1) * 4 * ldl;
#pragma unroll
                for (int b = 0; b < 4; ++b) b1[b] = wk[o1 + 16 * b];
                double a0 = xs[4 * st + ak][arow], a1 = xs[4 * st + ak][arow + 16];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    acc[0][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0[b], acc[0][b], 0, 0, 0);
                    acc[1][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0[b], acc[1][b], 0, 0, 0);
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) b0[b] = wk[o2 + 16 * b];
                a0 = xs[4 * st + 4 + ak][arow];
                a1 = xs[4 * st + 4 + ak][arow + 16];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    acc[0][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1[b], acc[0][b], 0, 0, 0);
                    acc[1][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1[b], acc[1][b], 0, 0, 0);
                }
            }
        }
        // D reg r of lane l: sample row (l >> 4) + 4 r of the block, model column l & 15
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t s = s0 + 32 * wm + 16 * a + (l >> 4) + 4 * r;
                const double y = yv[s < nv ? s : nv - 1];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const double v = acc[a][b][r];  // np.sign: 0 -> 0, NaN -> NaN
                    const double yh = v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : (v == 0.0 ? 0.0 : v));
                    mis[b] += (s < nv && !(yh == y)) ? 1u : 0u;
                }
            }
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        unsigned int tot = mis[b];
        tot += __shfl_xor(tot, 16);
        tot += __shfl_xor(tot, 32);
        const int64_t j = c0 + 16 * b + l;
        if (l < 16 && tot && j < nmod) atomicAdd(&cnt[j], tot);
    }
}

size_t roni_ws(int64_t n, int64_t d) {
    return (size_t)rmm_rows(d) * ((n + 1 + RMM_NT - 1) / RMM_NT * RMM_NT) * sizeof(double);
}

hipError_t launch_roni(const double *Xv, int64_t nv, int64_t d, int64_t ldv, const double *yv,
                       const double *ww, const double *deltas, int64_t n, int64_t ld,
                       double *ws, unsigned int *cnt, double *scores, hipStream_t st) {
    if (roni_valu() && d <= 1024)
        return launch_roni_valu(Xv, nv, d, ldv, yv, ww, deltas, n, ld, cnt, scores, st);
    const int64_t nmod = n + 1, ldl = (nmod + RMM_NT - 1) / RMM_NT * RMM_NT, rows = rmm_rows(d);
    hipError_t e = hipMemsetAsync(cnt, 0, (size_t)nmod * sizeof(unsigned int), st);
    if (e != hipSuccess) return e;
    const unsigned gx = (unsigned)((ldl + 255) / 256 < 64 ? (ldl + 255) / 256 : 64);
    const unsigned gy = (unsigned)(rows < 8192 ? rows : 8192);
    hipLaunchKernelGGL(k_roni_mm_prep<false>, dim3(gx, gy), dim3(256), 0, st, ww, deltas, ld, d, 1,
                       nmod, rows, ldl, ws, (double *)nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int64_t tiles = (nv + 64 * RSG_T - 1) / (64 * RSG_T);
    hipLaunchKernelGGL(k_roni_mm_sign, dim3((unsigned)tiles, (unsigned)(ldl / RMM_NT)), dim3(256), 0,
                       st, Xv, nv, d, ldv, yv, ws, ldl, nmod, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_roni_score, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cnt, n,
                       nv, scores);
    return hipGetLastError();
}

}  // namespace bk
