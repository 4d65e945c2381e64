/*
 * bk.h -- C ABI of the MI355X-native Multi-Krum engine (libbk.so).
 *
 * Drop-in boundary for Biscotti's verifier hot path.  The reference path is
 *
 *   Peer.VerifyUpdateKRUM          DistSys/krum.go:227-365
 *    -> KRUMValidator.computeScores  DistSys/krum.go:77-98
 *     -> KRUMValidator.getTopKRUMIndex(deltas [][]float64) []int
 *                                    DistSys/krum.go:100-166   <-- replaced
 *        (go-python: marshal n*d PyFloats, call numpy krum(deltas, clip),
 *         decode the int64 index bytes)
 *         -> krum(deltas, clip)      ML/code/logistic_validator.py:36-49
 *         -> get_krum_scores(X, g)   ML/code/logistic_validator.py:54-65
 *         (aggregate: np.mean(deltas[good_idx], 0), logistic_validator.py:51)
 *
 * A cgo shim with the same Go signature as getTopKRUMIndex calls bk_multikrum
 * (see INTEGRATION.md).  Plain pointers and sizes only; no torch, no HIP types.
 *
 * Conventions
 *   X        row-major n x d with leading dimension ld (elements), fp64 or fp32
 *            (fp32 is widened exactly; every accumulation is fp64).
 *   f        number of updates to reject ("clip"; krum.go:110 computes
 *            int(0.5*n)).  Valid iff 1 <= f < n (f = 0 makes the reference's
 *            np.argpartition raise ValueError, logistic_validator.py:45).
 *   m = n-f  number selected; k = max(0, n-f-2) neighbours summed per score.
 *   sel_idx  the m selected row indices, ASCENDING (a set: the only consumer,
 *            checkIfAccepted krum.go:47-73, tests membership).  Ties at the
 *            selection boundary resolve to the lower index; NaN scores order
 *            last (as numpy's sort/argpartition do).
 *   mean     (1/m) * sum of selected rows (fp64), the north-star aggregate.
 *
 * Errors: every entry returns 0 (BK_OK) or a negative bk_status; the message
 * is in bk_last_error() (thread-local).  Nothing aborts or throws across the
 * ABI.  Calls on one context are serialised internally; each entry selects the
 * context's device itself (goroutines migrate between OS threads).
 */
#ifndef BK_H_
#define BK_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BK_ABI_VERSION 14

typedef struct bk_ctx bk_ctx;

enum bk_status {
    BK_OK = 0,
    BK_EINVAL = -1,  /* bad n, d, f, ld, dtype, pointer or mode             */
    BK_ENOMEM = -2,  /* device / pinned allocation failed                    */
    BK_EHIP = -3,    /* a HIP runtime call failed                            */
    BK_ERCCL = -4,   /* an RCCL call failed / communicator missing          */
    BK_ENOTSUP = -5  /* shape outside what this build supports (n > BK_MAX_N) */
};

enum bk_dtype { BK_F64 = 0, BK_F32 = 1 };
enum bk_where { BK_HOST = 0, BK_HOST_PINNED = 1, BK_DEVICE = 2 };

#define BK_MAX_N 16384

/* ---- library ------------------------------------------------------------ */
int bk_abi_version(void);
const char *bk_last_error(void);
/* Argument check only (no GPU needed): BK_OK or BK_EINVAL / BK_ENOTSUP. */
int bk_check_args(int64_t n, int64_t d, int64_t f);

/* ---- context: replaces KRUMValidator.initialize() (krum.go:31-44), which
 *      bound pyKRUMFunc from the module imported in pyInit (honest.go:204-258) */
int bk_create(bk_ctx **out, int device);
void bk_destroy(bk_ctx *ctx);
/* Run on a caller stream (hipStream_t passed as void*); NULL = own stream. */
int bk_set_stream(bk_ctx *ctx, void *hip_stream);
void *bk_get_stream(bk_ctx *ctx);
/* Waits for the context stream (polling it for up to BK_SPIN_US, default
 * 2000 us, then blocking), then reports whether the last Multi-Krum call
 * on it produced valid outputs: BK_EHIP when k_small's hand-off wait gave up
 * (its sel entries are then -1), BK_ERCCL when a rank of a sharded call failed
 * before the exchange (bk_multikrum_sharded_device).  The asynchronous device
 * entries report these only here and through bk_selection_margin*. */
int bk_synchronize(bk_ctx *ctx);
/* C-owned pinned staging for callers that must copy (cgo: Go pointers may not
 * be retained by C, so the shim packs [][]float64 rows here). */
int bk_stage_alloc(bk_ctx *ctx, int64_t bytes, void **pinned);
int bk_stage_free(bk_ctx *ctx, void *pinned);

/* ---- the drop-in: getTopKRUMIndex (krum.go:100-166) + numpy krum ---------
 * X on host (BK_HOST / BK_HOST_PINNED: copied H2D) or device (BK_DEVICE).
 * Biscotti's deployed shapes (n <= 128, d <= 32768: the mnist and creditcard
 * verifiers, configs A and B) cross PCIe as ONE copy and run the one-launch
 * path (k_small / k_tiny, see bk_set_small_path); a BK_HOST_PINNED batch that
 * k_tiny takes whole (n <= 16, d <= 128) is not copied at all: the kernel
 * reads it over PCIe during the (synchronous) call.  A larger host batch crosses
 * PCIe in column chunks (BK_STAGE_CHUNK_BYTES, default 256 MiB) on a copy
 * stream while the previous chunk's partial Gram runs; the chunk partials are
 * summed in chunk order, so results are deterministic.
 * Outputs are HOST pointers: sel_idx (m entries), m_out, scores (n, nullable),
 * mean_out (d, nullable).  Synchronous; an invalid call (see bk_synchronize)
 * returns its error here. */
int bk_multikrum(bk_ctx *ctx, const void *X, int where, int dtype, int64_t n, int64_t d,
                 int64_t ld, int64_t f, int64_t *sel_idx, int64_t *m_out, double *scores,
                 double *mean_out);

/* The verifier's own input: n SEPARATE host rows (getTopKRUMIndex(deltas
 * [][]float64), krum.go:100-166 -- one slice per peer, as RPC decoded them,
 * replacing the shim's serial pack of the rows into a pinned batch,
 * krum.go:117-125's marshalling loop in the reference).  rows[i] points at
 * update i's d elements (dtype; pageable or pinned host memory, any
 * alignment); the rows are only read, during the call.  libbk packs them on
 * host threads (bk_set_host_threads) into a ring of C-owned pinned slots,
 * column chunk by column chunk, and each chunk's H2D and partial Gram start
 * as soon as it is packed.  Outputs and contract as bk_multikrum (host
 * outputs, synchronous); the selection and the mean are bitwise those of
 * bk_multikrum(BK_HOST_PINNED) on the same rows packed row-major.
 * cgo: the row pointers are Go pointers stored in C memory, which Go >= 1.21
 * allows while each row's backing array is pinned (runtime.Pinner) for the
 * call (go/bk/krum_bk.go).  A null row is BK_EINVAL. */
int bk_multikrum_rows(bk_ctx *ctx, const void *const *rows, int dtype, int64_t n, int64_t d,
                      int64_t f, int64_t *sel_idx, int64_t *m_out, double *scores,
                      double *mean_out);
/* Host threads that pack bk_multikrum_rows' rows, the caller's included (1:
 * the caller alone; 0: the default, BK_HOST_THREADS or min(8, hardware
 * threads)).  The workers are started on the next call and sleep between
 * calls. */
int bk_set_host_threads(bk_ctx *ctx, int threads);

/* Device-resident, asynchronous on the context stream.  All pointers are
 * device pointers; d_sel_idx gets m = n-f ascending indices; d_scores (n) and
 * d_mean (d) are nullable.  A failure inside the kernels (k_small's hand-off
 * timeout) cannot be returned here: bk_synchronize and bk_selection_margin*
 * report it, and every d_sel_idx entry is -1. */
int bk_multikrum_device(bk_ctx *ctx, const void *dX, int dtype, int64_t n, int64_t d,
                        int64_t ld, int64_t f, int64_t *d_sel_idx, double *d_scores,
                        double *d_mean);
/* Small batches (n <= 128, d <= 32768: Biscotti's deployed shapes, configs A
 * and B) run as ONE launch,
 * k_small: split-K Gram, reduce, scores, selection and mean pulled as work
 * items from a queue in dependency order (no co-residency assumed).  The same
 * results as the general path: selection, and the mean bitwise; scores within
 * rounding (another split of the Gram).  on = 0 forces the general path. */
int bk_set_small_path(bk_ctx *ctx, int on);
/* Replay bk_multikrum_device as a hipGraph (one captured launch sequence per
 * call signature: pointers, shape, f; up to 4 cached).  The first call of a
 * signature runs eagerly, the second captures, later ones replay; graphs are
 * bypassed while per-kernel timing is on, and retired when the context's
 * workspace is reallocated.  Off by default; on = 0 frees the cached graphs. */
int bk_graph_enable(bk_ctx *ctx, int on);

/* fp32 rows (dtype BK_F32): BK_F32_EXACT (default) widens every element onto
 * the fp64 MFMA, which is exact per product and accumulates in fp64.
 * BK_F32_MFMA (BASELINE config E's "fp32 MFMA path") runs
 * v_mfma_f32_16x16x4_f32 at twice the fp64 rate: products are rounded to fp32
 * and summed in fp32 within one K1 workgroup segment, and the segments'
 * partials are summed in fp64.  Tolerance, as SURVEY.md §8(d) restates it for
 * config E: the selection matches wherever the score gap at the boundary
 * exceeds the fp32 Gram error bound (~2 k gamma_d max|x_i|^2).  The mean is
 * unchanged (fp64 accumulation of the fp32 rows).  No effect on fp64 rows. */
enum bk_f32_mode {
    BK_F32_EXACT = 0,
    BK_F32_MFMA = 1,
    BK_F32_CERTIFIED = 2,
    BK_F32_I8 = 3,
    BK_F32_I8_CERTIFIED = 4,
    BK_F32_I8X2 = 5,
    BK_F32_I8X2_CERTIFIED = 6
};
/* BK_F32_I8: the Gram from exact int8 digit slices on v_mfma_i32_32x32x32_i8
 * (bk_i8.hip, K1i8; the Ozaki scheme).  Per range of columns (at least 8,
 * each row's slice <= 128 KiB) every row is scaled by a power of two >= its max |x| and cut into three
 * signed 7-bit digits; the six digit products of weight >= 2^-26 accumulate
 * exactly in int32 and combine exactly in fp64, so each range's partial is
 * exact for the truncated digits and the result deterministic.  The dropped
 * digits bound every Gram element's error ABSOLUTELY by
 *     sum_r 2^-21 (2 S_r L1_r + 2.03 d_r S_r^2)
 * (S_r the largest row scale, L1_r the largest ||x_i||_1 of range r, d_r its
 * columns), carried in the packed record and added to the selection margin's
 * bound: a selection that differs from the reference's comes with near_tie = 1.
 * Far tighter than the fp32 MFMA's gamma_d (config E: ~1e-4 against ~1.6e-2 of
 * max |x_i|^2) and several times faster.  Rows must be 16-B aligned (ld % 4 ==
 * 0, aligned base) and d >= 64; other batches take the exact path.  A
 * non-finite input makes the bound +inf (a near tie). */
/* BK_F32_I8X2: the same slicing with TWO digits (x / s = a0/64 + a1/2^13 +
 * rho, |rho| <= 2^-14) and the three digit products of weight >= 2^-19 (A0
 * A0^T, A0 A1^T, A1 A0^T) on 128 x 256 output tiles: half the products and
 * two thirds of the digit bytes of BK_F32_I8, under the absolute bound
 *     sum_r 2^-14 (2 S_r L1_r + 1.0001 d_r S_r^2)
 * (~2^7 looser than BK_F32_I8's; config E: still ~20x below its boundary
 * gap).  BK_F32_I8X2_CERTIFIED re-runs a near tie exact. */
/* BK_F32_CERTIFIED: the fp32 MFMA, then -- only when the selection margin
 * (bk_selection_margin) does not clear the fp32 bound -- the exact path on the
 * same device-resident batch, whose outputs replace the first run's.  Never
 * silently different from the reference where the exact path is not; the
 * entries become synchronous (the decision reads the margin on the host).
 * Only a Gram taken on the fp32 MFMA is re-run (the n <= 128 one-launch path
 * is always exact).  bk_group_multikrum honours it when it is set on the
 * group's contexts (bk_group_ctx): a near tie re-runs every device's shard
 * exact from device memory, then exchanges and finishes again. */
int bk_set_f32_mode(bk_ctx *ctx, int mode);
/* fp64 rows (dtype BK_F64): BK_F64_EXACT (default) runs the fp64 MFMA;
 * BK_F64_I8 takes the Gram from the same exact int8 digit slices as BK_F32_I8
 * (the digits of an fp64 row: every slicing step exact, only the remainder
 * past the third digit dropped) under the same absolute error bound;
 * BK_F64_I8_CERTIFIED re-runs the fp64 MFMA on a near tie, so its selected
 * set is always the reference's.  The mean is unchanged (K4 reads the fp64
 * rows).  Rows must be 16-B aligned (even ld) and d >= 64. */
enum bk_f64_mode {
    BK_F64_EXACT = 0,
    BK_F64_I8 = 3,
    BK_F64_I8_CERTIFIED = 4,
    BK_F64_I8X2 = 5,          /* the two-digit slicing of BK_F32_I8X2 on fp64 rows */
    BK_F64_I8X2_CERTIFIED = 6
};
int bk_set_f64_mode(bk_ctx *ctx, int mode);
/* BK_F32_I8_CERTIFIED: the same contract on the int8-sliced Gram.
 * exact re-runs BK_F32_CERTIFIED / BK_F32_I8_CERTIFIED have made on this context */
int64_t bk_certified_reruns(bk_ctx *ctx);

/* ---- selection margin: where the selection may legitimately differ from the
 * reference's (SURVEY.md §7 "Hard parts", §8(d); logistic_validator.py:45,
 * 59-63: argpartition over BLAS-rounded scores).  Every Multi-Krum call
 * (any entry) leaves on its context, computed on the device by the finish:
 *   gap       = s[rank m] - s[rank m-1], the lowest rejected score minus the
 *               highest selected one (+inf across a finite -> NaN boundary)
 *   err_bound = 2 (e_here + e_ref),  e = 4 k M' (gamma_{d+2}(u_G) + 2u + gamma_k(u))
 *               with M' >= max_i ||x_i||^2 (finite rows), u = 2^-53, u_G the
 *               Gram's unit roundoff here (2^-53, or 2^-24 once any of its
 *               columns ran on the fp32 MFMA), gamma_j(u) = j u / (1 - j u),
 *               d the Gram's total column count (after a multi-GPU exchange
 *               too; both come from the packed record's trailing pair), k =
 *               n - f - 2
 *   near_tie  = !(gap > err_bound); a record without a column count (d < 1,
 *               e.g. a caller's own packed Gram) has err_bound = +inf and
 *               near_tie = 1
 * Any fp64 computation of the reference formula in any summation order --
 * numpy's BLAS included -- gives scores within e of the exact ones, so when
 * near_tie = 0 the reference provably selects exactly sel_idx.  near_tie = 1
 * means the boundary is within rounding (or an exact tie, e.g. k = 0 where every
 * score is 0): the lower-index tie rule decided, and numpy's choice may differ.
 * Reads the record of the last call (synchronizes the context stream); returns
 * the errors bk_synchronize does when that call's outputs are invalid. */
int bk_selection_margin(bk_ctx *ctx, double *gap, double *err_bound, int *near_tie);
/* the whole record: {gap, err_bound, near_tie, M, s_lo, s_hi, d, k} (8 doubles) */
int bk_selection_margin_record(bk_ctx *ctx, double *record);

/* ---- dimension-sharded stages (one process / device per column shard) ----
 * Packed upper-triangle Gram: bk_upper_elems(n) doubles = the 64x64 upper
 * sub-tiles, then a trailing pair: the column count, and how many of those
 * columns were accumulated on the fp32 MFMA.  Summing the packed partials of
 * all shards (trailing pairs included) gives the Gram of the full batch, its
 * total d and its unit roundoff, which the selection margin uses. */
int64_t bk_upper_elems(int64_t n);
/* On failure d_upper's trailing pair is set to NaN (best effort): a caller
 * that still joins its exchange, so its peers are not left waiting, hands
 * every rank a record that bk_finish_device marks invalid (BK_ERCCL from
 * bk_synchronize / bk_selection_margin*). */
int bk_gram_upper_device(bk_ctx *ctx, const void *dX, int dtype, int64_t n, int64_t d,
                         int64_t ld, double *d_upper);
/* Scores + selection from a (summed) packed Gram, then the mean of this
 * shard's d columns of dX (d_mean nullable). */
int bk_finish_device(bk_ctx *ctx, const double *d_upper, const void *dX, int dtype, int64_t n,
                     int64_t d, int64_t ld, int64_t f, int64_t *d_sel_idx, double *d_scores,
                     double *d_mean);

/* ---- RCCL (one rank per process, xGMI) ------------------------------------ */
#define BK_UNIQUE_ID_BYTES 128
int bk_comm_unique_id(void *id_out /* BK_UNIQUE_ID_BYTES */);
int bk_comm_init(bk_ctx *ctx, int nranks, int rank, const void *id /* BK_UNIQUE_ID_BYTES */);
/* 0: ncclAllReduce(sum) of the packed Gram (default);
 * 1: deterministic -- ncclAllGather of the partials + fixed rank-order sum;
 * 2: the all-reduce overlapped with the Gram -- the packed upper cut into
 *    pieces by rows (BK_OVERLAP_PIECES, 2..8, default 2, each ~0.6 of the one
 *    before), each piece computed by its own launches and all-reduced on a
 *    communication stream while the next computes.  Every output is bitwise
 *    mode 0's (the pieces run the same segments / (tile, range) items; the
 *    sum is element-wise).  Applies where the Gram splits into such pieces
 *    (K1i8, and the K1 plans whose workgroups each stay in one piece: n >=
 *    ~2048, config E); elsewhere (config D's n = 512 plan) mode 0 runs.
 * Set on every rank alike. */
int bk_comm_set_mode(bk_ctx *ctx, int mode);
/* Partial Gram of the local column shard -> all-reduce -> scores/selection
 * (redundant on every rank) -> mean of the local columns.  Async on stream. */
/* d_local = 0 is allowed (an empty trailing shard: dX_local, ld and
 * d_mean_local unused); the rank still joins the exchange.
 * No rank strands its peers in the collective: the first call of a signature
 * (n, f, dtype, exchange mode) allocates the workspace and agrees on a status
 * word (one extra 8-B all-reduce and a host wait), so an allocation failure
 * is an error on every rank (BK_ERCCL on the peers); a later failure before
 * the exchange poisons the rank's partial and the rank still joins, so every
 * rank's bk_synchronize reports BK_ERCCL and the failing rank returns its own
 * error. */
int bk_multikrum_sharded_device(bk_ctx *ctx, const void *dX_local, int dtype, int64_t n,
                                int64_t d_local, int64_t ld, int64_t f, int64_t *d_sel_idx,
                                double *d_scores, double *d_mean_local);
/* the communicator's size and this rank (ncclCommCount / ncclCommUserRank);
 * nranks = 0 when bk_comm_init was not called */
int bk_comm_size(bk_ctx *ctx, int *nranks, int *rank);
/* exchanges of the packed Gram made on this context, and the bytes this rank
 * put into them (all-reduce: bk_upper_elems(n) * 8 each; all-gather: x nranks) */
int bk_comm_stats(bk_ctx *ctx, int64_t *exchanges, double *bytes);

/* ---- one process, G GPUs: the Go verifier's form ------
 * A verifier is ONE process holding [][]float64 in host memory
 * (VerifyUpdateKRUM, krum.go:227-365).  A group owns one context per device
 * and splits the columns like bk_multikrum_sharded_device: each device copies
 * its column shard over its own PCIe link, computes its partial Gram, the
 * partials are summed, every device scores and selects (identically) and
 * writes the mean of its columns into mean_out.
 *   mode BK_GROUP_ALLREDUCE:  ncclAllReduce over one communicator
 *                             (ncclCommInitAll), devices must be distinct;
 *   BK_GROUP_DETERMINISTIC:   ncclAllGather + fixed rank-order sum;
 *   BK_GROUP_HOST_EXCHANGE:   partials through pinned host memory, summed in
 *                             fixed rank order -- no RCCL; any device list,
 *                             repeats allowed (bitwise equal to DETERMINISTIC).
 * devices may be NULL (0..ngpus-1). */
typedef struct bk_group bk_group;
enum bk_group_mode { BK_GROUP_ALLREDUCE = 0, BK_GROUP_DETERMINISTIC = 1, BK_GROUP_HOST_EXCHANGE = 2 };
int bk_group_create(bk_group **out, int ngpus, const int *devices, int mode);
void bk_group_destroy(bk_group *g);
int bk_group_size(const bk_group *g);
/* bk_multikrum's contract (host X: BK_HOST or BK_HOST_PINNED; host outputs;
 * synchronous) over the group's devices.  shard_bounds: GPU r owns columns
 * [r*per, min(d, (r+1)*per)), per = ceil(d/G) rounded up to 8. */
int bk_group_multikrum(bk_group *g, const void *X, int where, int dtype, int64_t n, int64_t d,
                       int64_t ld, int64_t f, int64_t *sel_idx, int64_t *m_out, double *scores,
                       double *mean_out);
/* per-device context (timing, streams); r in [0, G) */
bk_ctx *bk_group_ctx(bk_group *g, int r);

/* ---- synthetic batches (spec: DESIGN.md "Synthetic inputs") --------------
 * Rows [0,n) x columns [c0, c0+d_local) of the n x d_total batch, generated on
 * the device bit-identically to oracle/krum_oracle.c and the numpy spec. */
#define BK_SYNTH_FP32ROUND 1
int bk_synth_fill_device(bk_ctx *ctx, void *dX, int dtype, int64_t n, int64_t d_local,
                         int64_t ld, int64_t c0, int64_t d_total, uint64_t seed, int64_t nbyz,
                         double mu_scale, double byz_scale, double sigma, int flags);

/* ---- the steps either side of Multi-Krum --- */

/* Block aggregation of the accepted updates -- replaces the update loop of
 * Honest.createBlock, DistSys/honest.go:360-375 (pulledGradientM.Add per
 * accepted update, in blockUpdates order):
 *     for r = 0 .. m-1:  global[c] = global[c] + X[idx[r]][c]
 * sequential fp64 adds in idx order, bit-identical to the Go loop.  idx lists
 * the accepted rows in the caller's update order (duplicates allowed); m = 0
 * leaves global unchanged.  The stake bookkeeping (+-STAKE_UNIT) stays above
 * the boundary.  Device variant: d_idx entries must lie in [0, n) (not checked
 * on the device); m <= BK_MAX_N. */
int bk_aggregate_device(bk_ctx *ctx, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld,
                        const int64_t *d_idx, int64_t m, double *d_global);
/* Host-buffer variant for the Go miner: X as in bk_multikrum (where), idx and
 * global (in/out, d entries) in host memory; idx is range-checked (BK_EINVAL). */
int bk_aggregate(bk_ctx *ctx, const void *X, int where, int dtype, int64_t n, int64_t d,
                 int64_t ld, const int64_t *idx, int64_t m, double *global);

/* Secure-aggregation quantised sum -- updateFloatToInt (DistSys/kyber.go:698-710)
 * of each accepted update, summed as the miners' share aggregation does before
 * recovery (honest.go:401-409, 442-502), and updateIntToFloat (kyber.go:745-757):
 *     d_sum[c]       = sum_r int64(X[idx[r]][c] * 10^precision)   (int64, wrapping)
 *     d_sum_float[c] = float64(d_sum[c]) / 10^precision           (nullable)
 * int64(float64) follows Go on amd64: truncation toward zero, NaN and
 * out-of-range values give INT64_MIN.  0 <= precision <= 18 (Biscotti uses
 * PRECISION = 4, main.go:45). */
int bk_quantized_sum_device(bk_ctx *ctx, const void *dX, int dtype, int64_t n, int64_t d,
                            int64_t ld, const int64_t *d_idx, int64_t m, int precision,
                            int64_t *d_sum, double *d_sum_float);

/* Noise application (client DP step) -- requestNoiseFromNoisers
 * (DistSys/main.go:1606-1653: noiseVec = 0 + v_0 + ... + v_{k-1}, then
 * /= float64(k)) and NoisedDelta = Delta + noise (main.go:1524-1537), batched
 * over n updates:
 *     out[i][c] = delta[i][c] + ((0 + noise[i][0][c]) + ... + noise[i][k-1][c]) / k
 * noise vector j of update i starts at d_noise + (i*k + j) * noise_ld.  out may
 * alias delta (out_ld == ld).  k = 0 gives NaN (0/0), as the Go code does. */
int bk_noise_apply_device(bk_ctx *ctx, const double *d_delta, int64_t n, int64_t d, int64_t ld,
                          const double *d_noise, int64_t k, int64_t noise_ld, double *d_out,
                          int64_t out_ld);

/* Noise application fused into the verifier's H2D staging (SURVEY.md §8(f)
 * row 3), then the drop-in Multi-Krum of bk_multikrum on the noised batch.
 * Replaces the host pass NoisedDelta = Delta + noise (main.go:1524-1537,
 * 1606-1653) that precedes getTopKRUMIndex (krum.go:100-166) when the batch is
 * noised where it is verified.  delta: host n x d (row stride ld); noise: host,
 * vector j of update i at noise + (i*k + j) * noise_ld.  Column chunks cross
 * PCIe on a copy stream while K6 noises, and K1 takes the partial Gram of, the
 * previous chunk on the context stream (as bk_multikrum's host path).
 * k = 0 means no noisers: NoisedDelta = Delta (main.go:1599-1602; unlike
 * bk_noise_apply_device, whose k = 0 is the literal 0/0).  where is BK_HOST or
 * BK_HOST_PINNED (pinned memory overlaps; pageable copies are staged by HIP).
 * Outputs as bk_multikrum, plus noised_out (nullable, host n x d, row stride
 * out_ld): the noised batch, bit-identical to bk_noise_apply_device.
 * Synchronous. */
int bk_multikrum_noised(bk_ctx *ctx, const double *delta, int64_t ld, const double *noise,
                        int64_t k, int64_t noise_ld, int where, int64_t n, int64_t d, int64_t f,
                        int64_t *sel_idx, int64_t *m_out, double *scores, double *mean_out,
                        double *noised_out, int64_t out_ld);

/* RONI verifier -- roni(ww, delta),
 * ML/code/logistic_validator.py:22-33, batched over n updates:
 *     score[i] = mean(sign(Xv . (ww + delta_i)) != yv) - mean(sign(Xv . ww) != yv)
 * with numpy's sign (0 -> 0, NaN -> NaN, which never equals a label).  Xv is
 * nv x d (row stride ldv), yv the nv labels as doubles (creditcard: -1 / +1,
 * utils.py:96-97), ww d weights, deltas n x d (row stride ld).  The Go verifier
 * rejects an update whose score exceeds 0.02 (main.go:213-226).  Any d
 * (creditcard d = 25), n <= 65534.  Each dot is the fp64 FMA chain over k
 * ascending (on the fp64 MFMA, which rounds exactly so). */
int bk_roni_device(bk_ctx *ctx, const double *d_Xv, int64_t nv, int64_t d, int64_t ldv,
                   const double *d_yv, const double *d_ww, const double *d_deltas, int64_t n,
                   int64_t ld, double *d_scores);
/* The Go verifier's shape: the validation set is uploaded once per context
 * (pyInit imports it with the module, honest.go:204-258), then verifyUpdate
 * (honest.go:598-629) scores host updates against the chain's latest model. */
int bk_roni_set_validation(bk_ctx *ctx, const double *Xv, int64_t nv, int64_t d, int64_t ldv,
                           const double *yv);
int bk_roni(bk_ctx *ctx, const double *ww, const double *deltas, int64_t n, int64_t d, int64_t ld,
            double *scores);

/* The torch-path RONI verifier (the mnist / lfw softmax models) --
 * client_obj.roni(ww, delta), ML/Pytorch/client_obj.py:100-112:
 *     updateModel(ww);         original = getTrainErr()
 *     updateModel(ww + delta); after    = getTrainErr();   score = after - original
 * err(w) = 1 - mean(argmax_c(x W^T + b) == y), with w = [W (n_classes x d_in,
 * row-major), b (n_classes)] (SoftmaxModel, ML/Pytorch/softmax_model.py:7-24;
 * d = n_classes * (d_in + 1): mnist 10 x 785 = 7,850) rounded to fp32 after
 * the fp64 add (torch.FloatTensor), each logit the fp64 sum over k ascending of
 * the exact fp32 products plus the bias, rounded once to fp32; argmax as
 * numpy's (first maximum, NaN wins).  Xv is nv x d_in fp32 (row stride ldv),
 * yv the nv labels (int32).  2 <= n_classes <= 16.
 *
 * WHICH SAMPLES: getTrainErr (ML/Pytorch/client.py:136-144) walks the client's
 * SHUFFLED trainloader (client.py:20, shuffle=True) and returns the error of
 * the LAST mini-batch only (its loop overwrites pred / labels), so the
 * reference scores `original` and `after` on two different random batches of
 * batch_size samples (10 in Biscotti, DistSys/honest.go:47).
 *   bk_roni_softmax_batches*  that semantics: the caller draws the batches (its
 *                             loader's shuffles) and passes, per update j, the
 *                             sample indices idx[(2 j) nb .. + nb) (original,
 *                             model ww) and idx[(2 j + 1) nb ..] (after, model
 *                             ww + delta_j); errors are over nb samples
 *   bk_roni_softmax*          every evaluation over the whole set: the
 *                             reference with batch_size >= nv (one batch)
 *
 * NEAR TIES: torch's CPU sgemm accumulates the logits in fp32 in its own
 * order, so its argmax can differ from this one only on samples whose top two
 * logits lie within that rounding.  near_ties (nullable) receives, per
 * evaluation, the number of samples for which
 *     !( l1 - l2 - u (|l1| + |l2|) > E_a + max_c E_c ),  E_c = g (|x| |w_c| + |b_c|),
 * u = 2^-24, g = gamma_{d_in+1}(u) (1 + 2^-10), or any logit is not finite
 * (l1: the winning logit, class a; l2: the best other).  A score can differ
 * from the reference's only if one of its two evaluations has a near tie, and
 * then by at most (near ties) / (samples).  Layout: bk_roni_softmax* n + 1
 * counts (ww, then each update's model); bk_roni_softmax_batches* 2 n (update
 * j: original, after).  A device-side batch index outside [0, nv) gives that
 * update score NaN and near ties -1 (nothing is read out of range); the host
 * form rejects it with BK_EINVAL. */
int bk_roni_softmax_device(bk_ctx *ctx, const float *d_Xv, int64_t nv, int64_t d_in, int64_t ldv,
                           const int32_t *d_yv, int64_t n_classes, const double *d_ww,
                           const double *d_deltas, int64_t n, int64_t ld, double *d_scores,
                           int32_t *d_near_ties);
int bk_roni_softmax_batches_device(bk_ctx *ctx, const float *d_Xv, int64_t nv, int64_t d_in,
                                   int64_t ldv, const int32_t *d_yv, int64_t n_classes,
                                   const double *d_ww, const double *d_deltas, int64_t n,
                                   int64_t ld, const int64_t *d_idx, int64_t nb, double *d_scores,
                                   int32_t *d_near_ties);
/* The Go verifier's shape (verifyUpdate, honest.go:598-629, bound to the
 * torch module's roni): the validation set (the client's training shard) once
 * per context, then host updates scored against the chain's latest model;
 * synchronous. */
int bk_roni_softmax_set_validation(bk_ctx *ctx, const float *Xv, int64_t nv, int64_t d_in,
                                   int64_t ldv, const int32_t *yv, int64_t n_classes);
int bk_roni_softmax(bk_ctx *ctx, const double *ww, const double *deltas, int64_t n, int64_t ld,
                    double *scores, int32_t *near_ties);
int bk_roni_softmax_batches(bk_ctx *ctx, const double *ww, const double *deltas, int64_t n,
                            int64_t ld, const int64_t *idx, int64_t nb, double *scores,
                            int32_t *near_ties);

/* ---- measurement: per-kernel HIP-event timing on the context stream ------- */
enum bk_kernel_id {
    BK_K_GRAM = 0,     /* K1  fp64-MFMA split-K upper-triangle Gram partials */
    BK_K_REDUCE = 1,   /* K1b fixed-order split-K reduce -> packed upper     */
    BK_K_EXPAND = 2,   /* K2t k_transpose: large n, K2's coalesced row copy  */
    BK_K_SCORES = 3,   /* K2  distance row, bitonic sort, sum ranks 1..k    */
    BK_K_RANK = 4,     /* K3  selection rank + mask                          */
    BK_K_COMPACT = 5,  /* K3b mask -> ascending sel_idx                      */
    BK_K_MEAN = 6,     /* K4  masked mean of the selected rows               */
    BK_K_ALLREDUCE = 7,/* C1  RCCL exchange of the packed Gram               */
    BK_K_SYNTH = 8,
    BK_K_H2D = 9,
    BK_K_D2H = 10,
    BK_K_AGGREGATE = 11, /* K4' block aggregation global += sum (bk_aggregate*) */
    BK_K_QSUM = 12,      /* K5  quantised int64 sum (bk_quantized_sum_device)  */
    BK_K_NOISE = 13,     /* K6  noise application (bk_noise_apply_device)      */
    BK_K_RONI = 14,      /* K7  RONI counts + scores (bk_roni*)                 */
    BK_K_SMALL = 15,     /* K1..K4 fused in one launch for n <= 128 (k_small)   */
    BK_K_SLICE = 16,     /* K1i8 digit slicing + error bound (BK_F32_I8)        */
    BK_K_SCORE_GATHER = 17, /* C2 RCCL all-gather of the split scores (n >= 2049) */
    /* bk_comm_set_mode 2: from the end of the last Gram piece to the end of
     * the last all-reduce -- the exchange time the overlap left exposed
     * (BK_K_ALLREDUCE is then the span from the first all-reduce's start) */
    BK_K_EXCHANGE_EXPOSED = 18,
    BK_NUM_KERNELS = 19
};
int bk_timing_enable(bk_ctx *ctx, int on);   /* all kernels; clears accumulated timings */
/* Time only the kernels whose bit (1u << kernel_id) is set: every timed kernel
 * adds two event records to the stream.  Clears accumulated timings. */
int bk_timing_select(bk_ctx *ctx, uint32_t kernel_mask);
int bk_timing_read(bk_ctx *ctx, int kernel_id, double *total_ms, int64_t *count);
/* Record the events of a timed kernel on every `every`-th launch only (1, the
 * default: every launch).  Two event records cost a few us of stream time, as
 * much as config B's whole one-launch step: sampling keeps the timed region's
 * step time honest while the kernel is still timed live.  Clears accumulated
 * timings. */
int bk_timing_stride(bk_ctx *ctx, int every);
const char *bk_kernel_name(int kernel_id);
/* The K1 plan for an aligned fp64 shape: S = workgroup groups (row-block
 * sets, bk_plan.hip), kc = columns per k-block, ntile = 64x64 upper sub-tiles,
 * nwg = workgroups of the launch.  Host-side only; ctx may be NULL. */
int bk_plan(bk_ctx *ctx, int64_t n, int64_t d, int64_t *S, int64_t *kc, int64_t *ntile,
            int64_t *nwg);
/* The same plan with the planner's mode forced (0: v7 interleave, 1: v8
 * round-aligned strides, 2: McNaughton pieces, 3: aligned pieces; -1: the
 * planner's own choice) and its round count (0: the planner's choice).  Every
 * mode computes the same Gram; this entry exists so the planner's coverage
 * check can be exercised for all of them (tests/test_abi.py).  Host-side
 * only; ctx may be NULL.  BK_EHIP if the plan fails its coverage check. */
int bk_plan_mode(bk_ctx *ctx, int64_t n, int64_t d, int mode, int rounds, int64_t *S,
                 int64_t *nwg);

#ifdef __cplusplus
}
#endif
#endif /* BK_H_ */
