// bk_internal.h -- shared declarations between the C ABI (bk_api.hip) and the
// kernels (bk_kernels.hip).  Not installed; the public surface is include/bk.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <vector>

#include "bk_synth.h"

namespace bk {

// the packed upper's trailing record (bk_upper_elems): {column count, columns
// accumulated on the fp32 MFMA, absolute Gram error bound of the int8-sliced
// columns (K1i8), 0}; every exchange sums it with the tiles
constexpr int BK_UPPER_TRAIL = 4;

// Probe knobs: timing-only ablations (BK_GRAM_MODE, BK_K2_MODE), planner and
// kernel-shape overrides and debug traces, read only by A/B builds
// (build(extra=["-DBK_PROBES"], out=tools/ab/...)).  The product libbk.so
// never reads them, so no environment variable can make it return a wrong
// result with BK_OK.  Knobs that only pick between
// bit-identical paths (BK_TINY, BK_SMALL, BK_STAGE_CHUNK_BYTES) and the test
// knobs that force a loud failure stay in the product.
#ifdef BK_PROBES
inline const char *probe_env(const char *name) { return getenv(name); }
constexpr bool kProbes = true;
#else
inline const char *probe_env(const char *) { return nullptr; }
constexpr bool kProbes = false;
#endif

// Split-K plan of K1 for one (n, d): T = ceil(n/64) sub-tile rows, ntile =
// T(T+1)/2 upper sub-tiles, S k-pieces of kc columns (multiple of 8), one wave
// per (sub-tile, piece) task, four tasks per 256-thread workgroup.
struct Plan {
    int n = 0, T = 0, ntile = 0, S = 0, nwg = 0;
    int64_t d = 0, kc = 0;
};

// K1 v3 (LDS-shared) plan -- DESIGN.md "K1".  Wave-tasks over the 64x64
// upper sub-tiles: OFF (one off-diagonal sub-tile, 16 MFMA per 4-column
// k-step), PAIR (the two diagonal sub-tiles of a 128-row super-block, upper
// 16x16 blocks only: 2 x 10 MFMA) and DIAG1 (one diagonal sub-tile, 10).  A
// group is <= 8 wave-tasks over <= 6 row-blocks; one 512-thread workgroup (8
// waves, 2 per SIMD) per (group, XCD, slice); see bk_plan.hip.
constexpr int G3_MAXB = 6;    // row-block slots staged per workgroup
constexpr int G3_BK = 16;     // columns per k-block (one LDS stage, 128 B per row)
constexpr int G3_STAGES = 3;  // LDS ring depth (2 k-blocks in flight)
constexpr int G3_BLK = 64 * G3_BK * 8;                     // 8 KiB per block per stage
constexpr int G3_STAGE = G3_MAXB * G3_BLK;                 // 48 KiB
constexpr int G3_LDS = G3_STAGES * G3_STAGE;               // 144 KiB
enum { T_NONE = 0, T_OFF = 1, T_PAIR = 2, T_DIAG1 = 3 };

// The exchange overlapped with the Gram (bk_comm_set_mode 2): ONE Gram launch
// whose workgroups are ordered piece by piece (piece p = launched workgroups
// [start[p], start[p + 1])); every workgroup, at its exit, counts itself into
// cnt[p] after an agent-scope release of its partials, and the communication
// stream waits on the count (hipStreamWaitValue32) before it reduces and
// all-reduces piece p -- so the pieces' exchanges overlap the later pieces'
// compute without a launch boundary (and its tail) between the pieces
struct PieceMarks {
    unsigned *cnt = nullptr;  // device memory: one arrival count per piece (zeroed per call)
    unsigned *sig[8] = {};    // signal memory (hipMallocSignalMemory): piece p done -> 1
    int k = 0;
    int start[9] = {};
    int nowt = 0;             // probe build only (BK_PIECES_NOWT): plain stores -- timing A/B, invalid
};
#ifdef __HIPCC__
// Only the pieces before the last are handed to the communication stream
// (the last is reduced behind the Gram on its own stream): their workgroups
// store their partials write-through (sc1) and count themselves -- the
// guide's write-through hand-off (MI355X_MICROARCH.md, correctness
// boundaries; the form k_small uses): every storing wave drains its sc1
// stores (vmcnt 0), a workgroup barrier, then one lane's relaxed agent-scope
// add on the piece's device counter; the workgroup whose add returns the
// piece's count - 1 saw every other one's drained stores, and raises the
// piece's signal word (one system-scope store) for the communication
// stream's hipStreamWaitValue32.  No release fence (a buffer_wbl2 writes back
// the XCD's whole dirty L2, ~6.5 us), and no per-workgroup atomic on the
// signal word itself: those serialised at ~0.15-0.3 us each and cost
// 0.25-0.3 ms per Gram (r6 A/B, tools/ab_overlap.py).
__device__ inline bool piece_handed(const PieceMarks &pm) {
    return pm.k > 1 && (int)blockIdx.x < pm.start[pm.k - 1];
}
__device__ inline void piece_done(const PieceMarks &pm) {
    if (!piece_handed(pm)) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int p = 0;
        while (p + 1 < pm.k && (int)blockIdx.x >= pm.start[p + 1]) ++p;
        const unsigned n_p = (unsigned)(pm.start[p + 1] - pm.start[p]);
        if (__hip_atomic_fetch_add(pm.cnt + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            n_p - 1u)
            __hip_atomic_store(pm.sig[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
// a partial's store: write-through (sc1) in a handed-off piece, plain otherwise
__device__ __forceinline__ void st_part(double *p, double v, bool wt) {
    if (wt)
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}
#endif

struct GroupDesc {
    int nb;               // row-blocks staged (even; padded with a duplicate)
    int blk[G3_MAXB];     // 64-row block index per slot
    int Q;                // workgroups of this group per XCD
    int wg0;              // offset of this group's list in wglist
    int cost;             // max over SIMDs of its two waves' MFMA units per k-step
    int task[8][5];       // per wave: {kind, slotA, slotB, u0, u1}
    // balanced band quads (bk_plan.hip): block (0,3) of each diagonal tile moves
    // from the PAIR wave to a super-tile OFF wave holding that row-block.
    // xt: PAIR 1 = skip block (0,3); OFF 1 / 2 = also compute block (0,3) of the
    // diagonal tile of its A / B row-block, into slab slot xslot (the PAIR's)
    int xt[8];
    int xslot[8];
};

struct Plan3 {
    int n = 0, T = 0, ntile = 0, ngroups = 0, nwg = 0, nfull = 0;
    int64_t d = 0;
    GroupDesc *d_groups = nullptr;  // device copies (owned by the context)
    int nvwg = 0;                   // virtual workgroups (segments): one partial slab each
    int *d_seg = nullptr;           // per launched workgroup: {first segment, segment count}
    int *d_wg = nullptr;            // per segment: {group, kstart, kstride, kend, tail}
    int *d_red = nullptr;           // per sub-tile u: {list offset, count, slot}
    int *d_wglist = nullptr;        // per group: its workgroups, in reduction order
};

// host planner (bk_plan.hip)
struct Plan3Host {
    int T = 0, ntile = 0, nfull = 0;
    std::vector<GroupDesc> groups;
    std::vector<int> seg;     // 2 per launched workgroup: its segments [v0, v0 + count)
    std::vector<int> wg;      // 5 per segment (a "virtual workgroup": one group, one slab)
    std::vector<int> red;     // 3 per sub-tile
    std::vector<int> wglist;  // concatenated per-group workgroup lists
};
// bk = columns per k-block: 16 for fp64 input, 32 for fp32 (128 B per row either way)
// mode / rounds >= 0 / > 0: force a planner mode (0 v7, 1 v8 strides, 2 McNaughton,
// 3 aligned pieces) and round count (bk_plan_mode); -1 / 0: the planner's choice
Plan3Host build_plan3(int n, int64_t d, int num_cu, int bk = G3_BK, int mode = -1, int rounds = 0);

// K1 v3: one launched workgroup runs its segments one after the other (a CU's
// share of the columns may span two groups: bk_plan.hip "McNaughton")
hipError_t launch_gram3(const void *X, int dtype, int64_t ld, int n, int64_t d, const Plan3 &pl,
                        double *part, hipStream_t st, int mode = 0, long long *trace = nullptr,
                        bool f32_mfma = false, const int *seg = nullptr, int nwg = -1,
                        const PieceMarks &pm = PieceMarks());
// fp32 rows for the fp32-MFMA K1 (a distinct element type selects the kernel)
struct f32m {
    float v;
    __host__ __device__ operator double() const { return v; }
};
// f32_mfma: K1 ran on the fp32 MFMA (the record's second trailing element)
// u0 / u1 / rec: only sub-tiles [u0, u1) (u1 < 0: all), the trailing record
// written only with rec -- one piece of an exchange overlapped with the Gram
hipError_t launch_reduce3(const double *part, const Plan3 &pl, double *U, hipStream_t st,
                          bool f32_mfma, int u0 = 0, int u1 = -1, bool rec = true);
// A split of K1 v3's plan into k launches whose sub-tiles are contiguous
// pieces [tile_end[p - 1], tile_end[p]) of the packed upper (rows of 64-row
// blocks), every launched workgroup's segments inside one piece: the same
// segments and slabs as the one launch, so every sub-tile's sum is bitwise
// the same.  seg: per piece, 2 ints per launched workgroup (as Plan3Host::seg,
// the XCD mapping b = 8 j + x kept).  False (k = 1) when the plan has no such
// split (a workgroup spanning two pieces: the McNaughton plans of n <= 1024)
bool plan3_pieces(const Plan3Host &H, int k, std::vector<int> &tile_end,
                  std::vector<std::vector<int>> &seg);
// the row-block cuts of a k-piece split: weights w[b] of the row blocks,
// valid[b] whether a cut before block b is allowed; the pieces shrink
// geometrically (x0.6) so the last exchange, the one left exposed, is small
std::vector<int> piece_cuts(const std::vector<double> &w, const std::vector<char> &valid, int k);
hipError_t configure_kernels();
hipError_t launch_gram(const void *X, int dtype, int64_t ld, int n, int64_t d, const Plan &pl,
                       double *part, hipStream_t st);
hipError_t launch_reduce(const double *part, const Plan &pl, double *U, hipStream_t st);
hipError_t launch_sum_ranks(const double *Ug, int R, int64_t stride, double *U, hipStream_t st);
hipError_t launch_add_upper(double *U, const double *P, int64_t count, hipStream_t st);
// Ut / dg: nullable (large n: k_transpose's transposed off-diagonal tiles and
// contiguous diagonal, for coalesced row reads)
// r0 / rows: score rows [r0, r0 + rows) only (rows < 0: to n), writing scores[i]
// and diag[i] for those rows (split scoring over the ranks of a sharded call)
hipError_t launch_scores(const double *U, const double *Ut, const double *dg, int T, int n,
                         int64_t k, double *scores, double *diag, hipStream_t st, int r0 = 0,
                         int rows = -1);
bool scores_transposed(int n);
// bj0 / bj1: transpose only the off-diagonal tiles of block-columns bj0..bj1
// (bj1 < 0: all); the diagonal always
hipError_t launch_transpose(const double *U, int T, double *Ut, double *dg, hipStream_t st,
                            int bj0 = 0, int bj1 = -1);
hipError_t launch_rank(const double *scores, int n, int m, int *mask, double *bnd,
                       hipStream_t st);
// split scoring: gathered {ch scores, status} slices -> n contiguous scores,
// and rec = dcols[0..2] (NaN when a rank's status is not 0)
hipError_t launch_split_unpack(const double *sg, int64_t ch, int parts, int n, const double *dcols,
                               double *scores, double *rec, hipStream_t st);
// The device margin record: MARGIN_WORDS doubles, the public 8 (bk.h
// bk_selection_margin_record) then u_G.  margin[2] codes besides 0 / 1 mark
// the call's outputs invalid (read_margin turns them into errors):
constexpr int MARGIN_WORDS = 9;
constexpr double MARGIN_HANDOFF_TIMEOUT = 2.0;  // k_small: a hand-off wait gave up
constexpr double MARGIN_POISONED = 3.0;         // a shard failed before the exchange
constexpr double MARGIN_QUEUE_DIRTY = 4.0;      // k_small (BK_SMALL_CHECK_LINES): a queue word
                                                // other than word 0 of its line was written
// margin: nullable (MARGIN_WORDS doubles, see k_compact); dcols: the packed upper's two
// trailing elements {column count, columns accumulated on the fp32 MFMA}
hipError_t launch_compact(const int *mask, int n, int64_t *sel, const double *diag,
                          const double *bnd, const double *dcols, int64_t k, double *margin,
                          hipStream_t st);
// K4 of a large selection (m >= MEAN_SEG_MIN) sums the selected rows in
// segments of MEAN_SEG_ROWS (seg_part: mean_segments(m) * d doubles), then
// the segments in order; the order depends on m only
constexpr int MEAN_SEG_MIN = 1024, MEAN_SEG_ROWS = 256;
inline int mean_segments(int m) { return m >= MEAN_SEG_MIN ? (m + MEAN_SEG_ROWS - 1) / MEAN_SEG_ROWS : 1; }
hipError_t launch_mean(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *sel, int m,
                       double *mean, int num_cu, hipStream_t st, double *seg_part = nullptr);
// global[c] += X[idx[0]][c] + X[idx[1]][c] + ... (sequential, idx order)
hipError_t launch_accumulate(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *idx,
                             int m, double *global, int num_cu, hipStream_t st);
// bk_aggregate.hip
hipError_t launch_qsum(const void *X, int dtype, int64_t ld, int64_t d, const int64_t *idx, int m,
                       double scale, int64_t *sum, double *sumf, int num_cu, hipStream_t st);
hipError_t launch_noise(const double *delta, int64_t ld, int64_t n, int64_t d, const double *noise,
                        int64_t k, int64_t nld, double *out, int64_t old, int num_cu,
                        hipStream_t st);
hipError_t configure_aggregate_kernels();
// bk_roni.hip
// K7: ws = roni_ws(n, d) bytes (the models' weights, k-major)
size_t roni_ws(int64_t n, int64_t d);
hipError_t launch_roni(const double *Xv, int64_t nv, int64_t d, int64_t ldv, const double *yv,
                       const double *ww, const double *deltas, int64_t n, int64_t ld,
                       double *ws, unsigned int *cnt, double *scores, hipStream_t st);
// the torch-path (softmax model) RONI, K8: ws = roni_softmax_ws(n, din, nv, C) bytes;
// good: 2 (n + 1) counters; xn: the samples' norms (nullable: computed into ws);
// near_out (nullable): the n + 1 near-tie counts (ww, then each update's model)
size_t roni_softmax_ws(int64_t n, int64_t din, int64_t nv, int C);
double roni_softmax_g(int64_t din);
hipError_t launch_roni_xnorm(const float *Xv, int64_t nv, int64_t din, int64_t ldv, double *xn,
                             hipStream_t st);
hipError_t launch_roni_softmax(const float *Xv, int64_t nv, int64_t din, int64_t ldv,
                               const int32_t *yv, int C, const double *ww, const double *deltas,
                               int64_t n, int64_t ld, double *ws, const double *xn,
                               unsigned int *good, double *scores, int32_t *near_out,
                               hipStream_t st);
// K8 on the last mini-batches (idx: n x 2 x nb sample indices; near_out nullable, 2 n)
hipError_t launch_roni_softmax_batches(const float *Xv, int64_t nv, int64_t din, int64_t ldv,
                                       const int32_t *yv, int C, const double *ww,
                                       const double *deltas, int64_t n, int64_t ld,
                                       const int64_t *idx, int64_t nb, double *scores,
                                       int32_t *near_out, hipStream_t st);
// bk_i8.hip: K1i8, the Gram of fp32 rows from exact int8 digit slices
// (BK_F32_I8): column ranges (one per XCD), digit planes [3][npad][dp] int8
struct I8Layout {
    // ns: digit planes (3: the six products of weight >= 2^-26; 2: the three of
    // weight >= 2^-19, BK_F32_I8X2); tj: the output tile's columns (128 / 256)
    int npad = 0, R = 0, T128 = 0, T64 = 0, es = 4, ns = 3, tj = 128;
    int64_t dp = 0, plane = 0, ntile64 = 0;
    std::vector<int64_t> rb;  // range boundaries (R + 1, multiples of 64 columns)
    std::vector<int> order;   // per workgroup {tile I | J << 16, range (-1: idle)}
    std::vector<int> tiles;   // the output tiles (I | J << 16), super-blocked
};
// k pieces of the tile list by 128-row blocks [I0, I1) (the exchange overlapping
// the Gram): per piece its workgroup order (as I8Layout::order) and the
// packed upper's sub-tile range; false when fewer than k cuts exist
bool i8_pieces(const I8Layout &L, int k, std::vector<int> &tile_end,
               std::vector<std::vector<int>> &orders);
I8Layout i8_layout(int n, int64_t d, int es, int num_cu, int ns = 3);
size_t i8_workspace(const I8Layout &L);
hipError_t configure_i8_kernels();
// tables: device copy of {rb (R + 1 int64), order (int pairs)}; ws:
// i8_workspace(L) bytes.  slice: digit planes + the error bound; gemm: the
// range partials; reduce: U (bk_upper_elems(n)) with the trailing record
// {d, 0, bound, 0}
hipError_t launch_i8_slice(const void *X, int dtype, int64_t ld, int n, int64_t d,
                           const I8Layout &L, void *ws, const void *tables, hipStream_t st);
// order / items: one piece's workgroup order (device int pairs), else the layout's
hipError_t launch_i8_gemm(int n, const I8Layout &L, void *ws, const void *tables, hipStream_t st,
                          const void *order = nullptr, int64_t items = -1,
                          const PieceMarks &pm = PieceMarks());
// [e0, e1) elements of U (e1 < 0: all); the record only with rec
hipError_t launch_i8_reduce(int64_t d, const I8Layout &L, void *ws, double *U, hipStream_t st,
                            int64_t e0 = 0, int64_t e1 = -1, bool rec = true);

// bk_small.hip: the whole Multi-Krum of a small batch (n <= 128) in one launch
struct SmallPlan {
    int nb16 = 0, nblk = 0, kc = 0, P = 0, ng = 0, Q = 0, nS = 0, C = 0;  // P chunks, ng G items
};
SmallPlan small_plan(int n, int64_t d, int num_cu);
// n <= 16 and d <= 128 (config A): launch_small runs k_tiny, one workgroup
bool tiny_ok(int n, int64_t d);
constexpr int SMALL_SPLIT_ITEMS = 4;       // G items per chunk (bk_small.hip SMALL_SPLIT)
constexpr int SMALL_CTR_WORDS = 71 * 32;  // 71 queue lines of 128 B (bk_small.hip)
constexpr uint64_t SMALL_SPIN_MAX = 1ull << 24;  // polls before a hand-off wait gives up (~1 s)
hipError_t launch_small(const void *X, int dtype, int64_t ld, int n, int64_t d, int f,
                        const SmallPlan &p, double *part, double *U, double *scores, double *diag,
                        int64_t *sel, double *mean, double *margin, unsigned *ctr, int num_cu,
                        hipStream_t st, long long *trace = nullptr,
                        uint64_t spin_max = SMALL_SPIN_MAX, int check_lines = 0,
                        double *scores_out = nullptr, int g0 = 0, int gn = -1, bool sm = true);
hipError_t launch_synth(void *X, int dtype, int64_t ld, int64_t n, int64_t dl, int64_t c0,
                        const int64_t *perm, const SynthParams &P, hipStream_t st);

}  // namespace bk
