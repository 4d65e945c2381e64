// bk_api.hip -- the C ABI (include/bk.h): context, workspace, orchestration,
// RCCL exchange, per-kernel HIP-event timing.  No torch, no C++ types across
// the boundary; every failure becomes a negative status + bk_last_error().
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/bk.h"
#include "bk_hostpool.h"
#include "bk_internal.h"
#include "bk_synth.h"

using namespace bk;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                      \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return fail(_e == hipErrorOutOfMemory ? BK_ENOMEM : BK_EHIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(_e), __FILE__, __LINE__);                \
    } while (0)

#define RCCLCHK(expr)                                                                        \
    do {                                                                                     \
        ncclResult_t _r = (expr);                                                            \
        if (_r != ncclSuccess)                                                               \
            return fail(BK_ERCCL, "%s: %s (%s:%d)", #expr, ncclGetErrorString(_r), __FILE__, \
                        __LINE__);                                                           \
    } while (0)

#define CHK(expr)              \
    do {                       \
        int _s = (expr);       \
        if (_s != BK_OK) return _s; \
    } while (0)

const char *kKernelNames[BK_NUM_KERNELS] = {"k_gram",    "k_reduce",  "k_transpose", "k_scores",
                                            "k_rank",    "k_compact", "k_mean",   "allreduce",
                                            "k_synth",   "h2d",       "d2h",
                                            "k_aggregate", "k_qsum",  "k_noise",
                                            "k_roni", "k_small", "k_slice", "score_gather",
                                            "exchange_exposed"};

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    uint64_t *epoch = nullptr;  // the owning context's ws_epoch (graph invalidation)
};

// A K1 plan's (or K1i8 layout's) split into k launches whose sub-tiles are
// contiguous pieces of the packed upper, for the exchange overlapped with
// the Gram (bk_comm_set_mode 2): piece p's elements are U[e[p], e[p + 1]),
// the last piece's range ending with the trailing record
struct Pieces {
    int k = 0;                // pieces built for (0: none yet)
    bool ok = false;          // false: the plan has no k-piece split
    std::vector<int64_t> e;   // k + 1 element bounds of U
    std::vector<int> nwg;     // per piece: launched workgroups (K1 v3) / items (K1i8)
    std::vector<size_t> off;  // per piece: its table's offset in d (ints)
    int *d = nullptr;         // device copy of the tables, concatenated
};

void free_pieces(Pieces &pc) {
    if (pc.d) (void)hipFree(pc.d);
    pc = Pieces();
}

}  // namespace

struct bk_ctx {
    int device = 0;
    int num_cu = 256;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // workspace (grow-only)
    DevBuf part, U, Ug, scores, mask, sel, X, mean, perm, trace, idx;
    // the selection margin of the last finish (K2 diag, K3 boundary scores, K3b record)
    DevBuf diag, bnd;
    DevBuf Ut;  // K2 at large n: transposed off-diagonal tiles + diagonal (k_transpose)
    // k_small (n <= 128, one launch): its queue counters (zeroed once; every
    // launch leaves them zero) and the split-K partials
    DevBuf small_ctr, small_part;
    DevBuf mean_part;  // K4 of a large selection: per-segment column sums (launch_mean)
    int small_on = 1;
    uint64_t small_spin_max = SMALL_SPIN_MAX;  // test knob BK_SMALL_SPIN_MAX=<polls>[,<launches>]
    int64_t small_spin_left = -1;              // ... for this many launches (-1: all)
    int small_check_lines = 0;                 // debug knob BK_SMALL_CHECK_LINES (bk_create)
    int margin_valid = 0;
    // a finish ran since its record's error codes were last read (bk_synchronize
    // reads them: an asynchronous caller learns of an invalid call there)
    int margin_unchecked = 0;
    int64_t spin_us = 2000;  // wait_stream: poll this long before blocking (BK_SPIN_US)
    // the record of the last finish, written by the kernels straight into mapped
    // pinned memory (GPU-cached, written back at the kernel's end): the host
    // reads it after the stream has finished, with no device-to-host copy
    double *hmargin = nullptr;
    double *dmargin = nullptr;  // its device address
    // pinned: the n <= 128 host entries' outputs {margin, sel, scores, mean},
    // read back in one copy (a D2H into pageable memory goes through HIP's
    // staging: ~20 us per copy at config B)
    void *hout = nullptr;  // the host small path's mapped output block (pinned)
    size_t hout_bytes = 0;
    double *hout_dev = nullptr;          // its device address
    const double *hout_host_margin = nullptr;  // its record, as the host reads it
    const double *margin_host = nullptr;  // non-null: the last call's record is there
    // BK_F32_CERTIFIED: 1 while the exact re-run of a near-tie call is in progress
    int force_exact = 0;
    int64_t certified_reruns = 0;
    // RONI: the validation set (bk_roni_set_validation) and per-call scratch
    DevBuf roni_X, roni_y, roni_w, roni_d, roni_cnt, roni_s;
    int64_t roni_nv = 0, roni_dim = 0;
    // the torch-path (softmax) RONI: its validation set (fp32 samples, int32
    // labels; bk_roni_softmax_set_validation) and the prepared models
    DevBuf rmc_X, rmc_y, rmc_ws, rmc_xn, rmc_idx, rmc_nt;
    int64_t rmc_nv = 0, rmc_din = 0, rmc_C = 0;
    // bk_multikrum_noised: a 2-slot ring of noise chunks, filled on a copy
    // stream while K6 consumes the previous chunk on `stream` (created lazily)
    DevBuf noise;
    hipStream_t copy = nullptr;
    hipEvent_t ev_go = nullptr, ev_cp[2] = {nullptr, nullptr}, ev_use[2] = {nullptr, nullptr};
    // host-side pinned allocations handed out by bk_stage_alloc
    std::vector<void *> staged;
    // bk_multikrum_rows: worker threads packing the caller's separate host rows
    // into a pinned ring (both created on first use), and the ring slots'
    // copy-done events
    bk::HostPool *hpool = nullptr;
    int hthreads = 0;  // packing threads incl. the caller (bk_set_host_threads; 0: default)
    void *rstage = nullptr;
    size_t rstage_bytes = 0;
    hipEvent_t ev_rows[4] = {nullptr, nullptr, nullptr, nullptr};
    // timing
    uint32_t timing = 0;  // bit k: record HIP events around kernel k (bk_timing_select)
    int tstride = 1;      // ... on every tstride-th launch of it (bk_timing_stride)
    int64_t tseq[BK_NUM_KERNELS] = {0};
    struct Ev {
        int kid;
        hipEvent_t a, b;
    };
    std::vector<Ev> pending;
    std::vector<hipEvent_t> pool;
    double tot_ms[BK_NUM_KERNELS] = {0};
    int64_t cnt[BK_NUM_KERNELS] = {0};
    // K1 v3 plans (device tables), cached per (n, d)
    struct CachedPlan {
        int n;
        int64_t d;
        int bk;  // columns per k-block (16 fp64, 32 fp32)
        Plan3 p;
        Pieces pc;
    };
    std::vector<CachedPlan> plans;
    // K1i8 (BK_F32_I8): layouts and device tables per (n, d), and the workspace
    struct I8Cached {
        int64_t n = 0, d = 0;
        I8Layout L;
        void *tables = nullptr;
        Pieces pc;
    };
    std::vector<I8Cached> i8;
    DevBuf i8ws;
    // K1i8 signatures {n, d, element size, digits} whose workspace failed to
    // allocate: they run exact until the mode is set again (bk_set_f*_mode)
    std::vector<std::array<int64_t, 4>> i8_failed;
    int gram_variant = 3;  // 3: LDS-shared v3 for aligned fp64; 1: v1 everywhere (BK_GRAM=v1)
    int gram_mode = 0;     // BK_GRAM_MODE: timing-only ablations of v3 (tools/, never tests)
    int f32_mode = BK_F32_EXACT;  // fp32 rows: widened onto the fp64 MFMA, or the fp32 MFMA
    int f64_mode = BK_F64_EXACT;  // fp64 rows: the fp64 MFMA, or K1i8 (bk_set_f64_mode)
    // hipGraph replay of bk_multikrum_device (bk_graph_enable): one captured
    // launch sequence per call signature; every workspace reallocation or plan
    // eviction bumps ws_epoch, which retires the graphs that baked the old
    // pointers in
    int graph_on = 0;
    uint64_t ws_epoch = 0;
    struct CachedGraph {
        const void *X;
        int dtype;
        int64_t n, d, ld, f;
        const void *sel, *scores, *mean;
        uint64_t epoch;
        hipGraph_t g;
        hipGraphExec_t exec;
    };
    std::vector<CachedGraph> graphs;
    // RCCL
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    int deterministic = 0;
    // the sharded entry's status agreement (sharded_once): the signature of the
    // last agreed call, and the device word the agreement all-reduces
    int64_t agreed_n = -1, agreed_f = -1;
    int agreed_dtype = -1, agreed_det = -1;
    DevBuf status;
    int test_fail_exchange = 0;  // test knob BK_TEST_FAIL_BEFORE_EXCHANGE (bk_create)
    int test_i8_enomem = 0;      // test knob BK_TEST_I8_ENOMEM: K1i8's workspace "fails" (bk_create)
    int test_fail_piece = 0;     // test knob BK_TEST_FAIL_PIECE=p: the overlapped Gram's piece p-1 fails
    int test_pieces_disagree = 0;  // test knob BK_TEST_PIECES_DISAGREE=1: act as if a peer cut the pieces differently
    // the overlapped exchange's piece layout as agreed at the signature's first
    // call: false when the ranks' layouts differed (every rank then exchanges
    // whole, serially, for that signature)
    bool overlap_agreed = true;
    // split scoring (stage_finish): at n >= split_min_n each rank of a sharded
    // call scores its share of the rows and the ranks all-gather the scores
    // (BK_SPLIT_SCORES_MIN_N; 0 turns it off).  Knobs for a 1-rank
    // communicator (bk_create): BK_TEST_SPLIT_SCORES=R scores in R row chunks,
    // one launch each, as R ranks would (the arithmetic of the split, tested on
    // one GPU); BK_EMU_SPLIT_SCORES=R scores only rank 0's chunk once a mode's
    // first call has scored them all (bench.py --emulate-ranks: one rank's time;
    // TIMING ONLY -- the other shares keep that first call's scores, so the
    // outputs and the margin of later calls are not valid, and new data at the
    // same n is not rescored)
    int64_t split_min_n = 2049;
    int test_split_scores = 0, emu_split_scores = 0;
    int test_split_fail = 0;   // BK_TEST_SPLIT_FAIL=p: under BK_TEST_SPLIT_SCORES, share p - 1 "fails"
    int64_t emu_split_n = -1;  // emulation: the n whose other chunks are scored
    DevBuf sgather;            // the gathered scores: parts x chunk doubles
    DevBuf pcnt;               // the overlapped exchange's per-piece arrival counts
    // bk_comm_set_mode 2: the exchange overlapped with the Gram in this many
    // pieces (BK_OVERLAP_PIECES, default 2; 0: off), all-reduced on cstream
    int overlap = 0;
    hipStream_t cstream = nullptr;
    hipEvent_t ev_piece[8] = {};
    hipEvent_t ev_cdone = nullptr;
    unsigned *sigcnt[8] = {};       // probe A/B only (BK_PIECES_DEVWAIT): signal memory for hipStreamWaitValue32
    // the pieces' completion words, polled by the host: fine-grained pinned
    // host memory, one 64-B line per piece (the Gram's last workgroup of a
    // piece stores 1 there, system scope)
    unsigned *hsig = nullptr;       // host address
    unsigned *hsig_d = nullptr;     // the same words as the device addresses them
    bool sig_pending = false;       // a launched Gram's piece words not all seen yet
    int wait_value_ok = -1;         // hipDeviceAttributeCanUseStreamWaitValue (-1: not asked)
    int64_t exchanges = 0;        // exchanges of the packed Gram (bk_comm_stats)
    double exchanged_bytes = 0;   // bytes each rank put into them
};

namespace {

int ensure(DevBuf &b, size_t bytes) {
    if (bytes <= b.bytes) return BK_OK;
    if (b.epoch) ++*b.epoch;  // pointers baked into captured graphs are about to change
    if (b.p) {
        hipError_t e = hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
        if (e != hipSuccess) return fail(BK_EHIP, "hipFree: %s", hipGetErrorString(e));
    }
    size_t want = bytes < 256 ? 256 : bytes;
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) {
        b.p = nullptr;
        return fail(BK_ENOMEM, "hipMalloc(%zu bytes): %s", want, hipGetErrorString(e));
    }
    b.bytes = want;
    return BK_OK;
}

void drop_graph(bk_ctx::CachedGraph &cg) {
    if (cg.exec) (void)hipGraphExecDestroy(cg.exec);
    if (cg.g) (void)hipGraphDestroy(cg.g);
    cg.exec = nullptr;
    cg.g = nullptr;
}

// every workspace buffer of c bumps c->ws_epoch when it is reallocated
void bind_epoch(bk_ctx *c) {
    DevBuf *bufs[] = {&c->part, &c->U,    &c->Ug,   &c->scores, &c->mask,   &c->sel,
                      &c->X,    &c->mean, &c->perm, &c->trace,  &c->idx,    &c->roni_X,
                      &c->roni_y, &c->roni_w, &c->roni_d, &c->roni_cnt, &c->roni_s,
                      &c->noise, &c->diag, &c->bnd, &c->Ut, &c->small_ctr, &c->small_part,
                      &c->mean_part, &c->status, &c->rmc_X, &c->rmc_y, &c->rmc_ws,
                      &c->rmc_xn, &c->rmc_idx, &c->rmc_nt, &c->i8ws, &c->sgather, &c->pcnt};
    for (DevBuf *b : bufs) b->epoch = &c->ws_epoch;
}

int get_event(bk_ctx *c, hipEvent_t *out) {
    if (!c->pool.empty()) {
        *out = c->pool.back();
        c->pool.pop_back();
        return BK_OK;
    }
    HIPCHK(hipEventCreate(out));
    return BK_OK;
}

// Bracket one launch with events when timing is on.
bool timing_on(bk_ctx *c, int kid) {
    if (!((c->timing >> kid) & 1u)) return false;
    return c->tstride <= 1 || (c->tseq[kid]++ % c->tstride) == 0;
}

template <typename F>
int timed(bk_ctx *c, int kid, F &&launch) {
    hipEvent_t a = nullptr, b = nullptr;
    const bool on = timing_on(c, kid);
    if (on) {
        CHK(get_event(c, &a));
        CHK(get_event(c, &b));
        HIPCHK(hipEventRecord(a, c->stream));
    }
    hipError_t e = launch();
    if (e != hipSuccess)
        return fail(BK_EHIP, "%s launch: %s", kKernelNames[kid], hipGetErrorString(e));
    if (on) {
        HIPCHK(hipEventRecord(b, c->stream));
        c->pending.push_back({kid, a, b});
    }
    return BK_OK;
}


Plan make_plan(int64_t n, int64_t d, int num_cu, size_t in_bytes) {
    Plan pl;
    pl.n = (int)n;
    pl.d = d;
    pl.T = (int)((n + 63) / 64);
    pl.ntile = pl.T * (pl.T + 1) / 2;
    const int64_t W = (int64_t)num_cu * 4;  // one wave per SIMD (K1 runs 1 workgroup per CU)
    const size_t part_cap = in_bytes / 16 > (64u << 20) ? in_bytes / 16 : (64u << 20);
    double best_cost = 1e300;
    int best_S = 1;
    for (int S = 1; S <= 4096; ++S) {
        const int64_t kc = ((d + S - 1) / S + 7) / 8 * 8;
        if (S > 1 && kc < 256) break;
        const int64_t Se = (d + kc - 1) / kc;
        if (Se != S) continue;
        if (S > 1 && (size_t)pl.ntile * S * 32768 > part_cap) break;
        const int64_t tasks = (int64_t)pl.ntile * S;
        const int64_t rounds = (tasks + W - 1) / W;
        const double cost = (double)rounds * (double)(kc + 64);  // +64: per-task fixed cost
        if (cost < best_cost * 0.99) {
            best_cost = cost;
            best_S = S;
        }
    }
    pl.S = best_S;
    pl.kc = ((d + best_S - 1) / best_S + 7) / 8 * 8;
    const int64_t tasks = (int64_t)pl.ntile * pl.S;
    pl.nwg = (int)((tasks + 3) / 4);
    return pl;
}

int check_common(bk_ctx *c, const void *X, int dtype, int64_t n, int64_t d, int64_t ld) {
    if (!c) return fail(BK_EINVAL, "null context");
    if (!X) return fail(BK_EINVAL, "null X");
    if (dtype != BK_F64 && dtype != BK_F32) return fail(BK_EINVAL, "bad dtype %d", dtype);
    if (n < 1 || d < 1) return fail(BK_EINVAL, "need n >= 1 and d >= 1 (n=%lld d=%lld)",
                                   (long long)n, (long long)d);
    if (n > BK_MAX_N) return fail(BK_ENOTSUP, "n=%lld exceeds BK_MAX_N=%d", (long long)n, BK_MAX_N);
    if (ld < d) return fail(BK_EINVAL, "ld=%lld < d=%lld", (long long)ld, (long long)d);
    return BK_OK;
}

size_t esize(int dtype) { return dtype == BK_F64 ? 8 : 4; }

void free_plan(Plan3 &p) {
    if (p.d_groups) (void)hipFree(p.d_groups);
    if (p.d_wg) (void)hipFree(p.d_wg);
    if (p.d_seg) (void)hipFree(p.d_seg);
    if (p.d_red) (void)hipFree(p.d_red);
    if (p.d_wglist) (void)hipFree(p.d_wglist);
    p.d_groups = nullptr;
    p.d_wg = p.d_red = p.d_wglist = p.d_seg = nullptr;
}

int get_plan3(bk_ctx *c, int64_t n, int64_t d, int bk, Plan3 **out) {
    for (auto &cp : c->plans)
        if (cp.n == n && cp.d == d && cp.bk == bk) {
            *out = &cp.p;
            return BK_OK;
        }
    Plan3Host H = build_plan3((int)n, d, c->num_cu, bk);
    for (int u = 0; u < H.ntile; ++u)
        if (H.red[3 * u + 1] < 0) return fail(BK_EHIP, "internal: K1 plan misses sub-tile %d", u);
    Plan3 p;
    p.n = (int)n;
    p.d = d;
    p.T = H.T;
    p.ntile = H.ntile;
    p.ngroups = (int)H.groups.size();
    p.nwg = (int)H.seg.size() / 2;
    p.nvwg = (int)H.wg.size() / 5;
    p.nfull = H.nfull;
    hipError_t e = hipMalloc(&p.d_groups, H.groups.size() * sizeof(GroupDesc));
    if (e == hipSuccess) e = hipMalloc(&p.d_wg, H.wg.size() * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&p.d_seg, H.seg.size() * sizeof(int));
    if (e == hipSuccess)
        e = hipMemcpy(p.d_seg, H.seg.data(), H.seg.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p.d_red, H.red.size() * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&p.d_wglist, H.wglist.size() * sizeof(int));
    if (e == hipSuccess)
        e = hipMemcpy(p.d_wglist, H.wglist.data(), H.wglist.size() * sizeof(int),
                      hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(p.d_groups, H.groups.data(), H.groups.size() * sizeof(GroupDesc),
                      hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(p.d_wg, H.wg.data(), H.wg.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(p.d_red, H.red.data(), H.red.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        free_plan(p);
        return fail(BK_ENOMEM, "K1 plan tables: %s", hipGetErrorString(e));
    }
    if (c->plans.size() >= 8) {
        free_plan(c->plans.front().p);
        free_pieces(c->plans.front().pc);
        c->plans.erase(c->plans.begin());
        ++c->ws_epoch;  // a captured graph may point at the evicted tables
    }
    c->plans.push_back({(int)n, d, bk, p});
    *out = &c->plans.back().p;
    return BK_OK;
}

// K1 v3 reads 16-B granules with global_load_lds: every row start must be
// 16-B aligned (fp64: ld even, fp32: ld a multiple of 4)
bool use_v3(bk_ctx *c, const void *dX, int dtype, int64_t ld) {
    const int64_t epg = dtype == BK_F64 ? 2 : 4;
    return c->gram_variant == 3 && (ld % epg) == 0 && ((uintptr_t)dX % 16) == 0;
}
int v3_bk(int dtype) { return dtype == BK_F64 ? G3_BK : 2 * G3_BK; }

// fp32 rows on the fp32 MFMA for this call: BK_F32_MFMA, or BK_F32_CERTIFIED
// unless its exact re-run of a near tie is in progress
bool f32_mfma_now(const bk_ctx *c, int dtype) {
    return dtype == BK_F32 && !c->force_exact &&
           (c->f32_mode == BK_F32_MFMA || c->f32_mode == BK_F32_CERTIFIED);
}

// rows on the int8-sliced Gram (K1i8) for this call: fp32 rows under
// BK_F32_I8* / BK_F32_I8X2*, fp64 rows under BK_F64_I8* / BK_F64_I8X2*,
// outside a certified exact re-run; 16-B aligned rows, d >= 64.  Returns the
// digit count (3, or 2 for the X2 modes), 0 when the call runs elsewhere
int i8_now(const bk_ctx *c, const void *dX, int dtype, int64_t d, int64_t ld) {
    const int mode = dtype == BK_F32 ? c->f32_mode : c->f64_mode;
    const int64_t epg = dtype == BK_F32 ? 4 : 2;
    if (c->force_exact || d < 64 || (ld % epg) != 0 || ((uintptr_t)dX % 16) != 0) return 0;
    if (mode == BK_F32_I8 || mode == BK_F32_I8_CERTIFIED) return 3;
    if (mode == BK_F32_I8X2 || mode == BK_F32_I8X2_CERTIFIED) return 2;
    return 0;
}

// K1i8's layout (ranges, tile order) and its device tables, cached per (n, d)
int get_i8(bk_ctx *c, int64_t n, int64_t d, int es, int ns, bk_ctx::I8Cached **out) {
    for (auto &e : c->i8)
        if (e.n == n && e.d == d && e.L.es == es && e.L.ns == ns) {
            *out = &e;
            return BK_OK;
        }
    bk_ctx::I8Cached e;
    e.n = n;
    e.d = d;
    e.L = i8_layout((int)n, d, es, c->num_cu, ns);
    const size_t tb = (size_t)(e.L.R + 1) * 8 + e.L.order.size() * sizeof(int);
    std::vector<char> h(tb);
    memcpy(h.data(), e.L.rb.data(), (size_t)(e.L.R + 1) * 8);
    memcpy(h.data() + (size_t)(e.L.R + 1) * 8, e.L.order.data(), e.L.order.size() * sizeof(int));
    hipError_t er = hipMalloc(&e.tables, tb);
    if (er == hipSuccess) er = hipMemcpy(e.tables, h.data(), tb, hipMemcpyHostToDevice);
    if (er != hipSuccess) {
        if (e.tables) (void)hipFree(e.tables);
        return fail(BK_ENOMEM, "K1i8 tables: %s", hipGetErrorString(er));
    }
    if (c->i8.size() >= 4) {
        (void)hipFree(c->i8.front().tables);
        free_pieces(c->i8.front().pc);
        c->i8.erase(c->i8.begin());
        ++c->ws_epoch;  // a captured graph may point at the evicted tables
    }
    c->i8.push_back(e);
    *out = &c->i8.back();
    return BK_OK;
}

// K1i8's layout and workspace for this call, or nullptr when the call does not
// take K1i8 -- or cannot: its range partials take R times the packed upper
// (~34 GB at n = 16,384, d = 1M fp32), and a batch the exact path can still
// take is not refused for them, it runs exact (its record then carries no
// int8 bound)
bk_ctx::I8Cached *i8_prepared(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d,
                              int64_t ld) {
    const int ns = i8_now(c, dX, dtype, d, ld);
    if (!ns) return nullptr;
    // a layout whose workspace could not be allocated goes straight to the
    // exact path on later calls: no repeated multi-GB hipMalloc attempts, no
    // workspace freed (and captured graphs retired) every call
    const std::array<int64_t, 4> sig{n, d, (int64_t)esize(dtype), ns};
    for (const auto &f : c->i8_failed)
        if (f == sig) return nullptr;
    const std::string keep = g_err;
    bk_ctx::I8Cached *e = nullptr;
    int st = c->test_i8_enomem ? BK_ENOMEM : get_i8(c, n, d, (int)esize(dtype), ns, &e);
    if (st == BK_OK) st = ensure(c->i8ws, i8_workspace(e->L));
    if (st == BK_OK) return e;
    (void)hipGetLastError();  // a failed hipMalloc must not surface at the next launch check
    g_err = keep;
    c->i8_failed.push_back(sig);
    return nullptr;
}

// Everything stage_gram allocates (K1's plan tables and split-K slabs), so a
// caller can learn of an allocation failure before it launches anything
int prepare_gram(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld) {
    if (i8_prepared(c, dX, dtype, n, d, ld)) return BK_OK;
    if (use_v3(c, dX, dtype, ld)) {
        Plan3 *p3 = nullptr;
        CHK(get_plan3(c, n, d, v3_bk(dtype), &p3));
        return ensure(c->part, (size_t)p3->nvwg * 16 * 4096 * sizeof(double));
    }
    const Plan pl = make_plan(n, d, c->num_cu, (size_t)n * d * esize(dtype));
    return ensure(c->part, (size_t)pl.ntile * pl.S * 4096 * sizeof(double));
}

// A partial that must still join an exchange after its rank failed: the
// trailing pair becomes NaN, every sum with it is NaN, and every rank's finish
// marks the call invalid (MARGIN_POISONED -> BK_ERCCL from bk_synchronize and
// the margin readers)
int poison_upper(bk_ctx *c, double *U, int64_t n) {
    const int64_t T = (n + 63) / 64;
    HIPCHK(hipMemsetAsync(U + T * (T + 1) / 2 * 4096, 0xFF, BK_UPPER_TRAIL * sizeof(double),
                          c->stream));
    return BK_OK;
}

// K1 + K1b: packed upper-triangle Gram of this call's columns into U (tiles,
// then the trailing pair {column count, columns on the fp32 MFMA}, bk_upper_elems)
int stage_gram(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld,
               double *U, Plan &pl) {
    if (bk_ctx::I8Cached *e = i8_prepared(c, dX, dtype, n, d, ld)) {
        // K1i8: digit slices + bound (k_slice), the int8 GEMM (k_gram), the
        // fixed-order sum of the range partials + the record (k_reduce)
        pl.n = (int)n;
        pl.d = d;
        pl.T = (int)((n + 63) / 64);
        pl.ntile = pl.T * (pl.T + 1) / 2;
        const I8Layout &L = e->L;
        void *ws = c->i8ws.p, *tb = e->tables;
        CHK(timed(c, BK_K_SLICE, [&] {
            return launch_i8_slice(dX, dtype, ld, (int)n, d, L, ws, tb, c->stream);
        }));
        CHK(timed(c, BK_K_GRAM, [&] { return launch_i8_gemm((int)n, L, ws, tb, c->stream); }));
        CHK(timed(c, BK_K_REDUCE, [&] { return launch_i8_reduce(d, L, ws, U, c->stream); }));
        return BK_OK;
    }
    if (use_v3(c, dX, dtype, ld)) {
        Plan3 *p3 = nullptr;
        CHK(get_plan3(c, n, d, v3_bk(dtype), &p3));
        pl.n = (int)n;
        pl.d = d;
        pl.T = p3->T;
        pl.ntile = p3->ntile;
        CHK(ensure(c->part, (size_t)p3->nvwg * 16 * 4096 * sizeof(double)));
        double *part = (double *)c->part.p;
        const Plan3 &P3 = *p3;
        long long *trace = nullptr;
        const char *tfile = probe_env("BK_TRACE_FILE");  // debug: per-workgroup timeline
        if (tfile) {
            CHK(ensure(c->trace, (size_t)P3.nwg * 24 * sizeof(long long)));
            HIPCHK(hipMemsetAsync(c->trace.p, 0, (size_t)P3.nwg * 24 * sizeof(long long), c->stream));
            trace = (long long *)c->trace.p;
        }
        CHK(timed(c, BK_K_GRAM, [&] {
            return launch_gram3(dX, dtype, ld, (int)n, d, P3, part, c->stream, c->gram_mode,
                                trace, f32_mfma_now(c, dtype));
        }));
        if (tfile) {
            std::vector<long long> h((size_t)P3.nwg * 24);
            HIPCHK(hipMemcpyAsync(h.data(), trace, h.size() * sizeof(long long),
                                  hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            if (FILE *fp = fopen(tfile, "ab")) {
                fwrite(h.data(), sizeof(long long), h.size(), fp);
                fclose(fp);
            }
        }
        CHK(timed(c, BK_K_REDUCE, [&] {
            return launch_reduce3(part, P3, U, c->stream, f32_mfma_now(c, dtype));
        }));
        return BK_OK;
    }
    pl = make_plan(n, d, c->num_cu, (size_t)n * d * esize(dtype));
    CHK(ensure(c->part, (size_t)pl.ntile * pl.S * 4096 * sizeof(double)));
    double *part = (double *)c->part.p;
    CHK(timed(c, BK_K_GRAM,
              [&] { return launch_gram(dX, dtype, ld, (int)n, d, pl, part, c->stream); }));
    CHK(timed(c, BK_K_REDUCE, [&] { return launch_reduce(part, pl, U, c->stream); }));
    return BK_OK;
}

// ---- the Gram in pieces, for an exchange overlapped with it ---------------
// (bk_comm_set_mode 2).  The packed upper is
// cut into k contiguous pieces by rows of sub-tiles; piece p is computed by its
// own launches (the same segments / (tile, range) items as the one launch, so
// every sub-tile is bitwise the same), and its all-reduce starts on the
// communication stream while the next pieces compute.

// the device copy of the pieces' tables
int upload_pieces(Pieces &pc, const std::vector<std::vector<int>> &tabs, int per_item) {
    size_t tot = 0;
    for (auto &t : tabs) {
        pc.off.push_back(tot);
        pc.nwg.push_back((int)(t.size() / per_item));
        tot += t.size();
    }
    std::vector<int> all;
    all.reserve(tot);
    for (auto &t : tabs) all.insert(all.end(), t.begin(), t.end());
    hipError_t e = hipMalloc(&pc.d, std::max<size_t>(tot, 1) * sizeof(int));
    if (e == hipSuccess && tot)
        e = hipMemcpy(pc.d, all.data(), tot * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        free_pieces(pc);
        return fail(BK_ENOMEM, "piece tables: %s", hipGetErrorString(e));
    }
    pc.ok = true;
    return BK_OK;
}

// The k-piece split of this call's Gram (built once per plan / layout and k):
// *out = nullptr when the call's Gram has none (K1 v1, a McNaughton plan
// whose workgroups span pieces, too few row blocks); then the caller computes
// the Gram whole and exchanges it after
int gram_pieces(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld, int k,
                const Pieces **out) {
    *out = nullptr;
    const int64_t usz = bk_upper_elems(n);
    auto finish = [&](Pieces &pc, const std::vector<int> &tile_end) {
        pc.e.assign(1, 0);
        for (size_t p = 0; p < tile_end.size(); ++p)
            pc.e.push_back(p + 1 < tile_end.size() ? (int64_t)tile_end[p] * 4096 : usz);
    };
    if (bk_ctx::I8Cached *e = i8_prepared(c, dX, dtype, n, d, ld)) {
        Pieces &pc = e->pc;
        if (pc.k != k) {
            free_pieces(pc);
            pc.k = k;
            std::vector<int> tile_end;
            std::vector<std::vector<int>> orders;
            if (i8_pieces(e->L, k, tile_end, orders)) {
                CHK(upload_pieces(pc, orders, 2));
                finish(pc, tile_end);
            }
        }
        if (pc.ok) *out = &pc;
        return BK_OK;
    }
    if (!use_v3(c, dX, dtype, ld)) return BK_OK;
    Plan3 *p3 = nullptr;
    const int bk = v3_bk(dtype);
    CHK(get_plan3(c, n, d, bk, &p3));
    for (auto &cp : c->plans)
        if (&cp.p == p3) {
            Pieces &pc = cp.pc;
            if (pc.k != k) {
                free_pieces(pc);
                pc.k = k;
                const Plan3Host H = build_plan3((int)n, d, c->num_cu, bk);
                std::vector<int> tile_end;
                std::vector<std::vector<int>> segs;
                if (plan3_pieces(H, k, tile_end, segs)) {
                    CHK(upload_pieces(pc, segs, 2));
                    finish(pc, tile_end);
                }
            }
            if (pc.ok) *out = &pc;
        }
    return BK_OK;
}

// the context's mapped margin record (allocated once: never moves, so a
// captured graph's pointer to it stays valid)
int margin_rec(bk_ctx *c) {
    if (c->hmargin) return BK_OK;
    void *p = nullptr, *dp = nullptr;
    HIPCHK(hipHostMalloc(&p, 128, hipHostMallocPortable | hipHostMallocMapped |
                                      hipHostMallocNonCoherent));
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) {
        (void)hipHostFree(p);
        return fail(BK_EHIP, "hipHostGetDevicePointer of the margin record failed");
    }
    memset(p, 0, 128);
    c->hmargin = (double *)p;
    c->dmargin = (double *)dp;
    return BK_OK;
}

// Split scoring over the ranks of a sharded call (after the
// exchange every rank holds the whole Gram, and K2 -- n sorts of n distances,
// 0.2 ms at n = 4,096 -- was repeated on every rank): rank r scores rows
// [r ch, r ch + ch), ch = ceil(n / parts), into slice r of a parts x (ch + 1)
// buffer whose last word is the rank's status (0, or NaN when its share
// failed), and ONE in-place RCCL all-gather hands every rank all n scores.
// Each row's score is K2's, bitwise, whichever rank computes it.
// k_split_unpack then copies the scores to the caller's array and hands K3b
// the Gram's trailing record, made NaN if any rank's status is not 0 -- so a
// rank that failed its share marks the call invalid on every rank
// (MARGIN_POISONED), as a shard that fails before the exchange does.  Only on
// the transposed K2 path (n >= 2049), whose contiguous diagonal K3b reads
// instead of the per-row diag K2 writes for its own rows only.
enum { SPLIT_NONE = 0, SPLIT_RCCL = 1, SPLIT_TEST = 2, SPLIT_EMU = 3 };
struct ScoreSplit {
    int mode = SPLIT_NONE;
    int parts = 1, part = 0;
};

ScoreSplit score_split(const bk_ctx *c, int64_t n) {
    ScoreSplit s;
    if (!c->comm || c->split_min_n <= 0 || n < c->split_min_n || !scores_transposed((int)n))
        return s;
    if (c->nranks > 1) {
        s.mode = SPLIT_RCCL;
        s.parts = c->nranks;
        s.part = c->rank;
    } else if (c->test_split_scores > 1) {
        s.mode = SPLIT_TEST;
        s.parts = c->test_split_scores;
    } else if (c->emu_split_scores > 1) {
        s.mode = SPLIT_EMU;
        s.parts = c->emu_split_scores;
    }
    return s;
}

// stage_finish's workspace, allocated before a sharded call's exchange so that
// a failure is caught by the ranks' status agreement: with split scoring
// stage_finish holds a collective, which no rank may skip
int prepare_finish(bk_ctx *c, int64_t n, const ScoreSplit &sp, bool own_scores) {
    if (sp.parts > 1) {  // first: a rank that fails below can still join the all-gather
        const int64_t ch = (n + sp.parts - 1) / sp.parts;
        CHK(ensure(c->sgather, ((size_t)(ch + 1) * sp.parts + 3) * sizeof(double)));
    }
    CHK(ensure(c->mask, (size_t)n * sizeof(int)));
    if (own_scores) CHK(ensure(c->scores, (size_t)n * sizeof(double)));
    CHK(ensure(c->diag, (size_t)n * sizeof(double)));
    CHK(ensure(c->bnd, 2 * sizeof(double)));
    CHK(margin_rec(c));
    const int T = (int)((n + 63) / 64);
    if (scores_transposed((int)n))
        CHK(ensure(c->Ut, ((size_t)T * (T + 1) / 2 * 4096 + (size_t)T * 64) * sizeof(double)));
    return BK_OK;
}

// a rank whose finish failed before its share still joins the score
// all-gather with a NaN status, so its peers mark the call invalid instead of
// waiting for it.  The gather buffer exists: it is sized by (n, ranks) alone
// and allocated first, on the call whose signature the ranks agreed on
void join_failed_share(bk_ctx *c, int64_t n, const ScoreSplit &sp) {
    const int64_t ch = (n + sp.parts - 1) / sp.parts;
    if (c->sgather.bytes < ((size_t)(ch + 1) * sp.parts + 3) * sizeof(double)) return;
    double *sg = (double *)c->sgather.p;
    (void)hipMemsetAsync(sg + (size_t)sp.part * (ch + 1) + ch, 0xFF, sizeof(double), c->stream);
    (void)ncclAllGather(sg + (size_t)sp.part * (ch + 1), sg, (size_t)(ch + 1), ncclDouble, c->comm,
                        c->stream);
}

// K2 + K3 + K4 from a packed upper Gram
int stage_finish(bk_ctx *c, const double *U, const Plan &pl, const void *dX, int dtype,
                 int64_t n, int64_t d, int64_t ld, int64_t f, int64_t *d_sel, double *d_scores,
                 double *d_mean, const ScoreSplit &sp = ScoreSplit()) {
    {
        const int pf = prepare_finish(c, n, sp, d_scores == nullptr);
        if (pf != BK_OK) {
            if (sp.mode == SPLIT_RCCL) {
                const std::string msg = g_err;
                join_failed_share(c, n, sp);
                g_err = msg;
            }
            return pf;
        }
    }
    double *sc = d_scores ? d_scores : (double *)c->scores.p;
    int *mask = (int *)c->mask.p;
    double *diag = (double *)c->diag.p, *bnd = (double *)c->bnd.p;
    const int64_t m = n - f;
    const int64_t k = n - f - 2 > 0 ? n - f - 2 : 0;
    // the packed upper's trailing record {column count, columns on the fp32
    // MFMA, int8 error bound, 0}: the margin's d, unit roundoff and absolute
    // Gram error, totals after an exchange
    const double *dcols = U + (size_t)pl.ntile * 4096;
    const double *Ut = nullptr, *dg = nullptr;
    int st = BK_OK;
    if (scores_transposed((int)n)) {
        // large n: transposed off-diagonal tiles + contiguous diagonal, so K2
        // reads rows in 512-B runs (the packed upper's lower half is strided)
        // (split scoring: each share transposes only what its rows read, below)
        const size_t tiles = (size_t)pl.ntile * 4096;
        double *ut = (double *)c->Ut.p;
        if (sp.parts <= 1)
            st = timed(c, BK_K_EXPAND, [&] { return launch_transpose(U, pl.T, ut, ut + tiles, c->stream); });
        Ut = ut;
        dg = ut + tiles;
    }
    if (sp.parts <= 1) {
        CHK(st);
        CHK(timed(c, BK_K_SCORES,
                  [&] { return launch_scores(U, Ut, dg, pl.T, (int)n, k, sc, diag, c->stream); }));
        CHK(timed(c, BK_K_RANK,
                  [&] { return launch_rank(sc, (int)n, (int)m, mask, bnd, c->stream); }));
    } else {
        const int64_t ch = (n + sp.parts - 1) / sp.parts;
        double *sg = (double *)c->sgather.p;
        // share p: the transposed tiles its rows read (block-columns of rows
        // [r0, r1), and the whole diagonal), then its K2, which writes
        // scores[i] of its rows through sg + p, i.e. at p (ch + 1) + (i - p ch);
        // its status word follows at p (ch + 1) + ch
        auto share = [&](int p, bool ok) {
            const int64_t r0 = (int64_t)p * ch, r1 = r0 + ch < n ? r0 + ch : n;
            int s2 = ok ? BK_OK : BK_EHIP;
            if (s2 == BK_OK) {
                const int b0 = r1 > r0 ? (int)(r0 >> 6) : 1, b1 = r1 > r0 ? (int)((r1 - 1) >> 6) : 0;
                double *ut = const_cast<double *>(Ut);
                s2 = timed(c, BK_K_EXPAND, [&] {
                    return launch_transpose(U, pl.T, ut, const_cast<double *>(dg), c->stream, b0, b1);
                });
            }
            if (s2 == BK_OK && r1 > r0)
                s2 = timed(c, BK_K_SCORES, [&] {
                    return launch_scores(U, Ut, dg, pl.T, (int)n, k, sg + p, diag, c->stream,
                                         (int)r0, (int)(r1 - r0));
                });
            const hipError_t e = hipMemsetAsync(sg + (size_t)p * (ch + 1) + ch, s2 == BK_OK ? 0 : 0xFF,
                                                sizeof(double), c->stream);
            if (s2 == BK_OK && e != hipSuccess)
                s2 = fail(BK_EHIP, "hipMemsetAsync: %s", hipGetErrorString(e));
            return s2;
        };
        if (sp.mode == SPLIT_RCCL) {
            // every rank joins the all-gather, whatever happened to its share
            // (test knob BK_TEST_SPLIT_FAIL=p: this rank's share fails when p - 1
            // is its rank -- tests/test_gpu_rccl_ranks.py, >= 2 GPUs)
            if (st == BK_OK && c->test_split_fail == sp.part + 1)
                st = fail(BK_EHIP, "test knob BK_TEST_SPLIT_FAIL=%d: this rank's share fails",
                          c->test_split_fail);
            const std::string pre = st == BK_OK ? std::string() : g_err;
            const int s2 = share(sp.part, st == BK_OK);
            if (st == BK_OK) st = s2;
            const std::string msg = st == BK_OK ? std::string() : (pre.empty() ? g_err : pre);
            // (timing is best effort here: nothing may keep a rank from the collective)
            hipEvent_t a = nullptr, b = nullptr;
            bool ton = timing_on(c, BK_K_SCORE_GATHER);
            if (ton) {
                const std::string keep = g_err;
                ton = get_event(c, &a) == BK_OK && get_event(c, &b) == BK_OK &&
                      hipEventRecord(a, c->stream) == hipSuccess;
                if (!ton) {
                    if (a) c->pool.push_back(a);
                    if (b) c->pool.push_back(b);
                    g_err = keep;
                }
            }
            RCCLCHK(ncclAllGather(sg + (size_t)sp.part * (ch + 1), sg, (size_t)(ch + 1), ncclDouble,
                                  c->comm, c->stream));
            if (ton) {
                HIPCHK(hipEventRecord(b, c->stream));
                c->pending.push_back({BK_K_SCORE_GATHER, a, b});
            }
            if (st != BK_OK) {
                g_err = msg;
                return st;
            }
        } else {
            CHK(st);
            // one GPU standing in for the ranks: every share (test), or rank
            // 0's once a mode's first call has scored them all (timing
            // emulation: the other shares' scores are that first call's)
            const bool all = sp.mode == SPLIT_TEST || c->emu_split_n != n;
            for (int p = 0; p < sp.parts; ++p) {
                // (test: a share that "fails" is another rank's failure seen
                // from this one -- its NaN status poisons the record below)
                const bool ok = !(sp.mode == SPLIT_TEST && c->test_split_fail == p + 1);
                if (all || p == 0) {
                    const int s2 = share(p, ok);
                    if (ok) CHK(s2);
                }
            }
            if (sp.mode == SPLIT_EMU) c->emu_split_n = n;
        }
        double *rec = sg + (size_t)(ch + 1) * sp.parts;
        HIPCHK(launch_split_unpack(sg, ch, sp.parts, (int)n, dcols, sc, rec, c->stream));
        dcols = rec;
        CHK(timed(c, BK_K_RANK,
                  [&] { return launch_rank(sc, (int)n, (int)m, mask, bnd, c->stream); }));
        diag = const_cast<double *>(dg);  // K2 wrote only its own rows' diag
    }
    CHK(timed(c, BK_K_COMPACT, [&] {
        return launch_compact(mask, (int)n, d_sel, diag, bnd, dcols, k, c->dmargin, c->stream);
    }));
    c->margin_valid = 1;
    c->margin_host = c->hmargin;
    c->margin_unchecked = 1;
    if (d_mean && d > 0) {
        double *seg = nullptr;
        if (mean_segments((int)m) > 1) {
            CHK(ensure(c->mean_part, (size_t)mean_segments((int)m) * (size_t)d * sizeof(double)));
            seg = (double *)c->mean_part.p;
        }
        CHK(timed(c, BK_K_MEAN, [&] {
            return launch_mean(dX, dtype, ld, d, d_sel, (int)m, d_mean, c->num_cu, c->stream, seg);
        }));
    }
    return BK_OK;
}

// k_small (bk_small.hip) takes the whole call for Biscotti's deployed shapes:
// n <= 128 (one 16x16-block grid per wave set) and d small enough that one
// launch beats the chain
bool small_ok(const bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld) {
    static const int64_t dmax = [] {
        const char *e = getenv("BK_SMALL_MAX_D");  // may only lower the cap
        const int64_t v = e ? atoll(e) : (int64_t)32768;
        return v < 32768 ? v : (int64_t)32768;  // d / 64 chunks: <= 1024 G items (k_small's groups)
    }();
    (void)dX;
    (void)dtype;
    (void)ld;  // unaligned rows take k_small's scalar-load variant
    return c->small_on && n <= 128 && d <= dmax;
}

// margin_out / scores_out: the host entry's mapped output block (the record
// and a second copy of the scores written by the kernel straight to host memory)
// g0 / gn / sm: this launch's share -- the G items of chunks [g0, g0 + gn)
// and, with sm, the S and M items (the pipelined host entry, below); the
// default is the whole call in one launch
int run_small(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld, int64_t f,
              int64_t *d_sel, double *d_scores, double *d_mean, double *margin_out = nullptr,
              double *scores_out = nullptr, int g0 = 0, int gn = -1, bool sm = true) {
    const SmallPlan sp = small_plan((int)n, d, c->num_cu);
    if (!c->small_ctr.p) {
        CHK(ensure(c->small_ctr, SMALL_CTR_WORDS * sizeof(unsigned)));
        HIPCHK(hipMemsetAsync(c->small_ctr.p, 0, SMALL_CTR_WORDS * sizeof(unsigned), c->stream));
    }
    // per chunk: the full-square partial Gram (16 nb16)^2 + its diagonal (bk_small.hip)
    const size_t np16 = (size_t)16 * sp.nb16;
    CHK(ensure(c->small_part, (size_t)sp.P * (np16 * np16 + np16) * sizeof(double)));
    CHK(ensure(c->U, (size_t)bk_upper_elems(n) * sizeof(double)));
    CHK(ensure(c->diag, (size_t)n * sizeof(double)));
    CHK(margin_rec(c));
    double *sc = d_scores;
    if (!sc) {
        CHK(ensure(c->scores, (size_t)n * sizeof(double)));
        sc = (double *)c->scores.p;
    }
    long long *trace = nullptr;
    const int items = SMALL_SPLIT_ITEMS * (gn < 0 ? sp.P : gn) + (sm ? sp.nS + (d_mean ? sp.C : 1) : 0);
    const int grid = items < c->num_cu ? items : c->num_cu;  // = launch_small's grid
    const size_t twords = (size_t)items * 8 + (size_t)grid * 2;  // + per workgroup {entry, exit}
    const char *tfile = probe_env("BK_SMALL_TRACE");  // debug: per-item timeline
    if (tfile) {
        CHK(ensure(c->trace, twords * sizeof(long long)));
        HIPCHK(hipMemsetAsync(c->trace.p, 0, twords * sizeof(long long), c->stream));
        trace = (long long *)c->trace.p;
    }
    // (the test knob's count goes to launches that wait: a G-only launch has no hand-off)
    const uint64_t spin = c->small_spin_left == 0 || !sm ? SMALL_SPIN_MAX : c->small_spin_max;
    if (c->small_spin_left > 0 && sm) --c->small_spin_left;
    CHK(timed(c, BK_K_SMALL, [&] {
        return launch_small(dX, dtype, ld, (int)n, d, (int)f, sp, (double *)c->small_part.p,
                            (double *)c->U.p, sc, (double *)c->diag.p, d_sel, d_mean,
                            margin_out ? margin_out : c->dmargin,
                            (unsigned *)c->small_ctr.p, c->num_cu, c->stream, trace, spin,
                            c->small_check_lines, scores_out, g0, gn, sm);
    }));
    if (sm) {
        c->margin_valid = 1;
        c->margin_host = margin_out ? c->hout_host_margin : c->hmargin;
        c->margin_unchecked = 1;
    }
    if (tfile) {
        std::vector<long long> h(twords + 6);
        h[0] = items;
        h[1] = SMALL_SPLIT_ITEMS * (gn < 0 ? sp.P : gn);  // G items
        h[2] = sp.Q;
        h[3] = sm ? sp.nS : 0;
        h[4] = sm ? (d_mean ? sp.C : 1) : 0;
        h[5] = grid;
        HIPCHK(hipMemcpyAsync(h.data() + 6, trace, twords * sizeof(long long),
                              hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (FILE *fp = fopen(tfile, "ab")) {
            fwrite(h.data(), sizeof(long long), h.size(), fp);
            fclose(fp);
        }
    }
    return BK_OK;
}

int run_device(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld, int64_t f,
               int64_t *d_sel, double *d_scores, double *d_mean) {
    if (small_ok(c, dX, dtype, n, d, ld))
        return run_small(c, dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean);
    Plan pl;
    const size_t usz = (size_t)bk_upper_elems(n);
    CHK(ensure(c->U, usz * sizeof(double)));
    double *U = (double *)c->U.p;
    CHK(stage_gram(c, dX, dtype, n, d, ld, U, pl));
    return stage_finish(c, U, pl, dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean);
}

// Wait for the context's stream: poll it for up to spin_us, then block.  A
// blocking wait sleeps the host thread until the GPU's completion interrupt;
// after the GPU has idled that wake-up was 40-75 us of a config-B call
// (tools/idle_probe.py: device-resident call after 200 ms idle 152 -> 77 us,
// host entry 229 -> 186 us, with the whole process set to spin).  Polling
// only inside libbk's own waits keeps that without a process-wide flag, and
// the cap bounds the CPU a long call (config D's 76 ms host entry) burns.
// The final hipStreamSynchronize returns at once on a finished stream.
hipError_t wait_stream(bk_ctx *c) {
    if (c->spin_us > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        const auto cap = std::chrono::microseconds(c->spin_us);
        for (;;) {
            const hipError_t q = hipStreamQuery(c->stream);
            if (q != hipErrorNotReady) {
                if (q != hipSuccess) return q;
                break;
            }
            if (std::chrono::steady_clock::now() - t0 > cap) break;
        }
    }
    return hipStreamSynchronize(c->stream);
}

// the error codes a finish can leave in margin[2] (bk_internal.h MARGIN_*)
int margin_status(const double *mg) {
    if (mg[2] == MARGIN_HANDOFF_TIMEOUT)
        return fail(BK_EHIP, "k_small: a hand-off wait timed out; the call's outputs are invalid "
                             "(sel entries are -1)");
    if (mg[2] == MARGIN_POISONED)
        return fail(BK_ERCCL, "a rank failed before the Gram exchange and poisoned its partial; "
                              "the call's outputs are invalid");
    if (mg[2] == MARGIN_QUEUE_DIRTY)
        return fail(BK_EHIP, "k_small: a queue word other than word 0 of its line was written "
                             "(BK_SMALL_CHECK_LINES)");
    return BK_OK;
}

// the last finish's margin record (k_compact: gap, err_bound, near_tie, M,
// s_lo, s_hi, d, k, then u_G), synchronously
int read_margin(bk_ctx *c, double (&mg)[MARGIN_WORDS]) {
    if (!c->margin_valid || !c->margin_host)
        return fail(BK_EINVAL, "no Multi-Krum call on this context yet");
    // the record sits in mapped host memory (the context's, or the n <= 128
    // host entry's output block): once the stream is done it is readable
    HIPCHK(wait_stream(c));
    memcpy(mg, c->margin_host, sizeof mg);
    c->margin_unchecked = 0;
    return margin_status(mg);
}

// Synchronous host entries: once their stream has synchronized, the record's
// error codes are checked (it is already in host memory)
int check_margin_readback(bk_ctx *c) {
    c->margin_unchecked = 0;
    return margin_status(c->margin_host);
}

// Error paths of the host entries: queued H2D copies may still read the
// caller's buffers, so both streams are drained unless the entry disarms this.
struct HostDrain {
    bk_ctx *c;
    bool armed = true;
    ~HostDrain() {
        if (!armed) return;
        if (c->copy) (void)hipStreamSynchronize(c->copy);
        (void)hipStreamSynchronize(c->stream);
    }
};

// the host entries' copy stream and its five events, created once: into locals,
// published together (a half-built set would break every later host call)
int ensure_copy_stream(bk_ctx *c) {
    if (c->copy) return BK_OK;
    hipStream_t cs = nullptr;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    hipError_t e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    for (int i = 0; i < 5 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        for (hipEvent_t x : ev)
            if (x) (void)hipEventDestroy(x);
        if (cs) (void)hipStreamDestroy(cs);
        return fail(BK_EHIP, "copy stream / events: %s", hipGetErrorString(e));
    }
    c->copy = cs;
    c->ev_go = ev[0];
    c->ev_cp[0] = ev[1];
    c->ev_cp[1] = ev[2];
    c->ev_use[0] = ev[3];
    c->ev_use[1] = ev[4];
    return BK_OK;
}

// The host entries' column chunk width: ~BK_STAGE_CHUNK_BYTES (default 256
// MiB) of the batch plus its k noise vectors per chunk, a multiple of 64
// columns (16-B aligned chunk starts), at most 64 chunks (every chunk writes
// and adds one packed partial Gram -- n^2/2 doubles, 1 GiB at n = 16384 --
// which must stay small against its copy).  bk_multikrum and
// bk_multikrum_rows chunk alike, so their chunk Grams sum in the same order.
int64_t host_chunk_cols(int64_t n, size_t es, int64_t k, int64_t d) {
    int64_t cap = (int64_t)256 << 20;
    if (const char *v = getenv("BK_STAGE_CHUNK_BYTES")) cap = atoll(v) > 0 ? atoll(v) : cap;
    const int64_t col_bytes = n * (int64_t)es + n * k * (int64_t)sizeof(double);
    int64_t W = cap / col_bytes;
    W = W < (d + 63) / 64 ? (d + 63) / 64 : W;
    W = W < 64 ? 64 : (W + 63) / 64 * 64;
    return W >= d ? d : W;
}

// Host entries (bk_multikrum, bk_multikrum_noised): the batch crosses PCIe in
// column chunks on a copy stream, and each chunk's partial Gram (K1 + K1b,
// after K6 when noise is applied) runs on the compute stream while the next
// chunk is in flight.  The Gram is additive over columns, so only the last
// chunk's K1 and the finish remain after the copies; the chunk partials are
// added to a running sum in chunk order (deterministic).  Noise: vector j of update i at
// noise + (i*k + j) * noise_ld, staged per chunk in a 2-slot device ring.
// On return (async) the device batch dX (row stride dld) is complete and
// noised and U holds the full packed Gram; pl describes it for stage_finish.
int stage_host_pipelined(bk_ctx *c, const void *X, int64_t ld, int dtype, const double *noise,
                         int64_t k, int64_t noise_ld, int64_t n, int64_t d, char *dX,
                         int64_t dld, double *U, Plan &pl) {
    const size_t es = esize(dtype);
    CHK(ensure_copy_stream(c));
    const int64_t W = host_chunk_cols(n, es, k, d);
    const int64_t C = (d + W - 1) / W;
    const size_t usz = (size_t)bk_upper_elems(n);
    double *P = nullptr;
    if (C > 1) {
        CHK(ensure(c->Ug, usz * sizeof(double)));
        P = (double *)c->Ug.p;
    }
    double *ring = nullptr;
    if (k > 0) {
        CHK(ensure(c->noise, (size_t)2 * n * k * W * sizeof(double)));
        ring = (double *)c->noise.p;
    }
    // on an error return, copies already queued may still read the caller's
    // host buffers: drain both streams before handing control back
    HostDrain drain{c};
    // earlier work on the compute stream may still read the batch / the ring
    HIPCHK(hipEventRecord(c->ev_go, c->stream));
    HIPCHK(hipStreamWaitEvent(c->copy, c->ev_go, 0));
    for (int64_t ch = 0; ch < C; ++ch) {
        const int64_t c0 = ch * W, wc = d - c0 < W ? d - c0 : W;
        const int s = (int)(ch & 1);
        double *slot = ring ? ring + (size_t)s * n * k * W : nullptr;
        if (ch >= 2 && k > 0) HIPCHK(hipStreamWaitEvent(c->copy, c->ev_use[s], 0));
        HIPCHK(hipMemcpy2DAsync(dX + c0 * es, (size_t)dld * es, (const char *)X + c0 * es,
                                (size_t)ld * es, (size_t)wc * es, (size_t)n,
                                hipMemcpyHostToDevice, c->copy));
        if (k > 0)
            HIPCHK(hipMemcpy2DAsync(slot, (size_t)wc * 8, noise + c0, (size_t)noise_ld * 8,
                                    (size_t)wc * 8, (size_t)(n * k), hipMemcpyHostToDevice,
                                    c->copy));
        HIPCHK(hipEventRecord(c->ev_cp[s], c->copy));
        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_cp[s], 0));
        double *xc = (double *)(dX + c0 * es);
        if (k > 0) {
            CHK(timed(c, BK_K_NOISE, [&] {
                return launch_noise(xc, dld, n, wc, slot, k, wc, xc, dld, c->num_cu, c->stream);
            }));
            HIPCHK(hipEventRecord(c->ev_use[s], c->stream));
        }
        // chunk 0 straight into U, later chunks added in chunk order
        CHK(stage_gram(c, dX + c0 * es, dtype, n, wc, dld, ch == 0 ? U : P, pl));
        if (ch > 0) HIPCHK(launch_add_upper(U, P, (int64_t)usz, c->stream));
    }
    pl.d = d;
    drain.armed = false;
    return BK_OK;
}

// K2..K4 on a batch staged by stage_host_pipelined, then the outputs back to
// the caller's host arrays (bk_multikrum, bk_multikrum_noised)
int run_host_outputs(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t dld,
                     int64_t f, const double *U, const Plan &pl, int64_t *sel_idx,
                     int64_t *m_out, double *scores, double *mean_out) {
    HostDrain drain{c};
    const int64_t m = n - f;
    CHK(ensure(c->sel, (size_t)n * sizeof(int64_t)));
    CHK(ensure(c->scores, (size_t)n * sizeof(double)));
    if (mean_out) CHK(ensure(c->mean, (size_t)d * sizeof(double)));
    int64_t *dsel = (int64_t *)c->sel.p;
    double *dsc = (double *)c->scores.p;
    double *dmean = mean_out ? (double *)c->mean.p : nullptr;
    CHK(stage_finish(c, U, pl, dX, dtype, n, d, dld, f, dsel, dsc, dmean));
    CHK(timed(c, BK_K_D2H, [&] {
        hipError_t e = hipMemcpyAsync(sel_idx, dsel, (size_t)m * sizeof(int64_t),
                                      hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess && scores)
            e = hipMemcpyAsync(scores, dsc, (size_t)n * sizeof(double), hipMemcpyDeviceToHost,
                               c->stream);
        if (e == hipSuccess && mean_out)
            e = hipMemcpyAsync(mean_out, dmean, (size_t)d * sizeof(double), hipMemcpyDeviceToHost,
                               c->stream);
        return e;
    }));
    HIPCHK(wait_stream(c));
    drain.armed = false;
    CHK(check_margin_readback(c));
    if (m_out) *m_out = m;
    return BK_OK;
}

// Host batches of Biscotti's deployed shapes (n <= 128: configs A and B, the
// mnist and creditcard verifiers) take the one-launch k_small / k_tiny path:
// ONE H2D of the 16-B-padded batch on the compute stream (<= 32 MiB: no column
// chunks, no copy stream), the noise added in place by K6 when the verifier
// noises the batch itself, the kernel, then the outputs and the margin record
// back, one synchronize.  The device-resident entry's arithmetic, so the same
// bits.  where == BK_DEVICE skips the copy, and so does a pinned batch that
// k_tiny reads over PCIe itself (below).
int run_host_small(bk_ctx *c, const void *X, int where, int64_t ld, int dtype, const double *noise,
                   int64_t k, int64_t noise_ld, int64_t n, int64_t d, int64_t f, int64_t *sel_idx,
                   int64_t *m_out, double *scores, double *mean_out, double *noised_out,
                   int64_t out_ld) {
    const size_t es = esize(dtype);
    const int64_t m = n - f;
    HostDrain drain{c};
    const void *dX = X;
    int64_t dld = ld;
    // a batch k_tiny takes whole (n <= 16, d <= 128: config A, a few KB) is
    // read by the kernel itself straight from the caller's pinned memory over
    // PCIe: no H2D copy, whose DMA set-up (~20 us) was most of the call
    // (BK_TINY_ZERO_COPY=0 copies it as before, for A/B)
    static const bool tiny_zc = [] {
        const char *e = getenv("BK_TINY_ZERO_COPY");
        return !(e && atoi(e) == 0);
    }();
    bool zero_copy = false;
    if (where == BK_HOST_PINNED && k == 0 && !noised_out && tiny_zc && tiny_ok((int)n, d) &&
        !probe_env("BK_SMALL_TRACE")) {
        void *hp = nullptr;
        if (hipHostGetDevicePointer(&hp, const_cast<void *>(X), 0) == hipSuccess && hp) {
            dX = hp;
            zero_copy = true;
        } else {
            (void)hipGetLastError();  // not mapped (pinned by other means): copy it
        }
    }
    // BK_SMALL_PIPE=<chunks> (A/B; default 0): the copy in that many column
    // chunks on the copy stream, each chunk's G items launched on the compute
    // stream as soon as it has landed (an event, no spinning), then one S + M
    // launch -- the same items and partials as the one-launch call, the same
    // bits.  Measured at config B (r4, tools/host_entry_ab.py): 0.157 ms per
    // call with one copy, 0.201 with 2 chunks, 0.234 with 4 -- a strided
    // column-chunk H2D and its launch cost more than the Gram they hide
    // (~14 us), so the one copy + one launch stays the default
    static const int pipe_env = [] {
        const char *e = getenv("BK_SMALL_PIPE");
        return e ? atoi(e) : 0;
    }();
    const SmallPlan sp = small_plan((int)n, d, c->num_cu);
    int nc = 0;
    if (where != BK_DEVICE && !zero_copy && k == 0 && !noised_out && !tiny_ok((int)n, d) &&
        !probe_env("BK_SMALL_TRACE") && pipe_env >= 2 && sp.P >= 2 * pipe_env)
        nc = pipe_env;
    if (nc) {
        const int64_t epg = (int64_t)(16 / es);
        dld = (d + epg - 1) / epg * epg;
        CHK(ensure(c->X, (size_t)n * dld * es));
        CHK(ensure_copy_stream(c));
        char *dx = (char *)c->X.p;
        // earlier work on the compute stream may still read the device batch
        HIPCHK(hipEventRecord(c->ev_go, c->stream));
        HIPCHK(hipStreamWaitEvent(c->copy, c->ev_go, 0));
        for (int q = 0; q < nc; ++q) {
            const int a0 = (int)((int64_t)sp.P * q / nc), a1 = (int)((int64_t)sp.P * (q + 1) / nc);
            const int64_t c0 = (int64_t)a0 * sp.kc, c1 = std::min<int64_t>((int64_t)a1 * sp.kc, d);
            HIPCHK(hipMemcpy2DAsync(dx + c0 * es, (size_t)dld * es, (const char *)X + c0 * es,
                                    (size_t)ld * es, (size_t)(c1 - c0) * es, (size_t)n,
                                    hipMemcpyHostToDevice, c->copy));
            HIPCHK(hipEventRecord(c->ev_cp[q & 1], c->copy));
            HIPCHK(hipStreamWaitEvent(c->stream, c->ev_cp[q & 1], 0));
            CHK(run_small(c, dx, dtype, n, d, dld, f, nullptr, nullptr, nullptr, nullptr, nullptr,
                          a0, a1 - a0, false));
        }
        dX = dx;
    }
    if (where != BK_DEVICE && !zero_copy && !nc) {
        const int64_t epg = (int64_t)(16 / es);
        dld = (d + epg - 1) / epg * epg;
        CHK(ensure(c->X, (size_t)n * dld * es));
        if (k > 0) CHK(ensure(c->noise, (size_t)n * k * d * sizeof(double)));
        CHK(timed(c, BK_K_H2D, [&] {
            // a contiguous batch (ld == d) whose rows are already 16-B
            // multiples (ld == dld): one linear copy.  A strided caller with
            // ld == dld != d (a numpy view X[:, :3] of an n x 4 array) takes
            // the 2-D copy: a linear n * d copy would shift every row after
            // the first
            hipError_t e = ld == dld && ld == d ? hipMemcpyAsync(c->X.p, X, (size_t)n * d * es,
                                                      hipMemcpyHostToDevice, c->stream)
                                     : hipMemcpy2DAsync(c->X.p, (size_t)dld * es, X,
                                                        (size_t)ld * es, (size_t)d * es, (size_t)n,
                                                        hipMemcpyHostToDevice, c->stream);
            if (e == hipSuccess && k > 0)
                e = hipMemcpy2DAsync(c->noise.p, (size_t)d * 8, noise, (size_t)noise_ld * 8,
                                     (size_t)d * 8, (size_t)(n * k), hipMemcpyHostToDevice,
                                     c->stream);
            return e;
        }));
        if (k > 0) {
            double *xd = (double *)c->X.p;
            CHK(timed(c, BK_K_NOISE, [&] {
                return launch_noise(xd, dld, n, d, (const double *)c->noise.p, k, d, xd, dld,
                                    c->num_cu, c->stream);
            }));
        }
        if (noised_out)
            HIPCHK(hipMemcpy2DAsync(noised_out, (size_t)out_ld * 8, c->X.p, (size_t)dld * 8,
                                    (size_t)d * 8, (size_t)n, hipMemcpyDeviceToHost, c->stream));
        dX = c->X.p;
    }
    // the outputs {margin (16 doubles), sel (n), scores (n), mean (d)} are
    // written by the kernel itself into one mapped pinned block:
    // no device-to-host copy after the kernel (a D2H costs ~15 us of PCIe
    // round trip at config B, more than the 63 KB it moves), one synchronize,
    // then copied to the caller's arrays on the host
    constexpr size_t MPAD = 16;
    const size_t words = MPAD + 2 * (size_t)n + (mean_out ? (size_t)d : 0);
    if (c->hout_bytes < words * sizeof(double)) {
        // an earlier asynchronous call's record may be unchecked: if it lives
        // in the block about to be freed, read it first (its stream is done
        // once wait_stream returns); a record in the context's own block stays
        if (c->margin_host && c->margin_host == c->hout_host_margin) {
            HIPCHK(wait_stream(c));
            if (c->margin_unchecked) {
                c->margin_unchecked = 0;
                CHK(margin_status(c->margin_host));
            }
            c->margin_host = nullptr;
            c->margin_valid = 0;
        }
        if (c->hout) (void)hipHostFree(c->hout);
        c->hout = nullptr;
        c->hout_bytes = 0;
        c->hout_dev = nullptr;
        c->hout_host_margin = nullptr;
        const size_t bytes = std::max<size_t>(words * sizeof(double), 64 * 1024);
#ifdef BK_HOUT_COHERENT  // ablation: uncached host block (each store crosses PCIe at once)
        const unsigned hflags = hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent;
#else  // GPU-cached, written back at the kernel's end: 156 vs 157 us per call at B
        const unsigned hflags = hipHostMallocPortable | hipHostMallocMapped | hipHostMallocNonCoherent;
#endif
        HIPCHK(hipHostMalloc(&c->hout, bytes, hflags));
        c->hout_bytes = bytes;
        void *dp = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dp, c->hout, 0));
        c->hout_dev = (double *)dp;
        c->hout_host_margin = (const double *)c->hout;
    }
    double *blk = c->hout_dev;
    int64_t *dsel = (int64_t *)(blk + MPAD);
    double *dmean = mean_out ? blk + MPAD + 2 * n : nullptr;
    CHK(run_small(c, dX, dtype, n, d, dld, f, dsel, nullptr, dmean, blk,
                  scores ? blk + MPAD + n : nullptr, 0, nc ? 0 : -1, true));
    HIPCHK(wait_stream(c));
    drain.armed = false;
    const double *h = (const double *)c->hout;
    c->margin_unchecked = 0;
    CHK(margin_status(h));
    memcpy(sel_idx, h + MPAD, (size_t)m * sizeof(int64_t));
    if (scores) memcpy(scores, h + MPAD + n, (size_t)n * sizeof(double));
    if (mean_out) memcpy(mean_out, h + MPAD + 2 * n, (size_t)d * sizeof(double));
    if (m_out) *m_out = m;
    return BK_OK;
}

// ---- the row-fed host entry (bk_multikrum_rows) ----------------------------
// Biscotti's verifier holds the batch as n separately allocated host rows
// (getTopKRUMIndex(deltas [][]float64), krum.go:100-166; each row a peer's
// RPC-decoded slice).  Before anything crosses PCIe the rows must be in
// pinned memory.  The cgo shim used to pack them serially into a pinned batch
// (one core, 4.3 GB at config D) and only then call bk_multikrum; here the
// packing runs on several host threads into a ring of pinned slots, and each
// slot's H2D (and the Gram of its columns) starts as soon as it is full.

// packing threads, the caller's included: bk_set_host_threads, else
// BK_HOST_THREADS, else min(8, the host's hardware threads) -- config D's
// pack keeps ahead of PCIe from 4 threads on (78-79 ms per call at 4, 8 and
// 16), and more threads only compete for the process's CPU share
int host_threads(const bk_ctx *c) {
    if (c->hthreads > 0) return c->hthreads;
    static const int def = [] {
        if (const char *v = getenv("BK_HOST_THREADS"))
            if (atoi(v) > 0) return std::min(atoi(v), 256);
        const unsigned hw = std::thread::hardware_concurrency();
        return (int)std::max(1u, std::min(8u, hw ? hw : 1u));
    }();
    return def;
}

// the context's worker pool (threads - 1 workers), or nullptr when the caller
// packs alone (one thread, or the workers could not be started)
bk::HostPool *get_pool(bk_ctx *c) {
    const int t = host_threads(c);
    if (c->hpool && c->hpool->workers() == t - 1) return c->hpool;
    delete c->hpool;
    c->hpool = nullptr;
    if (t <= 1) return nullptr;
    try {
        c->hpool = new bk::HostPool(t - 1);
    } catch (...) {
        c->hpool = nullptr;
    }
    return c->hpool;
}

// one packing job on the pool for the lifetime of this object: the pool's
// end() runs on every return path, so no worker still uses the job function
// (on the caller's stack) or writes into the stage after the entry returns
struct PoolJob {
    bk::HostPool *pool;
    PoolJob(bk::HostPool *p, int nitems, const std::function<void(int)> *fn) : pool(p) {
        if (pool) pool->begin(nitems, fn);
    }
    ~PoolJob() {
        if (pool) pool->end();
    }
};

// the pack's stores: non-temporal for the column-chunk ring (GBs streamed
// through it: the stores bypass the caches), cached memcpy for the small
// path's stage (<= 32 MiB, re-used every call: it stays in the L3, and r6's
// sweep at config B gave ~0.195 ms per call against ~0.205 non-temporal);
// BK_ROWS_COPY=nt|memcpy forces one (an A/B of the same bytes)
bool rows_copy_nt(bool dflt) {
    const char *e = getenv("BK_ROWS_COPY");
    if (e && strcmp(e, "memcpy") == 0) return false;
    if (e && strcmp(e, "nt") == 0) return true;
    return dflt;
}

// the pinned ring (grow-only; every call is synchronous, so no copy from the
// old ring is in flight when it is replaced)
int ensure_rows_stage(bk_ctx *c, size_t bytes) {
    if (c->rstage_bytes >= bytes) return BK_OK;
    if (c->rstage) (void)hipHostFree(c->rstage);
    c->rstage = nullptr;
    c->rstage_bytes = 0;
    HIPCHK(hipHostMalloc(&c->rstage, bytes, hipHostMallocPortable | hipHostMallocMapped));
    c->rstage_bytes = bytes;
    return BK_OK;
}

int ensure_rows_events(bk_ctx *c) {
    for (hipEvent_t &e : c->ev_rows)
        if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return BK_OK;
}

// Column chunks of the batch through a ring of S <= 3 pinned slots: chunk ch
// (columns [ch W, ch W + W)) is packed by the pool into slot ch mod S (row
// blocks of ~2 MiB are the items), crosses PCIe on the copy stream into the
// device batch dX (row stride dld), and its partial Gram runs on the compute
// stream, as in stage_host_pipelined.  A slot is handed back to the packers
// when its copy has landed, so the packing of chunks ch + 1 .. ch + S - 1
// overlaps the copy of chunk ch.  The chunks are bk_multikrum's
// (host_chunk_cols), summed in the same order: every output is bitwise that of
// bk_multikrum on the rows packed into one pinned batch.
int stage_rows_pipelined(bk_ctx *c, const char *const *rows, int dtype, int64_t n, int64_t d,
                         char *dX, int64_t dld, double *U, Plan &pl) {
    const size_t es = esize(dtype);
    CHK(ensure_copy_stream(c));
    CHK(ensure_rows_events(c));
    const int64_t W = host_chunk_cols(n, es, 0, d);
    const int64_t C = (d + W - 1) / W;
    const int S = (int)std::min<int64_t>(C, 3);
    const size_t slot = (size_t)n * W * es;
    CHK(ensure_rows_stage(c, slot * S));
    const size_t usz = (size_t)bk_upper_elems(n);
    double *P = nullptr;
    if (C > 1) {
        CHK(ensure(c->Ug, usz * sizeof(double)));
        P = (double *)c->Ug.p;
    }
    // items: blocks of rb rows of one chunk, ~2 MiB each
    const int64_t rb = std::max<int64_t>(1, std::min<int64_t>(n, ((int64_t)2 << 20) / (W * (int64_t)es)));
    const int64_t ipc = (n + rb - 1) / rb;
    std::unique_ptr<std::atomic<int64_t>[]> done(new std::atomic<int64_t>[C]);
    for (int64_t ch = 0; ch < C; ++ch) done[ch].store(0, std::memory_order_relaxed);
    char *stage = (char *)c->rstage;
    const bool nt = rows_copy_nt(true);
    const std::function<void(int)> fn = [&](int it) {
        const int64_t ch = it / ipc, r0 = (it % ipc) * rb, r1 = std::min(n, r0 + rb);
        const int64_t c0 = ch * W, wc = std::min(W, d - c0);
        char *sl = stage + (size_t)(ch % S) * slot;
        for (int64_t r = r0; r < r1; ++r)
            bk::copy_to_stage(sl + (size_t)r * wc * es, rows[r] + (size_t)c0 * es, (size_t)wc * es,
                              nt);
        _mm_sfence();
        done[ch].fetch_add(1, std::memory_order_release);
    };
    // on an error return, copies already queued may still read the stage and
    // write dX: drain both streams (after the pool has stopped, below)
    HostDrain drain{c};
    // earlier work on the compute stream may still read the device batch
    HIPCHK(hipEventRecord(c->ev_go, c->stream));
    HIPCHK(hipStreamWaitEvent(c->copy, c->ev_go, 0));
    bk::HostPool *pool = get_pool(c);
    PoolJob job(pool, (int)(C * ipc), &fn);
    if (pool) pool->release((int)(S * ipc));
    for (int64_t ch = 0; ch < C; ++ch) {
        const int64_t c0 = ch * W, wc = std::min(W, d - c0);
        const int s = (int)(ch % S);
        if (pool) {
            while (done[ch].load(std::memory_order_acquire) < ipc)
                if (!pool->help()) _mm_pause();
        } else {
            for (int64_t i = ch * ipc; i < (ch + 1) * ipc; ++i) fn((int)i);
        }
        HIPCHK(hipMemcpy2DAsync(dX + c0 * es, (size_t)dld * es, stage + (size_t)s * slot,
                                (size_t)wc * es, (size_t)wc * es, (size_t)n, hipMemcpyHostToDevice,
                                c->copy));
        HIPCHK(hipEventRecord(c->ev_rows[s], c->copy));
        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_rows[s], 0));
        CHK(stage_gram(c, dX + c0 * es, dtype, n, wc, dld, ch == 0 ? U : P, pl));
        if (ch > 0) HIPCHK(launch_add_upper(U, P, (int64_t)usz, c->stream));
        // chunk ch - 1's slot is free once its copy (queued before chunk ch's,
        // which keeps the copy engine busy meanwhile) has landed: chunk
        // ch - 1 + S goes into it
        if (ch >= 1 && ch - 1 + S < C) {
            HIPCHK(hipEventSynchronize(c->ev_rows[(ch - 1) % S]));
            if (pool) pool->release((int)((ch + S) * ipc));
        }
    }
    pl.d = d;
    drain.armed = false;
    return BK_OK;
}

// Biscotti's deployed shapes (n <= 128, d <= 32768: configs A and B) on the
// row-fed entry.  k_tiny's batches (n <= 16, d <= 128) are packed by the
// caller into the mapped pinned stage, which the kernel reads over PCIe (as
// bk_multikrum's pinned batches).  Larger ones are packed by the pool in
// row order into a stage laid out like the device batch (16-B rows), and
// each group of rows crosses PCIe as one linear copy on the compute stream
// as soon as it is packed (BK_ROWS_GROUPS groups, default 3, growing x1.5),
// so the copy engine starts after the first sixth of the pack instead of
// after all of it; then the one-launch k_small, as bk_multikrum's host path.
// (r6 sweep at config B, tools/rows_probe.py --sweep: every extra copy costs
// more than the pack it hides beyond 3-4 groups.)
int run_rows_small(bk_ctx *c, const char *const *rows, int dtype, int64_t n, int64_t d, int64_t f,
                   int64_t *sel_idx, int64_t *m_out, double *scores, double *mean_out) {
    const size_t es = esize(dtype);
    const int64_t epg = (int64_t)(16 / es);
    const int64_t dld = (d + epg - 1) / epg * epg;
    const size_t rowb = (size_t)dld * es;
    CHK(ensure_rows_stage(c, (size_t)n * rowb));
    char *stage = (char *)c->rstage;
    if (tiny_ok((int)n, d)) {
        for (int64_t r = 0; r < n; ++r) memcpy(stage + (size_t)r * rowb, rows[r], (size_t)d * es);
        return run_host_small(c, stage, BK_HOST_PINNED, dld, dtype, nullptr, 0, 0, n, d, f, sel_idx,
                              m_out, scores, mean_out, nullptr, 0);
    }
    const char *ge = getenv("BK_ROWS_GROUPS");
    const int groups_env = ge && atoi(ge) > 0 ? atoi(ge) : 3;
    CHK(ensure(c->X, (size_t)n * rowb));
    // items: ~128 KiB of rows each.  Groups grow geometrically (x1.5): the
    // copy engine starts after the first small group is packed, and each
    // later group is packed (by several threads, faster than PCIe drains
    // the stage) while the groups before it are in flight
    const int64_t ri = std::max<int64_t>(1, ((int64_t)128 << 10) / (d * (int64_t)es));
    const int64_t I = (n + ri - 1) / ri;
    const int64_t G = std::min<int64_t>(groups_env, I);
    std::vector<int64_t> gstart((size_t)G + 1);
    {
        double tot = 0, w = 1;
        for (int64_t g = 0; g < G; ++g, w *= 1.5) tot += w;
        double acc = 0;
        w = 1;
        gstart[0] = 0;
        for (int64_t g = 1; g <= G; ++g, w *= 1.5) {
            acc += w;
            gstart[(size_t)g] = std::max(gstart[(size_t)g - 1] + 1,
                                         std::min<int64_t>(I - (G - g), (int64_t)(I * acc / tot + 0.5)));
        }
        gstart[(size_t)G] = I;
    }
    std::unique_ptr<std::atomic<int64_t>[]> done(new std::atomic<int64_t>[G]);
    for (int64_t g = 0; g < G; ++g) done[g].store(0, std::memory_order_relaxed);
    const bool nt = rows_copy_nt(false);
    const std::function<void(int)> fn = [&](int it) {
        const int64_t r0 = it * ri, r1 = std::min(n, r0 + ri);
        for (int64_t r = r0; r < r1; ++r)
            bk::copy_to_stage(stage + (size_t)r * rowb, rows[r], (size_t)d * es, nt);
        _mm_sfence();
        int64_t g = 0;
        while (gstart[(size_t)g + 1] <= it) ++g;
        done[g].fetch_add(1, std::memory_order_release);
    };
    HostDrain drain{c};
    // debug (probe build): host timeline of the call, us from entry
    const bool trace = probe_env("BK_ROWS_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<double> tl;
    auto mark = [&] {
        if (trace)
            tl.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    };
    {
        // a stage of <= 8 MiB (config B: 6.3 MB) is packed by the caller
        // alone: waking the pool costs more than it saves there (B, per call:
        // 0.195 ms with 1-4 packing threads, 0.217 with 8; bench e2e_rows)
        bk::HostPool *pool = (size_t)n * rowb > ((size_t)8 << 20) ? get_pool(c) : nullptr;
        PoolJob job(pool, (int)I, &fn);
        if (pool) pool->release((int)I);
        mark();
        char *dx = (char *)c->X.p;
        for (int64_t g = 0; g < G; ++g) {
            const int64_t need = gstart[(size_t)g + 1] - gstart[(size_t)g];
            if (pool) {
                while (done[g].load(std::memory_order_acquire) < need)
                    if (!pool->help()) _mm_pause();
            } else {
                for (int64_t i = gstart[(size_t)g]; i < gstart[(size_t)g + 1]; ++i) fn((int)i);
            }
            mark();
            const int64_t r0 = gstart[(size_t)g] * ri, r1 = std::min(n, gstart[(size_t)g + 1] * ri);
            CHK(timed(c, BK_K_H2D, [&] {
                return hipMemcpyAsync(dx + (size_t)r0 * rowb, stage + (size_t)r0 * rowb,
                                      (size_t)(r1 - r0) * rowb, hipMemcpyHostToDevice, c->stream);
            }));
            mark();
        }
    }
    mark();
    const int st = run_host_small(c, c->X.p, BK_DEVICE, dld, dtype, nullptr, 0, 0, n, d, f, sel_idx,
                                  m_out, scores, mean_out, nullptr, 0);
    mark();
    if (trace) {
        fprintf(stderr, "rows_trace G=%lld I=%lld:", (long long)G, (long long)I);
        for (double t : tl) fprintf(stderr, " %.1f", t);
        fprintf(stderr, "\n");
    }
    drain.armed = st != BK_OK;
    return st;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

bool certified(const bk_ctx *c, int dtype) {
    if (dtype == BK_F64) return c->f64_mode == BK_F64_I8_CERTIFIED || c->f64_mode == BK_F64_I8X2_CERTIFIED;
    return c->f32_mode == BK_F32_CERTIFIED || c->f32_mode == BK_F32_I8_CERTIFIED ||
           c->f32_mode == BK_F32_I8X2_CERTIFIED;
}

// BK_F32_CERTIFIED: run on the fp32 MFMA; if the selection margin does not
// clear the fp32 error bound, run again on the exact path (fp32 widened onto
// the fp64 MFMA), whose outputs replace the first run's.  Synchronous (the
// decision needs the margin on the host).  In the sharded entry every rank
// holds the same summed Gram, hence the same margin and the same decision, so
// the re-run's exchange is joined by all ranks.
template <typename F>
int run_certified(bk_ctx *c, F &&run) {
    CHK(run());
    double mg[MARGIN_WORDS];
    CHK(read_margin(c, mg));
    // only a near tie of a call whose Gram ran on the fp32 MFMA (u_G > 2^-53)
    // is re-run: an exact first pass (k_small, n <= 128) would repeat itself
    if (mg[2] == 0.0 || !(mg[8] > 0x1p-53)) return BK_OK;
    // (BK_EMU_SPLIT_SCORES, timing only: the exact re-run's Gram is another
    // one, so its first call scores every share again, and so does the next
    // approximate call -- ADVICE r5)
    c->emu_split_n = -1;
    c->force_exact = 1;
    const int st = run();
    c->force_exact = 0;
    c->emu_split_n = -1;
    if (st == BK_OK) ++c->certified_reruns;
    return st;
}

// the host entries' certified modes: a near tie of an approximate Gram re-runs
// exact from the device-resident batch dX (row stride dld), whose outputs
// replace the first run's in the caller's arrays
int host_certified_rerun(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t dld,
                         int64_t f, double *U, int64_t *sel_idx, int64_t *m_out, double *scores,
                         double *mean_out) {
    if (!certified(c, dtype)) return BK_OK;
    double mg[MARGIN_WORDS];
    CHK(read_margin(c, mg));
    if (!(mg[2] != 0.0 && mg[8] > 0x1p-53)) return BK_OK;
    c->force_exact = 1;
    Plan pl2;
    int st = stage_gram(c, dX, dtype, n, d, dld, U, pl2);
    if (st == BK_OK)
        st = run_host_outputs(c, dX, dtype, n, d, dld, f, U, pl2, sel_idx, m_out, scores, mean_out);
    c->force_exact = 0;
    if (st == BK_OK) ++c->certified_reruns;
    return st;
}

}  // namespace

extern "C" {

int bk_abi_version(void) { return BK_ABI_VERSION; }

const char *bk_last_error(void) { return g_err.c_str(); }

int bk_check_args(int64_t n, int64_t d, int64_t f) {
    if (n < 1 || d < 1) return fail(BK_EINVAL, "need n >= 1 and d >= 1");
    if (f < 1 || f >= n)
        return fail(BK_EINVAL, "need 1 <= f < n (n=%lld f=%lld); f=0 is the reference's "
                               "argpartition ValueError",
                    (long long)n, (long long)f);
    if (n > BK_MAX_N) return fail(BK_ENOTSUP, "n=%lld exceeds BK_MAX_N=%d", (long long)n, BK_MAX_N);
    return BK_OK;
}

const char *bk_kernel_name(int kid) {
    return (kid >= 0 && kid < BK_NUM_KERNELS) ? kKernelNames[kid] : "?";
}

int64_t bk_upper_elems(int64_t n) {
    const int64_t T = (n + 63) / 64;
    // + the trailing record {column count, columns on the fp32 MFMA, the int8
    // Gram's absolute error bound, 0} (K3b's margin; summed by every exchange)
    return T * (T + 1) / 2 * 4096 + BK_UPPER_TRAIL;
}

int bk_create(bk_ctx **out, int device) {
    if (!out) return fail(BK_EINVAL, "null out");
    *out = nullptr;
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev)
        return fail(BK_EINVAL, "device %d out of range (%d visible)", device, ndev);
    bk_ctx *c = new (std::nothrow) bk_ctx();
    if (!c) return fail(BK_ENOMEM, "host allocation of bk_ctx failed");
    c->device = device;
    bind_epoch(c);
    DeviceGuard dg(device);
    // probe knob: how the host waits for the GPU (hipDeviceScheduleSpin 1,
    // Yield 2, BlockingSync 4; tools/idle_probe.py)
    if (const char *v = probe_env("BK_SCHED")) (void)hipSetDeviceFlags((unsigned)atoi(v));
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e == hipSuccess) c->num_cu = prop.multiProcessorCount;
    e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(BK_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    c->stream = c->own;
    if (const char *v = probe_env("BK_GRAM"))
        if (strcmp(v, "v1") == 0) c->gram_variant = 1;
    if (const char *v = probe_env("BK_GRAM_MODE")) c->gram_mode = atoi(v);
    if (const char *v = getenv("BK_SMALL")) c->small_on = atoi(v) != 0;
    if (const char *v = getenv("BK_SPIN_US")) c->spin_us = atoll(v);
    // test / debug knobs (tests/test_gpu_errors.py): a hand-off wait that gives
    // up after this many polls; the queue-line invariant check; a sharded call
    // that fails before its exchange
    if (const char *v = getenv("BK_SMALL_SPIN_MAX")) {
        char *end = nullptr;
        c->small_spin_max = strtoull(v, &end, 10);
        if (end && *end == ',') c->small_spin_left = strtoll(end + 1, nullptr, 10);
    }
    if (const char *v = getenv("BK_SMALL_CHECK_LINES")) c->small_check_lines = atoi(v) != 0;
    if (const char *v = getenv("BK_TEST_FAIL_BEFORE_EXCHANGE")) c->test_fail_exchange = atoi(v);
    if (const char *v = getenv("BK_TEST_I8_ENOMEM")) c->test_i8_enomem = atoi(v) != 0;
    if (const char *v = getenv("BK_TEST_FAIL_PIECE")) c->test_fail_piece = atoi(v);
    if (const char *v = getenv("BK_TEST_PIECES_DISAGREE")) c->test_pieces_disagree = atoi(v);
    if (const char *v = getenv("BK_SPLIT_SCORES_MIN_N")) c->split_min_n = atoll(v);
    if (const char *v = getenv("BK_TEST_SPLIT_SCORES")) c->test_split_scores = atoi(v);
    if (const char *v = getenv("BK_EMU_SPLIT_SCORES")) c->emu_split_scores = atoi(v);
    if (const char *v = getenv("BK_TEST_SPLIT_FAIL")) c->test_split_fail = atoi(v);
    e = configure_kernels();
    if (e == hipSuccess) e = configure_aggregate_kernels();
    if (e == hipSuccess) e = configure_i8_kernels();
    if (e != hipSuccess) {
        (void)hipStreamDestroy(c->own);
        delete c;
        return fail(BK_EHIP, "configure_kernels: %s", hipGetErrorString(e));
    }
    *out = c;
    return BK_OK;
}

void bk_destroy(bk_ctx *c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceGuard dg(c->device);
        (void)hipStreamSynchronize(c->stream);
        DevBuf *bufs[] = {&c->part, &c->U,    &c->Ug,  &c->scores,
                          &c->mask, &c->sel,  &c->X,   &c->mean, &c->perm, &c->trace, &c->idx,
                          &c->roni_X, &c->roni_y, &c->roni_w, &c->roni_d, &c->roni_cnt, &c->roni_s,
                          &c->noise, &c->diag, &c->bnd, &c->Ut, &c->small_ctr, &c->small_part,
                          &c->mean_part, &c->status, &c->rmc_X, &c->rmc_y, &c->rmc_ws,
                      &c->rmc_xn, &c->rmc_idx, &c->rmc_nt, &c->i8ws, &c->sgather, &c->pcnt};
        if (c->hmargin) (void)hipHostFree(c->hmargin);
        if (c->hout) (void)hipHostFree(c->hout);
        if (c->copy) (void)hipStreamSynchronize(c->copy);
        for (DevBuf *b : bufs)
            if (b->p) (void)hipFree(b->p);
        for (hipEvent_t ev : {c->ev_go, c->ev_cp[0], c->ev_cp[1], c->ev_use[0], c->ev_use[1],
                              c->ev_rows[0], c->ev_rows[1], c->ev_rows[2], c->ev_rows[3]})
            if (ev) (void)hipEventDestroy(ev);
        if (c->cstream) (void)hipStreamSynchronize(c->cstream);
        for (hipEvent_t ev : c->ev_piece)
            if (ev) (void)hipEventDestroy(ev);
        if (c->ev_cdone) (void)hipEventDestroy(c->ev_cdone);
        if (c->cstream) (void)hipStreamDestroy(c->cstream);
        for (unsigned *sgc : c->sigcnt)
            if (sgc) (void)hipFree(sgc);
        if (c->hsig) (void)hipHostFree(c->hsig);
        if (c->rstage) (void)hipHostFree(c->rstage);
        delete c->hpool;
        if (c->copy) (void)hipStreamDestroy(c->copy);
        for (void *p : c->staged) (void)hipHostFree(p);
        for (auto &ev : c->pending) {
            (void)hipEventDestroy(ev.a);
            (void)hipEventDestroy(ev.b);
        }
        for (hipEvent_t ev : c->pool) (void)hipEventDestroy(ev);
        for (auto &cp : c->plans) {
            free_plan(cp.p);
            free_pieces(cp.pc);
        }
        for (auto &e : c->i8) {
            if (e.tables) (void)hipFree(e.tables);
            free_pieces(e.pc);
        }
        for (auto &cg : c->graphs) drop_graph(cg);
        if (c->comm) (void)ncclCommDestroy(c->comm);
        if (c->own) (void)hipStreamDestroy(c->own);
    }
    delete c;
}

int bk_set_stream(bk_ctx *c, void *s) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    c->stream = s ? (hipStream_t)s : c->own;
    return BK_OK;
}

void *bk_get_stream(bk_ctx *c) { return c ? (void *)c->stream : nullptr; }

int bk_synchronize(bk_ctx *c) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    HIPCHK(wait_stream(c));
    if (c->margin_unchecked) {  // the last finish's error codes (an asynchronous caller's only check)
        double mg[MARGIN_WORDS];
        CHK(read_margin(c, mg));
    }
    return BK_OK;
}

int bk_stage_alloc(bk_ctx *c, int64_t bytes, void **pinned) {
    if (!c || !pinned || bytes <= 0) return fail(BK_EINVAL, "bad stage_alloc arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, (size_t)bytes, hipHostMallocPortable);
    if (e != hipSuccess) return fail(BK_ENOMEM, "hipHostMalloc(%lld): %s", (long long)bytes,
                                     hipGetErrorString(e));
    c->staged.push_back(p);
    *pinned = p;
    return BK_OK;
}

int bk_stage_free(bk_ctx *c, void *p) {
    if (!c || !p) return fail(BK_EINVAL, "bad stage_free arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    for (size_t i = 0; i < c->staged.size(); ++i) {
        if (c->staged[i] == p) {
            c->staged.erase(c->staged.begin() + i);
            HIPCHK(hipHostFree(p));
            return BK_OK;
        }
    }
    return fail(BK_EINVAL, "pointer was not allocated by bk_stage_alloc");
}

int bk_plan(bk_ctx *c, int64_t n, int64_t d, int64_t *S, int64_t *kc, int64_t *ntile,
            int64_t *nwg) {
    if (n < 1 || d < 1) return fail(BK_EINVAL, "need n, d >= 1");
    if (n > BK_MAX_N) return fail(BK_ENOTSUP, "n=%lld exceeds BK_MAX_N=%d", (long long)n, BK_MAX_N);
    // the K1 v3 plan for aligned fp64 rows (host tables only, nothing allocated)
    const Plan3Host H = build_plan3((int)n, d, c ? c->num_cu : 256, G3_BK);
    for (int u = 0; u < H.ntile; ++u)
        if (H.red[3 * u + 1] < 0) return fail(BK_EHIP, "internal: K1 plan fails its coverage check");
    if (S) *S = (int64_t)H.groups.size();
    if (kc) *kc = G3_BK;
    if (ntile) *ntile = H.ntile;
    if (nwg) *nwg = (int64_t)(H.seg.size() / 2);
    return BK_OK;
}

int bk_plan_mode(bk_ctx *c, int64_t n, int64_t d, int mode, int rounds, int64_t *S, int64_t *nwg) {
    if (n < 1 || d < 1) return fail(BK_EINVAL, "need n, d >= 1");
    if (n > BK_MAX_N) return fail(BK_ENOTSUP, "n=%lld exceeds BK_MAX_N=%d", (long long)n, BK_MAX_N);
    if (mode < -1 || mode > 3 || rounds < 0 || rounds > 16)
        return fail(BK_EINVAL, "bad planner mode %d / rounds %d", mode, rounds);
    const Plan3Host H = build_plan3((int)n, d, c ? c->num_cu : 256, G3_BK, mode, rounds);
    for (int u = 0; u < H.ntile; ++u)
        if (H.red[3 * u + 1] < 0) return fail(BK_EHIP, "internal: K1 plan fails its coverage check");
    if (S) *S = (int64_t)H.groups.size();
    if (nwg) *nwg = (int64_t)(H.seg.size() / 2);
    return BK_OK;
}

namespace {

// The 7-launch step (K1, K1b, K2, K3, K3b, K4) replayed as one hipGraph: the
// first call of a signature runs eagerly (allocating workspace and the K1
// plan), the second captures the same sequence, later ones replay it.  Only
// without per-kernel timing (events are not captured).
int run_device_graph(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld,
                     int64_t f, int64_t *d_sel, double *d_scores, double *d_mean) {
    for (size_t i = 0; i < c->graphs.size();) {  // retire graphs over stale workspace
        if (c->graphs[i].epoch != c->ws_epoch) {
            drop_graph(c->graphs[i]);
            c->graphs.erase(c->graphs.begin() + i);
        } else {
            ++i;
        }
    }
    for (auto &cg : c->graphs)
        if (cg.X == dX && cg.dtype == dtype && cg.n == n && cg.d == d && cg.ld == ld && cg.f == f &&
            cg.sel == d_sel && cg.scores == d_scores && cg.mean == d_mean) {
            HIPCHK(hipGraphLaunch(cg.exec, c->stream));
            // the captured finish (K3b / k_small) writes the context's record:
            // point the readers at it and arm bk_synchronize's check
            c->margin_valid = 1;
            c->margin_host = c->hmargin;
            c->margin_unchecked = 1;
            return BK_OK;
        }
    // eager run first: every ensure() / plan build happens outside the capture
    const uint64_t e0 = c->ws_epoch;
    CHK(run_device(c, dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean));
    if (c->ws_epoch != e0) return BK_OK;  // workspace moved: capture on the next call
    bk_ctx::CachedGraph cg{dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean, c->ws_epoch, nullptr,
                           nullptr};
    HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    const int st = run_device(c, dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean);
    hipGraph_t g = nullptr;
    const hipError_t ee = hipStreamEndCapture(c->stream, &g);
    if (st != BK_OK) {
        if (g) (void)hipGraphDestroy(g);
        return st;
    }
    if (ee != hipSuccess) return fail(BK_EHIP, "hipStreamEndCapture: %s", hipGetErrorString(ee));
    cg.g = g;
    const hipError_t ei = hipGraphInstantiate(&cg.exec, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
        drop_graph(cg);
        return fail(BK_EHIP, "hipGraphInstantiate: %s", hipGetErrorString(ei));
    }
    if (c->ws_epoch != e0) {  // cannot happen after an eager run of the same call; be safe
        drop_graph(cg);
        return BK_OK;
    }
    if (c->graphs.size() >= 4) {
        drop_graph(c->graphs.front());
        c->graphs.erase(c->graphs.begin());
    }
    c->graphs.push_back(cg);
    return BK_OK;  // the captured run is not executed: the eager one produced this call's outputs
}
}  // namespace

int bk_multikrum_device(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld,
                        int64_t f, int64_t *d_sel, double *d_scores, double *d_mean) {
    CHK(check_common(c, dX, dtype, n, d, ld));
    CHK(bk_check_args(n, d, f));
    if (!d_sel) return fail(BK_EINVAL, "null d_sel_idx");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    if (certified(c, dtype))
        return run_certified(c, [&] { return run_device(c, dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean); });
    // (the debug traces synchronize mid-call, which a stream capture refuses)
    if (c->graph_on && c->timing == 0 && !probe_env("BK_TRACE_FILE") && !probe_env("BK_SMALL_TRACE"))
        return run_device_graph(c, dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean);
    return run_device(c, dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean);
}

int bk_set_f32_mode(bk_ctx *c, int mode) {
    if (!c) return fail(BK_EINVAL, "null context");
    if (mode < BK_F32_EXACT || mode > BK_F32_I8X2_CERTIFIED)
        return fail(BK_EINVAL, "bad f32 mode %d", mode);
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->f32_mode != mode) ++c->ws_epoch;  // captured graphs baked the other kernel in
    c->f32_mode = mode;
    c->i8_failed.clear();  // a new mode tries K1i8's workspace again
    c->emu_split_n = -1;  // BK_EMU_SPLIT_SCORES: the new mode's first call scores every share
    return BK_OK;
}

int bk_set_f64_mode(bk_ctx *c, int mode) {
    if (!c) return fail(BK_EINVAL, "null context");
    if (mode != BK_F64_EXACT && mode != BK_F64_I8 && mode != BK_F64_I8_CERTIFIED &&
        mode != BK_F64_I8X2 && mode != BK_F64_I8X2_CERTIFIED)
        return fail(BK_EINVAL, "bad f64 mode %d", mode);
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->f64_mode != mode) ++c->ws_epoch;  // captured graphs baked the other kernel in
    c->f64_mode = mode;
    c->i8_failed.clear();
    c->emu_split_n = -1;
    return BK_OK;
}

int bk_graph_enable(bk_ctx *c, int on) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    c->graph_on = on ? 1 : 0;
    if (!on) {
        for (auto &cg : c->graphs) drop_graph(cg);
        c->graphs.clear();
    }
    return BK_OK;
}

int bk_multikrum(bk_ctx *c, const void *X, int where, int dtype, int64_t n, int64_t d, int64_t ld,
                 int64_t f, int64_t *sel_idx, int64_t *m_out, double *scores, double *mean_out) {
    CHK(check_common(c, X, dtype, n, d, ld));
    CHK(bk_check_args(n, d, f));
    if (!sel_idx) return fail(BK_EINVAL, "null sel_idx");
    if (where != BK_HOST && where != BK_HOST_PINNED && where != BK_DEVICE)
        return fail(BK_EINVAL, "bad where=%d", where);
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    // n <= 128: one copy and the one-launch path (always exact: no certified re-run)
    if (small_ok(c, X, dtype, n, d, ld))
        return run_host_small(c, X, where, ld, dtype, nullptr, 0, 0, n, d, f, sel_idx, m_out,
                              scores, mean_out, nullptr, 0);
    const size_t es = esize(dtype);
    const void *dX = X;
    int64_t dld = ld;
    CHK(ensure(c->U, (size_t)bk_upper_elems(n) * sizeof(double)));
    double *U = (double *)c->U.p;
    Plan pl;
    if (where != BK_DEVICE) {
        // device rows padded to 16 B so K1 v3 (global_load_lds granules) always applies
        const int64_t epg = (int64_t)(16 / es);
        dld = (d + epg - 1) / epg * epg;
        CHK(ensure(c->X, (size_t)n * dld * es));
        CHK(stage_host_pipelined(c, X, ld, dtype, nullptr, 0, 0, n, d, (char *)c->X.p, dld, U,
                                 pl));
        dX = c->X.p;
    } else {
        CHK(stage_gram(c, dX, dtype, n, d, dld, U, pl));
    }
    CHK(run_host_outputs(c, dX, dtype, n, d, dld, f, U, pl, sel_idx, m_out, scores, mean_out));
    return host_certified_rerun(c, dX, dtype, n, d, dld, f, U, sel_idx, m_out, scores, mean_out);
}

int bk_multikrum_rows(bk_ctx *c, const void *const *rows, int dtype, int64_t n, int64_t d,
                      int64_t f, int64_t *sel_idx, int64_t *m_out, double *scores,
                      double *mean_out) {
    CHK(check_common(c, rows, dtype, n, d, d));
    CHK(bk_check_args(n, d, f));
    if (!sel_idx) return fail(BK_EINVAL, "null sel_idx");
    for (int64_t i = 0; i < n; ++i)
        if (!rows[i]) return fail(BK_EINVAL, "null row %lld", (long long)i);
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    const char *const *R = (const char *const *)rows;
    if (small_ok(c, nullptr, dtype, n, d, d))
        return run_rows_small(c, R, dtype, n, d, f, sel_idx, m_out, scores, mean_out);
    const size_t es = esize(dtype);
    const int64_t epg = (int64_t)(16 / es);
    const int64_t dld = (d + epg - 1) / epg * epg;
    CHK(ensure(c->X, (size_t)n * dld * es));
    CHK(ensure(c->U, (size_t)bk_upper_elems(n) * sizeof(double)));
    double *U = (double *)c->U.p;
    Plan pl;
    CHK(stage_rows_pipelined(c, R, dtype, n, d, (char *)c->X.p, dld, U, pl));
    CHK(run_host_outputs(c, c->X.p, dtype, n, d, dld, f, U, pl, sel_idx, m_out, scores, mean_out));
    return host_certified_rerun(c, c->X.p, dtype, n, d, dld, f, U, sel_idx, m_out, scores, mean_out);
}

int bk_set_host_threads(bk_ctx *c, int threads) {
    if (!c) return fail(BK_EINVAL, "null context");
    if (threads < 0 || threads > 256) return fail(BK_EINVAL, "threads=%d out of [0, 256]", threads);
    std::lock_guard<std::mutex> lk(c->mu);
    c->hthreads = threads;
    return BK_OK;
}

// the noise application fused into the H2D staging of
// the verifier batch.  Rows go over in chunks on a copy stream (Delta rows
// straight into the padded device batch, their k noise vectors into a 2-slot
// ring); K6 adds each chunk's noise in place on the compute stream while the
// next chunk is in flight.  No host pass over n*d, and no n*k*d device buffer.
int bk_multikrum_noised(bk_ctx *c, const double *delta, int64_t ld, const double *noise,
                        int64_t k, int64_t noise_ld, int where, int64_t n, int64_t d, int64_t f,
                        int64_t *sel_idx, int64_t *m_out, double *scores, double *mean_out,
                        double *noised_out, int64_t out_ld) {
    CHK(check_common(c, delta, BK_F64, n, d, ld));
    CHK(bk_check_args(n, d, f));
    if (!sel_idx) return fail(BK_EINVAL, "null sel_idx");
    if (where != BK_HOST && where != BK_HOST_PINNED)
        return fail(BK_EINVAL, "bad where=%d (host batches only; device-resident batches use "
                               "bk_noise_apply_device + bk_multikrum_device)", where);
    if (k < 0) return fail(BK_EINVAL, "k=%lld < 0", (long long)k);
    if (k > 0 && !noise) return fail(BK_EINVAL, "null noise with k=%lld", (long long)k);
    if (k > 0 && noise_ld < d) return fail(BK_EINVAL, "noise_ld=%lld < d", (long long)noise_ld);
    if (noised_out && out_ld < d) return fail(BK_EINVAL, "out_ld=%lld < d", (long long)out_ld);
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    // n <= 128: one copy of the batch and its noise, K6, the one-launch path
    if (small_ok(c, delta, BK_F64, n, d, ld))
        return run_host_small(c, delta, where, ld, BK_F64, k > 0 ? noise : nullptr, k, noise_ld, n,
                              d, f, sel_idx, m_out, scores, mean_out, noised_out, out_ld);
    const int64_t dld = (d + 1) / 2 * 2;  // 16-B rows: K1 v3 applies
    CHK(ensure(c->X, (size_t)n * dld * sizeof(double)));
    double *dX = (double *)c->X.p;
    CHK(ensure(c->U, (size_t)bk_upper_elems(n) * sizeof(double)));
    double *U = (double *)c->U.p;
    Plan pl;
    // armed until the outputs have landed: on any error return, copies still
    // queued may read delta / noise or write noised_out
    HostDrain drain{c};
    // k = 0: no noisers, NoisedDelta = Delta (main.go:1599-1602)
    CHK(stage_host_pipelined(c, delta, ld, BK_F64, k > 0 ? noise : nullptr, k, noise_ld, n, d,
                             (char *)dX, dld, U, pl));
    if (noised_out)
        HIPCHK(hipMemcpy2DAsync(noised_out, (size_t)out_ld * 8, dX, (size_t)dld * 8,
                                (size_t)d * 8, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    CHK(run_host_outputs(c, dX, BK_F64, n, d, dld, f, U, pl, sel_idx, m_out, scores, mean_out));
    drain.armed = false;
    return BK_OK;
}

int bk_gram_upper_device(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld,
                         double *d_upper) {
    CHK(check_common(c, dX, dtype, n, d, ld));
    if (!d_upper) return fail(BK_EINVAL, "null d_upper");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    Plan pl;
    int st = c->test_fail_exchange == 2
                 ? fail(BK_EHIP, "test knob BK_TEST_FAIL_BEFORE_EXCHANGE=2: forced failure")
                 : stage_gram(c, dX, dtype, n, d, ld, d_upper, pl);
    if (st != BK_OK) {
        // a caller that exchanges the partial anyway (so its peers are not left
        // in the collective) hands every rank an invalid record, not a wrong Gram
        const std::string msg = g_err;
        (void)poison_upper(c, d_upper, n);
        g_err = msg;
    }
    return st;
}

int bk_finish_device(bk_ctx *c, const double *d_upper, const void *dX, int dtype, int64_t n,
                     int64_t d, int64_t ld, int64_t f, int64_t *d_sel, double *d_scores,
                     double *d_mean) {
    if (d_mean) CHK(check_common(c, dX, dtype, n, d, ld));
    if (!c) return fail(BK_EINVAL, "null context");
    CHK(bk_check_args(n, d < 1 ? 1 : d, f));
    if (!d_upper || !d_sel) return fail(BK_EINVAL, "null d_upper / d_sel_idx");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    Plan pl;
    pl.n = (int)n;
    pl.T = (int)((n + 63) / 64);
    pl.ntile = pl.T * (pl.T + 1) / 2;
    return stage_finish(c, d_upper, pl, dX, dtype, n, d, ld, f, d_sel, d_scores, d_mean);
}

int bk_comm_unique_id(void *id_out) {
    if (!id_out) return fail(BK_EINVAL, "null id");
    static_assert(sizeof(ncclUniqueId) == BK_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    RCCLCHK(ncclGetUniqueId(&id));
    memcpy(id_out, &id, sizeof id);
    return BK_OK;
}

int bk_comm_init(bk_ctx *c, int nranks, int rank, const void *id) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(BK_EINVAL, "bad comm_init arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    if (c->comm) {
        (void)ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    // the sharded entry's status agreement word, before the communicator (an
    // allocation failure then fails this rank's init, not a later collective)
    CHK(ensure(c->status, 4 * sizeof(double)));
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    RCCLCHK(ncclCommInitRank(&c->comm, nranks, uid, rank));
    c->nranks = nranks;
    c->rank = rank;
    c->agreed_n = c->agreed_f = -1;  // the next sharded call agrees again
    return BK_OK;
}

int bk_comm_set_mode(bk_ctx *c, int mode) {
    if (!c) return fail(BK_EINVAL, "null context");
    if (mode < 0 || mode > 2) return fail(BK_EINVAL, "bad exchange mode %d", mode);
    std::lock_guard<std::mutex> lk(c->mu);
    c->deterministic = mode == 1 ? 1 : 0;
    int k = 2;
    if (const char *v = getenv("BK_OVERLAP_PIECES")) k = atoi(v);
    c->overlap = mode == 2 ? std::max(2, std::min(8, k)) : 0;
    return BK_OK;
}

namespace {
// the communication stream of the overlapped exchange and its events (once)
int ensure_comm_stream(bk_ctx *c) {
    CHK(ensure(c->pcnt, 8 * sizeof(unsigned)));
    if (c->cstream) return BK_OK;
    if (!c->hsig) {
        void *hp = nullptr, *dp = nullptr;
        HIPCHK(hipHostMalloc(&hp, 8 * 64, hipHostMallocCoherent));
        memset(hp, 0, 8 * 64);
        const hipError_t e = hipHostGetDevicePointer(&dp, hp, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(hp);
            return fail(BK_EHIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
        }
        c->hsig = (unsigned *)hp;
        c->hsig_d = (unsigned *)dp;
    }

    // normal priority: a highest-priority stream was measured slower in every
    // form (two-digit certified 1.38 -> 1.77 ms, fp32 MFMA 4.39 -> 5.12 ms at
    // E's 8-rank shard)
    hipStream_t cs = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipError_t e = hipSuccess;
    hipEvent_t ev[9] = {};
    for (int i = 0; i < 9 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        for (hipEvent_t x : ev)
            if (x) (void)hipEventDestroy(x);
        (void)hipStreamDestroy(cs);
        return fail(BK_EHIP, "communication stream events: %s", hipGetErrorString(e));
    }
    for (int i = 0; i < 8; ++i) c->ev_piece[i] = ev[i];
    c->ev_cdone = ev[8];
    c->cstream = cs;
    return BK_OK;
}

// The sharded call with its exchange overlapped with the Gram (bk_comm_set_mode
// 2).  ONE Gram launch runs the pieces' workgroups in piece order, each
// workgroup counting itself into its piece's signal word at exit (PieceMarks).
// The communication stream waits for piece p's count (hipStreamWaitValue32),
// reduces piece p's sub-tiles (K1b, or K1i8's reduce of its range) and
// all-reduces them while the Gram's later pieces still run; the last piece is
// reduced on the context stream after the Gram, with the trailing record, and
// all-reduced last.  Every sub-tile is summed from the same partials in the
// same order as the serial path and the all-reduce sums element by element,
// so every output is bitwise that of mode 0.  A failure before the Gram's
// launch is queued poisons the record and joins every piece's all-reduce with
// no wait; the waits are queued only behind a launched Gram, whose every
// workgroup counts itself (idle ones included), so they always resolve.
int sharded_overlapped(bk_ctx *c, const Pieces &pc, const void *dX, int dtype, int64_t n,
                       int64_t dl, int64_t ld, int64_t f, double *U, Plan &pl, int64_t *d_sel,
                       double *d_scores, double *d_mean, const ScoreSplit &sp) {
    const int k = pc.k;
    pl.n = (int)n;
    pl.d = dl;
    pl.T = (int)((n + 63) / 64);
    pl.ntile = pl.T * (pl.T + 1) / 2;
    PieceMarks pm;
    pm.cnt = (unsigned *)c->pcnt.p;
    // r6: the host polls the piece words and queues each piece's reduce and
    // all-reduce as it completes.  A hipStreamWaitValue32 on the communication
    // stream (the probe build's BK_PIECES_DEVWAIT) held a command-processor
    // wait for the whole Gram and slowed it (E's 8-rank shard, exact: +0.85 ms
    // for the wait alone)
    if (probe_env("BK_PIECES_DEVWAIT") && !c->sigcnt[0])
        for (int i = 0; i < 8; ++i) {  // HIP hands signal memory out 8 bytes at a time
            void *sp = nullptr;
            HIPCHK(hipExtMallocWithFlags(&sp, 8, hipMallocSignalMemory));
            c->sigcnt[i] = (unsigned *)sp;
        }
    const bool devwait = probe_env("BK_PIECES_DEVWAIT") != nullptr && c->sigcnt[0];
    for (int p = 0; p < k; ++p) pm.sig[p] = devwait ? c->sigcnt[p] : c->hsig_d + 16 * p;
    if (c->sig_pending) {
        // a previous call's Gram may still store into the words (its host
        // wait was cut short): let it drain before they are reset
        (void)hipStreamSynchronize(c->stream);
        c->sig_pending = false;
    }
    for (int p = 0; p < 8; ++p) __atomic_store_n(c->hsig + 16 * p, 0u, __ATOMIC_RELEASE);
    pm.k = k;
    int tot = 0;
    for (int p = 0; p < k; ++p) {
        pm.start[p] = tot;
        tot += pc.nwg[(size_t)p];
    }
    pm.start[k] = tot;
    bk_ctx::I8Cached *e8 = i8_prepared(c, dX, dtype, n, dl, ld);
    Plan3 *p3 = nullptr;
    double *part = nullptr;
    const bool f32m = f32_mfma_now(c, dtype);
    int st = BK_OK;
    if (!e8) {
        st = get_plan3(c, n, dl, v3_bk(dtype), &p3);
        if (st == BK_OK) st = ensure(c->part, (size_t)p3->nvwg * 16 * 4096 * sizeof(double));
        if (st == BK_OK) part = (double *)c->part.p;
    }
    // 1. zero the piece counts; K1i8: the digit slices; then the one Gram launch
    bool launched = false;
    for (int p = 0; p < k && st == BK_OK && devwait; ++p) {
        const hipError_t e = hipMemsetAsync(c->sigcnt[p], 0, 8, c->stream);
        if (e != hipSuccess) st = fail(BK_EHIP, "hipMemsetAsync: %s", hipGetErrorString(e));
    }
    if (st == BK_OK) {
        const hipError_t e = hipMemsetAsync(c->pcnt.p, 0, 8 * sizeof(unsigned), c->stream);
        if (e != hipSuccess) st = fail(BK_EHIP, "hipMemsetAsync: %s", hipGetErrorString(e));
    }
    if (st == BK_OK && c->test_fail_piece)  // test knob BK_TEST_FAIL_PIECE (bk_create)
        st = fail(BK_EHIP, "test knob BK_TEST_FAIL_PIECE=%d: the Gram fails before its launch",
                  c->test_fail_piece);
    if (st == BK_OK && e8)
        st = timed(c, BK_K_SLICE, [&] {
            return launch_i8_slice(dX, dtype, ld, (int)n, dl, e8->L, c->i8ws.p, e8->tables, c->stream);
        });
    // probe build: BK_PIECES_NOMARK=1 -- the pieces' workgroup order with no
    // counts, every piece reduced on the context stream after the Gram (an A/B
    // of the order alone; timing only)
    const bool nomark = probe_env("BK_PIECES_NOMARK") != nullptr;
    if (nomark) pm.k = 0;
    // probe build, timing only (wrong results): BK_PIECES_NOWT=1 -- counts
    // without write-through stores; BK_PIECES_NOCSTREAM=1 -- counts and
    // write-through stores, but the communication stream neither reduces nor
    // all-reduces the early pieces
    if (probe_env("BK_PIECES_NOWT")) pm.nowt = 1;
    const bool nocs = probe_env("BK_PIECES_NOCSTREAM") != nullptr;
    // the communication stream starts behind everything queued before the
    // Gram (the counts' reset, the previous call's finish still reading U) --
    // NOT behind the Gram itself, whose pieces it takes as they complete
    // (r6 fix: this record sat after the Gram launch, so the early pieces'
    // work waited for the whole Gram and nothing overlapped)
    bool cs_started = false;
    if (st == BK_OK && !nomark) {
        HIPCHK(hipEventRecord(c->ev_piece[0], c->stream));
        HIPCHK(hipStreamWaitEvent(c->cstream, c->ev_piece[0], 0));
        cs_started = true;
    }
    if (st == BK_OK) {
        st = timed(c, BK_K_GRAM, [&] {
            return e8 ? launch_i8_gemm((int)n, e8->L, c->i8ws.p, e8->tables, c->stream, pc.d, tot, pm)
                      : launch_gram3(dX, dtype, ld, (int)n, dl, *p3, part, c->stream, c->gram_mode,
                                     nullptr, f32m, pc.d, tot, pm);
        });
        launched = st == BK_OK;
        if (launched && !devwait && !nomark) c->sig_pending = true;
    }
    if (nomark && launched) {
        for (int p = 0; p < k; ++p) {
            const int64_t e0 = pc.e[(size_t)p], e1 = p + 1 == k ? (int64_t)pl.ntile * 4096 : pc.e[(size_t)p + 1];
            HIPCHK(e8 ? launch_i8_reduce(dl, e8->L, c->i8ws.p, U, c->stream, e0, e1, p + 1 == k)
                      : launch_reduce3(part, *p3, U, c->stream, f32m, (int)(e0 / 4096), (int)(e1 / 4096),
                                       p + 1 == k));
        }
        const int64_t usz = bk_upper_elems(n);
        RCCLCHK(ncclAllReduce(U, U, (size_t)usz, ncclDouble, ncclSum, c->comm, c->stream));
        ++c->exchanges;
        return stage_finish(c, U, pl, dX, dtype, n, dl, ld, f, d_sel, d_scores, d_mean, sp);
    }
    const std::string st_msg = st == BK_OK ? std::string() : g_err;
    if (st != BK_OK) CHK(poison_upper(c, U, n));
    if (!cs_started || !launched) {
        // no Gram ran: the communication stream starts behind the poisoned record
        HIPCHK(hipEventRecord(c->ev_piece[0], c->stream));
        HIPCHK(hipStreamWaitEvent(c->cstream, c->ev_piece[0], 0));
    }
    hipEvent_t ar_a = nullptr, ar_b = nullptr, ex_a = nullptr, ex_b = nullptr;
    const bool t_ar = timing_on(c, BK_K_ALLREDUCE), t_ex = timing_on(c, BK_K_EXCHANGE_EXPOSED);
    auto reduce_piece = [&](int p, hipStream_t s, bool rec) -> hipError_t {
        const int64_t e0 = pc.e[(size_t)p], e1 = rec ? (int64_t)pl.ntile * 4096 : pc.e[(size_t)p + 1];
        if (e8) return launch_i8_reduce(dl, e8->L, c->i8ws.p, U, s, e0, e1, rec);
        return launch_reduce3(part, *p3, U, s, f32m, (int)(e0 / 4096), (int)(e1 / 4096), rec);
    };
    // pieces 0 .. k-2 on the communication stream, each as soon as its
    // workgroups are done; the last piece (and the record) on the context
    // stream after the Gram, all-reduced there too once the communication
    // stream's all-reduces are done -- one stream hop at the end, not two
    const bool nowait = probe_env("BK_PIECES_NOWAIT") != nullptr;  // probe: no wait, no early work
    for (int p = 0; p + 1 < k; ++p) {
        // the exchange's span starts when piece 0 is done (after its wait), so
        // span - exposed is the exchange work that ran under the Gram
        auto span_start = [&]() -> int {
            if (p == 0 && t_ar && !ar_a) {
                CHK(get_event(c, &ar_a));
                HIPCHK(hipEventRecord(ar_a, c->cstream));
            }
            return BK_OK;
        };
        if (nowait) {
            CHK(span_start());
            continue;
        }
        if (launched && devwait) {
            HIPCHK(hipStreamWaitValue32(c->cstream, c->sigcnt[p], 1u, hipStreamWaitValueGte,
                                        0xffffffffu));
        } else if (launched) {
            // until the piece's last workgroup stores its word -- or the
            // context stream has drained (the Gram done, or failed), which
            // the stream query below notices
            const volatile unsigned *w = c->hsig + 16 * p;
            for (unsigned spin = 1; __atomic_load_n(w, __ATOMIC_ACQUIRE) == 0u; ++spin) {
                _mm_pause();
                if ((spin & 1023u) == 0u && hipStreamQuery(c->stream) != hipErrorNotReady) break;
            }
            if (p + 2 == k) c->sig_pending = false;  // every word this Gram stores has been seen
        }
        CHK(span_start());
        if (launched) {
            if (nocs) continue;
            HIPCHK(reduce_piece(p, c->cstream, false));
        }
        if (nocs && launched) continue;
        const int64_t e0 = pc.e[(size_t)p], e1 = pc.e[(size_t)p + 1];
        RCCLCHK(ncclAllReduce(U + e0, U + e0, (size_t)(e1 - e0), ncclDouble, ncclSum, c->comm,
                              c->cstream));
    }
    HIPCHK(hipEventRecord(c->ev_cdone, c->cstream));
    if (launched) {
        const hipError_t e = reduce_piece(k - 1, c->stream, true);
        if (e != hipSuccess) {
            CHK(poison_upper(c, U, n));
            st = fail(BK_EHIP, "K1b of the last piece: %s", hipGetErrorString(e));
        }
    }
    if (t_ex) {  // the exposed part: the last piece reduced -> its all-reduce done
        CHK(get_event(c, &ex_a));
        HIPCHK(hipEventRecord(ex_a, c->stream));
    }
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_cdone, 0));
    {
        const int64_t e0 = pc.e[(size_t)k - 1], e1 = pc.e[(size_t)k];
        RCCLCHK(ncclAllReduce(U + e0, U + e0, (size_t)(e1 - e0), ncclDouble, ncclSum, c->comm,
                              c->stream));
    }
    if (t_ar) {  // the span: the first all-reduce's start -> the last one's end
        CHK(get_event(c, &ar_b));
        HIPCHK(hipEventRecord(ar_b, c->stream));
        c->pending.push_back({BK_K_ALLREDUCE, ar_a, ar_b});
    }
    if (t_ex) {
        CHK(get_event(c, &ex_b));
        HIPCHK(hipEventRecord(ex_b, c->stream));
        c->pending.push_back({BK_K_EXCHANGE_EXPOSED, ex_a, ex_b});
    }
    c->exchanged_bytes += (double)bk_upper_elems(n) * sizeof(double);
    ++c->exchanges;
    if (st != BK_OK) {
        (void)stage_finish(c, U, pl, dX, dtype, n, dl, ld, f, d_sel, d_scores, nullptr, sp);
        g_err = st_msg.empty() ? g_err : st_msg;
        return st;
    }
    return stage_finish(c, U, pl, dX, dtype, n, dl, ld, f, d_sel, d_scores, d_mean, sp);
}

// one pass of the sharded entry: partial Gram of the local columns (zeros for
// an empty shard), the exchange, then scores/selection and the local mean.
//
// No rank may leave its peers inside the collective.  Everything that can fail
// before it is an allocation (U, the all-gather buffer, K1's plan and slabs)
// or a launch.  On the first call of a signature (n, f, dtype, exchange mode),
// which every rank makes together, the workspace is allocated and the ranks
// all-reduce (max) a status word before the exchange, so an allocation
// failure on one rank is an error on every rank (BK_ERCCL on the others).
// Later calls of the same signature allocate nothing that depends on the rank
// alone but K1's slabs for a changed d_local; any failure there (or a failed
// launch) poisons the rank's partial (NaN trailing pair) and the rank still
// joins the exchange, so every rank's finish marks the call invalid
// (MARGIN_POISONED) and the failing rank returns its own error.
int sharded_once(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t dl, int64_t ld,
                 int64_t f, int64_t *d_sel, double *d_scores, double *d_mean) {
    const int64_t usz = bk_upper_elems(n);
    const bool exch = c->comm != nullptr;
    // the call's signature, the same on every rank by the API's contract: a
    // change makes the ranks agree again (status, and the overlapped piece layout)
    const int sig = c->deterministic + 2 * c->overlap +
                    32 * (dtype == BK_F32 ? c->f32_mode : c->f64_mode);
    const bool agree = exch && (c->nranks > 1 || c->test_fail_exchange) &&
                       (n != c->agreed_n || f != c->agreed_f || dtype != c->agreed_dtype ||
                        sig != c->agreed_det);
    const ScoreSplit sp = score_split(c, n);
    int prep = ensure(c->U, (size_t)usz * sizeof(double));
    if (prep == BK_OK && exch && c->deterministic)
        prep = ensure(c->Ug, (size_t)usz * c->nranks * sizeof(double));
    if (prep == BK_OK && sp.parts > 1) prep = prepare_finish(c, n, sp, d_scores == nullptr);
    if (prep == BK_OK && dl > 0) prep = prepare_gram(c, dX, dtype, n, dl, ld);
    // bk_comm_set_mode 2: the Gram in pieces, each all-reduced on the
    // communication stream while the next computes (nullptr: this call's
    // Gram has no such split -- it is computed whole and exchanged after)
    const Pieces *pcs = nullptr;
    if (prep == BK_OK && exch && c->overlap >= 2 && !c->deterministic && dl > 0) {
        if (c->wait_value_ok < 0) {
            int v = 0;
            c->wait_value_ok = hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue,
                                                     c->device) == hipSuccess && v ? 1 : 0;
            (void)hipGetLastError();
        }
        if (c->wait_value_ok) {
            prep = gram_pieces(c, dX, dtype, n, dl, ld, c->overlap, &pcs);
            if (prep == BK_OK && pcs) prep = ensure_comm_stream(c);
        }
    }
    if (prep == BK_OK && c->test_fail_exchange == (agree ? 1 : 2))
        prep = fail(BK_ENOMEM, "test knob BK_TEST_FAIL_BEFORE_EXCHANGE=%d: forced failure",
                    c->test_fail_exchange);
    const std::string prep_msg = prep == BK_OK ? std::string() : g_err;
    if (agree) {
        // one max-all-reduce of {status, piece layout, -piece layout}: the ranks
        // learn whether any failed, and whether they all cut the Gram into the
        // same pieces (the layout's fingerprint equal on every rank: max ==
        // -max(-fp)).  A rank whose plan does not split, or a different cut,
        // turns the overlapped exchange off on every rank for this signature:
        // each piece is one collective, so the ranks must agree on them.
        double *w = (double *)c->status.p;
        double v[3] = {prep == BK_OK ? 0.0 : 1.0, 0.0, 0.0};
        if (pcs) {
            uint64_t h = 1469598103934665603ull;
            auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
            mix((uint64_t)pcs->k);
            for (int64_t x : pcs->e) mix((uint64_t)x);
            v[1] = (double)(h >> 12) + 1.0;  // 52 bits: exact in a double, never 0
        }
        v[2] = -v[1] - (c->test_pieces_disagree ? 1.0 : 0.0);
        HIPCHK(hipMemcpyAsync(w, v, sizeof v, hipMemcpyHostToDevice, c->stream));
        RCCLCHK(ncclAllReduce(w, w, 3, ncclDouble, ncclMax, c->comm, c->stream));
        HIPCHK(hipMemcpyAsync(v, w, sizeof v, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        const double any = v[0];
        c->overlap_agreed = v[1] != 0.0 && v[1] == -v[2];
        if (prep != BK_OK) {
            g_err = prep_msg;
            return prep;
        }
        if (any != 0.0)
            return fail(BK_ERCCL, "a peer rank failed before the Gram exchange (status agreement "
                                  "of the call's first signature); no exchange was made");
        c->agreed_n = n;
        c->agreed_f = f;
        c->agreed_dtype = dtype;
        c->agreed_det = sig;
    } else if (prep != BK_OK && (!exch || c->U.bytes < (size_t)usz * sizeof(double))) {
        return prep;  // nothing to join (no communicator), or no partial to poison
    }
    double *U = (double *)c->U.p;
    Plan pl;
    pl.n = (int)n;
    pl.T = (int)((n + 63) / 64);
    pl.ntile = pl.T * (pl.T + 1) / 2;
    int st = prep;
    if (!c->overlap_agreed) pcs = nullptr;  // a peer cut the Gram differently (or not at all)
    if (pcs && st == BK_OK)
        return sharded_overlapped(c, *pcs, dX, dtype, n, dl, ld, f, U, pl, d_sel, d_scores, d_mean,
                                  sp);
    if (st == BK_OK) {
        if (dl > 0) {
            st = stage_gram(c, dX, dtype, n, dl, ld, U, pl);
        } else {
            // an empty column shard (d small against the rank count): a zero
            // partial (column counts 0 too), so this rank still joins the exchange
            const hipError_t e = hipMemsetAsync(U, 0, (size_t)usz * sizeof(double), c->stream);
            if (e != hipSuccess) st = fail(BK_EHIP, "hipMemsetAsync: %s", hipGetErrorString(e));
        }
    }
    const std::string st_msg = st == BK_OK ? std::string() : g_err;
    if (st != BK_OK) CHK(poison_upper(c, U, n));
    if (exch) {  // also at 1 rank, so the exchange is exercised on a 1-GPU box
        hipEvent_t a = nullptr, b = nullptr;
        const bool ton = timing_on(c, BK_K_ALLREDUCE);
        if (ton) {
            CHK(get_event(c, &a));
            CHK(get_event(c, &b));
            HIPCHK(hipEventRecord(a, c->stream));
        }
        if (!c->deterministic) {
            RCCLCHK(ncclAllReduce(U, U, (size_t)usz, ncclDouble, ncclSum, c->comm, c->stream));
        } else {
            double *Ug = (double *)c->Ug.p;
            RCCLCHK(ncclAllGather(U, Ug, (size_t)usz, ncclDouble, c->comm, c->stream));
            HIPCHK(launch_sum_ranks(Ug, c->nranks, usz, U, c->stream));
        }
        if (ton) {
            HIPCHK(hipEventRecord(b, c->stream));
            c->pending.push_back({BK_K_ALLREDUCE, a, b});
        }
        c->exchanged_bytes += (double)usz * sizeof(double) * (c->deterministic ? c->nranks : 1);
        ++c->exchanges;
    }
    if (st != BK_OK) {
        // the rest of the finish still runs, so this rank's record says so too
        (void)stage_finish(c, U, pl, dX, dtype, n, dl, ld, f, d_sel, d_scores, nullptr, sp);
        g_err = st_msg;
        return st;
    }
    return stage_finish(c, U, pl, dX, dtype, n, dl, ld, f, d_sel, d_scores,
                        dl > 0 ? d_mean : nullptr, sp);
}
}  // namespace

int bk_multikrum_sharded_device(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t dl,
                                int64_t ld, int64_t f, int64_t *d_sel, double *d_scores,
                                double *d_mean) {
    if (dl > 0) {
        CHK(check_common(c, dX, dtype, n, dl, ld));
    } else {
        // d_local = 0 is legal (an empty trailing shard): dX, ld and d_mean are unused
        if (!c) return fail(BK_EINVAL, "null context");
        if (dl < 0) return fail(BK_EINVAL, "d_local=%lld < 0", (long long)dl);
        if (dtype != BK_F64 && dtype != BK_F32) return fail(BK_EINVAL, "bad dtype %d", dtype);
    }
    CHK(bk_check_args(n, dl > 0 ? dl : 1, f));
    if (!d_sel) return fail(BK_EINVAL, "null d_sel_idx");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    if (c->nranks > 1 && !c->comm) return fail(BK_ERCCL, "bk_comm_init not called");
    auto once = [&] { return sharded_once(c, dX, dtype, n, dl, ld, f, d_sel, d_scores, d_mean); };
    if (certified(c, dtype)) return run_certified(c, once);
    return once();
}

int bk_comm_size(bk_ctx *c, int *nranks, int *rank) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    int nr = 1, rk = 0;
    if (c->comm) {
        RCCLCHK(ncclCommCount(c->comm, &nr));
        RCCLCHK(ncclCommUserRank(c->comm, &rk));
    }
    if (nranks) *nranks = c->comm ? nr : 0;
    if (rank) *rank = rk;
    return BK_OK;
}

int bk_comm_stats(bk_ctx *c, int64_t *exchanges, double *bytes) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    if (exchanges) *exchanges = c->exchanges;
    if (bytes) *bytes = c->exchanged_bytes;
    return BK_OK;
}

int bk_selection_margin(bk_ctx *c, double *gap, double *err_bound, int *near_tie) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    double mg[MARGIN_WORDS];
    CHK(read_margin(c, mg));
    if (gap) *gap = mg[0];
    if (err_bound) *err_bound = mg[1];
    if (near_tie) *near_tie = mg[2] != 0.0 ? 1 : 0;
    return BK_OK;
}

int bk_selection_margin_record(bk_ctx *c, double *record) {
    if (!c || !record) return fail(BK_EINVAL, "null context / record");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    double mg[MARGIN_WORDS];
    CHK(read_margin(c, mg));
    memcpy(record, mg, 8 * sizeof(double));  // the public record (u_G stays internal)
    return BK_OK;
}

int64_t bk_certified_reruns(bk_ctx *c) {
    if (!c) return 0;
    std::lock_guard<std::mutex> lk(c->mu);
    return c->certified_reruns;
}

int bk_set_small_path(bk_ctx *c, int on) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->small_on != (on ? 1 : 0)) ++c->ws_epoch;  // captured graphs baked the other path in
    c->small_on = on ? 1 : 0;
    return BK_OK;
}

// ---- one process, G GPUs --------------------------------------------------
}  // extern "C"

struct bk_group {
    std::vector<bk_ctx *> ctx;
    int mode = BK_GROUP_ALLREDUCE;
    std::mutex mu;
    // per-rank device buffers of the call (shard of X, packed Gram, outputs)
    std::vector<DevBuf> X, U, Ug, sel, sc, mean;
    // BK_GROUP_HOST_EXCHANGE: pinned partials [G][usz] and their sum
    void *hpart = nullptr, *hsum = nullptr;
    size_t hbytes = 0;
};

namespace {

// the column shard of rank r out of G (biscotti_amd/dist.py:shard_bounds)
void group_shard(int64_t d, int G, int r, int64_t *c0, int64_t *dl) {
    int64_t per = (d + G - 1) / G;
    per = (per + 7) / 8 * 8;
    const int64_t a = std::min<int64_t>(d, (int64_t)r * per);
    const int64_t b = std::min<int64_t>(d, a + per);
    *c0 = a;
    *dl = b - a;
}

// Error returns of bk_group_multikrum: every device's copy stream may still be
// reading the caller's X, and D2H copies may still be writing sel / scores /
// mean_out, so all streams of all contexts are drained unless disarmed.
struct GroupDrain {
    bk_group *g;
    bool armed = true;
    ~GroupDrain() {
        if (!armed) return;
        for (bk_ctx *c : g->ctx) {
            DeviceGuard dg(c->device);
            if (c->copy) (void)hipStreamSynchronize(c->copy);
            (void)hipStreamSynchronize(c->stream);
        }
    }
};

int group_free_host(bk_group *g) {
    if (g->hpart) (void)hipHostFree(g->hpart);
    if (g->hsum) (void)hipHostFree(g->hsum);
    g->hpart = g->hsum = nullptr;
    g->hbytes = 0;
    return BK_OK;
}

}  // namespace

extern "C" {

int bk_group_create(bk_group **out, int ngpus, const int *devices, int mode) {
    if (!out) return fail(BK_EINVAL, "null out");
    *out = nullptr;
    if (ngpus < 1 || ngpus > 64) return fail(BK_EINVAL, "ngpus=%d out of range", ngpus);
    if (mode < BK_GROUP_ALLREDUCE || mode > BK_GROUP_HOST_EXCHANGE)
        return fail(BK_EINVAL, "bad group mode %d", mode);
    std::vector<int> devs((size_t)ngpus);
    for (int r = 0; r < ngpus; ++r) devs[(size_t)r] = devices ? devices[r] : r;
    if (mode != BK_GROUP_HOST_EXCHANGE)
        for (int a = 0; a < ngpus; ++a)
            for (int b = a + 1; b < ngpus; ++b)
                if (devs[(size_t)a] == devs[(size_t)b])
                    return fail(BK_EINVAL, "RCCL group modes need distinct devices (device %d "
                                           "repeats); use BK_GROUP_HOST_EXCHANGE",
                                devs[(size_t)a]);
    bk_group *g = new (std::nothrow) bk_group();
    if (!g) return fail(BK_ENOMEM, "host allocation of bk_group failed");
    g->mode = mode;
    for (int r = 0; r < ngpus; ++r) {
        bk_ctx *c = nullptr;
        const int st = bk_create(&c, devs[(size_t)r]);
        if (st != BK_OK) {
            bk_group_destroy(g);
            return st;
        }
        g->ctx.push_back(c);
    }
    const size_t G = (size_t)ngpus;
    g->X.resize(G);
    g->U.resize(G);
    g->Ug.resize(G);
    g->sel.resize(G);
    g->sc.resize(G);
    g->mean.resize(G);
    if (mode != BK_GROUP_HOST_EXCHANGE) {
        std::vector<ncclComm_t> comms(G, nullptr);
        const ncclResult_t r = ncclCommInitAll(comms.data(), ngpus, devs.data());
        if (r != ncclSuccess) {
            bk_group_destroy(g);
            return fail(BK_ERCCL, "ncclCommInitAll(%d): %s", ngpus, ncclGetErrorString(r));
        }
        for (int k = 0; k < ngpus; ++k) {  // each context owns (and destroys) its rank
            g->ctx[(size_t)k]->comm = comms[(size_t)k];
            g->ctx[(size_t)k]->nranks = ngpus;
            g->ctx[(size_t)k]->rank = k;
        }
    }
    *out = g;
    return BK_OK;
}

void bk_group_destroy(bk_group *g) {
    if (!g) return;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        bk_ctx *c = g->ctx[r];
        {
            DeviceGuard dg(c->device);
            (void)hipStreamSynchronize(c->stream);
            for (auto *v : {&g->X, &g->U, &g->Ug, &g->sel, &g->sc, &g->mean})
                if (r < v->size() && (*v)[r].p) (void)hipFree((*v)[r].p);
        }
        bk_destroy(c);
    }
    group_free_host(g);
    delete g;
}

int bk_group_size(const bk_group *g) { return g ? (int)g->ctx.size() : 0; }

bk_ctx *bk_group_ctx(bk_group *g, int r) {
    if (!g || r < 0 || r >= (int)g->ctx.size()) return nullptr;
    return g->ctx[(size_t)r];
}

int bk_group_multikrum(bk_group *g, const void *X, int where, int dtype, int64_t n, int64_t d,
                       int64_t ld, int64_t f, int64_t *sel_idx, int64_t *m_out, double *scores,
                       double *mean_out) {
    if (!g || g->ctx.empty()) return fail(BK_EINVAL, "null group");
    CHK(check_common(g->ctx[0], X, dtype, n, d, ld));
    CHK(bk_check_args(n, d, f));
    if (!sel_idx) return fail(BK_EINVAL, "null sel_idx");
    if (where != BK_HOST && where != BK_HOST_PINNED)
        return fail(BK_EINVAL, "bk_group_multikrum takes host X (where=%d)", where);
    const int G = (int)g->ctx.size();
    // Biscotti's deployed shapes (n <= 128, small d: configs A and B) are one
    // launch on one device (k_small); splitting them over devices only adds
    // copies and an exchange
    if (small_ok(g->ctx[0], X, dtype, n, d, ld))
        return bk_multikrum(g->ctx[0], X, where, dtype, n, d, ld, f, sel_idx, m_out, scores,
                            mean_out);
    for (int r = 0; r < G; ++r) {
        int64_t c0, dl;
        group_shard(d, G, r, &c0, &dl);
        if (dl < 1)  // d too small to give every device a column: one device does it all
            return bk_multikrum(g->ctx[0], X, where, dtype, n, d, ld, f, sel_idx, m_out, scores,
                                mean_out);
    }
    std::lock_guard<std::mutex> lk(g->mu);
    std::vector<std::unique_lock<std::mutex>> locks;
    for (bk_ctx *c : g->ctx) locks.emplace_back(c->mu);  // fixed order: no deadlock
    const size_t es = esize(dtype);
    const int64_t m = n - f;
    const int64_t usz = bk_upper_elems(n);
    std::vector<Plan> pls((size_t)G);
    GroupDrain drain{g};
    // 1. per device: its column shard crosses PCIe in column chunks on the
    //    device's copy stream, each chunk's partial Gram (K1 + K1b) overlapped
    //    with the next chunk's copy (stage_host_pipelined)
    for (int r = 0; r < G; ++r) {
        bk_ctx *c = g->ctx[(size_t)r];
        DeviceGuard dg(c->device);
        int64_t c0, dl;
        group_shard(d, G, r, &c0, &dl);
        CHK(ensure(g->X[(size_t)r], (size_t)n * dl * es));
        CHK(ensure(g->U[(size_t)r], (size_t)usz * sizeof(double)));
        const char *src = (const char *)X + (size_t)c0 * es;
        CHK(stage_host_pipelined(c, src, ld, dtype, nullptr, 0, 0, n, dl, (char *)g->X[(size_t)r].p,
                                 dl, (double *)g->U[(size_t)r].p, pls[(size_t)r]));
    }
    // 2.-3. the exchange, then per device the finish and the outputs back
    auto exchange_finish = [&]() -> int {
    if (g->mode == BK_GROUP_ALLREDUCE) {
        RCCLCHK(ncclGroupStart());
        for (int r = 0; r < G; ++r) {
            bk_ctx *c = g->ctx[(size_t)r];
            double *U = (double *)g->U[(size_t)r].p;
            const ncclResult_t e =
                ncclAllReduce(U, U, (size_t)usz, ncclDouble, ncclSum, c->comm, c->stream);
            if (e != ncclSuccess) {
                (void)ncclGroupEnd();
                return fail(BK_ERCCL, "ncclAllReduce: %s", ncclGetErrorString(e));
            }
        }
        RCCLCHK(ncclGroupEnd());
    } else if (g->mode == BK_GROUP_DETERMINISTIC) {
        for (int r = 0; r < G; ++r) {
            DeviceGuard dg(g->ctx[(size_t)r]->device);
            CHK(ensure(g->Ug[(size_t)r], (size_t)usz * G * sizeof(double)));
        }
        RCCLCHK(ncclGroupStart());
        for (int r = 0; r < G; ++r) {
            bk_ctx *c = g->ctx[(size_t)r];
            const ncclResult_t e = ncclAllGather(g->U[(size_t)r].p, g->Ug[(size_t)r].p,
                                                 (size_t)usz, ncclDouble, c->comm, c->stream);
            if (e != ncclSuccess) {
                (void)ncclGroupEnd();
                return fail(BK_ERCCL, "ncclAllGather: %s", ncclGetErrorString(e));
            }
        }
        RCCLCHK(ncclGroupEnd());
        for (int r = 0; r < G; ++r) {
            bk_ctx *c = g->ctx[(size_t)r];
            DeviceGuard dg(c->device);
            HIPCHK(launch_sum_ranks((const double *)g->Ug[(size_t)r].p, G, usz,
                                    (double *)g->U[(size_t)r].p, c->stream));
        }
    } else {  // host exchange: D2H partials, fixed rank-order sum, H2D
        const size_t bytes = (size_t)usz * sizeof(double);
        if (g->hbytes < bytes) {
            group_free_host(g);
            HIPCHK(hipHostMalloc(&g->hpart, bytes * G, hipHostMallocPortable));
            HIPCHK(hipHostMalloc(&g->hsum, bytes, hipHostMallocPortable));
            g->hbytes = bytes;
        }
        double *hp = (double *)g->hpart, *hs = (double *)g->hsum;
        for (int r = 0; r < G; ++r) {
            bk_ctx *c = g->ctx[(size_t)r];
            DeviceGuard dg(c->device);
            HIPCHK(hipMemcpyAsync(hp + (size_t)r * usz, g->U[(size_t)r].p, bytes,
                                  hipMemcpyDeviceToHost, c->stream));
        }
        for (int r = 0; r < G; ++r) {
            DeviceGuard dg(g->ctx[(size_t)r]->device);
            HIPCHK(hipStreamSynchronize(g->ctx[(size_t)r]->stream));
        }
        for (int64_t e = 0; e < usz; ++e) {  // the order of k_sum_ranks: 0 + U_0 + U_1 + ...
            double acc = 0.0;
            for (int r = 0; r < G; ++r) acc += hp[(size_t)r * usz + e];
            hs[e] = acc;
        }
        for (int r = 0; r < G; ++r) {
            bk_ctx *c = g->ctx[(size_t)r];
            DeviceGuard dg(c->device);
            HIPCHK(hipMemcpyAsync(g->U[(size_t)r].p, hs, bytes, hipMemcpyHostToDevice, c->stream));
        }
    }
    // 3. per device: scores + selection (identical everywhere), mean of its columns
    for (int r = 0; r < G; ++r) {
        bk_ctx *c = g->ctx[(size_t)r];
        DeviceGuard dg(c->device);
        int64_t c0, dl;
        group_shard(d, G, r, &c0, &dl);
        CHK(ensure(g->sel[(size_t)r], (size_t)n * sizeof(int64_t)));
        CHK(ensure(g->sc[(size_t)r], (size_t)n * sizeof(double)));
        double *dmean = nullptr;
        if (mean_out) {
            CHK(ensure(g->mean[(size_t)r], (size_t)dl * sizeof(double)));
            dmean = (double *)g->mean[(size_t)r].p;
        }
        int64_t *dsel = (int64_t *)g->sel[(size_t)r].p;
        double *dsc = (double *)g->sc[(size_t)r].p;
        CHK(stage_finish(c, (const double *)g->U[(size_t)r].p, pls[(size_t)r], g->X[(size_t)r].p,
                         dtype, n, dl, dl, f, dsel, dsc, dmean));
        CHK(timed(c, BK_K_D2H, [&] {
            hipError_t e = hipSuccess;
            if (r == 0) {
                e = hipMemcpyAsync(sel_idx, dsel, (size_t)m * sizeof(int64_t),
                                   hipMemcpyDeviceToHost, c->stream);
                if (e == hipSuccess && scores)
                    e = hipMemcpyAsync(scores, dsc, (size_t)n * sizeof(double),
                                       hipMemcpyDeviceToHost, c->stream);
            }
            if (e == hipSuccess && mean_out)
                e = hipMemcpyAsync(mean_out + c0, dmean, (size_t)dl * sizeof(double),
                                   hipMemcpyDeviceToHost, c->stream);
            return e;
        }));
    }
    for (int r = 0; r < G; ++r) {
        DeviceGuard dg(g->ctx[(size_t)r]->device);
        HIPCHK(hipStreamSynchronize(g->ctx[(size_t)r]->stream));
    }
    for (int r = 0; r < G; ++r) CHK(check_margin_readback(g->ctx[(size_t)r]));
    return BK_OK;
    };
    CHK(exchange_finish());
    // BK_F32_CERTIFIED (set on the group's contexts): a near tie of a Gram
    // taken on the fp32 MFMA is re-run exact from the device-resident shards.
    // Every device holds the same summed record, so device 0's margin decides.
    bk_ctx *c0x = g->ctx[0];
    if (certified(c0x, dtype) && c0x->margin_host[2] == 1.0 && c0x->margin_host[8] > 0x1p-53) {
        for (bk_ctx *c : g->ctx) c->force_exact = 1;
        int st = BK_OK;
        for (int r = 0; r < G && st == BK_OK; ++r) {
            bk_ctx *c = g->ctx[(size_t)r];
            DeviceGuard dg(c->device);
            int64_t c0, dl;
            group_shard(d, G, r, &c0, &dl);
            st = stage_gram(c, g->X[(size_t)r].p, dtype, n, dl, dl, (double *)g->U[(size_t)r].p,
                            pls[(size_t)r]);
        }
        if (st == BK_OK) st = exchange_finish();
        for (bk_ctx *c : g->ctx) c->force_exact = 0;
        CHK(st);
        ++c0x->certified_reruns;
    }
    drain.armed = false;
    if (m_out) *m_out = m;
    return BK_OK;
}

int bk_synth_fill_device(bk_ctx *c, void *dX, int dtype, int64_t n, int64_t dl, int64_t ld,
                         int64_t c0, int64_t d_total, uint64_t seed, int64_t nbyz, double mu_scale,
                         double byz_scale, double sigma, int flags) {
    CHK(check_common(c, dX, dtype, n, dl, ld));
    if (c0 < 0 || c0 + dl > d_total || nbyz < 0 || nbyz > n)
        return fail(BK_EINVAL, "bad synth column range / nbyz");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    // Fisher-Yates on the host (sequential by definition), then upload
    std::vector<int64_t> perm((size_t)n);
    const uint64_t b3 = stream_base(seed, 3);
    for (int64_t i = 0; i < n; ++i) perm[(size_t)i] = i;
    for (int64_t i = n - 1; i >= 1; --i) {
        const int64_t j = (int64_t)(sm64(b3 + (uint64_t)i) % (uint64_t)(i + 1));
        const int64_t t = perm[(size_t)i];
        perm[(size_t)i] = perm[(size_t)j];
        perm[(size_t)j] = t;
    }
    CHK(ensure(c->perm, (size_t)n * sizeof(int64_t)));
    HIPCHK(hipMemcpyAsync(c->perm.p, perm.data(), (size_t)n * sizeof(int64_t),
                          hipMemcpyHostToDevice, c->stream));
    SynthParams P;
    P.b0 = stream_base(seed, 0);
    P.b1 = stream_base(seed, 1);
    P.b2 = stream_base(seed, 2);
    P.b4 = stream_base(seed, 4);
    P.n = n;
    P.nbyz = nbyz;
    P.d_total = d_total;
    P.mu_scale = mu_scale;
    P.byz_scale = byz_scale;
    P.sigma = sigma;
    P.flags = flags;
    const int64_t *dperm = (const int64_t *)c->perm.p;
    CHK(timed(c, BK_K_SYNTH,
              [&] { return launch_synth(dX, dtype, ld, n, dl, c0, dperm, P, c->stream); }));
    // the host perm vector dies here: make sure the (pageable) copy has landed
    HIPCHK(hipStreamSynchronize(c->stream));
    return BK_OK;
}

int bk_timing_enable(bk_ctx *c, int on) {
    return bk_timing_select(c, on ? ~0u : 0u);
}

namespace {
// drop the accumulated timings and pending events (under c->mu)
int timing_reset(bk_ctx *c) {
    DeviceGuard dg(c->device);
    HIPCHK(hipStreamSynchronize(c->stream));
    for (auto &ev : c->pending) {
        c->pool.push_back(ev.a);
        c->pool.push_back(ev.b);
    }
    c->pending.clear();
    for (int i = 0; i < BK_NUM_KERNELS; ++i) {
        c->tot_ms[i] = 0;
        c->cnt[i] = 0;
        c->tseq[i] = 0;
    }
    return BK_OK;
}
}  // namespace

int bk_timing_stride(bk_ctx *c, int every) {
    if (!c) return fail(BK_EINVAL, "null context");
    if (every < 1) return fail(BK_EINVAL, "timing stride %d < 1", every);
    std::lock_guard<std::mutex> lk(c->mu);
    c->tstride = every;
    return timing_reset(c);  // clears, keeps the selection
}

int bk_timing_select(bk_ctx *c, uint32_t mask) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    c->timing = mask;
    return timing_reset(c);
}

int bk_timing_read(bk_ctx *c, int kid, double *total_ms, int64_t *count) {
    if (!c || kid < 0 || kid >= BK_NUM_KERNELS) return fail(BK_EINVAL, "bad timing_read arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    if (!c->pending.empty()) {
        HIPCHK(hipStreamSynchronize(c->stream));
        for (auto &ev : c->pending) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, ev.a, ev.b));
            c->tot_ms[ev.kid] += ms;
            c->cnt[ev.kid] += 1;
            c->pool.push_back(ev.a);
            c->pool.push_back(ev.b);
        }
        c->pending.clear();
    }
    if (total_ms) *total_ms = c->tot_ms[kid];
    if (count) *count = c->cnt[kid];
    return BK_OK;
}

}  // extern "C"

// ---- block aggregation, quantised sum, noise ------
static int check_rows(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld,
                      int64_t m) {
    CHK(check_common(c, dX, dtype, n, d, ld));
    if (m < 0) return fail(BK_EINVAL, "m=%lld < 0", (long long)m);
    if (m > BK_MAX_N) return fail(BK_ENOTSUP, "m=%lld exceeds BK_MAX_N=%d", (long long)m, BK_MAX_N);
    return BK_OK;
}

int bk_aggregate_device(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d, int64_t ld,
                        const int64_t *d_idx, int64_t m, double *d_global) {
    CHK(check_rows(c, dX, dtype, n, d, ld, m));
    if (!d_global || (m > 0 && !d_idx)) return fail(BK_EINVAL, "null d_idx / d_global");
    if (m == 0) return BK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    return timed(c, BK_K_AGGREGATE, [&] {
        return launch_accumulate(dX, dtype, ld, d, d_idx, (int)m, d_global, c->num_cu, c->stream);
    });
}

int bk_aggregate(bk_ctx *c, const void *X, int where, int dtype, int64_t n, int64_t d, int64_t ld,
                 const int64_t *idx, int64_t m, double *global) {
    CHK(check_rows(c, X, dtype, n, d, ld, m));
    if (!global || (m > 0 && !idx)) return fail(BK_EINVAL, "null idx / global");
    if (where != BK_HOST && where != BK_HOST_PINNED && where != BK_DEVICE)
        return fail(BK_EINVAL, "bad where=%d", where);
    for (int64_t r = 0; r < m; ++r)
        if (idx[r] < 0 || idx[r] >= n)
            return fail(BK_EINVAL, "idx[%lld]=%lld out of [0,%lld)", (long long)r,
                        (long long)idx[r], (long long)n);
    if (m == 0) return BK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    // on an error return, queued copies may still read X / hidx / global
    HostDrain drain{c};
    const size_t es = esize(dtype);
    const void *dX = X;
    int64_t dld = ld;
    if (where != BK_DEVICE) {
        // only the accepted rows cross PCIe: gather them (in idx order) into the stage
        CHK(ensure(c->X, (size_t)m * d * es));
        char *dst = (char *)c->X.p;
        CHK(timed(c, BK_K_H2D, [&] {
            hipError_t e = hipSuccess;
            for (int64_t r = 0; r < m && e == hipSuccess; ++r)
                e = hipMemcpyAsync(dst + (size_t)r * d * es, (const char *)X + (size_t)idx[r] * ld * es,
                                   (size_t)d * es, hipMemcpyHostToDevice, c->stream);
            return e;
        }));
        dX = dst;
        dld = d;
    }
    CHK(ensure(c->idx, (size_t)m * sizeof(int64_t)));
    CHK(ensure(c->mean, (size_t)d * sizeof(double)));
    int64_t *didx = (int64_t *)c->idx.p;
    double *dglob = (double *)c->mean.p;
    std::vector<int64_t> hidx((size_t)m);
    for (int64_t r = 0; r < m; ++r) hidx[r] = where != BK_DEVICE ? r : idx[r];
    HIPCHK(hipMemcpyAsync(didx, hidx.data(), (size_t)m * sizeof(int64_t), hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(hipMemcpyAsync(dglob, global, (size_t)d * sizeof(double), hipMemcpyHostToDevice,
                          c->stream));
    CHK(timed(c, BK_K_AGGREGATE, [&] {
        return launch_accumulate(dX, dtype, dld, d, didx, (int)m, dglob, c->num_cu, c->stream);
    }));
    CHK(timed(c, BK_K_D2H, [&] {
        return hipMemcpyAsync(global, dglob, (size_t)d * sizeof(double), hipMemcpyDeviceToHost,
                              c->stream);
    }));
    HIPCHK(hipStreamSynchronize(c->stream));
    drain.armed = false;
    return BK_OK;
}

int bk_quantized_sum_device(bk_ctx *c, const void *dX, int dtype, int64_t n, int64_t d,
                            int64_t ld, const int64_t *d_idx, int64_t m, int precision,
                            int64_t *d_sum, double *d_sum_float) {
    CHK(check_rows(c, dX, dtype, n, d, ld, m));
    if (!d_sum || (m > 0 && !d_idx)) return fail(BK_EINVAL, "null d_idx / d_sum");
    if (precision < 0 || precision > 18)
        return fail(BK_EINVAL, "precision=%d outside [0, 18]", precision);
    double scale = 1.0;  // 10^p, exact for p <= 22 (what Go's math.Pow(10, p) returns)
    for (int i = 0; i < precision; ++i) scale *= 10.0;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    return timed(c, BK_K_QSUM, [&] {
        return launch_qsum(dX, dtype, ld, d, d_idx, (int)m, scale, d_sum, d_sum_float, c->num_cu,
                           c->stream);
    });
}

int bk_noise_apply_device(bk_ctx *c, const double *d_delta, int64_t n, int64_t d, int64_t ld,
                          const double *d_noise, int64_t k, int64_t noise_ld, double *d_out,
                          int64_t out_ld) {
    CHK(check_common(c, d_delta, BK_F64, n, d, ld));
    if (!d_out || (k > 0 && !d_noise)) return fail(BK_EINVAL, "null d_noise / d_out");
    if (k < 0) return fail(BK_EINVAL, "k=%lld < 0", (long long)k);
    if (k > 0 && noise_ld < d) return fail(BK_EINVAL, "noise_ld=%lld < d", (long long)noise_ld);
    if (out_ld < d) return fail(BK_EINVAL, "out_ld=%lld < d", (long long)out_ld);
    if (d_out == d_delta && out_ld != ld) return fail(BK_EINVAL, "in-place needs out_ld == ld");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    return timed(c, BK_K_NOISE, [&] {
        return launch_noise(d_delta, ld, n, d, d_noise, k, noise_ld, d_out, out_ld, c->num_cu,
                            c->stream);
    });
}

// ---- RONI ------------------------------------------
static int check_roni(int64_t nv, int64_t d, int64_t ldv, int64_t n, int64_t ld) {
    if (nv < 1 || d < 1) return fail(BK_EINVAL, "need nv >= 1 and d >= 1");
    if (ldv < d) return fail(BK_EINVAL, "ldv=%lld < d=%lld", (long long)ldv, (long long)d);
    if (n < 0) return fail(BK_EINVAL, "n=%lld < 0", (long long)n);
    if (n > 0 && ld < d) return fail(BK_EINVAL, "ld=%lld < d=%lld", (long long)ld, (long long)d);
    if (n > 65534) return fail(BK_ENOTSUP, "RONI n=%lld exceeds 65534", (long long)n);
    if (d > ((int64_t)1 << 21)) return fail(BK_ENOTSUP, "RONI d=%lld exceeds 2^21", (long long)d);
    return BK_OK;
}

int bk_roni_device(bk_ctx *c, const double *d_Xv, int64_t nv, int64_t d, int64_t ldv,
                   const double *d_yv, const double *d_ww, const double *d_deltas, int64_t n,
                   int64_t ld, double *d_scores) {
    if (!c) return fail(BK_EINVAL, "null context");
    CHK(check_roni(nv, d, ldv, n, ld));
    if (!d_Xv || !d_yv || !d_ww || (n > 0 && (!d_deltas || !d_scores)))
        return fail(BK_EINVAL, "null pointer argument");
    if (n == 0) return BK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    CHK(ensure(c->roni_cnt, (size_t)(n + 1) * sizeof(unsigned int)));
    CHK(ensure(c->rmc_ws, roni_ws(n, d)));
    unsigned int *cnt = (unsigned int *)c->roni_cnt.p;
    return timed(c, BK_K_RONI, [&] {
        return launch_roni(d_Xv, nv, d, ldv, d_yv, d_ww, d_deltas, n, ld, (double *)c->rmc_ws.p, cnt,
                           d_scores, c->stream);
    });
}

int bk_roni_set_validation(bk_ctx *c, const double *Xv, int64_t nv, int64_t d, int64_t ldv,
                           const double *yv) {
    if (!c) return fail(BK_EINVAL, "null context");
    CHK(check_roni(nv, d, ldv, 0, d));
    if (!Xv || !yv) return fail(BK_EINVAL, "null Xv / yv");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    c->roni_nv = 0;  // invalid until the new set has landed
    HostDrain drain{c};
    CHK(ensure(c->roni_X, (size_t)nv * d * sizeof(double)));
    CHK(ensure(c->roni_y, (size_t)nv * sizeof(double)));
    HIPCHK(hipMemcpy2DAsync(c->roni_X.p, (size_t)d * sizeof(double), Xv, (size_t)ldv * sizeof(double),
                            (size_t)d * sizeof(double), (size_t)nv, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->roni_y.p, yv, (size_t)nv * sizeof(double), hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    drain.armed = false;
    c->roni_nv = nv;
    c->roni_dim = d;
    return BK_OK;
}

int bk_roni(bk_ctx *c, const double *ww, const double *deltas, int64_t n, int64_t d, int64_t ld,
            double *scores) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);  // roni_nv / roni_dim change under it
    if (c->roni_nv < 1) return fail(BK_EINVAL, "no validation set: call bk_roni_set_validation");
    if (d != c->roni_dim)
        return fail(BK_EINVAL, "d=%lld != validation set's %lld", (long long)d, (long long)c->roni_dim);
    CHK(check_roni(c->roni_nv, d, d, n, ld));
    if (!ww || (n > 0 && (!deltas || !scores))) return fail(BK_EINVAL, "null pointer argument");
    if (n == 0) return BK_OK;
    DeviceGuard dg(c->device);
    HostDrain drain{c};  // error returns: queued H2D copies may still read ww / deltas
    CHK(ensure(c->roni_w, (size_t)d * sizeof(double)));
    CHK(ensure(c->roni_d, (size_t)n * d * sizeof(double)));
    CHK(ensure(c->roni_s, (size_t)n * sizeof(double)));
    CHK(ensure(c->roni_cnt, (size_t)(n + 1) * sizeof(unsigned int)));
    CHK(ensure(c->rmc_ws, roni_ws(n, d)));
    double *dw = (double *)c->roni_w.p, *dd = (double *)c->roni_d.p, *ds = (double *)c->roni_s.p;
    CHK(timed(c, BK_K_H2D, [&] {
        hipError_t e = hipMemcpyAsync(dw, ww, (size_t)d * sizeof(double), hipMemcpyHostToDevice,
                                      c->stream);
        if (e == hipSuccess)
            e = hipMemcpy2DAsync(dd, (size_t)d * sizeof(double), deltas, (size_t)ld * sizeof(double),
                                 (size_t)d * sizeof(double), (size_t)n, hipMemcpyHostToDevice,
                                 c->stream);
        return e;
    }));
    CHK(timed(c, BK_K_RONI, [&] {
        return launch_roni((const double *)c->roni_X.p, c->roni_nv, d, d,
                           (const double *)c->roni_y.p, dw, dd, n, d, (double *)c->rmc_ws.p,
                           (unsigned int *)c->roni_cnt.p, ds, c->stream);
    }));
    CHK(timed(c, BK_K_D2H, [&] {
        return hipMemcpyAsync(scores, ds, (size_t)n * sizeof(double), hipMemcpyDeviceToHost,
                              c->stream);
    }));
    HIPCHK(hipStreamSynchronize(c->stream));
    drain.armed = false;
    return BK_OK;
}

// ---- SURVEY.md §8(f) row 4, the torch path: the softmax-model RONI --------
static int check_roni_softmax(int64_t nv, int64_t din, int64_t ldv, int64_t C, int64_t n,
                              int64_t ld) {
    if (nv < 1 || din < 1) return fail(BK_EINVAL, "need nv >= 1 and d_in >= 1");
    if (ldv < din) return fail(BK_EINVAL, "ldv=%lld < d_in=%lld", (long long)ldv, (long long)din);
    if (C < 2 || C > 16) return fail(BK_ENOTSUP, "n_classes=%lld outside [2, 16]", (long long)C);
    if (n < 0) return fail(BK_EINVAL, "n=%lld < 0", (long long)n);
    if (n > 0 && ld < C * (din + 1))
        return fail(BK_EINVAL, "ld=%lld < n_classes * (d_in + 1) = %lld", (long long)ld,
                    (long long)(C * (din + 1)));
    if (n > 262139) return fail(BK_ENOTSUP, "RONI n=%lld exceeds 262139", (long long)n);
    if (nv > ((int64_t)1 << 31)) return fail(BK_ENOTSUP, "RONI nv=%lld too large", (long long)nv);
    if (din > ((int64_t)1 << 21)) return fail(BK_ENOTSUP, "RONI d_in=%lld exceeds 2^21", (long long)din);
    return BK_OK;
}

int bk_roni_softmax_device(bk_ctx *c, const float *d_Xv, int64_t nv, int64_t d_in, int64_t ldv,
                           const int32_t *d_yv, int64_t n_classes, const double *d_ww,
                           const double *d_deltas, int64_t n, int64_t ld, double *d_scores,
                           int32_t *d_near_ties) {
    if (!c) return fail(BK_EINVAL, "null context");
    CHK(check_roni_softmax(nv, d_in, ldv, n_classes, n, ld));
    if (!d_Xv || !d_yv || !d_ww || (n > 0 && (!d_deltas || !d_scores)))
        return fail(BK_EINVAL, "null pointer argument");
    if (n == 0) return BK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    CHK(ensure(c->rmc_ws, roni_softmax_ws(n, d_in, nv, (int)n_classes)));
    CHK(ensure(c->roni_cnt, (size_t)2 * (n + 1) * sizeof(unsigned int)));
    return timed(c, BK_K_RONI, [&] {
        return launch_roni_softmax(d_Xv, nv, d_in, ldv, d_yv, (int)n_classes, d_ww, d_deltas, n,
                                   ld, (double *)c->rmc_ws.p, nullptr, (unsigned int *)c->roni_cnt.p,
                                   d_scores, d_near_ties, c->stream);
    });
}

int bk_roni_softmax_batches_device(bk_ctx *c, const float *d_Xv, int64_t nv, int64_t d_in,
                                   int64_t ldv, const int32_t *d_yv, int64_t n_classes,
                                   const double *d_ww, const double *d_deltas, int64_t n,
                                   int64_t ld, const int64_t *d_idx, int64_t nb, double *d_scores,
                                   int32_t *d_near_ties) {
    if (!c) return fail(BK_EINVAL, "null context");
    CHK(check_roni_softmax(nv, d_in, ldv, n_classes, n, ld));
    if (nb < 1) return fail(BK_EINVAL, "need a batch of nb >= 1 samples (nb=%lld)", (long long)nb);
    if (n > 0x7fffffff) return fail(BK_ENOTSUP, "RONI n=%lld exceeds the grid", (long long)n);
    if (!d_Xv || !d_yv || !d_ww || (n > 0 && (!d_deltas || !d_scores || !d_idx)))
        return fail(BK_EINVAL, "null pointer argument");
    if (n == 0) return BK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    return timed(c, BK_K_RONI, [&] {
        return launch_roni_softmax_batches(d_Xv, nv, d_in, ldv, d_yv, (int)n_classes, d_ww,
                                           d_deltas, n, ld, d_idx, nb, d_scores, d_near_ties,
                                           c->stream);
    });
}

int bk_roni_softmax_set_validation(bk_ctx *c, const float *Xv, int64_t nv, int64_t d_in,
                                   int64_t ldv, const int32_t *yv, int64_t n_classes) {
    if (!c) return fail(BK_EINVAL, "null context");
    CHK(check_roni_softmax(nv, d_in, ldv, n_classes, 0, 0));
    if (!Xv || !yv) return fail(BK_EINVAL, "null Xv / yv");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    c->rmc_nv = 0;  // invalid until the new set has landed
    HostDrain drain{c};
    CHK(ensure(c->rmc_X, (size_t)nv * d_in * sizeof(float)));
    CHK(ensure(c->rmc_y, (size_t)nv * sizeof(int32_t)));
    CHK(ensure(c->rmc_xn, (size_t)nv * sizeof(double)));
    HIPCHK(hipMemcpy2DAsync(c->rmc_X.p, (size_t)d_in * sizeof(float), Xv, (size_t)ldv * sizeof(float),
                            (size_t)d_in * sizeof(float), (size_t)nv, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->rmc_y.p, yv, (size_t)nv * sizeof(int32_t), hipMemcpyHostToDevice,
                          c->stream));
    // the samples' norms (the near-tie bound), once per validation set
    HIPCHK(launch_roni_xnorm((const float *)c->rmc_X.p, nv, d_in, d_in, (double *)c->rmc_xn.p,
                             c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    drain.armed = false;
    c->rmc_nv = nv;
    c->rmc_din = d_in;
    c->rmc_C = n_classes;
    return BK_OK;
}

// the host forms: ww / deltas (and the batches' indices) to the device, K8,
// scores and near-tie counts back; synchronous
static int roni_softmax_host(bk_ctx *c, const double *ww, const double *deltas, int64_t n,
                             int64_t ld, const int64_t *idx, int64_t nb, double *scores,
                             int32_t *near_ties) {
    if (!c) return fail(BK_EINVAL, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->rmc_nv < 1) return fail(BK_EINVAL, "no validation set: call bk_roni_softmax_set_validation");
    const int64_t nv = c->rmc_nv, din = c->rmc_din, C = c->rmc_C, d = C * (din + 1);
    CHK(check_roni_softmax(nv, din, din, C, n, ld));
    if (!ww || (n > 0 && (!deltas || !scores))) return fail(BK_EINVAL, "null pointer argument");
    if (idx) {
        if (nb < 1) return fail(BK_EINVAL, "need a batch of nb >= 1 samples (nb=%lld)", (long long)nb);
        if (n > 0x7fffffff) return fail(BK_ENOTSUP, "RONI n=%lld exceeds the grid", (long long)n);
        for (int64_t i = 0; i < 2 * n * nb; ++i)
            if (idx[i] < 0 || idx[i] >= nv)
                return fail(BK_EINVAL, "batch index %lld = %lld outside [0, %lld)", (long long)i,
                            (long long)idx[i], (long long)nv);
    }
    if (n == 0) return BK_OK;
    DeviceGuard dg(c->device);
    HostDrain drain{c};  // error returns: queued H2D copies may still read ww / deltas
    const int64_t nnt = idx ? 2 * n : n + 1;
    CHK(ensure(c->roni_w, (size_t)d * sizeof(double)));
    CHK(ensure(c->roni_d, (size_t)n * d * sizeof(double)));
    CHK(ensure(c->roni_s, (size_t)n * sizeof(double)));
    CHK(ensure(c->rmc_nt, (size_t)nnt * sizeof(int32_t)));
    if (idx) CHK(ensure(c->rmc_idx, (size_t)2 * n * nb * sizeof(int64_t)));
    if (!idx) {
        CHK(ensure(c->rmc_ws, roni_softmax_ws(n, din, nv, (int)C)));
        CHK(ensure(c->roni_cnt, (size_t)2 * (n + 1) * sizeof(unsigned int)));
    }
    double *dw = (double *)c->roni_w.p, *dd = (double *)c->roni_d.p, *ds = (double *)c->roni_s.p;
    int32_t *dnt = (int32_t *)c->rmc_nt.p;
    CHK(timed(c, BK_K_H2D, [&] {
        hipError_t e = hipMemcpyAsync(dw, ww, (size_t)d * sizeof(double), hipMemcpyHostToDevice,
                                      c->stream);
        if (e == hipSuccess)
            e = hipMemcpy2DAsync(dd, (size_t)d * sizeof(double), deltas, (size_t)ld * sizeof(double),
                                 (size_t)d * sizeof(double), (size_t)n, hipMemcpyHostToDevice,
                                 c->stream);
        if (e == hipSuccess && idx)
            e = hipMemcpyAsync(c->rmc_idx.p, idx, (size_t)2 * n * nb * sizeof(int64_t),
                               hipMemcpyHostToDevice, c->stream);
        return e;
    }));
    CHK(timed(c, BK_K_RONI, [&] {
        if (idx)
            return launch_roni_softmax_batches((const float *)c->rmc_X.p, nv, din, din,
                                               (const int32_t *)c->rmc_y.p, (int)C, dw, dd, n, d,
                                               (const int64_t *)c->rmc_idx.p, nb, ds, dnt,
                                               c->stream);
        return launch_roni_softmax((const float *)c->rmc_X.p, nv, din, din,
                                   (const int32_t *)c->rmc_y.p, (int)C, dw, dd, n, d,
                                   (double *)c->rmc_ws.p, (const double *)c->rmc_xn.p,
                                   (unsigned int *)c->roni_cnt.p, ds, dnt, c->stream);
    }));
    CHK(timed(c, BK_K_D2H, [&] {
        hipError_t e = hipMemcpyAsync(scores, ds, (size_t)n * sizeof(double), hipMemcpyDeviceToHost,
                                      c->stream);
        if (e == hipSuccess && near_ties)
            e = hipMemcpyAsync(near_ties, dnt, (size_t)nnt * sizeof(int32_t),
                               hipMemcpyDeviceToHost, c->stream);
        return e;
    }));
    HIPCHK(hipStreamSynchronize(c->stream));
    drain.armed = false;
    return BK_OK;
}

int bk_roni_softmax(bk_ctx *c, const double *ww, const double *deltas, int64_t n, int64_t ld,
                    double *scores, int32_t *near_ties) {
    return roni_softmax_host(c, ww, deltas, n, ld, nullptr, 0, scores, near_ties);
}

int bk_roni_softmax_batches(bk_ctx *c, const double *ww, const double *deltas, int64_t n,
                            int64_t ld, const int64_t *idx, int64_t nb, double *scores,
                            int32_t *near_ties) {
    if (!idx && n > 0) return fail(BK_EINVAL, "null batch indices");
    return roni_softmax_host(c, ww, deltas, n, ld, idx, nb, scores, near_ties);
}
