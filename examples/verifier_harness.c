/*
 * examples/verifier_harness.c -- Biscotti's Krum verifier flow, replayed in C
 * with pthreads over libbk.so (no Go toolchain in this image; SURVEY.md §8(f)
 * row 1).  It mirrors, call for call, what the cgo shim go/bk/krum_bk.go does
 * inside DistSys/krum.go:
 *
 *   Peer.VerifyUpdateKRUM        krum.go:227-365   one thread per arriving peer:
 *     krumLock; if collecting: append to UpdateList; the KRUM_UPDATETHRESH-th
 *     arrival stops collecting, signals krumReceived, sorts by SourceID,
 *     computeScores, and hands krumAccepted to the THRESH-1 waiters; the others
 *     unlock and wait on krumAccepted; then checkIfAccepted(SourceID).
 *     Arrivals after collecting stopped get staleError.
 *   startKRUMDeadlineTimer       krum.go:178-224   a timer thread: on timeout
 *     (no krumReceived) it runs the same sort + computeScores on whatever
 *     arrived (n < threshold) and releases len(UpdateList) waiters.
 *   computeScores / getTopKRUMIndex  krum.go:77-166  through the shim's calls:
 *     bk_check_args -> the UpdateList's row pointers -> bk_multikrum_rows
 *     (libbk packs them on its host threads; BK_HARNESS_SERIAL_PACK=1 replays
 *     the pre-r6 shim instead: bk_stage_alloc + a serial pack +
 *     bk_multikrum(BK_HOST_PINNED)) -> bk_selection_margin; any error (e.g.
 *     n = 1: clip = int(0.5 * 1) = 0, the reference's argpartition ValueError)
 *     gives an empty AcceptedList: every update rejected.
 *   checkIfAccepted              krum.go:47-73
 *
 *   verifier_harness <file> <rows> <d> <threshold> <timeout_ms> <a_1> [<a_2> ...]
 *
 * file: rows x d little-endian float64.  Iteration k has a_k peers arriving
 * concurrently (peer p sends row p with SourceID sid(p) = (p * 7919) % 10007).
 * Output, per iteration:
 *   iter <k> path=<threshold|deadline> n=<n> f=<f> status=<st> near_tie=<0|1>
 *        batch=<sid,...> accepted=<sid,...> k_small=<launches> k_gram=<launches>
 * (the launches of the one-launch path and of the general chain's K1 this
 * iteration, from libbk's per-kernel timing: Biscotti's batch shapes must take
 * k_small straight from the host entry)
 *   peer <k> <sid> <accepted|rejected|stale>
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <semaphore.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "bk.h"

enum { V_NONE = 0, V_ACCEPTED, V_REJECTED, V_STALE };

static bk_ctx *g_ctx;
static const double *g_data;
static int64_t g_d, g_thresh;
static void *g_stage;
static int64_t g_stage_len;
static int g_serial_pack; /* BK_HARNESS_SERIAL_PACK=1: the shim's pre-r6 pinned pack */

/* KRUMValidator state (krum.go:22-29) and the verifier globals it uses */
static pthread_mutex_t krum_lock = PTHREAD_MUTEX_INITIALIZER;
static int collecting;               /* collectingUpdates */
static int64_t *upd_row, *upd_sid;   /* UpdateList: row index and SourceID */
static int64_t n_upd;
static int64_t *accepted;            /* AcceptedList (indices into UpdateList) */
static int64_t n_acc;
static sem_t krum_accepted;          /* the krumAccepted channel's tokens */
static pthread_mutex_t recv_lock = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t recv_cond = PTHREAD_COND_INITIALIZER;
static int krum_received;            /* the krumReceived channel */
/* what happened this iteration (printed by main) */
static const char *path;
static int64_t last_f;
static int last_status, last_near;

static int64_t sid_of(int64_t p) { return (p * 7919) % 10007; }

/* getTopKRUMIndex (krum.go:100-166) via the shim's exact calls */
static void compute_scores(void)
{
    const int64_t n = n_upd, d = g_d;
    const int64_t f = (int64_t)(0.5 * (double)n); /* krum.go:110 */
    last_f = f;
    last_near = 0;
    n_acc = 0;
    last_status = bk_check_args(n, d, f);
    if (last_status != BK_OK) return; /* reject all, as a failing Python call did */
    int64_t m = 0;
    if (g_serial_pack) {
        /* the shim's pre-r6 form: pack the rows into a C-owned pinned batch */
        const int64_t need = n * d * (int64_t)sizeof(double);
        if (need > g_stage_len) {
            if (g_stage) bk_stage_free(g_ctx, g_stage);
            g_stage = NULL;
            g_stage_len = 0;
            last_status = bk_stage_alloc(g_ctx, need, &g_stage);
            if (last_status != BK_OK) return;
            g_stage_len = need;
        }
        double *stage = (double *)g_stage;
        for (int64_t i = 0; i < n; ++i)
            memcpy(stage + i * d, g_data + upd_row[i] * d, (size_t)d * sizeof(double));
        last_status = bk_multikrum(g_ctx, stage, BK_HOST_PINNED, BK_F64, n, d, d, f, accepted, &m,
                                   NULL, NULL);
    } else {
        /* the shim's form: the UpdateList's rows as they are (one pointer per
         * update, in SourceID order), packed by libbk (bk_multikrum_rows) */
        const void **rows = (const void **)malloc((size_t)n * sizeof(void *));
        if (!rows) {
            last_status = BK_ENOMEM;
            return;
        }
        for (int64_t i = 0; i < n; ++i) rows[i] = g_data + upd_row[i] * d;
        last_status = bk_multikrum_rows(g_ctx, rows, BK_F64, n, d, f, accepted, &m, NULL, NULL);
        free(rows);
    }
    if (last_status != BK_OK) return;
    double gap, bound;
    if (bk_selection_margin(g_ctx, &gap, &bound, &last_near) != BK_OK) last_near = -1;
    n_acc = m;
}

static void sort_by_sid(void)
{
    for (int64_t i = 1; i < n_upd; ++i) /* insertion sort: n is small, stable */
        for (int64_t j = i; j > 0 && upd_sid[j - 1] > upd_sid[j]; --j) {
            int64_t t = upd_sid[j];
            upd_sid[j] = upd_sid[j - 1];
            upd_sid[j - 1] = t;
            t = upd_row[j];
            upd_row[j] = upd_row[j - 1];
            upd_row[j - 1] = t;
        }
}

static int check_if_accepted(int64_t sid) /* krum.go:47-73 */
{
    for (int64_t i = 0; i < n_acc; ++i)
        if (upd_sid[accepted[i]] == sid) return 1;
    return 0;
}

struct peer {
    int64_t row, sid;
    int verdict;
    unsigned delay_us;
};

static void *verify_update(void *arg) /* Peer.VerifyUpdateKRUM */
{
    struct peer *p = (struct peer *)arg;
    if (p->delay_us) usleep(p->delay_us);
    pthread_mutex_lock(&krum_lock);
    if (!collecting) {
        pthread_mutex_unlock(&krum_lock);
        p->verdict = V_STALE;
        return NULL;
    }
    upd_row[n_upd] = p->row;
    upd_sid[n_upd] = p->sid;
    ++n_upd;
    if (n_upd == g_thresh) {
        pthread_mutex_lock(&recv_lock); /* krumReceived <- true */
        krum_received = 1;
        pthread_cond_signal(&recv_cond);
        pthread_mutex_unlock(&recv_lock);
        collecting = 0;
        sort_by_sid();
        compute_scores();
        path = "threshold";
        for (int64_t i = 0; i < g_thresh - 1; ++i) sem_post(&krum_accepted);
        pthread_mutex_unlock(&krum_lock);
    } else {
        pthread_mutex_unlock(&krum_lock);
        sem_wait(&krum_accepted); /* <- krumAccepted */
    }
    p->verdict = check_if_accepted(p->sid) ? V_ACCEPTED : V_REJECTED;
    return NULL;
}

static long g_timeout_ms;

static void *deadline_timer(void *arg) /* startKRUMDeadlineTimer */
{
    (void)arg;
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    ts.tv_sec += g_timeout_ms / 1000;
    ts.tv_nsec += (g_timeout_ms % 1000) * 1000000L;
    if (ts.tv_nsec >= 1000000000L) {
        ts.tv_sec += 1;
        ts.tv_nsec -= 1000000000L;
    }
    int rc = 0;
    pthread_mutex_lock(&recv_lock);
    while (!krum_received && rc != ETIMEDOUT) rc = pthread_cond_timedwait(&recv_cond, &recv_lock, &ts);
    const int got = krum_received;
    pthread_mutex_unlock(&recv_lock);
    if (got) return NULL; /* case <- krumReceived */
    pthread_mutex_lock(&krum_lock);
    if (collecting) { /* time.After(timeoutKRUM): Krum on whatever arrived */
        collecting = 0;
        sort_by_sid();
        compute_scores();
        path = "deadline";
        for (int64_t i = 0; i < n_upd; ++i) sem_post(&krum_accepted);
    }
    pthread_mutex_unlock(&krum_lock);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 7) {
        fprintf(stderr, "usage: %s <file> <rows> <d> <threshold> <timeout_ms> <a_1> [<a_2> ...]\n",
                argv[0]);
        return 2;
    }
    const int64_t rows = atoll(argv[2]);
    g_d = atoll(argv[3]);
    g_thresh = atoll(argv[4]);
    g_timeout_ms = atol(argv[5]);
    if (rows < 1 || g_d < 1 || g_thresh < 1 || g_timeout_ms < 1) {
        fprintf(stderr, "bad sizes\n");
        return 2;
    }
    double *data = (double *)malloc((size_t)(rows * g_d) * sizeof(double));
    FILE *fp = fopen(argv[1], "rb");
    if (!data || !fp || fread(data, sizeof(double), (size_t)(rows * g_d), fp) != (size_t)(rows * g_d)) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 1;
    }
    fclose(fp);
    g_data = data;
    {
        const char *e = getenv("BK_HARNESS_SERIAL_PACK");
        g_serial_pack = e && atoi(e) != 0;
    }
    if (bk_create(&g_ctx, 0) != BK_OK) { /* KRUMValidator.initialize (krum.go:31-44) */
        fprintf(stderr, "bk_create: %s\n", bk_last_error());
        return 1;
    }
    /* count which path each Multi-Krum took (HIP events around k_small / K1) */
    bk_timing_select(g_ctx, (1u << BK_K_SMALL) | (1u << BK_K_GRAM));
    int64_t prev_small = 0, prev_gram = 0;
    upd_row = (int64_t *)calloc((size_t)rows, sizeof(int64_t));
    upd_sid = (int64_t *)calloc((size_t)rows, sizeof(int64_t));
    accepted = (int64_t *)calloc((size_t)rows, sizeof(int64_t));
    struct peer *peers = (struct peer *)calloc((size_t)rows, sizeof(struct peer));
    pthread_t *th = (pthread_t *)calloc((size_t)rows, sizeof(pthread_t));
    int rc = 0;
    for (int it = 6; it < argc && rc == 0; ++it) {
        const int64_t a = atoll(argv[it]);
        if (a < 0 || a > rows) {
            fprintf(stderr, "bad arrivals %lld\n", (long long)a);
            rc = 2;
            break;
        }
        /* prepareForNextIteration: flush and collect again (krum.go:169-176) */
        n_upd = n_acc = 0;
        collecting = 1;
        krum_received = 0;
        path = "none";
        last_status = 0;
        last_f = 0;
        last_near = 0;
        sem_init(&krum_accepted, 0, 0);
        pthread_t timer;
        pthread_create(&timer, NULL, deadline_timer, NULL);
        unsigned seed = 1234u + (unsigned)it;
        for (int64_t p = 0; p < a; ++p) {
            peers[p].row = p;
            peers[p].sid = sid_of(p);
            peers[p].verdict = V_NONE;
            peers[p].delay_us = (unsigned)(rand_r(&seed) % 3000); /* arrival order varies */
            pthread_create(&th[p], NULL, verify_update, &peers[p]);
        }
        for (int64_t p = 0; p < a; ++p) pthread_join(th[p], NULL);
        pthread_join(timer, NULL);
        sem_destroy(&krum_accepted);
        printf("iter %d path=%s n=%lld f=%lld status=%d near_tie=%d batch=", it - 5, path,
               (long long)n_upd, (long long)last_f, last_status, last_near);
        for (int64_t i = 0; i < n_upd; ++i) printf(i ? ",%lld" : "%lld", (long long)upd_sid[i]);
        printf(" accepted=");
        for (int64_t i = 0; i < n_acc; ++i)
            printf(i ? ",%lld" : "%lld", (long long)upd_sid[accepted[i]]);
        int64_t ns = 0, ng = 0;
        double ms = 0.0;
        bk_timing_read(g_ctx, BK_K_SMALL, &ms, &ns);
        bk_timing_read(g_ctx, BK_K_GRAM, &ms, &ng);
        printf(" k_small=%lld k_gram=%lld\n", (long long)(ns - prev_small), (long long)(ng - prev_gram));
        prev_small = ns;
        prev_gram = ng;
        for (int64_t p = 0; p < a; ++p)
            printf("peer %d %lld %s\n", it - 5, (long long)peers[p].sid,
                   peers[p].verdict == V_ACCEPTED   ? "accepted"
                   : peers[p].verdict == V_REJECTED ? "rejected"
                                                    : "stale");
    }
    if (g_stage) bk_stage_free(g_ctx, g_stage);
    bk_destroy(g_ctx);
    free(th);
    free(peers);
    free(accepted);
    free(upd_sid);
    free(upd_row);
    free(data);
    return rc;
}
