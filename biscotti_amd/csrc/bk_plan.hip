// bk_plan.hip -- host planner for K1 v3 (see bk_internal.h and DESIGN.md "K1").
//
// Turns (n, d, #CUs) into: wave-tasks over the 64x64 upper sub-tiles of the
// Gram, groups of <= 8 tasks sharing <= 6 row-blocks (one 512-thread
// workgroup each), and per-XCD slices of the columns whose counts balance the
// groups' per-SIMD MFMA cost so that the workgroups of a launch finish
// together.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <queue>
#include <vector>

#include "bk_internal.h"

namespace bk {

namespace {

constexpr int COST_OFF = 16, COST_PAIR = 20, COST_DIAG1 = 10;
// measured on MI355X (tools/trace_gram.py): a k-block of a group costs about
// 256 * cost + 191 * nb shader cycles -- each staged row-block adds ~0.75 cost
// units of memory stall.  Apportioning by this (not by MFMA cost alone) keeps
// the column fronts of all groups on an XCD together, so the row-blocks they
// share are re-read from L2 instead of HBM.
double eff_cost(const GroupDesc &g) {
    const char *v = getenv("BK_PLAN_NB_COST");
    const double a = v ? atof(v) : 0.75;
    return g.cost + a * g.nb;
}

struct Task {
    int kind;
    int ba, bb;  // row-blocks (OFF: bi, bj; PAIR: b0, b1; DIAG1: b0, b0)
    int cost;
};

int upper_index(int T, int bi, int bj) { return bi * T - bi * (bi - 1) / 2 + (bj - bi); }

int task_cost(int kind) {
    return kind == T_OFF ? COST_OFF : kind == T_PAIR ? COST_PAIR : kind == T_DIAG1 ? COST_DIAG1 : 0;
}

// waves w and w+4 share a SIMD (waves are dealt to SIMDs cyclically)
int group_cost(const std::vector<Task> &w8) {
    int c = 0;
    for (int s = 0; s < 4; ++s) {
        const int a = s < (int)w8.size() ? w8[s].cost : 0;
        const int b = s + 4 < (int)w8.size() ? w8[s + 4].cost : 0;
        c = std::max(c, a + b);
    }
    return c;
}

GroupDesc make_group(int T, const std::vector<Task> &tasks) {
    GroupDesc G{};
    std::vector<int> blocks;
    auto slot = [&](int b) {
        for (size_t i = 0; i < blocks.size(); ++i)
            if (blocks[i] == b) return (int)i;
        blocks.push_back(b);
        return (int)blocks.size() - 1;
    };
    for (int w = 0; w < 8; ++w) {
        int *t = G.task[w];
        t[0] = T_NONE;
        t[1] = t[2] = 0;
        t[3] = t[4] = -1;
        if (w >= (int)tasks.size() || tasks[w].kind == T_NONE) continue;
        const Task &k = tasks[w];
        t[0] = k.kind;
        t[1] = slot(k.ba);
        t[2] = slot(k.bb);
        if (k.kind == T_OFF) {
            t[3] = upper_index(T, k.ba, k.bb);
        } else if (k.kind == T_PAIR) {
            t[3] = upper_index(T, k.ba, k.ba);
            t[4] = upper_index(T, k.bb, k.bb);
        } else {
            t[3] = upper_index(T, k.ba, k.ba);
        }
    }
    if (blocks.empty()) blocks.push_back(0);
    G.nb = (int)blocks.size();
    for (int i = 0; i < G3_MAXB; ++i) G.blk[i] = i < G.nb ? blocks[i] : blocks[0];
    G.cost = group_cost(tasks);
    return G;
}

}  // namespace

Plan3Host build_plan3(int n, int64_t d, int num_cu, int bk) {
    Plan3Host H;
    const int T = (n + 63) / 64;
    const int TT = (T + 1) / 2;  // 128-row super-blocks
    H.T = T;
    H.ntile = T * (T + 1) / 2;
    H.nfull = (int)(d / bk);

    std::vector<std::vector<Task>> groups;  // each: 8 wave slots (waves w, w+4 pair on a SIMD)
    const Task none{T_NONE, 0, 0, 0};
    auto diag_task = [&](int I) {  // the diagonal sub-tiles of super-block I
        const int b0 = 2 * I, b1 = b0 + 1;
        return b1 < T ? Task{T_PAIR, b0, b1, COST_PAIR} : Task{T_DIAG1, b0, b0, COST_DIAG1};
    };
    auto near_task = [&](int I) {  // the off-diagonal sub-tile inside super-block I
        const int b0 = 2 * I, b1 = b0 + 1;
        return b1 < T ? Task{T_OFF, b0, b1, COST_OFF} : none;
    };
    auto super_tasks = [&](int I, int J) {  // the <= 4 OFF sub-tiles of super-tile (I < J)
        std::vector<Task> st;
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) {
                const int bi = 2 * I + a, bj = 2 * J + b;
                if (bi < T && bj < T) st.push_back(Task{T_OFF, bi, bj, COST_OFF});
            }
        return st;
    };
    // (1) the diagonal band in "quads" of two super-blocks (4 row-blocks):
    //     waves 0,1: PAIR tasks, 4,5: the near-diagonal OFF tasks (20 + 16 per
    //     SIMD), 2,3,6,7: the off-diagonal super-tile (I, I+1) between them
    std::vector<char> used((size_t)TT * TT, 0);
    for (int I = 0; I + 1 < TT; I += 2) {
        std::vector<Task> w(8, none);
        w[0] = diag_task(I);
        w[1] = diag_task(I + 1);
        w[4] = near_task(I);
        w[5] = near_task(I + 1);
        const std::vector<Task> st = super_tasks(I, I + 1);
        const int slots[4] = {2, 3, 6, 7};
        for (size_t k = 0; k < st.size(); ++k) w[slots[k]] = st[k];
        used[(size_t)I * TT + I + 1] = 1;
        groups.push_back(w);
    }
    if (TT & 1) {  // a last lone super-block
        std::vector<Task> w(8, none);
        w[0] = diag_task(TT - 1);
        w[4] = near_task(TT - 1);
        groups.push_back(w);
    }
    // (2) the other off-diagonal super-tiles, two per group along a super-row
    //     (6 row-blocks); leftovers paired when they share a super-block
    std::vector<std::pair<int, int>> singles;
    for (int I = 0; I < TT; ++I) {
        std::vector<int> row;
        for (int J = I + 1; J < TT; ++J)
            if (!used[(size_t)I * TT + J]) row.push_back(J);
        for (size_t k = 0; k + 1 < row.size(); k += 2) {
            std::vector<Task> w = super_tasks(I, row[k]);
            w.resize(4, none);
            for (const Task &t : super_tasks(I, row[k + 1])) w.push_back(t);
            w.resize(8, none);
            groups.push_back(w);
        }
        if (row.size() & 1) singles.push_back({I, row.back()});
    }
    std::vector<char> taken(singles.size(), 0);
    for (size_t a = 0; a < singles.size(); ++a) {
        if (taken[a]) continue;
        taken[a] = 1;
        std::vector<Task> w = super_tasks(singles[a].first, singles[a].second);
        w.resize(4, none);
        for (size_t b = a + 1; b < singles.size(); ++b) {
            if (taken[b]) continue;
            const auto &x = singles[a], &y = singles[b];
            if (x.first == y.first || x.first == y.second || x.second == y.first ||
                x.second == y.second) {
                taken[b] = 1;
                for (const Task &t : super_tasks(y.first, y.second)) w.push_back(t);
                break;
            }
        }
        w.resize(8, none);
        groups.push_back(w);
    }

    std::vector<GroupDesc> G;
    for (auto &w : groups) G.push_back(make_group(T, w));
    const int ng = (int)G.size();

    // (3) XCD-aware pieces.  Workgroups b and b+8 share an XCD (dispatch is
    //     round-robin; speed only, never correctness).  XCD x owns k-blocks
    //     [K_x, K_x+1), cut into R consecutive sub-ranges, one per dispatch
    //     round.  In round r group g runs Q_g workgroups, workgroup q taking
    //     k-blocks K_xr + q, + Q_g, ... < K_x(r+1), so within a round every
    //     group on an XCD sweeps the same sub-range with its column front
    //     level with the others', and the row-blocks the groups share are
    //     re-read from the XCD's L2 instead of HBM.  (Strided over the whole
    //     XCD range instead, a k-block would be read by one group in round 1
    //     and by another in round 2: v7 fetched 2x the unique bytes.)
    //     BK_PLAN_ALIGN=0 restores that v7 interleave for A/B runs.
    const int nfull = H.nfull;
    constexpr int NX = 8;
    const int per_xcd = std::max(1, num_cu / NX);
    std::vector<int64_t> K(NX + 1);
    for (int x = 0; x <= NX; ++x) K[x] = (int64_t)nfull * x / NX;
    // prologue (ring fill at loaded latency) + partial-slab write + reduce share,
    // in cost units (256 shader cycles): ~10 us per workgroup
    const char *ev = getenv("BK_PLAN_WGOH");
    const double wg_overhead = ev ? atof(ev) : 100.0;
    const char *er = getenv("BK_PLAN_ROUNDS");
    const int force_rounds = er ? atoi(er) : 0;
    const char *ea = getenv("BK_PLAN_ALIGN");
    const bool aligned = ea ? atoi(ea) != 0 : true;
    double best = 1e300;
    int bestR = 1;
    std::vector<int> bestQ(ng, 1);
    for (int rounds = 1; rounds <= 16; rounds *= 2) {
        if (force_rounds && rounds != force_rounds) continue;
        // aligned: Q_g workgroups per round on the XCD's slots; v7: Q_g over
        // all rounds' slots at once
        const double slots_total = aligned ? (double)std::max(per_xcd, ng)
                                           : (double)rounds * per_xcd;
        if (!aligned && ng > slots_total * 4) continue;
        // min-max apportionment of the slots (Q_g >= 1): repeatedly give a slot
        // to the group with the largest eff_g / Q_g.  Equal eff_g / Q_g both
        // balances the workgroups and makes every group's column front advance
        // at the same speed (shared row-blocks stay in L2).
        std::vector<int> Q(ng, 1);
        {
            std::priority_queue<std::pair<double, int>> pq;
            for (int g = 0; g < ng; ++g) pq.push({eff_cost(G[g]), g});
            for (int used = ng; used < (int)slots_total; ++used) {
                const int g = pq.top().second;
                pq.pop();
                Q[g]++;
                pq.push({eff_cost(G[g]) / Q[g], g});
            }
        }
        // list-schedule one XCD's workgroups in dispatch order on per_xcd slots
        std::vector<double> jobs;
        const int nr = aligned ? rounds : 1;
        for (int r = 0; r < nr; ++r) {
            const int64_t R = aligned ? (K[1] - K[0]) * (r + 1) / rounds - (K[1] - K[0]) * r / rounds
                                      : K[1] - K[0];
            for (int g = 0; g < ng; ++g)
                for (int q = 0; q < Q[g]; ++q) {
                    const int64_t nk = q < R ? (R - 1 - q) / Q[g] + 1 : 0;
                    jobs.push_back((double)nk * eff_cost(G[g]) + wg_overhead);
                }
        }
        std::priority_queue<double, std::vector<double>, std::greater<double>> slots;
        for (int i = 0; i < per_xcd; ++i) slots.push(0.0);
        double mk = 0;
        for (double j : jobs) {
            const double t1 = slots.top() + j;
            slots.pop();
            slots.push(t1);
            mk = std::max(mk, t1);
        }
        // + the split-K reduce (K1b) reading every workgroup's partial slabs
        // after K1, in cost units: bytes / ~4 TB/s / (256 cycles at ~2.25 GHz)
        double slab_bytes = 0;
        for (int g = 0; g < ng; ++g) {
            double b = 0;
            for (int w = 0; w < 8; ++w)
                b += G[g].task[w][0] == T_PAIR ? 65536.0 : G[g].task[w][0] != T_NONE ? 32768.0 : 0.0;
            slab_bytes += b * Q[g] * nr * NX;
        }
        mk += slab_bytes / 4e12 / (256.0 / 2.25e9);
        if (mk < best * 0.995) {
            best = mk;
            bestQ = Q;
            bestR = nr;
        }
    }
    // per-XCD launch lists (round-major, then q, then group); b = 8 j + x
    std::vector<std::vector<std::array<int, 5>>> lists(NX);
    int maxq = 0;
    for (int g = 0; g < ng; ++g) maxq = std::max(maxq, bestQ[g]);
    for (int x = 0; x < NX; ++x)
        for (int r = 0; r < bestR; ++r) {
            const int64_t span = K[x + 1] - K[x];
            const int k0 = (int)(K[x] + span * r / bestR), k1 = (int)(K[x] + span * (r + 1) / bestR);
            for (int q = 0; q < maxq; ++q)
                for (int g = 0; g < ng; ++g)
                    if (q < bestQ[g])
                        lists[x].push_back({g, k0 + q, bestQ[g], k1,
                                            (x == 0 && r == 0 && q == 0) ? 1 : 0});
        }
    size_t maxlen = 0;
    for (auto &l : lists) maxlen = std::max(maxlen, l.size());
    std::vector<std::vector<int>> gw(ng);
    for (size_t j = 0; j < maxlen; ++j)
        for (int x = 0; x < NX; ++x) {
            const int b = (int)(H.wg.size() / 5);
            if (j < lists[x].size()) {
                const auto &e = lists[x][j];
                H.wg.insert(H.wg.end(), e.begin(), e.end());
                gw[e[0]].push_back(b);
            } else {
                // keep b = 8j + x: an empty workgroup (no k-blocks) of group 0
                H.wg.insert(H.wg.end(), {0, 0, 1, 0, 0});
                gw[0].push_back(b);
            }
        }
    for (int g = 0; g < ng; ++g) {
        G[g].Q = bestQ[g] * bestR;
        G[g].wg0 = (int)H.wglist.size();
        H.wglist.insert(H.wglist.end(), gw[g].begin(), gw[g].end());
    }
    // every (group, k-block) exactly once, and exactly one tail workgroup per group
    bool covered = true;
    {
        std::vector<int> seen((size_t)ng * nfull, 0), tails(ng, 0);
        for (size_t b = 0; b < H.wg.size() / 5; ++b) {
            const int *e = &H.wg[5 * b];
            for (int64_t k = e[1]; k < e[3]; k += e[2]) seen[(size_t)e[0] * nfull + k]++;
            tails[e[0]] += e[4];
        }
        for (int v : seen) covered = covered && v == 1;
        for (int v : tails) covered = covered && v == 1;
    }
    // (4) reduce table: sub-tile u -> its group's workgroups, slot wave * 2 + t
    H.red.assign((size_t)H.ntile * 3, 0);
    std::vector<int> seen(H.ntile, 0);
    for (int g = 0; g < ng; ++g)
        for (int w = 0; w < 8; ++w)
            for (int t = 0; t < 2; ++t) {
                const int u = G[g].task[w][3 + t];
                if (u < 0) continue;
                H.red[3 * u] = G[g].wg0;
                H.red[3 * u + 1] = (int)gw[g].size();
                H.red[3 * u + 2] = w * 2 + t;
                seen[u]++;
            }
    bool ok = true;
    for (auto &g : G) ok = ok && g.nb <= G3_MAXB;
    ok = ok && covered;
    for (int u = 0; u < H.ntile; ++u)
        if (seen[u] != 1 || !ok) H.red[3 * u + 1] = -1;  // planner bug marker (checked by the caller)
    H.groups = G;
    return H;
}

}  // namespace bk
