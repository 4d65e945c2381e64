// bk_plan.hip -- host planner for K1 v3 (see bk_internal.h and DESIGN.md "K1").
//
// Turns (n, d, #CUs) into: wave-tasks over the 64x64 upper sub-tiles of the
// Gram, groups of <= 8 tasks sharing <= 8 row-blocks (one 512-thread
// workgroup each), and a per-group piece count P that balances the groups'
// per-SIMD MFMA cost so that every workgroup of a launch finishes together.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <functional>
#include <queue>
#include <vector>

#include "bk_internal.h"

namespace bk {

namespace {

constexpr int COST_OFF = 16, COST_PAIR = 20, COST_DIAG1 = 10;

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
    if (blocks.size() & 1) blocks.push_back(blocks[0]);  // glds issue needs an even count
    G.nb = (int)blocks.size();
    for (int i = 0; i < G3_MAXB; ++i) G.blk[i] = i < G.nb ? blocks[i] : blocks[0];
    G.cost = group_cost(tasks);
    return G;
}

}  // namespace

Plan3Host build_plan3(int n, int64_t d, int num_cu) {
    Plan3Host H;
    const int T = (n + 63) / 64;
    const int TT = (T + 1) / 2;
    H.T = T;
    H.ntile = T * (T + 1) / 2;
    H.nfull = (int)(d / G3_BK);

    std::vector<std::vector<Task>> groups;  // each: 8 wave slots (waves w, w+4 pair on a SIMD)

    // (1) the diagonal band, 4 super-blocks per group: PAIR tasks on waves 0-3,
    //     the near-diagonal OFF sub-tile (2I, 2I+1) on waves 4-7 -> 20 + 16 per SIMD
    for (int I0 = 0; I0 < TT; I0 += 4) {
        std::vector<Task> w(8, Task{T_NONE, 0, 0, 0});
        for (int k = 0; k < 4 && I0 + k < TT; ++k) {
            const int b0 = 2 * (I0 + k), b1 = b0 + 1;
            if (b1 < T) {
                w[k] = Task{T_PAIR, b0, b1, COST_PAIR};
                w[k + 4] = Task{T_OFF, b0, b1, COST_OFF};
            } else {
                w[k] = Task{T_DIAG1, b0, b0, COST_DIAG1};
            }
        }
        groups.push_back(w);
    }
    // (2) off-diagonal super-tiles (I < J): 4 OFF tasks each; two super-tiles of
    //     the same super-row per group (6 row-blocks), leftovers paired (<= 8)
    std::vector<std::vector<Task>> singles;
    for (int I = 0; I < TT; ++I) {
        std::vector<std::vector<Task>> row;
        for (int J = I + 1; J < TT; ++J) {
            std::vector<Task> st;
            for (int a = 0; a < 2; ++a)
                for (int b = 0; b < 2; ++b) {
                    const int bi = 2 * I + a, bj = 2 * J + b;
                    if (bi < T && bj < T) st.push_back(Task{T_OFF, bi, bj, COST_OFF});
                }
            row.push_back(st);
        }
        for (size_t k = 0; k + 1 < row.size(); k += 2) {
            std::vector<Task> w = row[k];
            w.resize(4, Task{T_NONE, 0, 0, 0});
            for (const Task &t : row[k + 1]) w.push_back(t);
            w.resize(8, Task{T_NONE, 0, 0, 0});
            groups.push_back(w);
        }
        if (row.size() & 1) singles.push_back(row.back());
    }
    for (size_t k = 0; k < singles.size(); k += 2) {
        std::vector<Task> w = singles[k];
        w.resize(4, Task{T_NONE, 0, 0, 0});
        if (k + 1 < singles.size())
            for (const Task &t : singles[k + 1]) w.push_back(t);
        w.resize(8, Task{T_NONE, 0, 0, 0});
        groups.push_back(w);
    }

    std::vector<GroupDesc> G;
    for (auto &w : groups) G.push_back(make_group(T, w));
    const int ng = (int)G.size();

    // (3) pieces: P_g ~ cost_g so per-WG time ~ (k-blocks / P_g) * cost_g is even;
    //     pick the total that minimises the simulated makespan on num_cu slots
    const int nfull = H.nfull;
    double csum = 0;
    for (auto &g : G) csum += g.cost;
    const double wg_overhead = 64.0 * 16.0;  // prologue + slab write, in cost*k-block units
    double best = 1e300;
    std::vector<int> bestP(ng, 1);
    for (int mult : {1, 2, 3, 4, 6, 8, 12, 16}) {
        const double target = (double)mult * num_cu;
        std::vector<int> P(ng);
        for (int g = 0; g < ng; ++g) {
            int p = (int)(target * G[g].cost / csum + 0.5);
            p = std::max(1, std::min(p, std::max(1, nfull)));
            P[g] = p;
        }
        // list-schedule in launch order on num_cu slots (1 workgroup per CU)
        std::priority_queue<double, std::vector<double>, std::greater<double>> slots;
        for (int i = 0; i < num_cu; ++i) slots.push(0.0);
        double mk = 0;
        for (int g = 0; g < ng; ++g)
            for (int p = 0; p < P[g]; ++p) {
                const int nk = p < nfull ? (nfull - 1 - p) / P[g] + 1 : 0;
                const double t0 = slots.top();
                slots.pop();
                const double t1 = t0 + (double)nk * G[g].cost + wg_overhead;
                mk = std::max(mk, t1);
                slots.push(t1);
            }
        if (mk < best * 0.995) {
            best = mk;
            bestP = P;
        }
    }
    int wg = 0;
    for (int g = 0; g < ng; ++g) {
        G[g].P = bestP[g];
        G[g].wg0 = wg;
        for (int p = 0; p < bestP[g]; ++p) {
            H.wg.push_back(g);
            H.wg.push_back(p);
        }
        wg += bestP[g];
    }
    // (4) reduce table: sub-tile u -> its slabs (wg0 + p) * 16 + wave * 2 + t
    H.red.assign((size_t)H.ntile * 3, 0);
    std::vector<int> seen(H.ntile, 0);
    for (int g = 0; g < ng; ++g)
        for (int w = 0; w < 8; ++w)
            for (int t = 0; t < 2; ++t) {
                const int u = G[g].task[w][3 + t];
                if (u < 0) continue;
                H.red[3 * u] = G[g].wg0 * 16 + w * 2 + t;
                H.red[3 * u + 1] = G[g].P;
                H.red[3 * u + 2] = 16;
                seen[u]++;
            }
    for (int u = 0; u < H.ntile; ++u)
        if (seen[u] != 1) H.red[3 * u + 1] = -1;  // planner bug marker (checked by the caller)
    H.groups = G;
    return H;
}

}  // namespace bk
