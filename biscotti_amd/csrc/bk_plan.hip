// bk_plan.hip -- host planner for K1 v3 (see bk_internal.h and DESIGN.md "K1").
//
// Turns (n, d, #CUs) into: wave-tasks over the 64x64 upper sub-tiles of the
// Gram, groups of <= 8 tasks sharing <= 6 row-blocks (one 512-thread
// workgroup each), and per-XCD slices of the columns whose counts balance the
// groups' per-SIMD MFMA cost so that the workgroups of a launch finish
// together.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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
// Per-k-block time of a group in cost units (256 shader cycles), fitted to the
// K1 timeline (tools/trace_gram.py, v8 at n = 512, d = 2^20 and 2^17): band
// quads (cost 36, 4 staged row-blocks) 9730 cycles, super-tile pairs (32, 6)
// 8880 -> 1.015 * cost + 0.37 * nb.  Only the ratios between groups matter:
// they set how the planner splits an XCD's columns between groups so that all
// its CUs finish together.
double eff_cost(const GroupDesc &g) {
    const char *v = probe_env("BK_PLAN_NB_COST");
    const double b = v ? atof(v) : 0.37;
    return 1.015 * g.cost + b * g.nb;
}

struct Task {
    int kind;
    int ba, bb;  // row-blocks (OFF: bi, bj; PAIR: b0, b1; DIAG1: b0, b0)
    int cost;
    int xt = 0, xslot = -1;  // balanced band quads (GroupDesc::xt)
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
        G.xt[w] = w < (int)tasks.size() ? tasks[w].xt : 0;
        G.xslot[w] = w < (int)tasks.size() ? tasks[w].xslot : -1;
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

// McNaughton's wrap-around rule, one XCD, one dispatch round: the groups'
// work over a column range of len k-blocks (e[g] per k-block) laid end to end
// and cut into P equal slot loads; a cut inside a group splits it into two
// contiguous k-block pieces.  Each slot becomes ONE launched workgroup that
// runs its pieces as consecutive segments, so the balance does not depend on
// which CU the dispatcher picks.
struct Piece {
    int g;
    int64_t a, b;  // k-blocks [a, b) relative to the range start
};
std::vector<std::vector<Piece>> mcnaughton(const std::vector<double> &e, int64_t len, int P) {
    std::vector<std::vector<Piece>> slot(P);
    if (len <= 0) return slot;
    const int ng = (int)e.size();
    // the work line: group g occupies [W[g], W[g+1]); cut c sits at c * L.
    // Each cut is rounded to a k-block boundary on its own (no accumulated
    // rounding: every slot is within one k-block of L).
    std::vector<double> W(ng + 1, 0.0);
    for (int g = 0; g < ng; ++g) W[g + 1] = W[g] + e[g] * (double)len;
    const double L = W[ng] / P;
    // cut positions as (group, k-block) pairs, in order
    std::vector<std::pair<int, int64_t>> cuts;
    cuts.push_back({0, 0});
    for (int c = 1; c < P; ++c) {
        const double pos = c * L;
        int g = 0;
        while (g < ng - 1 && W[g + 1] <= pos) ++g;
        int64_t k = (int64_t)((pos - W[g]) / e[g] + 0.5);
        k = std::max<int64_t>(0, std::min(len, k));
        std::pair<int, int64_t> cp{g, k};
        if (k == len && g < ng - 1) cp = {g + 1, 0};  // a cut at a group's end
        if (cp < cuts.back()) cp = cuts.back();
        cuts.push_back(cp);
    }
    cuts.push_back({ng - 1, len});
    for (int q = 0; q < P; ++q) {
        auto [g0, k0] = cuts[q];
        const auto [g1, k1] = cuts[q + 1];
        while (g0 < g1 || (g0 == g1 && k0 < k1)) {
            const int64_t end = g0 < g1 ? len : k1;
            if (end > k0) slot[q].push_back({g0, k0, end});
            if (g0 == g1) break;
            ++g0;
            k0 = 0;
        }
    }
    std::vector<std::vector<Piece>> out;
    for (auto &v : slot)
        if (!v.empty()) out.push_back(v);
    return out;
}

}  // namespace

Plan3Host build_plan3(int n, int64_t d, int num_cu, int bk, int mode_in, int rounds_in) {
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
        // Balance: the quad's 136 MFMA units sit 20 + 16 on SIMDs 0-1 and
        // 16 + 16 on SIMDs 2-3.  Block (0,3) of each of the four diagonal tiles
        // (1 unit) moves to the super-tile wave that already holds that
        // row-block's fragments: PAIR 20 -> 18, super waves 16 -> 17, every
        // SIMD 34.  Wave 2 = (2I, 2I+2) takes tile 2I from its A side (PAIR
        // wave 0, slab 0), 7 = (2I+1, 2I+3) tile 2I+1 (A, wave 0 slab 1),
        // 6 = (2I+1, 2I+2) tile 2I+2 (B, wave 1 slab 0), 3 = (2I, 2I+3) tile
        // 2I+3 (B, wave 1 slab 1).  Same MFMAs in the same order: bitwise equal.
        const char *eb = probe_env("BK_QUAD_BAL");
        const bool full = w[0].kind == T_PAIR && w[1].kind == T_PAIR && st.size() == 4;
        if (full && !(eb && atoi(eb) == 0)) {
            w[0].xt = w[1].xt = 1;
            w[0].cost = w[1].cost = COST_PAIR - 2;
            const int xs[4][3] = {{2, 1, 0}, {7, 1, 1}, {6, 2, 2}, {3, 2, 3}};  // wave, side, slab
            for (const auto &x : xs) {
                w[x[0]].xt = x[1];
                w[x[0]].xslot = x[2];
                w[x[0]].cost = COST_OFF + 1;
            }
        }
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
    //     round.  BK_PLAN_MODE picks how a round's sub-range is split:
    //   2 (default for ng <= per_xcd): McNaughton -- the groups' work (eff_cost per k-block)
    //     laid end to end and cut into per_xcd equal slot loads, each group a
    //     few contiguous k-block pieces, so every CU of the XCD finishes the
    //     round together whatever the groups' cost ratios (v8 gave each group
    //     the same workgroup count, and the cheaper super-tile groups idled
    //     ~8% of the kernel: fill 0.946);
    //   1 (default otherwise): v8 -- group g runs Q_g workgroups, workgroup q taking k-blocks
    //     x_r + q, + Q_g, ... (all groups' column fronts level, for L2 reuse,
    //     worth < 1%: DESIGN.md);
    //   0: v7 -- Q_g strided over the whole XCD range.
    const int nfull = H.nfull;
    constexpr int NX = 8;
    const int per_xcd = std::max(1, num_cu / NX);
    std::vector<int64_t> K(NX + 1);
    for (int x = 0; x <= NX; ++x) K[x] = (int64_t)nfull * x / NX;
    // prologue (ring fill at loaded latency) + partial-slab write + reduce share,
    // in cost units (256 shader cycles): ~10 us per workgroup
    const char *ev = probe_env("BK_PLAN_WGOH");
    const double wg_overhead = ev ? atof(ev) : 100.0;
    const char *er = probe_env("BK_PLAN_ROUNDS");
    const int force_rounds = rounds_in > 0 ? rounds_in : er ? atoi(er) : 0;
    // McNaughton where an XCD has at least as many CUs as groups (n <= 1024:
    // D -2.2%, its 8-GPU shard -2.0%, C -0.5% against v8); with more groups
    // (n = 4096: 256) each slot would run ~8 whole groups back to back, and
    // v8's one workgroup per group, handed to CUs as they free up, absorbs the
    // CUs' speed spread better (+3.3% for McNaughton there)
    int mode = ng <= per_xcd ? 2 : 1;
    if (const char *em = probe_env("BK_PLAN_MODE")) mode = atoi(em);
    if (mode_in >= 0) mode = mode_in;  // bk_plan_mode (the planner's coverage test)
    std::vector<double> eg(ng);
    for (int g = 0; g < ng; ++g) eg[g] = eff_cost(G[g]);
    auto slab_of = [&](int g) {
        double b = 0;
        for (int w = 0; w < 8; ++w)
            b += G[g].task[w][0] == T_PAIR ? 65536.0 : G[g].task[w][0] != T_NONE ? 32768.0 : 0.0;
        return b;
    };
    // one XCD's launch list for R rounds: launched workgroups, each a list of
    // segments {group, kstart, kstride, kend, tail}
    typedef std::array<int, 5> Seg;
    typedef std::vector<std::vector<std::vector<Seg>>> Lists;
    auto build_lists = [&](int rounds, Lists &lists) {
        lists.assign(NX, {});
        if (mode == 3 && per_xcd % ng == 0) {
            // aligned pieces: every group gets per_xcd / ng CUs of the XCD and
            // the same k-block pieces, so the q-th CUs of all groups stream the
            // same columns together and the row-blocks the groups share are
            // read from HBM once and then from L2 (at the price of the groups'
            // cost ratio in fill)
            const int pg = per_xcd / ng;
            for (int x = 0; x < NX; ++x)
                for (int r = 0; r < rounds; ++r) {
                    const int64_t span = K[x + 1] - K[x];
                    const int64_t k0 = K[x] + span * r / rounds, k1 = K[x] + span * (r + 1) / rounds;
                    for (int q = 0; q < pg; ++q)
                        for (int g = 0; g < ng; ++g)
                            lists[x].push_back({Seg{g, (int)(k0 + (k1 - k0) * q / pg), 1,
                                                    (int)(k0 + (k1 - k0) * (q + 1) / pg), 0}});
                }
            return std::vector<int>(ng, 0);
        }
        if (mode == 2 || mode == 3) {
            for (int x = 0; x < NX; ++x)
                for (int r = 0; r < rounds; ++r) {
                    const int64_t span = K[x + 1] - K[x];
                    const int64_t k0 = K[x] + span * r / rounds, k1 = K[x] + span * (r + 1) / rounds;
                    for (const auto &slot : mcnaughton(eg, k1 - k0, per_xcd)) {
                        std::vector<Seg> wg;
                        for (const Piece &pc : slot)
                            wg.push_back({pc.g, (int)(k0 + pc.a), 1, (int)(k0 + pc.b), 0});
                        lists[x].push_back(wg);
                    }
                }
            return std::vector<int>(ng, 0);
        }
        // modes 0 / 1: min-max apportionment of slots (Q_g >= 1): repeatedly
        // give a slot to the group with the largest eff_g / Q_g
        const double slots_total = mode == 1 ? (double)std::max(per_xcd, ng) : (double)rounds * per_xcd;
        std::vector<int> Q(ng, 1);
        std::priority_queue<std::pair<double, int>> pq;
        for (int g = 0; g < ng; ++g) pq.push({eg[g], g});
        for (int used = ng; used < (int)slots_total; ++used) {
            const int g = pq.top().second;
            pq.pop();
            Q[g]++;
            pq.push({eg[g] / Q[g], g});
        }
        int maxq = 0;
        for (int g = 0; g < ng; ++g) maxq = std::max(maxq, Q[g]);
        const int nr = mode == 1 ? rounds : 1;
        for (int x = 0; x < NX; ++x)
            for (int r = 0; r < nr; ++r) {
                const int64_t span = K[x + 1] - K[x];
                const int k0 = (int)(K[x] + span * r / nr), k1 = (int)(K[x] + span * (r + 1) / nr);
                for (int q = 0; q < maxq; ++q)
                    for (int g = 0; g < ng; ++g)
                        if (q < Q[g]) lists[x].push_back({Seg{g, k0 + q, Q[g], k1, 0}});
            }
        return Q;
    };
    auto model = [&](const std::vector<std::vector<Seg>> &l0) {
        // list-schedule XCD 0's workgroups in dispatch order on per_xcd slots,
        // + the split-K reduce (K1b) reading every segment's partial slabs
        // after K1: bytes / ~4 TB/s / (256 cycles at ~2.25 GHz)
        std::priority_queue<double, std::vector<double>, std::greater<double>> slots;
        for (int i = 0; i < per_xcd; ++i) slots.push(0.0);
        double mk = 0, slab_bytes = 0;
        for (const auto &wg : l0) {
            double t = 0;
            for (const Seg &e : wg) {
                const int64_t nk = e[1] < e[3] ? (e[3] - 1 - e[1]) / e[2] + 1 : 0;
                t += (double)nk * eg[e[0]] + wg_overhead;
                slab_bytes += slab_of(e[0]) * NX;
            }
            const double t1 = slots.top() + t;
            slots.pop();
            slots.push(t1);
            mk = std::max(mk, t1);
        }
        return mk + slab_bytes / 4e12 / (256.0 / 2.25e9);
    };
    double best = 1e300;
    int bestR = 1;
    for (int rounds = 1; rounds <= 16; rounds *= 2) {
        if (force_rounds && rounds != force_rounds) continue;
        if (mode == 0 && ng > rounds * per_xcd * 4) continue;
        Lists l;
        build_lists(rounds, l);
        const double mk = model(l[0]);
        if (mk < best * 0.995) {
            best = mk;
            bestR = rounds;
        }
    }
    Lists lists;
    const std::vector<int> bestQ = build_lists(bestR, lists);
    // exactly one ragged-tail segment per group (XCD 0's first of the group)
    {
        std::vector<char> has(ng, 0);
        for (auto &wg : lists[0])
            for (auto &e : wg)
                if (!has[e[0]]) {
                    has[e[0]] = 1;
                    e[4] = 1;
                }
        for (int g = 0; g < ng; ++g)
            if (!has[g]) lists[0].push_back({Seg{g, 0, 1, 0, 1}});  // no columns on XCD 0
    }
    // launched workgroup b = 8 j + x runs XCD x's j-th list entry; segments
    // are numbered in launch order (their slabs in part[])
    size_t maxlen = 0;
    for (auto &l : lists) maxlen = std::max(maxlen, l.size());
    std::vector<std::vector<int>> gw(ng);
    for (size_t j = 0; j < maxlen; ++j)
        for (int x = 0; x < NX; ++x) {
            const int v0 = (int)(H.wg.size() / 5);
            int cnt = 0;
            if (j < lists[x].size())
                for (const Seg &e : lists[x][j]) {
                    gw[e[0]].push_back((int)(H.wg.size() / 5));
                    H.wg.insert(H.wg.end(), e.begin(), e.end());
                    ++cnt;
                }
            H.seg.push_back(v0);
            H.seg.push_back(cnt);  // 0: an idle workgroup keeps b = 8 j + x
        }
    for (int g = 0; g < ng; ++g) {
        G[g].Q = mode >= 2 ? 0 : bestQ[g] * (mode == 1 ? bestR : 1);
        G[g].wg0 = (int)H.wglist.size();
        H.wglist.insert(H.wglist.end(), gw[g].begin(), gw[g].end());
    }
    // every (group, k-block) exactly once, and exactly one tail segment per group
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

std::vector<int> piece_cuts(const std::vector<double> &w, const std::vector<char> &valid, int k) {
    // target cumulative fractions: piece p's share of the work proportional
    // to 0.6^p, so each piece is ~0.6 of the one before (its compute hides
    // most of the previous piece's exchange) and the last one is small
    std::vector<int> cuts;
    const int B = (int)w.size();
    if (k < 2 || B < 2) return cuts;
    double tot = 0, wsum = 0, g = 1;
    for (int p = 0; p < k; ++p, g *= 0.6) wsum += g;
    for (double x : w) tot += x;
    std::vector<double> cum((size_t)B + 1, 0.0);
    for (int b = 0; b < B; ++b) cum[(size_t)b + 1] = cum[(size_t)b] + w[(size_t)b];
    double acc = 0;
    g = 1;
    int prev = 0;
    for (int p = 0; p + 1 < k; ++p, g *= 0.6) {
        acc += g / wsum;
        // the valid cut (strictly after the previous one, leaving room for
        // the pieces still to come) nearest the target
        int best = -1;
        for (int b = prev + 1; b <= B - (k - 1 - p); ++b)
            if (valid[(size_t)b] && (best < 0 || std::fabs(cum[(size_t)b] / tot - acc) <
                                                     std::fabs(cum[(size_t)best] / tot - acc)))
                best = b;
        if (best < 0) return std::vector<int>();
        cuts.push_back(best);
        prev = best;
    }
    return cuts;
}

bool plan3_pieces(const Plan3Host &H, int k, std::vector<int> &tile_end,
                  std::vector<std::vector<int>> &seg) {
    const int T = H.T, ng = (int)H.groups.size();
    // each group's row-block span: the rows of its sub-tiles (OFF tasks (ba <
    // bb): row ba; PAIR: rows ba and bb; DIAG1: ba)
    std::vector<int> lo(ng, T), hi(ng, -1);
    std::vector<double> w((size_t)T, 0.0);
    for (int g = 0; g < ng; ++g) {
        const GroupDesc &G = H.groups[g];
        for (int wv = 0; wv < 8; ++wv) {
            const int *t = G.task[wv];
            if (t[0] == T_NONE) continue;
            int rows[2] = {G.blk[t[1]], t[0] == T_PAIR ? G.blk[t[2]] : -1};
            for (int r : rows) {
                if (r < 0) continue;
                lo[g] = std::min(lo[g], r);
                hi[g] = std::max(hi[g], r);
                w[(size_t)r] += t[0] == T_PAIR ? 0.5 * G.cost : G.cost;
            }
        }
    }
    // a cut before row-block b is valid if no group has rows on both sides
    std::vector<char> valid((size_t)T, 1);
    for (int g = 0; g < ng; ++g)
        for (int b = lo[g] + 1; b <= hi[g]; ++b) valid[(size_t)b] = 0;
    const std::vector<int> cut = piece_cuts(w, valid, k);
    if ((int)cut.size() != k - 1) return false;
    auto piece_of_row = [&](int r) {
        int p = 0;
        while (p < k - 1 && r >= cut[(size_t)p]) ++p;
        return p;
    };
    // the launched workgroups by piece, each XCD's list order kept
    const int nwg = (int)H.seg.size() / 2;
    std::vector<std::vector<std::vector<int>>> per((size_t)k, std::vector<std::vector<int>>(8));
    for (int b = 0; b < nwg; ++b) {
        const int v0 = H.seg[2 * b], cnt = H.seg[2 * b + 1];
        if (cnt == 0) continue;  // an idle workgroup
        int p = -1;
        for (int v = v0; v < v0 + cnt; ++v) {
            const int g = H.wg[5 * v];
            const int pg = piece_of_row(lo[g]);
            if (p >= 0 && pg != p) return false;  // a workgroup spans two pieces
            p = pg;
        }
        per[(size_t)p][(size_t)(b % 8)].push_back(v0);
        per[(size_t)p][(size_t)(b % 8)].push_back(cnt);
    }
    tile_end.clear();
    seg.clear();
    for (int p = 0; p < k; ++p) {
        size_t mx = 0;
        for (auto &l : per[(size_t)p]) mx = std::max(mx, l.size() / 2);
        std::vector<int> tb;
        for (size_t j = 0; j < mx; ++j)
            for (int x = 0; x < 8; ++x) {
                const auto &l = per[(size_t)p][(size_t)x];
                tb.push_back(j < l.size() / 2 ? l[2 * j] : 0);
                tb.push_back(j < l.size() / 2 ? l[2 * j + 1] : 0);
            }
        seg.push_back(tb);
        const int b1 = p + 1 < k ? cut[(size_t)p] : T;
        tile_end.push_back(b1 * T - b1 * (b1 - 1) / 2);
    }
    return true;
}

}  // namespace bk
