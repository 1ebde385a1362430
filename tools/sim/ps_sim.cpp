// ps_sim — CPU simulator of the engine's bulk-synchronous ε-scaling push-relabel
// (design tool, not product code). Counts sweeps / global updates per phase for
// algorithm variants on the Quincy generator, so schedule changes can be judged
// without GPU time. Build: g++ -O2 -std=c++17 ps_sim.cpp ../../oracle/ks_oracle.c
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <queue>
#include <vector>
extern "C" {
#include "../../oracle/ks_oracle.h"
}
using i64 = long long;
static const i64 INF = 0x3fffffffffffffffLL;

struct G {
    int n;
    std::vector<int> first, head, rev;
    std::vector<i64> rcap, cost;
    std::vector<i64> excess, P, PN;
};

static i64 floordiv(i64 a, i64 b) { i64 q = a / b; if ((a % b) && (a < 0)) --q; return q; }

struct Opt {
    int alpha = 16, gi = 48, precise = 0, early_gu = 0, verbose = 1, sat_eps = 0, pref = 0, bfk = 0, tailT = 0;
};

struct Stats { i64 tail_sweeps = 0, sweeps = 0, gus = 0, bf_rounds = 0, visits = 0, relabels = 0, gu_scans = 0, gu_settled = 0; };

// global update: Dijkstra from deficits, length floor(rc/eps)+1; returns max hops
static int gu(G& g, i64 eps, bool early, Stats& st) {
    const int n = g.n;
    std::vector<i64> d(n, INF);
    std::vector<int> hops(n, 0);
    std::vector<char> done(n, 0);
    using QE = std::pair<i64, int>;
    std::priority_queue<QE, std::vector<QE>, std::greater<QE>> pq;
    int nex = 0;
    for (int v = 0; v < n; ++v) {
        if (g.excess[v] < 0) { d[v] = 0; pq.push({0, v}); }
        if (g.excess[v] > 0) ++nex;
    }
    i64 level = 0;
    int maxh = 0;
    while (!pq.empty()) {
        auto [dv, v] = pq.top(); pq.pop();
        if (done[v] || dv != d[v]) continue;
        done[v] = 1; level = dv;
        st.gu_settled++;
        st.gu_scans += g.first[v + 1] - g.first[v];
        maxh = std::max(maxh, hops[v]);
        if (early && g.excess[v] > 0 && --nex == 0) break;
        for (int a = g.first[v]; a < g.first[v + 1]; ++a) {
            int ra = g.rev[a];
            if (g.rcap[ra] <= 0) continue;
            int u = g.head[a];
            if (done[u]) continue;
            i64 rc = g.cost[ra] + g.P[u] - g.P[v];
            i64 nd = dv + std::max<i64>(0, floordiv(rc, eps) + 1);
            if (nd < d[u]) { d[u] = nd; hops[u] = hops[v] + 1; pq.push({nd, u}); }
        }
    }
    i64 dt = 0;
    for (int v = 0; v < n; ++v) if (done[v]) dt = std::max(dt, d[v]);
    if (early) dt = level;
    for (int v = 0; v < n; ++v) {
        i64 dd = done[v] ? d[v] : dt;
        g.P[v] -= eps * std::min(dd, dt);
        g.PN[v] = g.P[v];
    }
    st.gus++;
    st.bf_rounds += maxh + 1;
    return maxh;
}

// price refinement: Bellman-Ford (Jacobi rounds) on difference constraints
// d(u) <= d(v) + floor(rc(u,v)/eps) + 1 over residual arcs, d <= 0. Success -> prices
// p - eps*d make the current pseudoflow eps-optimal. Returns rounds used, -1 on failure.
static int price_refine(G& g, i64 eps, int max_rounds, Stats& st) {
    const int n = g.n;
    std::vector<i64> d(n, 0), nd(n);
    for (int r = 0; r < max_rounds; ++r) {
        bool changed = false;
        nd = d;
        for (int u = 0; u < n; ++u)
            for (int a = g.first[u]; a < g.first[u + 1]; ++a) {
                if (g.rcap[a] <= 0) continue;
                int v = g.head[a];
                i64 l = floordiv(g.cost[a] + g.P[u] - g.P[v], eps) + 1;
                if (d[v] + l < nd[u]) { nd[u] = d[v] + l; changed = true; }
            }
        d.swap(nd);
        st.bf_rounds++;
        if (!changed) {
            for (int v = 0; v < n; ++v) { g.P[v] -= eps * d[v]; g.PN[v] = g.P[v]; }
            return r + 1;
        }
    }
    return -1;
}

// GU by synchronous Bellman-Ford rounds from the deficits, truncated after kmax
// rounds: d' = min(d, L), L = min distance still on the frontier (valid cap).
static void gu_bf(G& g, i64 eps, int kmax, Stats& st) {
    const int n = g.n;
    std::vector<i64> d(n, INF);
    std::vector<char> fr(n, 0), nf(n, 0);
    for (int v = 0; v < n; ++v) if (g.excess[v] < 0) { d[v] = 0; fr[v] = 1; }
    int rounds = 0;
    bool any = true;
    while (any && rounds < kmax) {
        any = false;
        std::vector<i64> dn = d;
        for (int v = 0; v < n; ++v) {
            if (!fr[v]) continue;
            for (int a = g.first[v]; a < g.first[v + 1]; ++a) {
                int ra = g.rev[a];
                if (g.rcap[ra] <= 0) continue;
                int u = g.head[a];
                i64 rc = g.cost[ra] + g.P[u] - g.P[v];
                i64 nd = d[v] + std::max<i64>(0, floordiv(rc, eps) + 1);
                if (nd < dn[u]) { dn[u] = nd; nf[u] = 1; any = true; }
            }
        }
        d.swap(dn);
        fr.swap(nf);
        std::fill(nf.begin(), nf.end(), 0);
        rounds++;
    }
    i64 L = 0;
    if (any) {
        L = INF;
        for (int v = 0; v < n; ++v) if (fr[v]) L = std::min(L, d[v]);
    } else {
        for (int v = 0; v < n; ++v) if (d[v] < INF) L = std::max(L, d[v]);
    }
    for (int v = 0; v < n; ++v) {
        i64 dd = std::min(d[v], L);
        g.P[v] -= eps * dd;
        g.PN[v] = g.P[v];
    }
    st.gus++;
    st.bf_rounds += rounds;
}

int main(int argc, char** argv) {
    i64 T = 100000, M = 10000, R = 250, J = 1000; uint64_t seed = 3;
    Opt o;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-a")) o.alpha = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-g")) o.gi = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-p")) o.precise = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-e")) o.early_gu = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-c2")) { T = 10000; M = 1000; R = 25; J = 100; seed = 2; }
        else if (!strcmp(argv[i], "-q")) o.verbose = 0;
        else if (!strcmp(argv[i], "-s")) o.sat_eps = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-r")) o.pref = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-k")) o.bfk = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-t")) o.tailT = atoi(argv[++i]);
    }
    int64_t n, m;
    ko_quincy_sizes(T, M, R, J, &n, &m);
    ko_graph kg;
    std::vector<int32_t> nt(n); std::vector<int64_t> sup(n), src(m), dst(m), low(m), cap(m), cost(m);
    kg.ntype = nt.data(); kg.supply = sup.data(); kg.src = src.data(); kg.dst = dst.data();
    kg.low = low.data(); kg.cap = cap.data(); kg.cost = cost.data();
    ko_gen_quincy(T, M, R, J, seed, &kg);
    // residual CSR (arc order: by tail, stable over input order: fwd 2i, rev 2i+1)
    G g; g.n = (int)n;
    std::vector<int> deg(n + 1, 0);
    for (i64 i = 0; i < m; ++i) { deg[src[i] - 1]++; deg[dst[i] - 1]++; }
    g.first.assign(n + 1, 0);
    for (i64 v = 0; v < n; ++v) g.first[v + 1] = g.first[v] + deg[v];
    std::vector<int> pos(g.first.begin(), g.first.end() - 1);
    g.head.resize(2 * m); g.rev.resize(2 * m); g.rcap.resize(2 * m); g.cost.resize(2 * m);
    i64 mult = n + 1, maxc = 0;
    for (i64 i = 0; i < m; ++i) {
        int s = src[i] - 1, d = dst[i] - 1;
        int a = pos[s]++, b = pos[d]++;
        g.head[a] = d; g.head[b] = s; g.rev[a] = b; g.rev[b] = a;
        g.rcap[a] = cap[i]; g.rcap[b] = 0; g.cost[a] = cost[i] * mult; g.cost[b] = -cost[i] * mult;
        maxc = std::max<i64>(maxc, std::llabs(cost[i]));
    }
    g.excess.assign(sup.begin(), sup.end());
    g.P.assign(n, 0); g.PN.assign(n, 0);
    Stats tot;
    i64 eps = std::max<i64>(1, maxc * mult);
    std::vector<i64> esnap(n);
    std::vector<char> act(n);
    do {
        eps = std::max<i64>(1, eps / o.alpha);
        Stats ph;
        bool balanced = true;
        for (int v = 0; v < n; ++v) if (g.excess[v] != 0) { balanced = false; break; }
        if (o.pref && balanced) {
            int rr = price_refine(g, eps, o.pref, ph);
            if (o.verbose) printf("  price refine eps=%lld: %d rounds\n", eps, rr);
            if (rr > 0) { tot.bf_rounds += ph.bf_rounds; continue; }
        }
        for (int u = 0; u < n; ++u)
            for (int a = g.first[u]; a < g.first[u + 1]; ++a)
                if (g.rcap[a] > 0 && g.cost[a] + g.P[u] - g.P[g.head[a]] < (o.sat_eps ? -eps : 0)) {
                    i64 r = g.rcap[a]; g.rcap[a] = 0; g.rcap[g.rev[a]] += r;
                    g.excess[u] -= r; g.excess[g.head[a]] += r;
                }
        if (o.bfk) gu_bf(g, eps, o.bfk, ph); else gu(g, eps, o.early_gu, ph);
        int since = 0;
        for (;;) {
            int nact = 0;
            for (int v = 0; v < n; ++v) { esnap[v] = g.excess[v]; act[v] = esnap[v] > 0; nact += act[v]; }
            if (!nact) break;
            ph.sweeps++;
            const bool tail = o.tailT && nact <= o.tailT;
            if (tail) ph.tail_sweeps++;
            if (getenv("SIM_DUMP") && eps == atoll(getenv("SIM_DUMP")) && ph.sweeps >= 300 && ph.sweeps < 306) {
                int cnt[6] = {0};
                i64 ex[6] = {0};
                for (int v = 0; v < n; ++v) if (act[v]) { cnt[nt[v]]++; ex[nt[v]] += esnap[v]; }
                printf("sweep %lld active by type (0 other,1 task,2 pu,3 sink,4 mach): ", ph.sweeps);
                for (int k = 0; k < 5; ++k) printf("%d:%d/%lld ", k, cnt[k], ex[k]);
                int shown = 0;
                for (int v = 0; v < n && shown < 12; ++v) if (act[v]) { printf(" [%d t%d e%lld]", v, nt[v], esnap[v]); shown++; }
                printf("\n");
            }
            for (int v = 0; v < n; ++v) {
                if (!act[v]) continue;
                ph.visits++;
                i64 rem = esnap[v], minc = INF;
                const i64 pv = g.P[v];
                for (int a = g.first[v]; a < g.first[v + 1]; ++a) {
                    const i64 r = g.rcap[a];
                    const int w = g.head[a];
                    const i64 cr = g.cost[a] + pv - g.P[w];
                    if (cr < 0) {
                        if (r > 0) {
                            i64 d = std::min(r, rem);
                            g.rcap[a] -= d; g.rcap[g.rev[a]] += d; g.excess[w] += d; g.excess[v] -= d; rem -= d;
                            if (rem == 0) break;
                        }
                    } else if (r > 0 || (cr <= eps && (!o.precise || act[w]))) {
                        minc = std::min(minc, cr);
                    }
                }
                if (rem > 0) {
                    if (minc >= INF) { fprintf(stderr, "infeasible\n"); return 1; }
                    g.PN[v] = pv - (minc + eps);
                    ph.relabels++;
                }
            }
            for (int v = 0; v < n; ++v) g.P[v] = g.PN[v];
            if (tail) since = 0;
            if (++since >= o.gi) { if (o.bfk) gu_bf(g, eps, o.bfk, ph); else gu(g, eps, o.early_gu, ph); since = 0; }
            if (ph.sweeps > 2000000) { fprintf(stderr, "no convergence\n"); return 1; }
        }
        if (o.verbose)
            printf("eps=%lld tail=%lld sweeps=%lld gus=%lld bf_rounds=%lld visits=%lld relabels=%lld gu_settled/gu=%lld gu_scans/gu=%lld\n", eps, ph.tail_sweeps, ph.sweeps, ph.gus,
                   ph.bf_rounds, ph.visits, ph.relabels, ph.gu_settled / std::max<i64>(1, ph.gus), ph.gu_scans / std::max<i64>(1, ph.gus));
        tot.sweeps += ph.sweeps; tot.tail_sweeps += ph.tail_sweeps; tot.gus += ph.gus; tot.bf_rounds += ph.bf_rounds; tot.visits += ph.visits;
        tot.relabels += ph.relabels;
    } while (eps > 1);
    i64 c = 0;
    // cost = Σ over forward arcs of flow·cost; flow on arc a = rcap[rev a] for forward arcs (cost sign by construction)
    std::vector<char> isf(2 * m, 0);
    {
        std::vector<int> p2(g.first.begin(), g.first.end() - 1);
        for (i64 i = 0; i < m; ++i) { int s = src[i] - 1, d = dst[i] - 1; isf[p2[s]++] = 1; p2[d]++; }
    }
    for (i64 a = 0; a < 2 * m; ++a) if (isf[a]) c += g.rcap[g.rev[a]] * (g.cost[a] / mult);
    printf("TOTAL tail=%lld sat_eps=%d alpha=%d gi=%d precise=%d early=%d: cost=%lld sweeps=%lld gus=%lld bf_rounds=%lld visits=%lld relabels=%lld\n",
           tot.tail_sweeps, o.sat_eps, o.alpha, o.gi, o.precise, o.early_gu, c, tot.sweeps, tot.gus, tot.bf_rounds, tot.visits, tot.relabels);
}
