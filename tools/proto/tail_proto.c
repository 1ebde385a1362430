/* Design prototype (CPU, not part of the product or the oracle): how large is
 * the search a phase-tail "SSP in ε units" needs? Runs Goldberg cost scaling
 * with the engine's ε ladder (costs × (n+1), final phase at 1/48 unit) and,
 * once the final phase has ≤ K excess nodes, finishes it by multi-source
 * bounded Bellman-Ford searches from the excess nodes (lengths floor(rc/ε)+1),
 * price update p(v) −= ε·(D* − d(v)) on the nodes closer than the nearest
 * deficit D*, and one augmentation per search. Reports per-search visited
 * nodes, relaxations and BF rounds, and checks the final cost against a given
 * value. Build: gcc -O2 -o /tmp/tail_proto tools/proto/tail_proto.c oracle/ks_oracle.c -Ioracle */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ks_oracle.h"

#define INF ((int64_t)0x3fffffffffffffffLL)
typedef struct { int64_t n, m; int64_t *first, *head, *rcap, *cost, *rev, *ex; } R;

static int64_t fdiv(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b) && (a < 0)) --q; return q; }

int main(int argc, char** argv) {
    int64_t T = argc > 1 ? atoll(argv[1]) : 100000, M = T / 10, Rk = T / 400, J = T / 100;
    uint64_t seed = argc > 2 ? atoll(argv[2]) : 3;
    int K = argc > 3 ? atoi(argv[3]) : 64;
    int64_t n, m;
    ko_quincy_sizes(T, M, Rk, J, &n, &m);
    ko_graph g;
    g.ntype = calloc(n, 4); g.supply = calloc(n, 8);
    g.src = calloc(m, 8); g.dst = calloc(m, 8); g.low = calloc(m, 8); g.cap = calloc(m, 8); g.cost = calloc(m, 8);
    ko_gen_quincy(T, M, Rk, J, seed, &g);
    R r; r.n = n; r.m = m;
    r.first = calloc(n + 1, 8); r.head = malloc(16 * m); r.rcap = malloc(16 * m); r.cost = malloc(16 * m);
    r.rev = malloc(16 * m); r.ex = calloc(n, 8);
    for (int64_t i = 0; i < m; ++i) { r.first[g.src[i]]++; r.first[g.dst[i]]++; }
    for (int64_t v = 0; v < n; ++v) r.first[v + 1] += r.first[v];
    int64_t* pos = malloc(8 * (n + 1)); memcpy(pos, r.first, 8 * (n + 1));
    const int64_t mult = n + 1;
    int64_t maxc = 0;
    for (int64_t i = 0; i < m; ++i) {
        int64_t s = g.src[i] - 1, d = g.dst[i] - 1, a = pos[s]++, b = pos[d]++;
        r.head[a] = d; r.rcap[a] = g.cap[i]; r.cost[a] = g.cost[i] * mult; r.rev[a] = b;
        r.head[b] = s; r.rcap[b] = 0; r.cost[b] = -g.cost[i] * mult; r.rev[b] = a;
        if (g.cost[i] > maxc) maxc = g.cost[i];
    }
    for (int64_t v = 0; v < n; ++v) r.ex[v] = g.supply[v];
    int64_t* p = calloc(n, 8);
    /* the engine's ladder: final eps = (mult-1)/48, times 8 up to the first below max|cost|·mult/8 */
    int64_t e = (mult - 1) / 48, lo = maxc * mult / 64;
    while (e < lo) e *= 8;
    int64_t eps = e * 8;
    int64_t* q = malloc(8 * (n + 1)); char* inq = calloc(n, 1); int64_t* cur = malloc(8 * n);
    int64_t* d = malloc(8 * n); int64_t* pred = malloc(8 * n); char* seen = calloc(n, 1);
    int64_t* front = malloc(8 * n); int64_t* nxt = malloc(8 * n); int64_t* vis = malloc(8 * n);
    for (int64_t v = 0; v < n; ++v) d[v] = INF;
    int phase = 0;
    long long tot_iters = 0, tot_vis = 0, tot_relax = 0, tot_rounds = 0, max_vis = 0, max_rounds = 0;
    while (eps > 1) {
        eps = eps / 8 < 1 ? 1 : eps / 8;
        ++phase;
        const int final = eps * 48 < mult;
        for (int64_t u = 0; u < n; ++u)
            for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a)
                if (r.rcap[a] > 0 && r.cost[a] + p[u] - p[r.head[a]] < (getenv("SAT_EPS") ? -eps : 0)) {
                    int64_t x = r.rcap[a]; r.rcap[a] = 0; r.rcap[r.rev[a]] += x; r.ex[u] -= x; r.ex[r.head[a]] += x;
                }
        /* FIFO push-relabel until ≤ K excess nodes in the final phase (all excess elsewhere) */
        int64_t qh = 0, qt = 0, qn = 0, nexc = 0;
        for (int64_t v = 0; v < n; ++v) { cur[v] = r.first[v]; inq[v] = 0; if (r.ex[v] > 0) { q[qt++] = v; inq[v] = 1; ++qn; } }
        nexc = qn;
        const int all_bf = getenv("TAIL_ALL") != NULL;
        while (qn > 0 && !(all_bf || (final && nexc <= K))) {
            int64_t u = q[qh++]; if (qh == n + 1) qh = 0; --qn; inq[u] = 0;
            while (r.ex[u] > 0) {
                int64_t a = cur[u];
                for (; a < r.first[u + 1]; ++a) {
                    if (r.rcap[a] <= 0) continue;
                    int64_t v = r.head[a];
                    if (r.cost[a] + p[u] - p[v] >= 0) continue;
                    int64_t x = r.rcap[a] < r.ex[u] ? r.rcap[a] : r.ex[u];
                    int64_t old = r.ex[v];
                    r.rcap[a] -= x; r.rcap[r.rev[a]] += x; r.ex[u] -= x; r.ex[v] += x;
                    if (old <= 0 && r.ex[v] > 0) { ++nexc; if (!inq[v]) { q[qt++] = v; if (qt == n + 1) qt = 0; ++qn; inq[v] = 1; } }
                    if (r.ex[u] == 0) { --nexc; break; }
                }
                cur[u] = a;
                if (r.ex[u] == 0) break;
                int64_t mn = INF;
                for (int64_t b = r.first[u]; b < r.first[u + 1]; ++b)
                    if (r.rcap[b] > 0) { int64_t rc = r.cost[b] + p[u] - p[r.head[b]]; if (rc < mn) mn = rc; }
                p[u] -= mn + eps;
                cur[u] = r.first[u];
            }
        }
        if (!final && !all_bf) continue;
        if (getenv("TAIL_BLOCKING") && (final || all_bf)) {
            /* tail: global update from the deficits (exact BF, lengths floor(rc/eps)+1), price
             * update p -= eps*min(d, L), then a blocking flow by DFS with dead-end marks over the
             * admissible arcs toward no larger distance (rc' < 0, d(w) <= d(u), residual) */
            int64_t gus = 0, moved_total = 0;
            char* dead = calloc(n, 1);
            const int hub_rule = getenv("HUB_RULE") != NULL;
            const int unit = getenv("UNIT") != NULL;
            int64_t* stk = malloc(8 * (n + 1));
            for (;;) {
                int64_t nx = 0;
                for (int64_t v = 0; v < n; ++v) if (r.ex[v] > 0) ++nx;
                if (!nx) break;
                ++gus;
                /* BF from deficits over residual arcs (u -> w): d(u) = min d(w) + len */
                int64_t nf = 0;
                for (int64_t v = 0; v < n; ++v) { d[v] = r.ex[v] < 0 ? 0 : INF; if (r.ex[v] < 0) front[nf++] = v; }
                while (nf) {
                    int64_t nn2 = 0;
                    for (int64_t i = 0; i < nf; ++i) {
                        int64_t w = front[i];
                        for (int64_t a = r.first[w]; a < r.first[w + 1]; ++a) {
                            int64_t ra = r.rev[a];           /* arc u -> w */
                            if (r.rcap[ra] <= 0) continue;
                            int64_t u = r.head[a];
                            int64_t nd = d[w] + fdiv(r.cost[ra] + p[u] - p[w], eps) + 1;
                            if (nd < d[u]) { d[u] = nd; if (!seen[u]) { seen[u] = 1; nxt[nn2++] = u; } }
                        }
                    }
                    for (int64_t i = 0; i < nn2; ++i) seen[nxt[i]] = 0;
                    int64_t* t = front; front = nxt; nxt = t; nf = nn2;
                }
                int64_t L = 0;
                for (int64_t v = 0; v < n; ++v) if (d[v] < INF && d[v] > L) L = d[v];
                for (int64_t v = 0; v < n; ++v) p[v] -= eps * (d[v] < L ? d[v] : L);
                /* blocking flow */
                memset(dead, 0, n);
                int64_t moved = 0;
                for (int64_t s0 = 0; s0 < n; ++s0) {
                    while (r.ex[s0] > 0 && !dead[s0]) {
                        int64_t top = 0; stk[top] = -1;
                        int64_t u = s0, found = -1;
                        int64_t* path = malloc(8 * 4096); int64_t plen = 0;
                        for (int steps = 0; steps < 100000; ++steps) {
                            if (r.ex[u] < 0 && u != s0) { found = u; break; }
                            if (hub_rule && u != s0 && r.first[u + 1] - r.first[u] > 4096 && r.ex[u] <= 0) {
                                dead[u] = 1;   /* HUB_RULE: a hub without excess is a dead end (device list rule) */
                                u = r.head[r.rev[path[--plen]]];
                                continue;
                            }
                            int64_t best = -1, bd = INF;
                            for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a) {
                                if (r.rcap[a] <= 0) continue;
                                int64_t w = r.head[a];
                                if (dead[w]) continue;
                                int64_t rc = r.cost[a] + p[u] - p[w];
                                if (rc >= 0) continue;           /* admissible only */
                                if (d[w] > d[u] && d[u] < L) continue;
                                if (d[w] < bd) { bd = d[w]; best = a; }
                            }
                            if (best < 0) {                       /* dead end: retreat */
                                dead[u] = 1;
                                if (!plen) break;
                                u = r.head[r.rev[path[--plen]]];
                                continue;
                            }
                            if (plen >= 4096) break;
                            path[plen++] = best;
                            u = r.head[best];
                        }
                        if (found < 0) { free(path); break; }
                        int64_t delta = r.ex[s0] < -r.ex[found] ? r.ex[s0] : -r.ex[found];
                        if (unit) delta = 1;
                        for (int64_t i = 0; i < plen; ++i) if (r.rcap[path[i]] < delta) delta = r.rcap[path[i]];
                        for (int64_t i = 0; i < plen; ++i) { r.rcap[path[i]] -= delta; r.rcap[r.rev[path[i]]] += delta; }
                        r.ex[s0] -= delta; r.ex[found] += delta; moved += delta;
                        free(path);
                    }
                }
                moved_total += moved;
                if (getenv("TAIL_TRACE")) fprintf(stderr, "GU %lld: excess nodes %lld, moved %lld, L %lld\n", (long long)gus, (long long)nx, (long long)moved, (long long)L);
                if (!moved && gus > 200) break;
            }
            printf("phase %d eps %lld: blocking-flow: %lld global updates moved %lld units\n", phase, (long long)eps, (long long)gus, (long long)moved_total);
        }
        /* tail: SSP in eps units */
        int64_t nsrc = 0;
        for (int64_t v = 0; v < n; ++v) if (r.ex[v] > 0) ++nsrc;
        fprintf(stderr, "phase %d eps %lld: tail starts with %lld excess nodes\n", phase, (long long)eps, (long long)nsrc);
        for (;;) {
            int64_t nf = 0, nv = 0;
            for (int64_t v = 0; v < n; ++v) if (r.ex[v] > 0) { d[v] = 0; pred[v] = -1; front[nf++] = v; vis[nv++] = v; seen[v] = 1; }
            if (!nf) break;
            int64_t best = INF, tbest = -1, relax = 0, rounds = 0;
            while (nf) {
                ++rounds;
                int64_t nn2 = 0;
                for (int64_t i = 0; i < nf; ++i) {
                    int64_t u = front[i];
                    if (d[u] >= best || r.ex[u] < 0) continue;
                    for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a) {
                        if (r.rcap[a] <= 0) continue;
                        ++relax;
                        int64_t v = r.head[a];
                        int64_t nd = d[u] + fdiv(r.cost[a] + p[u] - p[v], eps) + 1;
                        if (nd < d[v] && nd < best) {
                            if (!seen[v]) { seen[v] = 1; vis[nv++] = v; }
                            d[v] = nd; pred[v] = a;
                            if (r.ex[v] < 0) { if (nd < best) { best = nd; tbest = v; } }
                            else nxt[nn2++] = v;
                        }
                    }
                }
                int64_t* t = front; front = nxt; nxt = t; nf = nn2;
            }
            if (tbest < 0) { fprintf(stderr, "infeasible tail\n"); return 1; }
            for (int64_t i = 0; i < nv; ++i) { int64_t v = vis[i]; if (d[v] < best) p[v] -= eps * (best - d[v]); }
            int64_t s = tbest, delta = -r.ex[tbest];
            while (pred[s] >= 0) { int64_t a = pred[s]; if (r.rcap[a] < delta) delta = r.rcap[a]; s = r.head[r.rev[a]]; }
            if (r.ex[s] < delta) delta = r.ex[s];
            for (int64_t v = tbest; pred[v] >= 0;) { int64_t a = pred[v]; r.rcap[a] -= delta; r.rcap[r.rev[a]] += delta; v = r.head[r.rev[a]]; }
            r.ex[s] -= delta; r.ex[tbest] += delta;
            if (getenv("TAIL_TRACE")) fprintf(stderr, "search %lld D* %lld units %.2f delta %lld nsrc-left\n", tot_iters, (long long)best, (double)best * eps / mult, (long long)delta);
            ++tot_iters; tot_vis += nv; tot_relax += relax; tot_rounds += rounds;
            if (nv > max_vis) max_vis = nv;
            if (rounds > max_rounds) max_rounds = rounds;
            for (int64_t i = 0; i < nv; ++i) { d[vis[i]] = INF; seen[vis[i]] = 0; }
        }
        /* price refinement would certify here; check optimality by the cost */
        if (final) break;
    }
    int64_t c = 0;
    for (int64_t u = 0; u < n; ++u)
        for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a)
            if (r.cost[a] > 0 && r.rcap[r.rev[a]] > 0) c += r.rcap[r.rev[a]] * (r.cost[a] / mult);
    int64_t left = 0;
    for (int64_t v = 0; v < n; ++v) if (r.ex[v] > 0) left += r.ex[v];
    printf("T %lld: final-phase tail searches %lld, visited avg %.0f max %lld, relaxations avg %.0f, rounds avg %.1f max %lld; cost %lld, excess left %lld\n",
           (long long)T, tot_iters, tot_iters ? (double)tot_vis / tot_iters : 0, max_vis,
           tot_iters ? (double)tot_relax / tot_iters : 0, tot_iters ? (double)tot_rounds / tot_iters : 0, max_rounds,
           (long long)c, (long long)left);
    return 0;
}
