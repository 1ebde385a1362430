/* Design prototype (CPU, not part of the product or the oracle): how far from
 * optimal is the flow of the last COARSE phase, measured as negative cycles?
 * Runs Goldberg cost scaling with the engine's ε ladder (costs × (n+1), final
 * phase at 1/D unit, α = 8; FIFO push-relabel, each phase drained), stops after
 * the phase at ε = STOP·(final ε) (STOP = 8: the phase before the final one),
 * then repeats: round-synchronous Bellman-Ford from d ≡ 0 over residual arcs with
 * the unscaled costs (the certificate's difference constraints), every 8 rounds
 * the predecessor graph is searched for cycles, and every cycle found is
 * cancelled (its bottleneck pushed around it) — as a GPU version would do in
 * parallel. Reports BF passes, rounds and cycles per pass, and the final cost.
 * Build: gcc -O2 -o /tmp/cc/cc tools/proto/cycle_cancel.c oracle/ks_oracle.c -Ioracle
 * Run:   /tmp/cc/cc [T=100000] [seed=3] [D=48] [STOP=8] */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ks_oracle.h"

#define INF ((int64_t)0x3fffffffffffffffLL)
typedef struct { int64_t n, m; int64_t *first, *head, *rcap, *cost, *rev, *ex; } R;

int main(int argc, char** argv) {
    int64_t T = argc > 1 ? atoll(argv[1]) : 100000, M = T / 10, Rk = T / 400, J = T / 100;
    uint64_t seed = argc > 2 ? atoll(argv[2]) : 3;
    int64_t D = argc > 3 ? atoll(argv[3]) : 48, STOP = argc > 4 ? atoll(argv[4]) : 8;
    const int64_t DET = getenv("CC_DET") ? atoll(getenv("CC_DET")) : 8;
    const int keep = getenv("CC_KEEP") != NULL;   /* continue the BF after cancelling instead of restarting */
    int64_t n, m;
    ko_quincy_sizes(T, M, Rk, J, &n, &m);
    ko_graph g;
    g.ntype = calloc(n, 4); g.supply = calloc(n, 8);
    g.src = calloc(m, 8); g.dst = calloc(m, 8); g.low = calloc(m, 8); g.cap = calloc(m, 8); g.cost = calloc(m, 8);
    ko_gen_quincy(T, M, Rk, J, seed, &g);
    R r; r.n = n; r.m = m;
    r.first = calloc(n + 1, 8); r.head = malloc(16 * m); r.rcap = malloc(16 * m); r.cost = malloc(16 * m);
    r.rev = malloc(16 * m); r.ex = calloc(n, 8);
    int64_t* tail = malloc(16 * m);
    for (int64_t i = 0; i < m; ++i) { r.first[g.src[i]]++; r.first[g.dst[i]]++; }
    for (int64_t v = 0; v < n; ++v) r.first[v + 1] += r.first[v];
    int64_t* pos = malloc(8 * (n + 1)); memcpy(pos, r.first, 8 * (n + 1));
    const int64_t mult = n + 1;
    int64_t maxc = 0;
    for (int64_t i = 0; i < m; ++i) {
        int64_t s = g.src[i] - 1, d = g.dst[i] - 1, a = pos[s]++, b = pos[d]++;
        r.head[a] = d; r.rcap[a] = g.cap[i]; r.cost[a] = g.cost[i] * mult; r.rev[a] = b; tail[a] = s;
        r.head[b] = s; r.rcap[b] = 0; r.cost[b] = -g.cost[i] * mult; r.rev[b] = a; tail[b] = d;
        if (g.cost[i] > maxc) maxc = g.cost[i];
    }
    for (int64_t v = 0; v < n; ++v) r.ex[v] = g.supply[v];
    int64_t* p = calloc(n, 8);
    int64_t efin = (mult - 1) / D, e = efin, lo = maxc * mult / 64;
    while (e < lo) e *= 8;
    int64_t eps = e * 8;
    int64_t* q = malloc(8 * (n + 1)); char* inq = calloc(n, 1); int64_t* cur = malloc(8 * n);
    int phase = 0;
    while (eps > efin * STOP) {
        eps = eps / 8 < 1 ? 1 : eps / 8;
        ++phase;
        for (int64_t u = 0; u < n; ++u)
            for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a)
                if (r.rcap[a] > 0 && r.cost[a] + p[u] - p[r.head[a]] < 0) {
                    int64_t x = r.rcap[a]; r.rcap[a] = 0; r.rcap[r.rev[a]] += x; r.ex[u] -= x; r.ex[r.head[a]] += x;
                }
        int64_t qh = 0, qt = 0, qn = 0;
        for (int64_t v = 0; v < n; ++v) { cur[v] = r.first[v]; inq[v] = 0; if (r.ex[v] > 0) { q[qt++] = v; inq[v] = 1; ++qn; } }
        const int64_t EARLY = getenv("CC_EARLY") ? atoll(getenv("CC_EARLY")) : 0;   /* last phase ends at <= EARLY excess nodes */
        const int lastc = !(eps > efin * STOP * 8);   /* the phase PRC follows */
        while (qn > 0) {
            if (EARLY && lastc && qn <= EARLY) break;
            int64_t u = q[qh++]; if (qh == n + 1) qh = 0; --qn; inq[u] = 0;
            while (r.ex[u] > 0) {
                int64_t a = cur[u];
                for (; a < r.first[u + 1]; ++a) {
                    if (r.rcap[a] <= 0) continue;
                    int64_t v = r.head[a];
                    if (r.cost[a] + p[u] - p[v] >= 0) continue;
                    int64_t x = r.rcap[a] < r.ex[u] ? r.rcap[a] : r.ex[u];
                    r.rcap[a] -= x; r.rcap[r.rev[a]] += x; r.ex[u] -= x; r.ex[v] += x;
                    if (r.ex[v] > 0 && !inq[v]) { q[qt++] = v; if (qt == n + 1) qt = 0; ++qn; inq[v] = 1; }
                    if (r.ex[u] == 0) break;
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
        {   /* forced routing of what an early end left: Dijkstra on max(0, rc) from each excess node */
            int64_t left = 0, nx = 0;
            for (int64_t v = 0; v < n; ++v) if (r.ex[v] > 0) { left += r.ex[v]; ++nx; }
            if (left) {
                int64_t* dd = malloc(8 * n); int64_t* pa = malloc(8 * n); char* done = calloc(n, 1);
                int64_t* hk = malloc(16 * m + 16); int64_t* hv = malloc(16 * m + 16);
                int64_t routed = 0;
                for (int64_t s0 = 0; s0 < n; ++s0) {
                    while (r.ex[s0] > 0) {
                        for (int64_t v = 0; v < n; ++v) { dd[v] = INF; pa[v] = -1; done[v] = 0; }
                        /* simple binary heap */
                        int64_t hn = 0; dd[s0] = 0; hk[hn] = 0; hv[hn++] = s0;
                        int64_t t = -1;
                        while (hn) {
                            int64_t bi = 0; for (int64_t i = 1; i < hn; ++i) if (hk[i] < hk[bi]) bi = i;   /* O(n) pop: prototype */
                            int64_t k0 = hk[bi], u = hv[bi]; hk[bi] = hk[--hn]; hv[bi] = hv[hn];
                            if (done[u] || k0 > dd[u]) continue;
                            done[u] = 1;
                            if (r.ex[u] < 0 && u != s0) { t = u; break; }
                            for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a) {
                                if (r.rcap[a] <= 0) continue;
                                int64_t w = r.head[a], rc = r.cost[a] + p[u] - p[w];
                                int64_t nd = dd[u] + (rc > 0 ? rc : 0);
                                if (nd < dd[w]) { dd[w] = nd; pa[w] = a; hk[hn] = nd; hv[hn++] = w; }
                            }
                        }
                        if (t < 0) { fprintf(stderr, "no route\n"); exit(3); }
                        int64_t dl = r.ex[s0] < -r.ex[t] ? r.ex[s0] : -r.ex[t];
                        for (int64_t v = t; v != s0; v = tail[pa[v]]) if (r.rcap[pa[v]] < dl) dl = r.rcap[pa[v]];
                        for (int64_t v = t; v != s0; v = tail[pa[v]]) { r.rcap[pa[v]] -= dl; r.rcap[r.rev[pa[v]]] += dl; }
                        r.ex[s0] -= dl; r.ex[t] += dl; routed += dl;
                    }
                }
                printf("  forced routing: %lld units from %lld excess nodes\n", (long long)routed, (long long)nx);
            }
        }
        int64_t c = 0;
        for (int64_t a = 0; a < 2 * m; ++a) if (r.cost[a] > 0 && r.rcap[r.rev[a]] > 0) c += r.rcap[r.rev[a]] * (r.cost[a] / mult);
        printf("phase %d eps %lld (1/%.1f unit): cost %lld\n", phase, (long long)eps, (double)mult / eps, (long long)c);
    }
    /* cycle cancelling with the unscaled costs */
    int64_t* d = malloc(8 * n); int64_t* pred = malloc(8 * n); int64_t* stamp = calloc(n, 8); char* oncyc = calloc(n, 1);
    int64_t* cyc = malloc(8 * n);
    int64_t* dold = malloc(8 * n);
    const int jacobi = getenv("CC_JACOBI") != NULL;   /* round-synchronous (the GPU's rounds) */
    int64_t passes = 0, tot_cycles = 0, tot_rounds = 0, stampc = 0;
    for (;;) {
        ++passes;
        for (int64_t v = 0; v < n; ++v) { d[v] = 0; pred[v] = -1; }
        int64_t rounds = 0, found = 0;
        int improved = 1;
        while (improved && rounds < 100000) {
            improved = 0;
            ++rounds;
            if (jacobi) memcpy(dold, d, 8 * n);
            const int64_t* dsrc = jacobi ? dold : d;
            for (int64_t a = 0; a < 2 * m; ++a) {
                if (r.rcap[a] <= 0) continue;
                int64_t u = tail[a], v = r.head[a];
                int64_t nd = dsrc[u] + r.cost[a] / mult;
                if (nd < d[v]) { d[v] = nd; pred[v] = a; improved = 1; }
            }
            if (rounds % DET == 0 || !improved) {
                /* cycles in the predecessor graph: each is negative */
                memset(oncyc, 0, n);
                for (int64_t s = 0; s < n; ++s) {
                    ++stampc;
                    int64_t v = s;
                    while (v >= 0 && pred[v] >= 0 && stamp[v] != stampc && !oncyc[v]) { stamp[v] = stampc; v = tail[pred[v]]; }
                    if (v < 0 || pred[v] < 0 || oncyc[v] || stamp[v] != stampc) continue;
                    /* v is on a cycle of this walk */
                    int64_t len = 0, w = v, delta = INF;
                    do { int64_t a = pred[w]; cyc[len++] = a; if (r.rcap[a] < delta) delta = r.rcap[a]; w = tail[a]; } while (w != v && len < n);
                    int64_t cc = 0;
                    for (int64_t i = 0; i < len; ++i) cc += r.cost[cyc[i]] / mult;
                    if (cc >= 0 || delta <= 0) continue;
                    for (int64_t i = 0; i < len; ++i) { r.rcap[cyc[i]] -= delta; r.rcap[r.rev[cyc[i]]] += delta; oncyc[tail[cyc[i]]] = 1; }
                    if (getenv("CC_TRACE")) printf("  cycle at round %lld: %lld arcs, cost %lld, delta %lld\n", (long long)rounds, (long long)len, (long long)cc, (long long)delta);
                    ++found;
                }
                if (found && !keep) break;
                if (found && keep) { tot_cycles += found; found = 0; improved = 1; memset(oncyc, 0, n); }
            }
        }
        tot_rounds += rounds;
        tot_cycles += found;
        printf("pass %lld: %lld rounds, %lld cycles cancelled\n", (long long)passes, (long long)rounds, (long long)found);
        if (!found) break;
    }
    int64_t c = 0;
    for (int64_t a = 0; a < 2 * m; ++a) if (r.cost[a] > 0 && r.rcap[r.rev[a]] > 0) c += r.rcap[r.rev[a]] * (r.cost[a] / mult);
    printf("after cancelling: cost %lld, %lld passes, %lld rounds, %lld cycles\n", (long long)c, (long long)passes,
           (long long)tot_rounds, (long long)tot_cycles);
    return 0;
}
