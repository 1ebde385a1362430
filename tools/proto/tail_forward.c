/* forward SSP tail simulation on a device dump: per update, Dijkstra from the excess nodes
   (lengths floor(rc/eps)+1 >= 0), D = nearest deficit, p -= eps*max(0, D - d), then one unit
   along each deficit-at-D's parent path (sequential, skipped if a capacity or the source ran out).
   KSRC: above this many excess nodes use the backward update + unit blocking flow instead. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef struct { long long cost, rcap, ucap; int head, rev; } Pos;
#define INF ((int64_t)0x3fffffffffffffffLL)
static int64_t fdiv(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b) && (a < 0)) --q; return q; }
/* binary heap on (d, v) */
static int64_t* hk; static int* hv; static int hn;
static void hpush(int64_t k, int v) { int i = hn++; while (i) { int p = (i - 1) / 2; if (hk[p] <= k) break; hk[i] = hk[p]; hv[i] = hv[p]; i = p; } hk[i] = k; hv[i] = v; }
static void hpop(int64_t* k, int* v) { *k = hk[0]; *v = hv[0]; int64_t lk = hk[--hn]; int lv = hv[hn]; int i = 0; for (;;) { int c = 2 * i + 1; if (c >= hn) break; if (c + 1 < hn && hk[c + 1] < hk[c]) ++c; if (hk[c] >= lk) break; hk[i] = hk[c]; hv[i] = hv[c]; i = c; } hk[i] = lk; hv[i] = lv; }
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb"); long long hdr[6]; if (!f || fread(hdr, 8, 6, f) != 6) return 2;
    const int64_t n = hdr[0], np = hdr[2], eps = hdr[3];
    int* first = malloc(4 * (n + 1)); int64_t* nd = malloc(32 * n); int64_t* ex = malloc(8 * n); Pos* pos = malloc(sizeof(Pos) * np);
    if (fread(first, 4, n + 1, f) != (size_t)(n + 1) || fread(nd, 8, 4 * n, f) != (size_t)(4 * n) || fread(ex, 8, n, f) != (size_t)n || fread(pos, sizeof(Pos), np, f) != (size_t)np) return 2;
    const int ksrc = getenv("KSRC") ? atoi(getenv("KSRC")) : 1000000;
    int64_t* p = malloc(8 * n); int* b0 = malloc(4 * n); int* b1 = malloc(4 * n);
    for (int64_t v = 0; v < n; ++v) { p[v] = nd[4 * v]; uint64_t w = (uint64_t)nd[4 * v + 3]; b0[v] = (int)(w & 0xffffffffu); b1[v] = (int)(w >> 32); }
    int* tail = malloc(4 * np); for (int64_t v = 0; v < n; ++v) for (int a = b0[v]; a < b1[v]; ++a) tail[a] = (int)v;
    int64_t* d = malloc(8 * n); int* par = malloc(4 * n); char* done = calloc(n, 1);
    hk = malloc(8 * (np + n)); hv = malloc(4 * (np + n));
    int* path = malloc(4 * 100000);
    int updates = 0; int64_t explored_tot = 0; int nback = 0, nfwd = 0; int dial_rounds = 0; int64_t dial_relax = 0; int64_t* sim_d = malloc(8 * n); char* fr = malloc(n); char* nfr = malloc(n);
    int* q = malloc(4 * n); char* inq = calloc(n, 1); char* dead = calloc(n, 1);
    for (; updates < 1000; ++updates) {
        int64_t nx = 0, ux = 0; for (int64_t v = 0; v < n; ++v) if (ex[v] > 0) { ++nx; ux += ex[v]; }
        if (!nx) break;
        int64_t moved = 0, explored = 0, D = INF;
        if (nx > ksrc) {
            /* backward: exact distances to the deficits, p -= eps*min(d, L), unit blocking flow */
            int qh = 0, qt = 0, qn = 0;
            for (int64_t v = 0; v < n; ++v) { d[v] = ex[v] < 0 ? 0 : INF; inq[v] = 0; if (ex[v] < 0) { q[qt++] = (int)v; inq[v] = 1; ++qn; } }
            while (qn) {
                const int w = q[qh++]; if (qh == n) qh = 0; --qn; inq[w] = 0;
                for (int a = b0[w]; a < b1[w]; ++a) {
                    const int ra = pos[a].rev; if (pos[ra].rcap <= 0) continue;
                    const int u = pos[a].head;
                    int64_t len = fdiv(pos[ra].cost + p[u] - p[w], eps) + 1; if (len < 0) len = 0;
                    if (d[w] + len < d[u]) { d[u] = d[w] + len; if (!inq[u]) { inq[u] = 1; q[qt++] = u; if (qt == n) qt = 0; ++qn; } }
                }
            }
            int64_t L = 0; for (int64_t v = 0; v < n; ++v) if (d[v] < INF && d[v] > L) L = d[v];
            for (int64_t v = 0; v < n; ++v) p[v] -= eps * (d[v] < L ? d[v] : L);
            memset(dead, 0, n);
            int64_t mv = 0;
            for (int64_t s0 = 0; s0 < n; ++s0) {
                while (ex[s0] > 0) {
                    int u = (int)s0, plen = 0, found = -1;
                    for (int steps = 0; steps < 1000000; ++steps) {
                        if (u != s0 && ex[u] < 0) { found = u; break; }
                        int best = -1; int64_t bd = INF;
                        for (int a = b0[u]; a < b1[u]; ++a) {
                            if (pos[a].rcap <= 0) continue; const int w = pos[a].head;
                            if (w == u || dead[w]) continue;
                            const int64_t rc = pos[a].cost + p[u] - p[w];
                            const int ok = (rc < 0 && d[w] <= d[u]) || (rc <= eps && d[w] < d[u]);
                            if (ok && d[w] < bd) { bd = d[w]; best = a; }
                        }
                        if (best < 0 || plen >= 100000) { dead[u] = 1; if (!plen) break; u = tail[path[--plen]]; continue; }
                        path[plen++] = best; u = pos[best].head;
                    }
                    if (found < 0) break;
                    for (int i = 0; i < plen; ++i) { pos[path[i]].rcap -= 1; pos[pos[path[i]].rev].rcap += 1; }
                    ex[s0] -= 1; ex[found] += 1; ++mv;
                }
            }
            ++nback;
            printf("update %d (backward): excess nodes %lld (%lld units), moved %lld\n", updates + 1, (long long)nx, (long long)ux, (long long)mv);
            continue;
        }
        ++nfwd;
        {   /* Dial: level by level, a level's zero-length BFS in synchronous waves */
            int64_t* dd = sim_d; int64_t relax = 0; int rounds = 0, levels = 0;
            for (int64_t v = 0; v < n; ++v) { dd[v] = ex[v] > 0 ? 0 : INF; fr[v] = ex[v] > 0; }
            int64_t L = 0, Dd = INF;
            for (;;) {
                /* process level L: waves over nodes with dd == L (fr marks those not yet expanded) */
                int any = 1;
                while (any) {
                    any = 0; ++rounds;
                    memset(nfr, 0, n);
                    for (int64_t u = 0; u < n; ++u) {
                        if (!fr[u] || dd[u] != L) continue;
                        fr[u] = 0;
                        if (ex[u] < 0) continue;
                        for (int a = b0[u]; a < b1[u]; ++a) {
                            ++relax;
                            if (pos[a].rcap <= 0) continue; const int w = pos[a].head;
                            int64_t len = fdiv(pos[a].cost + p[u] - p[w], eps) + 1; if (len < 0) len = 0;
                            const int64_t c = L + len;
                            if (c > Dd) continue;
                            if (c < dd[w]) { dd[w] = c; if (ex[w] < 0) { if (c < Dd) Dd = c; } else { nfr[w] = 1; if (c == L) any = 1; } }
                        }
                    }
                    for (int64_t v = 0; v < n; ++v) if (nfr[v]) fr[v] = 1;
                }
                ++levels;
                if (Dd <= L) break;
                /* next level: least tentative distance among unexpanded nodes */
                int64_t nl = INF; for (int64_t v = 0; v < n; ++v) if (fr[v] && dd[v] < nl) nl = dd[v];
                if (nl == INF || nl > Dd) break;
                L = nl; ++rounds;
            }
            printf("   dial: levels %d rounds %d relax %lld D %lld\n", levels, rounds, (long long)relax, (long long)Dd);
            dial_rounds += rounds; dial_relax += relax;
        }
        /* forward Dijkstra from the excess nodes */
        hn = 0; for (int64_t v = 0; v < n; ++v) { d[v] = INF; par[v] = -1; done[v] = 0; }
        for (int64_t v = 0; v < n; ++v) if (ex[v] > 0) { d[v] = 0; hpush(0, (int)v); }
        while (hn) {
            int64_t k; int u; hpop(&k, &u); if (done[u] || k != d[u]) continue; done[u] = 1; ++explored;
            if (k >= D) break;
            if (ex[u] < 0) { if (k < D) D = k; continue; }
            for (int a = b0[u]; a < b1[u]; ++a) {
                if (pos[a].rcap <= 0) continue; const int w = pos[a].head;
                int64_t len = fdiv(pos[a].cost + p[u] - p[w], eps) + 1; if (len < 0) len = 0;
                if (k + len < d[w]) { d[w] = k + len; par[w] = a; hpush(d[w], w); }
            }
        }
        explored_tot += explored;
        if (D == INF) { printf("no deficit reachable\n"); break; }
        for (int64_t v = 0; v < n; ++v) if (d[v] < D) p[v] -= eps * (D - d[v]);
        for (int64_t t = 0; t < n; ++t) {
            if (ex[t] >= 0 || d[t] != D) continue;
            int plen = 0, v = (int)t, ok = 1;
            while (!(d[v] == 0 && ex[v] > 0)) { const int a = par[v]; if (a < 0 || plen >= 100000) { ok = 0; break; } path[plen++] = a; v = tail[a]; }
            if (!ok || ex[v] <= 0) continue;
            for (int i = 0; i < plen; ++i) if (pos[path[i]].rcap < 1) ok = 0;
            if (!ok) continue;
            for (int i = 0; i < plen; ++i) { pos[path[i]].rcap -= 1; pos[pos[path[i]].rev].rcap += 1; }
            ex[v] -= 1; ex[t] += 1; ++moved;
        }
        printf("update %d: excess nodes %lld (%lld units), D %lld, explored %lld, moved %lld\n", updates + 1, (long long)nx, (long long)ux, (long long)D, (long long)explored, (long long)moved);
        (void)ksrc;
    }
    printf("dial total rounds %d relax %lld\n", dial_rounds, (long long)dial_relax);
    printf("backward %d, forward %d; forward SSP: %d updates, explored %lld nodes in total\n", nback, nfwd, updates, (long long)explored_tot);
    (void)0;
    return 0;
}
