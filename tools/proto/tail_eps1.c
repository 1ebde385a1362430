/* Design diagnostic (CPU, not part of the product or the oracle): reads the
 * residual state a -DKS_DUMP engine build writes at the first tail cycle of a
 * final phase (ks_engine.hip, KS_DUMP=<path>), recomputes the global update
 * (exact Bellman-Ford from the deficits, lengths floor(rc/ε)+1, p −= ε·min(d, L))
 * and runs sequential unit blocking flows under the device walkers' rules, to
 * tell the rules' reach apart from the device's concurrency:
 *   HUBS=0  walkers may pass every hub
 *   HUBS=1  hubs without excess are dead ends (the device's list-less hubs)
 *   SLACK=s the walk rule's slack (rc ≤ s·ε toward strictly smaller d)
 * Repeats update + blocking flow until no excess is left (or 200 updates).
 * Build: gcc -O2 -o /tmp/tail_dump tools/proto/tail_dump.c */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { long long cost, rcap, ucap; int head, rev; } Pos;
#define INF ((int64_t)0x3fffffffffffffffLL)

static int64_t fdiv(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b) && (a < 0)) --q; return q; }

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: tail_dump <dump>\n"); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror("open"); return 2; }
    long long hdr[6];
    if (fread(hdr, 8, 6, f) != 6) return 2;
    const int64_t n = hdr[0], hub_base = hdr[1], np = hdr[2], eps = hdr[3], mult = hdr[4];
    int* first = malloc(4 * (n + 1));
    int64_t* nd = malloc(32 * n);
    int64_t* ex = malloc(8 * n);
    Pos* pos = malloc(sizeof(Pos) * np);
    if (fread(first, 4, n + 1, f) != (size_t)(n + 1) || fread(nd, 8, 4 * n, f) != (size_t)(4 * n) ||
        fread(ex, 8, n, f) != (size_t)n || fread(pos, sizeof(Pos), np, f) != (size_t)np) { fprintf(stderr, "short dump\n"); return 2; }
    fclose(f);
    const int hubs_rule = getenv("HUBS") ? atoi(getenv("HUBS")) : 1;
    const int slack = getenv("SLACK") ? atoi(getenv("SLACK")) : 1;
    int64_t* p = malloc(8 * n);
    int* b0 = malloc(4 * n); int* b1 = malloc(4 * n);
    for (int64_t v = 0; v < n; ++v) {
        p[v] = nd[4 * v];
        const uint64_t w = (uint64_t)nd[4 * v + 3];
        b0[v] = (int)(w & 0xffffffffu); b1[v] = (int)(w >> 32);
    }
    int* tail = malloc(4 * np);
    for (int64_t v = 0; v < n; ++v) for (int a = b0[v]; a < b1[v]; ++a) tail[a] = (int)v;
    int64_t sx = 0, sd = 0, nx = 0, ndf = 0;
    for (int64_t v = 0; v < n; ++v) { if (ex[v] > 0) { sx += ex[v]; ++nx; } if (ex[v] < 0) { sd -= ex[v]; ++ndf; } }
    printf("n %lld hubs %lld positions %lld eps %lld mult %lld: excess %lld units at %lld nodes, deficit %lld at %lld\n",
           (long long)n, (long long)(n - hub_base), (long long)np, (long long)eps, (long long)mult, (long long)sx,
           (long long)nx, (long long)sd, (long long)ndf);
    int64_t viol = 0;
    for (int64_t v = 0; v < n; ++v)
        for (int a = b0[v]; a < b1[v]; ++a)
            if (pos[a].rcap > 0 && pos[a].cost + p[v] - p[pos[a].head] < -eps) ++viol;
    printf("arcs violating eps-optimality: %lld\n", (long long)viol);
    int64_t eps_run = eps;
    if (getenv("EPS1")) {
        /* price refinement at eps = 1 on the pseudoflow: SPFA from d = 0, lengths floor(rc/1)+1 = rc+1 */
        int64_t* dd = calloc(n, 8); int* qq = malloc(4 * n); char* iq = malloc(n); int* cn = calloc(n, 4);
        int qh = 0, qt = 0, qn = 0, neg = 0;
        for (int64_t v = 0; v < n; ++v) { qq[qt++] = (int)v; iq[v] = 1; ++qn; } qt %= n;
        while (qn && !neg) {
            const int w = qq[qh++]; if (qh == n) qh = 0; --qn; iq[w] = 0;
            /* relax in-arcs u -> w: d(u) <= len(u,w) + d(w) */
            for (int a = b0[w]; a < b1[w]; ++a) {
                const int ra = pos[a].rev; if (pos[ra].rcap <= 0) continue; const int u = pos[a].head;
                const int64_t len = pos[ra].cost + p[u] - p[w] + 1;
                if (dd[w] + len < dd[u]) { dd[u] = dd[w] + len; if (++cn[u] > n) { neg = 1; break; } if (!iq[u]) { iq[u] = 1; qq[qt++] = u; if (qt == n) qt = 0; ++qn; } }
            }
        }
        printf("price refinement at eps 1: %s\n", neg ? "FAILED (negative cycle)" : "converged");
        if (neg) return 0;
        for (int64_t v = 0; v < n; ++v) p[v] -= dd[v];
        int64_t viol1 = 0;
        for (int64_t v = 0; v < n; ++v) for (int a = b0[v]; a < b1[v]; ++a) if (pos[a].rcap > 0 && pos[a].cost + p[v] - p[pos[a].head] < -1) ++viol1;
        printf("arcs violating 1-optimality after refinement: %lld\n", (long long)viol1);
        eps_run = 1;
    }
    int64_t* d = malloc(8 * n);
    int* q = malloc(4 * n); char* inq = calloc(n, 1); char* dead = calloc(n, 1);
    int* path = malloc(4 * 65536);
    int64_t moved_total = 0;
    for (int gu = 1; gu <= 200; ++gu) {
        int64_t nxl = 0, exl = 0;
        for (int64_t v = 0; v < n; ++v) if (ex[v] > 0) { ++nxl; exl += ex[v]; }
        if (!nxl) { printf("done after %d updates\n", gu - 1); break; }
        /* exact distances to the deficits (SPFA over residual arcs, reversed) */
        int qh = 0, qt = 0, qn = 0;
        for (int64_t v = 0; v < n; ++v) { d[v] = ex[v] < 0 ? 0 : INF; inq[v] = 0; if (ex[v] < 0) { q[qt++] = (int)v; inq[v] = 1; ++qn; } }
        if (qt == n) qt = 0;
        while (qn) {
            const int w = q[qh++]; if (qh == n) qh = 0; --qn; inq[w] = 0;
            for (int a = b0[w]; a < b1[w]; ++a) {
                const int ra = pos[a].rev;   /* arc u -> w */
                if (pos[ra].rcap <= 0) continue;
                const int u = pos[a].head;
                int64_t len = fdiv(pos[ra].cost + p[u] - p[w], eps_run) + 1;
                if (len < 0) len = 0;
                const int64_t nd2 = d[w] + len;
                if (nd2 < d[u]) { d[u] = nd2; if (!inq[u]) { inq[u] = 1; q[qt++] = u; if (qt == n) qt = 0; ++qn; } }
            }
        }
        int64_t L = 0;
        for (int64_t v = 0; v < n; ++v) if (d[v] < INF && d[v] > L) L = d[v];
        for (int64_t v = 0; v < n; ++v) p[v] -= eps_run * (d[v] < L ? d[v] : L);
        if (gu == 1) {
            int shown = 0;
            for (int64_t v = 0; v < n && shown < 12; ++v)
                if (ex[v] > 0) { printf("  excess x%lld%s e %lld d %lld deg %d\n", (long long)v, v >= hub_base ? " (hub)" : "", (long long)ex[v], (long long)d[v], b1[v] - b0[v]); ++shown; }
            shown = 0;
            for (int64_t v = 0; v < n && shown < 12; ++v)
                if (ex[v] < 0) { printf("  deficit x%lld%s e %lld deg %d\n", (long long)v, v >= hub_base ? " (hub)" : "", (long long)ex[v], b1[v] - b0[v]); ++shown; }
        }
        /* unit blocking flow, sources in id order */
        memset(dead, 0, n);
        int64_t moved = 0, steps_run_tot = 0, plen_max = 0, hub_pass = 0;
        for (int64_t s0 = 0; s0 < n; ++s0) {
            if (hubs_rule && s0 >= hub_base) continue;   /* (hub sources: device lists; skipped here) */
            while (ex[s0] > 0) {
                int u = (int)s0, plen = 0, found = -1;
                for (int steps_run = 0; steps_run < 1000000; ++steps_run) {
                    ++steps_run_tot;
                    if (u != s0 && ex[u] < 0) { found = u; break; }
                    if (u != s0 && hubs_rule && u >= hub_base && ex[u] <= 0) {   /* list-less hub */
                        dead[u] = 1;
                        u = tail[path[--plen]];
                        continue;
                    }
                    int best = -1; int64_t bd = INF;
                    for (int a = b0[u]; a < b1[u]; ++a) {
                        if (pos[a].rcap <= 0) continue;
                        const int w = pos[a].head;
                        if (w == u || dead[w]) continue;
                        const int64_t rc = pos[a].cost + p[u] - p[w];
                        const int down = d[w] < d[u] || d[u] >= L;
                        const int ok = (rc < 0 && (d[w] <= d[u] || d[u] >= L)) || (rc <= slack * eps_run && down);
                        if (ok && d[w] < bd) { bd = d[w]; best = a; }
                    }
                    if (best < 0 || plen >= 65536) {
                        dead[u] = 1;
                        if (!plen) break;
                        u = tail[path[--plen]];
                        continue;
                    }
                    path[plen++] = best;
                    u = pos[best].head;
                }
                if (found < 0) break;
                for (int i = 0; i < plen; ++i) {
                    pos[path[i]].rcap -= 1; pos[pos[path[i]].rev].rcap += 1;
                    if (pos[path[i]].head >= hub_base && pos[path[i]].head != found) ++hub_pass;
                }
                ex[s0] -= 1; ex[found] += 1; ++moved;
                if (plen > plen_max) plen_max = plen;
            }
        }
        moved_total += moved;
        printf("update %d: excess nodes %lld (%lld units), L %lld, moved %lld, steps_run %lld, longest path %lld, hub passes %lld\n",
               gu, (long long)nxl, (long long)exl, (long long)L, (long long)moved, (long long)steps_run_tot,
               (long long)plen_max, (long long)hub_pass);
        if (!moved) {
            int64_t hx = 0;
            for (int64_t v = hub_base; v < n; ++v) if (ex[v] > 0) hx += ex[v];
            printf("no progress (%lld units at hubs)\n", (long long)hx);
            break;
        }
    }
    printf("moved %lld units in total\n", (long long)moved_total);
    return 0;
}
