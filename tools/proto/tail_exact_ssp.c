/* exact SSP finish on the device's tail state: (1) Bellman-Ford on the residual graph with
   scaled reduced costs from a virtual source (no negative cycle <=> the pseudoflow is optimal
   for its own supplies); (2) primal-dual: Dijkstra (unscaled integer lengths, potentials),
   D = nearest deficit, then a max flow over the tight arcs from every excess node to the
   deficits at distance D; repeat. Counts iterations and units per iteration. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef struct { long long cost, rcap, ucap; int head, rev; } Pos;
#define INF ((int64_t)0x3fffffffffffffffLL)
static int64_t* hk; static int* hv; static int hn;
static void hpush(int64_t k, int v) { int i = hn++; while (i) { int p = (i - 1) / 2; if (hk[p] <= k) break; hk[i] = hk[p]; hv[i] = hv[p]; i = p; } hk[i] = k; hv[i] = v; }
static void hpop(int64_t* k, int* v) { *k = hk[0]; *v = hv[0]; int64_t lk = hk[--hn]; int lv = hv[hn]; int i = 0; for (;;) { int c = 2 * i + 1; if (c >= hn) break; if (c + 1 < hn && hk[c + 1] < hk[c]) ++c; if (hk[c] >= lk) break; hk[i] = hk[c]; hv[i] = hv[c]; i = c; } hk[i] = lk; hv[i] = lv; }
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb"); long long hdr[6]; if (!f || fread(hdr, 8, 6, f) != 6) return 2;
    const int64_t n = hdr[0], np = hdr[2], mult = hdr[4];
    int* first = malloc(4 * (n + 1)); int64_t* nd = malloc(32 * n); int64_t* ex = malloc(8 * n); Pos* pos = malloc(sizeof(Pos) * np);
    if (fread(first, 4, n + 1, f) != (size_t)(n + 1) || fread(nd, 8, 4 * n, f) != (size_t)(4 * n) || fread(ex, 8, n, f) != (size_t)n || fread(pos, sizeof(Pos), np, f) != (size_t)np) return 2;
    int64_t* p = malloc(8 * n); int* b0 = malloc(4 * n); int* b1 = malloc(4 * n);
    for (int64_t v = 0; v < n; ++v) { p[v] = nd[4 * v]; uint64_t w = (uint64_t)nd[4 * v + 3]; b0[v] = (int)(w & 0xffffffffu); b1[v] = (int)(w >> 32); }
    int* tail = malloc(4 * np); for (int64_t v = 0; v < n; ++v) for (int a = b0[v]; a < b1[v]; ++a) tail[a] = (int)v;
    int64_t bad = 0; for (int64_t a = 0; a < np; ++a) if (pos[a].rcap > 0 && pos[a].cost % mult) ++bad;
    printf("positions with a cost not a multiple of mult: %lld\n", (long long)bad);
    /* (1) BF from a virtual source on unscaled costs: pi <= 0 potentials, SPFA with a pass limit */
    int64_t* pi = calloc(n, 8); int* q = malloc(4 * n); char* inq = malloc(n); int* cnt = calloc(n, 4);
    int qh = 0, qt = 0, qn = 0, negcyc = 0;
    for (int64_t v = 0; v < n; ++v) { q[qt++] = (int)v; inq[v] = 1; ++qn; } qt %= n;
    while (qn && !negcyc) {
        const int u = q[qh++]; if (qh == n) qh = 0; --qn; inq[u] = 0;
        for (int a = b0[u]; a < b1[u]; ++a) {
            if (pos[a].rcap <= 0) continue; const int w = pos[a].head;
            const int64_t c = pos[a].cost / mult;
            if (pi[u] + c < pi[w]) { pi[w] = pi[u] + c; if (++cnt[w] > n) { negcyc = 1; break; } if (!inq[w]) { inq[w] = 1; q[qt++] = w; if (qt == n) qt = 0; ++qn; } }
        }
    }
    printf("negative cycle in the residual graph (unscaled costs): %s\n", negcyc ? "YES" : "no");
    if (negcyc) return 0;
    /* (2) primal-dual with potentials pi (reduced c + pi[u] - pi[w] >= 0) */
    int64_t* d = malloc(8 * n); char* done = malloc(n); int* stk = malloc(4 * n); int* it = malloc(4 * n); char* vis = malloc(n);
    hk = malloc(8 * (np + n)); hv = malloc(4 * (np + n));
    int iters = 0;
    for (;;) {
        int64_t ux = 0; for (int64_t v = 0; v < n; ++v) if (ex[v] > 0) ux += ex[v];
        if (!ux) break;
        hn = 0; for (int64_t v = 0; v < n; ++v) { d[v] = INF; done[v] = 0; }
        for (int64_t v = 0; v < n; ++v) if (ex[v] > 0) { d[v] = 0; hpush(0, (int)v); }
        int64_t D = INF, explored = 0;
        while (hn) {
            int64_t k; int u; hpop(&k, &u); if (done[u] || k != d[u]) continue; done[u] = 1; ++explored;
            if (k > D) break;
            if (ex[u] < 0) { if (k < D) D = k; continue; }
            for (int a = b0[u]; a < b1[u]; ++a) {
                if (pos[a].rcap <= 0) continue; const int w = pos[a].head;
                const int64_t rc = pos[a].cost / mult + pi[u] - pi[w];
                if (rc < 0) { printf("negative reduced cost!\n"); return 1; }
                if (k + rc < d[w]) { d[w] = k + rc; hpush(d[w], w); }
            }
        }
        if (D == INF) { printf("no deficit reachable\n"); break; }
        for (int64_t v = 0; v < n; ++v) pi[v] += (d[v] < D ? d[v] : D);
        /* max flow over tight arcs (reduced cost 0) from excess nodes to deficits: DFS augmenting paths */
        int64_t moved = 0;
        for (int64_t s = 0; s < n; ++s) {
            while (ex[s] > 0) {
                memset(vis, 0, n);
                int sp = 0; stk[sp] = (int)s; it[sp] = b0[s]; vis[s] = 1; int found = -1;
                while (sp >= 0) {
                    const int u = stk[sp];
                    if (u != s && ex[u] < 0) { found = u; break; }
                    int advanced = 0;
                    while (it[sp] < b1[u]) {
                        const int a = it[sp]++;
                        if (pos[a].rcap <= 0) continue; const int w = pos[a].head;
                        if (vis[w]) continue;
                        if (pos[a].cost / mult + pi[u] - pi[w] != 0) continue;
                        vis[w] = 1; stk[++sp] = w; it[sp] = b0[w]; advanced = 1; break;
                    }
                    if (!advanced) --sp;
                }
                if (found < 0) break;
                /* path: stack nodes; arcs = it[k]-1 at each level */
                for (int k = 0; k < sp; ++k) { const int a = it[k] - 1; pos[a].rcap -= 1; pos[pos[a].rev].rcap += 1; }
                ex[s] -= 1; ex[found] += 1; ++moved;
            }
        }
        ++iters;
        printf("iteration %d: units left %lld, D %lld, explored %lld, moved %lld\n", iters, (long long)ux, (long long)D, (long long)explored, (long long)moved);
        if (!moved) break;
    }
    printf("exact SSP: %d iterations\n", iters);
    return 0;
}
