/*
 * ks_oracle.c — CPU restatement of the ksched placement hot path.
 * TEST INFRASTRUCTURE ONLY (see ks_oracle.h): never linked into ksched_amd.
 *
 * Reference citations are relative to the ksched tree (github.com/coreos/ksched
 * layout, mounted read-only as /root/reference in the build container).
 */
#include "ks_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define KO_INF ((int64_t)0x3fffffffffffffffLL)

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* ------------------------------------------------------------------------- */
/* splitmix64 counter stream: x_i = mix(seed + (i+1)·γ)          */
/* ------------------------------------------------------------------------- */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint64_t xs(uint64_t seed, uint64_t i) {
    return mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ULL);
}
static inline int64_t uab(int64_t a, int64_t b, uint64_t x) {
    return a + (int64_t)(x % (uint64_t)(b - a + 1));
}

void ko_quincy_sizes(int64_t T, int64_t M, int64_t R, int64_t J, int64_t* n, int64_t* m) {
    *n = T + J + R + 2 * M + 2;
    *m = 5 * T + R + 3 * M + J;
}

/* Quincy-shaped cell graph. Node ids: sink 1, cluster aggregator X 2,
 * racks 3.., machines, PUs (one per machine, as the fake topology of
 * cmd/k8sscheduler/scheduler.go:332-350), unscheduled aggregators U_j, tasks. */
int ko_gen_quincy(int64_t T, int64_t M, int64_t R, int64_t J, uint64_t seed, ko_graph* g) {
    if (T < 1 || M < 2 || R < 1 || J < 1 || R > M) return -1;
    const int64_t SINK = 1, X = 2, RACK0 = 3, MACH0 = RACK0 + R, PU0 = MACH0 + M,
                  U0 = PU0 + M, TASK0 = U0 + J;
    int64_t n, m;
    ko_quincy_sizes(T, M, R, J, &n, &m);
    g->n = n;
    g->m = m;
    for (int64_t v = 0; v < n; ++v) { g->supply[v] = 0; g->ntype[v] = 0; }
    g->ntype[SINK - 1] = 3;
    for (int64_t k = 0; k < M; ++k) { g->ntype[MACH0 + k - 1] = 4; g->ntype[PU0 + k - 1] = 2; }
    for (int64_t t = 0; t < T; ++t) { g->ntype[TASK0 + t - 1] = 1; g->supply[TASK0 + t - 1] = 1; }
    g->supply[SINK - 1] = -T;

    int64_t* slots = (int64_t*)malloc(sizeof(int64_t) * M);
    int64_t* rackslots = (int64_t*)calloc(R, sizeof(int64_t));
    int64_t* jobtasks = (int64_t*)calloc(J, sizeof(int64_t));
    for (int64_t k = 0; k < M; ++k) {
        slots[k] = uab(8, 12, xs(seed, k));
        rackslots[k % R] += slots[k];
    }
    int64_t a = 0;
#define ARC(s_, d_, lo_, ca_, co_) do { g->src[a] = (s_); g->dst[a] = (d_); g->low[a] = (lo_); \
        g->cap[a] = (ca_); g->cost[a] = (co_); ++a; } while (0)
    for (int64_t t = 0; t < T; ++t) {
        const uint64_t b = (uint64_t)M + 9 * (uint64_t)t;
        const int64_t j = (int64_t)(xs(seed, b + 0) % (uint64_t)J);
        const int64_t cU = uab(200, 1000, xs(seed, b + 1));
        const int64_t cX = uab(100, 400, xs(seed, b + 2));
        const int64_t rk = (int64_t)(xs(seed, b + 3) % (uint64_t)R);
        const int64_t cR = uab(20, 200, xs(seed, b + 4));
        const int64_t m1 = (int64_t)(xs(seed, b + 5) % (uint64_t)M);
        const int64_t m2 = (m1 + 1 + (int64_t)(xs(seed, b + 6) % (uint64_t)(M - 1))) % M;
        const int64_t c1 = uab(0, 100, xs(seed, b + 7));
        const int64_t c2 = uab(0, 100, xs(seed, b + 8));
        const int64_t tid = TASK0 + t;
        jobtasks[j] += 1;
        ARC(tid, U0 + j, 0, 1, cU);
        ARC(tid, X, 0, 1, cX);
        ARC(tid, RACK0 + rk, 0, 1, cR);
        ARC(tid, MACH0 + m1, 0, 1, c1);
        ARC(tid, MACH0 + m2, 0, 1, c2);
    }
    for (int64_t r = 0; r < R; ++r) ARC(X, RACK0 + r, 0, rackslots[r], 0);
    for (int64_t k = 0; k < M; ++k) ARC(RACK0 + (k % R), MACH0 + k, 0, slots[k], 0);
    for (int64_t k = 0; k < M; ++k) ARC(MACH0 + k, PU0 + k, 0, slots[k], 0);
    for (int64_t k = 0; k < M; ++k) ARC(PU0 + k, SINK, 0, slots[k], 0);
    for (int64_t j = 0; j < J; ++j) ARC(U0 + j, SINK, 0, jobtasks[j], 0);
#undef ARC
    free(slots); free(rackslots); free(jobtasks);
    return a == m ? 0 : -2;
}

void ko_trivial_sizes(int64_t machines, int64_t pods, int64_t* n, int64_t* m) {
    *n = 2 + 2 * machines + 2 + pods;
    *m = 4 * machines + 2 * pods + 1;
}

/* ksched's own topology (config 1): `k8sscheduler -fakeMachines -nm N -mt MT`
 * with P pods in one job, trivial cost model. Arc families and costs:
 * PU→sink (0,mt,0) graph_manager.go:1116-1129; machine→PU (0,mt,0) :624;
 * coordinator→machine (0,0,0) (NumSlotsBelow is 0 when the arc is created, :597-604);
 * EC→machine (0,free slots,0) :974-1010 + trivial_cost_modeler.go:76-83;
 * task→U (0,1,5) :1270-1285 + trivial :41-43; task→EC (0,1,2) :1197-1226 + trivial :69-74;
 * U→sink (0,#tasks,0) :1291-1305. Supplies: tasks +1, sink −P (:636-640). */
int ko_gen_trivial(int64_t machines, int64_t mt, int64_t pods, ko_graph* g) {
    int64_t n, m;
    ko_trivial_sizes(machines, pods, &n, &m);
    g->n = n;
    g->m = m;
    const int64_t SINK = 1, COORD = 2, U = 3 + 2 * machines, EC = U + 1, TASK0 = EC + 1;
    for (int64_t v = 0; v < n; ++v) { g->supply[v] = 0; g->ntype[v] = 0; }
    g->ntype[SINK - 1] = 3;
    g->supply[SINK - 1] = -pods;
    int64_t a = 0;
#define ARC(s_, d_, lo_, ca_, co_) do { g->src[a] = (s_); g->dst[a] = (d_); g->low[a] = (lo_); \
        g->cap[a] = (ca_); g->cost[a] = (co_); ++a; } while (0)
    for (int64_t k = 0; k < machines; ++k) {
        const int64_t mach = 3 + 2 * k, pu = mach + 1;
        g->ntype[mach - 1] = 4;
        g->ntype[pu - 1] = 2;
        ARC(pu, SINK, 0, mt, 0);
        ARC(mach, pu, 0, mt, 0);
        ARC(COORD, mach, 0, 0, 0);
    }
    ARC(U, SINK, 0, pods, 0);
    for (int64_t t = 0; t < pods; ++t) {
        const int64_t tid = TASK0 + t;
        g->ntype[tid - 1] = 1;
        g->supply[tid - 1] = 1;
        ARC(tid, U, 0, 1, 5);
        ARC(tid, EC, 0, 1, 2);
    }
    for (int64_t k = 0; k < machines; ++k) ARC(EC, 3 + 2 * k, 0, mt, 0);
#undef ARC
    return a == m ? 0 : -2;
}

/* ------------------------------------------------------------------------- */
/* residual graph (CSR by tail; lower bounds transformed away)                 */
/* ------------------------------------------------------------------------- */
typedef struct {
    int64_t n, m;
    int64_t* first;   /* n+1 */
    int64_t* head;    /* 2m  */
    int64_t* rcap;
    int64_t* cost;
    int64_t* rev;
    int64_t* fwd;     /* m: CSR slot of input arc i */
    int64_t* excess;  /* n  */
    int64_t  pos_supply;
} res_t;

static void res_free(res_t* r) {
    free(r->first); free(r->head); free(r->rcap); free(r->cost);
    free(r->rev); free(r->fwd); free(r->excess);
}

static int res_build(const ko_graph* g, res_t* r) {
    const int64_t n = g->n, m = g->m;
    memset(r, 0, sizeof(*r));
    r->n = n;
    r->m = m;
    r->first = (int64_t*)calloc(n + 1, sizeof(int64_t));
    r->head = (int64_t*)malloc(sizeof(int64_t) * (2 * m + 1));
    r->rcap = (int64_t*)malloc(sizeof(int64_t) * (2 * m + 1));
    r->cost = (int64_t*)malloc(sizeof(int64_t) * (2 * m + 1));
    r->rev = (int64_t*)malloc(sizeof(int64_t) * (2 * m + 1));
    r->fwd = (int64_t*)malloc(sizeof(int64_t) * (m + 1));
    r->excess = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    for (int64_t v = 0; v < n; ++v) {
        r->excess[v] = g->supply[v];
        if (g->supply[v] > 0) r->pos_supply += g->supply[v];
    }
    for (int64_t i = 0; i < m; ++i) {
        const int64_t s = g->src[i] - 1, d = g->dst[i] - 1;
        if (s < 0 || s >= n || d < 0 || d >= n || g->low[i] < 0 || g->low[i] > g->cap[i]) {
            res_free(r);
            return -1;
        }
        r->first[s + 1]++;
        r->first[d + 1]++;
    }
    for (int64_t v = 0; v < n; ++v) r->first[v + 1] += r->first[v];
    int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    memcpy(pos, r->first, sizeof(int64_t) * (n + 1));
    for (int64_t i = 0; i < m; ++i) {
        const int64_t s = g->src[i] - 1, d = g->dst[i] - 1;
        const int64_t pf = pos[s]++, pr = pos[d]++;
        r->head[pf] = d; r->rcap[pf] = g->cap[i] - g->low[i]; r->cost[pf] = g->cost[i]; r->rev[pf] = pr;
        r->head[pr] = s; r->rcap[pr] = 0; r->cost[pr] = -g->cost[i]; r->rev[pr] = pf;
        r->fwd[i] = pf;
        r->excess[s] -= g->low[i];   /* lower-bound transform */
        r->excess[d] += g->low[i];
    }
    free(pos);
    return 0;
}

static void res_flows(const ko_graph* g, const res_t* r, int64_t* flow_out) {
    for (int64_t i = 0; i < g->m; ++i)
        flow_out[i] = g->low[i] + (g->cap[i] - g->low[i]) - r->rcap[r->fwd[i]];
}

/* ------------------------------------------------------------------------- */
/* binary heap of (key, node)                                                   */
/* ------------------------------------------------------------------------- */
typedef struct { int64_t* k; int64_t* v; int64_t size, cap; } heap_t;
static void hp_init(heap_t* h, int64_t cap) {
    h->k = (int64_t*)malloc(sizeof(int64_t) * cap);
    h->v = (int64_t*)malloc(sizeof(int64_t) * cap);
    h->size = 0;
    h->cap = cap;
}
static void hp_free(heap_t* h) { free(h->k); free(h->v); }
static void hp_push(heap_t* h, int64_t key, int64_t val) {
    if (h->size == h->cap) {
        h->cap *= 2;
        h->k = (int64_t*)realloc(h->k, sizeof(int64_t) * h->cap);
        h->v = (int64_t*)realloc(h->v, sizeof(int64_t) * h->cap);
    }
    int64_t i = h->size++;
    while (i > 0) {
        int64_t p = (i - 1) >> 1;
        if (h->k[p] <= key) break;
        h->k[i] = h->k[p]; h->v[i] = h->v[p]; i = p;
    }
    h->k[i] = key; h->v[i] = val;
}
static void hp_pop(heap_t* h, int64_t* key, int64_t* val) {
    *key = h->k[0]; *val = h->v[0];
    const int64_t lk = h->k[--h->size], lv = h->v[h->size];
    int64_t i = 0;
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= h->size) break;
        if (c + 1 < h->size && h->k[c + 1] < h->k[c]) ++c;
        if (h->k[c] >= lk) break;
        h->k[i] = h->k[c]; h->v[i] = h->v[c]; i = c;
    }
    h->k[i] = lk; h->v[i] = lv;
}

/* ------------------------------------------------------------------------- */
/* successive shortest path (Flowlessly's configured algorithm, solver.go:32)  */
/* reduced cost rc(u,v) = c + pot[u] − pot[v] ≥ 0 on residual arcs            */
/* ------------------------------------------------------------------------- */

/* Augment every excess node's supply along shortest paths (Dijkstra with the
 * potentials, stopped at the first deficit settled). Requires rc ≥ 0 on every
 * residual arc; keeps it (pot[v] += dist[v] − D for settled v). Returns the
 * number of augmentations. */
static int64_t ssp_augment_all(res_t* rp, int64_t* pot) {
    res_t r = *rp;
    const int64_t n = r.n;
    int64_t* dist = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t* pred = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    char* done = (char*)calloc(n + 1, 1);
    int64_t* touched = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    for (int64_t v = 0; v < n; ++v) dist[v] = KO_INF;
    heap_t h;
    hp_init(&h, 1024);
    int64_t naug = 0;
    int progress = 1;
    while (progress) {
        progress = 0;
        for (int64_t s = 0; s < n; ++s) {
            while (r.excess[s] > 0) {
                /* Dijkstra from s until the first deficit node is settled */
                int64_t ntouch = 0, t = -1, D = 0;
                h.size = 0;
                dist[s] = 0; pred[s] = -1; touched[ntouch++] = s;
                hp_push(&h, 0, s);
                while (h.size > 0) {
                    int64_t du, u;
                    hp_pop(&h, &du, &u);
                    if (done[u] || du != dist[u]) continue;
                    done[u] = 1;
                    if (r.excess[u] < 0) { t = u; D = du; break; }
                    for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a) {
                        if (r.rcap[a] <= 0) continue;
                        const int64_t v = r.head[a];
                        if (done[v]) continue;
                        const int64_t nd = du + r.cost[a] + pot[u] - pot[v];
                        if (nd < dist[v]) {
                            if (dist[v] == KO_INF) touched[ntouch++] = v;
                            dist[v] = nd; pred[v] = a;
                            hp_push(&h, nd, v);
                        }
                    }
                }
                if (t >= 0) {
                    for (int64_t i = 0; i < ntouch; ++i) {
                        const int64_t v = touched[i];
                        if (done[v]) pot[v] += dist[v] - D;
                    }
                    /* bottleneck along the path t ← … ← s */
                    int64_t delta = r.excess[s] < -r.excess[t] ? r.excess[s] : -r.excess[t];
                    for (int64_t v = t; v != s;) {
                        const int64_t a = pred[v];
                        if (r.rcap[a] < delta) delta = r.rcap[a];
                        v = r.head[r.rev[a]];
                    }
                    for (int64_t v = t; v != s;) {
                        const int64_t a = pred[v];
                        r.rcap[a] -= delta; r.rcap[r.rev[a]] += delta;
                        v = r.head[r.rev[a]];
                    }
                    r.excess[s] -= delta; r.excess[t] += delta;
                    ++naug;
                    progress = 1;
                }
                for (int64_t i = 0; i < ntouch; ++i) { dist[touched[i]] = KO_INF; done[touched[i]] = 0; }
                if (t < 0) break;   /* s cannot reach a deficit now */
            }
        }
    }
    hp_free(&h);
    free(dist); free(pred); free(done); free(touched);
    return naug;
}

int ko_ssp(const ko_graph* g, int64_t* flow_out, int64_t* total_cost, int64_t* flow_value,
           int64_t* augmentations) {
    res_t r;
    if (res_build(g, &r)) return -1;
    const int64_t n = r.n;
    int64_t* pot = (int64_t*)calloc(n + 1, sizeof(int64_t));

    /* initial potentials: Bellman-Ford (SPFA) when a residual arc has negative cost */
    int neg = 0;
    for (int64_t a = 0; a < 2 * r.m; ++a) if (r.rcap[a] > 0 && r.cost[a] < 0) { neg = 1; break; }
    if (neg) {
        int64_t* q = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
        char* inq = (char*)malloc(n + 1);
        int64_t* cnt = (int64_t*)calloc(n + 1, sizeof(int64_t));
        int64_t qh = 0, qt = 0, qn = 0;
        for (int64_t v = 0; v < n; ++v) { pot[v] = 0; q[qt++] = v; inq[v] = 1; ++qn; }
        if (qt == n + 1) qt = 0;
        while (qn > 0) {
            const int64_t u = q[qh++]; if (qh == n + 1) qh = 0; --qn; inq[u] = 0;
            for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a) {
                if (r.rcap[a] <= 0) continue;
                const int64_t v = r.head[a];
                if (pot[u] + r.cost[a] < pot[v]) {
                    pot[v] = pot[u] + r.cost[a];
                    if (!inq[v]) {
                        if (++cnt[v] > n + 1) { /* negative cycle */
                            free(q); free(inq); free(cnt); free(pot); res_free(&r); return -3;
                        }
                        q[qt++] = v; if (qt == n + 1) qt = 0; ++qn; inq[v] = 1;
                    }
                }
            }
        }
        free(q); free(inq); free(cnt);
    }

    const int64_t naug = ssp_augment_all(&r, pot);

    int64_t left = 0;
    for (int64_t v = 0; v < n; ++v) if (r.excess[v] > 0) left += r.excess[v];
    res_flows(g, &r, flow_out);
    int64_t c = 0;
    for (int64_t i = 0; i < g->m; ++i) c += flow_out[i] * g->cost[i];
    *total_cost = c;
    *flow_value = r.pos_supply - left;
    if (augmentations) *augmentations = naug;
    free(pot);
    res_free(&r);
    return left > 0 ? 1 : 0;
}

/* ------------------------------------------------------------------------- */
/* incremental SSP: the daemon mode ksched runs Flowlessly in                   */
/* (solver.go:30-34 Incremental = true; later Solves send only the change     */
/* block, :86-89, and the solver re-solves from its previous state)            */
/* ------------------------------------------------------------------------- */
static inline uint64_t arc_key64(int64_t s, int64_t d) { return ((uint64_t)s << 32) | (uint64_t)d; }
static inline uint64_t key_hash(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33;
    return k;
}

/* The previous round's flow is carried by (src, dst) key onto the new graph
 * (clamped to the new bounds: a lowered capacity returns its surplus to the
 * endpoints, a deleted arc's flow leaves its endpoints unbalanced, a removed
 * node's arcs are gone), the previous potentials by node id (nodes created since
 * — fresh[v] = 1 — get the least potential under which none of their residual
 * out-arcs is negative). Every residual arc that the changes left with negative
 * reduced cost is then saturated, which restores rc ≥ 0 everywhere at the price
 * of more excess and deficit, and successive shortest paths route every excess
 * to a deficit from there. flow_out / pot_out: m / n entries for the next round.
 * ms[0] carry (hash the old arcs, seed the residual graph), ms[1] saturate,
 * ms[2] augment. */
int ko_ssp_incremental(const ko_graph* g, const int64_t* prev_src, const int64_t* prev_dst,
                       const int64_t* prev_flow, int64_t prev_m, const int64_t* prev_pot, int64_t prev_n,
                       const uint8_t* fresh, int64_t* flow_out, int64_t* pot_out, int64_t* total_cost,
                       int64_t* flow_value, int64_t* augmentations, double* ms) {
    const double t0 = now_ms();
    res_t r;
    if (res_build(g, &r)) return -1;
    const int64_t n = r.n, m = r.m;
    /* (src, dst) → previous flow */
    int64_t hcap = 16;
    while (hcap < 2 * prev_m + 2) hcap <<= 1;
    uint64_t* hk = (uint64_t*)calloc(hcap, sizeof(uint64_t));
    int64_t* hv = (int64_t*)malloc(sizeof(int64_t) * hcap);
    for (int64_t i = 0; i < prev_m; ++i) {
        if (prev_flow[i] <= 0) continue;
        const uint64_t k = arc_key64(prev_src[i], prev_dst[i]);
        uint64_t s = key_hash(k) & (uint64_t)(hcap - 1);
        while (hk[s] && hk[s] != k) s = (s + 1) & (uint64_t)(hcap - 1);
        hk[s] = k;
        hv[s] = prev_flow[i];
    }
    for (int64_t i = 0; i < m; ++i) {
        const uint64_t k = arc_key64(g->src[i], g->dst[i]);
        uint64_t s = key_hash(k) & (uint64_t)(hcap - 1);
        int64_t f = 0;
        while (hk[s]) {
            if (hk[s] == k) { f = hv[s]; break; }
            s = (s + 1) & (uint64_t)(hcap - 1);
        }
        if (f < g->low[i]) f = g->low[i];
        if (f > g->cap[i]) f = g->cap[i];
        const int64_t x = f - g->low[i];   /* residual-graph flow (lower bounds transformed) */
        if (x > 0) {
            const int64_t p = r.fwd[i];
            r.rcap[p] -= x;
            r.rcap[r.rev[p]] += x;
            r.excess[g->src[i] - 1] -= x;
            r.excess[g->dst[i] - 1] += x;
        }
    }
    free(hk); free(hv);
    int64_t* pot = (int64_t*)calloc(n + 1, sizeof(int64_t));
    for (int64_t v = 0; v < n && v < prev_n; ++v) pot[v] = prev_pot[v];
    for (int64_t v = 0; v < n; ++v) {
        if (v < prev_n && !(fresh && fresh[v])) continue;
        int64_t best = INT64_MIN;   /* rc(v, w) = c + pot[v] − pot[w] ≥ 0 ⇔ pot[v] ≥ pot[w] − c */
        for (int64_t a = r.first[v]; a < r.first[v + 1]; ++a)
            if (r.rcap[a] > 0 && pot[r.head[a]] - r.cost[a] > best) best = pot[r.head[a]] - r.cost[a];
        pot[v] = best == INT64_MIN ? 0 : best;
    }
    const double t1 = now_ms();
    for (int64_t u = 0; u < n; ++u)
        for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a) {
            if (r.rcap[a] <= 0) continue;
            const int64_t v = r.head[a];
            if (r.cost[a] + pot[u] - pot[v] < 0) {
                const int64_t d = r.rcap[a];
                r.rcap[a] = 0; r.rcap[r.rev[a]] += d;
                r.excess[u] -= d; r.excess[v] += d;
            }
        }
    const double t2 = now_ms();
    const int64_t naug = ssp_augment_all(&r, pot);
    const double t3 = now_ms();
    int64_t left = 0;
    for (int64_t v = 0; v < n; ++v) if (r.excess[v] > 0) left += r.excess[v];
    res_flows(g, &r, flow_out);
    int64_t c = 0;
    for (int64_t i = 0; i < g->m; ++i) c += flow_out[i] * g->cost[i];
    *total_cost = c;
    *flow_value = r.pos_supply - left;
    if (augmentations) *augmentations = naug;
    if (pot_out) memcpy(pot_out, pot, sizeof(int64_t) * n);
    if (ms) { ms[0] = t1 - t0; ms[1] = t2 - t1; ms[2] = t3 - t2; }
    free(pot);
    res_free(&r);
    return left > 0 ? 1 : 0;
}

/* ------------------------------------------------------------------------- */
/* Goldberg ε-scaling push-relabel (strong single-thread CPU baseline)         */
/* price convention: rc(u,v) = c'(u,v) + p[u] − p[v]; admissible iff rc < 0   */
/* ------------------------------------------------------------------------- */
static inline int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}

typedef struct {
    res_t* r;
    int64_t* p;
    int64_t* d;
    char* scanned;
    heap_t h;
} cs_t;

/* Dijkstra-based global price update from the deficit nodes over residual arcs,
 * arc length floor(rc/ε)+1. Returns −1 when an excess node cannot reach a deficit. */
static int cs_global_update(cs_t* c, int64_t eps) {
    res_t* r = c->r;
    const int64_t n = r->n;
    int64_t nexcess = 0;
    c->h.size = 0;
    for (int64_t v = 0; v < n; ++v) {
        c->scanned[v] = 0;
        if (r->excess[v] > 0) ++nexcess;
        if (r->excess[v] < 0) { c->d[v] = 0; hp_push(&c->h, 0, v); } else c->d[v] = KO_INF;
    }
    int64_t level = 0;
    while (c->h.size > 0 && nexcess > 0) {
        int64_t dv, v;
        hp_pop(&c->h, &dv, &v);
        if (c->scanned[v] || dv != c->d[v]) continue;
        c->scanned[v] = 1;
        level = dv;
        if (r->excess[v] > 0 && --nexcess == 0) break;
        for (int64_t a = r->first[v]; a < r->first[v + 1]; ++a) {
            const int64_t ra = r->rev[a];          /* arc (u, v) */
            if (r->rcap[ra] <= 0) continue;
            const int64_t u = r->head[a];
            if (c->scanned[u]) continue;
            const int64_t rc = r->cost[ra] + c->p[u] - c->p[v];
            const int64_t nd = dv + floordiv(rc, eps) + 1;
            if (nd < c->d[u]) { c->d[u] = nd; hp_push(&c->h, nd, u); }
        }
    }
    if (nexcess > 0) return -1;
    for (int64_t v = 0; v < n; ++v) {
        const int64_t dd = c->scanned[v] ? c->d[v] : level;
        c->p[v] -= eps * dd;
    }
    return 0;
}

int ko_cost_scaling(const ko_graph* g, int alpha, int64_t* flow_out, int64_t* total_cost,
                    int64_t* flow_value) {
    res_t r;
    if (res_build(g, &r)) return -1;
    const int64_t n = r.n;
    if (alpha < 2) alpha = 2;
    int64_t maxc = 0;
    for (int64_t i = 0; i < g->m; ++i) {
        const int64_t ac = g->cost[i] < 0 ? -g->cost[i] : g->cost[i];
        if (ac > maxc) maxc = ac;
    }
    const int64_t mult = n + 1;
    if (maxc > 0 && maxc > ((int64_t)1 << 62) / mult / (4 * (n + 1))) { res_free(&r); return -5; }
    for (int64_t a = 0; a < 2 * r.m; ++a) r.cost[a] *= mult;

    cs_t c;
    c.r = &r;
    c.p = (int64_t*)calloc(n + 1, sizeof(int64_t));
    c.d = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    c.scanned = (char*)malloc(n + 1);
    hp_init(&c.h, 1024);
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t* q = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    char* inq = (char*)calloc(n + 1, 1);
    int status = 0;

    int64_t eps = maxc * mult;
    if (eps < 1) eps = 1;
    for (;;) {
        eps = eps / alpha;
        if (eps < 1) eps = 1;
        /* refine: saturate every residual arc with negative reduced cost */
        for (int64_t u = 0; u < n; ++u)
            for (int64_t a = r.first[u]; a < r.first[u + 1]; ++a) {
                if (r.rcap[a] <= 0) continue;
                const int64_t v = r.head[a];
                if (r.cost[a] + c.p[u] - c.p[v] < 0) {
                    const int64_t dlt = r.rcap[a];
                    r.rcap[a] = 0; r.rcap[r.rev[a]] += dlt;
                    r.excess[u] -= dlt; r.excess[v] += dlt;
                }
            }
        if (cs_global_update(&c, eps)) { status = 1; break; }
        int64_t qh = 0, qt = 0, qn = 0;
        for (int64_t v = 0; v < n; ++v) {
            cur[v] = r.first[v];
            inq[v] = 0;
            if (r.excess[v] > 0) { q[qt++] = v; inq[v] = 1; ++qn; }
        }
        if (qt == n + 1) qt = 0;
        int64_t relabels = 0;
        while (qn > 0) {
            const int64_t u = q[qh++]; if (qh == n + 1) qh = 0; --qn; inq[u] = 0;
            while (r.excess[u] > 0) {
                int64_t a = cur[u];
                const int64_t e = r.first[u + 1];
                for (; a < e; ++a) {
                    if (r.rcap[a] <= 0) continue;
                    const int64_t v = r.head[a];
                    if (r.cost[a] + c.p[u] - c.p[v] >= 0) continue;
                    const int64_t dlt = r.rcap[a] < r.excess[u] ? r.rcap[a] : r.excess[u];
                    r.rcap[a] -= dlt; r.rcap[r.rev[a]] += dlt;
                    r.excess[u] -= dlt;
                    const int64_t old = r.excess[v];
                    r.excess[v] += dlt;
                    if (old <= 0 && r.excess[v] > 0 && !inq[v]) {
                        q[qt++] = v; if (qt == n + 1) qt = 0; ++qn; inq[v] = 1;
                    }
                    if (r.excess[u] == 0) break;
                }
                cur[u] = a;
                if (r.excess[u] == 0) break;
                /* relabel */
                int64_t minrc = KO_INF;
                for (int64_t b = r.first[u]; b < e; ++b) {
                    if (r.rcap[b] <= 0) continue;
                    const int64_t rc = r.cost[b] + c.p[u] - c.p[r.head[b]];
                    if (rc < minrc) minrc = rc;
                }
                if (minrc == KO_INF) { status = 1; break; }
                c.p[u] -= minrc + eps;
                cur[u] = r.first[u];
                if (++relabels > n) {
                    relabels = 0;
                    if (cs_global_update(&c, eps)) { status = 1; break; }
                    for (int64_t v = 0; v < n; ++v) cur[v] = r.first[v];
                }
            }
            if (status) break;
        }
        if (status || eps == 1) break;
    }

    int64_t left = 0;
    for (int64_t v = 0; v < n; ++v) if (r.excess[v] > 0) left += r.excess[v];
    for (int64_t a = 0; a < 2 * r.m; ++a) r.cost[a] /= mult;
    res_flows(g, &r, flow_out);
    int64_t tc = 0;
    for (int64_t i = 0; i < g->m; ++i) tc += flow_out[i] * g->cost[i];
    *total_cost = tc;
    *flow_value = r.pos_supply - left;
    hp_free(&c.h);
    free(c.p); free(c.d); free(c.scanned); free(cur); free(q); free(inq);
    res_free(&r);
    return status ? 1 : 0;
}

/* ------------------------------------------------------------------------- */
int ko_verify(const ko_graph* g, const int64_t* flow, int64_t* total_cost, int64_t* flow_value) {
    int64_t* bal = (int64_t*)calloc(g->n + 1, sizeof(int64_t));
    int st = 0;
    int64_t c = 0, pos = 0;
    for (int64_t i = 0; i < g->m; ++i) {
        if (flow[i] < g->low[i] || flow[i] > g->cap[i]) st = 1;
        bal[g->src[i] - 1] -= flow[i];
        bal[g->dst[i] - 1] += flow[i];
        c += flow[i] * g->cost[i];
    }
    for (int64_t v = 0; v < g->n; ++v) {
        if (g->supply[v] > 0) pos += g->supply[v];
        if (!st && g->supply[v] + bal[v] != 0) st = 2;
    }
    free(bal);
    *total_cost = c;
    *flow_value = pos;
    return st;
}

/* ------------------------------------------------------------------------- */
/* DIMACS text (dimacs/export.go:11-76) and the flow protocol (solver.go:134-179) */
/* ------------------------------------------------------------------------- */
static inline char* put_i64(char* p, int64_t v) {
    char tmp[24];
    int k = 0;
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    if (v < 0) *p++ = '-';
    do { tmp[k++] = (char)('0' + u % 10); u /= 10; } while (u);
    while (k) *p++ = tmp[--k];
    return p;
}
static inline char* put_s(char* p, const char* s) { while (*s) *p++ = *s++; return p; }

int64_t ko_export_dimacs(const ko_graph* g, char* buf, int64_t cap) {
    /* upper bound: 24 chars per integer field */
    const int64_t need = 256 + g->n * (4 + 3 * 24) + g->m * (4 + 5 * 24);
    if (!buf) return need;
    if (cap < need) return -1;
    char* p = buf;
    p = put_s(p, "c ===========================\np min ");
    p = put_i64(p, g->n); *p++ = ' '; p = put_i64(p, g->m); *p++ = '\n';
    p = put_s(p, "c ===========================\nc === ALL NODES FOLLOW ===\n");
    for (int64_t v = 0; v < g->n; ++v) {
        p = put_s(p, "n "); p = put_i64(p, v + 1); *p++ = ' ';
        p = put_i64(p, g->supply[v]); *p++ = ' '; p = put_i64(p, g->ntype[v]); *p++ = '\n';
    }
    p = put_s(p, "c === ALL ARCS FOLLOW ===\n");
    for (int64_t i = 0; i < g->m; ++i) {
        p = put_s(p, "a "); p = put_i64(p, g->src[i]); *p++ = ' '; p = put_i64(p, g->dst[i]); *p++ = ' ';
        p = put_i64(p, g->low[i]); *p++ = ' '; p = put_i64(p, g->cap[i]); *p++ = ' ';
        p = put_i64(p, g->cost[i]); *p++ = '\n';
    }
    p = put_s(p, "c EOI\n");
    *p = 0;
    return p - buf;
}

static inline const char* skip_ws(const char* p, const char* e) {
    while (p < e && (*p == ' ' || *p == '\t')) ++p;
    return p;
}
static inline const char* get_i64(const char* p, const char* e, int64_t* out, int* ok) {
    p = skip_ws(p, e);
    int neg = 0;
    if (p < e && *p == '-') { neg = 1; ++p; }
    if (p >= e || *p < '0' || *p > '9') { *ok = 0; return p; }
    int64_t v = 0;
    while (p < e && *p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
    *out = neg ? -v : v;
    return p;
}

void ko_free_graph(ko_graph* g) {
    free(g->ntype); free(g->supply); free(g->src); free(g->dst);
    free(g->low); free(g->cap); free(g->cost);
    memset(g, 0, sizeof(*g));
}

int ko_parse_dimacs(const char* text, int64_t len, ko_graph* out) {
    const char* p = text;
    const char* e = text + len;
    memset(out, 0, sizeof(*out));
    int64_t ia = 0;
    while (p < e) {
        const char* le = memchr(p, '\n', (size_t)(e - p));
        if (!le) le = e;
        int ok = 1;
        if (*p == 'p') {
            const char* q = p + 1;
            q = skip_ws(q, le);
            if (le - q < 3 || strncmp(q, "min", 3)) return -1;
            q += 3;
            q = get_i64(q, le, &out->n, &ok);
            q = get_i64(q, le, &out->m, &ok);
            if (!ok) return -1;
            out->ntype = (int32_t*)calloc(out->n + 1, sizeof(int32_t));
            out->supply = (int64_t*)calloc(out->n + 1, sizeof(int64_t));
            out->src = (int64_t*)malloc(sizeof(int64_t) * (out->m + 1));
            out->dst = (int64_t*)malloc(sizeof(int64_t) * (out->m + 1));
            out->low = (int64_t*)malloc(sizeof(int64_t) * (out->m + 1));
            out->cap = (int64_t*)malloc(sizeof(int64_t) * (out->m + 1));
            out->cost = (int64_t*)malloc(sizeof(int64_t) * (out->m + 1));
        } else if (*p == 'n') {
            int64_t id = 0, ex = 0, ty = 0;
            const char* q = get_i64(p + 1, le, &id, &ok);
            q = get_i64(q, le, &ex, &ok);
            if (!ok || !out->supply || id < 1 || id > out->n) return -1;
            int ok2 = 1;
            get_i64(q, le, &ty, &ok2);
            out->supply[id - 1] = ex;
            out->ntype[id - 1] = ok2 ? (int32_t)ty : 0;
        } else if (*p == 'a') {
            if (!out->src || ia >= out->m) return -1;
            const char* q = get_i64(p + 1, le, &out->src[ia], &ok);
            q = get_i64(q, le, &out->dst[ia], &ok);
            q = get_i64(q, le, &out->low[ia], &ok);
            q = get_i64(q, le, &out->cap[ia], &ok);
            q = get_i64(q, le, &out->cost[ia], &ok);
            if (!ok) return -1;
            ++ia;
        }
        p = le + 1;
    }
    if (!out->src || ia != out->m) return -1;
    return 0;
}

int64_t ko_flow_lines(const ko_graph* g, const int64_t* flow, int64_t cost, char* buf, int64_t cap) {
    int64_t nf = 0;
    for (int64_t i = 0; i < g->m; ++i) if (flow[i] > 0) ++nf;
    const int64_t need = 64 + nf * (4 + 3 * 24) + 32;
    if (!buf) return need;
    if (cap < need) return -1;
    char* p = buf;
    for (int64_t i = 0; i < g->m; ++i) {
        if (flow[i] <= 0) continue;
        p = put_s(p, "f "); p = put_i64(p, g->src[i]); *p++ = ' '; p = put_i64(p, g->dst[i]); *p++ = ' ';
        p = put_i64(p, flow[i]); *p++ = '\n';
    }
    p = put_s(p, "s "); p = put_i64(p, cost); *p++ = '\n';
    p = put_s(p, "c ALGORITHM TIME\nc EOI\n");
    *p = 0;
    return p - buf;
}

/* growable int64 vector */
typedef struct { int64_t* a; int64_t n, cap; } vec_t;
static inline void vpush(vec_t* v, int64_t x) {
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 4; v->a = (int64_t*)realloc(v->a, sizeof(int64_t) * v->cap); }
    v->a[v->n++] = x;
}

/* readFlowGraph (solver.go:134-179) + parseFlowToMapping/addPUToSourceNodes (:183-269).
 * Go map iteration is randomised; this restatement iterates leaves and flow
 * pairs in id / line order, which is one of the orders Go may produce. */
int64_t ko_bfs_mapping_from_lines(const ko_graph* g, const char* lines, int64_t len,
                                  int64_t* task_out, int64_t* pu_out) {
    const int64_t n = g->n;
    /* parse "f" lines into per-dst incoming lists (flow > 0 only, solver.go:157) */
    int64_t nf = 0, cap = 1024;
    int64_t *fs = (int64_t*)malloc(sizeof(int64_t) * cap), *fd = (int64_t*)malloc(sizeof(int64_t) * cap),
            *ff = (int64_t*)malloc(sizeof(int64_t) * cap);
    const char* p = lines;
    const char* e = lines + len;
    int eoi = 0;
    while (p < e && !eoi) {
        const char* le = memchr(p, '\n', (size_t)(e - p));
        if (!le) le = e;
        if (le > p) {
            if (*p == 'f') {
                int ok = 1;
                int64_t s = 0, d = 0, f = 0;
                const char* q = get_i64(p + 1, le, &s, &ok);
                q = get_i64(q, le, &d, &ok);
                q = get_i64(q, le, &f, &ok);
                if (!ok || s < 1 || s > n || d < 1 || d > n) { nf = -1; break; }
                if (f > 0) {
                    if (nf == cap) {
                        cap *= 2;
                        fs = (int64_t*)realloc(fs, sizeof(int64_t) * cap);
                        fd = (int64_t*)realloc(fd, sizeof(int64_t) * cap);
                        ff = (int64_t*)realloc(ff, sizeof(int64_t) * cap);
                    }
                    fs[nf] = s - 1; fd[nf] = d - 1; ff[nf] = f; ++nf;
                }
            } else if (*p == 'c') {
                if (le - p == 5 && !strncmp(p, "c EOI", 5)) eoi = 1;
            } else if (*p != 's') { nf = -1; break; }   /* solver.go:175 panic */
        }
        p = le + 1;
    }
    if (nf < 0 || !eoi) { free(fs); free(fd); free(ff); return -2; }   /* solver.go:178 */
    int64_t* ifirst = (int64_t*)calloc(n + 1, sizeof(int64_t));
    for (int64_t i = 0; i < nf; ++i) ifirst[fd[i] + 1]++;
    for (int64_t v = 0; v < n; ++v) ifirst[v + 1] += ifirst[v];
    int64_t* ipos = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    memcpy(ipos, ifirst, sizeof(int64_t) * (n + 1));
    int64_t* isrc = (int64_t*)malloc(sizeof(int64_t) * (nf + 1));
    int64_t* iflow = (int64_t*)malloc(sizeof(int64_t) * (nf + 1));
    for (int64_t i = 0; i < nf; ++i) { const int64_t k = ipos[fd[i]]++; isrc[k] = fs[i]; iflow[k] = ff[i]; }
    free(fs); free(fd); free(ff); free(ipos);

    int64_t sink = -1;
    for (int64_t v = 0; v < n; ++v) if (g->ntype[v] == 3) { sink = v; break; }
    vec_t* pus = (vec_t*)calloc(n, sizeof(vec_t));
    char* visited = (char*)calloc(n, 1);
    int64_t* queue = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t qh = 0, qt = 0, nmap = 0;
    for (int64_t v = 0; v < n && sink >= 0; ++v) {
        if (g->ntype[v] != 2) continue;                      /* LeafNodeIDs: PUs */
        visited[v] = 1;
        int64_t f = 0;
        for (int64_t k = ifirst[sink]; k < ifirst[sink + 1]; ++k) if (isrc[k] == v) { f = iflow[k]; break; }
        if (f <= 0) continue;
        for (int64_t i = 0; i < f; ++i) vpush(&pus[v], v);
        queue[qt++] = v;
    }
    int64_t rc = 0;
    while (qh < qt) {
        const int64_t v = queue[qh++];
        visited[v] = 1;
        if (g->ntype[v] == 1) {                              /* IsTaskNode */
            if (pus[v].n != 1) { rc = -1; break; }            /* solver.go:223-225 */
            task_out[nmap] = v + 1; pu_out[nmap] = pus[v].a[0] + 1; ++nmap;
            continue;
        }
        int64_t it = 0;
        for (int64_t k = ifirst[v]; k < ifirst[v + 1]; ++k) {
            const int64_t s = isrc[k];
            for (; iflow[k] > 0; iflow[k]--) {
                if (it == pus[v].n) break;
                vpush(&pus[s], pus[v].a[it]);
                ++it;
            }
            if (!visited[s]) { queue[qt++] = s; visited[s] = 1; }
            if (it == pus[v].n) break;
        }
    }
    for (int64_t v = 0; v < n; ++v) free(pus[v].a);
    free(pus); free(visited); free(queue); free(ifirst); free(isrc); free(iflow);
    return rc < 0 ? rc : nmap;
}

/* ExportIncremental (dimacs/export.go:31-38): one GenerateChange line per record
 * (add_node_change.go:57-61 "n id excess type", create_arc_change.go:44-51
 * "a src dst low cap cost type", update_arc_change.go:46-54
 * "x src dst low cap cost type oldcost", remove_node_change.go:26-28 "r id"),
 * then "c EOI". SET_EXCESS has no line (the reference never sends the sink's
 * drift). Returns bytes written or the required size when buf is NULL. */
int64_t ko_export_changes(const ko_delta* d, int64_t k, char* buf, int64_t cap) {
    const int64_t need = 16 + k * (4 + 8 * 24);
    if (!buf) return need;
    if (cap < need) return -1;
    char* p = buf;
    for (int64_t i = 0; i < k; ++i) {
        const ko_delta* x = &d[i];
        switch (x->kind) {
            case 0:
                p = put_s(p, "n "); p = put_i64(p, (int64_t)x->id); *p++ = ' ';
                p = put_i64(p, x->excess); *p++ = ' '; p = put_i64(p, x->type); *p++ = '\n';
                break;
            case 1:
                p = put_s(p, "r "); p = put_i64(p, (int64_t)x->id); *p++ = '\n';
                break;
            case 2: case 3:
                p = put_s(p, x->kind == 2 ? "a " : "x ");
                p = put_i64(p, (int64_t)x->src); *p++ = ' '; p = put_i64(p, (int64_t)x->dst); *p++ = ' ';
                p = put_i64(p, (int64_t)x->low); *p++ = ' '; p = put_i64(p, (int64_t)x->cap); *p++ = ' ';
                p = put_i64(p, x->cost); *p++ = ' '; p = put_i64(p, x->type);
                if (x->kind == 3) { *p++ = ' '; p = put_i64(p, x->old_cost); }
                *p++ = '\n';
                break;
            default:
                break;
        }
    }
    p = put_s(p, "c EOI\n");
    *p = 0;
    return p - buf;
}

/* The daemon's side of that stream: parse the change block back into records
 * until "c EOI". Returns the record count, or −1 on a malformed line. */
int64_t ko_parse_changes(const char* text, int64_t len, ko_delta* out, int64_t cap) {
    const char* p = text;
    const char* e = text + len;
    int64_t k = 0;
    while (p < e) {
        const char* le = memchr(p, '\n', (size_t)(e - p));
        if (!le) le = e;
        if (le > p) {
            int ok = 1;
            ko_delta x;
            memset(&x, 0, sizeof(x));
            int64_t v[7] = {0};
            const char* q = p + 1;
            if (*p == 'c') {
                if (le - p == 5 && !strncmp(p, "c EOI", 5)) break;
            } else if (*p == 'n') {
                for (int i = 0; i < 3; ++i) q = get_i64(q, le, &v[i], &ok);
                x.kind = 0; x.id = (uint64_t)v[0]; x.excess = v[1]; x.type = (int32_t)v[2];
            } else if (*p == 'r') {
                q = get_i64(q, le, &v[0], &ok);
                x.kind = 1; x.id = (uint64_t)v[0];
            } else if (*p == 'a' || *p == 'x') {
                const int nf = *p == 'a' ? 6 : 7;
                for (int i = 0; i < nf; ++i) q = get_i64(q, le, &v[i], &ok);
                x.kind = *p == 'a' ? 2 : 3;
                x.src = (uint64_t)v[0]; x.dst = (uint64_t)v[1]; x.low = (uint64_t)v[2]; x.cap = (uint64_t)v[3];
                x.cost = v[4]; x.type = (int32_t)v[5]; x.old_cost = v[6];
            } else {
                ok = 0;
            }
            if (!ok) return -1;
            if (*p != 'c') {
                if (k < cap && out) out[k] = x;
                ++k;
            }
        }
        p = le + 1;
    }
    return k;
}

/* The reference path of a later Solve (solver.go:84-90): the change block as
 * text and parsed back by the daemon, the incremental SSP re-solve, the "f"
 * lines of every positive-flow arc, and the BFS mapping over them.
 * ms[0..5] = export changes, parse, carry, saturate, augment, flines + bfs. */
int ko_reference_path_incremental(const ko_graph* g, const ko_delta* deltas, int64_t k,
                                  const int64_t* prev_src, const int64_t* prev_dst, const int64_t* prev_flow,
                                  int64_t prev_m, const int64_t* prev_pot, int64_t prev_n, const uint8_t* fresh,
                                  int64_t* flow_out, int64_t* pot_out, int64_t* total_cost, int64_t* flow_value,
                                  int64_t* n_mapped, double* ms) {
    const double t0 = now_ms();
    const int64_t need = ko_export_changes(deltas, k, NULL, 0);
    char* text = (char*)malloc((size_t)need + 1);
    const int64_t tl = ko_export_changes(deltas, k, text, need + 1);
    const double t1 = now_ms();
    ko_delta* back = (ko_delta*)malloc(sizeof(ko_delta) * (size_t)(k + 1));
    const int64_t kb = ko_parse_changes(text, tl, back, k + 1);
    free(text);
    free(back);
    if (kb < 0) return -1;
    const double t2 = now_ms();
    double sm[3] = {0, 0, 0};
    int64_t aug = 0;
    const int st = ko_ssp_incremental(g, prev_src, prev_dst, prev_flow, prev_m, prev_pot, prev_n, fresh, flow_out,
                                      pot_out, total_cost, flow_value, &aug, sm);
    if (st < 0) return st;
    const double t3 = now_ms();
    const int64_t fneed = ko_flow_lines(g, flow_out, *total_cost, NULL, 0);
    char* fl = (char*)malloc((size_t)fneed + 1);
    const int64_t fll = ko_flow_lines(g, flow_out, *total_cost, fl, fneed + 1);
    int64_t* tk = (int64_t*)malloc(sizeof(int64_t) * (g->n + 1));
    int64_t* pu = (int64_t*)malloc(sizeof(int64_t) * (g->n + 1));
    *n_mapped = ko_bfs_mapping_from_lines(g, fl, fll, tk, pu);
    const double t4 = now_ms();
    free(fl); free(tk); free(pu);
    if (ms) {
        ms[0] = t1 - t0; ms[1] = t2 - t1; ms[2] = sm[0]; ms[3] = sm[1]; ms[4] = sm[2]; ms[5] = t4 - t3;
    }
    (void)t3;
    return st;
}

int ko_reference_path(const ko_graph* g, int64_t* total_cost, int64_t* flow_value,
                      int64_t* n_mapped, double* ms) {
    double t0 = now_ms();
    const int64_t need = ko_export_dimacs(g, NULL, 0);
    char* text = (char*)malloc((size_t)need + 1);
    const int64_t tl = ko_export_dimacs(g, text, need + 1);
    double t1 = now_ms();
    ko_graph h;
    if (tl < 0 || ko_parse_dimacs(text, tl, &h)) { free(text); return -1; }
    free(text);
    double t2 = now_ms();
    int64_t* flow = (int64_t*)malloc(sizeof(int64_t) * (h.m + 1));
    int64_t aug = 0;
    const int st = ko_ssp(&h, flow, total_cost, flow_value, &aug);
    double t3 = now_ms();
    const int64_t fneed = ko_flow_lines(&h, flow, *total_cost, NULL, 0);
    char* fl = (char*)malloc((size_t)fneed + 1);
    const int64_t fll = ko_flow_lines(&h, flow, *total_cost, fl, fneed + 1);
    double t4 = now_ms();
    int64_t* tk = (int64_t*)malloc(sizeof(int64_t) * (h.n + 1));
    int64_t* pu = (int64_t*)malloc(sizeof(int64_t) * (h.n + 1));
    *n_mapped = ko_bfs_mapping_from_lines(&h, fl, fll, tk, pu);
    double t5 = now_ms();
    if (ms) { ms[0] = t1 - t0; ms[1] = t2 - t1; ms[2] = t3 - t2; ms[3] = t4 - t3; ms[4] = t5 - t4; }
    free(fl); free(tk); free(pu); free(flow);
    ko_free_graph(&h);
    return st;
}
