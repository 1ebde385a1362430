/*
 * ks_oracle_cli — TEST INFRASTRUCTURE ONLY.
 *
 *   ks_oracle_cli solve [ssp|cs]      read one full DIMACS export (export.go format)
 *                                     on stdin, print "f src dst flow" lines,
 *                                     "s cost", "c EOI" — the flow_scheduler
 *                                     protocol read by placement/solver.go:134-179
 *   ks_oracle_cli quincy T M R J SEED write a generated graph as DIMACS
 *   ks_oracle_cli trivial NM MT PODS  write the ksched trivial topology as DIMACS
 *   ks_oracle_cli refpath T M R J SEED  time the reference CPU path
 */
#include "ks_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static char* read_all(FILE* f, int64_t* len) {
    size_t cap = 1 << 20, n = 0;
    char* b = (char*)malloc(cap);
    for (;;) {
        if (n == cap) { cap *= 2; b = (char*)realloc(b, cap); }
        size_t r = fread(b + n, 1, cap - n, f);
        if (r == 0) break;
        n += r;
    }
    *len = (int64_t)n;
    return b;
}

static void alloc_graph(ko_graph* g, int64_t n, int64_t m) {
    g->n = n; g->m = m;
    g->ntype = (int32_t*)calloc(n, sizeof(int32_t));
    g->supply = (int64_t*)calloc(n, sizeof(int64_t));
    g->src = (int64_t*)malloc(sizeof(int64_t) * m);
    g->dst = (int64_t*)malloc(sizeof(int64_t) * m);
    g->low = (int64_t*)malloc(sizeof(int64_t) * m);
    g->cap = (int64_t*)malloc(sizeof(int64_t) * m);
    g->cost = (int64_t*)malloc(sizeof(int64_t) * m);
}

static void dump(const ko_graph* g) {
    int64_t need = ko_export_dimacs(g, NULL, 0);
    char* b = (char*)malloc((size_t)need + 1);
    int64_t l = ko_export_dimacs(g, b, need + 1);
    fwrite(b, 1, (size_t)l, stdout);
    free(b);
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: see header\n"); return 2; }
    if (!strcmp(argv[1], "solve")) {
        int64_t len;
        char* text = read_all(stdin, &len);
        ko_graph g;
        if (ko_parse_dimacs(text, len, &g)) { fprintf(stderr, "parse error\n"); return 1; }
        free(text);
        int64_t* flow = (int64_t*)malloc(sizeof(int64_t) * (g.m + 1));
        int64_t cost = 0, fv = 0, aug = 0;
        int st = (argc > 2 && !strcmp(argv[2], "cs")) ? ko_cost_scaling(&g, 12, flow, &cost, &fv)
                                                        : ko_ssp(&g, flow, &cost, &fv, &aug);
        if (st < 0) { fprintf(stderr, "solve error %d\n", st); return 1; }
        int64_t need = ko_flow_lines(&g, flow, cost, NULL, 0);
        char* b = (char*)malloc((size_t)need + 1);
        int64_t l = ko_flow_lines(&g, flow, cost, b, need + 1);
        fwrite(b, 1, (size_t)l, stdout);
        return 0;
    }
    if (!strcmp(argv[1], "quincy") && argc >= 7) {
        int64_t T = atoll(argv[2]), M = atoll(argv[3]), R = atoll(argv[4]), J = atoll(argv[5]);
        uint64_t seed = strtoull(argv[6], 0, 10);
        int64_t n, m;
        ko_quincy_sizes(T, M, R, J, &n, &m);
        ko_graph g;
        alloc_graph(&g, n, m);
        if (ko_gen_quincy(T, M, R, J, seed, &g)) return 1;
        dump(&g);
        return 0;
    }
    if (!strcmp(argv[1], "trivial") && argc >= 5) {
        int64_t nm = atoll(argv[2]), mt = atoll(argv[3]), pods = atoll(argv[4]);
        int64_t n, m;
        ko_trivial_sizes(nm, pods, &n, &m);
        ko_graph g;
        alloc_graph(&g, n, m);
        if (ko_gen_trivial(nm, mt, pods, &g)) return 1;
        dump(&g);
        return 0;
    }
    if (!strcmp(argv[1], "refpath") && argc >= 7) {
        int64_t T = atoll(argv[2]), M = atoll(argv[3]), R = atoll(argv[4]), J = atoll(argv[5]);
        uint64_t seed = strtoull(argv[6], 0, 10);
        int64_t n, m;
        ko_quincy_sizes(T, M, R, J, &n, &m);
        ko_graph g;
        alloc_graph(&g, n, m);
        if (ko_gen_quincy(T, M, R, J, seed, &g)) return 1;
        int64_t cost, fv, nm;
        double ms[5];
        int st = ko_reference_path(&g, &cost, &fv, &nm, ms);
        printf("status %d cost %lld flow %lld mapped %lld export %.2f parse %.2f ssp %.2f flines %.2f bfs %.2f ms\n",
               st, (long long)cost, (long long)fv, (long long)nm, ms[0], ms[1], ms[2], ms[3], ms[4]);
        int64_t* flow = (int64_t*)malloc(sizeof(int64_t) * m);
        int64_t c2, f2;
        int st2 = ko_cost_scaling(&g, 12, flow, &c2, &f2);
        printf("cs status %d cost %lld flow %lld\n", st2, (long long)c2, (long long)f2);
        return 0;
    }
    fprintf(stderr, "bad arguments\n");
    return 2;
}
