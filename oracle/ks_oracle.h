/*
 * ks_oracle — CPU restatement of the ksched placement hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in ksched_amd/ (the product) links,
 * loads or calls this code. It is imported only by tests/, by
 * __graft_entry__.smoke() as the checker, and by bench.py's cpu_baseline leg.
 *
 * Parity pinning: the reference's arithmetic lives in Flowlessly (external,
 * unpinned, absent offline — SURVEY §8c), so this oracle is pinned by
 *   (1) the known answers derived from the reference's own graph semantics
 *       (config 1: cost 200 / flow 100; TestMultiScheduleIteration rounds:
 *       9/15/15/9/5 with flows 3/5/3/3/3 — tests/golden/known_answers.json),
 *   (2) networkx.network_simplex goldens generated in the build container by
 *       tests/golden/gen_goldens.py (committed as (params, seed) → (cost, flow)),
 *   (3) agreement of two independent algorithms implemented here (successive
 *       shortest path = Flowlessly's configured algorithm, solver.go:32, and
 *       Goldberg cost scaling) with each other on every test graph.
 *
 * Contents:
 *   ko_gen_quincy / ko_gen_trivial   graph generators (trivial
 *                                    topology of cmd/k8sscheduler/scheduler.go:191-202,332-350
 *                                    with the arc families of graph_manager.go:1116-1305)
 *   ko_ssp                           successive shortest path min-cost max-flow
 *                                    (restates the Flowlessly algorithm ksched selects,
 *                                    placement/solver.go:30-34, 272-285)
 *   ko_cost_scaling                  Goldberg ε-scaling push-relabel (strong CPU baseline)
 *   ko_verify                        conservation / capacity / cost (integer)
 *   ko_export_dimacs                 dimacs/export.go:11-76 byte format
 *   ko_flow_lines / ko_parse_flow_lines   the "f src dst flow" protocol read by
 *                                    placement/solver.go:134-179
 *   ko_bfs_mapping                   parseFlowToMapping + addPUToSourceNodes,
 *                                    placement/solver.go:183-269
 *   ko_reference_path                export → parse → SSP → f lines → parse → BFS
 *   ko_ssp_incremental               SSP re-solve from the previous round's flow and
 *                                    potentials (Flowlessly's daemon mode, which ksched
 *                                    runs: solver.go:30-34 Incremental, :86-89)
 *   ko_export_changes / ko_parse_changes   the ExportIncremental change block
 *                                    (export.go:31-38, *_change.go GenerateChange)
 *   ko_reference_path_incremental    change text → parse → incremental SSP → f lines → BFS
 */
#ifndef KS_ORACLE_H
#define KS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Graph with 1-based node ids 1..n (index = id-1). */
typedef struct ko_graph {
    int64_t  n, m;
    int32_t* ntype;    /* n: DIMACS node type code                */
    int64_t* supply;   /* n: node excess                          */
    int64_t* src;      /* m: 1-based node ids                     */
    int64_t* dst;      /* m                                       */
    int64_t* low;      /* m                                       */
    int64_t* cap;      /* m                                       */
    int64_t* cost;     /* m                                       */
} ko_graph;

/* generator output sizes */
void ko_quincy_sizes(int64_t T, int64_t M, int64_t R, int64_t J, int64_t* n, int64_t* m);
void ko_trivial_sizes(int64_t machines, int64_t pods, int64_t* n, int64_t* m);

/* Fill caller-allocated arrays of a graph sized by the *_sizes call. */
int ko_gen_quincy(int64_t T, int64_t M, int64_t R, int64_t J, uint64_t seed, ko_graph* g);
int ko_gen_trivial(int64_t machines, int64_t mt, int64_t pods, ko_graph* g);

/* status: 0 feasible (all supply routed), 1 infeasible remainder, <0 error */
int ko_ssp(const ko_graph* g, int64_t* flow_out, int64_t* total_cost, int64_t* flow_value,
           int64_t* augmentations);
int ko_cost_scaling(const ko_graph* g, int alpha, int64_t* flow_out, int64_t* total_cost,
                    int64_t* flow_value);
/* 0 ok, 1 capacity violated, 2 conservation violated */
int ko_verify(const ko_graph* g, const int64_t* flow, int64_t* total_cost, int64_t* flow_value);

/* DIMACS text (export.go format). Returns bytes written (excluding NUL) or the
 * required size when buf is NULL. */
int64_t ko_export_dimacs(const ko_graph* g, char* buf, int64_t cap);
/* Parse DIMACS "p/n/a" text into a graph (allocates; free with ko_free_graph). */
int ko_parse_dimacs(const char* text, int64_t len, ko_graph* out);
void ko_free_graph(ko_graph* g);

/* "f src dst flow" lines for every arc with flow > 0, then "s cost", "c EOI". */
int64_t ko_flow_lines(const ko_graph* g, const int64_t* flow, int64_t cost, char* buf, int64_t cap);

/* BFS extraction (solver.go:183-269) over parsed f lines. task_out/pu_out sized n.
 * Returns the number of mapped tasks, or -1 on the 1:1 violation (solver.go:223-225). */
int64_t ko_bfs_mapping_from_lines(const ko_graph* g, const char* lines, int64_t len,
                                  int64_t* task_out, int64_t* pu_out);

/* The whole reference CPU path; ms[0..4] = export, parse, ssp, flines, bfs. */
int ko_reference_path(const ko_graph* g, int64_t* total_cost, int64_t* flow_value,
                      int64_t* n_mapped, double* ms);

/* One change record (the same 72-byte layout as the product's ks_delta; kinds:
 * 0 "n", 1 "r", 2 "a", 3 "x", 4 sink-excess drift with no line). */
typedef struct ko_delta {
    int32_t  kind, type;
    uint64_t id, src, dst, low, cap;
    int64_t  cost, old_cost, excess;
} ko_delta;

/* Incremental SSP re-solve (Flowlessly's daemon mode: solver.go:30-34, 86-89):
 * the previous round's flow (by (src, dst)) and potentials (by node id; fresh
 * nodes re-priced) are carried onto g, arcs the changes left with negative
 * reduced cost are saturated, and SSP routes the resulting excess.
 * pot_out (n) feeds the next round. ms[0..2] = carry, saturate, augment. */
int ko_ssp_incremental(const ko_graph* g, const int64_t* prev_src, const int64_t* prev_dst,
                       const int64_t* prev_flow, int64_t prev_m, const int64_t* prev_pot, int64_t prev_n,
                       const uint8_t* fresh, int64_t* flow_out, int64_t* pot_out, int64_t* total_cost,
                       int64_t* flow_value, int64_t* augmentations, double* ms);
/* ExportIncremental text of a change block (export.go:31-38) and its parse. */
int64_t ko_export_changes(const ko_delta* d, int64_t k, char* buf, int64_t cap);
int64_t ko_parse_changes(const char* text, int64_t len, ko_delta* out, int64_t cap);
/* A later Solve's reference path: change text → parse → incremental SSP →
 * f lines → BFS. ms[0..5] = export, parse, carry, saturate, augment, flines+bfs. */
int ko_reference_path_incremental(const ko_graph* g, const ko_delta* deltas, int64_t k,
                                  const int64_t* prev_src, const int64_t* prev_dst, const int64_t* prev_flow,
                                  int64_t prev_m, const int64_t* prev_pot, int64_t prev_n, const uint8_t* fresh,
                                  int64_t* flow_out, int64_t* pot_out, int64_t* total_cost, int64_t* flow_value,
                                  int64_t* n_mapped, double* ms);

#ifdef __cplusplus
}
#endif
#endif
