/*
 * ksmcmf.h — C-ABI of the MI355X-native min-cost max-flow solver that replaces
 * ksched's Flowlessly round-trip (the `placement.Solver` hot path).
 *
 * What each entry point replaces in the reference (paths relative to the
 * ksched tree, scheduling/flow/…):
 *
 *   ks_create / ks_destroy   placement/solver.go:49-55 NewSolver, :92-109 startSolver
 *                            (the exec'd flow_scheduler child becomes a device context)
 *   ks_load_graph            placement/solver.go:111-116 writeGraph → dimacs/export.go:11-29
 *                            (full "p/n/a" DIMACS text export becomes an array upload)
 *   ks_apply_deltas          placement/solver.go:118-123 writeIncremental →
 *                            dimacs/export.go:31-38 + the GenerateChange methods of
 *                            dimacs/{add_node,create_arc,update_arc,remove_node}_change.go
 *                            — validated on the host, applied IN PLACE on the device:
 *                            the graph (arc table, (src, dst) hash index, residual
 *                            CSR with slack) stays resident in HBM between rounds; a
 *                            stream is all-or-nothing (an invalid record applies none)
 *   ks_coalesce_deltas       the change optimisers graph_change_manager.go:220-279
 *                            (optimizeChanges: RemoveDuplicate, MergeToSameArc,
 *                            PurgeBeforeNodeRemoval — declared there, never implemented)
 *   ks_solve                 the external Flowlessly solve (solver.go:30-34, Dockerfile:10-12)
 *                            — min-cost flow, bit-exact total cost and flow value
 *   ks_get_flows             the "f src dst flow" lines read by readFlowGraph
 *                            (placement/solver.go:134-179); only arcs with flow > 0
 *   ks_get_task_mapping      parseFlowToMapping + addPUToSourceNodes
 *                            (placement/solver.go:183-269) → flowmanager.TaskMapping
 *                            (flowmanager/types.go:6)
 *   ks_last_error            the panics of solver.go:97-108, 148-153, 175-178, 223-225
 *                            become status codes + a message
 *
 * Semantics (flowgraph/graph.go:25-41, arc.go:26-36, node.go:76-106):
 *   - node ids are ksched NodeIDs (dense from 1, reused FIFO after removal,
 *     graph.go:169-182); excess is the node supply (tasks +1, sink −#tasks);
 *     type is the DIMACS node type code of export.go:56-68 (task 1, PU 2,
 *     sink 3, machine 4, numa/socket/cache/core 5, other 0).
 *   - arcs are (src, dst, low, cap, cost, type); at most one arc per ordered
 *     (src, dst) pair (node.go:118-131). ADD_ARC on an existing pair upserts.
 *   - UPDATE_ARC with low == cap == 0 REMOVES the arc (DeleteArc emits this
 *     record, graph_change_manager.go:184-193; ChangeArc to 0/0, :142-156, keeps
 *     a zero-capacity arc in the reference, which carries no flow either, so the
 *     two are equivalent for the solve). A later ADD_ARC / UPDATE_ARC re-creates
 *     it. The arc then no longer counts in n_arcs.
 *   - REMOVE_NODE drops every incident arc implicitly (the reference emits only
 *     "r id", graph_change_manager.go:129-139); the id may be reused later.
 *   - SET_EXCESS sets a node's supply explicitly (the sink's demand drifts in
 *     the reference without a message: graph_manager.go:640, 808). With
 *     ks_opts.auto_sink != 0 (default) the sink's demand is recomputed as
 *     −Σ(other supplies) at every solve, which is what keeps an incremental
 *     DIMACS stream balanced.
 *
 * Ownership: input arrays belong to the caller and are copied during the call.
 * Output buffers are caller-allocated; call with cap = 0 to get the count.
 * One context per thread; calls on one context are not reentrant
 * (placement/solver.go:59). Contexts on different devices may run concurrently.
 */
#ifndef KSMCMF_H
#define KSMCMF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSMCMF_ABI_VERSION 5   /* 2: ks_opts tuning fields, ks_result.recoveries, batch layout calls;
                                  3: ks_opts.cell_nodes, ks_result per-kind timing and cell-solver
                                  fields; 4: ks_opts.compact_pos (the last reserved word of
                                  ks_opts), and three words of ks_result repurposed:
                                  cell_fallbacks and cycles_cancelled (two reserved words)
                                  and compact (the former _pad3); 5: ks_result.fb_resets
                                  (the last reserved word), ks_result.cycles_rejected and
                                  gu_leaf_scans; ks_result grew to 352 B (2 reserved words).
                                  ks_opts (96 B) CHANGED SIZE in ABI 2 and ks_result in
                                  ABI 2, 3 and 5: a caller must check
                                  ks_abi_version() == KSMCMF_ABI_VERSION before ks_create. */

/* status codes (0 = OK) */
#define KS_OK            0
#define KS_E_INVALID    (-1)  /* bad argument / malformed graph or delta          */
#define KS_E_INFEASIBLE (-2)  /* supplies cannot be routed to the demands         */
#define KS_E_DEVICE     (-3)  /* HIP runtime error or device not available        */
#define KS_E_VERIFY     (-4)  /* on-device verification of the result failed      */
#define KS_E_RANGE      (-5)  /* value outside the solver's integer range         */

/* DIMACS node-type codes (dimacs/add_node_change.go:27-36, export.go:56-68) */
#define KS_NODE_OTHER    0
#define KS_NODE_TASK     1
#define KS_NODE_PU       2
#define KS_NODE_SINK     3
#define KS_NODE_MACHINE  4
#define KS_NODE_INTERMEDIATE 5

typedef struct ks_ctx ks_ctx;

typedef struct ks_opts {
    int32_t  alpha;            /* cost-scaling factor per ε-phase; 0 (ks_default_opts):
                                  8, or 32 for graphs under 32,768 nodes on the
                                  multi-kernel engine                                   */
    int32_t  verify;           /* run the on-device verifier after every solve (1)      */
    int32_t  auto_sink;        /* sink demand = −Σ other supplies at solve time (1)     */
    int32_t  price_refine;     /* certify optimality early [1]: 1 — the phase before the
                                  final one drains, then price refinement cancels the
                                  negative cycles it meets until it certifies the flow
                                  (the final phase runs only if it gives up); 2 — the
                                  final phase, then plain price refinement; 0 — off    */
    int32_t  gu_interval;      /* sweeps between global price updates (default 24)      */
    int32_t  warm_start;       /* 1: re-solve from the previous flow and prices after
                                  ks_apply_deltas (the first phase saturates only the
                                  arcs violating its ε); 2: every phase does; 0
                                  (default): every solve from scratch  */
    /* solver tuning; 0 selects the library default given in brackets.
       None of these changes the result — only how fast it is reached. */
    int32_t  walk_slack;       /* a phase's tail walkers take residual arcs of reduced cost
                                  ≤ walk_slack·ε toward a smaller distance while ε > 1
                                  [4]; < 0 disables the walkers                       */
    int32_t  final_div;        /* the phase price refinement certifies runs at 1/final_div
                                  of a cost unit [20 for cells and graphs under 32,768
                                  nodes, else 24 with the cycle-cancelling finish
                                  (price_refine 1) and 48 without]; < 0: the plain
                                  max|cost|/α^k ladder                                  */
    int32_t  pr_rounds;        /* Bellman-Ford rounds one price refinement may take [160] */
    int32_t  phase_exit;       /* a coarse phase ends once ≤ phase_exit nodes hold excess
                                  [256] ... */
    int32_t  phase_frac;       /* ... and ≤ 1/phase_frac of the phase's peak [128]; < 0 in
                                  phase_exit: coarse phases always drain completely   */
    int32_t  tail_sweeps;      /* sweeps per cycle once ≤ 64 nodes hold excess [4]      */
    int32_t  bf_margin;        /* Bellman-Ford rounds enqueued per cycle beyond the last
                                  update's count [6]                                    */
    int32_t  two_hop;          /* Bellman-Ford relaxes a task's / PU's in-arcs in the round
                                  its distance dropped [1]; < 0 off                     */
    int32_t  log_cycles;       /* 1: one diagnostic line per update cycle on stderr [0] */
    int32_t  fault_inject;     /* TESTS ONLY [0]: bit 0 — the last phase's walks use the
                                  coarse slack at ε = 1 (may end non-1-optimal); bit 1 —
                                  the final prices are perturbed before verification.
                                  Both must be repaired by the certificate recovery.
                                  Bit 2 (ks_batch_create*): global rank 0 fails to pack
                                  its rows in ks_batch_gather (every rank must still
                                  reach the collective and return the error). Bit 3
                                  (ks_batch_create*): rank 0's receive buffer
                                  allocation fails in ks_batch_gather (the same).
                                  Bit 4 (ks_batch_create*): the middle cell of the
                                  batch gives up in the cell solver and is re-solved
                                  on the engine; the result then reports solver 1,
                                  cells = the batch's cells, warm_started 1 (the
                                  other cells' optima are carried), cell_fallbacks 1
                                  and fb_resets. Bit 5: the cycle-cancelling finish gives
                                  up after its first batch (the final phase runs).
                                  Bit 6: one unit is moved on an arc after the solve
                                  without its endpoints' excess (the verifier's
                                  conservation check must fail: KS_E_VERIFY).
                                  Bit 7: every parent-graph search of the finish
                                  doubles only 5 steps (a 32-node window, shorter than
                                  the parent chains: their nodes are marked and meet
                                  cycles, and the union-of-cycles test must reject
                                  them — cycles_rejected). Bit 8 (engine): that test
                                  only counts, rejecting nothing (with bit 7 a chain
                                  is pushed along: the verifier must then fail the
                                  solve with KS_E_VERIFY, never return a wrong cost). */
    int32_t  walk_passes;      /* tail walker passes from the update's excess nodes per
                                  cycle [1]; later passes retry units left short        */
    int32_t  tail_nodes;       /* a phase's tail — walks over each update, few sweeps —
                                  starts once ≤ tail_nodes nodes hold excess [64]; at
                                  most 4096                                             */
    int32_t  bf_bound;         /* a global update with ≤ 64 excess nodes drops Bellman-Ford
                                  offers at or above the largest tentative distance of
                                  those nodes and caps prices there [on]; < 0 off       */
    int32_t  fwd_nodes;        /* in a coarse phase (one a finer phase follows), once
                                  ≤ fwd_nodes nodes hold excess, a cycle searches from them
                                  to the nearest deficit and pushes along the search's
                                  shortest paths instead of a global update [32 below
                                  32,768 nodes, else 64]; a search
                                  whose frontier grows past n/4 nodes, or that runs longer
                                  than twice the last global update's rounds, costs ONE
                                  global update and the next cycle searches forward again.
                                  The last phase always uses global updates. < 0 off      */
    int32_t  cell_nodes;       /* the cell solver (one workgroup per graph)
                                  solves every graph — or every cell of a ks_batch union —
                                  of at most cell_nodes node slots [0: a ks_batch cell up
                                  to what its LDS holds (13,1xx), a lone graph up to 4,096
                                  (larger ones solve sooner on the whole chip)]; < 0:
                                  always the multi-kernel engine                          */
    int32_t  warm_shift;       /* warm start: a node whose flow-carrying out-arc got dearer
                                  since the last solve (ksched's ageing of unscheduled
                                  arcs) is priced down by the rise, so that arc keeps its
                                  reduced cost [0: on]; < 0 off                          */
    int32_t  warm_canon;       /* warm start: each solve ends by replacing its prices with
                                  the flow's canonical ones (a Bellman-Ford at ε = 1 from
                                  d = p), so carried prices do not drift [0: on]; < 0 off.
                                  Multi-kernel engine only: a cell-solver solve keeps the
                                  prices its workgroup ended with                      */
    int32_t  compact_pos;      /* the multi-kernel engine's solve reads 16-byte residual
                                  records (32-bit residual, pair capacity, scaled cost,
                                  head) when every scaled cost and capacity fits, else
                                  the 32-byte ones [0: on]; < 0: always 32-byte (ABI 4)  */
} ks_opts;

typedef struct ks_node {       /* one "n id excess type" line                            */
    uint64_t id;
    int64_t  excess;
    int32_t  type;
    int32_t  _pad;
} ks_node;

typedef struct ks_arc {        /* one "a src dst low cap cost [type]" line               */
    uint64_t src, dst;
    uint64_t low, cap;
    int64_t  cost;
    int32_t  type;             /* flowgraph.ArcType: 0 other, 1 running (arc.go:18-23)   */
    int32_t  _pad;
} ks_arc;

enum ks_delta_kind {
    KS_ADD_NODE    = 0,        /* "n id excess type"                                     */
    KS_REMOVE_NODE = 1,        /* "r id"                                                 */
    KS_ADD_ARC     = 2,        /* "a src dst low cap cost type" (upsert)                 */
    KS_UPDATE_ARC  = 3,        /* "x src dst low cap cost type oldcost"                  */
    KS_SET_EXCESS  = 4         /* explicit supply change (sink drift)                    */
};

typedef struct ks_delta {
    int32_t  kind;             /* enum ks_delta_kind                                     */
    int32_t  type;             /* node type (ADD_NODE) or arc type (ADD/UPDATE_ARC)      */
    uint64_t id;               /* node id (ADD_NODE, REMOVE_NODE, SET_EXCESS)            */
    uint64_t src, dst;         /* arc endpoints (ADD_ARC, UPDATE_ARC)                    */
    uint64_t low, cap;
    int64_t  cost;
    int64_t  old_cost;         /* UPDATE_ARC only (informational, as in the "x" line)    */
    int64_t  excess;           /* ADD_NODE, SET_EXCESS                                   */
} ks_delta;

#define KS_N_PHASE_TIMERS 6    /* build, saturate, cycles, price-refine, verify, total   */

typedef struct ks_result {
    int64_t  total_cost;       /* Σ flow·cost over all arcs (lower bounds included)      */
    int64_t  flow_value;       /* units routed from supply nodes to demand nodes         */
    int32_t  status;           /* same code as the ks_solve return value                 */
    int32_t  phases;           /* ε-phases executed                                      */
    uint64_t sweeps;           /* push/relabel sweep kernels that did work               */
    uint64_t arc_scans;        /* residual-arc scans (device counter)                    */
    uint64_t node_visits;      /* active-node discharges (device counter)                */
    uint64_t pushes;
    uint64_t relabels;
    uint64_t global_updates;
    uint64_t gu_iterations;    /* Bellman-Ford rounds that did work (updates+refinement) */
    uint64_t gu_arc_scans;     /* in-arc relaxations inside Bellman-Ford rounds          */
    double   ms_phase[KS_N_PHASE_TIMERS];
    int64_t  n_nodes;          /* node slots on device                                   */
    int64_t  n_arcs;           /* live input arcs                                        */
    uint64_t sweep_launches;   /* push/relabel sweep kernel launches (incl. early exits) */
    double   ms_sweep_kernels; /* HIP-event-timed span of all sweep batches (ms)         */
    uint64_t gu_launches;      /* Bellman-Ford round launches (price updates, refinement)*/
    double   ms_gu_kernels;    /* HIP-event-timed span of all Bellman-Ford batches (ms)  */
    int32_t  warm_started;     /* 1 when this solve started from the previous solution   */
    int32_t  rebuilt;          /* 1 when this solve rebuilt the residual CSR from the arc
                                  table (after a load, or a delta that did not fit)     */
    int32_t  recoveries;       /* times the final optimality certificate failed and was
                                  repaired (price refinement, else one more ε = 1 phase
                                  from the current flow) before the solve returned      */
    int32_t  solver;           /* 0: multi-kernel engine; 1: cell solver (ABI 3)         */
    /* ABI 3. Per-kind device time: each span starts at an event recorded right before
       its first kernel and ends at one right after its last (no host gap inside).
       ms_gu_kernels / gu_launches: the backward Bellman-Ford rounds (global updates,
       price refinement); ms_sweep_kernels / sweep_launches: the sweep bursts;
       forward tail updates (k_fs_*) are their own kind:                               */
    uint64_t fs_launches;      /* forward search rounds launched (k_fs_round)           */
    double   ms_fs_kernels;    /* event-timed span of the forward-update batches (ms)   */
    uint64_t fwd_updates;      /* forward tail updates completed                        */
    int32_t  cells;            /* cells the cell solver ran (one workgroup each)        */
    int32_t  compact;          /* 1: the engine's solve read 16-byte residual records   */
    double   ms_cell_kernel;   /* event-timed duration of the cell-solver launches (ms) */
    uint64_t cell_ticks_max;   /* slowest cell's in-kernel solve time (100 MHz ticks)   */
    uint64_t cell_ticks_sum;   /* Σ over cells of their in-kernel solve times            */
    uint64_t fs_arc_scans;     /* residual out-arcs the forward tail searches examined    */
    uint64_t cell_fallbacks;   /* cells of this solve that did not converge in the cell
                                  solver (step cap or wall-clock limit) and were re-solved
                                  on the multi-kernel engine, the other cells' optima
                                  kept (the status stays KS_OK)                         */
    uint64_t cycles_cancelled; /* negative cycles the cycle-cancelling finish cancelled
                                  (ks_opts.price_refine 1)                  */
    uint64_t fb_resets;        /* ABI 5. A per-cell fallback solve: live arc slots plus
                                  node slots of the failing cells whose carried flow /
                                  price it reset (they restart cold; 0 otherwise)      */
    uint64_t cycles_rejected;  /* ABI 5. The finish's parent-graph searches: marked nodes
                                  the union-of-cycles test found with other than one
                                  member pointing at them (engine), or leader walks
                                  that did not close a cycle (cell solver)            */
    uint64_t gu_leaf_scans;    /* ABI 5. Bellman-Ford rounds also relax the in-arcs of a task
                                  or PU whose distance just dropped, in the same round
                                  (two hops per round): those second-hop in-arc positions
                                  examined (gu_arc_scans counts the first hop only)      */
    uint64_t reserved3[2];
} ks_result;

/* Counters of the device-resident graph store (ks_get_store_stats). */
typedef struct ks_store_stats {
    int64_t  live_arcs;        /* arcs in the store                                      */
    int64_t  inserted;         /* last ks_apply_deltas: arcs inserted in place           */
    int64_t  updated;          /*   arcs whose bounds / cost were edited in place        */
    int64_t  killed;           /*   arcs removed (UPDATE 0/0 or an endpoint removed)     */
    int64_t  superseded;       /*   records overridden by a later record for the arc     */
    int64_t  rebuilds;         /* CSR rebuilds since ks_load_graph (1 = the load's own)  */
    int64_t  residual_slots;   /* residual positions allocated (live pairs + slack)      */
    int64_t  reserved[4];
} ks_store_stats;

typedef struct ks_flow {       /* one "f src dst flow" line                              */
    uint64_t src, dst;
    int64_t  flow;
} ks_flow;

int         ks_abi_version(void);
void        ks_default_opts(ks_opts* opts);
ks_ctx*     ks_create(int device, const ks_opts* opts);
void        ks_destroy(ks_ctx* ctx);
const char* ks_last_error(ks_ctx* ctx);

/* Replace the whole graph (first Solve: solver.go:63-83). */
int ks_load_graph(ks_ctx* ctx, const ks_node* nodes, size_t n,
                  const ks_arc* arcs, size_t m);

/* Apply a delta stream in mutation order (later Solves: solver.go:86-88). */
int ks_apply_deltas(ks_ctx* ctx, const ks_delta* deltas, size_t k);

/* Shrink a delta stream without changing what ks_apply_deltas makes of it
 * (graph_change_manager.go:220-279): per arc only its last ADD/UPDATE record
 * survives (both are upserts; UPDATE 0/0 deletes); arc and SET_EXCESS records
 * touching a node before its REMOVE_NODE are dropped; per node only the last
 * SET_EXCESS survives. ADD_NODE / REMOVE_NODE records are kept; survivors keep
 * their order. Host-only (no context, no device). Writes at most `cap` records
 * to `out` (out == in allowed), *count = surviving records. KS_E_INVALID on a
 * zero or out-of-range node id. Validation errors a dropped record would have
 * raised in ks_apply_deltas are not reported. */
int ks_coalesce_deltas(const ks_delta* in, size_t k, ks_delta* out, size_t cap, size_t* count);

/* Solve min-cost flow on the current graph. result may be NULL. */
int ks_solve(ks_ctx* ctx, ks_result* result);

/* Solve k independent contexts concurrently (config 5: cluster cells /
 * what-if graphs). `workers` host threads (0 = min(k, 4)) each take the next
 * unsolved context and call ks_solve on it; contexts on one device run on
 * their own streams and overlap on the GPU. results[i] (may be NULL) receives
 * context i's result. Returns KS_OK, or the status of the first failing
 * context in index order (the others still ran). No reference counterpart:
 * ksched solves one graph per round (flowscheduler/scheduler.go:350). */
int ks_solve_many(ks_ctx* const* ctxs, size_t k, int workers, ks_result* results);

/* Arcs with positive flow from the last solve (the "f" lines). */
int ks_get_flows(ks_ctx* ctx, ks_flow* out, size_t cap, size_t* count);

/* task NodeID → PU NodeID for every task whose unit reaches a PU (TaskMapping).
 * The flow is decomposed on the device: each task's unit is followed along
 * positive-flow arcs (units numbered per node in arc order) to the sink, and
 * the last PU on the way is its placement. */
int ks_get_task_mapping(ks_ctx* ctx, uint64_t* task, uint64_t* pu,
                        size_t cap, size_t* count);

/* Device-resident mapping for RCCL gathers: for the i-th task node in id order
 * writes the PU node id it maps to, or 0 when unscheduled, computed on device
 * (nothing crosses PCIe). dev_out is a device pointer with room for `cap`
 * uint64 (KS_E_INVALID when cap < the task count); dev_out = NULL only sets
 * *count, the number of task nodes. */
int ks_get_task_pu_device(ks_ctx* ctx, uint64_t* dev_out, size_t cap, size_t* count);

/* The device-resident graph as it stands (the reference's dimacs.Export view,
 * export.go:11-29, e.g. for a checkpoint or a DIMACS dump): live nodes in id order
 * and live arcs in arc-slot order. Call with caps of 0 to size. */
int ks_get_graph(ks_ctx* ctx, ks_node* nodes, size_t ncap, size_t* n, ks_arc* arcs, size_t acap, size_t* m);

/* Store counters (no device work). */
int ks_get_store_stats(ks_ctx* ctx, ks_store_stats* out);

/* ---- scheduler-side sweeps of a round, on the device-resident graph ------- */

/* pb.SchedulingDelta_ChangeType (proto/scheduling_delta.proto:11-16) */
#define KS_DELTA_PLACE   0
#define KS_DELTA_PREEMPT 1
#define KS_DELTA_MIGRATE 2
#define KS_DELTA_NOOP    3

typedef struct ks_sched_delta {
    int32_t  type;             /* KS_DELTA_*                                             */
    int32_t  _pad;
    uint64_t task;             /* task NodeID                                            */
    uint64_t pu;               /* PU NodeID (PLACE / MIGRATE: the new one; PREEMPT: the
                                  one it leaves)                                         */
} ks_sched_delta;

/* Seed the device-kept task bindings (TaskBindings, flowscheduler/scheduler.go:421-437):
 * task NodeID → bound PU NodeID (0 = unbind). A REMOVE_NODE of a task unbinds it. */
int ks_set_bindings(ks_ctx* ctx, const uint64_t* task, const uint64_t* pu, size_t k);

/* Scheduling deltas of the last solve against the bindings, on device:
 * SchedulingDeltasForPreemptedTasks (graph_manager.go:297-339) — a bound task absent
 * from the mapping → PREEMPT, emitted first — then NodeBindingToSchedulingDelta
 * (:253-295) per mapped task: unbound → PLACE, bound elsewhere → MIGRATE, bound here
 * → nothing; each in task-id order. Every destination must be a PU (:259-262),
 * else KS_E_VERIFY. commit != 0 applies the deltas to the bindings
 * (applySchedulingDeltas, scheduler.go:377-412). out == NULL: *count only, nothing
 * committed; otherwise cap ≥ the count is required (KS_E_INVALID, nothing committed). */
int ks_scheduling_deltas(ks_ctx* ctx, int commit, ks_sched_delta* out, size_t cap, size_t* count);

#define KS_COST_SET 0
#define KS_COST_ADD 1

/* UpdateAllCostsToUnscheduledAggs (graph_manager.go:462-475, called by Solve before
 * every incremental export, solver.go:86) on device, in place: for every task with
 * an arc into an unscheduled aggregator, a running task (it has a running arc,
 * type 1) gets its running arc set to continuation_cost (TaskContinuationCost),
 * any other task its arc to the aggregator set to (KS_COST_SET) or raised by
 * (KS_COST_ADD: waiting-time ageing) unsched_cost (TaskToUnscheduledAggCost).
 * Aggregators: unsched_ids (k of them), or with unsched_ids == NULL every type-0
 * node with an arc into the sink. *changed (may be NULL) = arcs whose cost changed. */
int ks_update_unsched_costs(ks_ctx* ctx, const uint64_t* unsched_ids, size_t k, int32_t mode,
                            int64_t unsched_cost, int64_t continuation_cost, size_t* changed);

/* ComputeTopologyStatistics (graph_manager.go:480-511; trivial model PrepareStats /
 * GatherStats, costmodel/trivial_cost_modeler.go:147-176) on device: BFS from the
 * sink over in-arcs; a PU takes (len(CurrentRunningTasks), max_tasks_per_pu), every
 * resource node above sums its children. CurrentRunningTasks lengths: pu_running[i]
 * for PU pu_ids[i] (k of them), or with pu_ids == NULL the running arcs (type 1)
 * into each PU. Writes slots_below[id-1] / running_below[id-1] for ids 1..*count
 * (0 for nodes that are not resources); cap < *count → KS_E_INVALID. */
int ks_topology_stats(ks_ctx* ctx, uint64_t max_tasks_per_pu, const uint64_t* pu_ids,
                      const uint64_t* pu_running, size_t k, uint64_t* slots_below,
                      uint64_t* running_below, size_t cap, size_t* count);

/* ---- config 5: independent graphs sharded over GPUs (SURVEY §7 step 6, §8 row e) --
 * No reference counterpart (ksched solves one graph per round,
 * flowscheduler/scheduler.go:350); this is the north star's multi-GPU mode: cluster
 * cells / what-if graphs, graph g on global rank g mod world, each device solving
 * the disjoint union of its graphs, then ONE collective — every rank's per-graph
 * rows to rank 0 over RCCL (ncclSend/ncclRecv in a group), inside the library. */
typedef struct ks_batch ks_batch;
#define KS_UNIQUE_ID_BYTES 128

/* One process driving several devices (ncclCommInitAll over devices[0..ndev)). */
ks_batch*   ks_batch_create(const int* devices, int ndev, const ks_opts* opts);
/* One process per GPU (e.g. under torch.distributed.run): rank 0 makes the id with
 * ks_batch_unique_id and shares it out of band; every rank then calls this. */
int         ks_batch_unique_id(uint8_t* id /* KS_UNIQUE_ID_BYTES */);
ks_batch*   ks_batch_create_rank(int device, int nranks, int rank, const uint8_t* id, const ks_opts* opts);
void        ks_batch_destroy(ks_batch* b);
const char* ks_batch_last_error(ks_batch* b);
/* Every rank passes ALL ngraphs graphs (arrays as for ks_load_graph); each device
 * uploads the ones it owns. */
int ks_batch_load(ks_batch* b, size_t ngraphs, const ks_node* const* nodes, const size_t* n,
                  const ks_arc* const* arcs, const size_t* m);
/* Solve every local device's union concurrently; results[i] (may be NULL) for the
 * i-th local device. */
int ks_batch_solve(ks_batch* b, ks_result* results);
/* Collective (all ranks call it): per graph its cost, flow value and the PU node id
 * (local to the graph, 0 = unscheduled) of each of its task nodes in id order,
 * gathered to global rank 0, whose pu[g·max_tasks ..], cost[g], flow[g] receive
 * them (other ranks may pass NULL). A rank that fails to pack its rows still
 * enters the collective; every rank then returns that failure. */
int ks_batch_gather(ks_batch* b, size_t max_tasks, uint64_t* pu, int64_t* cost, int64_t* flow);

/* Layout of the gather (host-only, no device or RCCL: the packing and unpacking
 * of ks_batch_gather use exactly these). Graph g is owned by global rank
 * g mod world as its (g div world)-th graph; each rank sends one block of
 * ks_batch_block_len elements: [status][slots rows of 2 + max_tasks: cost, flow
 * value, PU per task]. ks_batch_unpack turns the world blocks rank 0 received (in
 * rank order) into graph order; it returns a rank's non-zero status word. */
size_t      ks_batch_slots(size_t ngraphs, int world);
int         ks_batch_owner(size_t g, int world, int* rank, size_t* slot);
size_t      ks_batch_block_len(size_t ngraphs, int world, size_t max_tasks);
int         ks_batch_unpack(const int64_t* gathered, size_t ngraphs, int world, size_t max_tasks, uint64_t* pu,
                            int64_t* cost, int64_t* flow);

#ifdef __cplusplus
}
#endif

#endif /* KSMCMF_H */
