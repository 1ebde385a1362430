// ks_cell.h — the cell solver of libksmcmf (internal): a whole ε-scaling
// min-cost-flow solve of one small graph inside ONE workgroup.
//
// A cell-sized graph (config 2: n = 12,127, 106k residual positions) is all
// latency for the multi-kernel engine: ~2,300 dependent launches of a few µs
// each. Here one 1024-thread workgroup runs every phase, global price update,
// push/relabel sweep and price refinement of the cell on one CU, separated by
// workgroup barriers instead of kernel boundaries, with the cell's prices and
// Bellman-Ford distances resident in LDS (12 B per node) and its frontiers as
// per-class lists compacted through an LDS bitmap. Independent cells (config 5)
// are independent workgroups of ONE launch: 64 cells run on 64 CUs at once.
//
// Memory model: a cell's state is touched only by its own workgroup, so plain
// loads/stores, workgroup-scope atomics (performed in the XCD's L2, never
// beyond it) and __syncthreads() are the whole protocol.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "ks_pos.h"

namespace ks {

constexpr int CELL_NCLS = 7;          // residual degree classes of a cell's nodes
constexpr int CELL_THREADS = 1024;    // one workgroup per cell

// ≤ 4, 8, 16, 32, 64 positions: one lane group of that width per node;
// ≤ 512: one wave per node; more (the cluster aggregator, a large sink): the
// whole workgroup per node.
__host__ __device__ inline int cell_class(int cap) {
    return cap <= 4 ? 0 : cap <= 8 ? 1 : cap <= 16 ? 2 : cap <= 32 ? 3 : cap <= 64 ? 4 : cap <= 512 ? 5 : 6;
}

// One cell: its nodes are the internal ids [cb[0], cb[7]), class c = [cb[c], cb[c+1]).
struct CellDesc {
    int cb[CELL_NCLS + 1];
};

// The cell solver's 16-byte copy of a residual position (packed before a solve
// from the 32-byte ks_pos.h record, its residual written back after): residual and
// pair capacity (int32), the SCALED cost (int32 — cost·(n+1) must fit, else the
// solve falls back to the engine; CELL_DEAD for an inert position), the head as a cell-local node index (14 bits) and the reverse
// position relative to the cell's first position (18 bits). A task's eight
// positions are one 128-byte line instead of two.
struct alignas(16) CellPos {
    int rcap;
    int ucap;
    int cost;
    unsigned hr;             // head_local | rev_rel << CELL_HEAD_BITS
};
constexpr int CELL_HEAD_BITS = 14;
constexpr int CELL_MAX_POS = 1 << (32 - CELL_HEAD_BITS);   // positions per cell the record addresses
constexpr int CELL_DEAD = 0x7fffffff;                       // an inert position's cost
constexpr long long CELL_MAX_CAP = (1LL << 24) - 1;         // capacities the cell solver takes (a lane group's
                                                            // admissible sum then fits int32) and |cost|
constexpr long long CELL_MAX_COST = (1LL << 31) - 2;        // |scaled cost| (CELL_DEAD = 2^31 − 1 marks inert)

enum CellStatus { CS_OK = 0, CS_INFEASIBLE = 1, CS_NOCONV = 2, CS_TIMEOUT = 3, CS_RANGE = 4 };

// Written by the cell's workgroup when it finishes.
struct CellOut {
    int status;            // CellStatus
    int phases;            // ε-phases run
    int updates;           // global price updates
    int pr_ok;             // price refinements that certified the flow
    int pr_tries;
    int last_eps;          // 1 when the solve ended at ε = 1 (scaled)
    int cycles;            // negative cycles the cycle-cancelling finish cancelled
    int searches;          // its parent-graph searches
    int rejected;          // leaders whose walk did not close a cycle (a chain, a longer cycle)
    unsigned cyc_dbg[4];   // diagnostics: nodes with a parent, marked on a cycle, leaders, closed walks
    unsigned long long sweeps, bf_rounds, scans, visits, pushes, relabels, gu_scans;
    unsigned long long ticks;   // s_memrealtime ticks (100 MHz) of the cell's solve
    // per operation kind (saturate, update init, Bellman-Ford round, update apply,
    // sweep, refinement init, refinement round, refinement apply): ticks incl. the
    // barriers and the controller, and counts
    unsigned long long op_ticks[9];      // (and the finish's parent-graph searches)
    unsigned op_n[9];
    unsigned long long item_ticks[9];    // diagnostics: op start → the last wave's items done
    unsigned long long first_ticks[9];   //              op start → the first wave's items done
    unsigned long long cls_ticks[32];    //              item ticks by step (sweep, BF, refinement, saturate) × class
    unsigned cls_n[32];                  //              and items (class 6: the workgroup-sized nodes)
    unsigned long long hist_t[12];       //              sweep (0–5) / BF round (6–11) ticks by frontier size
    unsigned hist_n[12];                 //              (≤ 16, 64, 256, 1k, 4k, more nodes) and counts
    unsigned long long phase_ticks[8];   //              ticks by ε-phase (the last slot: phases 8 and up,
                                         //              and the refinements)
};
constexpr int CELL_NOPS = 9;

struct CellArgs {
    Pos* pos;
    CellPos* cp;             // m2 compact positions (k_cell_pack before, k_cell_unpack after)
    const int* first;        // segment starts (a cell's positions begin at first[cb[0]])
    int m2;
    long long* nd;           // node records (p0, dist, p1, packed segment) × nn
    long long* excess;
    const CellDesc* cells;
    int ncells;
    int nn;                  // internal node ids
    int* lists;              // 2 × nn: two frontier buffers (a node's class slice at its class range)
    int* rl_node;            // nn: relabels pending until the end of a sweep
    long long* rl_p;         // nn
    CellOut* out;            // ncells
    long long mult;          // cost scaling (n + 1)
    long long eps_start;     // ε before the first phase's division by α
    long long sat_thr0;      // the first phase saturates arcs below −sat_thr0 (warm start), else 0
    int warm;                // 1: warm start (the first phase saturates only violations); 2: every phase
    int alpha;
    int pr_div;              // price refinement once ε·pr_div < mult
    int use_pr;
    int pr_cap;              // Bellman-Ford rounds a price refinement may take
    int use_prc;             // the cycle-cancelling finish (ks_opts.price_refine 1)
    int prc_cap;             // its rounds before it gives up (the final phase then runs)
    int gi;                  // sweeps between global updates
    int phase_exit, phase_frac;   // coarse phases end with few excess nodes left
    int mode;                // 0: solve from the state in place; 1: certificate recovery at ε = 1
    int max_nodes;           // largest cell (sizes the LDS)
    unsigned long long timeout_ticks;   // a cell's solve gives up after this many 100 MHz ticks
    int diag;                // per-item / per-class timing for the cycle log (ks_opts.log_cycles)
    int bound;               // 1: bounded global updates (ks_opts.bf_bound >= 0)
    const int* bad;          // set by k_cell_pack: a value the compact record cannot hold
    int fault_cell;          // TESTS ONLY (ks_opts.fault_inject bit 4): this cell stops after
    int fault_ops;           //   fault_ops operations with CS_NOCONV (−1: none)
    int cyc_lg;              // the finish's doubling steps (CYC_LOG; TESTS ONLY, fault_inject bit 7: 5)
};

// LDS one workgroup needs for cells of up to n nodes (0 when they do not fit in
// limit bytes: the device's opt-in LDS per workgroup, 160 KiB on gfx950).
size_t cell_lds_bytes(int n, size_t limit);
// Largest cell the LDS holds (and the compact record's head field addresses).
int cell_max_nodes(size_t limit);
// k_cell_pack → k_cell → k_cell_unpack on st; *bad (device int) is set when a
// position does not fit the compact record (every cell then returns CS_RANGE).
// *refused: the device will not run k_cell at this size (its LDS); any other
// error is a real launch failure
hipError_t cell_launch(const CellArgs& a, int* bad, size_t lds_limit, hipStream_t st, bool* refused);

}  // namespace ks
