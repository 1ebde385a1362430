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

enum CellStatus { CS_OK = 0, CS_INFEASIBLE = 1, CS_NOCONV = 2, CS_TIMEOUT = 3 };

// Written by the cell's workgroup when it finishes.
struct CellOut {
    int status;            // CellStatus
    int phases;            // ε-phases run
    int updates;           // global price updates
    int pr_ok;             // price refinements that certified the flow
    int pr_tries;
    int last_eps;          // 1 when the solve ended at ε = 1 (scaled)
    int pad[2];
    unsigned long long sweeps, bf_rounds, scans, visits, pushes, relabels, gu_scans;
    unsigned long long ticks;   // s_memrealtime ticks (100 MHz) of the cell's solve
    // per operation kind (saturate, update init, Bellman-Ford round, update apply,
    // sweep, refinement init, refinement round, refinement apply): ticks incl. the
    // barriers and the controller, and counts
    unsigned long long op_ticks[8];
    unsigned op_n[8];
};
constexpr int CELL_NOPS = 8;

struct CellArgs {
    Pos* pos;
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
    int warm;
    int alpha;
    int pr_div;              // price refinement once ε·pr_div < mult
    int use_pr;
    int pr_cap;              // Bellman-Ford rounds a price refinement may take
    int gi;                  // sweeps between global updates
    int phase_exit, phase_frac;   // coarse phases end with few excess nodes left
    int mode;                // 0: solve from the state in place; 1: certificate recovery at ε = 1
    int max_nodes;           // largest cell (sizes the LDS)
    unsigned long long timeout_ticks;   // a cell's solve gives up after this many 100 MHz ticks
};

// LDS one workgroup needs for cells of up to n nodes (0 when they do not fit).
size_t cell_lds_bytes(int n);
// Largest cell the LDS holds.
int cell_max_nodes();
hipError_t cell_launch(const CellArgs& a, hipStream_t st);

}  // namespace ks
